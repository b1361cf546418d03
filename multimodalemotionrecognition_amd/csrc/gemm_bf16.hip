// bf16 MFMA GEMM with fused epilogues -- the encoder workhorse.
//
//   C[m, n] = epi( sum_k A(m, k) * W[n, k] )        (nn.Linear / Conv1d-as-GEMM layout)
//   epi(v)  = act(v + bias[n]) (+ R[m, n])            fp32 accumulate, bf16 or fp32 output
//
// A-operand addressing modes (the K-contiguous "row" of the implicit im2col matrix):
//   mode 0 (rows):   row m starts at A + (m / rpg) * gstride + (m % rpg) * rstride.
//                    rpg = M, rstride = lda is a plain GEMM; with rpg = L_out, rstride = stride*C_in,
//                    gstride = L_in*C_in it is a channel-last Conv1d (WavLM feature extractor,
//                    TF:723-782): the k-window of output t is the contiguous slice x[b, t*s : t*s+k, :].
//   mode 1 (posconv): grouped Conv1d(768,768,k=128,pad=64,groups=16) of the WavLM positional embedding
//                    (TF:48-90): A(m=(b,t), k=(tap,c)) = x[b, t+tap-pad, g*Cg + c], zero outside [0,L);
//                    group g = blockIdx.z, output columns g*Cg + n.
//
// Tile 128x128x64, 256 threads = 4 waves (2x2), each wave 64x64 = 4x4 v_mfma_f32_16x16x32_bf16.
// Register-staged double-buffered LDS (one barrier per K step); LDS rows padded to 72 elements
// (144 B) so the 16 rows read by one ds_read_b128 lane group land on distinct banks.
#include "common.h"
#include "mer.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64, LDSK = BK + 8;

struct GemmArgs {
  int M, N, K;
  const bf16_t* A;
  long a_gstride, a_rstride;
  int a_rpg;
  int pc_L, pc_pad, pc_cg;
  long pc_ldx;
  const bf16_t* B;
  long ldb, b_zstride;
  void* C;
  long ldc, c_zoff;
  const float* bias;
  const bf16_t* R;
  long ldr;
  int act;
};

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

template <int AMODE>
__device__ __forceinline__ u32x4 load_a_chunk(const GemmArgs& g, int m, int k, int z) {
  u32x4 v = {0u, 0u, 0u, 0u};
  if (m >= g.M || k >= g.K) return v;
  if (AMODE == 0) {
    const bf16_t* p = g.A + (long)(m / g.a_rpg) * g.a_gstride + (long)(m % g.a_rpg) * g.a_rstride + k;
    v = *reinterpret_cast<const u32x4*>(p);
  } else {
    const int b = m / g.pc_L, t = m % g.pc_L;
    const int tap = k / g.pc_cg, c = k % g.pc_cg;
    const int src = t + tap - g.pc_pad;
    if (src >= 0 && src < g.pc_L) {
      const bf16_t* p = g.A + ((long)b * g.pc_L + src) * g.pc_ldx + (long)z * g.pc_cg + c;
      v = *reinterpret_cast<const u32x4*>(p);
    }
  }
  return v;
}

template <int AMODE, typename TOUT>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2][2][BM * LDSK];  // [buf][A/B][row*LDSK + k]
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int z = blockIdx.z;
  const int nx = (g.N + BN - 1) / BN, ny = (g.M + BM - 1) / BM;
  int tx, ty;
  xcd_tile(blockIdx.x, nx, nx * ny, tx, ty);
  const int m0 = ty * BM, n0 = tx * BN;
  const bf16_t* Bz = g.B + (long)z * g.b_zstride;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;

  // each thread stages 4 A chunks and 4 B chunks of 8 bf16 per K step
  const int crow = t >> 3, ckc = t & 7;
  u32x4 ra[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = crow + 32 * i;
      ra[i] = load_a_chunk<AMODE>(g, m0 + r, k0 + ckc * 8, z);
      const int n = n0 + r, k = k0 + ckc * 8;
      rb[i] = (n < g.N && k < g.K) ? *reinterpret_cast<const u32x4*>(Bz + (long)n * g.ldb + k) : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = crow + 32 * i;
      *reinterpret_cast<u32x4*>(&lds[buf][0][r * LDSK + ckc * 8]) = ra[i];
      *reinterpret_cast<u32x4*>(&lds[buf][1][r * LDSK + ckc * 8]) = rb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (g.K + BK - 1) / BK;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[4], bfr[4];
      const int kof = s * 32 + (lane >> 4) * 8;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(&lds[cur][0][(wm + i * 16 + (lane & 15)) * LDSK + kof]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(&lds[cur][1][(wn + j * 16 + (lane & 15)) * LDSK + kof]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

  // epilogue: row = (lane>>4)*4 + r, col = lane & 15 within each 16x16 tile
  TOUT* C = reinterpret_cast<TOUT*>(g.C) + (long)z * g.c_zoff;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wn + j * 16 + (lane & 15);
      if (col >= g.N) continue;
      const float bv = g.bias ? g.bias[(long)z * g.c_zoff + col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
        if (row >= g.M) continue;
        float v = apply_act(acc[i][j][r] + bv, g.act);
        if (g.R) v += bf2f(g.R[(long)row * g.ldr + (long)z * g.c_zoff + col]);
        stf<TOUT>(C, (long)row * g.ldc + col, v);
      }
    }
}

template <int AMODE>
int launch(const GemmArgs& g, int out_dtype, int groups, hipStream_t st) {
  dim3 grid(((g.N + BN - 1) / BN) * ((g.M + BM - 1) / BM), 1, groups);
  if (out_dtype == MER_BF16)
    hipLaunchKernelGGL((gemm_bf16_kernel<AMODE, bf16_t>), grid, dim3(256), 0, st, g);
  else
    hipLaunchKernelGGL((gemm_bf16_kernel<AMODE, float>), grid, dim3(256), 0, st, g);
  return (int)hipGetLastError();
}

}  // namespace

MER_API int mer_gemm_bf16(int M, int N, int K, const void* A, long a_gstride, long a_rstride, int a_rpg, const void* W,
                          long ldw, void* C, int c_dtype, long ldc, const float* bias, const void* R, long ldr, int act,
                          void* stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 8 != 0 || a_rpg <= 0 || (a_rstride % 8) != 0 || (a_gstride % 8) != 0 || (ldw % 8) != 0)
    return (int)hipErrorInvalidValue;
  if ((((uintptr_t)A) | ((uintptr_t)W)) & 15) return (int)hipErrorInvalidValue;
  GemmArgs g{};
  g.M = M; g.N = N; g.K = K;
  g.A = (const bf16_t*)A; g.a_gstride = a_gstride; g.a_rstride = a_rstride; g.a_rpg = a_rpg;
  g.B = (const bf16_t*)W; g.ldb = ldw; g.b_zstride = 0;
  g.C = C; g.ldc = ldc; g.c_zoff = 0;
  g.bias = bias; g.R = (const bf16_t*)R; g.ldr = ldr; g.act = act;
  return launch<0>(g, c_dtype, 1, (hipStream_t)stream);
}

MER_API int mer_posconv_gemm_bf16(int B, int L, int C_total, int groups, int taps, int pad, const void* X, long ldx,
                                  const void* Wp, void* out, int out_dtype, long ldo, const float* bias,
                                  const void* R, long ldr, int act, void* stream) {
  const int cg = C_total / groups;
  if (cg * groups != C_total || cg % 8 != 0 || (ldx % 8) != 0) return (int)hipErrorInvalidValue;
  GemmArgs g{};
  g.M = B * L; g.N = cg; g.K = taps * cg;
  g.A = (const bf16_t*)X; g.pc_L = L; g.pc_pad = pad; g.pc_cg = cg; g.pc_ldx = ldx;
  g.B = (const bf16_t*)Wp; g.ldb = (long)taps * cg; g.b_zstride = (long)cg * taps * cg;
  g.C = out; g.ldc = ldo; g.c_zoff = cg;
  g.bias = bias; g.R = (const bf16_t*)R; g.ldr = ldr; g.act = act;
  return launch<1>(g, out_dtype, groups, (hipStream_t)stream);
}
