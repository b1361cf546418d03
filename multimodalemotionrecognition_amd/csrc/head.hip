// fp32 kernels of the fusion head (fusion.py:153-184, 351-411, temporal.py:105-110, train.py:212-228).
//
// The head is tiny next to the encoders (1.1 GFLOP fwd at B=32) and the parity bar
// for it is "logits within 1e-3 of the fp32 CPU reference", so everything here computes
// in exact fp32: the GEMM uses the f32-input MFMA (v_mfma_f32_16x16x4_f32, bit-identical
// to an fma chain), softmax / LayerNorm reductions use wave64 shuffles.
#include "common.h"
#include "mer.h"

// ---------------------------------------------------------------------------------------
// Strided-batched fp32 GEMM on f32 MFMA:  C[m,n] (+)= act( sum_k A[m,k] B[k,n] + bias[n] )
// A(m,k) at A[m*sam + k*sak], B(k,n) at B[k*sbk + n*sbn]; C row-major with ldc.
// 64x64 tile, K chunks of 32, 256 threads = 4 waves of 32x32 (2x2 16x16 MFMA tiles).  Each thread
// moves 8 consecutive elements of A and of B per chunk (16-byte loads where the operand's unit-stride
// axis and alignment allow, VEC), the next chunk's loads are in flight while the current chunk is
// multiplied out of the other LDS buffer (one barrier per chunk).  LDS images are k-major [k][m|n]
// (+4 pad), so an MFMA operand read is 16 consecutive floats per k row.
// splitk > 1: each K slice stores its partial into the workspace [batch][splitk][M][N] and a fold kernel
// adds the slices into C in slice order (deterministic; caller pre-initialises C; act must be 0).
// ---------------------------------------------------------------------------------------
constexpr int GF_BK = 32, GF_LD = 64 + 4;

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float* v);
template <>
__device__ __forceinline__ void ld8<float>(const float* p, float* v) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}
template <>
__device__ __forceinline__ void ld8<bf16_t>(const bf16_t* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

// 8 elements of one operand: `lin` runs along the operand's unit-stride axis (8 consecutive
// elements starting at lin0, valid below lin_end), `fix` is the other coordinate (valid when ok).
template <typename T, bool VEC>
__device__ __forceinline__ void load_seg(const T* base, long s_lin, long s_fix, int lin0, int lin_end, int fix, bool ok,
                                         float* v) {
  if (!ok) {
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = 0.f;
    return;
  }
  const T* p = base + (long)fix * s_fix + (long)lin0 * s_lin;
  if (VEC && lin0 + 8 <= lin_end) {
    ld8<T>(p, v);
  } else {
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = lin0 + c < lin_end ? ldf<T>(p, (long)c * s_lin) : 0.f;
  }
}

template <typename TA, typename TB, bool A_KCONTIG, bool B_NCONTIG, bool VEC>
__global__ __launch_bounds__(256) void gemm_f32_kernel(int M, int N, int K, const TA* __restrict__ A, long sam,
                                                       long sak, long bsa, const TB* __restrict__ B, long sbk,
                                                       long sbn, long bsb, float* __restrict__ C, long ldc,
                                                       long bsc, const float* __restrict__ bias, int beta,
                                                       int act, int splitk, float* __restrict__ ws) {
  __shared__ float As[2][GF_BK][GF_LD];
  __shared__ float Bs[2][GF_BK][GF_LD];
  const int bz = blockIdx.z, batch = bz / splitk, ks = bz % splitk;
  A += batch * bsa;
  B += batch * bsb;
  C += batch * bsc;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int kchunk = ((K + splitk - 1) / splitk + GF_BK - 1) / GF_BK * GF_BK;
  const int kbeg = ks * kchunk, kend = min(K, kbeg + kchunk);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
  // this thread's segment: along k (row r = t>>2, k = (t&3)*8) or along m/n (k = t>>3, (t&7)*8)
  const int sr = t >> 2, sk = (t & 3) * 8, tk = t >> 3, tc = (t & 7) * 8;
  float ra[8], rb[8];
  auto gload = [&](int k0) {
    if (A_KCONTIG) load_seg<TA, VEC>(A, sak, sam, k0 + sk, kend, m0 + sr, m0 + sr < M, ra);
    else load_seg<TA, VEC>(A, sam, sak, m0 + tc, M, k0 + tk, k0 + tk < kend, ra);
    if (B_NCONTIG) load_seg<TB, VEC>(B, sbn, sbk, n0 + tc, N, k0 + tk, k0 + tk < kend, rb);
    else load_seg<TB, VEC>(B, sbk, sbn, k0 + sk, kend, n0 + sr, n0 + sr < N, rb);
  };
  auto lstore = [&](int buf) {
    if (A_KCONTIG) {
#pragma unroll
      for (int c = 0; c < 8; ++c) As[buf][sk + c][sr] = ra[c];
    } else {
      *reinterpret_cast<f32x4*>(&As[buf][tk][tc]) = f32x4{ra[0], ra[1], ra[2], ra[3]};
      *reinterpret_cast<f32x4*>(&As[buf][tk][tc + 4]) = f32x4{ra[4], ra[5], ra[6], ra[7]};
    }
    if (B_NCONTIG) {
      *reinterpret_cast<f32x4*>(&Bs[buf][tk][tc]) = f32x4{rb[0], rb[1], rb[2], rb[3]};
      *reinterpret_cast<f32x4*>(&Bs[buf][tk][tc + 4]) = f32x4{rb[4], rb[5], rb[6], rb[7]};
    } else {
#pragma unroll
      for (int c = 0; c < 8; ++c) Bs[buf][sk + c][sr] = rb[c];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kbeg < kend) {
    gload(kbeg);
    lstore(0);
  }
  __syncthreads();
  int buf = 0;
  for (int k0 = kbeg; k0 < kend; k0 += GF_BK, buf ^= 1) {
    const bool more = k0 + GF_BK < kend;
    if (more) gload(k0 + GF_BK);
#pragma unroll
    for (int kk = 0; kk < GF_BK / 4; ++kk) {
      const int kr = kk * 4 + (lane >> 4);
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[buf][kr][wm + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[buf][kr][wn + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) lstore(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
        const int col = n0 + wn + j * 16 + (lane & 15);
        if (row < M && col < N) {
          float v = acc[i][j][r];
          if (bias && ks == 0) v += bias[col];
          float* cp = C + (long)row * ldc + col;
          if (splitk > 1) {  // this K slice's own partial (summed in slice order by gemm_splitk_fold_kernel)
            ws[((long)bz * M + row) * N + col] = v;
          } else {
            if (beta) v += *cp;
            *cp = apply_act(v, act);
          }
        }
      }
}

// VEC: the unit-stride axis of both operands allows 16-byte segment loads (8 elements of bf16,
// 2 x 4 of fp32): base and every non-unit stride a multiple of the segment's alignment.
template <typename T>
static bool vec_ok(const void* p, long s1, long s2) {
  const long al = 16 / (long)sizeof(T) >= 8 ? 8 : 4;  // elements per 16-byte load
  return (((uintptr_t)p) & 15) == 0 && s1 % al == 0 && s2 % al == 0;
}

// C[b][m][n] += sum_{ks < splitk} ws[b][ks][m][n], slices in order
__global__ __launch_bounds__(256) void gemm_splitk_fold_kernel(int M, int N, int splitk, int batch,
                                                               const float* __restrict__ ws, float* __restrict__ C,
                                                               long ldc, long bsc) {
  const long total = (long)batch * M * N;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long b = e / ((long)M * N), mn = e - b * M * N;
    const int m = (int)(mn / N), n = (int)(mn - (long)m * N);
    const float* p = ws + (b * splitk) * M * N + mn;
    float acc = 0.f;
    for (int k = 0; k < splitk; ++k) acc += p[(long)k * M * N];
    C[b * bsc + (long)m * ldc + n] += acc;
  }
}

template <typename TA, typename TB>
static int launch_gemm_f32(int M, int N, int K, const void* A, long sam, long sak, long bsa, const void* B, long sbk,
                           long sbn, long bsb, float* C, long ldc, long bsc, const float* bias, int beta, int act,
                           int splitk, int batch, float* ws, hipStream_t st) {
  dim3 grid((N + 63) / 64, (M + 63) / 64, batch * splitk);
  const bool akc = (sak == 1), bnc = (sbn == 1);
  // the unit stride of each operand and its other strides must suit 16-byte loads
  const bool va = akc ? vec_ok<TA>(A, sam, bsa) : (sam == 1 && vec_ok<TA>(A, sak, bsa));
  const bool vb = bnc ? vec_ok<TB>(B, sbk, bsb) : (sbk == 1 && vec_ok<TB>(B, sbn, bsb));
  const bool vec = va && vb;
#define L(AK, BN, V)                                                                                                     \
  hipLaunchKernelGGL((gemm_f32_kernel<TA, TB, AK, BN, V>), grid, dim3(256), 0, st, M, N, K, (const TA*)A, sam, sak, \
                     bsa, (const TB*)B, sbk, sbn, bsb, C, ldc, bsc, bias, beta, act, splitk, ws)
  if (vec) {
    if (akc && bnc) L(true, true, true); else if (akc) L(true, false, true); else if (bnc) L(false, true, true); else L(false, false, true);
  } else {
    if (akc && bnc) L(true, true, false); else if (akc) L(true, false, false); else if (bnc) L(false, true, false); else L(false, false, false);
  }
#undef L
  if (splitk > 1) {
    const long total = (long)batch * M * N;
    const int grid = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(gemm_splitk_fold_kernel, dim3(grid), dim3(256), 0, st, M, N, splitk, batch, ws, C, ldc, bsc);
  }
  MER_LAUNCH_CHECK();
}

MER_API int mer_gemm_f32(int M, int N, int K, const void* A, int a_dtype, long sam, long sak, long bsa, const void* B,
                         int b_dtype, long sbk, long sbn, long bsb, float* C, long ldc, long bsc, const float* bias,
                         int beta, int act, int splitk, int batch, float* workspace, void* stream) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  if (splitk < 1) splitk = 1;
  if (splitk > 1 && (act != MER_ACT_NONE || !workspace)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (a_dtype == MER_F32 && b_dtype == MER_F32)
    return launch_gemm_f32<float, float>(M, N, K, A, sam, sak, bsa, B, sbk, sbn, bsb, C, ldc, bsc, bias, beta, act, splitk, batch, workspace, st);
  if (a_dtype == MER_BF16 && b_dtype == MER_F32)
    return launch_gemm_f32<bf16_t, float>(M, N, K, A, sam, sak, bsa, B, sbk, sbn, bsb, C, ldc, bsc, bias, beta, act, splitk, batch, workspace, st);
  if (a_dtype == MER_F32 && b_dtype == MER_BF16)
    return launch_gemm_f32<float, bf16_t>(M, N, K, A, sam, sak, bsa, B, sbk, sbn, bsb, C, ldc, bsc, bias, beta, act, splitk, batch, workspace, st);
  return launch_gemm_f32<bf16_t, bf16_t>(M, N, K, A, sam, sak, bsa, B, sbk, sbn, bsb, C, ldc, bsc, bias, beta, act, splitk, batch, workspace, st);
}

// ---------------------------------------------------------------------------------------
// Column sum (bias gradient): out[n] (+)= sum_m X[m*ldx + n]
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void colsum_kernel(int M, int N, const float* __restrict__ X, long ldx,
                                                     float* __restrict__ part, int rows_per_block) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float s = 0.f;
  if (c < N)
    for (int r = r0 + rg; r < r1; r += 4) s += X[(long)r * ldx + c];
  red[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && c < N) part[(long)blockIdx.y * N + c] = (red[0][threadIdx.x] + red[1][threadIdx.x]) +
                                                         (red[2][threadIdx.x] + red[3][threadIdx.x]);
}

// out0[e] (e < split) / out1[e - split] += sum_{r < rows} in[r*E + e]: fixed-order per-entry sums of
// per-block partial rows (64 entries per block, the 16 waves split the rows and meet in LDS in a fixed tree
// order; 16 rather than 4 waves: the per-thread row loop is a latency chain, 12.8 us at ~300 partial rows)
__global__ __launch_bounds__(1024) void rows_sum_add_kernel(int E, int rows, const float* __restrict__ in, int split,
                                                            float* __restrict__ out0, float* __restrict__ out1) {
  __shared__ float part[16][64];
  const int el = threadIdx.x & 63, pg = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + el;
  float a0 = 0.f, a1 = 0.f;
  if (e < E) {
    int r = pg;
    for (; r + 16 < rows; r += 32) {
      a0 += in[(long)r * E + e];
      a1 += in[(long)(r + 16) * E + e];
    }
    if (r < rows) a0 += in[(long)r * E + e];
  }
  part[pg][el] = a0 + a1;
  __syncthreads();
  if (pg == 0 && e < E) {
    float q[4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
      q[g] = (part[4 * g][el] + part[4 * g + 1][el]) + (part[4 * g + 2][el] + part[4 * g + 3][el]);
    const float v = (q[0] + q[1]) + (q[2] + q[3]);
    if (e < split) {
      if (out0) out0[e] += v;
    } else if (out1) {
      out1[e - split] += v;
    }
  }
}

static int colsum_rows_per_block(int M, int N) {
  const int nx = (N + 63) / 64;
  int rpb = (int)(((long)M * nx / 1024 + 3) / 4 * 4);  // ~1024 blocks: short per-thread row loops
  return rpb < 16 ? 16 : (rpb > 256 ? 256 : rpb);
}
MER_API int mer_colsum_f32(int M, int N, const float* X, long ldx, float* out, float* workspace, void* stream) {
  if (M <= 0 || N <= 0) return 0;
  const int rpb = colsum_rows_per_block(M, N);
  const int ny = (M + rpb - 1) / rpb;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(colsum_kernel, dim3((N + 63) / 64, ny), dim3(256), 0, st, M, N, X, ldx, workspace, rpb);
  hipLaunchKernelGGL(rows_sum_add_kernel, dim3((N + 63) / 64), dim3(1024), 0, st, N, ny, workspace, N, out,
                     (float*)nullptr);
  MER_LAUNCH_CHECK();
}

// (multi-head attention core: attn.hip)

// ---------------------------------------------------------------------------------------
// y = LayerNorm(x + s_b * r) (fusion.py:395,399 with StochasticDepth fusion.py:11-26):
// s_b = per-sample drop-path scale regenerated from (seed, b); r may be null.
// Saves the pre-norm sum (for backward), mean and rstd.  One wave per row.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void add_ln_fwd_kernel(int rows, int d, int rows_per_sample, const float* __restrict__ x,
                                                         const float* __restrict__ r, float dp_p,
                                                         const unsigned long long* __restrict__ seed_ptr,
    unsigned long long site, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float eps, float* __restrict__ y,
                                                         float* __restrict__ sum_out, float* __restrict__ mean_out,
                                                         float* __restrict__ rstd_out) {
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float sc = r ? dropout_scale(seed, row / rows_per_sample, dp_p) : 0.f;
  const float* xr = x + (long)row * d;
  const float* rr = r ? r + (long)row * d : nullptr;
  float s = 0.f;
  for (int c = lane; c < d; c += 64) {
    const float v = xr[c] + (rr ? sc * rr[c] : 0.f);
    if (sum_out) sum_out[(long)row * d + c] = v;
    s += v;
  }
  const float mean = wave_sum(s) / d;
  float q = 0.f;
  for (int c = lane; c < d; c += 64) {
    const float v = xr[c] + (rr ? sc * rr[c] : 0.f) - mean;
    q += v * v;
  }
  const float rstd = rsqrtf(wave_sum(q) / d + eps);
  for (int c = lane; c < d; c += 64) {
    const float v = xr[c] + (rr ? sc * rr[c] : 0.f);
    y[(long)row * d + c] = (v - mean) * rstd * gamma[c] + beta[c];
  }
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

MER_API int mer_add_ln_fwd(int rows, int d, int rows_per_sample, const float* x, const float* r, float dp_p,
                           const unsigned long long* seed, unsigned long long site, const float* gamma, const float* beta, float eps, float* y,
                           float* sum_out, float* mean_out, float* rstd_out, void* stream) {
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(add_ln_fwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, rows, d,
                     rows_per_sample, x, r, dp_p, seed, site, gamma, beta, eps, y, sum_out, mean_out, rstd_out);
  MER_LAUNCH_CHECK();
}

// dsum = rstd*(g - mean(g) - xhat*mean(g*xhat)), g = gamma*dy; dx = dsum, dr = s_b*dsum.
// dgamma += sum_rows dy*xhat, dbeta += sum_rows dy: each block stores its (dgamma | dbeta) partial row,
// rows_sum_add_kernel adds the rows in block order (deterministic).
__global__ __launch_bounds__(256) void add_ln_bwd_kernel(int rows, int d, int rows_per_sample, const float* __restrict__ dy,
                                                         const float* __restrict__ s, const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                         float dp_p, const unsigned long long* __restrict__ seed_ptr,
    unsigned long long site, float* __restrict__ dx,
                                                         float* __restrict__ dr, float* __restrict__ part,
                                                         int rows_per_block) {
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  extern __shared__ __attribute__((aligned(16))) float red[];  // [2][4][d]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int c = threadIdx.x; c < 8 * d; c += 256) red[c] = 0.f;
  __syncthreads();
  const int r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  for (int row = r0 + w; row < r1; row += 4) {
    const float mu = mean[row], rs = rstd[row];
    const float* dyr = dy + (long)row * d;
    const float* sr = s + (long)row * d;
    float a = 0.f, bsum = 0.f;
    for (int c = lane; c < d; c += 64) {
      const float xh = (sr[c] - mu) * rs;
      const float g = gamma[c] * dyr[c];
      a += g;
      bsum += g * xh;
      red[(0 * 4 + w) * d + c] += dyr[c] * xh;
      red[(1 * 4 + w) * d + c] += dyr[c];
    }
    a = wave_sum(a) / d;
    bsum = wave_sum(bsum) / d;
    const float sc = dr ? dropout_scale(seed, row / rows_per_sample, dp_p) : 0.f;
    for (int c = lane; c < d; c += 64) {
      const float xh = (sr[c] - mu) * rs;
      const float v = rs * (gamma[c] * dyr[c] - a - xh * bsum);
      dx[(long)row * d + c] = v;
      if (dr) dr[(long)row * d + c] = sc * v;
    }
  }
  __syncthreads();
  // this block's (dgamma | dbeta) partial row; rows_sum_add_kernel folds the rows in block order
  float* pr = part + (long)blockIdx.x * 2 * d;
  for (int c = threadIdx.x; c < d; c += 256) {
    pr[c] = red[0 * d + c] + red[1 * d + c] + red[2 * d + c] + red[3 * d + c];
    pr[d + c] = red[4 * d + c] + red[5 * d + c] + red[6 * d + c] + red[7 * d + c];
  }
}

MER_API int mer_add_ln_bwd(int rows, int d, int rows_per_sample, const float* dy, const float* s, const float* mean,
                           const float* rstd, const float* gamma, float dp_p, const unsigned long long* seed, unsigned long long site, float* dx,
                           float* dr, float* dgamma, float* dbeta, float* workspace, void* stream) {
  if (rows <= 0) return 0;
  if ((size_t)8 * d * sizeof(float) > 160 * 1024) return (int)hipErrorInvalidValue;
  // 16 rows per block (4 per wave): each row is a short chain of dependent loads and wave reductions, so the
  // kernel is latency-bound and wants many blocks (64 rows per block made it 31 us at 256 rows AND at 4,768)
  const int rpb = 16;
  const int nb = (rows + rpb - 1) / rpb;
  hipLaunchKernelGGL(add_ln_bwd_kernel, dim3(nb), dim3(256), 8 * d * sizeof(float), (hipStream_t)stream, rows, d,
                     rows_per_sample, dy, s, mean, rstd, gamma, dp_p, seed, site, dx, dr, workspace, rpb);
  hipLaunchKernelGGL(rows_sum_add_kernel, dim3((2 * d + 63) / 64), dim3(1024), 0, (hipStream_t)stream, 2 * d, nb,
                     workspace, d, dgamma, dbeta);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// Mean over dim 1 (TemporalPooler 'mean', temporal.py:108-109): [B,L,D] -> y[b*ldy + c].
// ---------------------------------------------------------------------------------------
// 64 columns x 4 row groups per block, combined in a fixed order (a single thread walking all L rows was a
// 149-long dependent load chain, ~20 us for the audio pooling)
__global__ __launch_bounds__(256) void mean_pool_fwd_kernel(int B, int L, int D, const float* __restrict__ x,
                                                            float* __restrict__ y, long ldy) {
  __shared__ float part[4][64];
  const int b = blockIdx.y, el = threadIdx.x & 63, g = threadIdx.x >> 6, c = blockIdx.x * 64 + el;
  float s0 = 0.f, s1 = 0.f;
  if (c < D) {
    int l = g;
    for (; l + 4 < L; l += 8) {
      s0 += x[((long)b * L + l) * D + c];
      s1 += x[((long)b * L + l + 4) * D + c];
    }
    if (l < L) s0 += x[((long)b * L + l) * D + c];
  }
  part[g][el] = s0 + s1;
  __syncthreads();
  if (g == 0 && c < D) y[(long)b * ldy + c] = ((part[0][el] + part[1][el]) + (part[2][el] + part[3][el])) / L;
}
__global__ void mean_pool_bwd_kernel(int B, int L, int D, const float* __restrict__ dy, long lddy, float* __restrict__ dx,
                                     int accumulate) {
  const long n = (long)B * L * D;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int c = e % D;
    const int b = e / ((long)L * D);
    const float g = dy[(long)b * lddy + c] / L;
    dx[e] = accumulate ? dx[e] + g : g;
  }
}
MER_API int mer_mean_pool_fwd(int B, int L, int D, const float* x, float* y, long ldy, void* stream) {
  hipLaunchKernelGGL(mean_pool_fwd_kernel, dim3((D + 63) / 64, B), dim3(256), 0, (hipStream_t)stream, B, L, D, x, y, ldy);
  MER_LAUNCH_CHECK();
}
MER_API int mer_mean_pool_bwd(int B, int L, int D, const float* dy, long lddy, float* dx, int accumulate, void* stream) {
  const long n = (long)B * L * D;
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(mean_pool_bwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, B, L, D, dy, lddy, dx, accumulate);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// Cross entropy with label smoothing (train.py:1033, mean reduction) fused with its gradient:
// loss = mean_b [(1-eps) * nll_b + eps * mean_c(-logp_bc)];  dlogits = (softmax - q) / B.
// late mode (train.py:212-214): inputs are probabilities p, loss = NLL(log(p + 1e-8)).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ bool argmax_better(float v, int i, float bv, int bi, int C) {
  if (i >= C) return false;
  if (bi >= C) return true;
  const bool vn = v != v, bn = bv != bv;
  if (vn != bn) return vn;
  if (vn) return i < bi;
  return v > bv || (v == bv && i < bi);
}
// One group of G lanes (G = pow2 >= C, at most 64; a lane loops over classes g, g + G, .. past that) per row, 256 / G
// rows in flight per pass: the rows' loads are issued together (one memory latency for B * C logits instead of B
// serial ones).  Per-row loss terms are summed in row order by thread 0 (deterministic).
template <int G>
__global__ __launch_bounds__(256) void ce_kernel(int B, int C, const float* __restrict__ logits,
                                                 const long long* __restrict__ labels, float eps_ls, int late,
                                                 float* __restrict__ loss, float* __restrict__ dlogits,
                                                 long long* __restrict__ preds) {
  constexpr int RPB = 256 / G;  // rows per pass
  __shared__ float rl[RPB];
  __shared__ float total;
  const int g = threadIdx.x % G, rg = threadIdx.x / G;
  if (threadIdx.x == 0) total = 0.f;
  for (int b0 = 0; b0 < B; b0 += RPB) {
    const int b = b0 + rg;
    const bool rv = b < B;
    const float* z = logits + (long)(rv ? b : B - 1) * C;
    const long long y = labels[rv ? b : B - 1];
    float term = 0.f;
    if (preds) {  // top-1 as torch.argmax: NaN counts as the maximum, the lowest index wins among equals
      float bv = 0.f;
      int bi = C;  // C = no candidate
      for (int c = g; c < C; c += G)
        if (argmax_better(z[c], c, bv, bi, C)) { bv = z[c]; bi = c; }
#pragma unroll
      for (int off = G / 2; off > 0; off >>= 1) {
        const float ov = __shfl_xor(bv, off, G);
        const int oi = __shfl_xor(bi, off, G);
        if (argmax_better(ov, oi, bv, bi, C)) { bv = ov; bi = oi; }
      }
      if (g == 0 && rv) preds[b] = bi < C ? bi : 0;
    }
    if (late) {
      for (int c = g; c < C; c += G) {
        const float pc = z[c];
        if (c == y) term += -logf(pc + 1e-8f);
        if (dlogits && rv) dlogits[(long)b * C + c] = (c == y) ? -1.0f / ((pc + 1e-8f) * B) : 0.f;
      }
#pragma unroll
      for (int off = G / 2; off > 0; off >>= 1) term += __shfl_xor(term, off, G);
    } else {
      float mx = -INFINITY;
      for (int c = g; c < C; c += G) mx = fmaxf(mx, z[c]);
#pragma unroll
      for (int off = G / 2; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, G));
      float se = 0.f, sz = 0.f, zy = 0.f;
      for (int c = g; c < C; c += G) {
        se += __expf(z[c] - mx);
        sz += z[c];
        if (c == y) zy = z[c];
      }
#pragma unroll
      for (int off = G / 2; off > 0; off >>= 1) {
        se += __shfl_xor(se, off, G);
        sz += __shfl_xor(sz, off, G);
        zy += __shfl_xor(zy, off, G);
      }
      const float lse = mx + logf(se);
      term = (1.f - eps_ls) * (lse - zy) + eps_ls * (lse - sz / C);
      if (dlogits && rv) {
        for (int c = g; c < C; c += G) {
          const float sm = __expf(z[c] - lse);
          const float q = (c == y ? 1.f - eps_ls : 0.f) + eps_ls / C;
          dlogits[(long)b * C + c] = (sm - q) / B;
        }
      }
    }
    if (g == 0) rl[rg] = rv ? term : 0.f;
    __syncthreads();
    if (threadIdx.x == 0) {
      float acc = total;
      for (int r = 0; r < RPB && b0 + r < B; ++r) acc += rl[r];
      total = acc;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = total / B;
}
MER_API int mer_cross_entropy(int B, int C, const float* logits, const long long* labels, float label_smoothing,
                              int late, float* loss, float* dlogits, long long* preds, void* stream) {
  if (B <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
#define MER_CE(G) hipLaunchKernelGGL(ce_kernel<G>, dim3(1), dim3(256), 0, st, B, C, logits, labels, label_smoothing, \
                                     late, loss, dlogits, preds)
  if (C <= 8) MER_CE(8);
  else if (C <= 16) MER_CE(16);
  else if (C <= 32) MER_CE(32);
  else MER_CE(64);
#undef MER_CE
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// RNG base of a training step (device-resident, see mer_site_seed in common.h)
// ---------------------------------------------------------------------------------------
__global__ void rng_advance_kernel(unsigned long long* state) {
  unsigned long long z = *state + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  *state = (z ^ (z >> 31)) & 0x3FFFFFFFFFFFFFFFull;
}
MER_API int mer_rng_advance(unsigned long long* state, void* stream) {
  hipLaunchKernelGGL(rng_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, state);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// Elementwise helpers
// ---------------------------------------------------------------------------------------
// y = x * s[0] (device scalar, e.g. autograd's grad_output of a 0-d loss)
__global__ void scale_dev_kernel(long n, const float* __restrict__ x, const float* __restrict__ s, float* __restrict__ y) {
  const float k = *s;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) y[e] = x[e] * k;
}
MER_API int mer_scale_dev(long n, const float* x, const float* s, float* y, void* stream) {
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(scale_dev_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, (hipStream_t)stream, n, x, s, y);
  MER_LAUNCH_CHECK();
}

// in-place dropout on rows with stride (nn.Dropout in train mode): x *= keep/(1-p)
__global__ void dropout_kernel(int rows, int cols, float* __restrict__ x, long ldx, float p, const unsigned long long* __restrict__ seed_ptr,
    unsigned long long site) {
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  const long n = (long)rows * cols;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int r = e / cols, c = e % cols;
    x[(long)r * ldx + c] *= dropout_scale(seed, e, p);
  }
}
MER_API int mer_dropout_inplace(int rows, int cols, float* x, long ldx, float p, const unsigned long long* seed, unsigned long long site, void* stream) {
  if (p <= 0.f) return 0;
  const long n = (long)rows * cols;
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(dropout_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, rows, cols, x, ldx, p, seed, site);
  MER_LAUNCH_CHECK();
}

// backward of y = dropout(relu(z)) given y: dz = dy * (y > 0) * drop_scale  (in place on dy)
__global__ void relu_dropout_bwd_kernel(int rows, int cols, float* __restrict__ dy, long lddy, const float* __restrict__ y,
                                        long ldy, float p, const unsigned long long* __restrict__ seed_ptr,
    unsigned long long site) {
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  const long n = (long)rows * cols;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int r = e / cols, c = e % cols;
    const float yy = y[(long)r * ldy + c];
    float g = dy[(long)r * lddy + c];
    g = yy > 0.f ? g * dropout_scale(seed, e, p) : 0.f;
    dy[(long)r * lddy + c] = g;
  }
}
MER_API int mer_relu_dropout_bwd(int rows, int cols, float* dy, long lddy, const float* y, long ldy, float p,
                                 const unsigned long long* seed, unsigned long long site, void* stream) {
  const long n = (long)rows * cols;
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(relu_dropout_bwd_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, (hipStream_t)stream, rows, cols,
                     dy, lddy, y, ldy, p, seed, site);
  MER_LAUNCH_CHECK();
}

// gated mix (fusion.py:408-411):  g = sigmoid(z[b]);  out = g*v + (1-g)*a
__global__ void gate_mix_fwd_kernel(int B, int D, const float* __restrict__ z, const float* __restrict__ v, long ldv,
                                    const float* __restrict__ a, long lda, float* __restrict__ out, float* __restrict__ g_out) {
  const int b = blockIdx.x;
  const float g = 1.f / (1.f + __expf(-z[b]));
  if (threadIdx.x == 0 && g_out) g_out[b] = g;
  for (int c = threadIdx.x; c < D; c += blockDim.x)
    out[(long)b * D + c] = g * v[(long)b * ldv + c] + (1.f - g) * a[(long)b * lda + c];
}
// dz = sum_c dout*(v-a) * g(1-g); dv = g*dout; da = (1-g)*dout  (dv/da accumulate into given buffers)
__global__ void gate_mix_bwd_kernel(int B, int D, const float* __restrict__ g_in, const float* __restrict__ v, long ldv,
                                    const float* __restrict__ a, long lda, const float* __restrict__ dout,
                                    float* __restrict__ dz, float* __restrict__ dv, long lddv, float* __restrict__ da,
                                    long ldda) {
  __shared__ float red[4];
  const int b = blockIdx.x;
  const float g = g_in[b];
  float s = 0.f;
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    const float d = dout[(long)b * D + c];
    s += d * (v[(long)b * ldv + c] - a[(long)b * lda + c]);
    dv[(long)b * lddv + c] += g * d;
    da[(long)b * ldda + c] += (1.f - g) * d;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) dz[b] = (red[0] + red[1] + red[2] + red[3]) * g * (1.f - g);
}
MER_API int mer_gate_mix_fwd(int B, int D, const float* z, const float* v, long ldv, const float* a, long lda,
                             float* out, float* g_out, void* stream) {
  hipLaunchKernelGGL(gate_mix_fwd_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, B, D, z, v, ldv, a, lda, out, g_out);
  MER_LAUNCH_CHECK();
}
MER_API int mer_gate_mix_bwd(int B, int D, const float* g, const float* v, long ldv, const float* a, long lda,
                             const float* dout, float* dz, float* dv, long lddv, float* da, long ldda, void* stream) {
  hipLaunchKernelGGL(gate_mix_bwd_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, B, D, g, v, ldv, a, lda, dout, dz,
                     dv, lddv, da, ldda);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// Emotion-prior token bias (fusion.py:170-176):
//   bias[b,i,j] = tanh(qt[b,i] + qp[b] + kt[b,j] + kp[b]) * scale
// where qt/kt are the token halves of query_head/key_head and qp/kp the prior halves (+bias).
// ---------------------------------------------------------------------------------------
__global__ void token_bias_fwd_kernel(int B, int Lq, int Lk, const float* __restrict__ qt, const float* __restrict__ qp,
                                      const float* __restrict__ kt, const float* __restrict__ kp,
                                      const float* __restrict__ scale, float* __restrict__ out) {
  const int b = blockIdx.y;
  const float s = *scale, base = qp[b] + kp[b];
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < Lq * Lk; e += gridDim.x * blockDim.x) {
    const int i = e / Lk, j = e % Lk;
    out[(long)b * Lq * Lk + e] = tanhf(qt[(long)b * Lq + i] + kt[(long)b * Lk + j] + base) * s;
  }
}
// g = dbias*scale*(1-tanh^2): dqt[b,i] = sum_j g, dkt[b,j] = sum_i g, dqp[b] = dkp[b] = sum g,
// dscale += sum dbias*tanh.  One workgroup per sample, deterministic.
__global__ __launch_bounds__(256) void token_bias_bwd_kernel(int B, int Lq, int Lk, const float* __restrict__ qt,
                                                             const float* __restrict__ qp, const float* __restrict__ kt,
                                                             const float* __restrict__ kp, const float* __restrict__ scale,
                                                             const float* __restrict__ dbias, float* __restrict__ dqt,
                                                             float* __restrict__ dkt, float* __restrict__ dqp,
                                                             float* __restrict__ dkp, float* __restrict__ dscale_part) {
  __shared__ float red[2][4];
  const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float s = *scale, base = qp[b] + kp[b];
  const float* db = dbias + (long)b * Lq * Lk;
  float tot = 0.f, dsc = 0.f;
  for (int i = w; i < Lq; i += 4) {
    float acc = 0.f;
    for (int j = lane; j < Lk; j += 64) {
      const float th = tanhf(qt[(long)b * Lq + i] + kt[(long)b * Lk + j] + base);
      const float d = db[(long)i * Lk + j];
      acc += d * s * (1.f - th * th);
      dsc += d * th;
    }
    acc = wave_sum(acc);
    if (lane == 0) dqt[(long)b * Lq + i] = acc;
    tot += lane == 0 ? acc : 0.f;
  }
  for (int j = threadIdx.x; j < Lk; j += 256) {
    float acc = 0.f;
    for (int i = 0; i < Lq; ++i) {
      const float th = tanhf(qt[(long)b * Lq + i] + kt[(long)b * Lk + j] + base);
      acc += db[(long)i * Lk + j] * s * (1.f - th * th);
    }
    dkt[(long)b * Lk + j] = acc;
  }
  tot = wave_sum(tot);
  dsc = wave_sum(dsc);
  if (lane == 0) { red[0][w] = tot; red[1][w] = dsc; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tt = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    dqp[b] = tt;
    dkp[b] = tt;
    dscale_part[b] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}
// Same sums with g staged once in LDS (Lq*Lk <= TB_LDS): row sums per wave, column sums per thread from LDS --
// the global-memory version walks a 149-long dependent column loop per thread (a2v: 32 us).
constexpr int TB_LDS = 4096;
__global__ __launch_bounds__(256) void token_bias_bwd_lds_kernel(int B, int Lq, int Lk, const float* __restrict__ qt,
                                                                 const float* __restrict__ qp, const float* __restrict__ kt,
                                                                 const float* __restrict__ kp, const float* __restrict__ scale,
                                                                 const float* __restrict__ dbias, float* __restrict__ dqt,
                                                                 float* __restrict__ dkt, float* __restrict__ dqp,
                                                                 float* __restrict__ dkp, float* __restrict__ dscale_part) {
  __shared__ float gs[TB_LDS];
  __shared__ float red[2][4];
  const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float s = *scale, base = qp[b] + kp[b];
  const float* db = dbias + (long)b * Lq * Lk;
  float dsc = 0.f;
  for (int e = threadIdx.x; e < Lq * Lk; e += 256) {
    const int i = e / Lk, j = e - i * Lk;
    const float th = tanhf(qt[(long)b * Lq + i] + kt[(long)b * Lk + j] + base);
    const float d = db[e];
    gs[e] = d * s * (1.f - th * th);
    dsc += d * th;
  }
  __syncthreads();
  float tot = 0.f;
  for (int i = w; i < Lq; i += 4) {
    float acc = 0.f;
    for (int j = lane; j < Lk; j += 64) acc += gs[i * Lk + j];
    acc = wave_sum(acc);
    if (lane == 0) dqt[(long)b * Lq + i] = acc;
    tot += lane == 0 ? acc : 0.f;
  }
  for (int j = threadIdx.x; j < Lk; j += 256) {
    float a0 = 0.f, a1 = 0.f;
    int i = 0;
    for (; i + 2 <= Lq; i += 2) {
      a0 += gs[i * Lk + j];
      a1 += gs[(i + 1) * Lk + j];
    }
    if (i < Lq) a0 += gs[i * Lk + j];
    dkt[(long)b * Lk + j] = a0 + a1;
  }
  tot = wave_sum(tot);
  dsc = wave_sum(dsc);
  if (lane == 0) { red[0][w] = tot; red[1][w] = dsc; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tt = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    dqp[b] = tt;
    dkp[b] = tt;
    dscale_part[b] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}
MER_API int mer_token_bias_fwd(int B, int Lq, int Lk, const float* qt, const float* qp, const float* kt, const float* kp,
                               const float* scale, float* out, void* stream) {
  dim3 grid((Lq * Lk + 255) / 256, B);
  hipLaunchKernelGGL(token_bias_fwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, B, Lq, Lk, qt, qp, kt, kp, scale, out);
  MER_LAUNCH_CHECK();
}
MER_API int mer_token_bias_bwd(int B, int Lq, int Lk, const float* qt, const float* qp, const float* kt, const float* kp,
                               const float* scale, const float* dbias, float* dqt, float* dkt, float* dqp, float* dkp,
                               float* dscale_part, void* stream) {
  if ((long)Lq * Lk <= TB_LDS)
    hipLaunchKernelGGL(token_bias_bwd_lds_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, B, Lq, Lk, qt, qp, kt, kp,
                       scale, dbias, dqt, dkt, dqp, dkp, dscale_part);
  else
    hipLaunchKernelGGL(token_bias_bwd_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, B, Lq, Lk, qt, qp, kt, kp,
                       scale, dbias, dqt, dkt, dqp, dkp, dscale_part);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// Sum of a small vector into a scalar (deterministic single-block reduce), optional accumulate.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void vec_sum_kernel(int n, const float* __restrict__ x, float* __restrict__ out, int acc) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += x[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float v = red[0] + red[1] + red[2] + red[3];
    *out = acc ? *out + v : v;
  }
}
MER_API int mer_vec_sum(int n, const float* x, float* out, int accumulate, void* stream) {
  hipLaunchKernelGGL(vec_sum_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, n, x, out, accumulate);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// Fused Adam over one flat fp32 buffer (torch.optim.Adam semantics, train.py:872,902):
//   g += wd*p; m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
// HBM-bound: 16 B read + 12 B written per parameter... vectorised 4-wide.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void adam_kernel(long n, float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, float lr, float b1,
                                                   float b2, float eps, float wd, float bc1, float bc2_sqrt,
                                                   float gscale) {
  const long n4 = n / 4;
  const float step = lr / bc1;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n4; e += (long)gridDim.x * blockDim.x) {
    float4 pp = reinterpret_cast<float4*>(p)[e];
    const float4 gg = reinterpret_cast<const float4*>(g)[e];
    float4 mm = reinterpret_cast<float4*>(m)[e];
    float4 vv = reinterpret_cast<float4*>(v)[e];
#define ADAM1(c)                                                  \
  {                                                               \
    const float gr = gscale * gg.c + wd * pp.c;                   \
    mm.c = b1 * mm.c + (1.f - b1) * gr;                           \
    vv.c = b2 * vv.c + (1.f - b2) * gr * gr;                      \
    pp.c -= step * mm.c / (sqrtf(vv.c) / bc2_sqrt + eps);         \
  }
    ADAM1(x) ADAM1(y) ADAM1(z) ADAM1(w)
#undef ADAM1
    reinterpret_cast<float4*>(p)[e] = pp;
    reinterpret_cast<float4*>(m)[e] = mm;
    reinterpret_cast<float4*>(v)[e] = vv;
  }
  for (long e = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const float gr = gscale * g[e] + wd * p[e];
    m[e] = b1 * m[e] + (1.f - b1) * gr;
    v[e] = b2 * v[e] + (1.f - b2) * gr * gr;
    p[e] -= step * m[e] / (sqrtf(v[e]) / bc2_sqrt + eps);
  }
}
MER_API int mer_adam_step(long n, float* p, const float* g, float* m, float* v, float lr, float b1, float b2, float eps,
                          float wd, int step, float grad_scale, void* stream) {
  if (n <= 0) return 0;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return (int)hipErrorInvalidValue;
  const float bc1 = 1.f - powf(b1, (float)step);
  const float bc2s = sqrtf(1.f - powf(b2, (float)step));
  const long n4 = (n + 3) / 4;
  const int grid = (int)((n4 + 255) / 256 < 2048 ? (n4 + 255) / 256 : 2048);
  hipLaunchKernelGGL(adam_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, n, p, g, m, v, lr, b1, b2, eps, wd,
                     bc1, bc2s, grad_scale);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// late fusion (fusion.py:358-363): out = (softmax(za) + softmax(zv)) / 2, one wave per row.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void softmax_row(const float* z, float* p, int C, int lane) {
  float mx = -INFINITY;
  for (int c = lane; c < C; c += 64) mx = fmaxf(mx, z[c]);
  mx = wave_max(mx);
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += __expf(z[c] - mx);
  s = wave_sum(s);
  for (int c = lane; c < C; c += 64) p[c] = __expf(z[c] - mx) / s;
}
__global__ void softmax_avg_fwd_kernel(int B, int C, const float* __restrict__ za, const float* __restrict__ zv,
                                       float* __restrict__ out, float* __restrict__ pa, float* __restrict__ pv) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= B) return;
  softmax_row(za + (long)b * C, pa + (long)b * C, C, lane);
  softmax_row(zv + (long)b * C, pv + (long)b * C, C, lane);
  __builtin_amdgcn_wave_barrier();
  for (int c = lane; c < C; c += 64) out[(long)b * C + c] = 0.5f * (pa[(long)b * C + c] + pv[(long)b * C + c]);
}
__global__ void softmax_avg_bwd_kernel(int B, int C, const float* __restrict__ pa, const float* __restrict__ pv,
                                       const float* __restrict__ dout, float* __restrict__ da, float* __restrict__ dv) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= B) return;
  const float* g = dout + (long)b * C;
  float sa = 0.f, sv = 0.f;
  for (int c = lane; c < C; c += 64) { sa += pa[(long)b * C + c] * g[c]; sv += pv[(long)b * C + c] * g[c]; }
  sa = wave_sum(sa);
  sv = wave_sum(sv);
  for (int c = lane; c < C; c += 64) {
    da[(long)b * C + c] = 0.5f * pa[(long)b * C + c] * (g[c] - sa);
    dv[(long)b * C + c] = 0.5f * pv[(long)b * C + c] * (g[c] - sv);
  }
}
MER_API int mer_softmax_avg_fwd(int B, int C, const float* za, const float* zv, float* out, float* pa, float* pv,
                                void* stream) {
  hipLaunchKernelGGL(softmax_avg_fwd_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, B, C, za, zv, out, pa, pv);
  MER_LAUNCH_CHECK();
}
MER_API int mer_softmax_avg_bwd(int B, int C, const float* pa, const float* pv, const float* dout, float* da, float* dv,
                                void* stream) {
  hipLaunchKernelGGL(softmax_avg_bwd_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, B, C, pa, pv, dout, da, dv);
  MER_LAUNCH_CHECK();
}
