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
  int vec_epi;  // pipelined kernels: 16-byte epilogue through LDS (N, ldc, ldr, c_zoff multiples of 8, aligned)
  // train-mode extras (mer_gemm_bf16_tr): dropout after the activation, before the residual (nn.Dropout of
  // WavLM's attention output / FFN, TF:286-294,323), mask index = row * N + col; and LayerDrop: the whole
  // launch is a no-op when bit skip_bit of *skip_mask is set (TF:417-419)
  float drop_p;
  const unsigned long long* drop_seed;
  unsigned long long drop_site;
  const long long* skip_mask;
  int skip_bit;
  // K-step order of overlapping-rows (convolution) A operands: K = kp_taps taps x kp_c channels; K-tile u reads
  // tap u % kp_taps of channel block u / kp_taps, so the taps that re-read the same input rows (stride < taps)
  // run back to back and hit L2 instead of re-fetching from HBM.  kp_taps = 0: natural order.
  int kp_taps, kp_c;
  // row bands of the XCD-grouped tile order (xcd_tile_grouped); 1 = plain row-major chunks, so the N-tiles of one
  // row panel run back to back on one XCD and share the A panel through its L2
  int tgroup;
};

// element offset of K-tile u (64 wide) in the K dimension
__device__ __forceinline__ int ktile_off(const GemmArgs& g, int u) {
  if (g.kp_taps <= 1) return u * 64;
  const int cb = u / g.kp_taps, tap = u - cb * g.kp_taps;
  return tap * g.kp_c + cb * 64;
}

__device__ __forceinline__ bool layer_skipped(const long long* mask, int bit) {
  return mask != nullptr && ((*mask >> bit) & 1ll);
}
// act -> dropout (train mode) of one epilogue element
__device__ __forceinline__ float epi_act_drop(float v, int act, float p, unsigned long long seed, long idx) {
  v = apply_act(v, act);
  return p > 0.f ? v * dropout_scale_pair(seed, (uint64_t)idx, p) : v;
}

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

template <typename T> __device__ __forceinline__ void store8(T* p, const float* v);
template <> __device__ __forceinline__ void store8<float>(float* p, const float* v) {
  *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4*>(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
}
template <> __device__ __forceinline__ void store8<bf16_t>(bf16_t* p, const float* v) {
  uint32_t w[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) w[e] = (uint32_t)f2bf(v[2 * e]) | ((uint32_t)f2bf(v[2 * e + 1]) << 16);
  *reinterpret_cast<u32x4*>(p) = u32x4{w[0], w[1], w[2], w[3]};
}

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
  if (layer_skipped(g.skip_mask, g.skip_bit)) return;
  const unsigned long long dseed = mer_site_seed(g.drop_seed, g.drop_site);
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
        float v = epi_act_drop(acc[i][j][r] + bv, g.act, g.drop_p, dseed, (long)row * g.N + col);
        if (g.R) v += bf2f(g.R[(long)row * g.ldr + (long)z * g.c_zoff + col]);
        stf<TOUT>(C, (long)row * g.ldc + col, v);
      }
    }
}


// ---------------------------------------------------------------------------------------------
// Pipelined variant (K % 64 == 0, mode 0): global_load_lds (16 B per lane) straight into a
// double-buffered LDS image, next K-tile issued BEFORE the current one is consumed, one
// vmcnt(0) + barrier per K-tile (cdna_hip_programming.md §5 "Minimum 2-phase").
// LDS image per operand: [rows][64 bf16] = 128-byte rows of eight 16-byte chunks; chunk c of
// row r lives at physical chunk c ^ ((r >> 1) & 7), so the 16 rows one ds_read_b128 lane group
// touches (same logical chunk) cover all sixteen 16-byte bank slots of a 256-byte bank row.
// glds writes lane-linear (base + 16*lane), so the XOR goes on each lane's SOURCE address and on
// the fragment read (rule 21: both sides).  Rows past M/N are clamped to the last valid row (their
// outputs are discarded); K is a multiple of 64, so no K tail.
template <int BM_, int BN_, int WM_, int WN_, int STAGES_ = 2, int KS_ = 64, int SA_ = 0, int SW_ = 0, int IL_ = 0>
struct PipeCfg {
  // IL (split ring only): the K-step's LDS-DMA issue goes between the first substep's MFMA rows instead of ahead of
  // the fragment reads, so its issue cost runs under the SIMD's MFMAs rather than in front of them
  static constexpr bool IL = IL_ != 0;
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;       // tile, waves along M / N
  // SW: operand-swapped MFMA (W fragment as the A operand): a lane's accumulator quad is then 4 consecutive COLUMNS
  // of one row, which the staged epilogue writes to LDS as one 16-byte fp32 or 8-byte bf16 vector
  static constexpr bool SW = SW_ != 0;
  static constexpr int STAGES = STAGES_;                            // LDS ring depth (K-tiles)
  // SA > 0: the A operand gets its own, deeper ring (SA = 3 with a 2-deep B ring): A is the HBM stream of the
  // conv-as-GEMMs (B, the weights, stays L2-resident), so A tiles are issued two K-steps ahead, B tiles one
  static constexpr int SA = SA_ > 0 ? SA_ : STAGES_, SB = STAGES_;
  static constexpr int LDS_ELEMS = SA * BM * KS_ + SB * BN * KS_;   // bf16 elements of the whole ring
  static constexpr int KS = KS_;                                    // K-tile width (64, or 32 for deep rings)
  static constexpr int CW = KS / 8, RPG = 64 / CW;                  // 16-byte chunks per LDS row, rows per glds
  static constexpr int WAVES = WM * WN, NT = 64 * WAVES;
  static constexpr int TM = BM / WM, TN = BN / WN;                  // per-wave output
  static constexpr int FM = TM / 16, FN = TN / 16;                  // 16x16 fragments per wave
  static constexpr int IA = BM / RPG / WAVES, IB = BN / RPG / WAVES;  // glds per wave per K-tile
  static constexpr int BUF = (BM + BN) * KS;                        // bf16 elements per LDS buffer
  static_assert(IA * RPG * WAVES == BM && IB * RPG * WAVES == BN, "tile rows must split into whole glds pieces");
  static_assert(KS == 64 || KS == 32, "K-tile");
};

__device__ __forceinline__ int swz_chunk(int row, int c) { return c ^ ((row >> 1) & 7); }
// CW chunks per row: 8 (128-byte rows) or 4 (64-byte rows: four rows share a 256-byte bank row, XOR by row bits 2-3)
template <int CW>
__device__ __forceinline__ int swz_k(int row, int c) {
  return CW == 8 ? (c ^ ((row >> 1) & 7)) : (c ^ ((row >> 2) & 3));
}
// element offset of K-tile u of width KS (the 32-wide tiles walk the 64-wide order in halves)
template <int KS>
__device__ __forceinline__ int ktile_off_k(const GemmArgs& g, int u) {
  return KS == 64 ? ktile_off(g, u) : ktile_off(g, u >> 1) + (u & 1) * 32;
}


// Phase timestamps of the pipelined GEMM (tools/gemm_phases.py builds a separate library with
// -DMER_GEMM_TIMING; the production library compiles GT() to nothing): wall_clock64() of workgroup blockIdx.x's
// thread 0 at phase k.
#ifdef MER_GEMM_TIMING
static __device__ long long mer_gt_buf[1024 * 8];
#define GT(k) \
  do { \
    if (threadIdx.x == 0 && blockIdx.x < 1024 && blockIdx.z == 0) mer_gt_buf[blockIdx.x * 8 + (k)] = wall_clock64(); \
  } while (0)
// shader-clock stamp (s_memtime, cycles at the in-kernel clock) beside GT(k): slot k + 4 (k = 1, 2 only)
#define GTC(k) \
  do { \
    if (threadIdx.x == 0 && blockIdx.x < 1024 && blockIdx.z == 0) \
      mer_gt_buf[blockIdx.x * 8 + 4 + (k)] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)
MER_API int mer_gt_reset() {
  static long long zeros[1024 * 8];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(mer_gt_buf), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice);
}
MER_API int mer_gt_read(long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(mer_gt_buf), sizeof(long long) * 1024 * 8, 0,
                                  hipMemcpyDeviceToHost);
}
#else
#define GT(k) \
  do { \
  } while (0)
#define GTC(k) \
  do { \
  } while (0)
#endif

__device__ __attribute__((aligned(16))) uint32_t mer_gemm_zero16[4] = {0u, 0u, 0u, 0u};

// AMODE 0: rows mode; AMODE 1: grouped positional conv (group = blockIdx.z), A chunks gathered per
// K-tile from x[b, t + tap - pad, z*cg + c] with out-of-range taps served from a zero chunk.
template <class CF, typename TOUT, int AMODE>
__global__ __launch_bounds__(CF::NT, 1) void gemm_pipe_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  if (layer_skipped(g.skip_mask, g.skip_bit)) return;
  GT(0);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int z = blockIdx.z;
  const int nx = (g.N + CF::BN - 1) / CF::BN, ny = (g.M + CF::BM - 1) / CF::BM;
  int tx, ty;
  xcd_tile_grouped(blockIdx.x, nx, ny, g.tgroup, tx, ty);
  const int m0 = ty * CF::BM, n0 = tx * CF::BN;
  const int wr = w / CF::WN, wc = w % CF::WN;

  // per-lane source pointers (fixed over K; advanced by 64 elements per K-tile)
  const bf16_t* pa[CF::IA];
  const bf16_t* pb[CF::IB];
  int at[CF::IA], acl[CF::IA];  // AMODE 1: the row's time index and logical chunk
  const int lrow = lane / CF::CW, lchunk = lane % CF::CW;
#pragma unroll
  for (int j = 0; j < CF::IA; ++j) {
    const int r = (w * CF::IA + j) * CF::RPG + lrow;
    int m = m0 + r;
    m = m < g.M ? m : g.M - 1;
    if (AMODE == 0) {
      pa[j] = g.A + (long)(m / g.a_rpg) * g.a_gstride + (long)(m % g.a_rpg) * g.a_rstride + swz_k<CF::CW>(r, lchunk) * 8;
    } else {
      const int b = m / g.pc_L;
      at[j] = m - b * g.pc_L;
      acl[j] = swz_k<CF::CW>(r, lchunk) * 8;
      pa[j] = g.A + (long)b * g.pc_L * g.pc_ldx + (long)z * g.pc_cg;
    }
  }
  const bf16_t* Bz = g.B + (long)z * g.b_zstride;
#pragma unroll
  for (int j = 0; j < CF::IB; ++j) {
    const int r = (w * CF::IB + j) * CF::RPG + lrow;
    int n = n0 + r;
    n = n < g.N ? n : g.N - 1;
    pb[j] = Bz + (long)n * g.ldb + swz_k<CF::CW>(r, lchunk) * 8;
  }
  const float inv_cg = AMODE == 1 ? 1.f / g.pc_cg : 0.f;
  auto stage_a = [&](bf16_t* la, int k0) {
#pragma unroll
    for (int j = 0; j < CF::IA; ++j) {
      if (AMODE == 0) {
        glds16(pa[j] + k0, la + (w * CF::IA + j) * 512);
      } else {
        const int k = k0 + acl[j];
        const int tap = fdiv(k, inv_cg), c = k - tap * g.pc_cg;
        const int src = at[j] + tap - g.pc_pad;
        const bool ok = src >= 0 && src < g.pc_L;
        glds16(ok ? pa[j] + (long)src * g.pc_ldx + c : reinterpret_cast<const bf16_t*>(mer_gemm_zero16),
               la + (w * CF::IA + j) * 512);
      }
    }
  };
  auto stage_b = [&](bf16_t* lb, int k0) {
#pragma unroll
    for (int j = 0; j < CF::IB; ++j)
      glds16(pb[j] + k0, lb + (w * CF::IB + j) * 512);
  };
  auto stage = [&](int buf, int k0) {
    bf16_t* la = smem + buf * CF::BUF;
    stage_a(la, k0);
    stage_b(la + CF::BM * CF::KS, k0);
  };

  f32x4 acc[CF::FM][CF::FN];
#pragma unroll
  for (int i = 0; i < CF::FM; ++i)
#pragma unroll
    for (int j = 0; j < CF::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (elements) inside one operand image, per k-step s: row*64 + phys_chunk*8
  const int fr = lane & 15, fq = lane >> 4;
  const int nk = g.K / CF::KS;
  constexpr int S = CF::STAGES, G = CF::IA + CF::IB;
  static_assert(S >= 2 && S <= 4 && (S - 2) * G < 64, "ring depth");
  // Ring of S LDS buffers: tiles kt+1 .. kt+S-2 stay in flight (counted vmcnt) across the barrier
  // that publishes tile kt; the barrier also retires every wave's reads of tile kt-1, whose buffer
  // the tile kt+S-1 DMA then reuses.  Raw s_barrier: __syncthreads() would drain vmcnt to 0.
  // split rings (SA = 3, SB = 2): A tiles at smem + (k % 3) * BM*KS, B tiles after the A ring at (k % 2) * BN*KS.
  // Issue order: prologue A(0) B(0) A(1); step kt issues B(kt+1) then A(kt+2), so when step kt starts the
  // youngest group is A(kt+1), issued after B(kt): vmcnt(IA) leaves exactly it in flight.  A(kt+2) reuses the
  // buffer of A(kt-1) and B(kt+1) that of B(kt-1), both read in step kt-1, before this step's barrier.
  constexpr bool SPLIT = CF::SA != CF::SB;
  static_assert(!SPLIT || (CF::SA == 3 && CF::SB == 2), "split ring: SA = 3, SB = 2");
  bf16_t* const ring_b = smem + CF::SA * CF::BM * CF::KS;
  if constexpr (SPLIT) {
    stage_a(smem, ktile_off_k<CF::KS>(g, 0));
    stage_b(ring_b, ktile_off_k<CF::KS>(g, 0));
    if (nk > 1) stage_a(smem + CF::BM * CF::KS, ktile_off_k<CF::KS>(g, 1));
  } else {
#pragma unroll
    for (int p = 0; p < S - 1; ++p)
      if (p < nk) stage(p, ktile_off_k<CF::KS>(g, p));
  }
  for (int kt = 0; kt < nk; ++kt) {
    if constexpr (SPLIT) {
      if (kt + 1 < nk) wait_vmcnt<CF::IA>(); else wait_vmcnt<0>();
    } else {
      const int ahead = (nk - 1 - kt) < (S - 2) ? (nk - 1 - kt) : (S - 2);
      wait_tiles_in_flight<G>(ahead);
    }
    __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));  // lgkmcnt(0) only
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt == 0) {
      GT(1);
      GTC(1);
    }
    const bf16_t* la;
    const bf16_t* lb;
    if constexpr (SPLIT) {
      if constexpr (!CF::IL) {
        if (kt + 1 < nk) stage_b(ring_b + ((kt + 1) & 1) * CF::BN * CF::KS, ktile_off_k<CF::KS>(g, kt + 1));
        if (kt + 2 < nk) stage_a(smem + ((kt + 2) % 3) * CF::BM * CF::KS, ktile_off_k<CF::KS>(g, kt + 2));
      }
      la = smem + (kt % 3) * CF::BM * CF::KS;
      lb = ring_b + (kt & 1) * CF::BN * CF::KS;
    } else {
      if (kt + S - 1 < nk) stage((kt + S - 1) % S, ktile_off_k<CF::KS>(g, kt + S - 1));
      la = smem + (kt % S) * CF::BUF;
      lb = la + CF::BM * CF::KS;
    }
#pragma unroll
    for (int s = 0; s < CF::KS / 32; ++s) {
      bf16x8 af[CF::FM], bfr[CF::FN];
#pragma unroll
      for (int i = 0; i < CF::FM; ++i) {
        const int r = wr * CF::TM + i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(la + r * CF::KS + swz_k<CF::CW>(r, s * 4 + fq) * 8);
      }
#pragma unroll
      for (int j = 0; j < CF::FN; ++j) {
        const int r = wc * CF::TN + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(lb + r * CF::KS + swz_k<CF::CW>(r, s * 4 + fq) * 8);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < CF::FM; ++i) {
#pragma unroll
        for (int j = 0; j < CF::FN; ++j)
          acc[i][j] = CF::SW ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0)
                             : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        if constexpr (CF::IL && SPLIT) {
          // same pieces, same issue order (B(kt+1) then A(kt+2)) as the non-interleaved ring: the vmcnt
          // bookkeeping at the top of the next step is unchanged
          if (s == 0 && i == 0 && kt + 1 < nk) {
            __builtin_amdgcn_sched_barrier(0);
            stage_b(ring_b + ((kt + 1) & 1) * CF::BN * CF::KS, ktile_off_k<CF::KS>(g, kt + 1));
            __builtin_amdgcn_sched_barrier(0);
          }
          if (s == 0 && i == 1 && kt + 2 < nk) {
            __builtin_amdgcn_sched_barrier(0);
            stage_a(smem + ((kt + 2) % 3) * CF::BM * CF::KS, ktile_off_k<CF::KS>(g, kt + 2));
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
      __builtin_amdgcn_s_setprio(0);
    }
  }

  GTC(2);
  GT(2);
  TOUT* C = reinterpret_cast<TOUT*>(g.C) + (long)z * g.c_zoff;
  const unsigned long long dseed = mer_site_seed(g.drop_seed, g.drop_site);
  if constexpr (CF::SW) {
    if (g.vec_epi) {
      // Operand-swapped epilogue: a lane holds row i*16 + fr, columns j*16 + fq*4 .. +3 of each fragment.  Without
      // residual or dropout on a bf16 output the result bf16(act(acc + bias)) is rounded before staging: 8-byte
      // writes of [row][TN + 8] bf16 (half the LDS bytes of the fp32 image, the whole sub-tile in one pass); else
      // act(acc + bias) is staged as fp32 [row][TN + 4], one 16-byte write per fragment, and the residual /
      // dropout pass below is the unswapped one.  Same arithmetic and rounding as the direct path.
      constexpr int WAVE_FLOATS = CF::LDS_ELEMS / 2 / CF::WAVES;
      constexpr int LPR = CF::TN / 8, RPP = 64 / LPR;
      // the lane's bias quads, loaded before the barrier that waits for the slowest wave's last MFMAs (their
      // latency was exposed at the first staging write); N % 8 == 0 here, so a quad is all in or all out
      // (bf16 outputs only: the fp32-output instantiation has no registers to spare and loads them per block j)
      constexpr bool PRE = std::is_same<TOUT, bf16_t>::value;
      f32x4 bq4[CF::FN];
      auto bias_quad = [&](int j) {
        const int col = n0 + wc * CF::TN + j * 16 + fq * 4;
        f32x4 q = f32x4{0.f, 0.f, 0.f, 0.f};
        if (g.bias && col < g.N) {
          const float* bp = g.bias + (long)z * g.c_zoff + col;
          q = f32x4{bp[0], bp[1], bp[2], bp[3]};
        }
        return q;
      };
      if constexpr (PRE) {
#pragma unroll
        for (int j = 0; j < CF::FN; ++j) bq4[j] = bias_quad(j);
      }
      __syncthreads();
      GT(4);
      auto bias4 = [&](int j, float* bq) {
        const f32x4 q = PRE ? bq4[j] : bias_quad(j);
#pragma unroll
        for (int e = 0; e < 4; ++e) bq[e] = q[e];
      };
      const int lr = lane / LPR, lc = (lane % LPR) * 8;
      const int colv = n0 + wc * CF::TN + lc;
      if (std::is_same<TOUT, bf16_t>::value && !g.R && !(g.drop_p > 0.f)) {
        constexpr int LDH = CF::TN + 8;
        constexpr int GH0 = 2 * WAVE_FLOATS / (16 * LDH);
        constexpr int GH = GH0 < CF::FM ? GH0 : CF::FM;
        static_assert(GH >= 1, "epilogue staging slice too small");
        bf16_t* hl = reinterpret_cast<bf16_t*>(smem) + w * 2 * WAVE_FLOATS;
#pragma unroll
        for (int i0 = 0; i0 < CF::FM; i0 += GH) {
#pragma unroll
          for (int j = 0; j < CF::FN; ++j) {
            float bq[4];
            bias4(j, bq);
#pragma unroll
            for (int ii = 0; ii < GH; ++ii) {
              if (i0 + ii >= CF::FM) break;
              uint32_t q[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) q[e] = (uint32_t)f2bf(apply_act(acc[i0 + ii][j][e] + bq[e], g.act));
              *reinterpret_cast<uint2*>(&hl[(ii * 16 + fr) * LDH + j * 16 + fq * 4]) =
                  make_uint2(q[0] | (q[1] << 16), q[2] | (q[3] << 16));
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          const int nrows = (CF::FM - i0 < GH ? CF::FM - i0 : GH) * 16;
#pragma unroll
          for (int rr = 0; rr < GH * 16; rr += RPP) {
            const int rl = rr + lr;
            const int row = m0 + wr * CF::TM + i0 * 16 + rl;
            if (rl < nrows && row < g.M && colv < g.N)
              *reinterpret_cast<u32x4*>(C + (long)row * g.ldc + colv) = *reinterpret_cast<const u32x4*>(&hl[rl * LDH + lc]);
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        GT(3);
        return;
      }
      constexpr int LDT = CF::TN + 4;
      constexpr int GI0 = WAVE_FLOATS / (16 * LDT);
      constexpr int GI = GI0 < CF::FM ? GI0 : CF::FM;
      static_assert(GI >= 1, "epilogue staging slice too small");
      float* wl = reinterpret_cast<float*>(smem) + w * WAVE_FLOATS;
#pragma unroll
      for (int i0 = 0; i0 < CF::FM; i0 += GI) {
        constexpr int NRR = (GI * 16 + RPP - 1) / RPP;
        u32x4 rres[NRR];
        if (g.R) {
#pragma unroll
          for (int q = 0; q < NRR; ++q) {
            const int row = m0 + wr * CF::TM + i0 * 16 + q * RPP + lr;
            const long rr = row < g.M ? row : g.M - 1;
            rres[q] = *reinterpret_cast<const u32x4*>(g.R + rr * g.ldr + (long)z * g.c_zoff + (colv < g.N ? colv : 0));
          }
        }
#pragma unroll
        for (int j = 0; j < CF::FN; ++j) {
          float bq[4];
          bias4(j, bq);
#pragma unroll
          for (int ii = 0; ii < GI; ++ii) {
            if (i0 + ii >= CF::FM) break;
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = apply_act(acc[i0 + ii][j][e] + bq[e], g.act);
            *reinterpret_cast<f32x4*>(&wl[(ii * 16 + fr) * LDT + j * 16 + fq * 4]) = v;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int nrows = (CF::FM - i0 < GI ? CF::FM - i0 : GI) * 16;
#pragma unroll
        for (int rr = 0; rr < GI * 16; rr += RPP) {
          const int rl = rr + lr;
          const int row = m0 + wr * CF::TM + i0 * 16 + rl;
          if (rl < nrows && row < g.M && colv < g.N) {
            const f32x4 lo = *reinterpret_cast<const f32x4*>(&wl[rl * LDT + lc]);
            const f32x4 hi = *reinterpret_cast<const f32x4*>(&wl[rl * LDT + lc + 4]);
            float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            if (g.drop_p > 0.f) dropout_pairs<8>(v, dseed, (uint64_t)((long)row * g.N + colv), g.drop_p);
            if (g.R) {
              const u32x4 rv = rres[rr / RPP];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                v[2 * e] += __uint_as_float(rv[e] << 16);
                v[2 * e + 1] += __uint_as_float(rv[e] & 0xffff0000u);
              }
            }
            store8<TOUT>(C + (long)row * g.ldc + colv, v);
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      GT(3);
      return;
    }
  }
  if (g.vec_epi) {
    // Epilogue through LDS (the ring is idle once every wave is past its last fragment read): each wave
    // stages act(acc + bias) of 16-row groups of its TM x TN sub-tile as fp32 [row][TN + 4] in its own slice
    // of the ring (conflict-free: the 4 row-quads of a fragment land 16 banks apart), then every lane moves
    // 8 consecutive columns of one row: a 16-byte residual load and 16-byte (bf16) / 2 x 16-byte (fp32)
    // stores instead of one 2- or 4-byte access per accumulator element.  Same arithmetic and rounding as
    // the direct path below.
    constexpr int LDT = CF::TN + 4;
    constexpr int WAVE_FLOATS = CF::LDS_ELEMS / 2 / CF::WAVES;  // bf16 ring elements / 2 = floats
    constexpr int GI0 = WAVE_FLOATS / (16 * LDT);
    constexpr int GI = GI0 < CF::FM ? GI0 : CF::FM;
    static_assert(GI >= 1, "epilogue staging slice too small");
    constexpr int LPR = CF::TN / 8, RPP = 64 / LPR;  // lanes per row, rows per pass
    float bv[CF::FN];  // loaded before the barrier: its wait for the slowest wave covers their latency
#pragma unroll
    for (int j = 0; j < CF::FN; ++j) {
      const int col = n0 + wc * CF::TN + j * 16 + fr;
      bv[j] = (g.bias && col < g.N) ? g.bias[(long)z * g.c_zoff + col] : 0.f;
    }
    __syncthreads();
    GT(4);
    float* wl = reinterpret_cast<float*>(smem) + w * WAVE_FLOATS;
    const int lr = lane / LPR, lc = (lane % LPR) * 8;
    const int colv = n0 + wc * CF::TN + lc;
#pragma unroll
    for (int i0 = 0; i0 < CF::FM; i0 += GI) {
      // this pass's residual vectors first: their latency overlaps the staging writes (a load inside the store
      // loop exposed it once per row group)
      constexpr int NRR = (GI * 16 + RPP - 1) / RPP;
      u32x4 rres[NRR];
      if (g.R) {
#pragma unroll
        for (int q = 0; q < NRR; ++q) {
          const int row = m0 + wr * CF::TM + i0 * 16 + q * RPP + lr;
          const long rr = row < g.M ? row : g.M - 1;
          rres[q] = *reinterpret_cast<const u32x4*>(g.R + rr * g.ldr + (long)z * g.c_zoff + (colv < g.N ? colv : 0));
        }
      }
#pragma unroll
      for (int ii = 0; ii < GI; ++ii) {
        if (i0 + ii >= CF::FM) break;
#pragma unroll
        for (int j = 0; j < CF::FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            wl[(ii * 16 + fq * 4 + r) * LDT + j * 16 + fr] = apply_act(acc[i0 + ii][j][r] + bv[j], g.act);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int nrows = (CF::FM - i0 < GI ? CF::FM - i0 : GI) * 16;
#pragma unroll
      for (int rr = 0; rr < GI * 16; rr += RPP) {
        const int rl = rr + lr;
        const int row = m0 + wr * CF::TM + i0 * 16 + rl;
        if (rl < nrows && row < g.M && colv < g.N) {
          const f32x4 lo = *reinterpret_cast<const f32x4*>(&wl[rl * LDT + lc]);
          const f32x4 hi = *reinterpret_cast<const f32x4*>(&wl[rl * LDT + lc + 4]);
          float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          if (g.drop_p > 0.f)  // N % 8 == 0 on this path: the 8 indices start even
            dropout_pairs<8>(v, dseed, (uint64_t)((long)row * g.N + colv), g.drop_p);
          if (g.R) {
            const u32x4 rv = rres[rr / RPP];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[2 * e] += __uint_as_float(rv[e] << 16);
              v[2 * e + 1] += __uint_as_float(rv[e] & 0xffff0000u);
            }
          }
          store8<TOUT>(C + (long)row * g.ldc + colv, v);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    GT(3);
    return;
  }
  if constexpr (CF::SW) {
#pragma unroll
    for (int j = 0; j < CF::FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = n0 + wc * CF::TN + j * 16 + fq * 4 + r;  // swapped: element r is column fq*4 + r of row fr
        if (col >= g.N) continue;
        const float bv = g.bias ? g.bias[(long)z * g.c_zoff + col] : 0.f;
#pragma unroll
        for (int i = 0; i < CF::FM; ++i) {
          const int row = m0 + wr * CF::TM + i * 16 + fr;
          if (row >= g.M) continue;
          float v = epi_act_drop(acc[i][j][r] + bv, g.act, g.drop_p, dseed, (long)row * g.N + col);
          if (g.R) v += bf2f(g.R[(long)row * g.ldr + (long)z * g.c_zoff + col]);
          stf<TOUT>(C, (long)row * g.ldc + col, v);
        }
      }
    return;
  }
#pragma unroll
  for (int j = 0; j < CF::FN; ++j) {
    const int col = n0 + wc * CF::TN + j * 16 + fr;
    if (col >= g.N) continue;
    const float bv = g.bias ? g.bias[(long)z * g.c_zoff + col] : 0.f;
#pragma unroll
    for (int i = 0; i < CF::FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wr * CF::TM + i * 16 + fq * 4 + r;
        if (row >= g.M) continue;
        float v = epi_act_drop(acc[i][j][r] + bv, g.act, g.drop_p, dseed, (long)row * g.N + col);
        if (g.R) v += bf2f(g.R[(long)row * g.ldr + (long)z * g.c_zoff + col]);
        stf<TOUT>(C, (long)row * g.ldc + col, v);
      }
  }
}

using CfgP = PipeCfg<128, 64, 2, 2>;   // 4 waves, 64x32 per wave, 48 KiB LDS (pos-conv gather: 48 columns per group)
using CfgT3 = PipeCfg<128, 64, 2, 2, 3>;   // v7: 128x64 tiles, 3-deep ring, 72 KiB LDS (2 blocks / CU)
using CfgW2 = PipeCfg<128, 128, 2, 4, 2>;  // v9: 8 waves (64x32 each), 2-deep, 64 KiB LDS (2 blocks / CU)
using CfgY2 = PipeCfg<256, 256, 4, 4, 2>;  // v13: 16 waves (64x64 each), 2-deep, 128 KiB LDS
using CfgY32 = PipeCfg<256, 256, 4, 4, 2, 64, 3>;  // v18: 16 waves, A 3-deep + B 2-deep rings, 160 KiB LDS
using CfgY32i = PipeCfg<256, 256, 4, 4, 2, 64, 3, 0, 1>;  // v22: v18, DMA issue between MFMA rows
// v23: v18 operand-swapped (bf16 staging, see the epilogue) with the DMA issued between MFMA rows.  (The swapped form
// without the DMA interleave, v21, lost its train-step A/B and was never picked: removed in round 6.)
using CfgY32si = PipeCfg<256, 256, 4, 4, 2, 64, 3, 1, 1>;

template <class CF, typename TOUT, int AMODE>
int launch_pipe_t(const GemmArgs& g, int groups, hipStream_t st) {
  const long tiles = (long)((g.N + CF::BN - 1) / CF::BN) * ((g.M + CF::BM - 1) / CF::BM);
  const size_t lds = CF::LDS_ELEMS * sizeof(bf16_t);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_pipe_kernel<CF, TOUT, AMODE>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return (int)hipErrorInvalidConfiguration;
  hipLaunchKernelGGL((gemm_pipe_kernel<CF, TOUT, AMODE>), dim3((unsigned)tiles, 1, groups), dim3(CF::NT), lds, st, g);
  return (int)hipGetLastError();
}

template <class CF, int AMODE = 0>
int launch_pipe(const GemmArgs& g, int out_dtype, hipStream_t st, int groups = 1) {
  return out_dtype == MER_BF16 ? launch_pipe_t<CF, bf16_t, AMODE>(g, groups, st)
                               : launch_pipe_t<CF, float, AMODE>(g, groups, st);
}

// Tile choice.  variant -1 = the WALL-TIME pick (tools/bench_gemm.py on the B=32 WavLM shapes): occupancy (waves
// per CU) hides the DMA latency of the 2-deep pipeline, so the 16-wave 256x256 tile (v13) wins wherever its grid
// covers most of the 256 CUs (QKV, FFN-up: 0.49 / 0.64 PF); conv1 (1,200 tiles streaming a 314 MB A operand) takes
// the split ring (v18, A three K-tiles deep: 278.6 -> 271.4 us); the 768-column GEMMs and the 512-column convs
// below conv1 have too few such tiles: 128x64 tiles on a 3-deep ring for K >= 2048 (FFN-down), 128x128 8-wave
// tiles otherwise.  variant -2 = the CU-TIME pick for the train step's frozen forward, which runs on a side stream
// beside the trunk: every shape on the v18 split ring.  On the few-tile shapes that is LONGER wall time (FFN-down
// 33 -> 66 us on 57 CUs) but about half the CU-time (57 CUs x 66 us vs 228 x 33), and the two-stream step is bound
// by CU-time: same-box +1.1 % (twice), split ring over the plain ring +0.3 % (profiles/r04j).  All variants are
// bit-identical (same fragments, same k order).
int pick_variant(int M, int N, int K, int rule) {
  if (rule == -2) return 18;
  const long tl = (long)((M + 255) / 256) * ((N + 255) / 256);
  if (tl >= 1200 && N <= 512) return 18;
  if (tl >= 160 && N > 512) return 13;
  return K >= 2048 ? 7 : 9;
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

namespace {
// Tile order: with at most 4 column tiles of 256 (conv1..6: N = 512) the B operand is a few hundred KB and always
// L2-resident, while the A row panel is the stream: keep a panel's N-tiles adjacent (group 1) so they run in lockstep
// on one XCD and fetch the panel once.  Wider outputs (QKV, FFN-up) walk 8-row bands (the B panels dominate).
int tile_group(int N) { return (N + 255) / 256 <= 4 ? 1 : 8; }

// 16-byte epilogue accesses: 8-column runs never straddle N, and every row start is 16-byte aligned
bool vec_epilogue_ok(int N, const void* C, long ldc, const void* R, long ldr, long c_zoff) {
  if (N % 8 || ldc % 8 || c_zoff % 8 || (((uintptr_t)C) & 15)) return false;
  if (R && (ldr % 8 || (((uintptr_t)R) & 15))) return false;
  return true;
}
}  // namespace

MER_API int mer_gemm_bf16(int M, int N, int K, const void* A, long a_gstride, long a_rstride, int a_rpg, const void* W,
                          long ldw, void* C, int c_dtype, long ldc, const float* bias, const void* R, long ldr, int act,
                          void* stream) {
  return mer_gemm_bf16_ex(M, N, K, A, a_gstride, a_rstride, a_rpg, W, ldw, C, c_dtype, ldc, bias, R, ldr, act, -1,
                          stream);
}

MER_API int mer_gemm_bf16_ex(int M, int N, int K, const void* A, long a_gstride, long a_rstride, int a_rpg,
                             const void* W, long ldw, void* C, int c_dtype, long ldc, const float* bias, const void* R,
                             long ldr, int act, int variant, void* stream) {
  return mer_gemm_bf16_tr(M, N, K, A, a_gstride, a_rstride, a_rpg, W, ldw, C, c_dtype, ldc, bias, R, ldr, act, 0.f,
                          nullptr, 0ull, nullptr, 0, variant, stream);
}

MER_API int mer_gemm_bf16_tr(int M, int N, int K, const void* A, long a_gstride, long a_rstride, int a_rpg,
                             const void* W, long ldw, void* C, int c_dtype, long ldc, const float* bias, const void* R,
                             long ldr, int act, float drop_p, const unsigned long long* drop_seed,
                             unsigned long long drop_site, const long long* skip_mask, int skip_bit, int variant,
                             void* stream) {
  if (M <= 0 || N <= 0) return 0;
  if (drop_p < 0.f || drop_p >= 1.f || (drop_p > 0.f && !drop_seed) || skip_bit < 0 || skip_bit > 62)
    return (int)hipErrorInvalidValue;
  if (!(variant == -2 || variant == -1 || variant == 0 || variant == 7 || variant == 9 || variant == 13 ||
        variant == 18 || variant == 22 || variant == 23))
    return (int)hipErrorInvalidValue;
  if (K % 8 != 0 || a_rpg <= 0 || (a_rstride % 8) != 0 || (a_gstride % 8) != 0 || (ldw % 8) != 0)
    return (int)hipErrorInvalidValue;
  if ((((uintptr_t)A) | ((uintptr_t)W)) & 15) return (int)hipErrorInvalidValue;
  GemmArgs g{};
  g.M = M; g.N = N; g.K = K;
  g.A = (const bf16_t*)A; g.a_gstride = a_gstride; g.a_rstride = a_rstride; g.a_rpg = a_rpg;
  g.B = (const bf16_t*)W; g.ldb = ldw; g.b_zstride = 0;
  g.C = C; g.ldc = ldc; g.c_zoff = 0;
  g.bias = bias; g.R = (const bf16_t*)R; g.ldr = ldr; g.act = act;
  g.vec_epi = vec_epilogue_ok(N, C, ldc, R, ldr, 0);
  g.tgroup = tile_group(N);
  g.drop_p = drop_p; g.drop_seed = drop_seed; g.drop_site = drop_site; g.skip_mask = skip_mask; g.skip_bit = skip_bit;
  if (a_rstride > 0 && a_rstride < K) {  // overlapping rows = a strided conv: taps of gcd(stride, K) channels
    long a = a_rstride, b = K;
    while (b) { const long t = a % b; a = b; b = t; }
    if (a % 64 == 0 && K / a > 1) {
      g.kp_taps = (int)(K / a);
      g.kp_c = (int)a;
    }
  }
  const hipStream_t st = (hipStream_t)stream;
  if (K % 64 != 0) variant = 0;  // the register-staged kernel takes any K (multiple of 8)
  if (variant < 0) {
    const int rule = variant;
    variant = pick_variant(M, N, K, rule);
    // The split ring with its LDS-DMA issued between the first substep's MFMA rows (v22); a bf16 output without
    // residual or dropout also rounds before staging on the operand-swapped form (v23: half the epilogue's LDS
    // bytes).  tools/bench_gemm.py, 20 back-to-back launches on the split ring: conv1 with GELU 300 -> 274 us,
    // conv2 150 -> 143, FFN-up 35.9 -> 33.9, QKV 28.9 -> 27.7 (profiles/r05/gemm_swap); bit-identical to v18.
    // Wall-time rule: wherever it picks the split ring (conv1).  CU-time rule (-2, the train step's side-stream
    // forward): the feature-extractor convs only (N <= 512) -- with every shape the same-box ABBA bench ran 204.0
    // vs 204.6 steps/s (6 pairs, profiles/r05/gemm_swap/ab_il_abba.txt), with the convs only 207.25 vs 206.91
    // (5 of 6 pairs, ab_conv_abba.txt): within the box's noise either way, and the convs keep their gain.
    if (variant == 18 && (rule == -1 || N <= 512))
      variant = (c_dtype == MER_BF16 && !R && !(drop_p > 0.f) && g.vec_epi) ? 23 : 22;
  }
  switch (variant) {
    case 7: return launch_pipe<CfgT3>(g, c_dtype, st);
    case 9: return launch_pipe<CfgW2>(g, c_dtype, st);
    case 13: return launch_pipe<CfgY2>(g, c_dtype, st);
    case 18: return launch_pipe<CfgY32>(g, c_dtype, st);
    case 22: return launch_pipe<CfgY32i>(g, c_dtype, st);
    case 23: return launch_pipe<CfgY32si>(g, c_dtype, st);
    default: return launch<0>(g, c_dtype, 1, st);
  }
}

namespace {
// ---------------------------------------------------------------------------------------------------------------
// Positional conv (grouped Conv1d(768, 768, k=128, pad=64, groups=16), TF:82-90) as a Toeplitz product.  The
// implicit GEMM above gathers its A operand per K-tile from x[b, t + tap - pad, c]: with 128 taps every x row is
// fetched 128 times through L2 (~0.94 GB of operand loads per launch for a 7 MB input), which bounded it at ~115 us
// (380 TF/s).  Here one block owns one (clip, group): the clip's rows of that group's 48 channels are loaded ONCE
// into an LDS strip of L + taps - 1 rows (zero rows for the padding), and the A fragment of tap j, time t is strip
// row t + j -- the same 16 bytes the gather produced.  The weights stream through a double-buffered LDS chunk of
// PS_KC k-columns.  Every output element accumulates the same bf16 fragments in the same k-block order on the same
// MFMA as gemm_pipe_kernel<CfgP, 1>, and the epilogue is the same arithmetic (act(acc + bias) rounded through a
// register, then + residual, then bf16), so the result is bit-identical (tests/test_wavlm_gpu.py).
// Limits: L <= PS_MAXL, taps <= PS_MAXT, cg = CG (a multiple of 16), taps * CG % PS_KC == 0.
constexpr int PS_MAXL = 160, PS_MAXT = 128, PS_KC = 192;

template <int CG, int NW>
__global__ __launch_bounds__(64 * NW, 2) void posconv_strip_kernel(int L, int taps, int pad, const bf16_t* __restrict__ X,
                                                               long ldx, const bf16_t* __restrict__ Wp,
                                                               bf16_t* __restrict__ out, long ldo,
                                                               const float* __restrict__ bias,
                                                               const bf16_t* __restrict__ R, long ldr, int act) {
  // wave w owns M fragments w, w + NW, ... (16 time steps each): MI per wave, computed for every wave whether or not
  // the clip has that many rows (branch-free fragment loop; rows past L are discarded by the epilogue), so the strip
  // covers NW * MI fragments
  constexpr int MI = (PS_MAXL / 16 + NW - 1) / NW;
  constexpr int NF = CG / 16, CH = CG / 8, WROW = PS_KC + 8, SROWS = NW * MI * 16 + PS_MAXT;
  constexpr int NT = 64 * NW;
  constexpr int WCH = PS_KC / 8;  // 16-byte chunks per weight row of one K-chunk
  constexpr int WIT = (CG * WCH + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) bf16_t strip[SROWS * CG];
  __shared__ __attribute__((aligned(16))) bf16_t wbuf[2][CG * WROW];
  // grid (groups, clips): linear block id = clip * groups + group, so with groups % 8 == 0 every block of a group
  // lands on the same XCD (ids round-robin over the 8 XCDs) and that XCD's L2 holds only its 2 groups' weights
  // (2 x 590 KB) instead of all 16 (9.4 MB, more than the 4 MB L2: every chunk re-fetched)
  const int z = blockIdx.x, b = blockIdx.y, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int K = taps * CG, nkc = K / PS_KC;
  const bf16_t* Xb = X + (long)b * L * ldx + (long)z * CG;
  const bf16_t* Wz = Wp + (long)z * CG * K;
  const u32x4 zero4 = {0u, 0u, 0u, 0u};
  // strip row u = input time u - pad (zero outside the clip; rows past L + taps - 1 are zero too)
  for (int i = t; i < SROWS * CH; i += NT) {
    const int u = i / CH, ch = i - u * CH, tt = u - pad;
    const bool ok = tt >= 0 && tt < L;
    const u32x4 v = *reinterpret_cast<const u32x4*>(ok ? Xb + (long)tt * ldx + ch * 8 : Xb);
    *reinterpret_cast<u32x4*>(strip + u * CG + ch * 8) = ok ? v : zero4;
  }
  // the next weight chunk in registers, loaded at the top of a chunk and stored to the other buffer at its end (two
  // register sets loading two chunks ahead measured no faster: 77.5 vs 75.8 us)
  u32x4 wr[WIT];
  auto wload = [&](int kc) {
#pragma unroll
    for (int j = 0; j < WIT; ++j) {
      const int i = t + NT * j, n = i / WCH, ch = i - n * WCH;
      wr[j] = i < CG * WCH ? *reinterpret_cast<const u32x4*>(Wz + (long)n * K + kc * PS_KC + ch * 8) : zero4;
    }
  };
  auto wstore = [&](int buf) {
#pragma unroll
    for (int j = 0; j < WIT; ++j) {
      const int i = t + NT * j, n = i / WCH, ch = i - n * WCH;
      if (i < CG * WCH) *reinterpret_cast<u32x4*>(wbuf[buf] + n * WROW + ch * 8) = wr[j];
    }
  };
  const int nmf = (L + 15) / 16;
  f32x4 acc[MI][NF];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  wload(0);
  wstore(0);
  __syncthreads();
  for (int kc = 0; kc < nkc; ++kc) {
    if (kc + 1 < nkc) wload(kc + 1);  // in flight across this chunk's MFMAs
    const bf16_t* wb = wbuf[kc & 1];
#pragma unroll
    for (int kb = 0; kb < PS_KC / 32; ++kb) {
      const int kl = kb * 32 + fq * 8, kg = kc * PS_KC + kl;
      const int tap = kg / CG, c0 = kg - tap * CG;
      bf16x8 bq[NF], af[MI];
#pragma unroll
      for (int j = 0; j < NF; ++j) bq[j] = *reinterpret_cast<const bf16x8*>(wb + (j * 16 + fr) * WROW + kl);
#pragma unroll
      for (int i = 0; i < MI; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(strip + ((w + NW * i) * 16 + fr + tap) * CG + c0);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bq[j], acc[i][j], 0, 0, 0);
    }
    if (kc + 1 < nkc) wstore((kc + 1) & 1);  // the other buffer: its last reader (chunk kc - 1) passed the barrier
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int mf = w + NW * i;
    if (mf >= nmf) break;
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int n = j * 16 + fr;
      const float bv = bias ? bias[z * CG + n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int tt = mf * 16 + fq * 4 + r;
        if (tt >= L) continue;
        float v = apply_act(acc[i][j][r] + bv, act);
        asm volatile("" : "+v"(v));  // round to fp32 here, as the LDS-staged epilogue does: no fma with the add
        const long row = (long)b * L + tt;
        if (R) v += bf2f(R[row * ldr + z * CG + n]);
        out[row * ldo + z * CG + n] = f2bf(v);
      }
    }
  }
}
}  // namespace

MER_API int mer_posconv_gemm_bf16(int B, int L, int C_total, int groups, int taps, int pad, const void* X, long ldx,
                                  const void* Wp, void* out, int out_dtype, long ldo, const float* bias,
                                  const void* R, long ldr, int act, int variant, void* stream) {
  const int cg = C_total / groups;
  if (cg * groups != C_total || cg % 8 != 0 || (ldx % 8) != 0) return (int)hipErrorInvalidValue;
  GemmArgs g{};
  g.M = B * L; g.N = cg; g.K = taps * cg;
  g.A = (const bf16_t*)X; g.pc_L = L; g.pc_pad = pad; g.pc_cg = cg; g.pc_ldx = ldx;
  g.B = (const bf16_t*)Wp; g.ldb = (long)taps * cg; g.b_zstride = (long)cg * taps * cg;
  g.C = out; g.ldc = ldo; g.c_zoff = cg;
  g.bias = bias; g.R = (const bf16_t*)R; g.ldr = ldr; g.act = act;
  g.vec_epi = vec_epilogue_ok(cg, out, ldo, R, ldr, g.c_zoff);
  g.tgroup = 8;
  // variant -1: the Toeplitz strip kernel where it applies, else the gather GEMM; 0: the gather GEMM (the strip
  // kernel's bit-exact reference, tests/test_wavlm_gpu.py)
  if (variant < -1 || variant > 0) return (int)hipErrorInvalidValue;
  if (variant == -1 && cg == 48 && L <= PS_MAXL && taps <= PS_MAXT && (taps * cg) % PS_KC == 0 && out_dtype == MER_BF16 &&
      (ldx % 8) == 0 && (((uintptr_t)X | (uintptr_t)Wp) & 15) == 0) {
    // 4 waves of 3 fragments each (8 or 10 waves per block measured 77-89 us vs 75)
    hipLaunchKernelGGL((posconv_strip_kernel<48, 4>), dim3(groups, B), dim3(256), 0, (hipStream_t)stream, L, taps, pad,
                       (const bf16_t*)X, ldx, (const bf16_t*)Wp, (bf16_t*)out, ldo, bias, (const bf16_t*)R, ldr, act);
    return (int)hipGetLastError();
  }
  if (g.K % 64 == 0 && (((uintptr_t)X | (uintptr_t)Wp) & 15) == 0) {
    return launch_pipe<CfgP, 1>(g, out_dtype, (hipStream_t)stream, groups);
  }
  return launch<1>(g, out_dtype, groups, (hipStream_t)stream);
}
