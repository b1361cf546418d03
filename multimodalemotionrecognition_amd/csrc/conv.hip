// ResNet18 frame trunk (VideoNet.backbone, video.py:21-23 -> torchvision resnet18) on MFMA.
//
// Activations are NHWC bf16 (channels padded to a multiple of 8 so every 16-byte chunk of an
// im2col row is 8 channels of ONE tap).  Convolutions are implicit GEMMs on
// v_mfma_f32_16x16x32_bf16 with fp32 accumulation:
//   fwd   : Y[m=(n,oh,ow)][k]      = sum_{r,s,c} X[n, oh*st-pad+r, ow*st-pad+s, c] W[k][r][s][c]
//   dgrad : dX[m=(n,h,w)][c]       = sum_{r,s,k} dY[n, (h+pad-r)/st, (w+pad-s)/st, k] W'[c][r][s][k]
//           (taps whose (h+pad-r) is not a multiple of st contribute zero)
//   wgrad : dW[k][(r,s,c)]         = sum_{p=(n,oh,ow)} dY[p][k] X[n, oh*st-pad+r, ow*st-pad+s, c]
// fwd/dgrad stage K-contiguous tiles (ds_read_b128 fragments); wgrad reduces over pixels, so both
// operands are staged [pixel][channel] and read with the gfx950 LDS transpose (ds_read_b64_tr_b16).
// BatchNorm (train mode: batch statistics, running-stat update with momentum 0.1 / unbiased var)
// is split into a stats reduction fused into the conv epilogue, a finalize, and an apply pass.
#include <type_traits>

#include "common.h"
#include "mer.h"

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;

// Phase timestamps of the halo conv (tools/halo_phases.py builds a separate library with -DMER_CONV_TIMING; the
// production library compiles CT() to nothing): wall_clock64() of workgroup blockIdx.x's thread 0 at slot k.
#ifdef MER_CONV_TIMING
static __device__ long long mer_ct_buf[512 * 64];
#define CT(k) \
  do { \
    if (threadIdx.x == 0 && blockIdx.x < 512 && (k) < 64) mer_ct_buf[blockIdx.x * 64 + (k)] = wall_clock64(); \
  } while (0)
MER_API int mer_ct_reset() {
  static long long zeros[512 * 64];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(mer_ct_buf), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice);
}
MER_API int mer_ct_read(long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(mer_ct_buf), sizeof(long long) * 512 * 64, 0, hipMemcpyDeviceToHost);
}
// conv_pipe_kernel's phases (tools/pipe_phases.py): slot k of the linear block id (blockIdx.y * gridDim.x + blockIdx.x)
static __device__ long long mer_ctp_buf[4096 * 8];
#define CTP(k) \
  do { \
    const unsigned b_ = blockIdx.y * gridDim.x + blockIdx.x; \
    if (threadIdx.x == 0 && b_ < 4096) mer_ctp_buf[b_ * 8 + (k)] = wall_clock64(); \
  } while (0)
MER_API int mer_ctp_reset() {
  static long long zeros[4096 * 8];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(mer_ctp_buf), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice);
}
MER_API int mer_ctp_read(long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(mer_ctp_buf), sizeof(long long) * 4096 * 8, 0, hipMemcpyDeviceToHost);
}
#else
#define CT(k) \
  do { \
  } while (0)
#define CTP(k) \
  do { \
  } while (0)
#endif

namespace {

constexpr int CBK = 64;  // K step

struct ConvGeom {
  int N, OH, OW;          // GEMM output spatial dims (fwd: Ho,Wo; dgrad: H,W)
  int IH, IW, IC;         // A-source spatial dims / channels (fwd: H,W,C; dgrad: Ho,Wo,K)
  int R, S, st, pad;
  int Ncols;              // GEMM N (fwd: Cout; dgrad: Cin)
  int Kred;               // R*S*IC
  const bf16_t* X;        // A source
  const bf16_t* Wt;       // [Ncols][Kred]
  bf16_t* Y;              // [M][ldy]
  long ldy;
  float* stats;           // fwd: per column (sum, sumsq), may be null
  const bf16_t* R_;       // residual added in the epilogue (dgrad), may be null
  const bf16_t* Rmask;    // residual is added only where Rmask > 0 (relu mask), may be null
  // dgrad only: the BatchNorm-backward reduction of the BN whose relu'd output this gradient flows
  // into, fused into the epilogue (bn_bwd_reduce semantics; NULL bnr_red = off).  g = (mask > 0) * y,
  // red[p][c] += (sum g, sum g * (x - mean) * rstd); red2 likewise for a second BN reading the same g
  // (the downsample branch).  One stored row per output row tile (MER_BN_RED_ROWS), like the forward statistics.
  const bf16_t* bnr_mask;
  const bf16_t* bnr_x;
  const float* bnr_ms;
  float* bnr_red;
  const bf16_t* bnr_x2;
  const float* bnr_ms2;
  float* bnr_red2;
  int vec;                // 16-byte epilogue (Ncols, ldy multiples of 8, every operand 16-byte aligned)
  // stride-2 dgrad only: a 1x1 / stride-2 / pad-0 downsample of the same input fused as an extra K segment of parity
  // class (0, 0) -- the only class its taps reach: dx[2i, 2j] += sum_k dY2[i, j, k] W2t[c][k] (NULL X2 = off)
  const bf16_t* X2;       // [N][IH][IW][K2], the downsample branch's output gradient
  const bf16_t* Wt2;      // [Ncols][K2]
  int K2;
};

__host__ __device__ inline bool conv_vec_ok(const ConvGeom& g) {
  const uintptr_t a = (uintptr_t)g.Y | (uintptr_t)g.R_ | (uintptr_t)g.Rmask | (uintptr_t)g.bnr_mask |
                      (uintptr_t)g.bnr_x | (uintptr_t)g.bnr_x2 | (uintptr_t)g.stats | (uintptr_t)g.bnr_red |
                      (uintptr_t)g.bnr_red2;
  return g.Ncols % 8 == 0 && g.ldy % 8 == 0 && (a & 15) == 0;
}

template <bool DGRAD>
__device__ __forceinline__ u32x4 conv_a_chunk(const ConvGeom& g, int n, int oh, int ow, bool rowok, int kk, int tap,
                                              int c, int r, int s) {
  u32x4 v = {0u, 0u, 0u, 0u};
  if (!rowok || kk >= g.Kred) return v;
  int ih, iw;
  if (!DGRAD) {
    ih = oh * g.st - g.pad + r;
    iw = ow * g.st - g.pad + s;
  } else {
    const int th = oh + g.pad - r, tw = ow + g.pad - s;
    if (th < 0 || tw < 0) return v;
    if (g.st == 1) {
      ih = th;
      iw = tw;
    } else if (g.st == 2) {
      if ((th | tw) & 1) return v;
      ih = th >> 1;
      iw = tw >> 1;
    } else {
      if ((th % g.st) || (tw % g.st)) return v;
      ih = th / g.st;
      iw = tw / g.st;
    }
  }
  if (ih < 0 || ih >= g.IH || iw < 0 || iw >= g.IW) return v;
  return *reinterpret_cast<const u32x4*>(g.X + (((long)n * g.IH + ih) * g.IW + iw) * g.IC + c);
}

// fwd / dgrad implicit GEMM. BM_ x BN_ tile, 4 waves as 2x2.
template <bool DGRAD, int BM_, int BN_>
__global__ __launch_bounds__(256, 2) void conv_kernel(ConvGeom g) {
  constexpr int LDK = CBK + 8;
  constexpr int IT = BM_ / 32, JT = BN_ / 32;           // 16x16 tiles per wave
  constexpr int ACH = BM_ * 8 / 256, BCH = BN_ * 8 / 256;  // 16B chunks per thread per K step
  __shared__ __attribute__((aligned(16))) bf16_t lds[2][(BM_ + BN_) * LDK];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int M = g.N * g.OH * g.OW;
  const int nx = (g.Ncols + BN_ - 1) / BN_, ny = (M + BM_ - 1) / BM_;
  int tx, ty;
  xcd_tile(blockIdx.x, nx, nx * ny, tx, ty);
  const int m0 = ty * BM_, n0 = tx * BN_;
  const int wm = (w >> 1) * (BM_ / 2), wn = (w & 1) * (BN_ / 2);
  const int crow = t >> 3, ckc = t & 7;

  int an[ACH], aoh[ACH], aow[ACH];
  bool aok[ACH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    const int m = m0 + crow + 32 * i;
    aok[i] = m < M;
    const int mm = aok[i] ? m : 0;
    an[i] = mm / (g.OH * g.OW);
    const int rem = mm - an[i] * g.OH * g.OW;
    aoh[i] = rem / g.OW;
    aow[i] = rem - aoh[i] * g.OW;
  }
  u32x4 ra[ACH], rb[BCH];
  const float inv_IC = 1.f / g.IC, inv_S = 1.f / g.S;
  auto gload = [&](int k0) {
    const int kk = k0 + ckc * 8;
    const int tap = fdiv(kk, inv_IC), c = kk - tap * g.IC;
    const int r = fdiv(tap, inv_S), s = tap - r * g.S;
#pragma unroll
    for (int i = 0; i < ACH; ++i) ra[i] = conv_a_chunk<DGRAD>(g, an[i], aoh[i], aow[i], aok[i], kk, tap, c, r, s);
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int n = n0 + crow + 32 * i;
      rb[i] = (n < g.Ncols && kk < g.Kred) ? *reinterpret_cast<const u32x4*>(g.Wt + (long)n * g.Kred + kk)
                                            : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < ACH; ++i)
      *reinterpret_cast<u32x4*>(&lds[buf][(crow + 32 * i) * LDK + ckc * 8]) = ra[i];
#pragma unroll
    for (int i = 0; i < BCH; ++i)
      *reinterpret_cast<u32x4*>(&lds[buf][(BM_ + crow + 32 * i) * LDK + ckc * 8]) = rb[i];
  };
  f32x4 acc[IT][JT];
#pragma unroll
  for (int i = 0; i < IT; ++i)
#pragma unroll
    for (int j = 0; j < JT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (g.Kred + CBK - 1) / CBK;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * CBK);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int kof = s * 32 + (lane >> 4) * 8;
      bf16x8 af[IT], bfr[JT];
#pragma unroll
      for (int i = 0; i < IT; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(&lds[cur][(wm + i * 16 + (lane & 15)) * LDK + kof]);
#pragma unroll
      for (int j = 0; j < JT; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(&lds[cur][(BM_ + wn + j * 16 + (lane & 15)) * LDK + kof]);
#pragma unroll
      for (int i = 0; i < IT; ++i)
#pragma unroll
        for (int j = 0; j < JT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int j = 0; j < JT; ++j) {
    const int col = n0 + wn + j * 16 + (lane & 15);
    float csum = 0.f, csq = 0.f;
#pragma unroll
    for (int i = 0; i < IT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
        if (row < M && col < g.Ncols) {
          float v = acc[i][j][r];
          if (g.R_) {
            const long ri = (long)row * g.ldy + col;
            if (!g.Rmask || bf2f(g.Rmask[ri]) > 0.f) v += bf2f(g.R_[ri]);
          }
          const bf16_t h = f2bf(v);
          g.Y[(long)row * g.ldy + col] = h;
          const float hv = bf2f(h);
          csum += hv;
          csq += hv * hv;
        }
      }
    if (g.stats) {
      csum += __shfl_xor(csum, 16, 64);
      csum += __shfl_xor(csum, 32, 64);
      csq += __shfl_xor(csq, 16, 64);
      csq += __shfl_xor(csq, 32, 64);
      if ((lane >> 4) == 0 && col < g.Ncols) {
        float* slab = g.stats + (long)ty * g.Ncols * 2;  // this row tile's own stats row (exactly 2 adds onto 0: order-free)
        atomicAdd(slab + 2 * col, csum);
        atomicAdd(slab + 2 * col + 1, csq);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// wgrad: dW[k][(r,s,c)] += sum_p dY[p][k] X(p; r,s,c).  Split-K over pixels (grid z): each split
// stores a coalesced fp32 slab, wgrad_reduce sums them into the PyTorch-layout gradient [Cout][Cin][R][S]
// (scattered fp32 atomics at stride R*S ran ~17x under the atomic peak: MI355X_MICROARCH 'Global float atomics').
// LDS images [pixel][channel] (+16 pad); MFMA fragments via ds_read_b64_tr_b16.
// ---------------------------------------------------------------------------------------
struct WgradGeom {
  int N, H, W, C;         // X (input activation, NHWC, C padded)
  int Ho, Wo, K;          // dY
  int R, S, st, pad;
  int Creal;              // real input channels (<= C) of the weight
  const bf16_t* X;
  const bf16_t* dY;
  float* ws;              // [splits][K][R*S*C] fp32 partial slabs
  int pix_per_split;
  long ldy;               // dY row stride (elements; K for a conv, a column slice of a wider matrix for a Linear)
  int flat;               // wgrad_pipe_kernel: 1-D grid of splits x tiles, a split's tiles on one XCD (see there)
};

template <int BM_, int BN_, int WM = 2, int WN = 2, int PF = 1>
__global__ __launch_bounds__(64 * WM * WN, 2) void wgrad_kernel(WgradGeom g) {
  constexpr int NT = 64 * WM * WN;
  constexpr int LDM = BM_ + 16, LDN = BN_ + 16;
  constexpr int IT = BM_ / WM / 16, JT = BN_ / WN / 16;
  constexpr int ACH = BM_ * 64 / 8 / NT, BCH = BN_ * 64 / 8 / NT;  // 16B chunks per thread
  static_assert(ACH * NT * 8 == BM_ * 64 && BCH * NT * 8 == BN_ * 64, "staging split");
  __shared__ __attribute__((aligned(16))) bf16_t lds[2][64 * LDM + 64 * LDN];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int Ntot = g.R * g.S * g.C;
  const int P = g.N * g.Ho * g.Wo;
  const int wnx = (Ntot + BN_ - 1) / BN_, wny = (g.K + BM_ - 1) / BM_;
  int wtx, wty;
  xcd_tile(blockIdx.x, wnx, wnx * wny, wtx, wty);
  const int m0 = wty * BM_, n0 = wtx * BN_;
  const int p_beg = blockIdx.z * g.pix_per_split, p_end = min(P, p_beg + g.pix_per_split);
  const int wm = (w / WN) * (BM_ / WM), wn = (w % WN) * (BN_ / WN);
  constexpr int ACPR = BM_ / 8, BCPR = BN_ / 8;  // chunks per LDS row

  // PF = 1: one register set, the next K-step's loads in flight during this one's MFMAs, __syncthreads per step.
  // PF = 2: two register sets, K-steps kt+1 and kt+2 in flight; the per-step barrier is a raw s_barrier after
  // lgkmcnt(0) (this wave's LDS traffic), so the younger register loads stay in flight across it (a
  // __syncthreads would drain vmcnt to 0 and leave one step of latency hiding).
  u32x4 ra[ACH], rb[BCH], ra2[ACH], rb2[BCH];
  // Per-thread constants: a thread always stages the same 16-byte column chunk, so its (tap, c) and the
  // row offsets of its chunks are fixed; only the pixel base moves (by 64) per K step.
  const int a_cc = t % ACPR, a_pr0 = t / ACPR;
  const int b_cc = t % BCPR, b_pr0 = t / BCPR;
  const int b_nn = n0 + b_cc * 8;
  const bool b_colok = b_nn < Ntot;
  const float inv_C = 1.f / g.C, inv_S = 1.f / g.S, inv_HoWo = 1.f / (g.Ho * g.Wo), inv_Wo = 1.f / g.Wo;
  const int b_tap = b_colok ? fdiv(b_nn, inv_C) : 0;
  const int b_c = b_colok ? b_nn - b_tap * g.C : 0;
  const int b_r = fdiv(b_tap, inv_S), b_s = b_tap - fdiv(b_tap, inv_S) * g.S;
  const int HoWo = g.Ho * g.Wo;
  // Branch-free staging: every load is unconditional from a clamped (valid) address, its validity kept in a
  // bit of `okm`; the zeroing select happens at the LDS store, after this K-step's MFMAs.  (A per-lane
  // condition around a load compiles to a branch and a wait for that load: the staging loads of a K-step
  // were serialised on the memory latency.)
  unsigned okm = 0u, okm2 = 0u;
  auto gload = [&](u32x4* ra, u32x4* rb, unsigned& okm, int p0) {
    okm = 0u;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int p = p0 + a_pr0 + i * (NT / ACPR), k = m0 + a_cc * 8;
      const bool ok = p < p_end && k < g.K;
      ra[i] = *reinterpret_cast<const u32x4*>(g.dY + (long)(p < p_end ? p : p_beg) * g.ldy + (k < g.K ? k : 0));
      okm |= (ok ? 1u : 0u) << i;
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int p = p0 + b_pr0 + i * (NT / BCPR);
      const int pc = p < p_end ? p : p_beg;
      const int n = fdiv(pc, inv_HoWo);
      const int rem = pc - n * HoWo;
      const int oh = fdiv(rem, inv_Wo), ow = rem - oh * g.Wo;
      const int ih = oh * g.st - g.pad + b_r, iw = ow * g.st - g.pad + b_s;
      const bool ok = p < p_end && b_colok && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
      const int ihc = ih < 0 ? 0 : (ih >= g.H ? g.H - 1 : ih), iwc = iw < 0 ? 0 : (iw >= g.W ? g.W - 1 : iw);
      rb[i] = *reinterpret_cast<const u32x4*>(g.X + (((long)n * g.H + ihc) * g.W + iwc) * g.C + b_c);
      okm |= (ok ? 1u : 0u) << (ACH + i);
    }
  };
  auto lstore = [&](int buf, const u32x4* ra, const u32x4* rb, unsigned okm) {
    const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int ch = t + NT * i;
      *reinterpret_cast<u32x4*>(&lds[buf][(ch / ACPR) * LDM + (ch % ACPR) * 8]) = ((okm >> i) & 1u) ? ra[i] : z;
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int ch = t + NT * i;
      *reinterpret_cast<u32x4*>(&lds[buf][64 * LDM + (ch / BCPR) * LDN + (ch % BCPR) * 8]) =
          ((okm >> (ACH + i)) & 1u) ? rb[i] : z;
    }
  };
  // transposed fragment: elements j=0..7 = Img[k0 + 8*(lane>>4) + j][c0 + (lane&15)]
  auto tr_frag = [&](const bf16_t* img, int ld, int k0, int c0) -> bf16x8 {
    const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4;
    const int kr = k0 + 8 * (lane >> 4);
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + (kr + q) * ld + c0 + p4));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + (kr + 4 + q) * ld + c0 + p4));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  };

  f32x4 acc[IT][JT];
#pragma unroll
  for (int i = 0; i < IT; ++i)
#pragma unroll
    for (int j = 0; j < JT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p_end - p_beg + 63) / 64;
  auto compute = [&](int cur) {
    const bf16_t* Aimg = &lds[cur][0];
    const bf16_t* Bimg = &lds[cur][64 * LDM];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[IT], bfr[JT];
#pragma unroll
      for (int i = 0; i < IT; ++i) af[i] = tr_frag(Aimg, LDM, s * 32, wm + i * 16);
#pragma unroll
      for (int j = 0; j < JT; ++j) bfr[j] = tr_frag(Bimg, LDN, s * 32, wn + j * 16);
#pragma unroll
      for (int i = 0; i < IT; ++i)
#pragma unroll
        for (int j = 0; j < JT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  if (PF == 1) {
    if (nk > 0) {
      gload(ra, rb, okm, p_beg);
      lstore(0, ra, rb, okm);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      gload(ra, rb, okm, p_beg + (kt + 1 < nk ? kt + 1 : kt) * 64);  // unconditional (the last one re-reads, unused)
      compute(cur);
      if (kt + 1 < nk) lstore(cur ^ 1, ra, rb, okm);
      __syncthreads();
    }
  } else {
    // set 1 (ra, rb) carries the even K-steps, set 2 the odd ones; loads past the end re-read step nk-1, unused
    auto kstep = [&](int k) { return p_beg + (k < nk ? k : nk - 1) * 64; };
    if (nk > 0) {
      gload(ra, rb, okm, p_beg);
      gload(ra2, rb2, okm2, kstep(1));
      lstore(0, ra, rb, okm);
    }
    lds_barrier();
    for (int kt = 0; kt < nk; kt += 2) {
      gload(ra, rb, okm, kstep(kt + 2));  // set 1 was stored into LDS by the previous step
      compute(0);
      if (kt + 1 < nk) lstore(1, ra2, rb2, okm2);
      lds_barrier();
      if (kt + 1 >= nk) break;
      gload(ra2, rb2, okm2, kstep(kt + 3));
      compute(1);
      if (kt + 2 < nk) lstore(0, ra, rb, okm);
      lds_barrier();
    }
  }
  // partial tile -> this split's fp32 slab [K][R*S*C] (plain coalesced stores; summed by wgrad_reduce)
  float* slab = g.ws + (long)blockIdx.z * g.K * Ntot;
#pragma unroll
  for (int i = 0; i < IT; ++i)
#pragma unroll
    for (int j = 0; j < JT; ++j) {
      const int nn = n0 + wn + j * 16 + (lane & 15);
      if (nn >= Ntot) continue;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int k = m0 + wm + i * 16 + (lane >> 4) * 4 + rr;
        if (k < g.K) slab[(long)k * Ntot + nn] = acc[i][j][rr];
      }
    }
}

// wgrad on a global_load_lds ring (the conv_pipe_kernel structure): no staging registers, STAGES-1 K-steps of
// 64 pixels in flight across each barrier (counted vmcnt + raw s_barrier).  LDS images [64 pixels][BM | BN]
// are dense rows of 16-byte chunks, chunk c of row r stored at c ^ wswz(r) (the DMA writes lane-linear, so the
// XOR is applied to each lane's SOURCE chunk and to the transposed fragment read): the 4 rows one
// ds_read_b64_tr_b16 lane group reads land on distinct bank groups.  Spatial padding, pixels past the split
// and channels past K / R*S*C read a 16-byte zero chunk in global memory.  Same partial slabs as wgrad_kernel.
__device__ __attribute__((aligned(16))) uint32_t mer_conv_zero16[4] = {0u, 0u, 0u, 0u};

__device__ __forceinline__ int wswz(int row, int nchunks) { return ((row & 7) << 1) & (nchunks - 1); }

// KG > 1: in-workgroup split-K over the pixels, as in conv_pipe_kernel: KG groups of WM x WN waves, each with its own
// ring and a contiguous 1/KG of the split's K-steps; the groups' tiles are summed in LDS in group order before the one
// slab store.  A KG = 2 launch covers the pixels of two one-group splits with the same waves per CU, so it writes (and
// the fold re-reads) half the fp32 slabs -- ~0.5 of the ~1 GB per step the trunk's weight gradients moved.
template <int BM_, int BN_, int WM, int WN, int STAGES, int KS = 64, int KG = 1>
__global__ __launch_bounds__(64 * WM * WN * KG, KG > 1 ? WM * WN * KG / 4 : 2) void wgrad_pipe_kernel(WgradGeom g) {
  constexpr int WAVES = WM * WN;  // per K-group
  constexpr int ACW = BM_ / 8, BCW = BN_ / 8;           // 16-byte chunks per LDS row
  constexpr int ARI = 64 / ACW, BRI = 64 / BCW;         // rows per glds instruction
  constexpr int IA = KS / ARI / WAVES, IB = KS / BRI / WAVES;  // glds per wave per K-step of KS pixels
  static_assert(IA * ARI * WAVES == KS && IB * BRI * WAVES == KS, "the K-step must split into whole glds rows");
  static_assert(KS % 32 == 0, "MFMA k = 32 pixels");
  constexpr int IT = BM_ / WM / 16, JT = BN_ / WN / 16;
  constexpr int BUF = KS * (BM_ + BN_);                 // bf16 elements per ring slot
  extern __shared__ __attribute__((aligned(16))) bf16_t smem_all[];
  const int t = threadIdx.x, lane = t & 63, kg = (t >> 6) / WAVES, w = (t >> 6) % WAVES;
  bf16_t* const smem = smem_all + kg * STAGES * BUF;  // this K-group's ring
  const int Ntot = g.R * g.S * g.C;
  const int P = g.N * g.Ho * g.Wo;
  const int wnx = (Ntot + BN_ - 1) / BN_, wny = (g.K + BM_ - 1) / BM_;
  int wtx, wty, zs;
  if (g.flat) {
    // Every tile of one split reads the same pixel range (dY rows and, for an R x S conv, R*S shifted windows of X
    // rows).  Split-major over the bijective XCD chunks (xcd_tile on the flattened (split, tile) index): an XCD runs
    // whole splits, so their tiles fetch the rows into ITS L2 once.  With the z grid the T tiles of a split went
    // to T different XCDs (linear dispatch order round-robins XCDs) and each re-fetched the rows from HBM:
    // layer1's 3x3 wgrad read 244 MB per launch for 51 MB of operands (gpurun_out/pmcstep).
    int tile;
    xcd_tile(blockIdx.x, wnx * wny, (int)gridDim.x, tile, zs);
    wty = tile / wnx;
    wtx = tile - wty * wnx;
  } else {
    xcd_tile(blockIdx.x, wnx, wnx * wny, wtx, wty);
    zs = blockIdx.z;
  }
  const int m0 = wty * BM_, n0 = wtx * BN_;
  const int p_beg = zs * g.pix_per_split, p_end = min(P, p_beg + g.pix_per_split);
  const int wm = (w / WN) * (BM_ / WM), wn = (w % WN) * (BN_ / WN);
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(mer_conv_zero16);

  // per-lane constants of each glds: its LDS row inside the K-step and its (logical) column chunk
  int arow[IA], acol[IA];
  bool acok[IA];
#pragma unroll
  for (int j = 0; j < IA; ++j) {
    const int row = (w * IA + j) * ARI + lane / ACW;
    arow[j] = row;
    acol[j] = m0 + ((lane % ACW) ^ wswz(row, ACW)) * 8;
    acok[j] = acol[j] < g.K;
  }
  int brow[IB], bc[IB], br[IB], bs[IB];
  bool bcok[IB];
  const float inv_C = 1.f / g.C, inv_S = 1.f / g.S, inv_HoWo = 1.f / (g.Ho * g.Wo), inv_Wo = 1.f / g.Wo;
#pragma unroll
  for (int j = 0; j < IB; ++j) {
    const int row = (w * IB + j) * BRI + lane / BCW;
    brow[j] = row;
    const int col = n0 + ((lane % BCW) ^ wswz(row, BCW)) * 8;
    bcok[j] = col < Ntot;
    const int cc = bcok[j] ? col : 0;
    const int tap = fdiv(cc, inv_C);
    bc[j] = cc - tap * g.C;
    br[j] = fdiv(tap, inv_S);
    bs[j] = tap - br[j] * g.S;
  }
  const int HoWo = g.Ho * g.Wo;
  auto stage = [&](int slot, int p0) {
    bf16_t* la = smem + slot * BUF;
    bf16_t* lb = la + KS * BM_;
#pragma unroll
    for (int j = 0; j < IA; ++j) {
      const int p = p0 + arow[j];
      glds16(p < p_end && acok[j] ? g.dY + (long)p * g.ldy + acol[j] : zero, la + (w * IA + j) * 512);
    }
#pragma unroll
    for (int j = 0; j < IB; ++j) {
      const int p = p0 + brow[j];
      const int pc = p < p_end ? p : p_beg;
      const int n = fdiv(pc, inv_HoWo);
      const int rem = pc - n * HoWo;
      const int oh = fdiv(rem, inv_Wo), ow = rem - oh * g.Wo;
      const int ih = oh * g.st - g.pad + br[j], iw = ow * g.st - g.pad + bs[j];
      const bool ok = p < p_end && bcok[j] && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
      glds16(ok ? g.X + (((long)n * g.H + ih) * g.W + iw) * g.C + bc[j] : zero, lb + (w * IB + j) * 512);
    }
  };
  // transposed fragment from a swizzled image with CW chunks per row: elements j = 0..7 =
  // Img[k0 + 8*(lane>>4) + j][c0 + (lane&15)]
  auto tr_frag = [&](const bf16_t* img, int CW, int k0, int c0) -> bf16x8 {
    const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4;
    const int kr = k0 + 8 * (lane >> 4);
    const int lc = (c0 + p4) >> 3, sub = (c0 + p4) & 7;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const int r0 = kr + q, r1 = kr + 4 + q;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(img + r0 * CW * 8 + ((lc ^ wswz(r0, CW)) << 3) + sub));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(img + r1 * CW * 8 + ((lc ^ wswz(r1, CW)) << 3) + sub));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  };

  f32x4 acc[IT][JT];
#pragma unroll
  for (int i = 0; i < IT; ++i)
#pragma unroll
    for (int j = 0; j < JT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // this K-group's K-steps [kb, kb + nk) of the split's nk_all (every group runs the loop nkg times: workgroup-wide
  // barriers)
  const int nk_all = (p_end - p_beg + KS - 1) / KS;
  const int nkg = (nk_all + KG - 1) / KG, kb = kg * nkg;
  const int nk = nk_all - kb < nkg ? (nk_all - kb > 0 ? nk_all - kb : 0) : nkg;
  const int pk0 = p_beg + kb * KS;
  constexpr int G = IA + IB;
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) stage(s, pk0 + s * KS);
  for (int kt = 0; kt < nkg; ++kt) {
    const int left = nk - 1 - kt;
    const int ahead = left < (STAGES - 2) ? left : (STAGES - 2);
    wait_tiles_in_flight<G>(ahead);
    lds_barrier();
    if (kt + STAGES - 1 < nk) stage((kt + STAGES - 1) % STAGES, pk0 + (kt + STAGES - 1) * KS);
    if (KG > 1 && kt >= nk) continue;
    const bf16_t* Aimg = smem + (kt % STAGES) * BUF;
    const bf16_t* Bimg = Aimg + KS * BM_;
#pragma unroll
    for (int s = 0; s < KS / 32; ++s) {
      bf16x8 af[IT], bfr[JT];
#pragma unroll
      for (int i = 0; i < IT; ++i) af[i] = tr_frag(Aimg, ACW, s * 32, wm + i * 16);
#pragma unroll
      for (int j = 0; j < JT; ++j) bfr[j] = tr_frag(Bimg, BCW, s * 32, wn + j * 16);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < IT; ++i)
#pragma unroll
        for (int j = 0; j < JT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  if constexpr (KG > 1) {  // groups 1.. hand their tiles to group 0 through LDS; group 0 sums in group order
    constexpr int LDR = BN_ + 4;
    __syncthreads();  // every group's last fragment reads are done before the exchange reuses the rings
    float* const part = reinterpret_cast<float*>(smem_all);
    if (kg > 0) {
      float* mine = part + (kg - 1) * BM_ * LDR;
#pragma unroll
      for (int i = 0; i < IT; ++i)
#pragma unroll
        for (int j = 0; j < JT; ++j)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            mine[(wm + i * 16 + (lane >> 4) * 4 + rr) * LDR + wn + j * 16 + (lane & 15)] = acc[i][j][rr];
    }
    lds_barrier();
    if (kg > 0) return;
#pragma unroll
    for (int i = 0; i < IT; ++i)
#pragma unroll
      for (int j = 0; j < JT; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
#pragma unroll
          for (int q = 1; q < KG; ++q)
            acc[i][j][rr] += part[(q - 1) * BM_ * LDR + (wm + i * 16 + (lane >> 4) * 4 + rr) * LDR + wn + j * 16 +
                                  (lane & 15)];
  }
  float* slab = g.ws + (long)zs * g.K * Ntot;
#pragma unroll
  for (int i = 0; i < IT; ++i)
#pragma unroll
    for (int j = 0; j < JT; ++j) {
      const int nn = n0 + wn + j * 16 + (lane & 15);
      if (nn >= Ntot) continue;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int k = m0 + wm + i * 16 + (lane >> 4) * 4 + rr;
        if (k < g.K) slab[(long)k * Ntot + nn] = acc[i][j][rr];
      }
    }
}

template <int BM_, int BN_, int WM, int WN, int STAGES, int KS = 64, int KG = 1>
void launch_wgrad_pipe(const WgradGeom& g0, dim3 grid, hipStream_t st) {
  const size_t ring = (size_t)KG * STAGES * KS * (BM_ + BN_) * sizeof(bf16_t);
  const size_t xchg = (size_t)(KG - 1) * BM_ * (BN_ + 4) * sizeof(float);
  const size_t lds = ring > xchg ? ring : xchg;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_pipe_kernel<BM_, BN_, WM, WN, STAGES, KS, KG>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return;
  // split-major 1-D grid over xcd_tile's XCD chunks: the tiles of one split (same dY rows, same shifted X windows)
  // share an L2 (DESIGN.md section 4e'': layer1 / stem wgrad fetch 244 -> 67 MB per launch)
  WgradGeom g = g0;
  g.flat = 1;
  const dim3 gr(grid.x * grid.z, 1, 1);
  hipLaunchKernelGGL((wgrad_pipe_kernel<BM_, BN_, WM, WN, STAGES, KS, KG>), gr, dim3(64 * WM * WN * KG), lds, st, g);
}

// slab0[i] = sum_z ws[z][i] over the flat [K][R*S*C] index.  A block owns E = 256/SG consecutive elements
// and SG split-groups: thread (sg, e) sums splits sg, sg+SG, ... with 4 independent loads in flight (the
// split count reaches ~100 on the stem / layer1, where one serial chain per element was latency-bound),
// and the SG partials meet in LDS.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(int K, int C, int Creal, int RS, int splits, int SG,
                                                           float* __restrict__ ws) {
  __shared__ float part[256];
  const int E = 256 / SG, e = threadIdx.x % E, sg = threadIdx.x / E;
  const long total = (long)K * RS * C;
  const long idx = (long)blockIdx.x * E + e;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (idx < total) {
    int z = sg;
    for (; z + 3 * SG < splits; z += 4 * SG) {
      a0 += ws[(long)z * total + idx];
      a1 += ws[(long)(z + SG) * total + idx];
      a2 += ws[(long)(z + 2 * SG) * total + idx];
      a3 += ws[(long)(z + 3 * SG) * total + idx];
    }
    for (; z < splits; z += SG) a0 += ws[(long)z * total + idx];
  }
  part[threadIdx.x] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (sg != 0 || idx >= total) return;
  float s = 0.f;
  for (int q = 0; q < SG; ++q) s += part[q * E + e];
  ws[idx] = s;  // slab 0 (only this block ever reads element idx)
}

// dw[k][c][r][s] += sum_z ws[z][k][(r*S+s)*C + c] for c < Creal, in split order: one pass replacing the
// reduce + scatter pair.  Block (channel group of 32, k): each thread sums its (tap, channel) elements over
// the splits (8 loads in flight, clamped, branch-free) into an LDS [tap][32] tile, written back in the
// PyTorch order (c, r, s) -- a contiguous run of 32*R*S floats.
__global__ __launch_bounds__(256) void wgrad_fold_scatter_kernel(int K, int C, int Creal, int RS, int splits,
                                                                 const float* __restrict__ ws, float* __restrict__ dw) {
  __shared__ float tile[49 * 32];  // R*S <= 49 (7x7 stem)
  const int k = blockIdx.y, c0 = blockIdx.x * 32;
  const long slab = (long)K * RS * C;
  const float* src = ws + (long)k * RS * C;
  for (int i = threadIdx.x; i < RS * 32; i += 256) {
    const int tap = i >> 5, c = c0 + (i & 31);
    const float* e = src + tap * C + (c < Creal ? c : 0);
    float s = 0.f;
    for (int z0 = 0; z0 < splits; z0 += 8) {
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = e[(long)(z0 + q < splits ? z0 + q : splits - 1) * slab];
#pragma unroll
      for (int q = 0; q < 8; ++q) s += z0 + q < splits ? v[q] : 0.f;
    }
    tile[i] = c < Creal ? s : 0.f;
  }
  __syncthreads();
  const int ncl = min(32, Creal - c0);
  const float inv_RS = 1.f / RS;
  float* dst = dw + ((long)k * Creal + c0) * RS;
  for (int i = threadIdx.x; i < ncl * RS; i += 256) {  // i = cl*RS + tap
    const int cl = fdiv(i, inv_RS), tap = i - cl * RS;
    dst[i] += tile[tap * 32 + cl];
  }
}

// dw[k][c][r][s] += slab0[k][(r*S+s)*C + c] for c < Creal.  Block (channel group of 32, k): reads coalesced
// along c (one 128-byte segment per tap) into an LDS [tap][32] tile, written back in the PyTorch order
// (c, r, s) -- a contiguous run of 32*R*S floats.
__global__ __launch_bounds__(256) void wgrad_scatter_kernel(int C, int Creal, int RS, const float* __restrict__ ws,
                                                            float* __restrict__ dw) {
  __shared__ float tile[49 * 32];  // R*S <= 49 (7x7 stem)
  const int k = blockIdx.y, c0 = blockIdx.x * 32;
  const float* src = ws + (long)k * RS * C;
  for (int i = threadIdx.x; i < RS * 32; i += 256) {
    const int tap = i >> 5, c = c0 + (i & 31);
    tile[i] = c < Creal ? src[tap * C + c] : 0.f;
  }
  __syncthreads();
  const int ncl = min(32, Creal - c0);
  const float inv_RS = 1.f / RS;
  float* dst = dw + ((long)k * Creal + c0) * RS;
  for (int i = threadIdx.x; i < ncl * RS; i += 256) {  // i = cl*RS + tap
    const int cl = fdiv(i, inv_RS), tap = i - cl * RS;
    dst[i] += tile[tap * 32 + cl];
  }
}

// Batched fold of deferred split-K partial slabs: every weight gradient of one backward segment in ONE launch
// instead of one or two per convolution (the folds were ~30 launches of 5-12 us each on the critical stream).
// Record r: dw_r[k][c][tap] += sum_z ws_r[z][k][tap*C + c] (c < Creal), or with a scatter map
// dw_r[k][map[j]] for source column j = tap*C + c (-1: dropped) -- the stem's 4x4 space-to-depth form
// gathered back to 7x7x3.  Threads walk the SOURCE order (coalesced slab reads, the bulk of the bytes): a thread
// owns 4 consecutive source elements (one 16-byte load per split), a block E = 256/SG threads and SG split-groups
// (thread (sg, e) sums splits sg, sg+SG, ... in batches of 8 loads issued before their adds, the SG partials meet in
// LDS in order) -- fixed order, deterministic.  The thread's four read-modify-writes of dw issue their loads
// together: written as four `+=`, each waited for the previous store (possible aliasing), and the 16-byte form ran
// 245 us per trunk fold (tools/bench_fold.py) against 157 us for the 4-byte form it replaces; now ~146 us.
struct FoldRec {
  const float* ws;
  float* dw;
  const int* map;
  int K, C, Creal, RS, splits, SG, blk0, nblk;
};
constexpr int kFoldMaxRecs = 32;
struct FoldTable {
  int n;
  FoldRec r[kFoldMaxRecs];
};

__global__ __launch_bounds__(256) void wgrad_fold_batch_kernel(FoldTable t) {
  __shared__ f32x4 part[256];
  const int v = blockIdx.x;
  const int ri = table_find(t.n, v, [&](int i) { return t.r[i].blk0; });
  const FoldRec& R = t.r[ri];
  const int SG = R.SG, E = 256 / SG, e = threadIdx.x % E, sg = threadIdx.x / E;
  const long row = (long)R.RS * R.C, total = (long)R.K * row;
  const int lb = v - R.blk0;
  const long idx = ((long)lb * E + e) * 4;
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 a0 = zero4, a1 = zero4, a2 = zero4, a3 = zero4;
  const int splits = R.splits;
  if (idx < total) {
    const f32x4* __restrict__ src = reinterpret_cast<const f32x4*>(R.ws + idx);
    const long st = total / 4;
    // this thread's splits z = sg + SG * i, i < n: batches of 8 loads issued before their adds (clamped
    // addresses, zero-selected), chains a0..a3 by i % 4 -- no serial tail
    const int n = splits > sg ? (splits - sg + SG - 1) / SG : 0;
    for (int i0 = 0; i0 < n; i0 += 8) {
      f32x4 w[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int i = i0 + q < n ? i0 + q : n - 1;
        w[q] = src[(long)(sg + SG * i) * st];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (i0 + q < n) {
          if ((q & 3) == 0) a0 += w[q];
          else if ((q & 3) == 1) a1 += w[q];
          else if ((q & 3) == 2) a2 += w[q];
          else a3 += w[q];
        }
    }
  }
  part[threadIdx.x] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (sg != 0 || idx >= total) return;
  f32x4 s4 = zero4;
  for (int q = 0; q < SG; ++q) s4 += part[q * E + e];
  const long per_k = R.map ? (long)R.Creal : (long)R.Creal * R.RS;
  const int k = (int)(idx / row), j0 = (int)(idx - (long)k * row);
  int o[4];
  float d[4];
  float* __restrict__ dwk = R.dw + (long)k * per_k;
#pragma unroll
  for (int c4 = 0; c4 < 4; ++c4) {
    const int j = j0 + c4;
    if (R.map) {
      o[c4] = R.map[j];
    } else {
      const int tap = j / R.C, c = j - tap * R.C;
      o[c4] = c < R.Creal ? c * R.RS + tap : -1;
    }
  }
#pragma unroll
  for (int c4 = 0; c4 < 4; ++c4) d[c4] = dwk[o[c4] >= 0 ? o[c4] : 0];  // the 4 read-modify-writes' loads together
#pragma unroll
  for (int c4 = 0; c4 < 4; ++c4)
    if (o[c4] >= 0) dwk[o[c4]] = d[c4] + s4[c4];
}


// ---------------------------------------------------------------------------------------
// Pipelined fwd / dgrad implicit GEMM: the im2col A tile and the weight tile are DMA'd straight into
// LDS with global_load_lds (16 B per lane), the next K-tile issued before the current one is consumed
// (cdna_hip_programming.md §5 "Minimum 2-phase").  Same XOR-swizzled [rows][64] LDS image as
// gemm_bf16.hip's pipelined kernel.  Zero padding (spatial borders, dgrad's stride holes, K tail,
// rows past M / N) is served by pointing the lane at a 16-byte zero chunk in global memory.
// ---------------------------------------------------------------------------------------

__device__ __forceinline__ int cswz(int row, int c) { return c ^ ((row >> 1) & 7); }
// K-step of CW 16-byte chunks per LDS row: 8 (64-wide, 128-byte rows) or 4 (32-wide, 64-byte rows; four rows share
// a 256-byte bank row, so the XOR takes row bits 2-3 -- the 16 rows one ds_read_b128 lane group reads then cover
// all 16 bank slots)
template <int CW>
__device__ __forceinline__ int cswz_k(int row, int c) {
  return CW == 8 ? (c ^ ((row >> 1) & 7)) : (c ^ ((row >> 2) & 3));
}

template <bool DGRAD>
__device__ __forceinline__ const bf16_t* conv_a_src(const ConvGeom& g, int n, int oh, int ow, bool rowok, int kk,
                                                    float inv_IC, float inv_S) {
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(mer_conv_zero16);
  if (!rowok || kk >= g.Kred) return zero;
  const int tap = fdiv(kk, inv_IC), c = kk - tap * g.IC;
  const int r = fdiv(tap, inv_S), s = tap - r * g.S;
  int ih, iw;
  if (!DGRAD) {
    ih = oh * g.st - g.pad + r;
    iw = ow * g.st - g.pad + s;
  } else {
    const int th = oh + g.pad - r, tw = ow + g.pad - s;
    if (th < 0 || tw < 0) return zero;
    if (g.st == 1) {
      ih = th;
      iw = tw;
    } else {
      if ((th | tw) & 1) return zero;  // st == 2 (checked on the host)
      ih = th >> 1;
      iw = tw >> 1;
    }
  }
  if (ih < 0 || ih >= g.IH || iw < 0 || iw >= g.IW) return zero;
  return g.X + (((long)n * g.IH + ih) * g.IW + iw) * g.IC + c;
}

// Stride-2 dgrad, parity-decomposed (PAR): an input pixel (h, w) only receives taps with
// (h + pad - r) and (w + pad - s) even, so the 4 parity classes (h&1, w&1) (blockIdx.y) are 4 dense
// implicit GEMMs over just their taps -- 1/4 of the MFMA work of the masked 9-tap form for 3x3 and none
// of its zero staging.  Class c: rows (n, hh, ww) -> pixel (n, 2hh+ph, 2ww+pw); taps r = r0 + 2ri,
// s = s0 + 2si with r0 = (ph + pad) & 1; source row ih = hh + (ph + pad - r0)/2 - ri.
struct ParClass {
  int ph, pw, Hc, Wc, r0, s0, nr, ns, dh0, dw0;
};

// Parity class of this block: grid.y walks the classes longest first (3 = odd/odd: 4 taps of a 3x3, then 2, 2, 1)
// -- blocks dispatch y-major, so the long class-3 tiles start first and the short ones fill the tail.
__device__ __forceinline__ int par_cls() { return 3 - (int)blockIdx.y; }

__device__ __forceinline__ ParClass par_class(const ConvGeom& g, int cls) {
  ParClass c;
  c.ph = cls >> 1;
  c.pw = cls & 1;
  c.Hc = (g.OH - c.ph + 1) >> 1;
  c.Wc = (g.OW - c.pw + 1) >> 1;
  c.r0 = (c.ph + g.pad) & 1;
  c.s0 = (c.pw + g.pad) & 1;
  c.nr = (g.R - c.r0 + 1) >> 1;
  c.ns = (g.S - c.s0 + 1) >> 1;
  c.dh0 = (c.ph + g.pad - c.r0) >> 1;
  c.dw0 = (c.pw + g.pad - c.s0) >> 1;
  return c;
}

// Forward BatchNorm statistics of one output tile from the accumulator layout (column = lane & 15: two shuffles per
// value; acc holds the stored, bf16-rounded outputs).  The cross-wave exchanges here and in conv_epilogue_vec go
// through LDS only, so they use lds_barrier() (lgkmcnt(0) + s_barrier): a __syncthreads() would also drain every
// outstanding global store and DMA (vmcnt(0)), which the persistent halo kernel overlaps with its next tile.  The WM waves sharing a column meet in LDS (red: >= WM*WN*TN*2
// idle floats) in wave order; the block then STORES its per-column (sum, sumsq) into stats row stat_row -- every (row
// tile, column) has exactly one writer, so the statistics (and every BatchNorm output) are bitwise deterministic.
// the lane's partial (sum, sumsq) of its accumulator-layout columns j * 16 + (lane & 15) over its rows (< M)
template <int FM, int FN, int WM, int WN>
__device__ __forceinline__ void conv_tile_stats_lane(const ConvGeom& g, const f32x4 (&acc)[FM][FN], int w, int lane,
                                                     int m0, int n0, int M, float (&part)[FN][2]) {
  constexpr int TM = FM * 16, TN = FN * 16;
  const int wr = w / WN, wc = w % WN, fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = n0 + wc * TN + j * 16 + fr;
    float csum = 0.f, csq = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wr * TM + i * 16 + fq * 4 + r;
        if (row < M && col < g.Ncols) {
          const float hv = acc[i][j][r];
          csum += hv;
          csq += hv * hv;
        }
      }
    part[j][0] = csum;
    part[j][1] = csq;
  }
}

// lane partials -> the block's per-column (sum, sumsq) row: two shuffles per value, the WM waves of a column meet in
// LDS (red) in wave order, one writer per element
template <int FN, int WM, int WN>
__device__ __forceinline__ void conv_stats_finish(const ConvGeom& g, float (&part)[FN][2], float* red, int w, int lane,
                                                  int n0, long stat_row) {
  constexpr int TN = FN * 16;
  const int wr = w / WN, wc = w % WN, fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      part[j][q] += __shfl_xor(part[j][q], 16, 64);
      part[j][q] += __shfl_xor(part[j][q], 32, 64);
    }
  lds_barrier();
  if (wr > 0 && fq == 0)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      red[((wr * WN + wc) * FN * 16 + j * 16 + fr) * 2] = part[j][0];
      red[((wr * WN + wc) * FN * 16 + j * 16 + fr) * 2 + 1] = part[j][1];
    }
  lds_barrier();
  if (wr == 0 && fq == 0) {
    float* slab = g.stats + stat_row * g.Ncols * 2;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = n0 + wc * TN + j * 16 + fr;
      float t0 = part[j][0], t1 = part[j][1];
#pragma unroll
      for (int q = 1; q < WM; ++q) {
        t0 += red[((q * WN + wc) * FN * 16 + j * 16 + fr) * 2];
        t1 += red[((q * WN + wc) * FN * 16 + j * 16 + fr) * 2 + 1];
      }
      if (col < g.Ncols) {
        slab[2 * col] = t0;
        slab[2 * col + 1] = t1;
      }
    }
  }
}

template <int FM, int FN, int WM, int WN>
__device__ __forceinline__ void conv_tile_stats(const ConvGeom& g, const f32x4 (&acc)[FM][FN], float* red, int w,
                                                int lane, int m0, int n0, int M, long stat_row) {
  float part[FN][2];
  conv_tile_stats_lane<FM, FN, WM, WN>(g, acc, w, lane, m0, n0, M, part);
  conv_stats_finish<FN, WM, WN>(g, part, red, w, lane, n0, stat_row);
}

// Running per-lane partial sums of a persistent workgroup's tiles (conv_halo_kernel): each tile's fused column
// reductions add into these -- every tile of a workgroup covers the same output columns -- and the cross-lane /
// cross-wave reduction and the partial-row store run ONCE per workgroup (conv_epilogue_acc_finish), not once per tile.
// (vector types rather than arrays: a float[8] member left in scratch once the finish's 16-byte stores were
// vectorised over it)
typedef __attribute__((ext_vector_type(8))) float f32x8;
template <int FN>
struct EpiAcc {
  f32x8 sA, sB, sC;  // dgrad: the BN-backward sums of the lane's 8 pass-layout columns
  float fs[FN][2];   // fwd: the BN statistics of the lane's accumulator-layout columns
  __device__ void zero() {
    sA = sB = sC = f32x8{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < FN; ++j) fs[j][0] = fs[j][1] = 0.f;
  }
};
struct EpiNoAcc {};

// The 16-byte conv epilogue: each wave stages fp32 accumulators of 16-row groups of its TM x TN sub-tile in its own
// slice (WAVE_FLOATS floats at smemf + w * WAVE_FLOATS, idle LDS), then every lane owns 8 consecutive columns of one
// row per pass: 16-byte residual / mask / BN-operand loads and one 16-byte bf16 store instead of 2-byte accesses per
// element.  The fused column reductions (forward BN statistics of the stored bf16 values into stats row stat_row; the
// dgrad's BN-backward sums into bnr_red row red_row_id) accumulate per lane over its rows, then meet across the lanes
// sharing the columns (xor tree) and across the WM waves of a column (LDS, wave order): one writer per partial-row
// element, fixed order.  out_row(row) = the output pixel of GEMM row `row`.  Called by every wave of the workgroup.
// The epilogue's pass geometry: each wave stages GI 16-row groups at a time; a pass moves RPP rows, one per lane
// group of LPR lanes (8 columns each)
template <int FM, int FN, int WAVE_FLOATS>
struct EpiGeo {
  static constexpr int TM = FM * 16, TN = FN * 16, LDT = TN + 4;
  static constexpr int GI0 = WAVE_FLOATS / (16 * LDT);
  static constexpr int GI = GI0 < FM ? GI0 : FM;
  static constexpr int LPR = TN / 8, RPP = 64 / LPR;
  static constexpr int PPG = (GI * 16 + RPP - 1) / RPP;  // passes per staged group
  static constexpr int NP = ((FM + GI - 1) / GI) * PPG;  // passes per tile
};

// The dgrad epilogue's global operands (residual, residual mask, BN mask, BN input(s), BN (mean, rstd) of its 8
// columns), loaded AHEAD of the epilogue -- conv_halo_kernel issues them before its K loop, so their latency hides
// under the MFMAs instead of stalling the epilogue's passes one after another.  Same addresses as the in-epilogue
// loads (rows past M clamped to row M - 1; those passes discard them).
template <int NP>
struct EpiPre {
  u32x4 r[NP], m[NP], bm[NP], x[NP], x2[NP];
  float mu[8], rs[8], mu2[8], rs2[8];
};
struct EpiNone {};

template <bool DGRAD, int FM, int FN, int WM, int WN, int WAVE_FLOATS, class OutRow, int NP, bool X2 = true>
__device__ __forceinline__ void conv_epilogue_prefetch(const ConvGeom& g, EpiPre<NP>& pre, int w, int lane, int m0,
                                                       int n0, int M, OutRow out_row) {
  using E = EpiGeo<FM, FN, WAVE_FLOATS>;
  static_assert(NP == E::NP, "prefetch pass count");
  const int wr = w / WN, wc = w % WN;
  const int lr = lane / E::LPR, lc = (lane % E::LPR) * 8;
  const int colv = n0 + wc * E::TN + lc;
  const bool cok = colv < g.Ncols;
  const bool do_bnr = DGRAD && g.bnr_red != nullptr;
  const bool has_x2 = X2 && do_bnr && g.bnr_x2 != nullptr;
  const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int col = cok ? colv + e : 0;
    pre.mu[e] = do_bnr ? g.bnr_ms[2 * col] : 0.f;
    pre.rs[e] = do_bnr ? g.bnr_ms[2 * col + 1] : 0.f;
    pre.mu2[e] = has_x2 ? g.bnr_ms2[2 * col] : 0.f;
    pre.rs2[e] = has_x2 ? g.bnr_ms2[2 * col + 1] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int i0 = (q / E::PPG) * E::GI, rr = (q % E::PPG) * E::RPP;
    int row = m0 + wr * E::TM + i0 * 16 + rr + lr;
    row = row < M ? row : M - 1;
    const long e0 = out_row(row) * g.ldy + (cok ? colv : 0);
    pre.r[q] = (DGRAD && g.R_) ? *reinterpret_cast<const u32x4*>(g.R_ + e0) : z;
    pre.m[q] = (DGRAD && g.R_ && g.Rmask) ? *reinterpret_cast<const u32x4*>(g.Rmask + e0) : z;
    pre.bm[q] = do_bnr ? *reinterpret_cast<const u32x4*>(g.bnr_mask + e0) : z;
    pre.x[q] = do_bnr ? *reinterpret_cast<const u32x4*>(g.bnr_x + e0) : z;
    pre.x2[q] = has_x2 ? *reinterpret_cast<const u32x4*>(g.bnr_x2 + e0) : z;
  }
}

template <bool DGRAD, int FM, int FN, int WM, int WN, int WAVE_FLOATS, class OutRow, class Pre = EpiNone,
          bool DEFER = false, bool X2 = true, class AccT = EpiNoAcc>
__device__ __forceinline__ void conv_epilogue_vec(const ConvGeom& g, f32x4 (&acc)[FM][FN], float* smemf, int w,
                                                  int lane, int m0, int n0, int M, long red_row_id, long stat_row,
                                                  OutRow out_row, const Pre* pre = nullptr, int ct_slot = -1,
                                                  AccT* accp = nullptr) {
  constexpr bool PREF = !std::is_same<Pre, EpiNone>::value;
  constexpr bool ACC = !std::is_same<AccT, EpiNoAcc>::value;  // add the reductions into *accp, store nothing
  using E = EpiGeo<FM, FN, WAVE_FLOATS>;
  constexpr int TM = FM * 16, TN = FN * 16;
  const int wr = w / WN, wc = w % WN, fr = lane & 15, fq = lane >> 4;
  constexpr int LDT = TN + 4;
  constexpr int GI = E::GI;
  static_assert(GI >= 1, "epilogue staging slice too small");
  constexpr int LPR = TN / 8, RPP = 64 / LPR;
  float* wl = smemf + w * WAVE_FLOATS;
  const int lr = lane / LPR, lc = (lane % LPR) * 8;
  const int colv = n0 + wc * TN + lc;
  const bool cok = colv < g.Ncols;
  const bool do_bnr = DGRAD && g.bnr_red != nullptr;
  const bool has_x2 = X2 && do_bnr && g.bnr_x2 != nullptr;  // X2 = false: compiled out (24 VGPRs)
  float mu[8], rs[8], mu2[8], rs2[8];
  float sA[8], sB[8], sC[8];
  // DEFER (the halo kernel): the 16-byte output stores are issued LAST, after the cross-wave reductions -- a wave
  // stalled issuing stores would otherwise hold every other wave at the reductions' barriers (the store queue
  // drains ~16 B/clk per CU).  The deferred stores hold ~40 VGPRs, which cost conv_pipe_kernel's 8-wave dgrad
  // tiles their second block per CU (127 -> 150 VGPRs: layer2's dgrads 37 -> 56 us), so it stores per pass.
  constexpr int NPS = DEFER ? E::NP : 1;
  u32x4 pend[NPS];
  long pend_at[NPS];
  bool pend_ok[NPS];
#pragma unroll
  for (int q = 0; q < NPS; ++q) pend_ok[q] = false;
  auto flush = [&]() {
#pragma unroll
    for (int q = 0; q < NPS; ++q)
      if (pend_ok[q]) *reinterpret_cast<u32x4*>(g.Y + pend_at[q]) = pend[q];
  };
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if constexpr (PREF) {
      mu[e] = pre->mu[e];
      rs[e] = pre->rs[e];
      mu2[e] = pre->mu2[e];
      rs2[e] = pre->rs2[e];
    } else {
      const int col = cok ? colv + e : 0;
      mu[e] = do_bnr ? g.bnr_ms[2 * col] : 0.f;
      rs[e] = do_bnr ? g.bnr_ms[2 * col + 1] : 0.f;
      mu2[e] = has_x2 ? g.bnr_ms2[2 * col] : 0.f;
      rs2[e] = has_x2 ? g.bnr_ms2[2 * col + 1] : 0.f;
    }
    sA[e] = sB[e] = sC[e] = 0.f;
  }
#pragma unroll
  for (int i0 = 0; i0 < FM; i0 += GI) {
#pragma unroll
    for (int ii = 0; ii < GI; ++ii) {
      if (i0 + ii >= FM) break;
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) wl[(ii * 16 + fq * 4 + r) * LDT + j * 16 + fr] = acc[i0 + ii][j][r];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int nrows = (FM - i0 < GI ? FM - i0 : GI) * 16;
#pragma unroll
    for (int rr = 0; rr < GI * 16; rr += RPP) {
      const int rl = rr + lr;
      const int row = m0 + wr * TM + i0 * 16 + rl;
      if (rl < nrows && row < M && cok) {
        const f32x4 lo = *reinterpret_cast<const f32x4*>(&wl[rl * LDT + lc]);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(&wl[rl * LDT + lc + 4]);
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const long e0 = out_row(row) * g.ldy + colv;
        const int q = (i0 / GI) * E::PPG + rr / RPP;  // this pass's prefetch slot (static once the loops unroll)
        if (DGRAD && g.R_) {
          u32x4 rv, mv;
          if constexpr (PREF) {
            rv = pre->r[q];
            mv = g.Rmask ? pre->m[q] : u32x4{1u, 1u, 1u, 1u};
          } else {
            rv = *reinterpret_cast<const u32x4*>(g.R_ + e0);
            mv = g.Rmask ? *reinterpret_cast<const u32x4*>(g.Rmask + e0) : u32x4{1u, 1u, 1u, 1u};
          }
          const bf16_t* rh = reinterpret_cast<const bf16_t*>(&rv);
          const bf16_t* mh = reinterpret_cast<const bf16_t*>(&mv);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (!g.Rmask || bf2f(mh[e]) > 0.f) v[e] += bf2f(rh[e]);
        }
        u32x4 ov;
        bf16_t* oh = reinterpret_cast<bf16_t*>(&ov);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          oh[e] = f2bf(v[e]);
          v[e] = bf2f(oh[e]);  // the stored value feeds the reductions
        }
        if constexpr (DEFER) {
          pend[q] = ov;
          pend_at[q] = e0;
          pend_ok[q] = true;
        } else {
          *reinterpret_cast<u32x4*>(g.Y + e0) = ov;
        }
        if (do_bnr) {
          u32x4 mv, xv, x2v;
          if constexpr (PREF) {
            mv = pre->bm[q];
            xv = pre->x[q];
            x2v = pre->x2[q];
          } else {
            mv = *reinterpret_cast<const u32x4*>(g.bnr_mask + e0);
            xv = *reinterpret_cast<const u32x4*>(g.bnr_x + e0);
            x2v = has_x2 ? *reinterpret_cast<const u32x4*>(g.bnr_x2 + e0) : u32x4{0u, 0u, 0u, 0u};
          }
          const bf16_t* mh = reinterpret_cast<const bf16_t*>(&mv);
          const bf16_t* xh = reinterpret_cast<const bf16_t*>(&xv);
          const bf16_t* x2h = reinterpret_cast<const bf16_t*>(&x2v);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float gv = bf2f(mh[e]) > 0.f ? v[e] : 0.f;
            sA[e] += gv;
            sB[e] += gv * (bf2f(xh[e]) - mu[e]) * rs[e];
            if (has_x2) sC[e] += gv * (bf2f(x2h[e]) - mu2[e]) * rs2[e];
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (ct_slot >= 0) CT(ct_slot);
  if constexpr (ACC) {
    if (do_bnr) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        accp->sA[e] += sA[e];
        accp->sB[e] += sB[e];
        accp->sC[e] += sC[e];
      }
      flush();
      return;
    }
  }
  if (do_bnr) {
  // lanes sharing this lane's 8 columns: lane % LPR equal -> xor over the row bits of the lane index
#pragma unroll
  for (int o = LPR; o < 64; o <<= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sA[e] += __shfl_xor(sA[e], o, 64);
      sB[e] += __shfl_xor(sB[e], o, 64);
      if (has_x2) sC[e] += __shfl_xor(sC[e], o, 64);
    }
  if (ct_slot >= 0) CT(ct_slot + 3);
  // the WM waves of a column range meet in LDS: red[(wr*WN + wc)][TN][3]
  float* red = smemf;
  lds_barrier();  // every wave is past its staging slice
  if (ct_slot >= 0) CT(ct_slot + 4);
  if (wr > 0 && lane < LPR)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float* o = red + ((wr * WN + wc) * TN + lc + e) * 3;
      o[0] = sA[e];
      o[1] = sB[e];
      o[2] = sC[e];
    }
  lds_barrier();
  if (wr != 0 || lane >= LPR || !cok) {
    flush();
    return;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int q = 1; q < WM; ++q) {
      const float* o = red + ((q * WN + wc) * TN + lc + e) * 3;
      sA[e] += o[0];
      sB[e] += o[1];
      sC[e] += o[2];
    }
  {
    const long slab = red_row_id * g.Ncols * 2 + 2 * colv;
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      *reinterpret_cast<f32x4*>(g.bnr_red + slab + 2 * e) = f32x4{sA[e], sB[e], sA[e + 1], sB[e + 1]};
      if (g.bnr_red2)
        *reinterpret_cast<f32x4*>(g.bnr_red2 + slab + 2 * e) = f32x4{sA[e], sC[e], sA[e + 1], sC[e + 1]};
    }
  }
  if (ct_slot >= 0) CT(ct_slot + 1);
  flush();
  if (ct_slot >= 0) CT(ct_slot + 2);
  return;
  }  // do_bnr
  if (!g.stats) {
    flush();
    return;
  }
  // forward BN statistics from the accumulator layout (column = lane & 15: two shuffles per value, cheaper than
  // the 8-column lane reduction) over the stored, bf16-rounded values
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = bf2f(f2bf(acc[i][j][r]));
  if constexpr (ACC) {
    float part[FN][2];
    conv_tile_stats_lane<FM, FN, WM, WN>(g, acc, w, lane, m0, n0, M, part);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      accp->fs[j][0] += part[j][0];
      accp->fs[j][1] += part[j][1];
    }
    flush();
    return;
  }
  conv_tile_stats<FM, FN, WM, WN>(g, acc, smemf, w, lane, m0, n0, M, stat_row);
  if (ct_slot >= 0) CT(ct_slot + 1);
  flush();
  if (ct_slot >= 0) CT(ct_slot + 2);
}

// The workgroup's accumulated reductions (EpiAcc) -> its one partial row: the dgrad's BN-backward sums meet across the
// lanes sharing columns (xor tree) and the WM waves (LDS, wave order) as in conv_epilogue_vec; the forward statistics
// as in conv_stats_finish.  Called by every wave, with smemf free LDS.
template <bool DGRAD, int FM, int FN, int WM, int WN, int WAVE_FLOATS, bool X2 = true>
__device__ __forceinline__ void conv_epilogue_acc_finish(const ConvGeom& g, EpiAcc<FN>& a, float* smemf, int w,
                                                         int lane, int n0, long row_id) {
  if constexpr (DGRAD) {
    if (!g.bnr_red) return;
    using E = EpiGeo<FM, FN, WAVE_FLOATS>;
    constexpr int TN = FN * 16, LPR = E::LPR;
    const int wr = w / WN, wc = w % WN;
    const int lc = (lane % LPR) * 8;
    const int colv = n0 + wc * TN + lc;
    const bool cok = colv < g.Ncols;
    const bool has_x2 = X2 && g.bnr_x2 != nullptr;
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        a.sA[e] += __shfl_xor(a.sA[e], o, 64);
        a.sB[e] += __shfl_xor(a.sB[e], o, 64);
        if (has_x2) a.sC[e] += __shfl_xor(a.sC[e], o, 64);
      }
    float* red = smemf;
    lds_barrier();
    if (wr > 0 && lane < LPR)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float* o = red + ((wr * WN + wc) * TN + lc + e) * 3;
        o[0] = a.sA[e];
        o[1] = a.sB[e];
        o[2] = a.sC[e];
      }
    lds_barrier();
    if (wr != 0 || lane >= LPR || !cok) return;
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int q = 1; q < WM; ++q) {
        const float* o = red + ((q * WN + wc) * TN + lc + e) * 3;
        a.sA[e] += o[0];
        a.sB[e] += o[1];
        a.sC[e] += o[2];
      }
    const long slab = row_id * g.Ncols * 2 + 2 * colv;
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      *reinterpret_cast<f32x4*>(g.bnr_red + slab + 2 * e) = f32x4{a.sA[e], a.sB[e], a.sA[e + 1], a.sB[e + 1]};
      if (g.bnr_red2)
        *reinterpret_cast<f32x4*>(g.bnr_red2 + slab + 2 * e) = f32x4{a.sA[e], a.sC[e], a.sA[e + 1], a.sC[e + 1]};
    }
  } else {
    if (!g.stats) return;
    conv_stats_finish<FN, WM, WN>(g, a.fs, smemf, w, lane, n0, row_id);
  }
}

// Minimum waves per SIMD of a conv_pipe_kernel block of nw waves: 16-wave blocks 1 per CU, 8-wave blocks 2 per CU --
// except the tiles that would spill at 128 VGPRs (the 256-row dgrad tiles and the 3-deep 128 x 128 dgrad ring, none of
// them a default pick), which keep one block per CU; 4-wave blocks 2 per CU.
// A block whose LDS leaves no room for a second one on the CU (160 KB) asks for nw / 4 (its own waves only).
constexpr int conv_pipe_wpe(int nw, int bm, int bn, int stages, bool dgrad, bool par, int lds_bytes = 0) {
  return (nw >= 16 || 2 * lds_bytes > 160 * 1024)
             ? (nw >= 4 ? nw / 4 : 1)
             : nw == 8 ? ((dgrad && (bm == 256 || (!par && bm == 128 && bn == 128 && stages == 3))) ? 2 : 4) : 2;
}
// dynamic LDS of a conv_pipe_kernel instantiation: KG rings, or the split-K tile exchange if larger
constexpr int conv_pipe_lds(int bm, int bn, int stages, int ks, int kg) {
  return kg * stages * (bm + bn) * ks * 2 > (kg > 1 ? kg * bm * (bn + 4) * 4 : 0)
             ? kg * stages * (bm + bn) * ks * 2
             : kg * bm * (bn + 4) * 4;
}

// The wave layout of the in-workgroup split-K reduction (KG > 1): WAVES * KG waves over the BM x BN tile, 4 wave
// rows when that leaves >= 16-row / 16-column sub-tiles.
template <int BM_, int BN_, int NW>
struct KgLayout {
  static constexpr int WM = (NW >= 4 && BM_ / 4 >= 16) ? 4 : (NW >= 2 ? 2 : 1);
  static constexpr int WN = NW / WM;
  static_assert(WM * WN == NW && BM_ % (16 * WM) == 0 && BN_ % (16 * WN) == 0, "split-K epilogue layout");
};

// STAGES-deep LDS ring (cdna_hip_programming.md "Pipelining across barriers"): tiles kt+1 .. kt+STAGES-2 stay
// in flight across the barrier that publishes tile kt (counted vmcnt, raw s_barrier); the barrier also retires
// every wave's reads of tile kt-1, whose buffer the DMA of tile kt+STAGES-1 then reuses.
//
// KG > 1: in-workgroup split-K.  The small-M layers (ResNet18 layer3 / layer4: 12,544 / 4,096 GEMM rows) have one
// 64 x 128 tile per CU, and one 8-wave tile per CU leaves the K loop latency-bound (0.15-0.18 of the MFMA peak).
// KG K-groups of WM x WN waves each own a ring of their own and a contiguous 1/KG of the K-steps, all groups stepping
// through the same barriers; at the end every group stores its fp32 tile to LDS and the WAVES * KG waves re-split the
// tile (KgLayout), each element summed over the groups in group order -- deterministic, no global partials, and the
// fused epilogue (BN statistics / BN-backward sums) runs unchanged on the summed tile.
template <bool DGRAD, bool PAR, int BM_, int BN_, int WM = 2, int WN = 2, int STAGES = 2, int KS = 64, bool X2 = true,
          int KG = 1>
// (__launch_bounds__'s second argument is amdgpu_waves_per_eu, a minimum of waves per SIMD: two 8-wave blocks per CU need
// 4, i.e. <= 128 VGPRs -- with 2, the parity-class dgrad tile took 131 VGPRs and ran one block per CU)
__global__ __launch_bounds__(64 * WM * WN * KG, conv_pipe_wpe(WM * WN * KG, BM_, BN_, STAGES, DGRAD, PAR,
                                                              conv_pipe_lds(BM_, BN_, STAGES, KS, KG))) void conv_pipe_kernel(ConvGeom g) {
  constexpr int WAVES = WM * WN;  // per K-group
  constexpr int CW = KS / 8, RPG = 64 / CW;  // 16-byte chunks per LDS row, rows per glds instruction
  constexpr int IA = BM_ / RPG / WAVES, IB = BN_ / RPG / WAVES;  // glds per wave per K-tile
  static_assert(IA * RPG * WAVES == BM_ && IB * RPG * WAVES == BN_, "tile rows must split into whole glds pieces");
  static_assert(KS == 64 || KS == 32, "K-tile");
  static_assert(KG == 1 || KG == 2 || KG == 4, "K-groups");
  constexpr int TM = BM_ / WM, TN = BN_ / WN, FM = TM / 16, FN = TN / 16;
  constexpr int BUF = (BM_ + BN_) * KS;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem_all[];
  const int t = threadIdx.x, lane = t & 63, kg = (t >> 6) / WAVES, w = (t >> 6) % WAVES;
  bf16_t* const smem = smem_all + kg * STAGES * BUF;  // this K-group's ring
  ParClass pc{};
  int M, Kr, rowsH, rowsW;  // this launch's GEMM rows / reduction length, row -> (n, a, b) grid
  int Kr0 = 0;              // PAR: the 3x3 taps' share of Kr (the fused downsample segment follows it in class 0)
  if (PAR) {
    pc = par_class(g, par_cls());
    M = g.N * pc.Hc * pc.Wc;
    Kr0 = pc.nr * pc.ns * g.IC;
    Kr = Kr0 + ((g.X2 && pc.ph == 0 && pc.pw == 0) ? g.K2 : 0);
    rowsH = pc.Hc;
    rowsW = pc.Wc;
  } else {
    M = g.N * g.OH * g.OW;
    Kr = g.Kred;
    rowsH = g.OH;
    rowsW = g.OW;
  }
  const int nx = (g.Ncols + BN_ - 1) / BN_, ny = (M + BM_ - 1) / BM_;
  if ((int)blockIdx.x >= nx * ny) return;  // grid sized for the largest parity class
  CTP(0);
  int tx, ty;
  xcd_tile(blockIdx.x, nx, nx * ny, tx, ty);
  const int m0 = ty * BM_, n0 = tx * BN_;
  const int wr = w / WN, wc = w % WN;

  int an[IA], aoh[IA], aow[IA], acl[IA];
  bool aok[IA];
#pragma unroll
  for (int j = 0; j < IA; ++j) {
    const int r = (w * IA + j) * RPG + lane / CW;
    const int m = m0 + r;
    aok[j] = m < M;
    const int mm = aok[j] ? m : 0;
    an[j] = mm / (rowsH * rowsW);
    const int rem = mm - an[j] * rowsH * rowsW;
    aoh[j] = rem / rowsW;
    aow[j] = rem - aoh[j] * rowsW;
    acl[j] = cswz_k<CW>(r, lane % CW) * 8;
  }
  const bf16_t* pb[IB];
  const bf16_t* pb2[IB];
  int bcl[IB];
  bool bok[IB];
#pragma unroll
  for (int j = 0; j < IB; ++j) {
    const int r = (w * IB + j) * RPG + lane / CW;
    const int n = n0 + r;
    bok[j] = n < g.Ncols;
    pb[j] = g.Wt + (long)(bok[j] ? n : 0) * g.Kred;
    pb2[j] = g.Wt2 + (long)(bok[j] ? n : 0) * g.K2;  // (unused unless the downsample segment is fused)
    bcl[j] = cswz_k<CW>(r, lane % CW) * 8;
  }
  const float inv_IC = 1.f / g.IC, inv_S = 1.f / g.S, inv_ns = PAR ? 1.f / pc.ns : 1.f;
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(mer_conv_zero16);
  // class-local reduction index kk -> (ri, si, c) -> source; the weight operand's offset of the same kk
  auto par_a_src = [&](int n, int hh, int ww, bool rowok, int kk) -> const bf16_t* {
    if (!rowok || kk >= Kr) return zero;
    if (kk >= Kr0)  // the fused downsample segment (class 0): its output pixel (hh, ww) is the input pixel (2hh, 2ww)
      return g.X2 + (((long)n * g.IH + hh) * g.IW + ww) * g.K2 + (kk - Kr0);
    const int tap = fdiv(kk, inv_IC), c = kk - tap * g.IC;
    const int ri = fdiv(tap, inv_ns), si = tap - ri * pc.ns;
    const int ih = hh + pc.dh0 - ri, iw = ww + pc.dw0 - si;
    if (ih < 0 || ih >= g.IH || iw < 0 || iw >= g.IW) return zero;
    return g.X + (((long)n * g.IH + ih) * g.IW + iw) * g.IC + c;
  };
  auto par_b_off = [&](int kk) -> int {
    const int tap = fdiv(kk, inv_IC), c = kk - tap * g.IC;
    const int ri = fdiv(tap, inv_ns), si = tap - ri * pc.ns;
    return ((pc.r0 + 2 * ri) * g.S + pc.s0 + 2 * si) * g.IC + c;
  };
  auto stage = [&](int buf, int k0) {
    bf16_t* la = smem + buf * BUF;
    bf16_t* lb = la + BM_ * KS;
#pragma unroll
    for (int j = 0; j < IA; ++j) {
      const bf16_t* src = PAR ? par_a_src(an[j], aoh[j], aow[j], aok[j], k0 + acl[j])
                              : conv_a_src<DGRAD>(g, an[j], aoh[j], aow[j], aok[j], k0 + acl[j], inv_IC, inv_S);
      glds16(src, la + (w * IA + j) * 512);
    }
#pragma unroll
    for (int j = 0; j < IB; ++j) {
      const int kk = k0 + bcl[j];
      const bool ok = bok[j] && kk < Kr;
      const bf16_t* src = !PAR ? pb[j] + kk : (kk >= Kr0 ? pb2[j] + (kk - Kr0) : pb[j] + par_b_off(kk));
      glds16(ok ? src : zero, lb + (w * IB + j) * 512);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  // this K-group's K-steps: [kb, kb + nk) of the tile's nk_all; every group runs the loop nkg times (the barriers are
  // workgroup-wide), a group with fewer steps idles through its last ones
  const int nk_all = (Kr + KS - 1) / KS;
  const int nkg = (nk_all + KG - 1) / KG, kb = kg * nkg;
  const int nk = nk_all - kb < nkg ? (nk_all - kb > 0 ? nk_all - kb : 0) : nkg;
  const int kofs = kb * KS;
  constexpr int G = IA + IB;
  static_assert(STAGES >= 2 && STAGES <= 4, "ring depth");
#pragma unroll
  for (int p = 0; p < STAGES - 1; ++p)
    if (p < nk) stage(p, kofs + p * KS);
  CTP(1);
  for (int kt = 0; kt < nkg; ++kt) {
    const int left = nk - 1 - kt;
    const int ahead = left < (STAGES - 2) ? left : (STAGES - 2);
    wait_tiles_in_flight<G>(ahead);
    lds_barrier();
    if (kt + STAGES - 1 < nk) stage((kt + STAGES - 1) % STAGES, kofs + (kt + STAGES - 1) * KS);
    if (KG > 1 && kt >= nk) continue;
    const bf16_t* la = smem + (kt % STAGES) * BUF;
    const bf16_t* lb = la + BM_ * KS;
#pragma unroll
    for (int s = 0; s < KS / 32; ++s) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wr * TM + i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(la + r * KS + cswz_k<CW>(r, s * 4 + fq) * 8);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wc * TN + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(lb + r * KS + cswz_k<CW>(r, s * 4 + fq) * 8);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  CTP(2);

  // output row -> element offset of the pixel in Y
  auto out_row = [&](int row) -> long {
    if (!PAR) return (long)row;
    const int n = row / (pc.Hc * pc.Wc);
    const int rem = row - n * pc.Hc * pc.Wc;
    const int hh = rem / pc.Wc, ww = rem - hh * pc.Wc;
    return ((long)n * g.OH + 2 * hh + pc.ph) * g.OW + 2 * ww + pc.pw;
  };
  // partial-row index of this tile for the fused reductions: ty, after the row tiles of the preceding parity
  // classes in the PAR (stride-2) form
  auto red_row = [&]() -> long {
    long row_id = ty;
    if (PAR)
      for (int c2 = 0; c2 < par_cls(); ++c2) {
        const ParClass q = par_class(g, c2);
        row_id += (g.N * q.Hc * q.Wc + BM_ - 1) / BM_;
      }
    return row_id;
  };
  // One-pass input-gradient epilogues load their operands (residual, its mask, the BN mask and input(s), BN (mean, rstd))
  // right after the K loop, so the latency hides under the barrier / split-K exchange.  (Loading every pass's operands
  // there for the multi-pass tiles needs 20 VGPRs per pass: the 128 x 128 tiles then spill.)
  constexpr int EWF = STAGES * BUF / 2 / WAVES;  // epilogue staging floats per wave
  const int ct_slot = 10;  // (timing build: stamps inside the epilogue, CT slots 10..12)
  if constexpr (KG > 1) {  // (the launcher takes KG > 1 only with the 16-byte epilogue)
    using L = KgLayout<BM_, BN_, WAVES * KG>;
    constexpr int LDR = BN_ + 4;  // padded fp32 rows: a fragment's 4 row quads fall on distinct bank groups
    constexpr int TM2 = BM_ / L::WM, TN2 = BN_ / L::WN, FM2 = TM2 / 16, FN2 = TN2 / 16;
    using E2 = EpiGeo<FM2, FN2, EWF>;
    const int w2 = t >> 6, wr2 = w2 / L::WN, wc2 = w2 % L::WN;
    constexpr bool PF = DGRAD && E2::NP == 1;
    EpiPre<E2::NP> pre;
    if constexpr (PF)
      conv_epilogue_prefetch<DGRAD, FM2, FN2, L::WM, L::WN, EWF, decltype(out_row), E2::NP, X2>(g, pre, w2, lane, m0,
                                                                                                n0, M, out_row);
    __syncthreads();  // every wave's last fragment reads are done before the exchange reuses the ring
    float* const part = reinterpret_cast<float*>(smem_all);
    {
      float* mine = part + kg * BM_ * LDR;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) mine[(wr * TM + i * 16 + fq * 4 + r) * LDR + wc * TN + j * 16 + fr] = acc[i][j][r];
    }
    lds_barrier();
    f32x4 acc2[FM2][FN2];
#pragma unroll
    for (int i = 0; i < FM2; ++i)
#pragma unroll
      for (int j = 0; j < FN2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int e = (wr2 * TM2 + i * 16 + fq * 4 + r) * LDR + wc2 * TN2 + j * 16 + fr;
          float s = part[e];
#pragma unroll
          for (int q = 1; q < KG; ++q) s += part[q * BM_ * LDR + e];  // group order: fixed
          acc2[i][j][r] = s;
        }
    lds_barrier();  // every wave holds its sums before the epilogue reuses the LDS
    CTP(3);
    if constexpr (PF)
      conv_epilogue_vec<DGRAD, FM2, FN2, L::WM, L::WN, EWF, decltype(out_row), decltype(pre), false, X2>(
          g, acc2, reinterpret_cast<float*>(smem_all), w2, lane, m0, n0, M, g.bnr_red ? red_row() : 0l, ty, out_row,
          &pre, ct_slot);
    else
      conv_epilogue_vec<DGRAD, FM2, FN2, L::WM, L::WN, EWF, decltype(out_row), EpiNone, false, X2>(
          g, acc2, reinterpret_cast<float*>(smem_all), w2, lane, m0, n0, M, (DGRAD && g.bnr_red) ? red_row() : 0l, ty,
          out_row, static_cast<const EpiNone*>(nullptr), ct_slot);
    CTP(4);
    return;
  }
  if (g.vec) {
    using E1 = EpiGeo<FM, FN, EWF>;
    if constexpr (DGRAD && E1::NP == 1) {
      EpiPre<E1::NP> pre;
      conv_epilogue_prefetch<DGRAD, FM, FN, WM, WN, EWF, decltype(out_row), E1::NP, X2>(g, pre, w, lane, m0, n0, M,
                                                                                         out_row);
      __syncthreads();  // every wave's last fragment reads are done before the epilogue reuses the ring
      CTP(3);
      conv_epilogue_vec<DGRAD, FM, FN, WM, WN, EWF, decltype(out_row), decltype(pre), false, X2>(
          g, acc, reinterpret_cast<float*>(smem), w, lane, m0, n0, M, g.bnr_red ? red_row() : 0l, ty, out_row, &pre,
          ct_slot);
    } else {
      __syncthreads();  // every wave's last fragment reads are done before the epilogue reuses the ring
      CTP(3);
      conv_epilogue_vec<DGRAD, FM, FN, WM, WN, EWF, decltype(out_row), EpiNone, false, X2>(
          g, acc, reinterpret_cast<float*>(smem), w, lane, m0, n0, M, (DGRAD && g.bnr_red) ? red_row() : 0l, ty,
          out_row, static_cast<const EpiNone*>(nullptr), ct_slot);
    }
    CTP(4);
    return;
  } else {
  __syncthreads();
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wr * TM + i * 16 + fq * 4 + r;
      if (row >= M) continue;
      const long orow = out_row(row) * g.ldy;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = n0 + wc * TN + j * 16 + fr;
        if (col >= g.Ncols) continue;
        float v = acc[i][j][r];
        if (g.R_) {
          const long ri = orow + col;
          if (!g.Rmask || bf2f(g.Rmask[ri]) > 0.f) v += bf2f(g.R_[ri]);
        }
        const bf16_t h = f2bf(v);
        g.Y[orow + col] = h;
        acc[i][j][r] = bf2f(h);  // the stored value feeds the BN statistics
      }
    }
  if (DGRAD && g.bnr_red) {
    // fused bn_bwd_reduce over this tile's stored gradient: 3 sums per column (g, g*xhat, g*xhat2)
    float ps[FN][3];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = n0 + wc * TN + j * 16 + fr;
      const bool cok = col < g.Ncols;
      const float mu = cok ? g.bnr_ms[2 * col] : 0.f, rs = cok ? g.bnr_ms[2 * col + 1] : 0.f;
      const float mu2 = (cok && g.bnr_x2) ? g.bnr_ms2[2 * col] : 0.f;
      const float rs2 = (cok && g.bnr_x2) ? g.bnr_ms2[2 * col + 1] : 0.f;
      float s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wr * TM + i * 16 + fq * 4 + r;
          if (row < M && cok) {
            const long e = out_row(row) * g.ldy + col;
            const float gv = bf2f(g.bnr_mask[e]) > 0.f ? acc[i][j][r] : 0.f;
            s1 += gv;
            s2 += gv * (bf2f(g.bnr_x[e]) - mu) * rs;
            if (g.bnr_x2) s3 += gv * (bf2f(g.bnr_x2[e]) - mu2) * rs2;
          }
        }
#pragma unroll
      for (int o = 16; o < 64; o <<= 1) {
        s1 += __shfl_xor(s1, o, 64);
        s2 += __shfl_xor(s2, o, 64);
        s3 += __shfl_xor(s3, o, 64);
      }
      ps[j][0] = s1;
      ps[j][1] = s2;
      ps[j][2] = s3;
    }
    // the WM waves sharing a column meet in LDS (staging buffers idle now): red[wr][col][3]
    float* red = reinterpret_cast<float*>(smem);
    __syncthreads();
    if (wr > 0 && fq == 0)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int q = 0; q < 3; ++q) red[((wr * WN + wc) * FN * 16 + j * 16 + fr) * 3 + q] = ps[j][q];
    __syncthreads();
    if (wr == 0 && fq == 0) {
      // this block's own partial row (single writer per element -> deterministic after the fixed-order fold):
      // row = ty, after the row tiles of the preceding parity classes in the PAR (stride-2) form
      long row_id = ty;
      if (PAR)
        for (int c2 = 0; c2 < par_cls(); ++c2) {
          const ParClass q = par_class(g, c2);
          row_id += (g.N * q.Hc * q.Wc + BM_ - 1) / BM_;
        }
      const long slab = row_id * g.Ncols * 2;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = n0 + wc * TN + j * 16 + fr;
        float t0 = ps[j][0], t1 = ps[j][1], t2 = ps[j][2];
#pragma unroll
        for (int q = 1; q < WM; ++q) {
          const float* o = red + ((q * WN + wc) * FN * 16 + j * 16 + fr) * 3;
          t0 += o[0];
          t1 += o[1];
          t2 += o[2];
        }
        if (col < g.Ncols) {
          g.bnr_red[slab + 2 * col] = t0;
          g.bnr_red[slab + 2 * col + 1] = t1;
          if (g.bnr_red2) {
            g.bnr_red2[slab + 2 * col] = t0;
            g.bnr_red2[slab + 2 * col + 1] = t2;
          }
        }
      }
    }
  }
  }  // !g.vec
  if (g.stats) conv_tile_stats<FM, FN, WM, WN>(g, acc, reinterpret_cast<float*>(smem), w, lane, m0, n0, M, ty);
}

template <bool DGRAD, bool PAR, int BM_, int BN_, int WM = 2, int WN = 2, int STAGES = 2, int KS = 64, int KG = 1>
int launch_conv_pipe_t(ConvGeom& g, hipStream_t st) {
  // PAR: grid.x covers the largest parity class (ph = pw = 0), grid.y = the 4 classes
  const int Mg = PAR ? g.N * ((g.OH + 1) / 2) * ((g.OW + 1) / 2) : g.N * g.OH * g.OW;
  const long tiles = (long)((Mg + BM_ - 1) / BM_) * ((g.Ncols + BN_ - 1) / BN_);
  const size_t ring = (size_t)KG * STAGES * (BM_ + BN_) * KS * sizeof(bf16_t);
  const size_t kgred = KG > 1 ? (size_t)KG * BM_ * (BN_ + 4) * sizeof(float) : 0;  // the split-K tile exchange
  const size_t lds = ring > kgred ? ring : kgred;
  if (KG > 1 && !g.vec) return (int)hipErrorInvalidValue;  // the split-K form has the 16-byte epilogue only
  // a stride-1 input gradient whose BN-backward target has no second (downsample) branch runs the instantiation
  // without the x2 terms: 24 fewer VGPRs, which keeps the 8-wave tiles at 2 blocks per CU
  if constexpr (DGRAD && !PAR) {
    if (!g.bnr_x2) {
      if (hipFuncSetAttribute(
              reinterpret_cast<const void*>(&conv_pipe_kernel<DGRAD, PAR, BM_, BN_, WM, WN, STAGES, KS, false, KG>),
              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return (int)hipErrorInvalidConfiguration;
      hipLaunchKernelGGL((conv_pipe_kernel<DGRAD, PAR, BM_, BN_, WM, WN, STAGES, KS, false, KG>),
                         dim3((unsigned)tiles, 1), dim3(64 * WM * WN * KG), lds, st, g);
      return (int)hipGetLastError();
    }
  }
  if (hipFuncSetAttribute(
          reinterpret_cast<const void*>(&conv_pipe_kernel<DGRAD, PAR, BM_, BN_, WM, WN, STAGES, KS, true, KG>),
          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return (int)hipErrorInvalidConfiguration;
  hipLaunchKernelGGL((conv_pipe_kernel<DGRAD, PAR, BM_, BN_, WM, WN, STAGES, KS, true, KG>),
                     dim3((unsigned)tiles, PAR ? 4 : 1), dim3(64 * WM * WN * KG), lds, st, g);
  return (int)hipGetLastError();
}

// variant 1: 4-wave tiles; variant 2 (default): 8-wave tiles -- more waves per CU hide the DMA latency of
// the 2-deep pipeline (tools/bench_conv.py: 1.1-1.3x on every ResNet layer), cf. gemm_bf16.hip
// pick_variant; variant 3: 16-wave 256-row tiles on the large-M layers.
template <bool DGRAD, bool PAR>
int launch_conv_pipe(ConvGeom& g, hipStream_t st, int variant) {
  const int M = PAR ? g.N * g.OH * g.OW / 4 : g.N * g.OH * g.OW;
  const int bn = g.Ncols <= 64 ? 64 : 128;
  const long tiles128 = (long)((M + 127) / 128) * ((g.Ncols + bn - 1) / bn) * (PAR ? 4 : 1);
  // below 384 128-row tiles, 64-row tiles (128-row tiles on the deep layers lose 3.5 % of the step)
  const bool small_m = tiles128 < 384;
  if (variant == 7) {  // in-workgroup split-K (two K-groups) on the 64-row tiles
    if (bn == 64)
      return PAR ? launch_conv_pipe_t<DGRAD, PAR, 64, 64, 2, 2, 2, 64, 2>(g, st)
                 : launch_conv_pipe_t<DGRAD, PAR, 64, 64, 2, 2, 3, 64, 2>(g, st);
    return PAR ? launch_conv_pipe_t<DGRAD, PAR, 64, 128, 2, 4, 2, 64, 2>(g, st)
               : launch_conv_pipe_t<DGRAD, PAR, 64, 128, 2, 4, 3, 64, 2>(g, st);
  }
  if (variant == 3 && !small_m) {  // 256-row tiles (8 / 16 waves) for the large-M layers
    // (the 16-wave dgrad tile needs more than 128 VGPRs and would spill to scratch: 8-wave 256 x 64 tiles instead;
    // tools/check_scratch.py keeps every kernel of the library scratch-free)
    if constexpr (DGRAD) {
      return launch_conv_pipe_t<DGRAD, PAR, 256, 64, 4, 2>(g, st);
    } else {
      if (bn == 64) return launch_conv_pipe_t<DGRAD, PAR, 256, 64, 4, 2>(g, st);
      return launch_conv_pipe_t<DGRAD, PAR, 256, 128, 4, 4>(g, st);
    }
  }
  if (variant == 5) {  // 32-wide K-tiles on a 4-deep ring (three K-tiles in flight), 4-wave tiles
    if (bn == 64)
      return small_m ? launch_conv_pipe_t<DGRAD, PAR, 64, 64, 2, 2, 4, 32>(g, st)
                     : launch_conv_pipe_t<DGRAD, PAR, 128, 64, 2, 2, 4, 32>(g, st);
    return small_m ? launch_conv_pipe_t<DGRAD, PAR, 64, 128, 2, 2, 4, 32>(g, st)
                   : launch_conv_pipe_t<DGRAD, PAR, 128, 128, 2, 4, 4, 32>(g, st);
  }
  if (variant == 4) {  // variant-2 tiles on a 3-deep ring (two K-tiles in flight across each barrier)
    if (bn == 64)
      return small_m ? launch_conv_pipe_t<DGRAD, PAR, 64, 64, 2, 2, 3>(g, st)
                     : launch_conv_pipe_t<DGRAD, PAR, 128, 64, 4, 2, 3>(g, st);
    return small_m ? launch_conv_pipe_t<DGRAD, PAR, 64, 128, 2, 4, 3>(g, st)
                   : launch_conv_pipe_t<DGRAD, PAR, 128, 128, 2, 4, 3>(g, st);
  }
  if (variant >= 2) {
    // deep layers (small M, one 64-row tile per CU or fewer): a 3-deep ring keeps two K-tiles in flight
    // (tools/bench_conv.py: layer4 3x3 fwd 54.6 -> 44.8 us, dgrad 55.1 -> 47.1 us; the parity-class dgrad
    // and the large-M layers run best on the 2-deep ring at 2 blocks per CU)
    if (bn == 64)
      return small_m ? (PAR ? launch_conv_pipe_t<DGRAD, PAR, 64, 64, 2, 2>(g, st)
                            : launch_conv_pipe_t<DGRAD, PAR, 64, 64, 2, 2, 3>(g, st))
                     : launch_conv_pipe_t<DGRAD, PAR, 128, 64, 4, 2>(g, st);
    // (a stride-1 input gradient with a second BN-backward branch -- x2: the block-0 output of layers 2-4 -- used to
    // take the 64 x 128 tile because the 128 x 128 one needed 138 VGPRs; bounded to 128 (conv_pipe_wpe) it runs two
    // blocks per CU without spilling: layer2.1.conv1's dgrad 54.0 -> 39.4 us, profiles/r06/bench_conv_x2.txt)
    return small_m ? (PAR ? launch_conv_pipe_t<DGRAD, PAR, 64, 128, 2, 4>(g, st)
                          : launch_conv_pipe_t<DGRAD, PAR, 64, 128, 2, 4, 3>(g, st))
                   : launch_conv_pipe_t<DGRAD, PAR, 128, 128, 2, 4>(g, st);
  }
  if (bn == 64)
    return small_m ? launch_conv_pipe_t<DGRAD, PAR, 64, 64>(g, st) : launch_conv_pipe_t<DGRAD, PAR, 128, 64>(g, st);
  return small_m ? launch_conv_pipe_t<DGRAD, PAR, 64, 128>(g, st) : launch_conv_pipe_t<DGRAD, PAR, 128, 128>(g, st);
}

template <bool DGRAD>
int launch_conv(ConvGeom& g, hipStream_t st) {
  const int M = g.N * g.OH * g.OW;
  const int bn = g.Ncols <= 64 ? 64 : 128;
  const long tiles128 = (long)((M + 127) / 128) * ((g.Ncols + bn - 1) / bn);
  const bool small_m = tiles128 < 384;  // deep layers (layer3/4): halve BM so the grid fills 256 CUs
  const int nx = (g.Ncols + bn - 1) / bn;
  if (bn == 64) {
    if (small_m) {
      hipLaunchKernelGGL((conv_kernel<DGRAD, 64, 64>), dim3(nx * ((M + 63) / 64)), dim3(256), 0, st, g);
    } else {
      hipLaunchKernelGGL((conv_kernel<DGRAD, 128, 64>), dim3(nx * ((M + 127) / 128)), dim3(256), 0, st, g);
    }
  } else {
    if (small_m) {
      hipLaunchKernelGGL((conv_kernel<DGRAD, 64, 128>), dim3(nx * ((M + 63) / 64)), dim3(256), 0, st, g);
    } else {
      hipLaunchKernelGGL((conv_kernel<DGRAD, 128, 128>), dim3(nx * ((M + 127) / 128)), dim3(256), 0, st, g);
    }
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Stride-1 convolutions of 64 output channels with the whole weight resident in LDS: ResNet18 layer1 (3x3, pad 1,
// 64 -> 64 channels on 28x28 maps at 112^2 frames; forward and input gradient) and the stem in its space-to-depth form
// (4x4, pad 0, 16 -> 64 channels: 59x59 -> 56x56).  conv_pipe_kernel re-fetches every input pixel from L2 once per
// tap and waits one DMA round trip per 64-deep K-step with ~8 MFMAs per wave behind it: latency-bound, layer1 ran at
// 200-380 TF/s and the stem at ~195.  Here persistent workgroups keep the packed weight [64][R*S*C] resident in LDS
// (layer1 73.7 KB, stem 32 KB) and stage, per 128-pixel output tile, the HALO its taps read -- the input rows the
// tile's output rows need, (W + R - 1) pixels wide with zero border columns -- double-buffered, so tile i+1's halo
// streams in while tile i computes.  The K loop is LDS -> MFMA only: no global load, no barrier.  The A fragment of
// tap (r, s) for output pixel (n, y, x) is halo pixel (n*IH + y + r - pad - base, x + s), the same 16 bytes
// conv_pipe_kernel gathers; K-steps run in the same (tap, channel) order on the same MFMA with the same wave layout
// and epilogue (conv_epilogue_vec), so outputs and BN statistics are bit-identical to conv_pipe_kernel's
// (tests/test_resnet_gpu.py).  Both LDS images are XOR-swizzled per 16-byte chunk so a fragment's 16 rows fall on 16
// distinct bank slots.
// ---------------------------------------------------------------------------------------
namespace halo {
constexpr int BM = 128;  // output pixels per tile
// C input channels, R x R taps, pad, W output width, IHX = IH - OH (input rows beyond the output rows: the stem's 3),
// ROWS halo rows: the image rows 128 consecutive output pixels span + R - 1, + IHX when a tile may straddle frames
template <int C_, int R_, int PAD_, int W_, int IHX_>
struct Geo {
  static constexpr int C = C_, R = R_, PAD = PAD_, W = W_, IHX = IHX_;
  static constexpr int KRED = R * R * C, WCH = KRED / 8;    // reduction, 16-byte chunks per weight row
  static constexpr int CPP = C / 8;                         // chunks per halo pixel
  static constexpr int HW = W + R - 1;                      // halo row width (pixels)
  static constexpr int ROWS = (W + BM - 2) / W + 1 + (R - 1) + IHX;
  static constexpr int CH = (ROWS * HW * CPP + 63) / 64 * 64;  // 16-byte chunks per halo buffer (whole glds pieces)
  static constexpr int ELEMS = CH * 8;                         // bf16 elements per halo buffer
  static constexpr int LDS_ELEMS = 64 * KRED + 2 * ELEMS + C;  // weights, two halo buffers, one zero pixel
  static constexpr int KSTEPS = KRED / 32;
  static constexpr int HSHIFT = CPP == 8 ? 1 : 3;  // halo swizzle: chunk c of pixel p at c ^ ((p >> HSHIFT) & (CPP-1))
  static_assert(CPP == 8 || CPP == 2, "halo layouts for 16 or 64 channels");
  static_assert(WCH % 16 == 0 || WCH % 16 == 8, "weight-row swizzle");
};
// physical chunk of logical weight chunk c in row n (16 consecutive rows at one c cover all 16 bank slots)
template <int WCH>
__device__ __forceinline__ int wchunk(int n, int c) {
  return WCH % 16 == 0 ? ((c & ~15) | ((c & 15) ^ (n & 15))) : ((c & ~7) | ((c & 7) ^ ((n >> 1) & 7)));
}
}  // namespace halo

// X2: the dgrad's second fused BN (bnr_x2) may be present (false: its sums and registers are compiled out)
template <bool DGRAD, class GE, int WM, int WN, int OCC, bool X2 = true>
__global__ __launch_bounds__(64 * WM * WN, OCC) void conv_halo_kernel(ConvGeom g) {
  constexpr int WAVES = WM * WN;
  constexpr int TM = halo::BM / WM, TN = 64 / WN, FM = TM / 16, FN = TN / 16;
  constexpr int HW = GE::HW, CPP = GE::CPP, C = GE::C, R = GE::R, PAD = GE::PAD, W_ = GE::W;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  bf16_t* const wlds = smem;
  bf16_t* const hbuf = smem + 64 * GE::KRED;
  bf16_t* const zpix = hbuf + 2 * GE::ELEMS;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w / WN, wc = w % WN, fr = lane & 15, fq = lane >> 4;
  const int OH = g.OH, IH = g.IH, IW = g.IW, M = g.N * g.OH * W_, in_rows = g.N * g.IH;
  const int ntiles = (M + halo::BM - 1) / halo::BM;
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(mer_conv_zero16);
  int tile = blockIdx.x;
  CT(0);
  // global input row of output row (frame n, row y) at tap row 0: n * IH + y - pad
  auto in_row0 = [&](int m) {
    const int go = m / W_, n = go / OH;
    return n * IH + (go - n * OH) - PAD;
  };
  // halo of tile `tl`: global input rows base .. base + ROWS - 1 (base = in_row0 of the tile's first pixel), input
  // columns -pad .. W + R - 2 - pad; chunk L of the buffer holds halo pixel L / CPP, logical channel chunk
  // (L % CPP) ^ ((pixel >> HSHIFT) & (CPP - 1))
  auto stage_halo = [&](bf16_t* hb, int tl) {
    const int base = in_row0(tl * halo::BM);
    for (int j = w; j < GE::CH / 64; j += WAVES) {
      const int L = j * 64 + lane;
      const int hp = L / CPP, c = (L % CPP) ^ ((hp >> GE::HSHIFT) & (CPP - 1));
      const int hr = hp / HW, x = hp - hr * HW - PAD, gr = base + hr;
      const bool ok = hr < GE::ROWS && gr >= 0 && gr < in_rows && x >= 0 && x < IW;
      glds16(ok ? g.X + ((long)gr * IW + x) * C + c * 8 : zero, hb + j * 512);
    }
  };
  // resident weights: row n (output column) x WCH chunks, swizzled by halo::wchunk
  for (int j = w; j < GE::WCH; j += WAVES) {  // 64 rows x WCH chunks = WCH glds pieces of 64 chunks
    const int L = j * 64 + lane;
    const int n = L / GE::WCH, pc = L - n * GE::WCH;
    glds16(g.Wt + (long)n * GE::KRED + halo::wchunk<GE::WCH>(n, pc) * 8, wlds + j * 512);  // (an involution)
  }
  stage_halo(hbuf, tile);
  if (t < CPP) *reinterpret_cast<u32x4*>(zpix + t * 8) = u32x4{0u, 0u, 0u, 0u};
  wait_vmcnt<0>();
  __syncthreads();
  CT(1);

  // Per tile: issue the next tile's halo DMA, run the K loop on this one, wait for that DMA (and the previous tile's
  // epilogue stores -- both had the whole K loop to land), then the epilogue (staged through this tile's halo buffer,
  // now free).  No vmcnt wait follows the epilogue: its stores drain under the next K loop.  The fused column
  // reductions (forward BN statistics, the dgrad's BN-backward sums) accumulate per lane over the workgroup's tiles --
  // all of them cover the same 64 output columns -- and are reduced and stored once, as partial row blockIdx.x, after
  // the loop (round 6: one cross-lane / cross-wave reduction per workgroup instead of per tile, and grid-size partial
  // rows instead of one per tile for the folds).
  EpiAcc<FN> eacc;
  eacc.zero();
  for (int cur = 0, it = 0; tile < ntiles; tile += gridDim.x, cur ^= 1, ++it) {
    bf16_t* const hb = hbuf + cur * GE::ELEMS;
    if (tile + (int)gridDim.x < ntiles) stage_halo(hbuf + (cur ^ 1) * GE::ELEMS, tile + gridDim.x);
    CT(it < 11 ? 2 + 5 * it : 63);
    const int m0 = tile * halo::BM, base = in_row0(m0);
    const auto out_row = [](int row) { return (long)row; };
    constexpr int EWF = GE::ELEMS / 2 / WAVES;  // epilogue staging floats per wave (this tile's halo buffer)
    EpiPre<EpiGeo<FM, FN, EWF>::NP> pre;
    if constexpr (DGRAD)
      conv_epilogue_prefetch<DGRAD, FM, FN, WM, WN, EWF, decltype(out_row), EpiGeo<FM, FN, EWF>::NP, X2>(
          g, pre, w, lane, m0, 0, M, out_row);
    int hpb[FM], yv[FM];  // per fragment row of this lane: halo pixel of tap (0, 0), input row of tap row 0
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      int m = m0 + wr * TM + i * 16 + fr;
      m = m < M ? m : M - 1;  // rows past M compute garbage that the epilogue discards
      const int go = m / W_, x = m - go * W_, n = go / OH, y = go - n * OH;
      yv[i] = y - PAD;
      hpb[i] = (n * IH + y - PAD - base) * HW + x;
    }
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // k-steps of 32 in the packed (tap, channel) order: the fragments of step u + 1 are read while step u's MFMAs run
    // (two register sets, static indices: the loop is fully unrolled)
    bf16x8 af[2][FM], bfr[2][FN];
    auto frags = [&](int u, bf16x8 (&a)[FM], bf16x8 (&b)[FN]) {
      const int kk = u * 32 + fq * 8;       // this lane's 8 reduction indices start here
      const int tap = kk / C, c = (kk % C) / 8;
      const int r = tap / R, s = tap - R * (tap / R);
      // dgrad: tap (r, s) of the packed transposed weight reads dy at (h + pad - r, w + pad - s): the halo row / col
      // of output (y, x) then sits at offset (R - 1 - r, R - 1 - s) from (y - pad, x - pad) when pad = (R - 1) / 2
      const int hr = DGRAD ? R - 1 - r : r, hs = DGRAD ? R - 1 - s : s;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int hp = hpb[i] + hr * HW + hs;
        const bool ok = (unsigned)(yv[i] + hr) < (unsigned)IH;  // rows outside the frame read the zero pixel
        a[i] = *reinterpret_cast<const bf16x8*>(
            ok ? hb + hp * C + ((c ^ ((hp >> GE::HSHIFT) & (CPP - 1))) << 3) : zpix);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = wc * TN + j * 16 + fr, cb = u * 4 + fq;
        b[j] = *reinterpret_cast<const bf16x8*>(wlds + n * GE::KRED + (halo::wchunk<GE::WCH>(n, cb) << 3));
      }
    };
    frags(0, af[0], bfr[0]);
#pragma unroll
    for (int u = 0; u < GE::KSTEPS; ++u) {
      if (u + 1 < GE::KSTEPS) frags(u + 1, af[(u + 1) & 1], bfr[(u + 1) & 1]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[u & 1][i], bfr[u & 1][j], acc[i][j], 0, 0, 0);
    }
    CT(it < 11 ? 3 + 5 * it : 63);
    wait_vmcnt<0>();  // this wave's share of the next halo (and the previous epilogue's stores) has landed
    lds_barrier();    // every wave's: the next halo is complete and no wave still reads hb
    CT(it < 11 ? 4 + 5 * it : 63);
    const int ct_slot = it == 1 ? 60 : -1;  // (timing build: stamps inside the second tile's epilogue)
    if constexpr (DGRAD)
      conv_epilogue_vec<DGRAD, FM, FN, WM, WN, EWF, decltype(out_row), decltype(pre), true, X2, EpiAcc<FN>>(
          g, acc, reinterpret_cast<float*>(hb), w, lane, m0, 0, M, (long)tile, (long)tile, out_row, &pre, ct_slot,
          &eacc);
    else
      conv_epilogue_vec<DGRAD, FM, FN, WM, WN, EWF, decltype(out_row), EpiNone, true, true, EpiAcc<FN>>(
          g, acc, reinterpret_cast<float*>(hb), w, lane, m0, 0, M, (long)tile, (long)tile, out_row,
          static_cast<const EpiNone*>(nullptr), ct_slot, &eacc);
    CT(it < 11 ? 5 + 5 * it : 63);
    lds_barrier();    // every wave is past its epilogue's use of hb before the DMA two tiles on refills it
    CT(it < 11 ? 6 + 5 * it : 63);
  }
  // (no DMA is in flight after the last tile: the halo buffers are free)
  conv_epilogue_acc_finish<DGRAD, FM, FN, WM, WN, GE::ELEMS / 2 / WAVES, X2>(g, eacc, reinterpret_cast<float*>(hbuf), w,
                                                                          lane, 0, (long)blockIdx.x);
}

using HaloL1 = halo::Geo<64, 3, 1, 28, 0>;    // layer1: 3x3 / pad 1, 64 -> 64, 28x28
using HaloStem = halo::Geo<16, 4, 0, 56, 3>;  // the stem's space-to-depth form: 4x4 / pad 0, 16 -> 64, 59x59 -> 56x56

// which halo kernel applies (0: none): 3x3 / stride 1 / pad 1, 64 -> 64 channels on 28-wide maps (fwd and dgrad), or
// 4x4 / stride 1 / pad 0, 16 -> 64 channels, 59 -> 56 (fwd); 64 output columns, 16-byte epilogue, no fused downsample
int halo_kind(const ConvGeom& g, bool dgrad) {
  if (g.st != 1 || g.Ncols != 64 || g.ldy != 64 || !g.vec || g.X2 != nullptr ||
      ((((uintptr_t)g.X) | ((uintptr_t)g.Wt)) & 15) != 0)
    return 0;
  if (g.R == 3 && g.S == 3 && g.pad == 1 && g.IC == 64 && g.IW == 28 && g.OW == 28 && g.IH == g.OH && g.Kred == 576)
    return 1;
  if (!dgrad && g.R == 4 && g.S == 4 && g.pad == 0 && g.IC == 16 && g.IW == 59 && g.OW == 56 && g.IH == 59 &&
      g.OH == 56 && g.Kred == 256)
    return 2;
  return 0;
}

int cu_count() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || v <= 0)
      return 256;
    return v;
  }();
  return n;
}

template <bool DGRAD, class GE, int OCC, bool X2 = true>
int launch_halo_t(ConvGeom& g, hipStream_t st) {
  constexpr int WM = 4, WN = 2;  // 8 waves, 32 x 32 each: conv_pipe_kernel's 128 x 64 tile (variant 2)
  const size_t lds = GE::LDS_ELEMS * sizeof(bf16_t);
  static_assert(GE::LDS_ELEMS * 2 * OCC <= 160 * 1024, "LDS per CU");
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_halo_kernel<DGRAD, GE, WM, WN, OCC, X2>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return (int)hipErrorInvalidConfiguration;
  const int M = g.N * g.OH * g.OW, ntiles = (M + halo::BM - 1) / halo::BM;
  const int slots = OCC * cu_count();
  hipLaunchKernelGGL((conv_halo_kernel<DGRAD, GE, WM, WN, OCC, X2>), dim3(ntiles < slots ? ntiles : slots),
                     dim3(64 * WM * WN), lds, st, g);
  return (int)hipGetLastError();
}

template <bool DGRAD>
int launch_conv_halo(ConvGeom& g, hipStream_t st, int kind) {
  // (the dgrad without a second fused BN -- every layer1 dgrad of the train step -- drops its registers: the
  // per-workgroup accumulators otherwise spill)
  if constexpr (DGRAD)
    if (kind == 1 && !g.bnr_x2) return launch_halo_t<DGRAD, HaloL1, 1, false>(g, st);
  if (kind == 1) return launch_halo_t<DGRAD, HaloL1, 1>(g, st);
  if constexpr (!DGRAD) return launch_halo_t<false, HaloStem, 2>(g, st);  // 71 KB of LDS: two workgroups per CU
  return (int)hipErrorInvalidValue;
}

// Default tile for a non-parity-class conv (forward, or stride-1 input gradient): the in-workgroup split-K form (7: 64-row
// tiles, two K-groups) when one such tile per CU covers the output (ResNet18 layer4: 256 tiles) and each K-group gets
// >= 4 K-steps; otherwise the one-group tiles (`fallback`).  Serialized trunk at B = 32 (profiles/r06/trunk_table_serial
// .txt vs r05): layer4 3x3 fwd 44 -> 36.5 us, dgrad 50-53 -> 41-46.5; layer4.0 stride-2 fwd 24.2 -> 22.1.  Measured and
// dropped: 128-row tiles with two K-groups for layer3 (196 tiles) won standalone with warm operands (34.1 -> 28.2 us)
// but not in the trunk (33.4 -> 34.0, dgrad 39 -> 42) nor in a same-box step A/B (205.17 vs 205.35 steps/s, 4 pairs);
// 64 x 64 per-wave sub-tiles with four / two K-groups lost on every layer (profiles/r06/bench_conv_v10_v11_lost.txt).
int conv_default_variant(const ConvGeom& g, int fallback) {
  if (!g.vec || g.Kred < 8 * CBK) return fallback;
  const long M = (long)g.N * g.OH * g.OW;
  const long nt = (g.Ncols + (g.Ncols <= 64 ? 63 : 127)) / (g.Ncols <= 64 ? 64 : 128);
  if (((M + 63) / 64) * nt <= cu_count()) return 7;
  return fallback;
}

int wgrad_default_variant(int K) {
  (void)K;
  return 4;
}

bool vec_epilogue_enabled() { return true; }

}  // namespace

MER_API int mer_conv_fwd(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* x,
                         const void* w_packed, void* y, float* stats, void* stream) {
  return mer_conv_fwd_ex(N, H, W, C, K, R, S, stride, pad, x, w_packed, y, stats, -1, stream);
}

namespace {
ConvGeom fwd_geom(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* x,
                  const void* w_packed, void* y, float* stats) {
  ConvGeom g{};
  g.N = N; g.IH = H; g.IW = W; g.IC = C;
  g.OH = (H + 2 * pad - R) / stride + 1; g.OW = (W + 2 * pad - S) / stride + 1;
  g.R = R; g.S = S; g.st = stride; g.pad = pad;
  g.Ncols = K; g.Kred = R * S * C;
  g.X = (const bf16_t*)x; g.Wt = (const bf16_t*)w_packed; g.Y = (bf16_t*)y; g.ldy = K; g.stats = stats;
  g.vec = vec_epilogue_enabled() && conv_vec_ok(g);
  return g;
}

ConvGeom dgrad_geom(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* dy,
                    const void* wt_packed, const void* ds_dy) {
  ConvGeom g{};
  g.N = N; g.OH = H; g.OW = W;
  g.IH = (H + 2 * pad - R) / stride + 1; g.IW = (W + 2 * pad - S) / stride + 1; g.IC = K;
  g.R = R; g.S = S; g.st = stride; g.pad = pad;
  g.Ncols = C; g.Kred = R * S * K;
  g.X = (const bf16_t*)dy; g.Wt = (const bf16_t*)wt_packed; g.ldy = C; g.stats = nullptr;
  g.X2 = (const bf16_t*)ds_dy;
  g.vec = vec_epilogue_enabled() && conv_vec_ok(g);
  return g;
}

// workgroups of a halo launch (launch_halo_t): one partial row each
int halo_rows(const ConvGeom& g, int kind) {
  const long M = (long)g.N * g.OH * g.OW, ntiles = (M + halo::BM - 1) / halo::BM;
  const long slots = (long)(kind == 1 ? 1 : 2) * cu_count();
  return (int)(ntiles < slots ? ntiles : slots);
}
}  // namespace

MER_API int mer_conv_fwd_rows(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* x,
                              const void* w_packed, int variant) {
  if (N <= 0 || C % 8 || variant < -1 || variant > 7) return -(int)hipErrorInvalidValue;
  const ConvGeom g = fwd_geom(N, H, W, C, K, R, S, stride, pad, x, w_packed, nullptr, nullptr);
  if (variant == -1 || variant == 6) {
    const int hk = halo_kind(g, false);
    if (hk) return halo_rows(g, hk);
  }
  const long M = (long)N * g.OH * g.OW;
  if (variant == -1) {  // the default pipelined tile: one statistics row per BM-row tile (launch_conv_pipe's choice)
    const int v = conv_default_variant(g, 2);
    const int bn = g.Ncols <= 64 ? 64 : 128;
    const bool small_m = ((M + 127) / 128) * ((g.Ncols + bn - 1) / bn) < 384;
    const int BM = (v == 7 || small_m) ? 64 : 128;
    return (int)((M + BM - 1) / BM);
  }
  return (int)((M + 63) / 64);  // an upper bound: rows past the tiles stay as the caller left them (zeroed)
}

MER_API int mer_conv_dgrad_rows(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* dy,
                                const void* wt_packed, const void* ds_dy, int variant) {
  if (N <= 0 || K % 8 || C % 8 || variant < -1 || variant > 7) return -(int)hipErrorInvalidValue;
  const ConvGeom g = dgrad_geom(N, H, W, C, K, R, S, stride, pad, dy, wt_packed, ds_dy);
  if (variant == -1 || variant == 6) {
    const int hk = halo_kind(g, true);
    if (hk) return halo_rows(g, hk);
  }
  if (variant == -1 && (stride == 1 || stride == 2)) {
    // the default pipelined tile (mer_conv_dgrad_ds's variant resolution, launch_conv_pipe's tile rule): one reduction
    // row per BM-row tile, per parity class for the stride-2 form (red_row: the classes' tiles back to back) -- exact
    int v = C <= 64 ? 5 : 2;
    if (stride == 1) v = conv_default_variant(g, v);
    const bool par = stride == 2;
    const long Mq = par ? (long)N * H * W / 4 : (long)N * H * W;
    const int bn = C <= 64 ? 64 : 128;
    const bool small_m = ((Mq + 127) / 128) * ((C + bn - 1) / bn) * (par ? 4 : 1) < 384;
    const int BM = (v == 7 || small_m) ? 64 : 128;
    if (!par) return (int)(((long)N * H * W + BM - 1) / BM);
    long rows = 0;
    for (int cls = 0; cls < 4; ++cls) {
      const int ph = cls >> 1, pw = cls & 1;
      const long Mc = (long)N * ((H - ph + 1) >> 1) * ((W - pw + 1) >> 1);
      rows += (Mc + BM - 1) / BM;
    }
    return (int)rows;
  }
  return (int)(((long)N * H * W + 63) / 64 + 4);  // MER_BN_RED_ROWS(M) - 64: an upper bound (zero the buffer)
}

MER_API int mer_conv_fwd_ex(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* x,
                            const void* w_packed, void* y, float* stats, int variant, void* stream) {
  if (C % 8 || variant < -1 || variant > 7) return (int)hipErrorInvalidValue;
  ConvGeom g = fwd_geom(N, H, W, C, K, R, S, stride, pad, x, w_packed, y, stats);
  // default: the halo kernel where it applies (layer1), else the 8-wave pipelined tiles; variant 6 = halo or fail
  // (mer_conv_fwd_rows makes the same choice from the same geometry)
  if (variant == -1 || variant == 6) {
    const int hk = halo_kind(g, false);
    if (hk) return launch_conv_halo<false>(g, (hipStream_t)stream, hk);
  }
  if (variant == 6) return (int)hipErrorInvalidValue;
  if (variant == -1) variant = conv_default_variant(g, 2);
  if (variant == 0) return launch_conv<false>(g, (hipStream_t)stream);
  return launch_conv_pipe<false, false>(g, (hipStream_t)stream, variant);
}

MER_API int mer_conv_dgrad(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* dy,
                           const void* wt_packed, void* dx, const void* residual, const void* residual_mask,
                           void* stream) {
  return mer_conv_dgrad_ex(N, H, W, C, K, R, S, stride, pad, dy, wt_packed, dx, residual, residual_mask, -1, stream);
}

MER_API int mer_conv_dgrad_ex(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* dy,
                              const void* wt_packed, void* dx, const void* residual, const void* residual_mask,
                              int variant, void* stream) {
  return mer_conv_dgrad_bnr(N, H, W, C, K, R, S, stride, pad, dy, wt_packed, dx, residual, residual_mask, nullptr,
                            nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, variant, stream);
}

MER_API int mer_conv_dgrad_bnr(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* dy,
                               const void* wt_packed, void* dx, const void* residual, const void* residual_mask,
                               const void* bn_mask, const void* bn_x, const float* bn_ms, float* bn_red,
                               const void* bn_x2, const float* bn_ms2, float* bn_red2, int variant, void* stream) {
  return mer_conv_dgrad_ds(N, H, W, C, K, R, S, stride, pad, dy, wt_packed, dx, residual, residual_mask, bn_mask, bn_x,
                           bn_ms, bn_red, bn_x2, bn_ms2, bn_red2, nullptr, nullptr, 0, variant, stream);
}

MER_API int mer_conv_dgrad_ds(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* dy,
                              const void* wt_packed, void* dx, const void* residual, const void* residual_mask,
                              const void* bn_mask, const void* bn_x, const float* bn_ms, float* bn_red,
                              const void* bn_x2, const float* bn_ms2, float* bn_red2, const void* ds_dy,
                              const void* ds_wt_packed, int ds_K, int variant, void* stream) {
  if (K % 8 || C % 8 || variant < -1 || variant > 7) return (int)hipErrorInvalidValue;
  const bool auto_variant = variant == -1;
  // 64-channel outputs (layer1, the layer2.0 input gradients): 32-wide K-tiles on a 4-deep ring with 4-wave tiles
  // (tools/bench_conv.py --fused: layer1 101 -> 65 us, layer2.0 s2 74 -> 51, downsample 48 -> 31); wider outputs
  // keep the 64-wide 2-deep ring (the deep ring loses 10-50% there).  The layer1 shapes take the halo kernel (6).
  if (variant == -1) variant = C <= 64 ? 5 : 2;
  // the fused downsample: a 1x1 / stride-2 / pad-0 conv of the same input with ds_K output channels, beside a
  // 3x3 / stride-2 / pad-1 conv (its taps land in parity class (0, 0) only, at pixel (2i, 2j)); K-tile aligned.
  // Checked AFTER the variant is resolved: only the pipelined kernels (variants 1..5) read the second K segment.
  if (ds_dy && (stride != 2 || R != 3 || S != 3 || pad != 1 || !ds_wt_packed || ds_K <= 0 || ds_K % 64 || K % 64 ||
                variant < 1))
    return (int)hipErrorInvalidValue;
  if (bn_red && (!bn_mask || !bn_x || !bn_ms || (bn_x2 && (!bn_ms2 || !bn_red2)))) return (int)hipErrorInvalidValue;
  if (bn_red && (variant == 0 || stride > 2)) return (int)hipErrorInvalidValue;  // fused only in the pipelined kernel
  ConvGeom g = dgrad_geom(N, H, W, C, K, R, S, stride, pad, dy, wt_packed, ds_dy);
  g.Y = (bf16_t*)dx;
  g.R_ = (const bf16_t*)residual; g.Rmask = (const bf16_t*)residual_mask;
  g.bnr_mask = (const bf16_t*)bn_mask; g.bnr_x = (const bf16_t*)bn_x; g.bnr_ms = bn_ms; g.bnr_red = bn_red;
  g.bnr_x2 = (const bf16_t*)bn_x2; g.bnr_ms2 = bn_ms2; g.bnr_red2 = bn_red2;
  g.Wt2 = (const bf16_t*)ds_wt_packed; g.K2 = ds_dy ? ds_K : 0;
  // (mer_conv_dgrad_rows makes the same choice from the same geometry)
  if (auto_variant || variant == 6) {
    const int hk = halo_kind(g, true);
    if (hk) return launch_conv_halo<true>(g, (hipStream_t)stream, hk);
  }
  if (variant == 6) return (int)hipErrorInvalidValue;
  if (auto_variant && stride == 1) variant = conv_default_variant(g, variant);
  if (variant == 0 || stride > 2) return launch_conv<true>(g, (hipStream_t)stream);
  if (stride == 2) return launch_conv_pipe<true, true>(g, (hipStream_t)stream, variant);
  return launch_conv_pipe<true, false>(g, (hipStream_t)stream, variant);
}

MER_API int mer_conv_wgrad(int N, int H, int W, int C, int Creal, int K, int R, int S, int stride, int pad,
                           const void* x, const void* dy, float* dw, int splits, float* workspace, void* stream) {
  return mer_conv_wgrad_ex(N, H, W, C, Creal, K, R, S, stride, pad, x, dy, dw, splits, workspace, -1, stream);
}

static int conv_wgrad_impl(int N, int H, int W, int C, int Creal, int K, int R, int S, int stride, int pad,
                           const void* x, const void* dy, long ldy, float* dw, int splits, float* workspace,
                           int variant, void* stream, bool fold = true) {
  if (C % 8 || K % 8 || variant < -1 || variant > 8 || R * S > 49) return (int)hipErrorInvalidValue;
  if (variant == -1) variant = wgrad_default_variant(K);
  WgradGeom g{};
  g.N = N; g.H = H; g.W = W; g.C = C; g.Creal = Creal;
  g.Ho = (H + 2 * pad - R) / stride + 1; g.Wo = (W + 2 * pad - S) / stride + 1; g.K = K;
  g.R = R; g.S = S; g.st = stride; g.pad = pad;
  g.X = (const bf16_t*)x; g.dY = (const bf16_t*)dy; g.ws = workspace;
  g.ldy = ldy > 0 ? ldy : K;
  const int P = N * g.Ho * g.Wo;
  if (splits < 1) splits = 1;
  g.pix_per_split = ((P + splits - 1) / splits + 63) / 64 * 64;
  splits = (P + g.pix_per_split - 1) / g.pix_per_split;  // every split non-empty (<= requested)
  const int Ntot = R * S * C;
  hipStream_t st = (hipStream_t)stream;
  if (K <= 64) {
    dim3 grid(((Ntot + 127) / 128) * ((K + 63) / 64), 1, splits);
    if (variant == 1)
      hipLaunchKernelGGL((wgrad_kernel<64, 128>), grid, dim3(256), 0, st, g);
    else if (variant == 4)
      launch_wgrad_pipe<64, 128, 2, 4, 2>(g, grid, st);
    else if (variant == 8)
      launch_wgrad_pipe<64, 128, 2, 4, 2, 64, 2>(g, grid, st);
    else if (variant == 5 || variant == 6)
      launch_wgrad_pipe<64, 128, 2, 4, 3>(g, grid, st);
    else if (variant == 3)
      hipLaunchKernelGGL((wgrad_kernel<64, 128, 2, 4, 2>), grid, dim3(512), 0, st, g);
    else
      hipLaunchKernelGGL((wgrad_kernel<64, 128, 2, 4>), grid, dim3(512), 0, st, g);
  } else {
    dim3 grid(((Ntot + 127) / 128) * ((K + 127) / 128), 1, splits);
    if (variant == 1)
      hipLaunchKernelGGL((wgrad_kernel<128, 128>), grid, dim3(256), 0, st, g);
    else if (variant == 4)
      launch_wgrad_pipe<128, 128, 2, 4, 2>(g, grid, st);
    else if (variant == 8)
      launch_wgrad_pipe<128, 128, 2, 4, 2, 64, 2>(g, grid, st);
    else if (variant == 5)
      launch_wgrad_pipe<128, 128, 2, 4, 3>(g, grid, st);
    else if (variant == 6)
      launch_wgrad_pipe<128, 128, 2, 4, 4, 32>(g, grid, st);
    else if (variant == 7)
      launch_wgrad_pipe<128, 128, 2, 4, 3, 32>(g, grid, st);
    else if (variant == 3)
      hipLaunchKernelGGL((wgrad_kernel<128, 128, 2, 4, 2>), grid, dim3(512), 0, st, g);
    else
      hipLaunchKernelGGL((wgrad_kernel<128, 128, 2, 4>), grid, dim3(512), 0, st, g);
  }
  if (!fold) MER_LAUNCH_CHECK();  // partial slabs left for mer_wgrad_fold_batch
  constexpr int fold_max = 16;  // most slabs folded in the single fold+scatter pass
  if (splits > fold_max) {  // many partial slabs: a wide reduce first (one serial chain per element was latency-bound)
    const int SG = splits >= 64 ? 16 : 8;
    const long total = (long)K * R * S * C;
    const int E = 256 / SG;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((total + E - 1) / E)), dim3(256), 0, st, K, C, Creal, R * S,
                       splits, SG, workspace);
    hipLaunchKernelGGL(wgrad_scatter_kernel, dim3((Creal + 31) / 32, K), dim3(256), 0, st, C, Creal, R * S, workspace,
                       dw);
  } else {  // few slabs: fold and scatter in one pass
    hipLaunchKernelGGL(wgrad_fold_scatter_kernel, dim3((Creal + 31) / 32, K), dim3(256), 0, st, K, C, Creal, R * S,
                       splits, workspace, dw);
  }
  MER_LAUNCH_CHECK();
}

MER_API int mer_conv_wgrad_ex(int N, int H, int W, int C, int Creal, int K, int R, int S, int stride, int pad,
                              const void* x, const void* dy, float* dw, int splits, float* workspace, int variant,
                              void* stream) {
  return conv_wgrad_impl(N, H, W, C, Creal, K, R, S, stride, pad, x, dy, K, dw, splits, workspace, variant, stream);
}

MER_API int mer_conv_wgrad_partials(int N, int H, int W, int C, int K, int R, int S, int stride, int pad,
                                    const void* x, const void* dy, int splits, float* workspace, int variant,
                                    void* stream) {
  return conv_wgrad_impl(N, H, W, C, C, K, R, S, stride, pad, x, dy, K, nullptr, splits, workspace, variant, stream,
                         false);
}

static int fold_sg_max() { return 8; }  // split groups per block for many-slab records

// rows: n x 8 int64 {ws, dw, map, K, C, Creal (map records: output floats per k), R*S, splits}
MER_API int mer_wgrad_fold_batch(int n, const long long* rows, void* stream) {
  if (n < 1 || n > kFoldMaxRecs) return (int)hipErrorInvalidValue;
  FoldTable t{};
  t.n = n;
  int blk = 0;
  for (int i = 0; i < n; ++i) {
    const long long* q = rows + 8 * i;
    FoldRec& r = t.r[i];
    r.ws = (const float*)q[0]; r.dw = (float*)q[1]; r.map = (const int*)q[2];
    r.K = (int)q[3]; r.C = (int)q[4]; r.Creal = (int)q[5]; r.RS = (int)q[6]; r.splits = (int)q[7];
    if (!r.ws || !r.dw || r.K < 1 || r.C < 1 || r.C % 4 || r.RS < 1 || r.splits < 1 || r.Creal < 1 ||
        (!r.map && r.Creal > r.C) || ((uintptr_t)r.ws & 15))
      return (int)hipErrorInvalidValue;
    // SG <= 8: E >= 32 consecutive floats per split group, i.e. whole 128-byte lines (SG 16 read half lines: the
    // slabs are cold by the time the segment folds, so half-used lines cost HBM bytes)
    r.SG = r.splits > 48 ? fold_sg_max() : (r.splits > 12 ? 4 : 1);
    const long total = (long)r.K * r.RS * r.C;
    r.blk0 = blk;
    r.nblk = (int)((total + 4 * (256 / r.SG) - 1) / (4 * (256 / r.SG)));
    blk += r.nblk;
  }
  hipLaunchKernelGGL(wgrad_fold_batch_kernel, dim3(blk), dim3(256), 0, (hipStream_t)stream, t);
  MER_LAUNCH_CHECK();
}

// Linear weight gradient as a 1x1 convolution over M "pixels": dw[n][k] += sum_m dy[m][n] x[m][k].
MER_API int mer_linear_wgrad(int M, int N, int K, const void* x, const void* dy, long ldy, float* dw, int splits,
                             float* workspace, void* stream) {
  if (ldy < N || ldy % 8) return (int)hipErrorInvalidValue;
  return conv_wgrad_impl(1, 1, M, K, K, N, 1, 1, 1, 0, x, dy, ldy, dw, splits, workspace, -1, stream);
}

// ---------------------------------------------------------------------------------------
// Packing kernels
// ---------------------------------------------------------------------------------------
// video frames NCHW fp32 -> NHWC bf16 with channels zero-padded to Cp
// one frame per blockIdx.y; Cp == 8: one 16-byte store per pixel
__global__ void pack_input_kernel(int C, int HW, const float* __restrict__ x, bf16_t* __restrict__ y) {
  const int n = blockIdx.y;
  const float* xn = x + (long)n * C * HW;
  u32x4* yn = reinterpret_cast<u32x4*>(y + (long)n * HW * 8);
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += gridDim.x * blockDim.x) {
    u32x4 o = {0u, 0u, 0u, 0u};
    bf16_t* oh = reinterpret_cast<bf16_t*>(&o);
    for (int c = 0; c < C; ++c) oh[c] = f2bf(xn[(long)c * HW + p]);
    yn[p] = o;
  }
}
MER_API int mer_pack_input_nhwc(int N, int C, int H, int W, int Cp, const float* x, void* y, void* stream) {
  if (Cp != 8 || C > 8) return (int)hipErrorInvalidValue;
  const int HW = H * W;
  dim3 grid((HW + 255) / 256 < 64 ? (HW + 255) / 256 : 64, N);
  hipLaunchKernelGGL(pack_input_kernel, grid, dim3(256), 0, (hipStream_t)stream, C, HW, x, (bf16_t*)y);
  MER_LAUNCH_CHECK();
}

// Space-to-depth stem input (ResNet conv1: 7x7, stride 2, pad 3 on C <= 4 channels, H and W even):
// fp32 NCHW [N][C][H][W] -> bf16 [N][H/2+3][W/2+3][16], pixel (j, i) = 2x2 block (j-2, i-2) of the frame
// with channel (dy*2 + dx)*C + c (zero for the 2 leading / 1 trailing border rows and columns and for
// channels >= 4C).  The stride-2 7x7 conv then is a stride-1 4x4 conv with no padding on 16 channels
// (K = 256 instead of 7*7*8 = 392 for the 8-channel-padded direct form); weights: pack mode 2 below.
template <int C>  // compile-time channel count: the (dy, dx, c) -> s2d channel map unrolls to fixed registers
__global__ void pack_input_s2d_kernel(int N, int H, int W, const float* __restrict__ x, bf16_t* __restrict__ y) {
  const int Hs = H / 2 + 3, Ws = W / 2 + 3;
  const int total = N * Hs * Ws;  // (< 2^22, checked on the host: 32-bit index math, exact float-reciprocal divides --
                                  // the 64-bit divisions of a long index were most of this kernel's time)
  const float inv_Ws = 1.f / Ws, inv_Hs = 1.f / Hs;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < total; p += gridDim.x * blockDim.x) {
    const int q = fdiv(p, inv_Ws);
    const int i = p - q * Ws;
    const int n = fdiv(q, inv_Hs);
    const int j = q - n * Hs;
    uint32_t o[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    const int jj = j - 2, ii = i - 2;
    if (jj >= 0 && jj < H / 2 && ii >= 0 && ii < W / 2) {
      // the 2x2 block's two rows of each channel as float2 loads (adjacent lanes read adjacent 8-byte pairs: one
      // coalesced 512-byte run per wave instruction)
      const float* xn = x + (long)n * C * H * W + (long)(2 * jj) * W + 2 * ii;
      float v[C][4];  // [c][dydx]
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) {
          const float2 q2 = *reinterpret_cast<const float2*>(xn + (long)c * H * W + dy * W);
          v[c][2 * dy] = q2.x;
          v[c][2 * dy + 1] = q2.y;
        }
#pragma unroll
      for (int ch = 0; ch < 4 * C; ++ch)
        o[ch >> 1] |= (uint32_t)f2bf(v[ch % C][ch / C]) << ((ch & 1) * 16);
    }
    u32x4* dst = reinterpret_cast<u32x4*>(y + (long)p * 16);
    dst[0] = u32x4{o[0], o[1], o[2], o[3]};
    dst[1] = u32x4{o[4], o[5], o[6], o[7]};
  }
}
MER_API int mer_pack_input_s2d(int N, int C, int H, int W, const float* x, void* y, void* stream) {
  if (C < 1 || C > 4 || (H & 1) || (W & 1) || ((uintptr_t)x & 7)) return (int)hipErrorInvalidValue;
  const long per_frame = (long)(H / 2 + 3) * (W / 2 + 3);
  if (N < 0 || per_frame >= (1L << 22)) return (int)hipErrorInvalidValue;
  // the kernel's fdiv index math holds below 2^22 pixels per launch: larger batches go in frame chunks
  const int chunk = (int)(((1L << 22) - 1) / per_frame);
  const hipStream_t st = (hipStream_t)stream;
  for (int n0 = 0; n0 < N; n0 += chunk) {
    const int nc = N - n0 < chunk ? N - n0 : chunk;
    const long total = (long)nc * per_frame;
    const int grid = (int)((total + 255) / 256 < 16384 ? (total + 255) / 256 : 16384);
    const float* xc = x + (long)n0 * C * H * W;
    bf16_t* yc = (bf16_t*)y + n0 * per_frame * 16;
    if (C == 3) hipLaunchKernelGGL(pack_input_s2d_kernel<3>, dim3(grid), dim3(256), 0, st, nc, H, W, xc, yc);
    else if (C == 1) hipLaunchKernelGGL(pack_input_s2d_kernel<1>, dim3(grid), dim3(256), 0, st, nc, H, W, xc, yc);
    else if (C == 2) hipLaunchKernelGGL(pack_input_s2d_kernel<2>, dim3(grid), dim3(256), 0, st, nc, H, W, xc, yc);
    else hipLaunchKernelGGL(pack_input_s2d_kernel<4>, dim3(grid), dim3(256), 0, st, nc, H, W, xc, yc);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

// PyTorch conv weight [K][C][R][S] fp32 -> fwd [K][R][S][Cp] (transpose=0) or dgrad [Cp][R][S][Kp] (transpose=1)
__global__ void pack_w_kernel(int K, int C, int R, int S, int Cp, int transpose, const float* __restrict__ w,
                              bf16_t* __restrict__ out) {
  const long total = (long)K * R * S * Cp;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    int k, r, s, c;
    if (!transpose) {
      c = e % Cp; long q = e / Cp; s = q % S; q /= S; r = q % R; k = q / R;
    } else {
      k = e % K; long q = e / K; s = q % S; q /= S; r = q % R; c = q / R;
    }
    out[e] = c < C ? f2bf(w[(((long)k * C + c) * R + r) * S + s]) : (bf16_t)0;
  }
}
MER_API int mer_pack_conv_weight(int K, int C, int R, int S, int Cp, int transpose, const float* w, void* out,
                                 void* stream) {
  const long total = (long)K * R * S * Cp;
  const int grid = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
  hipLaunchKernelGGL(pack_w_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, K, C, R, S, Cp, transpose, w,
                     (bf16_t*)out);
  MER_LAUNCH_CHECK();
}

// All of a trunk's weight packs in ONE launch (the per-step re-pack in training is ~40 small layouts
// whose separate launches cost more than their bytes).  desc: n records of 9 int64 =
// {w, out, K, C, R, S, Cp, transpose (0, 1, or 2 = space-to-depth stem), first element (unused here)};
// grid.y = record.  Both layouts go
// through an LDS tile so global reads AND writes are contiguous runs:
//   transpose 0: block = one output channel k: w[k][c][rs] (C*RS contiguous floats) -> out[k][rs][c<Cp];
//   transpose 1: block = (input channel c, 64 output channels k0..): w[k][c][rs] (runs of RS) ->
//                out[c][rs][k0..k0+63].
// FLAT: one-dimensional grid over every record's blocks (column 8 = the record's first block): no idle blocks (the
// 2-D form launches 4,096 blocks per record, most of which only exit -- that dispatch was most of its time)
template <bool FLAT>
__global__ __launch_bounds__(256) void pack_w_batched_kernel(const long long* __restrict__ desc, int n) {
  __shared__ float tile[4608];  // max C*RS (512 * 9) or 64 * RS (RS <= 49 -> 3136)
  int rec = FLAT ? 0 : (int)blockIdx.y;
  if (FLAT)
    for (int i = 1; i < n; ++i)
      if (desc[i * 9 + 8] <= (long long)blockIdx.x) rec = i;
  const long long* r = desc + rec * 9;
  const int bx = FLAT ? (int)(blockIdx.x - r[8]) : (int)blockIdx.x;
  const float* w = reinterpret_cast<const float*>(r[0]);
  bf16_t* out = reinterpret_cast<bf16_t*>(r[1]);
  const int K = (int)r[2], C = (int)r[3], RS = (int)(r[4] * r[5]), Cp = (int)r[6];
  if (r[7] == 3) {  // transposed pack from the forward bf16 pack: src [K][RS][C] -> out [C][RS][K] (C, K % 64 == 0)
    // block = (tap, 64-channel tile, 64-output tile): 16-byte loads of 64 k-rows into LDS, 16-byte stores of 64 c-rows
    const uint16_t* src = reinterpret_cast<const uint16_t*>(r[0]);
    uint16_t* lds = reinterpret_cast<uint16_t*>(tile);  // [64 k][72] (row pad spreads the column gathers)
    const int kbn = K >> 6, cbn = C >> 6;
    const int rs = bx / (kbn * cbn), rem = bx - rs * kbn * cbn, cb = rem / kbn, kb = rem - cb * kbn;
    if (rs >= RS) return;
    const int k0 = kb * 64, c0 = cb * 64;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = threadIdx.x + 256 * j, kk = i >> 3, ch = (i & 7) * 8;
      const uint4 v = *reinterpret_cast<const uint4*>(src + ((long)(k0 + kk) * RS + rs) * C + c0 + ch);
      *reinterpret_cast<uint4*>(lds + kk * 72 + ch) = v;
    }
    __syncthreads();
    uint16_t* ob = reinterpret_cast<uint16_t*>(out);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = threadIdx.x + 256 * j, cc = i >> 3, kc = (i & 7) * 8;
      uint32_t pk[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        pk[e] = (uint32_t)lds[(kc + 2 * e) * 72 + cc] | ((uint32_t)lds[(kc + 2 * e + 1) * 72 + cc] << 16);
      *reinterpret_cast<uint4*>(ob + ((long)(c0 + cc) * RS + rs) * K + k0 + kc) = uint4{pk[0], pk[1], pk[2], pk[3]};
    }
    return;
  }
  if (r[7] == 2) {  // space-to-depth stem: out[k][ry][rx][ch], tap (r, s) = (2ry+dy-1, 2rx+dx-1), ch = (dy*2+dx)*C + c
    const int k = bx;
    const int R = (int)r[4], S = (int)r[5], Ro = (R + 2) / 2, So = (S + 2) / 2;
    if (k >= K) return;
    const float* src = w + (long)k * C * RS;
    for (int i = threadIdx.x; i < C * RS; i += 256) tile[i] = src[i];
    __syncthreads();
    bf16_t* dst = out + (long)k * Ro * So * Cp;
    for (int i = threadIdx.x; i < Ro * So * Cp; i += 256) {
      const int ch = i % Cp, q = i / Cp, rx = q % So, ry = q / So;
      const int dydx = ch / C, c = ch - dydx * C;
      const int rr = 2 * ry + (dydx >> 1) - 1, ss = 2 * rx + (dydx & 1) - 1;
      const bool ok = dydx < 4 && rr >= 0 && rr < R && ss >= 0 && ss < S;
      dst[i] = ok ? f2bf(tile[c * RS + rr * S + ss]) : (bf16_t)0;
    }
  } else if (!r[7]) {
    const int k = bx;
    if (k >= K) return;
    const float* src = w + (long)k * C * RS;
    const int n = C * RS;
    if ((n & 3) == 0 && (((uintptr_t)src) & 15) == 0) {
      for (int i = threadIdx.x; i < n / 4; i += 256)
        reinterpret_cast<f32x4*>(tile)[i] = reinterpret_cast<const f32x4*>(src)[i];  // [c][rs]
    } else {
      for (int i = threadIdx.x; i < n; i += 256) tile[i] = src[i];
    }
    __syncthreads();
    bf16_t* dst = out + (long)k * RS * Cp;
    // 8 consecutive channels of one tap per thread, one 16-byte store (Cp % 8 == 0); i / Cp by reciprocal
    const float inv_Cp = 1.f / Cp;
    for (int i = threadIdx.x; i < RS * Cp / 8; i += 256) {  // i*8 = rs*Cp + c0
      const int rs = fdiv(i * 8, inv_Cp), c0 = i * 8 - rs * Cp;
      uint32_t pk[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = c0 + 2 * e;
        const uint32_t lo = c < C ? f2bf(tile[c * RS + rs]) : 0u, hi = c + 1 < C ? f2bf(tile[(c + 1) * RS + rs]) : 0u;
        pk[e] = lo | (hi << 16);
      }
      *reinterpret_cast<uint4*>(dst + (long)i * 8) = uint4{pk[0], pk[1], pk[2], pk[3]};
    }
  } else {
    const int kb = (K + 63) / 64;
    const int c = bx / kb, k0 = (bx - c * kb) * 64;
    if (c >= Cp) return;
    const int nk = min(64, K - k0);
    const float inv_RS = 1.f / RS;
    for (int i = threadIdx.x; i < nk * RS; i += 256) {  // [kk][rs]
      const int kk = fdiv(i, inv_RS), rs = i - kk * RS;
      tile[i] = c < C ? w[((long)(k0 + kk) * C + c) * RS + rs] : 0.f;
    }
    __syncthreads();
    bf16_t* dst = out + (long)c * RS * K + k0;
    if (nk == 64 && (K & 7) == 0) {  // 8 consecutive output channels per thread, one 16-byte store
      for (int i = threadIdx.x; i < RS * 8; i += 256) {  // i = rs*8 + kk0/8
        const int rs = i >> 3, kk0 = (i & 7) * 8;
        uint32_t pk[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          pk[e] = (uint32_t)f2bf(tile[(kk0 + 2 * e) * RS + rs]) | ((uint32_t)f2bf(tile[(kk0 + 2 * e + 1) * RS + rs]) << 16);
        *reinterpret_cast<uint4*>(dst + (long)rs * K + kk0) = uint4{pk[0], pk[1], pk[2], pk[3]};
      }
    } else {
      for (int i = threadIdx.x; i < RS * nk; i += 256) {  // i = rs*nk + kk
        const int rs = i / nk, kk = i - rs * nk;
        dst[(long)rs * K + kk] = f2bf(tile[kk * RS + rs]);
      }
    }
  }
}
MER_API int mer_pack_conv_weights(int n, const long long* desc, long total, void* stream) {
  (void)total;
  if (n <= 0 || n > 64) return (int)hipErrorInvalidValue;
  // grid.x covers the largest record: 512 output channels (layout 0) or 512 x 8 (c, k-block) tiles
  hipLaunchKernelGGL(pack_w_batched_kernel<false>, dim3(512 * 8, n), dim3(256), 0, (hipStream_t)stream, desc, n);
  MER_LAUNCH_CHECK();
}
MER_API int mer_pack_conv_weights_flat(int n, const long long* desc, long total_blocks, void* stream) {
  if (n <= 0 || n > 64 || total_blocks <= 0 || total_blocks > (1L << 30)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(pack_w_batched_kernel<true>, dim3((unsigned)total_blocks), dim3(256), 0, (hipStream_t)stream, desc,
                     n);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// BatchNorm2d (train mode), channel-last.  stats[c] = (sum, sumsq) over M = N*H*W values.
// finalize: ms[c] = (mean, rstd); running_mean = (1-mom) rm + mom*mean; running_var uses the
// unbiased variance (torch semantics); num_batches_tracked += 1.
// ---------------------------------------------------------------------------------------
// Forward statistics layout (mer.h MER_BN_STAT_ROWS): one row per output row tile of the conv (<= ceil(M/64)
// rows, unused rows zero) followed by 64 scratch rows.  Rows are summed in a fixed order: stage 1 (when
// there are more than 64 rows) folds contiguous row groups into the 64 scratch rows, stage 2 folds <= 64
// rows per channel -- deterministic whatever the tile size and block schedule were.
// Latency: a block here is a short chain (one wave-row of loads, a sum, an LDS meet), so every load of a
// thread's rows is issued before the first add (batches of 16 from clamped addresses, zero-selected) -- the
// loop that added as it loaded waited one memory latency per two rows.  The sum order is unchanged: a0 takes
// the thread's rows 0, 2, 4, ... and a1 rows 1, 3, 5, ... (rows r0 + pg + 4 i).
__global__ __launch_bounds__(256) void bn_stat_rows_fold_kernel(int C2, int rows, int per, const float* __restrict__ in,
                                                                float* __restrict__ out) {
  __shared__ float part[4][64];
  const int el = threadIdx.x & 63, pg = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + el, grp = blockIdx.y;
  const int r0 = grp * per, r1 = min(rows, r0 + per);
  const int ec = e < C2 ? e : C2 - 1;
  const int n = r1 - (r0 + pg) > 0 ? (r1 - (r0 + pg) + 3) / 4 : 0;  // this thread's rows
  float a0 = 0.f, a1 = 0.f;
  for (int i0 = 0; i0 < n; i0 += 16) {
    float x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = r0 + pg + 4 * (i0 + i);
      x[i] = in[(long)(r < r1 ? r : r1 - 1) * C2 + ec];
    }
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      if (i0 + i < n) a0 += x[i];
      if (i0 + i + 1 < n) a1 += x[i + 1];
    }
  }
  part[pg][el] = a0 + a1;
  __syncthreads();
  if (pg == 0 && e < C2) out[(long)grp * C2 + e] = (part[0][el] + part[1][el]) + (part[2][el] + part[3][el]);
}

// 64 channels per block; the 4 waves split the (<= 64) rows, then meet in LDS
__global__ __launch_bounds__(256) void bn_finalize_kernel(int C, long M, int rows, const float* __restrict__ stats,
                                                          float eps, float momentum, float* __restrict__ ms,
                                                          float* __restrict__ rmean, float* __restrict__ rvar,
                                                          long long* __restrict__ nbt) {
  __shared__ float part[4][64][2];
  const int cl = threadIdx.x & 63, pg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  if (!stats) {  // eval mode: normalise with the running statistics, no update
    if (pg == 0 && c < C) {
      ms[2 * c] = rmean[c];
      ms[2 * c + 1] = rsqrtf(rvar[c] + eps);
    }
    return;
  }
  float sum = 0.f, sq = 0.f;
  {  // rows <= 64: this wave's <= 16 rows all in flight before the first add (same order)
    const int cc = c < C ? c : C - 1;
    float xs[16], xq[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int p = pg + 4 * i, pc = p < rows ? p : rows - 1;
      xs[i] = stats[(long)pc * 2 * C + 2 * cc];
      xq[i] = stats[(long)pc * 2 * C + 2 * cc + 1];
    }
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (pg + 4 * i < rows) {
        sum += xs[i];
        sq += xq[i];
      }
  }
  part[pg][cl][0] = sum;
  part[pg][cl][1] = sq;
  __syncthreads();
  if (pg != 0 || c >= C) return;
  sum = part[0][cl][0] + part[1][cl][0] + part[2][cl][0] + part[3][cl][0];
  sq = part[0][cl][1] + part[1][cl][1] + part[2][cl][1] + part[3][cl][1];
  const float mean = sum / M;
  const float var = fmaxf(sq / M - mean * mean, 0.f);
  ms[2 * c] = mean;
  ms[2 * c + 1] = rsqrtf(var + eps);
  if (rmean) rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
  if (rvar) rvar[c] = (1.f - momentum) * rvar[c] + momentum * var * ((float)M / (float)(M > 1 ? M - 1 : 1));
  if (nbt && c == 0) *nbt += 1;
}
// 64 < rows <= BN_WIDE_ROWS: the fold and the finalize in ONE launch (round 6).  16 waves per block; wave w sums rows
// w, w + 16, ... of the block's 64 columns (lane = column), the 16 wave partials meet in LDS and wave 0 adds them in a
// fixed pairwise order -- deterministic, like the two-stage form it replaces for ResNet18 layer2 / layer3 (784 / 196
// rows at B = 32), one ~5 us launch less per BatchNorm.  Every load of a thread's rows (NB <= 64 of them) is issued
// before the first add: the batches-of-16 loop waited one memory latency per batch, 4 per pass at 784 rows, and the
// finalize ran its sums and its sums of squares as two such passes (13.4 us per launch in the step trace).  The
// forward finalize's columns are the interleaved (sum, sumsq) pairs of 32 channels, so one pass carries both and the
// grid has twice the blocks.  The per-element order (even-ordinal rows into a0, odd into a1, then the wave tree) is
// the batched loop's, so the results are bitwise those of the round-6 kernels.
constexpr int BN_WIDE_ROWS = 1024;

template <int N>
__device__ __forceinline__ float pair_tree(const float* v, int stride) {
  if constexpr (N == 1) {
    return v[0];
  } else {
    return pair_tree<N / 2>(v, stride) + pair_tree<N / 2>(v + (N / 2) * stride, stride);
  }
}

// per-(wave, element) partial over rows w, w + 16, ... (< rows <= 16 * NB): x[r * ld + e]
// (32-bit offsets from the column's base: rows * ld < 2^31 for every caller, and 64 loads in flight fit in 128 VGPRs)
template <int NB>
__device__ __forceinline__ float wide_rows_sum(const float* __restrict__ x, int rows, int ld, int e, int w) {
  float v[NB];
  const float* __restrict__ xe = x + e;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int r = w + 16 * i;
    v[i] = xe[(r < rows ? r : rows - 1) * ld];
  }
  float a0 = 0.f, a1 = 0.f;
#pragma unroll
  for (int i = 0; i < NB; i += 2) {
    if (w + 16 * i < rows) a0 += v[i];
    if (w + 16 * (i + 1) < rows) a1 += v[i + 1];
  }
  return a0 + a1;
}

template <int NB>
__device__ __forceinline__ void bn_finalize_wide_body(int C, long M, int rows, const float* __restrict__ stats,
                                                      float eps, float momentum, float* __restrict__ ms,
                                                      float* __restrict__ rmean, float* __restrict__ rvar,
                                                      long long* __restrict__ nbt, float (*part)[64]) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + l;  // column of the [rows][C][2] layout: channel col / 2, sum (even) / sumsq (odd)
  if (blockIdx.x * 64 >= 2 * C) return;  // (block-uniform: the paired launch's grid covers the wider record)
  part[w][l] = wide_rows_sum<NB>(stats, rows, 2 * C, col < 2 * C ? col : 2 * C - 1, w);
  __syncthreads();
  if (w != 0) return;
  const float tot = pair_tree<16>(&part[0][l], 64);
  const float sq = __shfl_xor(tot, 1, 64);
  const int c = col >> 1;
  if ((l & 1) || c >= C) return;
  const float sum = tot;
  const float mean = sum / M;
  const float var = fmaxf(sq / M - mean * mean, 0.f);
  ms[2 * c] = mean;
  ms[2 * c + 1] = rsqrtf(var + eps);
  if (rmean) rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
  if (rvar) rvar[c] = (1.f - momentum) * rvar[c] + momentum * var * ((float)M / (float)(M > 1 ? M - 1 : 1));
  if (nbt && c == 0) *nbt += 1;
}

template <int NB>
__global__ __launch_bounds__(1024) void bn_finalize_wide_kernel(int C, long M, int rows, const float* __restrict__ stats,
                                                                float eps, float momentum, float* __restrict__ ms,
                                                                float* __restrict__ rmean, float* __restrict__ rvar,
                                                                long long* __restrict__ nbt) {
  __shared__ float part[16][64];
  bn_finalize_wide_body<NB>(C, M, rows, stats, eps, momentum, ms, rmean, rvar, nbt, part);
}

// Two BatchNorms' finalizes in one launch (blockIdx.y = record): a stride-2 BasicBlock's bn2 and downsample BN, whose
// convs both end before either BatchNorm is applied -- one ~4-7 us launch less on the trunk stream per such block.
struct BnFinRec {
  int C, rows;
  long M;
  const float* stats;
  float *ms, *rmean, *rvar;
  long long* nbt;
};
struct BnFinPair {
  BnFinRec r[2];
};
template <int NB>
__global__ __launch_bounds__(1024) void bn_finalize_wide2_kernel(BnFinPair t, float eps, float momentum) {
  __shared__ float part[16][64];
  const bool y = blockIdx.y != 0;  // (uniform selects: an indexed kernel-argument record cost scratch at NB = 64)
  bn_finalize_wide_body<NB>(y ? t.r[1].C : t.r[0].C, y ? t.r[1].M : t.r[0].M, y ? t.r[1].rows : t.r[0].rows,
                            y ? t.r[1].stats : t.r[0].stats, eps, momentum, y ? t.r[1].ms : t.r[0].ms,
                            y ? t.r[1].rmean : t.r[0].rmean, y ? t.r[1].rvar : t.r[0].rvar,
                            y ? t.r[1].nbt : t.r[0].nbt, part);
}

// out[e] = sum over parts rows of in[p][e], e < 2C, for 64 < parts <= BN_WIDE_ROWS (one launch; see above)
template <int NB>
__global__ __launch_bounds__(1024) void partials_sum_wide_kernel(int C2, int parts, const float* __restrict__ in,
                                                                 float* __restrict__ out) {
  __shared__ float part[16][64];
  const int el = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + el, ec = e < C2 ? e : C2 - 1;
  part[w][el] = wide_rows_sum<NB>(in, parts, C2, ec, w);
  __syncthreads();
  if (w == 0 && e < C2) out[e] = pair_tree<16>(&part[0][el], 64);
}
// two buffers of the same shape in one launch (blockIdx.y): a stride-2 block's bn2 and downsample-BN backward sums,
// which one fused dgrad epilogue produced
template <int NB>
__global__ __launch_bounds__(1024) void partials_sum_wide2_kernel(int C2, int parts, const float* __restrict__ in0,
                                                                  float* __restrict__ out0,
                                                                  const float* __restrict__ in1,
                                                                  float* __restrict__ out1) {
  __shared__ float part[16][64];
  const float* in = blockIdx.y ? in1 : in0;
  float* out = blockIdx.y ? out1 : out0;
  const int el = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + el, ec = e < C2 ? e : C2 - 1;
  part[w][el] = wide_rows_sum<NB>(in, parts, C2, ec, w);
  __syncthreads();
  if (w == 0 && e < C2) out[e] = pair_tree<16>(&part[0][el], 64);
}

// the wide launches by row count: NB = 16 / 32 / 64 loads per thread
template <class F16, class F32, class F64>
static inline void wide_pick(int rows, F16 f16, F32 f32, F64 f64) {
  if (rows <= 256) f16();
  else if (rows <= 512) f32();
  else f64();
}

MER_API int mer_bn_finalize(int C, long M, const float* stats, float eps, float momentum, float* ms, float* rmean,
                            float* rvar, long long* num_batches_tracked, void* stream) {
  return mer_bn_finalize_rows(C, M, (int)((M + 63) / 64), stats, eps, momentum, ms, rmean, rvar, num_batches_tracked,
                              stream);
}

MER_API int mer_bn_finalize_rows2(int C, long M, int data_rows, const float* stats, float* ms, float* rmean, float* rvar,
                                  long long* nbt, int C2, long M2, int data_rows2, const float* stats2, float* ms2,
                                  float* rmean2, float* rvar2, long long* nbt2, float eps, float momentum,
                                  void* stream) {
  if (!stats || !stats2 || C <= 0 || C2 <= 0 || data_rows <= 0 || data_rows > (M + 63) / 64 || data_rows2 <= 0 ||
      data_rows2 > (M2 + 63) / 64)
    return (int)hipErrorInvalidValue;
  const int rows = data_rows > data_rows2 ? data_rows : data_rows2;
  if (rows > BN_WIDE_ROWS) {  // the two-stage folds, one after the other
    const int rc = mer_bn_finalize_rows(C, M, data_rows, stats, eps, momentum, ms, rmean, rvar, nbt, stream);
    return rc ? rc : mer_bn_finalize_rows(C2, M2, data_rows2, stats2, eps, momentum, ms2, rmean2, rvar2, nbt2, stream);
  }
  BnFinPair t{};
  t.r[0] = BnFinRec{C, data_rows, M, stats, ms, rmean, rvar, nbt};
  t.r[1] = BnFinRec{C2, data_rows2, M2, stats2, ms2, rmean2, rvar2, nbt2};
  const int cmax = C > C2 ? C : C2;
  const dim3 grid((2 * cmax + 63) / 64, 2);
  hipStream_t st = (hipStream_t)stream;
#define MER_BN_FIN2(NB) [&] { hipLaunchKernelGGL(bn_finalize_wide2_kernel<NB>, grid, dim3(1024), 0, st, t, eps, momentum); }
  wide_pick(rows, MER_BN_FIN2(16), MER_BN_FIN2(32), MER_BN_FIN2(64));
#undef MER_BN_FIN2
  MER_LAUNCH_CHECK();
}

MER_API int mer_bn_finalize_rows(int C, long M, int data_rows, const float* stats, float eps, float momentum, float* ms,
                                 float* rmean, float* rvar, long long* num_batches_tracked, void* stream) {
  if (!stats && (!rmean || !rvar)) return (int)hipErrorInvalidValue;
  const int all_rows = (int)((M + 63) / 64);  // MER_BN_STAT_ROWS(M) - 64: the scratch rows follow them
  if (data_rows <= 0 || data_rows > all_rows) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int tiles = data_rows;
  const float* src = stats;
  int rows = tiles;
  if (stats && tiles > 64 && tiles <= BN_WIDE_ROWS) {
    const dim3 grid((2 * C + 63) / 64);
#define MER_BN_FIN_WIDE(NB)                                                                                          \
  [&] {                                                                                                              \
    hipLaunchKernelGGL(bn_finalize_wide_kernel<NB>, grid, dim3(1024), 0, st, C, M, tiles, stats, eps, momentum, ms, \
                       rmean, rvar, num_batches_tracked);                                                            \
  }
    wide_pick(tiles, MER_BN_FIN_WIDE(16), MER_BN_FIN_WIDE(32), MER_BN_FIN_WIDE(64));
#undef MER_BN_FIN_WIDE
    MER_LAUNCH_CHECK();
  }
  if (stats && tiles > 64) {
    float* scratch = const_cast<float*>(stats) + (long)all_rows * 2 * C;
    const int per = (tiles + 63) / 64;
    hipLaunchKernelGGL(bn_stat_rows_fold_kernel, dim3((2 * C + 63) / 64, 64), dim3(256), 0, st, 2 * C, tiles, per,
                       stats, scratch);
    src = scratch;
    rows = 64;
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 63) / 64), dim3(256), 0, st, C, M, rows, src, eps, momentum, ms,
                     rmean, rvar, num_batches_tracked);
  MER_LAUNCH_CHECK();
}

// y = [relu]( bn(x) + (res_bn ? bn2(res) : res) ), 8 channels per thread (C % 8 == 0).
// ms = (mean, rstd) pairs; eval mode passes (running_mean, 1/sqrt(running_var+eps)) the same way.
// BN is folded into one (scale, shift) per channel, computed once per block into LDS (C <= 512); a
// thread always owns the same 8 channels (256 % (C/8) == 0 and the grid stride is a multiple of 256) and
// streams two 16-byte vectors per iteration so the loads of both are in flight together.
__global__ __launch_bounds__(256) void bn_apply_kernel(long M, int C, const bf16_t* __restrict__ x,
                                                       const float* __restrict__ ms, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, const bf16_t* __restrict__ res,
                                                       const float* __restrict__ ms2, const float* __restrict__ gamma2,
                                                       const float* __restrict__ beta2, int relu,
                                                       bf16_t* __restrict__ y) {
  __shared__ __attribute__((aligned(16))) float coef[4][512];  // scale, shift, scale2, shift2
  for (int c = threadIdx.x; c < C; c += 256) {
    const float sc = ms[2 * c + 1] * gamma[c];
    coef[0][c] = sc;
    coef[1][c] = beta[c] - ms[2 * c] * sc;
    float sc2 = 1.f, sh2 = 0.f;
    if (ms2) {
      sc2 = ms2[2 * c + 1] * gamma2[c];
      sh2 = beta2[c] - ms2[2 * c] * sc2;
    }
    coef[2][c] = sc2;
    coef[3][c] = sh2;
  }
  __syncthreads();
  const long nvec = M * C / 8;
  const long stride = (long)gridDim.x * blockDim.x;
  const long tid0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int c0 = (int)(tid0 % (C / 8)) * 8;
  float sc[8], sh[8], sc2[8], sh2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = coef[0][c0 + i];
    sh[i] = coef[1][c0 + i];
    sc2[i] = coef[2][c0 + i];
    sh2[i] = coef[3][c0 + i];
  }
  auto one = [&](const u32x4& xv, const u32x4& rv) -> u32x4 {
    const bf16_t* xh = reinterpret_cast<const bf16_t*>(&xv);
    const bf16_t* rh = reinterpret_cast<const bf16_t*>(&rv);
    u32x4 ov;
    bf16_t* oh = reinterpret_cast<bf16_t*>(&ov);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float v = bf2f(xh[i]) * sc[i] + sh[i];
      if (res) v += bf2f(rh[i]) * sc2[i] + sh2[i];
      if (relu) v = fmaxf(v, 0.f);
      oh[i] = f2bf(v);
    }
    return ov;
  };
  const u32x4 z = {0u, 0u, 0u, 0u};
  long e = tid0;
  for (; e + stride < nvec; e += 2 * stride) {
    const u32x4 x0 = *reinterpret_cast<const u32x4*>(x + e * 8);
    const u32x4 x1 = *reinterpret_cast<const u32x4*>(x + (e + stride) * 8);
    const u32x4 r0 = res ? *reinterpret_cast<const u32x4*>(res + e * 8) : z;
    const u32x4 r1 = res ? *reinterpret_cast<const u32x4*>(res + (e + stride) * 8) : z;
    *reinterpret_cast<u32x4*>(y + e * 8) = one(x0, r0);
    *reinterpret_cast<u32x4*>(y + (e + stride) * 8) = one(x1, r1);
  }
  if (e < nvec) {
    const u32x4 x0 = *reinterpret_cast<const u32x4*>(x + e * 8);
    const u32x4 r0 = res ? *reinterpret_cast<const u32x4*>(res + e * 8) : z;
    *reinterpret_cast<u32x4*>(y + e * 8) = one(x0, r0);
  }
}
static int bn_stream_grid(long nvec) {
  const long g = (nvec + 1023) / 1024;  // ~4 vectors per thread
  return (int)(g < 1 ? 1 : g > 2048 ? 2048 : g);
}

MER_API int mer_bn_apply(long M, int C, const void* x, const float* ms, const float* gamma, const float* beta,
                         const void* res, const float* ms2, const float* gamma2, const float* beta2, int relu, void* y,
                         void* stream) {
  if (C % 8 || C > 512 || 256 % (C / 8)) return (int)hipErrorInvalidValue;
  const long nvec = M * C / 8;
  const int grid = bn_stream_grid(nvec);
  hipLaunchKernelGGL(bn_apply_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, M, C, (const bf16_t*)x, ms,
                     gamma, beta, (const bf16_t*)res, ms2, gamma2, beta2, relu, (bf16_t*)y);
  MER_LAUNCH_CHECK();
}

// BatchNorm folded to (scale, shift) for channel c from ms = (mean, rstd) pairs
__device__ __forceinline__ void stem_bn_coef(int c, const float* ms, const float* gamma, const float* beta, float& sc,
                                             float& sh) {
  sc = ms[2 * c + 1] * gamma[c];
  sh = beta[c] - ms[2 * c] * sc;
}

// BN backward reduction: g = dy * (mask > 0) (mask = the ReLU output, or null), xhat from x and ms:
//   red[c] = (sum g, sum g*xhat), one partial row per block folded in block order.  C <= 512, C % 8 == 0.
// BNMASK: no mask tensor; the ReLU mask is recomputed as bf16(relu(x*scale + shift)) > 0 from (ms, mgamma,
// mbeta) -- the fused stem, whose activation is never stored.
template <bool BNMASK>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(long M, int C, const bf16_t* __restrict__ dy,
                                                            const bf16_t* __restrict__ mask,
                                                            const bf16_t* __restrict__ x, const float* __restrict__ ms,
                                                            const float* __restrict__ mgamma,
                                                            const float* __restrict__ mbeta,
                                                            float* __restrict__ rows, long rows_per_block) {
  // per-thread sums over this block's rows, then the rows_per_iter threads of a channel chunk meet in LDS in
  // thread order and the block STORES its partial row: no atomics, deterministic
  __shared__ float part[2][2048];  // [s1|s2][tr * C + c], rows_per_iter * C <= 2048
  const int cpr = C / 8;                     // 16B chunks per row
  const int rows_per_iter = 256 / cpr > 0 ? 256 / cpr : 1;
  const int tc = threadIdx.x % cpr, tr = threadIdx.x / cpr;
  const long r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float s1[8] = {0.f}, s2[8] = {0.f};
  if (tr < rows_per_iter) {
    float mean[8], rstd[8], msc[8], msh[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      mean[i] = ms[2 * (tc * 8 + i)];
      rstd[i] = ms[2 * (tc * 8 + i) + 1];
      if (BNMASK) stem_bn_coef(tc * 8 + i, ms, mgamma, mbeta, msc[i], msh[i]);
    }
    // 4 rows per iteration with every load issued first (unconditional, from clamped rows; a row past r1
    // contributes exact zeros), so a thread has 8-12 loads in flight instead of one row's 2-3: the same rows
    // in the same order as a one-row loop, bit-identical sums
    for (long rb = r0 + tr; rb < r1; rb += 4 * rows_per_iter) {
      u32x4 gv[4], xv[4], mv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long r = rb + u * rows_per_iter;
        const long off = (r < r1 ? r : r1 - 1) * C + tc * 8;
        gv[u] = *reinterpret_cast<const u32x4*>(dy + off);
        xv[u] = *reinterpret_cast<const u32x4*>(x + off);
        mv[u] = u32x4{1u, 1u, 1u, 1u};
        if (!BNMASK && mask) mv[u] = *reinterpret_cast<const u32x4*>(mask + off);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool rowok = rb + u * rows_per_iter < r1;
        const bf16_t* gh = reinterpret_cast<const bf16_t*>(&gv[u]);
        const bf16_t* xh = reinterpret_cast<const bf16_t*>(&xv[u]);
        const bf16_t* mh = reinterpret_cast<const bf16_t*>(&mv[u]);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const bool live = BNMASK ? bf2f(f2bf(fmaxf(bf2f(xh[i]) * msc[i] + msh[i], 0.f))) > 0.f
                                   : (!mask || bf2f(mh[i]) > 0.f);
          const float g = (live && rowok) ? bf2f(gh[i]) : 0.f;
          if (rowok) {  // (a select: the loads above are unconditional)
            s1[i] += g;
            s2[i] += g * (bf2f(xh[i]) - mean[i]) * rstd[i];
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      part[0][tr * C + tc * 8 + i] = s1[i];
      part[1][tr * C + tc * 8 + i] = s2[i];
    }
  }
  __syncthreads();
  float* out = rows + (long)blockIdx.x * C * 2;
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int q = 0; q < rows_per_iter; ++q) {
      a += part[0][q * C + c];
      b += part[1][q * C + c];
    }
    out[2 * c] = a;
    out[2 * c + 1] = b;
  }
}
// rows_per_block keeps the block count <= 512 (the workspace holds MER_BN_RED_WS_ROWS = 512 + 64 rows)
static long bn_bwd_reduce_rpb(long M) { return (M + 511) / 512 > 32 ? (M + 511) / 512 : 32; }
static int partials_fold(int C, int parts, float* in, float* out, hipStream_t st);
MER_API int mer_bn_bwd_reduce(long M, int C, const void* dy, const void* mask, const void* x, const float* ms,
                              float* red, float* workspace, void* stream) {
  if (C % 8 || C > 512) return (int)hipErrorInvalidValue;
  const long rpb = bn_bwd_reduce_rpb(M);
  const int blocks = (int)((M + rpb - 1) / rpb);
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<false>), dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, M, C,
                     (const bf16_t*)dy, (const bf16_t*)mask, (const bf16_t*)x, ms, (const float*)nullptr,
                     (const float*)nullptr, workspace, rpb);
  return partials_fold(C, blocks, workspace, red, (hipStream_t)stream);
}

// out[c] = sum_p in[p][c] over `parts` partial rows of (a, b) pairs (fused-epilogue reductions), in a fixed
// order; 64 entries per block, the 4 waves split the rows, then meet in LDS.  More than 64 rows are first
// folded (bn_stat_rows_fold_kernel) into the 64 scratch rows the caller provides after them.
__global__ __launch_bounds__(256) void partials_sum_kernel(int C, int parts, const float* __restrict__ in,
                                                           float* __restrict__ out) {
  __shared__ float part[4][64];
  const int el = threadIdx.x & 63, pg = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + el;
  float acc = 0.f;
  {  // parts <= 64: this wave's <= 16 rows all in flight before the first add (same order)
    const int ec = e < 2 * C ? e : 2 * C - 1;
    float x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int p = pg + 4 * i;
      x[i] = in[(long)(p < parts ? p : parts - 1) * 2 * C + ec];
    }
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (pg + 4 * i < parts) acc += x[i];
  }
  part[pg][el] = acc;
  __syncthreads();
  if (pg == 0 && e < 2 * C) out[e] = part[0][el] + part[1][el] + part[2][el] + part[3][el];
}
static int partials_fold(int C, int parts, float* in, float* out, hipStream_t st) {
  const float* src = in;
  if (parts > 64 && parts <= BN_WIDE_ROWS) {
    const dim3 grid((2 * C + 63) / 64);
#define MER_PSUM_WIDE(NB) \
  [&] { hipLaunchKernelGGL(partials_sum_wide_kernel<NB>, grid, dim3(1024), 0, st, 2 * C, parts, in, out); }
    wide_pick(parts, MER_PSUM_WIDE(16), MER_PSUM_WIDE(32), MER_PSUM_WIDE(64));
#undef MER_PSUM_WIDE
    MER_LAUNCH_CHECK();
  }
  if (parts > 64) {
    float* scratch = in + (long)parts * 2 * C;
    const int per = (parts + 63) / 64;
    hipLaunchKernelGGL(bn_stat_rows_fold_kernel, dim3((2 * C + 63) / 64, 64), dim3(256), 0, st, 2 * C, parts, per, in,
                       scratch);
    src = scratch;
    parts = 64;
  }
  hipLaunchKernelGGL(partials_sum_kernel, dim3((2 * C + 63) / 64), dim3(256), 0, st, C, parts, src, out);
  MER_LAUNCH_CHECK();
}
MER_API int mer_partials_sum(int C, int parts, float* in, float* out, void* stream) {
  if (C <= 0 || parts <= 0) return (int)hipErrorInvalidValue;
  return partials_fold(C, parts, in, out, (hipStream_t)stream);
}

MER_API int mer_partials_sum2(int C, int parts, float* in, float* out, float* in2, float* out2, void* stream) {
  if (C <= 0 || parts <= 0 || !in || !out || !in2 || !out2) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (parts > BN_WIDE_ROWS) {  // the two-stage folds, one after the other
    const int rc = partials_fold(C, parts, in, out, st);
    return rc ? rc : partials_fold(C, parts, in2, out2, st);
  }
  const dim3 grid((2 * C + 63) / 64, 2);
#define MER_PSUM2(NB) \
  [&] { hipLaunchKernelGGL(partials_sum_wide2_kernel<NB>, grid, dim3(1024), 0, st, 2 * C, parts, in, out, in2, out2); }
  wide_pick(parts, MER_PSUM2(16), MER_PSUM2(32), MER_PSUM2(64));
#undef MER_PSUM2
  MER_LAUNCH_CHECK();
}

// dx = gamma*rstd*(g - s1/M - xhat*s2/M) (bf16), and (block 0) dgamma += s2, dbeta += s1.
// Affine in (g, x) once the sums are known: dx = k1*g + k2*x + k0 per channel, the constants computed once
// per block into LDS; same thread/channel ownership and 2-vector streaming as bn_apply_kernel.
// (BNMASK as in bn_bwd_reduce_kernel; dy and dx may alias: every element is read, then written, by one thread)
template <bool BNMASK>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(long M, int C, const bf16_t* dy,
                                                           const bf16_t* __restrict__ mask,
                                                           const bf16_t* __restrict__ x, const float* __restrict__ ms,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ mbeta,
                                                           const float* __restrict__ red, int batch_stats,
                                                           bf16_t* dx, float* __restrict__ dgamma,
                                                           float* __restrict__ dbeta) {
  __shared__ __attribute__((aligned(16))) float coef[5][512];
  const float invM = 1.f / (float)M;
  for (int c = threadIdx.x; c < C; c += 256) {
    if (blockIdx.x == 0) {
      if (dgamma) dgamma[c] += red[2 * c + 1];
      if (dbeta) dbeta[c] += red[2 * c];
    }
    const float mu = ms[2 * c], rs = ms[2 * c + 1], gr = gamma[c] * rs;
    // batch statistics (train): the mean/var terms carry gradient; running stats (eval): they do not
    const float a = batch_stats ? red[2 * c] * invM : 0.f;
    const float b = batch_stats ? red[2 * c + 1] * invM : 0.f;
    const float t = gr * b * rs;  // (explicit rounding steps, shared with bn_bwd_apply2_kernel)
    coef[0][c] = gr;
    coef[1][c] = -t;
    coef[2][c] = fmaf(-gr, a, t * mu);
    if (BNMASK) stem_bn_coef(c, ms, gamma, mbeta, coef[3][c], coef[4][c]);
  }
  __syncthreads();
  const long nvec = M * C / 8;
  const long stride = (long)gridDim.x * blockDim.x;
  const long tid0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int c0 = (int)(tid0 % (C / 8)) * 8;
  float k1[8], k2[8], k0[8], msc[8], msh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    k1[i] = coef[0][c0 + i];
    k2[i] = coef[1][c0 + i];
    k0[i] = coef[2][c0 + i];
    msc[i] = BNMASK ? coef[3][c0 + i] : 0.f;
    msh[i] = BNMASK ? coef[4][c0 + i] : 0.f;
  }
  auto one = [&](const u32x4& gv, const u32x4& xv, const u32x4& mv) -> u32x4 {
    const bf16_t* gh = reinterpret_cast<const bf16_t*>(&gv);
    const bf16_t* xh = reinterpret_cast<const bf16_t*>(&xv);
    const bf16_t* mh = reinterpret_cast<const bf16_t*>(&mv);
    u32x4 ov;
    bf16_t* oh = reinterpret_cast<bf16_t*>(&ov);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bool live = BNMASK ? bf2f(f2bf(fmaxf(bf2f(xh[i]) * msc[i] + msh[i], 0.f))) > 0.f
                               : (!mask || bf2f(mh[i]) > 0.f);
      const float g = live ? bf2f(gh[i]) : 0.f;
      oh[i] = f2bf(fmaf(k1[i], g, fmaf(k2[i], bf2f(xh[i]), k0[i])));  // explicit: apply2 rounds the same
    }
    return ov;
  };
  const u32x4 one16 = {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};  // bf16 1.0 (no mask)
  long e = tid0;
  for (; e + stride < nvec; e += 2 * stride) {
    const long e1 = e + stride;
    const u32x4 g0 = *reinterpret_cast<const u32x4*>(dy + e * 8);
    const u32x4 g1 = *reinterpret_cast<const u32x4*>(dy + e1 * 8);
    const u32x4 x0 = *reinterpret_cast<const u32x4*>(x + e * 8);
    const u32x4 x1 = *reinterpret_cast<const u32x4*>(x + e1 * 8);
    const u32x4 m0 = (!BNMASK && mask) ? *reinterpret_cast<const u32x4*>(mask + e * 8) : one16;
    const u32x4 m1 = (!BNMASK && mask) ? *reinterpret_cast<const u32x4*>(mask + e1 * 8) : one16;
    *reinterpret_cast<u32x4*>(dx + e * 8) = one(g0, x0, m0);
    *reinterpret_cast<u32x4*>(dx + e1 * 8) = one(g1, x1, m1);
  }
  if (e < nvec) {
    const u32x4 g0 = *reinterpret_cast<const u32x4*>(dy + e * 8);
    const u32x4 x0 = *reinterpret_cast<const u32x4*>(x + e * 8);
    const u32x4 m0 = (!BNMASK && mask) ? *reinterpret_cast<const u32x4*>(mask + e * 8) : one16;
    *reinterpret_cast<u32x4*>(dx + e * 8) = one(g0, x0, m0);
  }
}
MER_API int mer_bn_bwd_apply(long M, int C, const void* dy, const void* mask, const void* x, const float* ms,
                             const float* gamma, const float* red, int batch_stats, void* dx, float* dgamma,
                             float* dbeta, void* stream) {
  if (C % 8 || C > 512 || 256 % (C / 8)) return (int)hipErrorInvalidValue;
  const long nvec = M * C / 8;
  const int grid = bn_stream_grid(nvec);
  hipLaunchKernelGGL((bn_bwd_apply_kernel<false>), dim3(grid), dim3(256), 0, (hipStream_t)stream, M, C,
                     (const bf16_t*)dy, (const bf16_t*)mask, (const bf16_t*)x, ms, gamma, (const float*)nullptr, red,
                     batch_stats, (bf16_t*)dx, dgamma, dbeta);
  MER_LAUNCH_CHECK();
}

// Two BatchNorm backward applies that read the same gradient and ReLU mask: a stride-2 BasicBlock's bn2 and its
// downsample BN (the block output relu(bn2(c2) + bn_d(cd)) fans its gradient out to both).  One pass loads g and the
// mask once for both outputs -- 12 instead of 16 bytes per element and one launch less -- with each output's
// per-element arithmetic exactly bn_bwd_apply_kernel<false>'s (bit-identical to two launches).
__global__ __launch_bounds__(256) void bn_bwd_apply2_kernel(long M, int C, const bf16_t* __restrict__ dy,
                                                            const bf16_t* __restrict__ mask,
                                                            const bf16_t* __restrict__ x, const float* __restrict__ ms,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ red,
                                                            const bf16_t* __restrict__ x2,
                                                            const float* __restrict__ ms2,
                                                            const float* __restrict__ gamma2,
                                                            const float* __restrict__ red2, int batch_stats,
                                                            bf16_t* __restrict__ dx, bf16_t* __restrict__ dx2,
                                                            float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                            float* __restrict__ dgamma2, float* __restrict__ dbeta2) {
  __shared__ __attribute__((aligned(16))) float coef[6][512];
  const float invM = 1.f / (float)M;
  for (int c = threadIdx.x; c < C; c += 256) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float* rd = h ? red2 : red;
      const float* m = h ? ms2 : ms;
      if (blockIdx.x == 0) {
        float* dg = h ? dgamma2 : dgamma;
        float* db = h ? dbeta2 : dbeta;
        if (dg) dg[c] += rd[2 * c + 1];
        if (db) db[c] += rd[2 * c];
      }
      const float mu = m[2 * c], rs = m[2 * c + 1], gr = (h ? gamma2 : gamma)[c] * rs;
      const float a = batch_stats ? rd[2 * c] * invM : 0.f;
      const float b = batch_stats ? rd[2 * c + 1] * invM : 0.f;
      const float t = gr * b * rs;
      coef[3 * h + 0][c] = gr;
      coef[3 * h + 1][c] = -t;
      coef[3 * h + 2][c] = fmaf(-gr, a, t * mu);
    }
  }
  __syncthreads();
  const long nvec = M * C / 8;
  const long stride = (long)gridDim.x * blockDim.x;
  const long tid0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int c0 = (int)(tid0 % (C / 8)) * 8;
  float k[6][8];
#pragma unroll
  for (int j = 0; j < 6; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) k[j][i] = coef[j][c0 + i];
  for (long e = tid0; e < nvec; e += stride) {
    const u32x4 gv = *reinterpret_cast<const u32x4*>(dy + e * 8);
    const u32x4 mv = *reinterpret_cast<const u32x4*>(mask + e * 8);
    const u32x4 xv = *reinterpret_cast<const u32x4*>(x + e * 8);
    const u32x4 x2v = *reinterpret_cast<const u32x4*>(x2 + e * 8);
    const bf16_t* gh = reinterpret_cast<const bf16_t*>(&gv);
    const bf16_t* mh = reinterpret_cast<const bf16_t*>(&mv);
    const bf16_t* xh = reinterpret_cast<const bf16_t*>(&xv);
    const bf16_t* x2h = reinterpret_cast<const bf16_t*>(&x2v);
    u32x4 ov, o2v;
    bf16_t* oh = reinterpret_cast<bf16_t*>(&ov);
    bf16_t* o2h = reinterpret_cast<bf16_t*>(&o2v);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float g = bf2f(mh[i]) > 0.f ? bf2f(gh[i]) : 0.f;
      oh[i] = f2bf(fmaf(k[0][i], g, fmaf(k[1][i], bf2f(xh[i]), k[2][i])));
      o2h[i] = f2bf(fmaf(k[3][i], g, fmaf(k[4][i], bf2f(x2h[i]), k[5][i])));
    }
    *reinterpret_cast<u32x4*>(dx + e * 8) = ov;
    *reinterpret_cast<u32x4*>(dx2 + e * 8) = o2v;
  }
}
MER_API int mer_bn_bwd_apply2(long M, int C, const void* dy, const void* mask, const void* x, const float* ms,
                              const float* gamma, const float* red, const void* x2, const float* ms2,
                              const float* gamma2, const float* red2, int batch_stats, void* dx, void* dx2,
                              float* dgamma, float* dbeta, float* dgamma2, float* dbeta2, void* stream) {
  if (C % 8 || C > 512 || 256 % (C / 8) || !mask || !x2 || !dx2 || dx == dy || dx2 == dy)
    return (int)hipErrorInvalidValue;
  const long nvec = M * C / 8;
  const int grid = bn_stream_grid(nvec);
  hipLaunchKernelGGL(bn_bwd_apply2_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, M, C, (const bf16_t*)dy,
                     (const bf16_t*)mask, (const bf16_t*)x, ms, gamma, red, (const bf16_t*)x2, ms2, gamma2, red2,
                     batch_stats, (bf16_t*)dx, (bf16_t*)dx2, dgamma, dbeta, dgamma2, dbeta2);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// MaxPool2d(3, 2, 1) (resnet stem) channel-last, with the argmax tap (0..8) saved for backward.
// ---------------------------------------------------------------------------------------
// 8 channels (16 B) per thread; pixel index decomposed with fdiv (N*Ho*Wo < 2^22)
__global__ void maxpool_fwd_kernel(int N, int H, int W, int C, int Ho, int Wo, const bf16_t* __restrict__ x,
                                   bf16_t* __restrict__ y, uint8_t* __restrict__ arg) {
  const int cpr = C / 8;
  const int total = N * Ho * Wo * cpr;
  const float inv_cpr = 1.f / cpr, inv_Wo = 1.f / Wo, inv_Ho = 1.f / Ho;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int q = fdiv(e, inv_cpr);
    const int c0 = (e - q * cpr) * 8;
    const int q2 = fdiv(q, inv_Wo);
    const int ow = q - q2 * Wo;
    const int n = fdiv(q2, inv_Ho);
    const int oh = q2 - n * Ho;
    float best[8];
    int bi[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { best[i] = -INFINITY; bi[i] = 0; }
    for (int r = 0; r < 3; ++r)
      for (int s = 0; s < 3; ++s) {
        const int ih = oh * 2 - 1 + r, iw = ow * 2 - 1 + s;
        if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
        const u32x4 v = *reinterpret_cast<const u32x4*>(x + (((long)n * H + ih) * W + iw) * C + c0);
        const bf16_t* vh = reinterpret_cast<const bf16_t*>(&v);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float f = bf2f(vh[i]);
          if (f > best[i]) { best[i] = f; bi[i] = r * 3 + s; }  // first max wins, like torch
        }
      }
    u32x4 o;
    bf16_t* oh8 = reinterpret_cast<bf16_t*>(&o);
    uint2 a;
    uint8_t* a8 = reinterpret_cast<uint8_t*>(&a);
#pragma unroll
    for (int i = 0; i < 8; ++i) { oh8[i] = f2bf(best[i]); a8[i] = (uint8_t)bi[i]; }
    *reinterpret_cast<u32x4*>(y + (long)q * C + c0) = o;
    *reinterpret_cast<uint2*>(arg + (long)q * C + c0) = a;
  }
}
MER_API int mer_maxpool_fwd(int N, int H, int W, int C, const void* x, void* y, void* argmax, void* stream) {
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  if (C % 8 || (long)N * H * W >= (1L << 22)) return (int)hipErrorInvalidValue;
  const long total = (long)N * Ho * Wo * C / 8;
  const int grid = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, N, H, W, C, Ho, Wo,
                     (const bf16_t*)x, (bf16_t*)y, (uint8_t*)argmax);
  MER_LAUNCH_CHECK();
}
// gather backward: dx[n,h,w,c] = sum of dy over the (<= 4) windows whose argmax is (h,w)
__global__ void maxpool_bwd_kernel(int N, int H, int W, int C, int Ho, int Wo, const bf16_t* __restrict__ dy,
                                   const uint8_t* __restrict__ arg, bf16_t* __restrict__ dx) {
  const int cpr = C / 8;
  const int total = N * H * W * cpr;
  const float inv_cpr = 1.f / cpr, inv_W = 1.f / W, inv_H = 1.f / H;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int q = fdiv(e, inv_cpr);
    const int c0 = (e - q * cpr) * 8;
    const int q2 = fdiv(q, inv_W);
    const int w = q - q2 * W;
    const int n = fdiv(q2, inv_H);
    const int h = q2 - n * H;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // the (<= 4) candidate windows: every load unconditional from a clamped window, invalid ones masked by the
    // tap test (a load under a per-lane branch waits for itself: 4 dependent round trips per thread)
    u32x4 gq[2][2];
    uint2 aq[2][2];
    int tap[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int oh = (h + 1) / 2 - 1 + a, ow = (w + 1) / 2 - 1 + b;
        const int r = h - (oh * 2 - 1), s = w - (ow * 2 - 1);
        const bool ok = oh >= 0 && oh < Ho && ow >= 0 && ow < Wo && r >= 0 && r <= 2 && s >= 0 && s <= 2;
        const int ohc = oh < 0 ? 0 : (oh >= Ho ? Ho - 1 : oh), owc = ow < 0 ? 0 : (ow >= Wo ? Wo - 1 : ow);
        const long oi = (((long)n * Ho + ohc) * Wo + owc) * C + c0;
        gq[a][b] = *reinterpret_cast<const u32x4*>(dy + oi);
        aq[a][b] = *reinterpret_cast<const uint2*>(arg + oi);
        tap[a][b] = ok ? r * 3 + s : -1;  // -1 matches no argmax
      }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const bf16_t* gh = reinterpret_cast<const bf16_t*>(&gq[a][b]);
        const uint8_t* a8 = reinterpret_cast<const uint8_t*>(&aq[a][b]);
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if ((int)a8[i] == tap[a][b]) acc[i] += bf2f(gh[i]);
      }
    u32x4 o;
    bf16_t* oh8 = reinterpret_cast<bf16_t*>(&o);
#pragma unroll
    for (int i = 0; i < 8; ++i) oh8[i] = f2bf(acc[i]);
    *reinterpret_cast<u32x4*>(dx + (long)q * C + c0) = o;
  }
}
MER_API int mer_maxpool_bwd(int N, int H, int W, int C, const void* dy, const void* argmax, void* dx, void* stream) {
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  if (C % 8 || (long)N * H * W >= (1L << 22)) return (int)hipErrorInvalidValue;
  const long total = (long)N * H * W * C / 8;
  const int grid = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, N, H, W, C, Ho, Wo,
                     (const bf16_t*)dy, (const uint8_t*)argmax, (bf16_t*)dx);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// Fused ResNet stem tail (video.py:21-23 -> torchvision conv1/bn1/relu/maxpool), channel-last, C = 64:
//   forward:  p = maxpool3x3s2p1( a ),  a = bf16(relu(x * scale + shift))  -- a is never stored;
//   backward: da = maxpool gather of dp (materialised once by maxpool_bwd), g = da * (a > 0) with the ReLU
//             mask recomputed from (x, BN) in the BatchNorm reduction and apply passes, so a is never stored
//             (gathering dp inside both passes instead was measured 2x slower: DESIGN.md section 4e).
// Same roundings, tap order and tie rule as bn_apply -> maxpool_fwd / maxpool_bwd -> bn_bwd_*.
// ---------------------------------------------------------------------------------------

__global__ void stem_bnrelu_maxpool_kernel(int N, int H, int W, int C, int Ho, int Wo, const bf16_t* __restrict__ x,
                                           const float* __restrict__ ms, const float* __restrict__ gamma,
                                           const float* __restrict__ beta, bf16_t* __restrict__ y,
                                           uint8_t* __restrict__ arg) {
  const int cpr = C / 8;
  const int total = N * Ho * Wo * cpr;
  const float inv_cpr = 1.f / cpr, inv_Wo = 1.f / Wo, inv_Ho = 1.f / Ho;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int q = fdiv(e, inv_cpr);
    const int c0 = (e - q * cpr) * 8;
    const int q2 = fdiv(q, inv_Wo);
    const int ow = q - q2 * Wo;
    const int n = fdiv(q2, inv_Ho);
    const int oh = q2 - n * Ho;
    float sc[8], sh[8], best[8];
    int bi[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      stem_bn_coef(c0 + i, ms, gamma, beta, sc[i], sh[i]);
      best[i] = -INFINITY;
      bi[i] = 0;
    }
    // all 9 taps loaded first, unconditionally from clamped pixels (branch-free: the loads are in flight
    // together), out-of-frame taps masked to -inf so they never win; same tap order and first-max tie rule
    u32x4 v[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ih = oh * 2 - 1 + t / 3, iw = ow * 2 - 1 + t % 3;
      const int ihc = ih < 0 ? 0 : (ih >= H ? H - 1 : ih), iwc = iw < 0 ? 0 : (iw >= W ? W - 1 : iw);
      v[t] = *reinterpret_cast<const u32x4*>(x + (((long)n * H + ihc) * W + iwc) * C + c0);
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ih = oh * 2 - 1 + t / 3, iw = ow * 2 - 1 + t % 3;
      const bool ok = ih >= 0 && ih < H && iw >= 0 && iw < W;
      const bf16_t* vh = reinterpret_cast<const bf16_t*>(&v[t]);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float f = ok ? bf2f(f2bf(fmaxf(bf2f(vh[i]) * sc[i] + sh[i], 0.f))) : -INFINITY;
        if (f > best[i]) { best[i] = f; bi[i] = t; }
      }
    }
    u32x4 o;
    bf16_t* oh8 = reinterpret_cast<bf16_t*>(&o);
    uint2 a;
    uint8_t* a8 = reinterpret_cast<uint8_t*>(&a);
#pragma unroll
    for (int i = 0; i < 8; ++i) { oh8[i] = f2bf(best[i]); a8[i] = (uint8_t)bi[i]; }
    *reinterpret_cast<u32x4*>(y + (long)q * C + c0) = o;
    *reinterpret_cast<uint2*>(arg + (long)q * C + c0) = a;
  }
}

MER_API int mer_stem_bnrelu_maxpool_fwd(int N, int H, int W, int C, const void* x, const float* ms, const float* gamma,
                                        const float* beta, void* y, void* argmax, void* stream) {
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  if (C % 8 || C > 512 || (long)N * H * W >= (1L << 22)) return (int)hipErrorInvalidValue;
  const long total = (long)N * Ho * Wo * C / 8;
  const int grid = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
  hipLaunchKernelGGL(stem_bnrelu_maxpool_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, N, H, W, C, Ho, Wo,
                     (const bf16_t*)x, ms, gamma, beta, (bf16_t*)y, (uint8_t*)argmax);
  MER_LAUNCH_CHECK();
}

MER_API int mer_stem_pool_bn_bwd(int N, int H, int W, int C, const void* dy, const void* argmax, const void* x,
                                 const float* ms, const float* gamma, const float* beta, float* red, int batch_stats,
                                 void* dx, float* dgamma, float* dbeta, float* workspace, void* stream) {
  if (C % 8 || C > 512 || 256 % (C / 8) || (long)N * H * W >= (1L << 22)) return (int)hipErrorInvalidValue;
  const hipStream_t st = (hipStream_t)stream;
  const long M = (long)N * H * W;
  // 1) maxpool gather backward into dx (as the pre-BN gradient); 2) BN reduction with the ReLU mask
  // recomputed from (x, BN); 3) BN apply in place over dx (each element read, then written, by one thread)
  int rc = mer_maxpool_bwd(N, H, W, C, dy, argmax, dx, stream);
  if (rc) return rc;
  const long rpb = bn_bwd_reduce_rpb(M);
  const int blocks = (int)((M + rpb - 1) / rpb);
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<true>), dim3((unsigned)blocks), dim3(256), 0, st, M, C, (const bf16_t*)dx,
                     (const bf16_t*)nullptr, (const bf16_t*)x, ms, gamma, beta, workspace, rpb);
  rc = partials_fold(C, blocks, workspace, red, st);
  if (rc) return rc;
  hipLaunchKernelGGL((bn_bwd_apply_kernel<true>), dim3(bn_stream_grid(M * C / 8)), dim3(256), 0, st, M, C,
                     (const bf16_t*)dx, (const bf16_t*)nullptr, (const bf16_t*)x, ms, gamma, beta, red, batch_stats,
                     (bf16_t*)dx, dgamma, dbeta);
  MER_LAUNCH_CHECK();
}

// global average pool (AdaptiveAvgPool2d(1)): NHWC bf16 -> [N, C] fp32; backward broadcasts dy/HW.
__global__ void avgpool_fwd_kernel(int N, int HW, int C, const bf16_t* __restrict__ x, float* __restrict__ y) {
  const int n = blockIdx.y, c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int p = 0; p < HW; ++p) s += bf2f(x[((long)n * HW + p) * C + c]);
  y[(long)n * C + c] = s / HW;
}
__global__ void avgpool_bwd_kernel(int N, int HW, int C, const float* __restrict__ dy, bf16_t* __restrict__ dx) {
  const int n = blockIdx.y;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < HW * C; e += gridDim.x * blockDim.x) {
    const int c = e % C;
    dx[(long)n * HW * C + e] = f2bf(dy[(long)n * C + c] / HW);
  }
}
MER_API int mer_avgpool_fwd(int N, int HW, int C, const void* x, float* y, void* stream) {
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3((C + 255) / 256, N), dim3(256), 0, (hipStream_t)stream, N, HW, C,
                     (const bf16_t*)x, y);
  MER_LAUNCH_CHECK();
}
MER_API int mer_avgpool_bwd(int N, int HW, int C, const float* dy, void* dx, void* stream) {
  dim3 grid((HW * C + 255) / 256, N);
  hipLaunchKernelGGL(avgpool_bwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, N, HW, C, dy, (bf16_t*)dx);
  MER_LAUNCH_CHECK();
}
