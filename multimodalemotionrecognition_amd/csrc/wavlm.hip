// WavLM-base forward kernels (frozen encoder of the north-star path, wavlm_audio.py:165-183).
// Citations TF:<line> are transformers' modeling_wavlm.py (installed 5.15.0).
#include "common.h"
#include "mer.h"

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(8))) float f32x8;

// ---------------------------------------------------------------------------------------
// Feature-extractor layer 0 (TF:723-745): conv0 = Conv1d(1, 512, k=10, s=5, bias=False) on the raw
// waveform, GroupNorm(512, 512) over time per (clip, channel), GELU; channel-last bf16 output.
// The conv is 10 MACs per output, so instead of writing the conv output, reading it back for the
// statistics and again for the normalisation (3 x 314 MB at B=32), pass 1 computes the conv tile by
// tile and keeps only per-tile partial (sum, sumsq) rows, a finalize reduces them in a fixed order
// (deterministic), and pass 2 recomputes the conv, normalises, applies GELU and writes once.
// Statistics are taken over the bf16-ROUNDED conv outputs, the values GroupNorm sees in the bf16 path.
//
// The conv runs on v_mfma_f32_16x16x32_bf16 at fp32-class accuracy: waveform and weights are split exactly
// into three bf16 planes (x = xh + xm + xl, 8 + 8 + 8 mantissa bits) and the six products down to 2^-24
// relative (xh.wh, xh.wm, xm.wh, xh.wl, xm.wm, xl.wh) are stacked along K: 6 terms x 10 taps = 60 of the 64
// K slots of two MFMAs per 16 channels x 16 time steps (the dropped xm.wl, xl.wm, xl.wl are below fp32's own
// rounding; the high-pass / DC-offset case of tests/test_wavlm_gpu.py is the one that needs all six).  The
// 10 VALU FMAs per output (plus their LDS sample reads) were half of both passes' VALU time; what is left is
// GroupNorm + GELU.  Operand roles: A = weights (row = channel), B = samples (column = time step), so a lane's
// accumulator holds 4 ADJACENT channels of one time step: one 8-byte store of the channel-last output.
// Block = 128 output steps of one clip x 512 channels, 4 waves x 128 channels.
// ---------------------------------------------------------------------------------------
namespace {
constexpr int C0_TS = 128, C0_KW = 10, C0_ST = 5;
constexpr int C0_PL = C0_TS * C0_ST + C0_KW;  // samples per tile (one plane)
constexpr int C0_ZERO = 3 * C0_PL;            // index of the zero slot after the three planes
// term t (K slots 10t .. 10t+9) of the split product: sample plane and weight plane (0 = hi, 1 = mid, 2 = lo)
__device__ __forceinline__ int c0_xplane(int t) { return (0x210100 >> (4 * t)) & 15; }  // h h m h m l
__device__ __forceinline__ int c0_wplane(int t) { return (0x012010 >> (4 * t)) & 15; }  // h m h l m h

__device__ __forceinline__ void split3(float x, bf16_t& h, bf16_t& m, bf16_t& l) {
  h = f2bf(x);
  const float r1 = x - bf2f(h);  // exact
  m = f2bf(r1);
  l = f2bf(r1 - bf2f(m));        // exact remainder, <= 8 significant bits
}

// the tile's samples t0*5 .. t0*5 + 649 as three bf16 planes (zero past the clip), plus the zero slot
__device__ __forceinline__ void conv0_tile_split(const float* __restrict__ x, int S, int t0, bf16_t* xs3) {
  for (int i = threadIdx.x; i < C0_PL; i += blockDim.x) {
    const long si = (long)t0 * C0_ST + i;
    bf16_t h, m, l;
    split3(si < S ? x[si] : 0.f, h, m, l);
    xs3[i] = h;
    xs3[C0_PL + i] = m;
    xs3[2 * C0_PL + i] = l;
  }
  if (threadIdx.x == 0) xs3[C0_ZERO] = 0;
}

// B-fragment gather table of this lane (col = time l & 15, K slots 32m + 8(l>>4) + i): LDS index of slot i
// at local time 0, and the per-time-step stride mask (samples advance 5 per step; the 4 empty slots 60..63
// read the zero slot at stride 0)
struct C0Gather {
  int off[16], msk[16];
  __device__ __forceinline__ void init(int lane) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int k = 32 * (s >> 3) + 8 * (lane >> 4) + (s & 7), t = k / 10, j = k - 10 * t;
      off[s] = t < 6 ? c0_xplane(t) * C0_PL + j : C0_ZERO;
      msk[s] = t < 6 ? -1 : 0;
    }
  }
  // the two B fragments (K 0..31, 32..63) of local time step tl
  __device__ __forceinline__ void load(const bf16_t* xs3, int tl, bf16x8& b0, bf16x8& b1) const {
    const int t5 = tl * C0_ST;
    uint32_t u[8];
#pragma unroll
    for (int p = 0; p < 8; ++p)
      u[p] = (uint32_t)xs3[off[2 * p] + (t5 & msk[2 * p])] | ((uint32_t)xs3[off[2 * p + 1] + (t5 & msk[2 * p + 1])] << 16);
    b0 = __builtin_bit_cast(bf16x8, u32x4{u[0], u[1], u[2], u[3]});
    b1 = __builtin_bit_cast(bf16x8, u32x4{u[4], u[5], u[6], u[7]});
  }
};

__device__ __forceinline__ f32x4 c0_mfma(const bf16x8* a, bf16x8 b0, bf16x8 b1) {
  f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b0, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b1, d, 0, 0, 0);
}
}  // namespace

// A fragments of the split weights, once per call: wfrag[(g16 * 2 + m) * 64 + lane] = 8 bf16 of channel
// 16 g16 + (lane & 15), K slots 32m + 8(lane>>4) .. +7.  Grid 32 (16-channel groups) x 128 threads.
__global__ __launch_bounds__(128) void wavlm_conv0_wfrag_kernel(const float* __restrict__ w,
                                                                bf16x8* __restrict__ wfrag) {
  const int m = threadIdx.x >> 6, lane = threadIdx.x & 63, c = blockIdx.x * 16 + (lane & 15);
  uint32_t u[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    bf16_t v[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int k = 32 * m + 8 * (lane >> 4) + 2 * p + e, t = k / 10, j = k - 10 * t;
      v[e] = 0;
      if (t < 6) {
        bf16_t pl[3];
        split3(w[c * C0_KW + j], pl[0], pl[1], pl[2]);
        v[e] = pl[c0_wplane(t)];
      }
    }
    u[p] = (uint32_t)v[0] | ((uint32_t)v[1] << 16);
  }
  wfrag[(blockIdx.x * 2 + m) * 64 + lane] = __builtin_bit_cast(bf16x8, u32x4{u[0], u[1], u[2], u[3]});
}

// pass 1: per-tile (sum, sumsq) of the bf16-rounded conv outputs per channel.  Wave w, channel group cb
// (16 channels) outer, the tile's 8 column blocks of 16 time steps inner; a lane sums its 4 channels over its
// 8 time steps, then the 16 lanes of a channel quad meet in a fixed xor tree (deterministic)
__global__ __launch_bounds__(256) void wavlm_conv0_stats_kernel(int S, int Lout, const float* __restrict__ wav,
                                                                const bf16x8* __restrict__ wfrag,
                                                                float* __restrict__ part) {
  __shared__ bf16_t xs3[C0_ZERO + 2];
  const int b = blockIdx.y, t0 = blockIdx.x * C0_TS, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  conv0_tile_split(wav + (long)b * S, S, t0, xs3);
  C0Gather gt;
  gt.init(lane);
  const int tn = min(C0_TS, Lout - t0);
  __syncthreads();
  bf16x8 bq[8][2];
#pragma unroll
  for (int tb = 0; tb < 8; ++tb) gt.load(xs3, 16 * tb + (lane & 15), bq[tb][0], bq[tb][1]);
  float* pr = part + ((long)b * gridDim.x + blockIdx.x) * 1024;
  const bf16x8* wf = wfrag + wv * 8 * 2 * 64 + lane;
  bf16x8 an[2] = {wf[0], wf[64]};  // the next channel group's A fragments, one group ahead
  for (int cb = 0; cb < 8; ++cb) {
    const bf16x8 af[2] = {an[0], an[1]};
    if (cb + 1 < 8) {
      an[0] = wf[(cb + 1) * 128];
      an[1] = wf[(cb + 1) * 128 + 64];
    }
    f32x4 s = {0.f, 0.f, 0.f, 0.f}, q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tb = 0; tb < 8; ++tb) {
      const f32x4 d = c0_mfma(af, bq[tb][0], bq[tb][1]);
      const float vm = 16 * tb + (lane & 15) < tn ? 1.f : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = bf2f(f2bf(d[r])) * vm;
        s[r] += v;
        q[r] += v * v;
      }
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s[r] += __shfl_xor(s[r], o, 64);
        q[r] += __shfl_xor(q[r], o, 64);
      }
    if ((lane & 15) == 0) {
      const int c = wv * 128 + cb * 16 + 4 * (lane >> 4);
      *reinterpret_cast<f32x4*>(pr + c * 2) = f32x4{s[0], q[0], s[1], q[1]};
      *reinterpret_cast<f32x4*>(pr + c * 2 + 4) = f32x4{s[2], q[2], s[3], q[3]};
    }
  }
}

// coef[b][c] = (scale, shift) of GroupNorm from the tile partials, summed in tile order (one serial chain per
// channel: the statistics feed a test whose score-path gradients are rounding-chaotic, so the order stays
// fixed); one wave per 64 channels, the loads unrolled so a chain's operands are in flight together
__global__ __launch_bounds__(64) void wavlm_gn_finalize_kernel(int ntiles, int Lout, const float* __restrict__ part,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, float eps,
                                                               float* __restrict__ coef) {
  const int b = blockIdx.y, c = blockIdx.x * 64 + threadIdx.x;
  const float2* p = reinterpret_cast<const float2*>(part + (long)b * ntiles * 1024) + c;
  float s = 0.f, q = 0.f;
#pragma unroll 16
  for (int t = 0; t < ntiles; ++t) {
    const float2 v = p[(long)t * 512];
    s += v.x;
    q += v.y;
  }
  const float mu = s / Lout;
  const float var = fmaxf(q / Lout - mu * mu, 0.f);
  const float sc = rsqrtf(var + eps) * gamma[c];
  coef[((long)b * 512 + c) * 2] = sc;
  coef[((long)b * 512 + c) * 2 + 1] = beta[c] - mu * sc;
}

// pass 2: conv recompute, GroupNorm affine, GELU, one bf16 write.  Column block (16 time steps) outer so each
// wave finishes its 256-byte row segments of 16 output rows back to back; the (scale, shift) table of the
// clip's 512 channels sits in LDS
__global__ __launch_bounds__(256) void wavlm_conv0_gn_gelu_kernel(int S, int Lout, const float* __restrict__ wav,
                                                                  const bf16x8* __restrict__ wfrag,
                                                                  const float* __restrict__ coef,
                                                                  bf16_t* __restrict__ out) {
  __shared__ bf16_t xs3[C0_ZERO + 2];
  __shared__ f32x4 cf[256];  // (scale, shift) of channels 2i, 2i+1
  const int b = blockIdx.y, t0 = blockIdx.x * C0_TS, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  conv0_tile_split(wav + (long)b * S, S, t0, xs3);
  cf[threadIdx.x] = reinterpret_cast<const f32x4*>(coef + (long)b * 1024)[threadIdx.x];
  C0Gather gt;
  gt.init(lane);
  bf16x8 af[8][2];
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) {
    af[cb][0] = wfrag[((wv * 8 + cb) * 2) * 64 + lane];
    af[cb][1] = wfrag[((wv * 8 + cb) * 2 + 1) * 64 + lane];
  }
  const int tn = min(C0_TS, Lout - t0);
  __syncthreads();
  for (int tb = 0; tb < 8; ++tb) {
    const int tl = 16 * tb + (lane & 15);
    bf16x8 b0, b1;
    gt.load(xs3, tl, b0, b1);
    bf16_t* orow = out + ((long)b * Lout + t0 + tl) * 512 + wv * 128 + 4 * (lane >> 4);
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) {
      const f32x4 d = c0_mfma(af[cb], b0, b1);
      const int c2 = (wv * 128 + cb * 16 + 4 * (lane >> 4)) >> 1;  // channel pair index
      const f32x4 p0 = cf[c2], p1 = cf[c2 + 1];                    // sc0 sh0 sc1 sh1 | sc2 sh2 sc3 sh3
      const float y0 = gelu_erf(bf2f(f2bf(d[0])) * p0[0] + p0[1]), y1 = gelu_erf(bf2f(f2bf(d[1])) * p0[2] + p0[3]);
      const float y2 = gelu_erf(bf2f(f2bf(d[2])) * p1[0] + p1[1]), y3 = gelu_erf(bf2f(f2bf(d[3])) * p1[2] + p1[3]);
      if (tl < tn)
        *reinterpret_cast<uint2*>(orow + cb * 16) = uint2{(uint32_t)f2bf(y0) | ((uint32_t)f2bf(y1) << 16),
                                                          (uint32_t)f2bf(y2) | ((uint32_t)f2bf(y3) << 16)};
    }
  }
}

MER_API int mer_wavlm_conv0_gn_gelu(int B, int S, int Lout, const float* wav, const float* w0, const float* gamma,
                                    const float* beta, float eps, float* workspace, void* out, void* stream) {
  if (B <= 0 || Lout != (S - C0_KW) / C0_ST + 1) return (int)hipErrorInvalidValue;
  const int ntiles = (Lout + C0_TS - 1) / C0_TS;
  float* part = workspace;                             // [B][ntiles][512][2]
  float* coef = workspace + (long)B * ntiles * 1024;   // [B][512][2]
  bf16x8* wfrag = reinterpret_cast<bf16x8*>(coef + (long)B * 1024);  // [32][2][64] split weight fragments
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(wavlm_conv0_wfrag_kernel, dim3(32), dim3(128), 0, st, w0, wfrag);
  hipLaunchKernelGGL(wavlm_conv0_stats_kernel, dim3(ntiles, B), dim3(256), 0, st, S, Lout, wav, wfrag, part);
  hipLaunchKernelGGL(wavlm_gn_finalize_kernel, dim3(8, B), dim3(64), 0, st, ntiles, Lout, part, gamma, beta, eps, coef);
  hipLaunchKernelGGL(wavlm_conv0_gn_gelu_kernel, dim3(ntiles, B), dim3(256), 0, st, S, Lout, wav, wfrag, coef,
                     (bf16_t*)out);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// Row LayerNorm (feature projection TF:93-105, encoder LN TF:418, post-LN layers TF:314-336).
// x fp32 or bf16 [rows, d] (ldx), y bf16 or fp32 [rows, d] (ldy).  One wave per row.
// ---------------------------------------------------------------------------------------
template <typename T> __device__ __forceinline__ f32x4 ld4(const T* p);
template <> __device__ __forceinline__ f32x4 ld4<float>(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
template <> __device__ __forceinline__ f32x4 ld4<bf16_t>(const bf16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
               __uint_as_float(u.y & 0xffff0000u)};
}
template <typename T> __device__ __forceinline__ void st4(T* p, f32x4 v);
template <> __device__ __forceinline__ void st4<float>(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
template <> __device__ __forceinline__ void st4<bf16_t>(bf16_t* p, f32x4 v) {
  *reinterpret_cast<uint2*>(p) = uint2{(uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                       (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16)};
}

// VEC: d % 256 == 0 and 4-element aligned rows -- each lane moves 4 consecutive elements per access.
// Train mode (mer_layernorm_tr): dropout on the OUTPUT (WavLMEncoder.dropout after the encoder LayerNorm,
// TF:406-407; mask index row * d + c) and the LayerDrop skip of the layer the LN belongs to (TF:417-419).
template <typename TI, typename TO, bool VEC>
__global__ __launch_bounds__(256) void layernorm_kernel(int rows, int d, const TI* __restrict__ x, long ldx,
                                                        const float* __restrict__ gamma, const float* __restrict__ beta,
                                                        float eps, TO* __restrict__ y, long ldy, float drop_p,
                                                        const unsigned long long* __restrict__ seed_ptr,
                                                        unsigned long long site, const long long* __restrict__ skip,
                                                        int skip_bit) {
  if (skip && ((*skip >> skip_bit) & 1ll)) return;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  const TI* xr = x + (long)row * ldx;
  TO* yr = y + (long)row * ldy;
  float vals[16];  // d <= 1024
  float s = 0.f;
  if (VEC) {
    const int nv = d >> 8;
    f32x4 gv[4], bv[4];  // issued with the row loads: their latency overlaps the row's, not the reductions'
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i >= nv) break;
      gv[i] = *reinterpret_cast<const f32x4*>(gamma + (i * 64 + lane) * 4);
      bv[i] = *reinterpret_cast<const f32x4*>(beta + (i * 64 + lane) * 4);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i >= nv) break;
      const f32x4 v = ld4<TI>(xr + (i * 64 + lane) * 4);
      vals[4 * i] = v[0]; vals[4 * i + 1] = v[1]; vals[4 * i + 2] = v[2]; vals[4 * i + 3] = v[3];
      s += (v[0] + v[1]) + (v[2] + v[3]);
    }
    const float mean = wave_sum(s) / d;
    float q = 0.f;
    for (int i = 0; i < 4 * nv; ++i) { const float v = vals[i] - mean; q += v * v; }
    const float rstd = rsqrtf(wave_sum(q) / d + eps);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i >= nv) break;
      const int c = (i * 64 + lane) * 4;
      const f32x4 g = gv[i], b = bv[i];
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (vals[4 * i + e] - mean) * rstd * g[e] + b[e];
      if (drop_p > 0.f) {  // d % 256 == 0: the 4 indices start even
        float ov[4] = {o[0], o[1], o[2], o[3]};
        dropout_pairs<4>(ov, seed, (uint64_t)((long)row * d + c), drop_p);
        o = f32x4{ov[0], ov[1], ov[2], ov[3]};
      }
      st4<TO>(yr + c, o);
    }
    return;
  }
  int n = 0;
  for (int c = lane; c < d; c += 64, ++n) {
    vals[n] = ldf<TI>(xr, c);
    s += vals[n];
  }
  const float mean = wave_sum(s) / d;
  float q = 0.f;
  for (int i = 0; i < n; ++i) { const float v = vals[i] - mean; q += v * v; }
  const float rstd = rsqrtf(wave_sum(q) / d + eps);
  n = 0;
  for (int c = lane; c < d; c += 64, ++n) {
    float o = (vals[n] - mean) * rstd * gamma[c] + beta[c];
    if (drop_p > 0.f) o *= dropout_scale_pair(seed, (uint64_t)((long)row * d + c), drop_p);
    stf<TO>(yr, c, o);
  }
}

MER_API int mer_layernorm(int rows, int d, const void* x, int x_dtype, long ldx, const float* gamma,
                          const float* beta, float eps, void* y, int y_dtype, long ldy, void* stream) {
  return mer_layernorm_tr(rows, d, x, x_dtype, ldx, gamma, beta, eps, y, y_dtype, ldy, 0.f, nullptr, 0ull, nullptr, 0,
                          stream);
}

MER_API int mer_layernorm_tr(int rows, int d, const void* x, int x_dtype, long ldx, const float* gamma,
                             const float* beta, float eps, void* y, int y_dtype, long ldy, float drop_p,
                             const unsigned long long* seed, unsigned long long site, const long long* skip_mask,
                             int skip_bit, void* stream) {
  if (d > 1024 || rows <= 0) return rows <= 0 ? 0 : (int)hipErrorInvalidValue;
  if (drop_p < 0.f || drop_p >= 1.f || (drop_p > 0.f && !seed) || skip_bit < 0 || skip_bit > 62)
    return (int)hipErrorInvalidValue;
  dim3 grid((rows + 3) / 4);
  hipStream_t st = (hipStream_t)stream;
  const bool vec = d % 256 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && ((((uintptr_t)x) | ((uintptr_t)y)) & 7) == 0 &&
                   (((uintptr_t)x) & (x_dtype == MER_F32 ? 15 : 7)) == 0 &&
                   (((uintptr_t)y) & (y_dtype == MER_F32 ? 15 : 7)) == 0 &&
                   ((((uintptr_t)gamma) | ((uintptr_t)beta)) & 15) == 0;
#define L(TI, TO)                                                                                              \
  do {                                                                                                         \
    if (vec)                                                                                                   \
      hipLaunchKernelGGL((layernorm_kernel<TI, TO, true>), grid, dim3(256), 0, st, rows, d, (const TI*)x, ldx, \
                         gamma, beta, eps, (TO*)y, ldy, drop_p, seed, site, skip_mask, skip_bit);             \
    else                                                                                                       \
      hipLaunchKernelGGL((layernorm_kernel<TI, TO, false>), grid, dim3(256), 0, st, rows, d, (const TI*)x, ldx, \
                         gamma, beta, eps, (TO*)y, ldy, drop_p, seed, site, skip_mask, skip_bit);             \
  } while (0)
  if (x_dtype == MER_F32 && y_dtype == MER_BF16) L(float, bf16_t);
  else if (x_dtype == MER_BF16 && y_dtype == MER_BF16) L(bf16_t, bf16_t);
  else if (x_dtype == MER_F32 && y_dtype == MER_F32) L(float, float);
  else L(bf16_t, float);
#undef L
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// Self-attention with WavLM's gated relative position bias (TF:147-241):
//   gate_i = sigmoid(a_i) * (sigmoid(b_i) * const_h - 1) + 2,  (a_i, b_i) = pair-sums of
//            gru_rel_pos_linear(x_i[h*dh:(h+1)*dh])                          (TF:163-177)
//   S_ij   = scale * q_i.k_j + gate_i * emb[bucket(j - i), h]                 (TF:243-271)
//   O_i    = softmax_j(S_i) V
// Q/K/V come from one fused projection [B*L, 3*768] (q | k | v).  L <= 256, dh = 64.
// Grid (B*H, ceil(L/(16 NW))): a workgroup stages K (row-major) and V^T of its (b, h) in LDS, and each
// of its NW waves (default 5) owns 16 query rows.  The scores are computed TRANSPOSED, S^T = K Q^T
// (v_mfma_f32_16x16x32_bf16, key j on the accumulator rows, query i = lane & 15), so every lane holds
// whole key columns of one query: the softmax reduces in-lane plus two xor-shuffles, the gate is one
// register per lane, and the accumulator tiles ARE the B operand of O^T = V^T P^T on
// v_mfma_f32_16x16x16_bf16 (k = 4*(lane>>4) + e) -- P never goes through LDS.
// ---------------------------------------------------------------------------------------
// Phase timestamps for tuning (tools/attn_phases.py builds a separate library with -DMER_ATTN_TIMING; the production
// library compiles AT() to nothing): wall_clock64() of each block's thread 0 at phase k.
#ifdef MER_ATTN_TIMING
static __device__ long long mer_at_buf[2048 * 8];
#define AT(k) \
  do { \
    if (threadIdx.x == 0 && blockIdx.x < 2048) mer_at_buf[blockIdx.x * 8 + (k)] = wall_clock64(); \
  } while (0)
MER_API int mer_at_read(long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(mer_at_buf), sizeof(long long) * 2048 * 8, 0, hipMemcpyDeviceToHost);
}
#else
#define AT(k) \
  do { \
  } while (0)
#endif

namespace {
constexpr int ADH = 64, APAD = ADH + 8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
}

// KT: key tiles held in registers (compile time, >= ceil(L / 16)): 10 for L <= 160 (the 3 s clips: L = 149), 16 up to
// L = 256.  NW waves per block, one 16-row query tile each.  (Waves owning 2 tiles so that one 8-wave block stages
// K / V once per (b, h) need > 128 VGPRs -- 3 waves per SIMD, one such block per CU -- or spill: measured no gain.)
template <int NW, int KT>
__global__ __launch_bounds__(64 * NW) void wavlm_attn_kernel(
    int L, int H, const bf16_t* __restrict__ qkv, long ldqkv,
                                                         const bf16_t* __restrict__ x, long ldx,
                                                         const float* __restrict__ gw, const float* __restrict__ gb,
                                                         const float* __restrict__ gconst,
                                                         const float* __restrict__ rel_emb,
                                                         const int* __restrict__ bucket, bf16_t* __restrict__ out,
                                                         long ldo, float scale, float drop_p,
                                                         const unsigned long long* __restrict__ seed_ptr,
                                                         unsigned long long site, const long long* __restrict__ skip,
                                                         int skip_bit) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  AT(0);
#ifdef MER_ATTN_TIMING
  if (threadIdx.x == 0 && blockIdx.x < 2048)  // HW_ID (wave / SIMD / CU / SE) and XCC_ID of wave 0
    mer_at_buf[blockIdx.x * 8 + 7] = ((long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                                     (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
#endif
  if (skip && ((*skip >> skip_bit) & 1ll)) return;
  constexpr int KP = 16 * KT;  // keys held (zero rows / columns past L)
  constexpr int VTP = KP + 8;
  const int NTL = (L + 15) / 16;  // query tiles
  bf16_t* Ks = reinterpret_cast<bf16_t*>(smem_raw);   // [KP][APAD]
  bf16_t* Vt = Ks + KP * APAD;                        // [ADH][VTP]
  // this head's relative-position bias row, tbl[16 + r] = bias(r - (L - 1)) for r in [0, 2L-1), zero padding of 16
  // entries before and KP - L after: every (i < 16 NTL, j < KP) reads tbl[16 + j - i + L - 1] without clamping
  // (padding values only reach masked scores)
  float* tbl = reinterpret_cast<float*>(Vt + ADH * VTP);
  constexpr int NTH = 64 * NW;
  constexpr int KIT = (KP * 8 + NTH - 1) / NTH, VIT = (KP * 2 + NTH - 1) / NTH;
  constexpr int TIT = (16 + 2 * 256 + KP + NTH - 1) / NTH;  // table entries (L <= 256) per thread
  // one-dimensional grid, XCD-aware: the row blocks of one (b, h) run on one XCD and share its K / V in L2
  const int nrb = (NTL + NW - 1) / NW;
  int rbk, bh;
  xcd_tile(blockIdx.x, nrb, gridDim.x, rbk, bh);  // gridDim.x = nrb * B * H
  const int b = bh / H, h = bh % H;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int D = H * ADH;
  const int rb = rbk * NW + w;  // this wave's 16-row query tile

  // Loads are unconditional from clamped (valid) rows, zeroed by a select at the LDS store: a load under a
  // per-lane condition compiles to a branch around it and a wait for it, serialising the prologue's loads.
  // Prologue: the 8 gru_rel_pos_linear weight rows as MFMA A fragments (row n = lane&15 < 8, zero above; split
  // into bf16 hi + lo at use), the relative-position bias row of this head (precomputed table [H][2L-1] when
  // bucket == nullptr, else gathered through the bucket index), K (row-major 16-byte chunks) and V (4-row groups
  // for the V^T image); rows >= L are zero.
  const int gn = lane & 15;
  f32x4 gwr[2][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const float* wp = gw + (gn < 8 ? gn : 7) * ADH + kk * 32 + (lane >> 4) * 8;
    gwr[kk][0] = *reinterpret_cast<const f32x4*>(wp);
    gwr[kk][1] = *reinterpret_cast<const f32x4*>(wp + 4);
  }
  const int ntbl = 16 + 2 * L - 1 + (KP - L);
  float tb[TIT];
#pragma unroll
  for (int k = 0; k < TIT; ++k) {
    const int r = min(max(t + NTH * k - 16, 0), 2 * L - 2);
    tb[k] = bucket ? rel_emb[(long)bucket[r] * H + h] : rel_emb[(long)h * (2 * L - 1) + r];
  }
  {
    u32x4 kr[KIT];
#pragma unroll
    for (int it = 0; it < KIT; ++it) {
      const int c = t + it * NTH, row = min(c >> 3, L - 1), ch = c & 7;
      kr[it] = *reinterpret_cast<const u32x4*>(qkv + ((long)b * L + row) * ldqkv + D + h * ADH + ch * 8);
    }
    u32x4 vr[VIT][4];
#pragma unroll
    for (int it = 0; it < VIT; ++it) {
      const int q = t + it * NTH, rq = q >> 3, ch = q & 7;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = min(rq * 4 + e, L - 1);
        vr[it][e] = *reinterpret_cast<const u32x4*>(qkv + ((long)b * L + row) * ldqkv + 2 * D + h * ADH + ch * 8);
      }
    }
    AT(1);
#pragma unroll
    for (int k = 0; k < TIT; ++k) {
      const int r = t + NTH * k;
      if (r < ntbl) tbl[r] = (r >= 16 && r < 16 + 2 * L - 1) ? tb[k] : 0.f;
    }
#pragma unroll
    for (int it = 0; it < KIT; ++it) {
      const int c = t + it * NTH, row = c >> 3, ch = c & 7;
      if (c < KP * 8) *reinterpret_cast<u32x4*>(&Ks[row * APAD + ch * 8]) = row < L ? kr[it] : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int it = 0; it < VIT; ++it) {
      const int q = t + it * NTH, rq = q >> 3, ch = q & 7;
      if (q < KP * 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (rq * 4 + e >= L) vr[it][e] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < 8; ++i) {  // channel d = ch*8 + i: (V[4rq][d], .., V[4rq+3][d])
          const int sh = (i & 1) * 16, wd = i >> 1;
          const uint32_t v0 = (vr[it][0][wd] >> sh) & 0xffffu, v1 = (vr[it][1][wd] >> sh) & 0xffffu;
          const uint32_t v2 = (vr[it][2][wd] >> sh) & 0xffffu, v3 = (vr[it][3][wd] >> sh) & 0xffffu;
          *reinterpret_cast<uint2*>(&Vt[(ch * 8 + i) * VTP + rq * 4]) = uint2{v0 | (v1 << 16), v2 | (v3 << 16)};
        }
      }
    }
  }
  // the gate weights as split bf16 A fragments (kept for every tile of this wave)
  bf16x8 whi[2], wlo[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x8 wv = __builtin_shufflevector(gn < 8 ? gwr[kk][0] : z, gn < 8 ? gwr[kk][1] : z, 0, 1, 2, 3, 4, 5, 6, 7);
    whi[kk] = __builtin_convertvector(wv, bf16x8);
    wlo[kk] = __builtin_convertvector(wv - __builtin_convertvector(whi[kk], f32x8), bf16x8);
  }
  const float gc = gconst[h];
  const unsigned long long dseed = mer_site_seed(seed_ptr, site);
  // the paired dropout mask (common.h dropout_scale_pair) over index ((b*H+h)*L + i)*LE + j, LE = L rounded up to
  // even: the seed mix of mer_hash, the 16-bit keep threshold, and whether every index fits 32 bits
  const int LE = L + (L & 1);
  const uint32_t hseed = (uint32_t)dseed ^ ((uint32_t)(dseed >> 32) * 0x85EBCA6Bu);
  const uint32_t keep_thr = drop_thr16(drop_p);
  const bool idx32 = (unsigned long long)(gridDim.x / nrb) * (unsigned long long)(L + 1) * (unsigned long long)LE <
                     (1ull << 32);
  __syncthreads();
  AT(2);

  if (rb < NTL) {  // wave-uniform
    // this tile's Q (B operand of S^T = K Q^T) and x rows (B operand of the gate product): Q[i = lane&15][d =
    // kk*32 + 8*(lane>>4) ..]; rows past L read row L - 1 (their outputs are never stored)
    const int qrow = min(rb * 16 + (lane & 15), L - 1);
    bf16x8 qb[2], xb[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      qb[kk] = *reinterpret_cast<const bf16x8*>(qkv + ((long)b * L + qrow) * ldqkv + h * ADH + kk * 32 + (lane >> 4) * 8);
      xb[kk] = *reinterpret_cast<const bf16x8*>(x + ((long)b * L + qrow) * ldx + h * ADH + kk * 32 + (lane >> 4) * 8);
    }
    // gate of the tile's 16 rows: the 8 gru_rel_pos_linear outputs G^T[n][i] = sum_k W[n][k] x[i][k] on MFMA (the
    // fp32 weight split into bf16 hi + lo; x is exact bf16).  Lane (i = lane&15, group q = lane>>4) holds outputs
    // n = 4q .. 4q+3 of row i: group 0 sums a_i (TF:163-177 .view(.., 2, 4).sum(-1)), group 1 b_i.
    const int i = rb * 16 + (lane & 15);
    float gi;
    {
      f32x4 g = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        g = __builtin_amdgcn_mfma_f32_16x16x32_bf16(whi[kk], xb[kk], g, 0, 0, 0);
        g = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wlo[kk], xb[kk], g, 0, 0, 0);
      }
      // sum_{r} (z + b) in the order of the stage-2 backward's recompute (wavlm_train.hip), so a trainable layer's
      // backward differentiates exactly the gate its forward applied
      float zs = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) zs += g[r] + gb[(4 * (lane >> 4) + r) & 7];
      const float ga = 1.f / (1.f + __expf(-__shfl(zs, lane & 15, 64)));
      const float gbv = 1.f / (1.f + __expf(-__shfl(zs, 16 + (lane & 15), 64)));
      gi = i < L ? ga * (gbv * gc - 1.f) + 2.f : 1.f;
    }
    AT(3);
    // S^T tiles: s[ct][r] = S[i][j = ct*16 + 4*(lane>>4) + r]; key tiles past L are zero rows of Ks (LDS sized for
    // KT tiles), masked to -inf below
    f32x4 s[KT];
#pragma unroll
    for (int ct = 0; ct < KT; ++ct) s[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int ct = 0; ct < KT; ++ct) {
        const bf16x8 ka = *reinterpret_cast<const bf16x8*>(&Ks[(ct * 16 + (lane & 15)) * APAD + kk * 32 + (lane >> 4) * 8]);
        s[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qb[kk], s[ct], 0, 0, 0);
      }
    float mx = -INFINITY;
    const float* trow = tbl + 16 + (lane >> 4) * 4 - i + L - 1;  // + j - 4*(lane>>4) = ct*16 + r
#pragma unroll
    for (int ct = 0; ct < KT; ++ct) {
#pragma unroll
      for (int r = 0; r < 4; ++r) s[ct][r] = s[ct][r] * scale + gi * trow[ct * 16 + r];
      if (ct * 16 + 15 >= L) {  // (wave-uniform) the tile holds keys past L
#pragma unroll
        for (int r = 0; r < 4; ++r) s[ct][r] = ct * 16 + (lane >> 4) * 4 + r < L ? s[ct][r] : -INFINITY;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[ct][r]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    AT(4);
    // P^T = exp(S^T - max) rounded to bf16 (the weights that enter PV also form the normaliser).  Train mode:
    // attention-probability dropout (F.multi_head_attention_forward dropout_p, TF:206-228): dropped weights do
    // not enter PV, the kept ones are rescaled by 1/(1-p) with the normaliser
    const long mrow = (((long)b * H + h) * L + i) * LE;  // even: the lane's keys pair up as (r0, r1), (r2, r3)
    float sum = 0.f;
    // P^T as packed bf16 pairs: word pw[ct][rp] = keys (2 rp, 2 rp + 1) of the tile (low half first), the layout of
    // the PV A operand -- the dropout mask then clears whole 16-bit halves with one AND per pair (per-element
    // inserts into a short vector compiled to ~25 permutes + an exec-mask branch each)
    uint32_t pw[KT][2];
#pragma unroll
    for (int ct = 0; ct < KT; ++ct)
#pragma unroll
      for (int rp = 0; rp < 2; ++rp) {
        const bf16_t p0 = f2bf(__expf(s[ct][2 * rp] - mx)), p1 = f2bf(__expf(s[ct][2 * rp + 1] - mx));
        sum += bf2f(p0);
        sum += bf2f(p1);
        pw[ct][rp] = (uint32_t)p0 | ((uint32_t)p1 << 16);
      }
    if (drop_p > 0.f) {  // (uniform) the keep mask, dropout_scale_pair(dseed, mrow + j, p) != 0
      if (idx32) {
        // every mask index is < 2^32: mer_hash's first product distributes over the pair index (mrow + j) / 2 =
        // mrow / 2 + 8 ct + 2 (lane >> 4) + r / 2, so each pair costs one add + the two-multiply finaliser
        const uint32_t qb0 = (uint32_t)(mrow >> 1) * 0x9E3779B9u + hseed + (uint32_t)(2 * (lane >> 4)) * 0x9E3779B9u;
#pragma unroll
        for (int ct = 0; ct < KT; ++ct)
#pragma unroll
          for (int rp = 0; rp < 2; ++rp) {
            uint32_t xh = qb0 + (uint32_t)(ct * 8 + rp) * 0x9E3779B9u;
            xh ^= xh >> 16;
            xh *= 0x7FEB352Du;
            xh ^= xh >> 15;
            xh *= 0x846CA68Bu;
            xh ^= xh >> 16;
            const uint32_t keep = ((xh & 0xFFFFu) < keep_thr ? 0u : 0x0000FFFFu) | ((xh >> 16) < keep_thr ? 0u : 0xFFFF0000u);
            pw[ct][rp] &= keep;
          }
      } else {
#pragma unroll
        for (int ct = 0; ct < KT; ++ct)
#pragma unroll
          for (int rp = 0; rp < 2; ++rp) {
            const int j = ct * 16 + (lane >> 4) * 4 + 2 * rp;
            const bool k0 = dropout_scale_pair(dseed, (uint64_t)(mrow + j), drop_p) != 0.f;
            const bool k1 = dropout_scale_pair(dseed, (uint64_t)(mrow + j + 1), drop_p) != 0.f;
            pw[ct][rp] &= (k0 ? 0x0000FFFFu : 0u) | (k1 ? 0xFFFF0000u : 0u);
          }
      }
    }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    AT(5);
    // O^T[d][i] = sum_j V^T[d][j] P^T[j][i]: A = V^T (d = lane&15, j = ct*16 + 4*(lane>>4) + e)
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ct = 0; ct < KT; ++ct)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const s16x4 va = *reinterpret_cast<const s16x4*>(&Vt[(dt * 16 + (lane & 15)) * VTP + ct * 16 + (lane >> 4) * 4]);
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(va, __builtin_bit_cast(s16x4, u32x2{pw[ct][0], pw[ct][1]}),
                                                          o[dt], 0, 0, 0);
      }
    if (i < L) {
      const float inv = (drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f) / sum;
      bf16_t* orow = out + ((long)b * L + i) * ldo + h * ADH + (lane >> 4) * 4;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const uint32_t lo = (uint32_t)f2bf(o[dt][0] * inv) | ((uint32_t)f2bf(o[dt][1] * inv) << 16);
        const uint32_t hi = (uint32_t)f2bf(o[dt][2] * inv) | ((uint32_t)f2bf(o[dt][3] * inv) << 16);
        *reinterpret_cast<uint2*>(orow + dt * 16) = uint2{lo, hi};
      }
    }
  }
  AT(6);
}

MER_API int mer_wavlm_attention(int B, int L, int H, const void* qkv, long ldqkv, const void* x, long ldx,
                                const float* gate_w, const float* gate_b, const float* gate_const,
                                const float* rel_emb, const int* bucket, void* out, long ldo, float scale,
                                void* stream) {
  return mer_wavlm_attention_tr(B, L, H, qkv, ldqkv, x, ldx, gate_w, gate_b, gate_const, rel_emb, bucket, out, ldo,
                                scale, 0.f, nullptr, 0ull, nullptr, 0, stream);
}

MER_API int mer_wavlm_attention_tr(int B, int L, int H, const void* qkv, long ldqkv, const void* x, long ldx,
                                   const float* gate_w, const float* gate_b, const float* gate_const,
                                   const float* rel_emb, const int* bucket, void* out, long ldo, float scale,
                                   float drop_p, const unsigned long long* seed, unsigned long long site,
                                   const long long* skip_mask, int skip_bit, void* stream) {
  if (L > 256 || L <= 0) return (int)hipErrorInvalidValue;
  if (drop_p < 0.f || drop_p >= 1.f || (drop_p > 0.f && !seed) || skip_bit < 0 || skip_bit > 62)
    return (int)hipErrorInvalidValue;
  if ((ldqkv % 8) || (ldx % 8) || (ldo % 4) || ((((uintptr_t)qkv) | ((uintptr_t)x)) & 15) || (((uintptr_t)out) & 7))
    return (int)hipErrorInvalidValue;
  const int LP = (L + 15) / 16 * 16;
  // 5 waves (80 query rows) per block: 2 blocks per (b, h) at L = 149.  The workgroup's waves land on SIMDs
  // 0,1,2,3,0, so SIMD 0 holds 2 of every block: at <= 4 waves per SIMD 2 blocks run per CU (the 768 blocks of
  // B = 32 in 2 rounds).  4 waves (1.5 rounds) lost 1.5 %, one 10-wave block per (b, h) (K/V staged once) 0.5 %
  // of the step.
#define MER_ATTN_LAUNCH(NW, KT)                                                                                   \
  do {                                                                                                           \
    const size_t lds = sizeof(bf16_t) * ((size_t)16 * KT * APAD + (size_t)ADH * (16 * KT + 8)) +                 \
                       sizeof(float) * (16 + 2 * L + 16 * KT);                                                    \
    hipLaunchKernelGGL((wavlm_attn_kernel<NW, KT>), dim3(B * H * ((LP / 16 + NW - 1) / NW)), dim3(64 * NW), lds,   \
                       (hipStream_t)stream, L, H, (const bf16_t*)qkv, ldqkv, (const bf16_t*)x, ldx, gate_w, gate_b, \
                       gate_const, rel_emb, bucket, (bf16_t*)out, ldo, scale, drop_p, seed, site, skip_mask,      \
                       skip_bit);                                                                                 \
  } while (0)
  if (LP <= 160)  // 10 key tiles in registers: the 3 s clip (L = 149)
    MER_ATTN_LAUNCH(5, 10);
  else
    MER_ATTN_LAUNCH(5, 16);
#undef MER_ATTN_LAUNCH
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// Weight preparation (frozen weights: run once per weight version, never in the hot loop).
// dst[i0][i1][i2] = bf16(src[i0*s0 + i1*s1 + i2*s2] * (scale ? scale[i1] : 1))
// e.g. Conv1d [Cout][Cin][k] -> [Cout][k][Cin] (K-contiguous im2col order).
// ---------------------------------------------------------------------------------------
__global__ void permute3_bf16_kernel(int n0, int n1, int n2, const float* __restrict__ src, long s0, long s1, long s2,
                                     const float* __restrict__ scale, bf16_t* __restrict__ dst) {
  const long n = (long)n0 * n1 * n2;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int i2 = e % n2;
    const int i1 = (e / n2) % n1;
    const int i0 = e / ((long)n1 * n2);
    float v = src[(long)i0 * s0 + (long)i1 * s1 + (long)i2 * s2];
    if (scale) v *= scale[i1];
    dst[e] = f2bf(v);
  }
}
MER_API int mer_permute3_bf16(int n0, int n1, int n2, const float* src, long s0, long s1, long s2, const float* scale,
                              void* dst, void* stream) {
  const long n = (long)n0 * n1 * n2;
  const int grid = (int)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
  hipLaunchKernelGGL(permute3_bf16_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, (hipStream_t)stream, n0, n1, n2,
                     src, s0, s1, s2, scale, (bf16_t*)dst);
  MER_LAUNCH_CHECK();
}

// weight_norm(dim=2) scale of the positional conv (TF:58-78): scale[k] = g[k] / ||v[:, :, k]||_2
__global__ __launch_bounds__(256) void weightnorm_scale_kernel(int n01, int taps, const float* __restrict__ v,
                                                               const float* __restrict__ g, float* __restrict__ scale) {
  __shared__ float red[4];
  const int k = blockIdx.x;
  float s = 0.f;
  for (int i = threadIdx.x; i < n01; i += 256) {
    const float x = v[(long)i * taps + k];
    s += x * x;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) scale[k] = g[k] / sqrtf(red[0] + red[1] + red[2] + red[3]);
}
MER_API int mer_weightnorm_scale(int n01, int taps, const float* v, const float* g, float* scale, void* stream) {
  hipLaunchKernelGGL(weightnorm_scale_kernel, dim3(taps), dim3(256), 0, (hipStream_t)stream, n01, taps, v, g, scale);
  MER_LAUNCH_CHECK();
}

// fp32 -> bf16 cast (contiguous), 4 elements per thread-iteration.
__global__ void cast_bf16_kernel(long n, const float* __restrict__ x, bf16_t* __restrict__ y) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) y[e] = f2bf(x[e]);
}
MER_API int mer_cast_bf16(long n, const float* x, void* y, void* stream) {
  const int grid = (int)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, (hipStream_t)stream, n, x, (bf16_t*)y);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// SpecAugment time masking of WavLM in train mode (WavLMModel._mask_hidden_states TF:985-1015 with
// _compute_mask_indices TF:834-950, config mask_time_prob 0.05 / mask_time_length 10 / min_masks 2): the
// projected features h [B*L, D] get `n` spans of `span` frames replaced by masked_spec_embed, n =
// max(int(prob * L / span + eps), min_masks) capped as TF does, eps ~ U[0,1) shared by the batch, span starts
// distinct and uniform over [0, L - span] per sample (Floyd's sampling without replacement -- the distribution
// of TF's np.random.choice(..., replace=False); the random stream is the device hash, not numpy's).
// One workgroup per sample; mask_out (optional, uint8 [B, L]) records the masked frames.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void wavlm_time_mask_kernel(int L, int D, bf16_t* __restrict__ h, long ldh,
                                                              const float* __restrict__ embed, float prob, int span,
                                                              int min_masks, const unsigned long long* __restrict__ seed_ptr,
                                                              unsigned long long site, unsigned char* __restrict__ mask_out) {
  __shared__ int starts[64];
  __shared__ int nsp;
  const int b = blockIdx.x;
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  if (threadIdx.x == 0) {
    const float eps = (mer_hash(seed, 0) >> 8) * (1.0f / 16777216.0f);
    int n = (int)(prob * (float)L / (float)span + eps);
    n = n > min_masks ? n : min_masks;
    if (n * span > L) n = L / span;
    if (L - (span - 1) < n) n = L - (span - 1) > 0 ? L - (span - 1) : 0;
    n = n < 64 ? n : 64;
    const int N = L - span + 1;
    int cnt = 0;
    for (int jj = N - n; jj < N; ++jj) {  // Floyd: uniform n-subset of [0, N)
      const uint32_t r = mer_hash(seed, 1 + (uint64_t)b * 64 + cnt);
      const int t = (int)(((uint64_t)r * (uint64_t)(jj + 1)) >> 32);
      bool present = false;
      for (int k = 0; k < cnt; ++k) present |= starts[k] == t;
      starts[cnt++] = present ? jj : t;
    }
    nsp = cnt;
  }
  __syncthreads();
  const int n = nsp;
  if (mask_out) {
    for (int r = threadIdx.x; r < L; r += blockDim.x) {
      bool m = false;
      for (int k = 0; k < n; ++k) m |= r >= starts[k] && r < starts[k] + span;
      mask_out[(long)b * L + r] = m ? 1 : 0;
    }
  }
  const long tot = (long)n * span * D;
  for (long e = threadIdx.x; e < tot; e += blockDim.x) {
    const int k = (int)(e / ((long)span * D));
    const int rem = (int)(e - (long)k * span * D);
    const int r = starts[k] + rem / D, c = rem % D;
    h[((long)b * L + r) * ldh + c] = f2bf(embed[c]);
  }
}

MER_API int mer_wavlm_time_mask(int B, int L, int D, void* h, long ldh, const float* embed, float mask_prob,
                                int mask_len, int min_masks, const unsigned long long* seed, unsigned long long site,
                                unsigned char* mask_out, void* stream) {
  if (B <= 0) return 0;
  if (mask_len < 1 || mask_len > L || !seed || mask_prob < 0.f) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(wavlm_time_mask_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, L, D, (bf16_t*)h, ldh, embed,
                     mask_prob, mask_len, min_masks, seed, site, mask_out);
  MER_LAUNCH_CHECK();
}

// y = x (bf16 -> bf16 or fp32), contiguous: the train-mode encoder output leaves the in-place layer buffer
__global__ void bf16_convert_kernel(long n, const bf16_t* __restrict__ x, void* __restrict__ y, int to_f32) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    if (to_f32) reinterpret_cast<float*>(y)[e] = bf2f(x[e]);
    else reinterpret_cast<bf16_t*>(y)[e] = x[e];
  }
}
MER_API int mer_bf16_convert(long n, const void* x, void* y, int y_dtype, void* stream) {
  if (n <= 0) return 0;
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(bf16_convert_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, n, (const bf16_t*)x, y,
                     y_dtype == MER_F32 ? 1 : 0);
  MER_LAUNCH_CHECK();
}
