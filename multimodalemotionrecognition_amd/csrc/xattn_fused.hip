// Fused xattn head forward (fusion.py:366-411, the north-star block) on split-bf16 MFMA.
//
// Arithmetic: every matrix product runs on v_mfma_f32_16x16x32_bf16 with each fp32 operand split into
// bf16 hi + lo planes (x = hi + lo to ~16 mantissa bits, both RNE): A.B ~= Ah.Bh + Ah.Bl + Al.Bh with fp32
// accumulation (the dropped Al.Bl term is ~2^-16 relative).  Operands that are bf16 to begin with (the WavLM
// features) have no lo plane and skip that pass.  This keeps the head at fp32-class accuracy (logits within
// 1e-4 of the reference goldens) at 16/3 x the exact-f32 MFMA rate.  Weights are split once per step by
// mer_xh_split (they change every Adam step); activations are split in registers as fragments are built.
//
// Four launches replace the ~40-launch schedule of xattn_head.py (mean temporal pooling; concat / gated):
//   F1 xh_audio_fwd (grid B*Ta/32 + B*T/16): a_seq(bf16) -> a_s = audio_seq_proj -> a = a_in_proj -> [q2 | k1 v1]
//      (the a2v query projection and the v2a key/value projections share the input a); the trailing blocks
//      project the video rows: v = v_in_proj(v_feat), q1
//   F2 xh_v2a_fwd (grid B): MHA of q1 over the sample's Ta keys -> out-proj ->
//      drop-path + residual + LayerNorm -> v1 -> [k2 v2] (the a2v key/value projections) + mean-pool of v1
//   F3 xh_a2v_fwd (grid B * ceil(Ta/16)): MHA of 16 query rows over the sample's T keys -> out-proj ->
//      drop-path + residual + LayerNorm -> a1, per-tile column sums of a1 (the a-side mean pool)
//   F4 xh_mlp_fwd (grid B): a-pool fold, concat MLP (or gated head) -> logits, exact fp32 FMA
// Every tensor the backward (xattn_head.head_backward) reads is written out with the same layout as the
// unfused schedule.  Fragment maps (v_mfma_f32_16x16x32_bf16): A lane l = row l&15, k = 8*(l>>4)..+7;
// B lane l = col l&15, same k; C/D col = l&15, row = 4*(l>>4) + r.
#include "common.h"
#include "mer.h"
#include "xattn_common.h"

using namespace xh;

// ---------------------------------------------------------------------------------------------
// weight split: for each descriptor row (src, hi, lo, rows, cols, trans, dst_ld) of a [rows][cols] fp32 weight,
// hi / lo (bf16) = split(src) in the same layout (trans 0, dst contiguous) or transposed (trans 1:
// dst[c * dst_ld + r], the [in][out] planes the backward's data-gradient products read)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void xh_split_kernel(const long long* __restrict__ desc) {
  __shared__ float tileL[32][33];
  const long long* d = desc + 7 * blockIdx.y;
  // pointers read from a table are FLAT accesses unless typed global (a flat access also waits for LDS traffic)
  typedef __attribute__((address_space(1))) const float gcf;
  typedef __attribute__((address_space(1))) bf16_t gbf;
  gcf* src = (gcf*)(d[0]);
  gbf* hi = (gbf*)(d[1]);
  gbf* lo = (gbf*)(d[2]);
  // 32-bit index math (the head's weights: well below 2^31 elements)
  const unsigned rows = (unsigned)d[3], cols = (unsigned)d[4], n = rows * cols, dld = (unsigned)d[6];
  auto split1 = [](float x, bf16_t& h, bf16_t& l) {
    h = f2bf(x);
    l = f2bf(x - bf2f(h));
  };
  if (d[5] == 0) {  // same layout: element e
    for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
      bf16_t h, l;
      split1(src[e], h, l);
      hi[e] = h;
      lo[e] = l;
    }
    return;
  }
  // transposed (dst[c * dld + r]): 32 x 32 tiles through LDS, so both the source rows and the destination rows
  // are read / written contiguously (the element-wise form wrote 2 bytes per lane to 64 different rows)
  const unsigned tr = (rows + 31) / 32, tc = (cols + 31) / 32;
  const int t = threadIdx.x, ty = t >> 3, tx = (t & 7) * 4;
  for (unsigned tile = blockIdx.x; tile < tr * tc; tile += gridDim.x) {
    const unsigned r0 = (tile / tc) * 32, c0 = (tile % tc) * 32;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const unsigned r = r0 + ty, c = c0 + tx + e;
      tileL[ty][tx + e] = (r < rows && c < cols) ? src[r * cols + c] : 0.f;
    }
    __syncthreads();
    const unsigned c = c0 + ty;  // destination row
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const unsigned r = r0 + tx + e;
      if (c < cols && r < rows) {
        bf16_t h, l;
        split1(tileL[tx + e][ty], h, l);
        hi[c * dld + r] = h;
        lo[c * dld + r] = l;
      }
    }
    __syncthreads();
  }
}

#ifdef MER_XH_TIMING
MER_API int mer_xt_read_fwd(long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(mer_xt_buf), sizeof(long long) * 4 * 512 * 16, 0,
                                  hipMemcpyDeviceToHost);
}
#endif

MER_API int mer_xh_split(int n_items, const long long* desc, void* stream) {
  if (n_items <= 0) return 0;
  hipLaunchKernelGGL(xh_split_kernel, dim3(64, n_items), dim3(256), 0, (hipStream_t)stream, desc);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// F1: audio token chain, 32 rows per block, 8 waves; the trailing ceil(B*T/16) blocks run the video rows'
// input and query projections (v, q1), which depend on nothing the audio chain makes.
// These blocks are latency chains (one block per CU, three dependent products): every weight fragment a wave
// needs for the short products is loaded into registers at block entry (WRegs), so its L2 latency overlaps
// the first phase instead of recurring at each k step of each product (phase stamps, B = 32: the video
// blocks' 512-deep product 25.3 us with a 3-deep k-step pipeline from L2; the a / [q2 | k1 v1] products
// 3.0 / 9.2 us).  The video rows' fp32 features are staged once into LDS (zero past vdim).
// ---------------------------------------------------------------------------------------------
constexpr int F1_WAVES = 8;
constexpr int F1_VROWS = 16;     // video rows per block
constexpr int F1_VK = 512;       // video feature depth bound (ResNet18: 512)
constexpr int F1_VLD = F1_VK + 4;  // LDS row stride of the staged video features

struct XhVideo {
  int M, vdim;
  const float* vfeat;
  SplitW Wv;
  const float* bv;
  SplitW Wq1;
  const float* bq1;
  float* v;
  float* q1;
};

// TA bf16: the WavLM features (exact, two passes); float: fp32 features (split, three passes).  PAIR: the first
// product was computed beforehand as ONE bf16 GEMM of the WavLM features with the stacked [hi; lo] planes of
// audio_seq_proj (mer_gemm_bf16: 256 output columns, a well-pipelined 768-deep product) and aseq is that fp32
// [M][256] pair; a_s = pair[:, :128] + pair[:, 128:] + bs.
template <typename TA, bool PAIR = false>
__global__ __launch_bounds__(64 * F1_WAVES) void xh_audio_fwd_kernel(int M, int S, const TA* __restrict__ aseq,
                                                                     long ldas, SplitW Ws, const float* __restrict__ bs,
                                                                     SplitW Wa, const float* __restrict__ ba, SplitW Wc,
                                                                     const float* __restrict__ bq2,
                                                                     const float* __restrict__ bkv1,
                                                                     float* __restrict__ a_s, float* __restrict__ a,
                                                                     float* __restrict__ q2, float* __restrict__ kv1,
                                                                     XhVideo vid) {
  __shared__ __attribute__((aligned(16))) float smem[64 * LDA];  // asL | aL; the video blocks: [16][F1_VLD]
  float* asL = smem;
  float* aL = smem + 32 * LDA;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fk = (lane >> 4) * 8;
  const int na = (M + 31) / 32;
  if ((int)blockIdx.x >= na) {  // video rows: v = v_feat Wv^T + bv, q1 = v Wq1^T + bq1 (16 columns per wave)
    XT(2, 8);
    const long v0 = (long)(blockIdx.x - na) * F1_VROWS;
    const int vmax = (int)(vid.M - v0 < F1_VROWS ? vid.M - v0 : F1_VROWS), vd = vid.vdim;
    f32x4 x[F1_VROWS * F1_VK / 4 / (64 * F1_WAVES)];
#pragma unroll
    for (int q = 0; q < F1_VROWS * F1_VK / 4 / (64 * F1_WAVES); ++q) {  // the rows first (clamped addresses)
      const int e = threadIdx.x + 64 * F1_WAVES * q, r = e / (F1_VK / 4), k = 4 * (e % (F1_VK / 4));
      x[q] = *reinterpret_cast<const f32x4*>(vid.vfeat + (v0 + (r < vmax ? r : vmax - 1)) * vd + (k < vd ? k : vd - 4));
    }
    WRegs<F1_VK / 32, 1> wv;  // then every weight fragment: their latency overlaps the staging
    wregs_load(wv, vid.Wv, vd, 16 * w, vd / 32);
    WRegs<XD / 32, 1> wq;
    wregs_load(wq, vid.Wq1, XD, 16 * w, XD / 32);
#pragma unroll
    for (int q = 0; q < F1_VROWS * F1_VK / 4 / (64 * F1_WAVES); ++q) {  // zero past vmax / vdim
      const int e = threadIdx.x + 64 * F1_WAVES * q, r = e / (F1_VK / 4), k = 4 * (e % (F1_VK / 4));
      *reinterpret_cast<f32x4*>(smem + r * F1_VLD + k) = (r < vmax && k < vd) ? x[q] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    lds_sync();  // LDS only: the weight loads stay in flight
    f32x4 acc[1][1];
    {  // two accumulator chains (even / odd k steps) so consecutive MFMAs do not wait on each other
      f32x4 c2[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int s = 0; s < F1_VK / 32; ++s) {
        bf16x8 ah, al;
        frag_row(smem + fr * F1_VLD + 32 * s + fk, true, ah, al);
        Frag H, L;
        H.u = wv.h[s][0];
        L.u = wv.l[s][0];
        c2[s & 1] = mma3(ah, al, H.v, L.v, c2[s & 1]);
      }
      acc[0][0] = c2[0] + c2[1];
    }
    lds_sync();  // the staged features are dead: v goes to LDS rows 0..15
    store_acc(acc, 16 * w, vid.bv, smem, LDA, vid.v, XD, v0, vmax);
    lds_sync();
    XT(2, 9);
    zero(acc);
    mm_lw<1, 1, XD / 32>(acc, smem, LDA, wq);
    store_acc(acc, 16 * w, vid.bq1, nullptr, 0, vid.q1, XD, v0, vmax);
    XT(2, 10);
    return;
  }
  XT(2, 0);
  const long r0 = (long)blockIdx.x * 32;
  const int rmax = (int)(M - r0 < 32 ? M - r0 : 32);
  WRegs<XD / 32, 1> wa;
  WRegs<XD / 32, 3> wc;
  // a_s = a_seq Ws^T + bs  (bf16 A is exact: two passes; fp32 A: split, three passes); wave (w & 3) owns 32
  // columns, wave half (w >> 2) one half of K
  if constexpr (PAIR) {
    const float* pr = reinterpret_cast<const float*>(aseq);
    f32x4 x0[2], x1[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {  // 32 rows x 32 float4 per half, two per thread
      const int e = threadIdx.x + 64 * F1_WAVES * q, r = e >> 5, c = 4 * (e & 31);
      const long rc = r0 + (r < rmax ? r : rmax - 1);
      x0[q] = *reinterpret_cast<const f32x4*>(pr + rc * ldas + c);
      x1[q] = *reinterpret_cast<const f32x4*>(pr + rc * ldas + XD + c);
    }
    wregs_load(wa, Wa, XD, 16 * w, XD / 32);  // issued after the pair loads: their latency overlaps the sum
    wregs_load(wc, Wc, XD, 48 * w, XD / 32);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int e = threadIdx.x + 64 * F1_WAVES * q, r = e >> 5, c = 4 * (e & 31);
      const f32x4 v = (x0[q] + x1[q]) + *reinterpret_cast<const f32x4*>(bs + c);
      *reinterpret_cast<f32x4*>(asL + r * LDA + c) = r < rmax ? v : f32x4{0.f, 0.f, 0.f, 0.f};
      if (r < rmax) *reinterpret_cast<f32x4*>(a_s + (r0 + r) * XD + c) = v;
    }
    XT(2, 1);
  } else {
    f32x4 acc[2][2];
    zero(acc);
    const int c0 = 32 * (w & 3), kh = w >> 2, Kh = S / 2, kbase = kh * Kh;
    if constexpr (sizeof(TA) == 2) {  // pipelined like mm_aw, F1_D k steps in flight
      constexpr int F1_D = 6;
      u4 sa[F1_D][2], sb[F1_D][2][2];
      auto load = [&](int k, u4 (&ra)[2], u4 (&rb)[2][2]) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const long off = (long)(c0 + 16 * j + fr) * S + kbase + k + fk;
          rb[j][0] = *reinterpret_cast<const u4*>(Ws.hi + off);
          rb[j][1] = *reinterpret_cast<const u4*>(Ws.lo + off);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r = 16 * i + fr;
          ra[i] = *reinterpret_cast<const u4*>(aseq + (r0 + (r < rmax ? r : rmax - 1)) * ldas + kbase + k + fk);
        }
      };
      const int nsteps = Kh / 32;  // branch-free pipeline, as mm_aw
#pragma unroll
      for (int d = 0; d < F1_D; ++d) load(32 * (d < nsteps ? d : nsteps - 1), sa[d], sb[d]);
      for (int s0 = 0; s0 < nsteps; s0 += F1_D) {
#pragma unroll
        for (int d = 0; d < F1_D; ++d) {
          const bool live = s0 + d < nsteps;
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            Frag A;
            A.u = live ? sa[d][i] : u4{0u, 0u, 0u, 0u};
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              Frag H, L;
              H.u = sb[d][j][0];
              L.u = sb[d][j][1];
              acc[i][j] = mma(A.v, H.v, acc[i][j]);
              acc[i][j] = mma(A.v, L.v, acc[i][j]);
            }
          }
          const int nx = s0 + d + F1_D;
          load(32 * (nx < nsteps ? nx : nsteps - 1), sa[d], sb[d]);
        }
      }
    } else {
      mm_aw(acc, reinterpret_cast<const float*>(aseq) + r0 * ldas + kbase, ldas, rmax, Kh,
            SplitW{Ws.hi + kbase, Ws.lo + kbase}, S, c0);
    }
    wregs_load(wa, Wa, XD, 16 * w, XD / 32);
    wregs_load(wc, Wc, XD, 48 * w, XD / 32);
    // the upper K half's partial sums through aL (free until the second product), added in a fixed order
    if (kh == 1) store_acc(acc, c0, nullptr, aL, LDA, nullptr, 0, 0, 32);
    __syncthreads();
    if (kh == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += aL[(16 * i + 4 * (lane >> 4) + r) * LDA + c0 + 16 * j + fr];
      store_acc(acc, c0, bs, asL, LDA, a_s, XD, r0, rmax);
    }
  }
  lds_sync();  // LDS only: the weight loads and the a_s stores stay in flight
  XT(2, 2);
  {  // a = a_s Wa^T + ba (16 columns per wave)
    f32x4 acc[2][1];
    zero(acc);
    mm_lw<2, 1, XD / 32>(acc, asL, LDA, wa);
    store_acc(acc, 16 * w, ba, aL, LDA, a, XD, r0, rmax);
  }
  lds_sync();
  XT(2, 3);
  {  // [q2 | k1 v1] = a Wc^T + [bq2 | bkv1]: 384 columns, 48 per wave in ONE pipelined pass (K = 128: 4 steps)
    f32x4 acc[2][3];
    zero(acc);
    const int c0 = 48 * w;
    mm_lw<2, 3, XD / 32>(acc, aL, LDA, wc);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int col = c0 + 16 * j + fr;
      const bool isq = col < XD;
      const float bv = isq ? bq2[col] : bkv1[col - XD];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * i + 4 * (lane >> 4) + r;
          if (row >= rmax) continue;
          const float v = acc[i][j][r] + bv;
          if (isq) q2[(r0 + row) * XD + col] = v;
          else kv1[(r0 + row) * 2 * XD + col - XD] = v;
        }
    }
  }
  XT(2, 4);
}

MER_API int mer_xh_audio_fwd_pair(int M, const float* pair, long ldp, const float* bs, const void* Wa_hi,
                                  const void* Wa_lo, const float* ba, const void* Wc_hi, const void* Wc_lo,
                                  const float* bq2, const float* bkv1, float* a_s, float* a, float* q2, float* kv1, int Mv,
                                  int vdim, const float* vfeat, const void* Wv_hi, const void* Wv_lo, const float* bv,
                                  const void* Wq1_hi, const void* Wq1_lo, const float* bq1, float* v, float* q1,
                                  void* stream) {
  if (M <= 0 || Mv < 0 || ldp < 2 * XD || ldp % 4 || ((uintptr_t)pair & 15) ||
      (Mv > 0 && (vdim <= 0 || vdim % 32 || vdim > F1_VK || ((uintptr_t)vfeat & 15))))
    return (int)hipErrorInvalidValue;
  const SplitW wa{(const bf16_t*)Wa_hi, (const bf16_t*)Wa_lo}, wc{(const bf16_t*)Wc_hi, (const bf16_t*)Wc_lo};
  const XhVideo vid{Mv, vdim, vfeat, SplitW{(const bf16_t*)Wv_hi, (const bf16_t*)Wv_lo}, bv,
                    SplitW{(const bf16_t*)Wq1_hi, (const bf16_t*)Wq1_lo}, bq1, v, q1};
  const dim3 grid((M + 31) / 32 + (Mv + F1_VROWS - 1) / F1_VROWS);
  hipLaunchKernelGGL((xh_audio_fwd_kernel<float, true>), grid, dim3(64 * F1_WAVES), 0, (hipStream_t)stream, M, 2 * XD,
                     pair, ldp, SplitW{nullptr, nullptr}, bs, wa, ba, wc, bq2, bkv1, a_s, a, q2, kv1, vid);
  MER_LAUNCH_CHECK();
}

MER_API int mer_xh_audio_fwd(int M, int S, const void* aseq, int aseq_dtype, long ldas, const void* Ws_hi,
                             const void* Ws_lo, const float* bs, const void* Wa_hi, const void* Wa_lo, const float* ba,
                             const void* Wc_hi, const void* Wc_lo, const float* bq2, const float* bkv1, float* a_s,
                             float* a, float* q2, float* kv1, int Mv, int vdim, const float* vfeat, const void* Wv_hi,
                             const void* Wv_lo, const float* bv, const void* Wq1_hi, const void* Wq1_lo,
                             const float* bq1, float* v, float* q1, void* stream) {
  // M = 0: the video rows alone; Mv = 0: the audio chain alone (the head's audio-first schedule launches them
  // separately, the audio chain on a side stream beside the frame trunk)
  if (M < 0 || Mv < 0 || M + Mv == 0) return (int)hipErrorInvalidValue;
  if ((M > 0 && (S % 64 || ldas % 8 || ((uintptr_t)aseq & 15))) ||
      (Mv > 0 && (vdim <= 0 || vdim % 32 || vdim > F1_VK || ((uintptr_t)vfeat & 15))))
    return (int)hipErrorInvalidValue;
  const SplitW ws{(const bf16_t*)Ws_hi, (const bf16_t*)Ws_lo}, wa{(const bf16_t*)Wa_hi, (const bf16_t*)Wa_lo},
      wc{(const bf16_t*)Wc_hi, (const bf16_t*)Wc_lo};
  const XhVideo vid{Mv, vdim, vfeat, SplitW{(const bf16_t*)Wv_hi, (const bf16_t*)Wv_lo}, bv,
                    SplitW{(const bf16_t*)Wq1_hi, (const bf16_t*)Wq1_lo}, bq1, v, q1};
  const dim3 grid((M + 31) / 32 + (Mv + F1_VROWS - 1) / F1_VROWS);
  if (aseq_dtype == MER_BF16)
    hipLaunchKernelGGL(xh_audio_fwd_kernel<bf16_t>, grid, dim3(64 * F1_WAVES), 0, (hipStream_t)stream, M, S,
                       (const bf16_t*)aseq, ldas, ws, bs, wa, ba, wc, bq2, bkv1, a_s, a, q2, kv1, vid);
  else
    hipLaunchKernelGGL(xh_audio_fwd_kernel<float>, grid, dim3(64 * F1_WAVES), 0, (hipStream_t)stream, M, S,
                       (const float*)aseq, ldas, ws, bs, wa, ba, wc, bq2, bkv1, a_s, a, q2, kv1, vid);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// Shared attention pieces.  One wave owns one head: S (16 query rows x up to 16*NT keys) in registers,
// softmax by in-lane + 16-lane xor reductions, P (pre-dropout) to global, P' = dropout(P) through the
// wave's LDS tile into O_h = P' V_h.
// ---------------------------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ void head_attention(int b, int h, int i0, int Lq, int Lk, const float* Qrows, long ldq,
                                               const float* Krows, const float* Vrows, long ldkv, float scale,
                                               float* P, float drop_p, unsigned long long dseed, float* PL, int pld,
                                               float* oL, const float* __restrict__ bias) {
  const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4, fk = fq * 8;
  constexpr int KP = 16 * NT;               // keys padded to the tile
  constexpr int KC = (KP + 31) / 32 * 32;   // PV contracts over KP rounded up to 32
  // Every global load of the head is issued up front, so the whole attention waits on ONE memory latency: the
  // K fragments of the NT key tiles and the V column gathers of the PV contraction (raw fp32, split at use).
  f32x4 kraw[NT][2];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int j = 16 * t + fr;
    const float* kp = Krows + (long)(j < Lk ? j : Lk - 1) * ldkv + h * XDH + fk;
    kraw[t][0] = *reinterpret_cast<const f32x4*>(kp);
    kraw[t][1] = *reinterpret_cast<const f32x4*>(kp + 4);
  }
  float vraw[KC / 32][2][8];
#pragma unroll
  for (int k = 0; k < KC / 32; ++k)
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int kk = 32 * k + fk + e;
        vraw[k][jt][e] = Vrows[(long)(kk < Lk ? kk : Lk - 1) * ldkv + h * XDH + 16 * jt + fr];
      }
  // the emotion-prior attention bias of this sample (fusion.py:390-398 attn_mask, added after the scaling):
  // bias[b][i][j], the same for every head
  float bv[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * fq + r, j = 16 * t + fr;
      const long bi = ((long)b * Lq + (i < Lq ? i : Lq - 1)) * Lk + (j < Lk ? j : Lk - 1);
      bv[t][r] = bias ? bias[bi] : 0.f;
    }
  // S = Q_h K_h^T: A = Q rows (k = head dims), B[n = key][k] = K rows
  f32x4 s[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    bf16x8 ah, al;
    frag_row(Qrows + (long)(i0 + fr < Lq ? fr : Lq - 1 - i0) * ldq + h * XDH + fk, i0 + fr < Lq, ah, al);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const bool ok = 16 * t + fr < Lk;
      float x[8] = {kraw[t][0][0], kraw[t][0][1], kraw[t][0][2], kraw[t][0][3],
                    kraw[t][1][0], kraw[t][1][1], kraw[t][1][2], kraw[t][1][3]};
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = ok ? x[e] : 0.f;
      bf16x8 bh, bl;
      split8(x, bh, bl);
      s[t] = mma3(ah, al, bh, bl, s[t]);
    }
  }
  float mx[4], sum[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) mx[r] = -INFINITY;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * t + fr;
      s[t][r] = j < Lk ? s[t][r] * scale + bv[t][r] : -INFINITY;
      mx[r] = fmaxf(mx[r], s[t][r]);
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], o, 64));
    sum[r] = 0.f;
  }
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = 16 * t + fr < Lk ? __expf(s[t][r] - mx[r]) : 0.f;
      s[t][r] = e;
      sum[r] += e;
    }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) sum[r] += __shfl_xor(sum[r], o, 64);
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * fq + r, j = 16 * t + fr;
      float pd = 0.f;
      if (i < Lq && j < Lk) {
        const float pr = s[t][r] / sum[r];
        const long pi = (((long)b * XH + h) * Lq + i) * Lk + j;
        P[pi] = pr;
        pd = pr * dropout_scale(dseed, pi, drop_p);
      }
      PL[(4 * fq + r) * pld + j] = pd;
    }
  if (KP % 32) {  // zero the pad chunk the contraction reads
    for (int e = lane; e < 16 * 16; e += 64) PL[(e >> 4) * pld + KP + (e & 15)] = 0.f;
  }
  wave_sync_lds();
  // O_h = P' V_h: A = P' (16 x KC), B[n = head dim][k = key] = the preloaded V gathers
  f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int k = 0; k < KC / 32; ++k) {
    bf16x8 ah, al;
    frag_row(PL + fr * pld + 32 * k + fk, true, ah, al);
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = 32 * k + fk + e < Lk ? vraw[k][jt][e] : 0.f;
      bf16x8 bh, bl;
      split8(x, bh, bl);
      o[jt] = mma3(ah, al, bh, bl, o[jt]);
    }
  }
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) oL[(4 * fq + r) * LDA + h * XDH + 16 * jt + fr] = o[jt][r];
}

// s = x + keep_b * y; LayerNorm(s) over 128 columns for `nrows` rows of LDS tiles (one wave per row);
// saves s / mean / rstd (global rows grow0 + r) and writes the normalised row to out (LDS) and / or g_out
__device__ __forceinline__ void add_ln_rows(int nrows, const float* xL, const float* yL, float keep_scale,
                                            const float* gamma, const float* beta, float* outL, float* s_g,
                                            float* mean_g, float* rstd_g, long grow0) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int r = w; r < nrows; r += 4) {
    const float v0 = xL[r * LDA + lane] + keep_scale * yL[r * LDA + lane];
    const float v1 = xL[r * LDA + 64 + lane] + keep_scale * yL[r * LDA + 64 + lane];
    const float mean = wave_sum(v0 + v1) / XD;
    const float d0 = v0 - mean, d1 = v1 - mean;
    const float rstd = rsqrtf(wave_sum(d0 * d0 + d1 * d1) / XD + 1e-5f);
    outL[r * LDA + lane] = d0 * rstd * gamma[lane] + beta[lane];
    outL[r * LDA + 64 + lane] = d1 * rstd * gamma[64 + lane] + beta[64 + lane];
    s_g[(grow0 + r) * XD + lane] = v0;
    s_g[(grow0 + r) * XD + 64 + lane] = v1;
    if (lane == 0) {
      mean_g[grow0 + r] = mean;
      rstd_g[grow0 + r] = rstd;
    }
  }
}

constexpr int F2_KT = 10;  // 16-key tiles of the v2a attention (Ta <= 160: F4 folds up to this many F3 tiles)

// ---------------------------------------------------------------------------------------------
// F2: the v2a block as two launches.  F2a = the v2a attention, one workgroup per (sample, head) -- 128 workgroups
// at B = 32 (the one-workgroup-per-sample version, a wave per head, ran 32), each wave walking a quarter of the
// keys --; F2b = its out-projection, drop-path + residual + LayerNorm, v-pool and [k2 v2] projection, one
// workgroup per sample.
//
// F2a: wave w owns the 32-key chunk c = w of the sample's Ta keys (8 waves: Ta <= 256; with 4 waves and two chunks on
// wave 0 at Ta = 149, the PV phase of that wave set the block time -- tools/xt_phases.py: 3.0 of 7.4 us).  Scores
// S = Q_h K^T (+ the emotion-prior bias), the row max and then the row sum of exp(S - max) meet across the waves in LDS
// (fixed order), P = exp / sum is saved (pre-dropout, as the unfused schedule saves it), and each wave's P' V_h partial
// is summed in a fixed order into o1's 32 columns of head h.  Loads are issued up front (one memory latency).
// ---------------------------------------------------------------------------------------------
constexpr int F2A_W = 8;                  // waves = 32-key chunks: Ta <= F2A_W * 32 = 256
constexpr int F2A_PLD = 36;               // P' chunk stride

// fixed-order sum of v[0..N) (N a power of two): pairwise, the same tree whatever the wave schedule
template <int N>
__device__ __forceinline__ float tree_sum(const float* v, int stride) {
  if constexpr (N == 1) {
    return v[0];
  } else {
    return tree_sum<N / 2>(v, stride) + tree_sum<N / 2>(v + (N / 2) * stride, stride);
  }
}

__global__ __launch_bounds__(64 * F2A_W) void xh_v2a_attn_kernel(int T, int Ta, const float* __restrict__ q1,
                                                                 const float* __restrict__ kv1, XhDrop dr, float scale,
                                                                 float* __restrict__ P1, float* __restrict__ o1,
                                                                 const float* __restrict__ bias) {
  __shared__ float red[2][F2A_W][16];                                    // per-wave row max / row sum
  __shared__ __attribute__((aligned(16))) float PL[F2A_W][16 * F2A_PLD];  // per-wave P' chunk (PV A operand)
  __shared__ float oP[F2A_W][16][33];                                    // per-wave P' V partials
  XT(3, 0);
  const int b = blockIdx.x >> 2, h = blockIdx.x & 3;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4, fk = fq * 8;
  const long ldkv = 2 * XD;
  const float* Kr = kv1 + (long)b * Ta * ldkv + h * XDH;       // key j: Kr[j * ldkv + d]
  const float* Vr = Kr + XD;                                   // value j: Vr[j * ldkv + d]
  const int c = w;                                             // this wave's chunk
  const bool live = 32 * c < Ta;                               // (wave-uniform)
  const unsigned long long dseed = mer_site_seed(dr.seed, dr.site_attn);
  // every global load first: K fragments and V gathers of this wave's chunk (clamped rows), the prior bias
  f32x4 kraw[2][2];
  float vraw[2][8];
  float bv[2][4];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int j = 32 * c + 16 * tt + fr, jc = j < Ta ? j : Ta - 1;
    kraw[tt][0] = *reinterpret_cast<const f32x4*>(Kr + (long)jc * ldkv + fk);
    kraw[tt][1] = *reinterpret_cast<const f32x4*>(Kr + (long)jc * ldkv + fk + 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * fq + r;
      const long bi = ((long)b * T + (i < T ? i : T - 1)) * Ta + jc;
      bv[tt][r] = bias ? bias[bi] : 0.f;
    }
  }
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kk = 32 * c + fk + e;
      vraw[jt][e] = Vr[(long)(kk < Ta ? kk : Ta - 1) * ldkv + 16 * jt + fr];
    }
  bf16x8 qh, ql;
  frag_row(q1 + ((long)b * T + (fr < T ? fr : T - 1)) * XD + h * XDH + fk, fr < T, qh, ql);
  XT(3, 1);
  f32x4 s[2];
  float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int j = 32 * c + 16 * tt + fr;
    float x[8] = {kraw[tt][0][0], kraw[tt][0][1], kraw[tt][0][2], kraw[tt][0][3],
                  kraw[tt][1][0], kraw[tt][1][1], kraw[tt][1][2], kraw[tt][1][3]};
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = j < Ta ? x[e] : 0.f;
    bf16x8 bh, bl;
    split8(x, bh, bl);
    s[tt] = mma3(qh, ql, bh, bl, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[tt][r] = j < Ta ? s[tt][r] * scale + bv[tt][r] : -INFINITY;
      mx[r] = fmaxf(mx[r], s[tt][r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], o, 64));
    if (fr == 0) red[0][w][4 * fq + r] = mx[r];
  }
  __syncthreads();
  float sum[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 4 * fq + r;
    float m = red[0][0][i];
#pragma unroll
    for (int q = 1; q < F2A_W; ++q) m = fmaxf(m, red[0][q][i]);
    mx[r] = m;
    sum[r] = 0.f;
  }
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 32 * c + 16 * tt + fr;
      const float e = j < Ta ? __expf(s[tt][r] - mx[r]) : 0.f;
      s[tt][r] = e;
      sum[r] += e;
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) sum[r] += __shfl_xor(sum[r], o, 64);
    if (fr == 0) red[1][w][4 * fq + r] = sum[r];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) sum[r] = tree_sum<F2A_W>(&red[1][0][4 * fq + r], 16);
  XT(3, 2);
  // P (saved, pre-dropout), P' = dropout(P) through LDS into O_w = P'_w V_w
  f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  float* pl = PL[w];
  if (live) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 4 * fq + r, j = 32 * c + 16 * tt + fr;
        float pd = 0.f;
        if (i < T && j < Ta) {
          const float pr = s[tt][r] / sum[r];
          const long pi = (((long)b * XH + h) * T + i) * Ta + j;
          P1[pi] = pr;
          pd = pr * dropout_scale(dseed, pi, dr.attn);
        }
        pl[i * F2A_PLD + 16 * tt + fr] = pd;
      }
    wave_sync_lds();
    bf16x8 ah, al;
    frag_row(pl + fr * F2A_PLD + fk, true, ah, al);
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = 32 * c + fk + e < Ta ? vraw[jt][e] : 0.f;
      bf16x8 bh, bl;
      split8(x, bh, bl);
      o[jt] = mma3(ah, al, bh, bl, o[jt]);
    }
  }
  XT(3, 3);
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) oP[w][4 * fq + r][16 * jt + fr] = o[jt][r];
  __syncthreads();
  for (int e = threadIdx.x; e < T * XDH; e += 64 * F2A_W) {
    const int i = e / XDH, d = e - i * XDH;
    o1[((long)b * T + i) * XD + h * XDH + d] = tree_sum<F2A_W>(&oP[0][i][d], 16 * 33);
  }
  XT(3, 4);
}

// F2b: F2's second half on o1 (one workgroup per sample): v2 = o1 Wo1^T + bo1, v1 = LN(v + keep_b v2), v-pool,
// [k2 v2] = v1 Wkv2^T + bkv2
__global__ __launch_bounds__(256) void xh_v2a_post_kernel(
    int T, const float* __restrict__ v, const float* __restrict__ o1, SplitW Wo1, const float* __restrict__ bo1,
    const float* __restrict__ gamma, const float* __restrict__ beta, SplitW Wkv2, const float* __restrict__ bkv2,
    XhDrop dr, float* __restrict__ s_v, float* __restrict__ mean_v, float* __restrict__ rstd_v, float* __restrict__ v1,
    float* __restrict__ kv2, float* __restrict__ emb, long ld_emb) {
  __shared__ __attribute__((aligned(16))) float vL[16 * LDA];
  __shared__ __attribute__((aligned(16))) float oL[16 * LDA];
  __shared__ __attribute__((aligned(16))) float tL[16 * LDA];
  const int b = blockIdx.x, w = threadIdx.x >> 6;
  const long row0 = (long)b * T;
  const unsigned long long seed_path = mer_site_seed(dr.seed, dr.site_path);
  // every weight fragment of both products first (registers), then the rows: one memory latency for all
  WRegs<XD / 32, 2> wo;
  wregs_load(wo, Wo1, XD, 32 * w, XD / 32);
  WRegs<XD / 32, 4> wkv;
  wregs_load(wkv, Wkv2, XD, 64 * w, XD / 32);
  {
    f32x4 xv[16 * XD / 4 / 256], xo[16 * XD / 4 / 256];
#pragma unroll
    for (int q = 0; q < 16 * XD / 4 / 256; ++q) {
      const int e = threadIdx.x + 256 * q, r = e / (XD / 4), c = 4 * (e % (XD / 4));
      const long rc = row0 + (r < T ? r : T - 1);
      xv[q] = *reinterpret_cast<const f32x4*>(v + rc * XD + c);
      xo[q] = *reinterpret_cast<const f32x4*>(o1 + rc * XD + c);
    }
#pragma unroll
    for (int q = 0; q < 16 * XD / 4 / 256; ++q) {
      const int e = threadIdx.x + 256 * q, r = e / (XD / 4), c = 4 * (e % (XD / 4));
      const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f32x4*>(vL + r * LDA + c) = r < T ? xv[q] : z;
      *reinterpret_cast<f32x4*>(oL + r * LDA + c) = r < T ? xo[q] : z;
    }
  }
  lds_sync();
  {  // v2 = o Wo1^T + bo1
    f32x4 acc[1][2];
    zero(acc);
    mm_lw<1, 2, XD / 32>(acc, oL, LDA, wo);
    store_acc(acc, 32 * w, bo1, tL, LDA, nullptr, 0, 0, 16);
  }
  lds_sync();
  // v1 = LN(v + keep_b * v2)  (StochasticDepth: one keep draw per sample, fusion.py:11-26)
  add_ln_rows(T, vL, tL, dropout_scale(seed_path, b, dr.path), gamma, beta, oL, s_v, mean_v, rstd_v, row0);
  lds_sync();
  for (int e = threadIdx.x; e < T * XD; e += 256) v1[row0 * XD + e] = oL[(e / XD) * LDA + e % XD];
  for (int e = threadIdx.x; e < (16 - T) * XD; e += 256) oL[(T + e / XD) * LDA + e % XD] = 0.f;
  if (threadIdx.x < XD) {  // mean temporal pool of v1 (temporal.py:108-109) -> emb[b, 0:d]
    float s = 0.f;
    for (int r = 0; r < T; ++r) s += oL[r * LDA + threadIdx.x];
    emb[(long)b * ld_emb + threadIdx.x] = s / T;
  }
  lds_sync();
  {  // [k2 v2] = v1 Wkv2^T + bkv2: 256 columns, 64 per wave
    f32x4 acc[1][4];
    zero(acc);
    mm_lw<1, 4, XD / 32>(acc, oL, LDA, wkv);
    store_acc(acc, 64 * w, bkv2, nullptr, 0, kv2, 2 * XD, row0, T);
  }
}

MER_API int mer_xh_v2a_fwd(int B, int T, int Ta, const float* v, const float* q1, const float* kv1, const void* Wo1_hi,
                            const void* Wo1_lo, const float* bo1, const float* gamma, const float* beta,
                            const void* Wkv2_hi, const void* Wkv2_lo, const float* bkv2, float attn_p, float path_p,
                            const unsigned long long* seed, unsigned long long site_attn, unsigned long long site_path,
                            float scale, float* P1, float* o1, float* s_v, float* mean_v, float* rstd_v, float* v1,
                            float* kv2, float* emb, long ld_emb, const float* bias, void* stream) {
  if (B <= 0) return 0;
  if (T <= 0 || T > 16 || Ta <= 0 || Ta > F2A_W * 32) return (int)hipErrorInvalidValue;
  if ((attn_p > 0.f || path_p > 0.f) && !seed) return (int)hipErrorInvalidValue;
  XhDrop dr{attn_p, path_p, seed, site_attn, site_path};
  hipLaunchKernelGGL(xh_v2a_attn_kernel, dim3(B * XH), dim3(64 * F2A_W), 0, (hipStream_t)stream, T, Ta, q1, kv1, dr,
                     scale, P1, o1, bias);
  hipLaunchKernelGGL(xh_v2a_post_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, T, v, o1,
                     SplitW{(const bf16_t*)Wo1_hi, (const bf16_t*)Wo1_lo}, bo1, gamma, beta,
                     SplitW{(const bf16_t*)Wkv2_hi, (const bf16_t*)Wkv2_lo}, bkv2, dr, s_v, mean_v, rstd_v, v1, kv2,
                     emb, ld_emb);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// F3: a2v block, one workgroup per (sample, 16 query rows); keys = the sample's T (<= 16) v1 rows.
// ---------------------------------------------------------------------------------------------
constexpr int F3_PLD = 36;

__global__ __launch_bounds__(256) void xh_a2v_fwd_kernel(int T, int Ta, int ntiles, const float* __restrict__ q2,
                                                         const float* __restrict__ kv2, const float* __restrict__ a,
                                                         SplitW Wo2, const float* __restrict__ bo2,
                                                         const float* __restrict__ gamma, const float* __restrict__ beta,
                                                         XhDrop dr, float scale, float* __restrict__ P2,
                                                         float* __restrict__ o2, float* __restrict__ s_a,
                                                         float* __restrict__ mean_a, float* __restrict__ rstd_a,
                                                         float* __restrict__ part, const float* __restrict__ bias) {
  __shared__ __attribute__((aligned(16))) float aL[16 * LDA];
  __shared__ __attribute__((aligned(16))) float oL[16 * LDA];
  __shared__ __attribute__((aligned(16))) float tL[16 * LDA];
  __shared__ __attribute__((aligned(16))) float PL[XH * 16 * F3_PLD];
  const int b = blockIdx.x / ntiles, tile = blockIdx.x - b * ntiles, w = threadIdx.x >> 6;
  const int i0 = tile * 16;
  const int nr = Ta - i0 < 16 ? Ta - i0 : 16;
  const long row0 = (long)b * Ta + i0;
  const unsigned long long seed_attn = mer_site_seed(dr.seed, dr.site_attn);
  const unsigned long long seed_path = mer_site_seed(dr.seed, dr.site_path);
  XT(1, 0);
  // the residual rows and the out-projection's weight fragments are loaded before the attention (their latency
  // overlaps it)
  f32x4 ar[16 * XD / 4 / 256];
#pragma unroll
  for (int q = 0; q < 16 * XD / 4 / 256; ++q) {
    const int e = threadIdx.x + 256 * q, r = e / (XD / 4), c = 4 * (e % (XD / 4));
    ar[q] = *reinterpret_cast<const f32x4*>(a + (row0 + (r < nr ? r : nr - 1)) * XD + c);
  }
  WRegs<XD / 32, 2> wo;
  wregs_load(wo, Wo2, XD, 32 * w, XD / 32);
  head_attention<1>(b, w, i0, Ta, T, q2 + row0 * XD, XD, kv2 + (long)b * T * 2 * XD, kv2 + (long)b * T * 2 * XD + XD,
                    2 * XD, scale, P2, dr.attn, seed_attn, PL + w * 16 * F3_PLD, F3_PLD, oL, bias);
  XT(1, 1);
#pragma unroll
  for (int q = 0; q < 16 * XD / 4 / 256; ++q) {
    const int e = threadIdx.x + 256 * q, r = e / (XD / 4), c = 4 * (e % (XD / 4));
    *reinterpret_cast<f32x4*>(aL + r * LDA + c) = r < nr ? ar[q] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  lds_sync();
  for (int e = threadIdx.x; e < nr * XD; e += 256) o2[row0 * XD + e] = oL[(e / XD) * LDA + e % XD];
  {  // a2 = o Wo2^T + bo2
    f32x4 acc[1][2];
    zero(acc);
    mm_lw<1, 2, XD / 32>(acc, oL, LDA, wo);
    store_acc(acc, 32 * w, bo2, tL, LDA, nullptr, 0, 0, 16);
  }
  lds_sync();
  add_ln_rows(nr, aL, tL, dropout_scale(seed_path, b, dr.path), gamma, beta, oL, s_a, mean_a, rstd_a, row0);
  lds_sync();
  if (threadIdx.x < XD) {  // this tile's column sums of a1 (the a-side mean pool, folded in tile order by F4)
    float s = 0.f;
    for (int r = 0; r < nr; ++r) s += oL[r * LDA + threadIdx.x];
    part[((long)b * ntiles + tile) * XD + threadIdx.x] = s;
  }
  XT(1, 2);
}

MER_API int mer_xh_a2v_fwd(int B, int T, int Ta, const float* q2, const float* kv2, const float* a, const void* Wo2_hi,
                           const void* Wo2_lo, const float* bo2, const float* gamma, const float* beta, float attn_p,
                           float path_p, const unsigned long long* seed, unsigned long long site_attn,
                           unsigned long long site_path, float scale, float* P2, float* o2, float* s_a, float* mean_a,
                           float* rstd_a, float* part, const float* bias, void* stream) {
  if (B <= 0) return 0;
  if (T <= 0 || T > 16 || Ta <= 0) return (int)hipErrorInvalidValue;
  if ((attn_p > 0.f || path_p > 0.f) && !seed) return (int)hipErrorInvalidValue;
  const int ntiles = (Ta + 15) / 16;
  XhDrop dr{attn_p, path_p, seed, site_attn, site_path};
  hipLaunchKernelGGL(xh_a2v_fwd_kernel, dim3(B * ntiles), dim3(256), 0, (hipStream_t)stream, T, Ta, ntiles, q2, kv2,
                     a, SplitW{(const bf16_t*)Wo2_hi, (const bf16_t*)Wo2_lo}, bo2, gamma, beta, dr, scale, P2, o2, s_a,
                     mean_a, rstd_a, part, bias);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// F4: a-pool fold + classifier head (fusion.py:404-411), ONE sample per workgroup, exact fp32 FMA.
//   concat: h = dropout(relu(emb W0^T + b0)), logits = h W3^T + b3
//   gated:  h = dropout(relu(emb Wg0^T + b)), z = h Wg3^T + b, g = sigmoid(z),
//           fused = g v_emb + (1 - g) a_emb, logits = fused Wc^T + bc
// Every product is rows . vector with k across the 64 lanes (each weight row is one coalesced 512 B / 1 KB
// load per wave, 8 rows in flight per wave), the 8 per-lane partials of a row group reduced by a transposing
// butterfly (dot_rows8).  The per-sample chain is a handful of dependent L2 round trips; B workgroups.
// ---------------------------------------------------------------------------------------------

// v[j] (j < 8: partial sums of 8 rows) -> every lane holds the full sum of row 4*b5 + 2*b4 + b3 (lane bits)
__device__ __forceinline__ float xpose_sum8(float (&v)[8]) {
  const int lane = threadIdx.x & 63;
  const bool h5 = lane & 32, h4 = lane & 16, h3 = lane & 8;
  float u[4], q[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float send = h5 ? v[i] : v[4 + i];
    u[i] = (h5 ? v[4 + i] : v[i]) + __shfl_xor(send, 32, 64);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float send = h4 ? u[i] : u[2 + i];
    q[i] = (h4 ? u[2 + i] : u[i]) + __shfl_xor(send, 16, 64);
  }
  float r = (h3 ? q[1] : q[0]) + __shfl_xor(h3 ? q[0] : q[1], 8, 64);
  r += __shfl_xor(r, 4, 64);
  r += __shfl_xor(r, 2, 64);
  r += __shfl_xor(r, 1, 64);
  return r;
}

// rows [r0, r0 + 8) of W ([nrows][K], row stride ldw) dotted with x (LDS, K floats): returns the sum of row
// r0 + ((lane >> 3) & 7) in every lane (rows >= nrows read row nrows - 1: callers drop them).  K = 64 * KL.
template <int KL>
__device__ __forceinline__ float dot_rows8(const float* __restrict__ W, long ldw, int nrows, int r0, const float* xL) {
  const int lane = threadIdx.x & 63;
  float xv[KL];
#pragma unroll
  for (int e = 0; e < KL; ++e) xv[e] = xL[KL * lane + e];
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r = r0 + j < nrows ? r0 + j : nrows - 1;
    const float* wr = W + (long)r * ldw + KL * lane;
    float wv[KL];
    if constexpr (KL == 4) {
      const f32x4 q = *reinterpret_cast<const f32x4*>(wr);
      wv[0] = q[0]; wv[1] = q[1]; wv[2] = q[2]; wv[3] = q[3];
    } else {
#pragma unroll
      for (int e = 0; e < KL; ++e) wv[e] = wr[e];
    }
    float acc = 0.f;
#pragma unroll
    for (int e = 0; e < KL; ++e) acc = fmaf(wv[e], xv[e], acc);
    v[j] = acc;
  }
  return xpose_sum8(v);
}

template <bool GATED>
__global__ __launch_bounds__(256) void xh_mlp_fwd_kernel(int Ta, int ntiles, int H1, int C,
                                                         const float* __restrict__ part, float* __restrict__ emb,
                                                         const float* __restrict__ W0, const float* __restrict__ b0,
                                                         const float* __restrict__ W3, const float* __restrict__ b3,
                                                         const float* __restrict__ Wc, const float* __restrict__ bc,
                                                         float mlp_p, const unsigned long long* __restrict__ seed_ptr,
                                                         unsigned long long site, float* __restrict__ hsave,
                                                         float* __restrict__ gsave, float* __restrict__ fsave,
                                                         float* __restrict__ logits) {
  __shared__ __attribute__((aligned(16))) float eL[2 * XD];
  __shared__ __attribute__((aligned(16))) float hL[256];
  __shared__ __attribute__((aligned(16))) float fL[XD];
  __shared__ float zL;
  const int t = threadIdx.x, b = blockIdx.x, w = t >> 6, lane = t & 63, sub = (lane >> 3) & 7;
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  {  // emb = [v-pool (F2) | a-pool = the F3 tile partials folded in tile order / Ta]
    float val;
    if (t < XD) {
      val = emb[(long)b * 2 * XD + t];
    } else {
      float acc = 0.f;
#pragma unroll
      for (int q = 0; q < F2_KT; ++q) {
        const float x = part[((long)b * ntiles + (q < ntiles ? q : ntiles - 1)) * XD + t - XD];
        acc += q < ntiles ? x : 0.f;
      }
      val = acc / Ta;
      emb[(long)b * 2 * XD + t] = val;
    }
    eL[t] = val;
  }
  __syncthreads();
  // h = dropout(relu(emb W0^T + b0)): wave w takes the 8-row groups w, w + 4, ..., four groups' weight rows in
  // flight at once (a group at a time waited one L2 round trip per 8 rows: 8 per wave at H1 = 256)
  for (int g0 = w; 8 * g0 < H1; g0 += 16) {
    float sv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int g = g0 + 4 * q;
      sv[q] = dot_rows8<4>(W0, 2 * XD, H1, 8 * (8 * g < H1 ? g : g0), eL);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int g = g0 + 4 * q, r = 8 * g + sub;
      if ((lane & 7) == 0 && 8 * g < H1 && r < H1) {
        float hv = sv[q] + b0[r];
        hv = (hv > 0.f ? hv : 0.f) * dropout_scale(seed, (uint64_t)((long)b * H1 + r), mlp_p);
        hL[r] = hv;
        hsave[(long)b * H1 + r] = hv;
      }
    }
  }
  for (int r = H1 + t; r < 256; r += 256) hL[r] = 0.f;  // (H1 % 4 == 0: the k-split reads whole float4)
  __syncthreads();
  if constexpr (!GATED) {  // logits = h W3^T + b3
    for (int g = w; 8 * g < C; g += 4) {
      const float s = dot_rows8<4>(W3, H1, C, 8 * g, hL);
      const int c = 8 * g + sub;
      if ((lane & 7) == 0 && c < C) logits[(long)b * C + c] = s + b3[c];
    }
    return;
  } else {
    if (w == 0) {  // z = h Wg3^T + b, g = sigmoid(z)
      float a = 0.f;
      for (int k = lane; k < H1; k += 64) a = fmaf(hL[k], W3[k], a);
      a = wave_sum(a) + b3[0];
      if (lane == 0) {
        const float gv = 1.f / (1.f + expf(-a));
        zL = gv;
        gsave[b] = gv;
      }
    }
    __syncthreads();
    if (t < XD) {
      const float gv = zL;
      const float f = gv * eL[t] + (1.f - gv) * eL[XD + t];
      fL[t] = f;
      fsave[(long)b * XD + t] = f;
    }
    __syncthreads();
    for (int g = w; 8 * g < C; g += 4) {  // logits = fused Wc^T + bc
      const float s = dot_rows8<2>(Wc, XD, C, 8 * g, fL);
      const int c = 8 * g + sub;
      if ((lane & 7) == 0 && c < C) logits[(long)b * C + c] = s + bc[c];
    }
  }
}

MER_API int mer_xh_mlp_fwd(int B, int Ta, int gated, int H1, int C, const float* part, float* emb, const float* W0,
                           const float* b0, const float* W3, const float* b3, const float* Wc, const float* bc,
                           float mlp_p, const unsigned long long* seed, unsigned long long site, float* hsave,
                           float* gsave, float* fsave, float* logits, void* stream) {
  if (B <= 0) return 0;
  if (H1 <= 0 || H1 > 256 || H1 % 4 || C <= 0 || C > 32 || Ta > 16 * F2_KT || (mlp_p > 0.f && !seed))
    return (int)hipErrorInvalidValue;
  if (gated && (!Wc || !bc || !gsave || !fsave)) return (int)hipErrorInvalidValue;
  const int ntiles = (Ta + 15) / 16;
  if (gated)
    hipLaunchKernelGGL(xh_mlp_fwd_kernel<true>, dim3(B), dim3(256), 0, (hipStream_t)stream, Ta, ntiles, H1, C, part,
                       emb, W0, b0, W3, b3, Wc, bc, mlp_p, seed, site, hsave, gsave, fsave, logits);
  else
    hipLaunchKernelGGL(xh_mlp_fwd_kernel<false>, dim3(B), dim3(256), 0, (hipStream_t)stream, Ta, ntiles, H1, C, part,
                       emb, W0, b0, W3, b3, Wc, bc, mlp_p, seed, site, hsave, gsave, fsave, logits);
  MER_LAUNCH_CHECK();
}
