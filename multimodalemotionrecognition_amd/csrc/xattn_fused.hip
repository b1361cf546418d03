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
//   F1 xh_audio_fwd (grid B*Ta/32 + B*T/32): a_seq(bf16) -> a_s = audio_seq_proj -> a = a_in_proj -> [q2 | k1 v1]
//      (the a2v query projection and the v2a key/value projections share the input a); the trailing blocks
//      project the video rows: v = v_in_proj(v_feat), q1
//   F2 xh_v2a_fwd (grid B): MHA of q1 over the sample's Ta keys -> out-proj ->
//      drop-path + residual + LayerNorm -> v1 -> [k2 v2] (the a2v key/value projections) + mean-pool of v1
//   F3 xh_a2v_fwd (grid B * ceil(Ta/16)): MHA of 16 query rows over the sample's T keys -> out-proj ->
//      drop-path + residual + LayerNorm -> a1, per-tile column sums of a1 (the a-side mean pool)
//   F4 xh_mlp_fwd (grid ceil(B/4)): a-pool fold, concat MLP (or gated head) -> logits, exact fp32 FMA
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
__global__ void xh_split_kernel(const long long* __restrict__ desc) {
  const long long* d = desc + 7 * blockIdx.y;
  const float* src = reinterpret_cast<const float*>(d[0]);
  bf16_t* hi = reinterpret_cast<bf16_t*>(d[1]);
  bf16_t* lo = reinterpret_cast<bf16_t*>(d[2]);
  const long rows = d[3], cols = d[4], n = rows * cols, dld = d[6];
  const bool trans = d[5] != 0;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const float x = src[e];
    const bf16_t h = f2bf(x);
    const long o = trans ? (e % cols) * dld + e / cols : e;
    hi[o] = h;
    lo[o] = f2bf(x - bf2f(h));
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
// F1: audio token chain, 32 rows per block, 4 waves; the trailing ceil(B*T/32) blocks run the video rows'
// input and query projections (v, q1), which depend on nothing the audio chain makes.
// ---------------------------------------------------------------------------------------------
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

template <typename TA>  // bf16: the WavLM features (exact, two passes); float: fp32 features (split, three passes)
__global__ __launch_bounds__(256) void xh_audio_fwd_kernel(int M, int S, const TA* __restrict__ aseq, long ldas,
                                                           SplitW Ws, const float* __restrict__ bs, SplitW Wa,
                                                           const float* __restrict__ ba, SplitW Wc,
                                                           const float* __restrict__ bq2, const float* __restrict__ bkv1,
                                                           float* __restrict__ a_s, float* __restrict__ a,
                                                           float* __restrict__ q2, float* __restrict__ kv1, XhVideo vid) {
  __shared__ __attribute__((aligned(16))) float asL[32 * LDA];
  __shared__ __attribute__((aligned(16))) float aL[32 * LDA];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fk = (lane >> 4) * 8;
  const int na = (M + 31) / 32;
  if ((int)blockIdx.x >= na) {  // video rows: v = v_feat Wv^T + bv, q1 = v Wq1^T + bq1
    const long v0 = (long)(blockIdx.x - na) * 32;
    const int vmax = (int)(vid.M - v0 < 32 ? vid.M - v0 : 32);
    {
      f32x4 acc[2][2];
      zero(acc);
      mm_aw(acc, vid.vfeat + v0 * vid.vdim, vid.vdim, vmax, vid.vdim, vid.Wv, vid.vdim, 32 * w);
      store_acc(acc, 32 * w, vid.bv, asL, LDA, vid.v, XD, v0, vmax);
    }
    __syncthreads();
    f32x4 acc[2][2];
    zero(acc);
    mm_aw(acc, asL, LDA, 32, XD, vid.Wq1, XD, 32 * w);
    store_acc(acc, 32 * w, vid.bq1, nullptr, 0, vid.q1, XD, v0, vmax);
    return;
  }
  XT(2, 0);
  const long r0 = (long)blockIdx.x * 32;
  const int rmax = (int)(M - r0 < 32 ? M - r0 : 32);
  // a_s = a_seq Ws^T + bs  (bf16 A is exact: two passes; fp32 A: split, three passes)
  {
    f32x4 acc[2][2];
    zero(acc);
    const int c0 = 32 * w;
    if constexpr (sizeof(TA) == 2) {  // pipelined like mm_aw, F1_D k steps in flight
      constexpr int F1_D = 4;
      u4 sa[F1_D][2], sb[F1_D][2][2];
      auto load = [&](int k, u4 (&ra)[2], u4 (&rb)[2][2]) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const long off = (long)(c0 + 16 * j + fr) * S + k + fk;
          rb[j][0] = *reinterpret_cast<const u4*>(Ws.hi + off);
          rb[j][1] = *reinterpret_cast<const u4*>(Ws.lo + off);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r = 16 * i + fr;
          ra[i] = *reinterpret_cast<const u4*>(aseq + (r0 + (r < rmax ? r : rmax - 1)) * ldas + k + fk);
        }
      };
      const int nsteps = S / 32;  // branch-free pipeline, as mm_aw
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
      mm_aw(acc, reinterpret_cast<const float*>(aseq) + r0 * ldas, ldas, rmax, S, Ws, S, c0);
    }
    store_acc(acc, c0, bs, asL, LDA, a_s, XD, r0, rmax);
  }
  __syncthreads();
  XT(2, 1);
  {  // a = a_s Wa^T + ba
    f32x4 acc[2][2];
    zero(acc);
    mm_aw(acc, asL, LDA, 32, XD, Wa, XD, 32 * w);
    store_acc(acc, 32 * w, ba, aL, LDA, a, XD, r0, rmax);
  }
  __syncthreads();
  XT(2, 2);
  {  // [q2 | k1 v1] = a Wc^T + [bq2 | bkv1]: 384 columns, 96 per wave
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      f32x4 acc[2][3];
      zero(acc);
      const int c0 = 96 * w + 48 * half;
      mm_aw(acc, aL, LDA, 32, XD, Wc, XD, c0);
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
  }
  XT(2, 3);
}

MER_API int mer_xh_audio_fwd(int M, int S, const void* aseq, int aseq_dtype, long ldas, const void* Ws_hi,
                             const void* Ws_lo, const float* bs, const void* Wa_hi, const void* Wa_lo, const float* ba,
                             const void* Wc_hi, const void* Wc_lo, const float* bq2, const float* bkv1, float* a_s,
                             float* a, float* q2, float* kv1, int Mv, int vdim, const float* vfeat, const void* Wv_hi,
                             const void* Wv_lo, const float* bv, const void* Wq1_hi, const void* Wq1_lo,
                             const float* bq1, float* v, float* q1, void* stream) {
  if (M <= 0 || Mv < 0) return (int)hipErrorInvalidValue;
  if (S % 32 || ldas % 8 || ((uintptr_t)aseq & 15) || (Mv > 0 && (vdim <= 0 || vdim % 32))) return (int)hipErrorInvalidValue;
  const SplitW ws{(const bf16_t*)Ws_hi, (const bf16_t*)Ws_lo}, wa{(const bf16_t*)Wa_hi, (const bf16_t*)Wa_lo},
      wc{(const bf16_t*)Wc_hi, (const bf16_t*)Wc_lo};
  const XhVideo vid{Mv, vdim, vfeat, SplitW{(const bf16_t*)Wv_hi, (const bf16_t*)Wv_lo}, bv,
                    SplitW{(const bf16_t*)Wq1_hi, (const bf16_t*)Wq1_lo}, bq1, v, q1};
  const dim3 grid((M + 31) / 32 + (Mv + 31) / 32);
  if (aseq_dtype == MER_BF16)
    hipLaunchKernelGGL(xh_audio_fwd_kernel<bf16_t>, grid, dim3(256), 0, (hipStream_t)stream, M, S,
                       (const bf16_t*)aseq, ldas, ws, bs, wa, ba, wc, bq2, bkv1, a_s, a, q2, kv1, vid);
  else
    hipLaunchKernelGGL(xh_audio_fwd_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, M, S,
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
                                               float* oL) {
  const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4, fk = fq * 8;
  // S = Q_h K_h^T: A = Q rows (k = head dims), B[n = key][k] = K rows
  f32x4 s[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    bf16x8 ah, al;
    frag_row(Qrows + (long)(i0 + fr < Lq ? fr : Lq - 1 - i0) * ldq + h * XDH + fk, i0 + fr < Lq, ah, al);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int j = 16 * t + fr;
      bf16x8 bh, bl;
      frag_row(Krows + (long)(j < Lk ? j : Lk - 1) * ldkv + h * XDH + fk, j < Lk, bh, bl);
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
      s[t][r] = j < Lk ? s[t][r] * scale : -INFINITY;
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
  constexpr int KP = 16 * NT;  // keys padded to the tile; PV contracts over KP rounded up to 32
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
  // O_h = P' V_h: A = P' (16 x KP32), B[n = head dim][k = key] = V rows (gathered with stride ldkv)
  constexpr int KC = (KP + 31) / 32 * 32;
  f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int k = 0; k < KC; k += 32) {
    bf16x8 ah, al;
    frag_row(PL + fr * pld + k + fk, true, ah, al);
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      bf16x8 bh, bl;
      frag_col(Vrows + (long)(k + fk) * ldkv + h * XDH + 16 * jt + fr, ldkv, k + fk, Lk, bh, bl);
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

// ---------------------------------------------------------------------------------------------
// F2: v2a block, one workgroup per sample (T <= 16 query rows).
// ---------------------------------------------------------------------------------------------
constexpr int F2_KT = 10;                 // Ta <= 160 keys
constexpr int F2_PLD = 16 * F2_KT + 20;   // P' tile stride (>= 32-padded keys)

__global__ __launch_bounds__(256) void xh_v2a_fwd_kernel(
    int T, int Ta, const float* __restrict__ v, const float* __restrict__ q1, const float* __restrict__ kv1,
    SplitW Wo1, const float* __restrict__ bo1, const float* __restrict__ gamma, const float* __restrict__ beta,
    SplitW Wkv2, const float* __restrict__ bkv2, XhDrop dr, float scale, float* __restrict__ P1,
    float* __restrict__ o1, float* __restrict__ s_v, float* __restrict__ mean_v, float* __restrict__ rstd_v,
    float* __restrict__ v1, float* __restrict__ kv2, float* __restrict__ emb, long ld_emb) {
  extern __shared__ __attribute__((aligned(16))) float f2smem[];  // F2_LDS_BYTES
  float* vL = f2smem;
  float* qL = vL + 16 * LDA;
  float* oL = qL + 16 * LDA;
  float* PL = oL + 16 * LDA;  // [XH][16][F2_PLD]
  float* tL = PL;             // the out-projection tile reuses P' once the attention is done
  const int b = blockIdx.x, w = threadIdx.x >> 6;
  const long row0 = (long)b * T;
  const unsigned long long seed_attn = mer_site_seed(dr.seed, dr.site_attn);
  const unsigned long long seed_path = mer_site_seed(dr.seed, dr.site_path);
#pragma unroll
  for (int e = threadIdx.x; e < 16 * XD; e += 256) {  // v, q1 (F1's video blocks)
    const int r = e / XD, c = e - r * XD;
    const long rc = row0 + (r < T ? r : T - 1);
    const float xv = v[rc * XD + c], xq = q1[rc * XD + c];
    vL[r * LDA + c] = r < T ? xv : 0.f;
    qL[r * LDA + c] = r < T ? xq : 0.f;
  }
  XT(3, 0);
  __syncthreads();
  XT(3, 1);
  // attention: wave w = head w, keys = this sample's Ta rows of kv1 (k | v)
  head_attention<F2_KT>(b, w, 0, T, Ta, qL, LDA, kv1 + (long)b * Ta * 2 * XD, kv1 + (long)b * Ta * 2 * XD + XD, 2 * XD,
                        scale, P1, dr.attn, seed_attn, PL + w * 16 * F2_PLD, F2_PLD, oL);
  __syncthreads();
  XT(3, 2);
  for (int e = threadIdx.x; e < T * XD; e += 256) o1[row0 * XD + e] = oL[(e / XD) * LDA + e % XD];
  {  // v2 = o Wo1^T + bo1
    f32x4 acc[1][2];
    zero(acc);
    mm_aw(acc, oL, LDA, 16, XD, Wo1, XD, 32 * w);
    store_acc(acc, 32 * w, bo1, tL, LDA, nullptr, 0, 0, 16);
  }
  __syncthreads();
  XT(3, 3);
  // v1 = LN(v + keep_b * v2)  (StochasticDepth: one keep draw per sample, fusion.py:11-26)
  add_ln_rows(T, vL, tL, dropout_scale(seed_path, b, dr.path), gamma, beta, qL, s_v, mean_v, rstd_v, row0);
  __syncthreads();
  for (int e = threadIdx.x; e < T * XD; e += 256) v1[row0 * XD + e] = qL[(e / XD) * LDA + e % XD];
  for (int e = threadIdx.x; e < (16 - T) * XD; e += 256) qL[(T + e / XD) * LDA + e % XD] = 0.f;
  if (threadIdx.x < XD) {  // mean temporal pool of v1 (temporal.py:108-109) -> emb[b, 0:d]
    float s = 0.f;
    for (int r = 0; r < T; ++r) s += qL[r * LDA + threadIdx.x];
    emb[(long)b * ld_emb + threadIdx.x] = s / T;
  }
  __syncthreads();
  {  // [k2 v2] = v1 Wkv2^T + bkv2: 256 columns, 64 per wave
    f32x4 acc[1][4];
    zero(acc);
    mm_aw(acc, qL, LDA, 16, XD, Wkv2, XD, 64 * w);
    store_acc(acc, 64 * w, bkv2, nullptr, 0, kv2, 2 * XD, row0, T);
  }
  XT(3, 4);
}

constexpr size_t F2_LDS_BYTES = sizeof(float) * (3 * 16 * LDA + XH * 16 * F2_PLD);

MER_API int mer_xh_v2a_fwd(int B, int T, int Ta, const float* v, const float* q1, const float* kv1, const void* Wo1_hi,
                           const void* Wo1_lo, const float* bo1, const float* gamma, const float* beta,
                           const void* Wkv2_hi, const void* Wkv2_lo, const float* bkv2, float attn_p, float path_p,
                           const unsigned long long* seed, unsigned long long site_attn, unsigned long long site_path,
                           float scale, float* P1, float* o1, float* s_v, float* mean_v, float* rstd_v, float* v1,
                           float* kv2, float* emb, long ld_emb, void* stream) {
  if (B <= 0) return 0;
  if (T <= 0 || T > 16 || Ta <= 0 || Ta > 16 * F2_KT) return (int)hipErrorInvalidValue;
  if ((attn_p > 0.f || path_p > 0.f) && !seed) return (int)hipErrorInvalidValue;
  XhDrop dr{attn_p, path_p, seed, site_attn, site_path};
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&xh_v2a_fwd_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)F2_LDS_BYTES) != hipSuccess)
    return (int)hipErrorInvalidConfiguration;
  hipLaunchKernelGGL(xh_v2a_fwd_kernel, dim3(B), dim3(256), F2_LDS_BYTES, (hipStream_t)stream, T, Ta, v, q1, kv1,
                     SplitW{(const bf16_t*)Wo1_hi, (const bf16_t*)Wo1_lo}, bo1, gamma, beta,
                     SplitW{(const bf16_t*)Wkv2_hi, (const bf16_t*)Wkv2_lo}, bkv2, dr, scale, P1, o1, s_v, mean_v,
                     rstd_v, v1, kv2, emb, ld_emb);
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
                                                         float* __restrict__ part) {
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
  head_attention<1>(b, w, i0, Ta, T, q2 + row0 * XD, XD, kv2 + (long)b * T * 2 * XD, kv2 + (long)b * T * 2 * XD + XD,
                    2 * XD, scale, P2, dr.attn, seed_attn, PL + w * 16 * F3_PLD, F3_PLD, oL);
#pragma unroll
  for (int e = threadIdx.x; e < 16 * XD; e += 256) {
    const int r = e / XD, c = e - r * XD;
    const float x = a[(row0 + (r < nr ? r : nr - 1)) * XD + c];
    aL[r * LDA + c] = r < nr ? x : 0.f;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < nr * XD; e += 256) o2[row0 * XD + e] = oL[(e / XD) * LDA + e % XD];
  {  // a2 = o Wo2^T + bo2
    f32x4 acc[1][2];
    zero(acc);
    mm_aw(acc, oL, LDA, 16, XD, Wo2, XD, 32 * w);
    store_acc(acc, 32 * w, bo2, tL, LDA, nullptr, 0, 0, 16);
  }
  __syncthreads();
  add_ln_rows(nr, aL, tL, dropout_scale(seed_path, b, dr.path), gamma, beta, oL, s_a, mean_a, rstd_a, row0);
  __syncthreads();
  if (threadIdx.x < XD) {  // this tile's column sums of a1 (the a-side mean pool, folded in tile order by F4)
    float s = 0.f;
    for (int r = 0; r < nr; ++r) s += oL[r * LDA + threadIdx.x];
    part[((long)b * ntiles + tile) * XD + threadIdx.x] = s;
  }
}

MER_API int mer_xh_a2v_fwd(int B, int T, int Ta, const float* q2, const float* kv2, const float* a, const void* Wo2_hi,
                           const void* Wo2_lo, const float* bo2, const float* gamma, const float* beta, float attn_p,
                           float path_p, const unsigned long long* seed, unsigned long long site_attn,
                           unsigned long long site_path, float scale, float* P2, float* o2, float* s_a, float* mean_a,
                           float* rstd_a, float* part, void* stream) {
  if (B <= 0) return 0;
  if (T <= 0 || T > 16 || Ta <= 0) return (int)hipErrorInvalidValue;
  if ((attn_p > 0.f || path_p > 0.f) && !seed) return (int)hipErrorInvalidValue;
  const int ntiles = (Ta + 15) / 16;
  XhDrop dr{attn_p, path_p, seed, site_attn, site_path};
  hipLaunchKernelGGL(xh_a2v_fwd_kernel, dim3(B * ntiles), dim3(256), 0, (hipStream_t)stream, T, Ta, ntiles, q2, kv2,
                     a, SplitW{(const bf16_t*)Wo2_hi, (const bf16_t*)Wo2_lo}, bo2, gamma, beta, dr, scale, P2, o2, s_a,
                     mean_a, rstd_a, part);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// F4: a-pool fold + classifier head (fusion.py:404-411), 4 samples per workgroup, exact fp32 FMA.
//   concat: h = dropout(relu(emb W0^T + b0)), logits = h W3^T + b3
//   gated:  h = dropout(relu(emb Wg0^T + b)), z = h Wg3^T + b, g = sigmoid(z),
//           fused = g v_emb + (1 - g) a_emb, logits = fused Wc^T + bc
// ---------------------------------------------------------------------------------------------
constexpr int F4_KC = 32;  // W0 k-chunk staged in LDS

__global__ __launch_bounds__(256) void xh_mlp_fwd_kernel(int B, int Ta, int ntiles, int gated, int H1, int C,
                                                         const float* __restrict__ part, float* __restrict__ emb,
                                                         const float* __restrict__ W0, const float* __restrict__ b0,
                                                         const float* __restrict__ W3, const float* __restrict__ b3,
                                                         const float* __restrict__ Wc, const float* __restrict__ bc,
                                                         float mlp_p, const unsigned long long* __restrict__ seed_ptr,
                                                         unsigned long long site, float* __restrict__ hsave,
                                                         float* __restrict__ gsave, float* __restrict__ fsave,
                                                         float* __restrict__ logits) {
  __shared__ float eL[4][2 * XD];
  __shared__ float hL[4][256];
  __shared__ float wL[256 * (F4_KC + 1)];  // W0[:, k0 : k0 + 32], row stride 33 (conflict-free column reads)
  __shared__ float zL[4];
  const int t = threadIdx.x, s0 = blockIdx.x * 4, w = t >> 6, lane = t & 63;
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
#pragma unroll
  for (int e = t; e < 4 * 2 * XD; e += 256) {
    const int s = e / (2 * XD), c = e - s * 2 * XD, bb = s0 + s;
    float val = 0.f;
    if (bb < B) {
      if (c < XD) {
        val = emb[(long)bb * 2 * XD + c];
      } else {
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < F2_KT; ++q) {
          const float x = part[((long)bb * ntiles + (q < ntiles ? q : ntiles - 1)) * XD + c - XD];
          acc += q < ntiles ? x : 0.f;
        }
        val = acc / Ta;
        emb[(long)bb * 2 * XD + c] = val;
      }
    }
    eL[s][c] = val;
  }
  // h = relu(emb W0^T + b0): thread t = output t for the 4 samples, W0 staged 32 columns at a time; the next
  // chunk's loads (thread t: column t & 31 of rows t / 32 + 8 i) are in flight while this chunk is consumed
  float acc[4];
  for (int s = 0; s < 4; ++s) acc[s] = t < H1 ? b0[t] : 0.f;
  float pre[256 / 8];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 256 / 8; ++i) {
      const int r = (t >> 5) + 8 * i;
      const float x = W0[(long)(r < H1 ? r : H1 - 1) * 2 * XD + k0 + (t & 31)];
      pre[i] = r < H1 ? x : 0.f;
    }
  };
  load(0);
  for (int k0 = 0; k0 < 2 * XD; k0 += F4_KC) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 256 / 8; ++i) wL[((t >> 5) + 8 * i) * (F4_KC + 1) + (t & 31)] = pre[i];
    __syncthreads();
    if (k0 + F4_KC < 2 * XD) load(k0 + F4_KC);
    if (t < H1) {
#pragma unroll 8
      for (int kk = 0; kk < F4_KC; ++kk) {
        const float wv = wL[t * (F4_KC + 1) + kk];
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[s] = fmaf(eL[s][k0 + kk], wv, acc[s]);
      }
    }
  }
  if (t < H1) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int bb = s0 + s;
      float hv = acc[s] > 0.f ? acc[s] : 0.f;
      if (bb < B) {
        hv *= dropout_scale(seed, (uint64_t)((long)bb * H1 + t), mlp_p);
        hsave[(long)bb * H1 + t] = hv;
      }
      hL[s][t] = hv;
    }
  }
  __syncthreads();
  if (!gated) {  // logits: one wave per (sample, class) dot over H1
    for (int o = w; o < 4 * C; o += 4) {
      const int s = o / C, c = o - s * C, bb = s0 + s;
      float a = 0.f;
      for (int k = lane; k < H1; k += 64) a = fmaf(hL[s][k], W3[(long)c * H1 + k], a);
      a = wave_sum(a);
      if (lane == 0 && bb < B) logits[(long)bb * C + c] = a + b3[c];
    }
    return;
  }
  {  // z = h Wg3^T + b (one output per sample, wave s), g = sigmoid(z)
    const int s = w, bb = s0 + s;
    float a = 0.f;
    for (int k = lane; k < H1; k += 64) a = fmaf(hL[s][k], W3[k], a);
    a = wave_sum(a) + b3[0];
    const float g = 1.f / (1.f + expf(-a));
    if (lane == 0) {
      zL[s] = g;
      if (bb < B) gsave[bb] = g;
    }
  }
  __syncthreads();
  for (int e = t; e < 4 * XD; e += 256) {
    const int s = e / XD, c = e - s * XD, bb = s0 + s;
    const float g = zL[s];
    const float f = g * eL[s][c] + (1.f - g) * eL[s][XD + c];
    hL[s][c] = f;  // h no longer needed
    if (bb < B) fsave[(long)bb * XD + c] = f;
  }
  __syncthreads();
  for (int o = w; o < 4 * C; o += 4) {
    const int s = o / C, c = o - s * C, bb = s0 + s;
    float a = 0.f;
    for (int k = lane; k < XD; k += 64) a = fmaf(hL[s][k], Wc[(long)c * XD + k], a);
    a = wave_sum(a);
    if (lane == 0 && bb < B) logits[(long)bb * C + c] = a + bc[c];
  }
}

MER_API int mer_xh_mlp_fwd(int B, int Ta, int gated, int H1, int C, const float* part, float* emb, const float* W0,
                           const float* b0, const float* W3, const float* b3, const float* Wc, const float* bc,
                           float mlp_p, const unsigned long long* seed, unsigned long long site, float* hsave,
                           float* gsave, float* fsave, float* logits, void* stream) {
  if (B <= 0) return 0;
  if (H1 <= 0 || H1 > 256 || C <= 0 || 4 * C > 256 || Ta > 16 * F2_KT || (mlp_p > 0.f && !seed))
    return (int)hipErrorInvalidValue;
  if (gated && (!Wc || !bc || !gsave || !fsave || H1 > 256)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(xh_mlp_fwd_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, B, Ta, (Ta + 15) / 16,
                     gated, H1, C, part, emb, W0, b0, W3, b3, Wc, bc, mlp_p, seed, site, hsave, gsave, fsave, logits);
  MER_LAUNCH_CHECK();
}
