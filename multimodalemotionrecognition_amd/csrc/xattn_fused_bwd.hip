// Fused xattn head backward: the reverse of xattn_fused.hip (fusion.py:366-411 + the two nn.MultiheadAttention
// blocks, TORCH:6576-6606) on split-bf16 MFMA.  Four data-gradient launches plus one grouped weight-gradient
// launch and its fixed-order fold replace the ~25 backward launches of xattn_head.head_backward:
//   G4 xh_mlp_bwd   (grid B): classifier head -> dh (dz), demb (exact fp32 FMA); its weight gradients go to W
//   G3 xh_a2v_bwd   (grid B * ceil(Ta/16)): a-pool / LayerNorm / out-proj / attention backward of 16 query rows
//                   -> da (LN residual part), da2, dq2, per-tile partials of dK2 dV2 and of dgamma / dbeta
//   G2 xh_v2a_bwd   (grid B): dK2 dV2 fold -> dv1 -> LayerNorm / out-proj / attention backward over the
//                   sample's Ta keys -> dq1, dK1 dV1 and the residual part of dv
//   G1 xh_audio_bwd (grid B*Ta/32 + B*T/32): da += [dq2 | dK1 dV1] . [Wq2 ; Wkv1], da_s = da . Wa; the trailing
//                   blocks: dv += dq1 . Wq1, dv_feat = dv . Wv (the ResNet18 trunk's input gradient)
//   W  xh_wgrad + xh_wfold: every dW = dY^T X and bias / LayerNorm-affine gradient as ONE grouped launch of
//      (problem, 64 x 64 tile, row split) blocks writing partials, folded in split order (deterministic, no
//      atomics) and added into the caller's gradient buffers
// Dropout / drop-path / attention-dropout masks are regenerated from the forward's (seed, site, index).
// Data-gradient products read the TRANSPOSED split planes ([in][out]) that mer_xh_split writes (trans = 1).
#include "common.h"
#include "mer.h"
#include "xattn_common.h"

using namespace xh;

namespace {

// LayerNorm backward of one 128-wide row, wave-wide: dy = (dy0, dy1) at columns (lane, 64 + lane).  Returns
// d(pre-LN sum) in (ds0, ds1) and accumulates the row's dgamma / dbeta terms into (g0, g1, bb0, bb1).
__device__ __forceinline__ void ln_row_bwd(float dy0, float dy1, const float* srow, float mean, float rstd,
                                           const float* gamma, float& ds0, float& ds1, float& g0, float& g1,
                                           float& bb0, float& bb1) {
  const int lane = threadIdx.x & 63;
  const float xh0 = (srow[lane] - mean) * rstd, xh1 = (srow[64 + lane] - mean) * rstd;
  const float gg0 = gamma[lane] * dy0, gg1 = gamma[64 + lane] * dy1;
  const float a = wave_sum(gg0 + gg1) / XD;
  const float bs = wave_sum(gg0 * xh0 + gg1 * xh1) / XD;
  ds0 = rstd * (gg0 - a - xh0 * bs);
  ds1 = rstd * (gg1 - a - xh1 * bs);
  g0 += dy0 * xh0;
  g1 += dy1 * xh1;
  bb0 += dy0;
  bb1 += dy1;
}

// per-wave (g0 g1 b0 b1) -> block sums in wave order -> part[0:128] = dgamma, part[128:256] = dbeta
__device__ __forceinline__ void ln_part_store(float g0, float g1, float b0, float b1, float* red, float* part) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  red[w * 256 + lane] = g0;
  red[w * 256 + 64 + lane] = g1;
  red[w * 256 + 128 + lane] = b0;
  red[w * 256 + 192 + lane] = b1;
  lds_sync();
  if (threadIdx.x < 256) {
    float s = 0.f;
    for (int q = 0; q < 4; ++q) s += red[q * 256 + threadIdx.x];
    part[threadIdx.x] = s;
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// G4: classifier head backward, ONE sample per workgroup (the data gradients only; the head's weight and bias
// gradients dW0 = dh^T emb, dW3 = dl^T h (gated: dWg3 = dz^T h, dWc = dl^T fused) are problems of the grouped
// W launch, which runs after G1).  Unfused: xattn_head.py:207-225.
//   concat: dh = relu' . dropout' . (dl W3),                   demb = dh W0
//   gated:  dfused = dl Wc, dz = sum_c dfused (v - a) g (1 - g), dh = relu' . dropout' . dz Wg3,
//           demb = dh Wg0 + [g dfused | (1 - g) dfused]
// demb = W0^T dh runs with the 256 emb columns across the lanes (one coalesced 1 KB row load per wave and row,
// 16 rows in flight) and the rows split over the 4 waves, folded in wave order.  Exact fp32 FMA.
// ---------------------------------------------------------------------------------------------
template <bool GATED>
__global__ __launch_bounds__(256) void xh_mlp_bwd_kernel(int C, int H1, const float* __restrict__ dl,
                                                         const float* __restrict__ emb, const float* __restrict__ h,
                                                         const float* __restrict__ gsave, const float* __restrict__ W0,
                                                         const float* __restrict__ W3, const float* __restrict__ Wc,
                                                         float mlp_p, const unsigned long long* __restrict__ seed_ptr,
                                                         unsigned long long site, float* __restrict__ dh_out,
                                                         float* __restrict__ dz_out, float* __restrict__ demb) {
  __shared__ float dlL[32];
  __shared__ __attribute__((aligned(16))) float dhL[256];
  __shared__ float dfL[XD];
  __shared__ float red[4][2 * XD];
  __shared__ float dzL;
  const int t = threadIdx.x, b = blockIdx.x, w = t >> 6, lane = t & 63;
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  if (t < C) dlL[t] = dl[(long)b * C + t];
  __syncthreads();
  float gv = 0.f;
  if constexpr (GATED) {
    gv = gsave[b];
    if (t < XD) {  // dfused = dl Wc  ([C][128])
      float acc = 0.f;
      for (int q = 0; q < C; ++q) acc = fmaf(dlL[q], Wc[(long)q * XD + t], acc);
      dfL[t] = acc;
    }
    __syncthreads();
    if (w < 2) {  // dz over the 128 columns (waves 0, 1), folded in wave order
      const int c = 64 * w + lane;
      const float x = dfL[c] * (emb[(long)b * 2 * XD + c] - emb[(long)b * 2 * XD + XD + c]);
      const float s = wave_sum(x);
      if (lane == 0) red[0][w] = s;
    }
    __syncthreads();
    if (t == 0) {
      const float dz = (red[0][0] + red[0][1]) * gv * (1.f - gv);
      dzL = dz;
      dz_out[b] = dz;
    }
    __syncthreads();
  }
  // dh (thread = hidden unit); h is the saved post-dropout activation: relu' . dropout' = (h > 0) * mask scale
  for (int r = t; r < 256; r += 256) {
    float dhv = 0.f;
    if (r < H1) {
      float acc;
      if constexpr (GATED) {
        acc = dzL * W3[r];
      } else {
        acc = 0.f;
        for (int q = 0; q < C; ++q) acc = fmaf(dlL[q], W3[(long)q * H1 + r], acc);
      }
      const float hv = h[(long)b * H1 + r];
      dhv = hv > 0.f ? acc * dropout_scale(seed, (uint64_t)((long)b * H1 + r), mlp_p) : 0.f;
      dh_out[(long)b * H1 + r] = dhv;
    }
    dhL[r] = dhv;
  }
  __syncthreads();
  {  // demb partial of this wave's rows: column 4 * lane .. + 3
    const int per = (H1 + 3) / 4, r0 = w * per, r1 = r0 + per < H1 ? r0 + per : H1;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int U = 16;
    for (int rb = r0; rb < r1; rb += U) {
      f32x4 wv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = rb + u < r1 ? rb + u : r1 - 1;
        wv[u] = *reinterpret_cast<const f32x4*>(W0 + (long)r * 2 * XD + 4 * lane);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float d = rb + u < r1 ? dhL[rb + u] : 0.f;
        acc[0] = fmaf(d, wv[u][0], acc[0]);
        acc[1] = fmaf(d, wv[u][1], acc[1]);
        acc[2] = fmaf(d, wv[u][2], acc[2]);
        acc[3] = fmaf(d, wv[u][3], acc[3]);
      }
    }
    *reinterpret_cast<f32x4*>(&red[w][4 * lane]) = acc;
  }
  __syncthreads();
  {
    float s = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
    if constexpr (GATED) s += t < XD ? dfL[t] * gv : dfL[t - XD] * (1.f - gv);
    demb[(long)b * 2 * XD + t] = s;
  }
}

MER_API int mer_xh_mlp_bwd(int B, int C, int H1, int gated, const float* dlogits, const float* emb, const float* h,
                           const float* g, const float* W0, const float* W3, const float* Wc, float mlp_p,
                           const unsigned long long* seed, unsigned long long site, float* dh, float* dz, float* demb,
                           void* stream) {
  if (B <= 0) return 0;
  if (H1 <= 0 || H1 > 256 || C <= 0 || C > 32 || (mlp_p > 0.f && !seed) || !dh || !demb ||
      (gated && (!Wc || !g || !dz)))
    return (int)hipErrorInvalidValue;
  if (gated)
    hipLaunchKernelGGL(xh_mlp_bwd_kernel<true>, dim3(B), dim3(256), 0, (hipStream_t)stream, C, H1, dlogits, emb, h, g,
                       W0, W3, Wc, mlp_p, seed, site, dh, dz, demb);
  else
    hipLaunchKernelGGL(xh_mlp_bwd_kernel<false>, dim3(B), dim3(256), 0, (hipStream_t)stream, C, H1, dlogits, emb, h, g,
                       W0, W3, Wc, mlp_p, seed, site, dh, dz, demb);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// G3: a2v block backward, one workgroup per (sample, 16 query rows), wave = head.  Unfused: xattn_head.py:237-252
// ---------------------------------------------------------------------------------------------
constexpr int G3_TLD = 36;  // per-head 16 x 32 LDS tiles (dS, P'), keys padded to the MFMA K of 32

__global__ __launch_bounds__(256) void xh_a2v_bwd_kernel(
    int T, int Ta, int ntiles, const float* __restrict__ demb, const float* __restrict__ s_a,
    const float* __restrict__ mean_a, const float* __restrict__ rstd_a, const float* __restrict__ gamma,
    const float* __restrict__ P2, const float* __restrict__ kv2, const float* __restrict__ q2, SplitW WoT2, XhDrop dr,
    float scale, float* __restrict__ da, float* __restrict__ da2, float* __restrict__ dqkv,
    float* __restrict__ dkv2_part, float* __restrict__ ln_part, float* __restrict__ dbias) {
  __shared__ __attribute__((aligned(16))) float d2L[16 * LDA];
  __shared__ __attribute__((aligned(16))) float oL[16 * LDA];
  __shared__ __attribute__((aligned(16))) float tiles[XH * 2 * 16 * G3_TLD];
  __shared__ float red[4 * 256];
  XT(3, 0);
  const int b = blockIdx.x / ntiles, tile = blockIdx.x - b * ntiles, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int fr = lane & 15, fq = lane >> 4, fk = fq * 8;
  const int i0 = tile * 16, nr = Ta - i0 < 16 ? Ta - i0 : 16;
  const long row0 = (long)b * Ta + i0;
  const unsigned long long seed_attn = mer_site_seed(dr.seed, dr.site_attn);
  const unsigned long long seed_path = mer_site_seed(dr.seed, dr.site_path);
  const float keep = dropout_scale(seed_path, b, dr.path);
  WRegs<XD / 32, 2> wo;  // do2's weight fragments first: their latency overlaps the LayerNorm backward
  wregs_load(wo, WoT2, XD, 32 * w, XD / 32);
  {  // a-pool (mean over Ta) + LayerNorm backward; da = ds (residual), da2 = keep * ds
    float g0 = 0.f, g1 = 0.f, b0 = 0.f, b1 = 0.f;
    const float dy0 = demb[(long)b * 2 * XD + XD + lane] / Ta, dy1 = demb[(long)b * 2 * XD + XD + 64 + lane] / Ta;
    for (int r = w; r < 16; r += 4) {
      float ds0 = 0.f, ds1 = 0.f;
      if (r < nr) {
        const long gr = row0 + r;
        ln_row_bwd(dy0, dy1, s_a + gr * XD, mean_a[gr], rstd_a[gr], gamma, ds0, ds1, g0, g1, b0, b1);
        da[gr * XD + lane] = ds0;
        da[gr * XD + 64 + lane] = ds1;
        da2[gr * XD + lane] = keep * ds0;
        da2[gr * XD + 64 + lane] = keep * ds1;
      }
      d2L[r * LDA + lane] = keep * ds0;
      d2L[r * LDA + 64 + lane] = keep * ds1;
    }
    ln_part_store(g0, g1, b0, b1, red, ln_part + (long)blockIdx.x * 256);
  }
  lds_sync();
  {  // do2 = da2 . Wo2
    f32x4 acc[1][2];
    zero(acc);
    mm_lw<1, 2, XD / 32>(acc, d2L, LDA, wo);
    store_acc(acc, 32 * w, nullptr, oL, LDA, nullptr, 0, 0, 16);
  }
  lds_sync();
  XT(3, 1);
  // attention backward of head h = w over the sample's T keys
  const int h = w;
  float* dSt = tiles + (h * 2) * 16 * G3_TLD;
  float* Pdt = dSt + 16 * G3_TLD;
  const float* kb = kv2 + (long)b * T * 2 * XD;
  f32x4 dp = f32x4{0.f, 0.f, 0.f, 0.f};
  {  // dP' = do2_h . V2_h^T
    bf16x8 ah, al, bh, bl;
    frag_row(oL + fr * LDA + h * XDH + fk, true, ah, al);
    frag_row(kb + (long)(fr < T ? fr : T - 1) * 2 * XD + XD + h * XDH + fk, fr < T, bh, bl);
    dp = mma3(ah, al, bh, bl, dp);
  }
  float pv[4], rs[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * fq + r, j = fr;
    const bool ok = (4 * fq + r) < nr && j < T;
    const long pi = (((long)b * XH + h) * Ta + i) * T + j;
    const long pc = (((long)b * XH + h) * Ta + (ok ? i : i0)) * T + (ok ? j : 0);  // always in range
    const float m = ok ? dropout_scale(seed_attn, pi, dr.attn) : 0.f;
    const float pl = P2[pc];
    pv[r] = ok ? pl : 0.f;
    dp[r] *= m;  // dP
    Pdt[(4 * fq + r) * G3_TLD + j] = pv[r] * m;
    rs[r] = pv[r] * dp[r];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) rs[r] += __shfl_xor(rs[r], o, 64);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    dSt[(4 * fq + r) * G3_TLD + fr] = pv[r] * (dp[r] - rs[r]);
    dSt[(4 * fq + r) * G3_TLD + 16 + fr] = 0.f;  // key pad 16..31
  }
  wave_sync_lds();
  {  // dq2_h = dS . K2_h * scale -> dqkv[:, h * 32 ..]
    f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    bf16x8 ah, al;
    frag_row(dSt + fr * G3_TLD + fk, true, ah, al);
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      bf16x8 bh, bl;
      frag_col(kb + (long)fk * 2 * XD + h * XDH + 16 * jt + fr, 2 * XD, fk, T, bh, bl);
      o[jt] = mma3(ah, al, bh, bl, o[jt]);
    }
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = 4 * fq + r;
        if (rr < nr) dqkv[(row0 + rr) * 3 * XD + h * XDH + 16 * jt + fr] = o[jt][r] * scale;
      }
  }
  {  // dK2_h = dS^T . q2_h * scale, dV2_h = P'^T . do2_h: rows = keys, contraction over this tile's 16 rows
    f32x4 dk[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    f32x4 dv[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    bf16x8 sh, sl, ph, pl;
    frag_col(dSt + (long)fk * G3_TLD + fr, G3_TLD, fk, 16, sh, sl);
    frag_col(Pdt + (long)fk * G3_TLD + fr, G3_TLD, fk, 16, ph, pl);
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      bf16x8 qh, ql, gh, gl;
      frag_col(q2 + (row0 + fk) * XD + h * XDH + 16 * jt + fr, XD, fk, nr, qh, ql);
      frag_col(oL + fk * LDA + h * XDH + 16 * jt + fr, LDA, fk, 16, gh, gl);
      dk[jt] = mma3(sh, sl, qh, ql, dk[jt]);
      dv[jt] = mma3(ph, pl, gh, gl, dv[jt]);
    }
    float* pt = dkv2_part + ((long)b * ntiles + tile) * 16 * 2 * XD;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = 4 * fq + r;
        pt[j * 2 * XD + h * XDH + 16 * jt + fr] = dk[jt][r] * scale;
        pt[j * 2 * XD + XD + h * XDH + 16 * jt + fr] = dv[jt][r];
      }
  }
  XT(3, 2);
  if (dbias) {  // the prior bias gradient: dS summed over the heads in head order (mha_dbias_kernel's order)
    __syncthreads();
    for (int e = threadIdx.x; e < nr * T; e += 256) {
      const int i = e / T, j = e - i * T;
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < XH; ++q) s += tiles[(q * 2) * 16 * G3_TLD + i * G3_TLD + j];
      dbias[((long)b * Ta + i0 + i) * T + j] = s;
    }
  }
  XT(3, 3);
}

MER_API int mer_xh_a2v_bwd(int B, int T, int Ta, const float* demb, const float* s_a, const float* mean_a,
                           const float* rstd_a, const float* gamma, const float* P2, const float* kv2, const float* q2,
                           const void* WoT2_hi, const void* WoT2_lo, float attn_p, float path_p,
                           const unsigned long long* seed, unsigned long long site_attn, unsigned long long site_path,
                           float scale, float* da, float* da2, float* dqkv, float* dkv2_part, float* ln_part,
                           float* dbias, void* stream) {
  if (B <= 0) return 0;
  if (T <= 0 || T > 16 || Ta <= 0 || ((attn_p > 0.f || path_p > 0.f) && !seed)) return (int)hipErrorInvalidValue;
  const int ntiles = (Ta + 15) / 16;
  XhDrop dr{attn_p, path_p, seed, site_attn, site_path};
  hipLaunchKernelGGL(xh_a2v_bwd_kernel, dim3(B * ntiles), dim3(256), 0, (hipStream_t)stream, T, Ta, ntiles, demb, s_a,
                     mean_a, rstd_a, gamma, P2, kv2, q2, SplitW{(const bf16_t*)WoT2_hi, (const bf16_t*)WoT2_lo}, dr,
                     scale, da, da2, dqkv, dkv2_part, ln_part, dbias);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// G2: v2a block backward as two launches (xattn_head.py:252-269 + the v-pool half of 229-231).
// G2a, one workgroup per sample: dkv2 = the a2v tiles' dK2 dV2 partials summed in tile order, dv1 = dkv2 Wkv2 +
// v-pool gradient, LayerNorm backward (dv = its residual part, dv2 = keep * ds, dgamma / dbeta partials),
// do1 = dv2 Wo1 (to global: G2b reads it).
// G2b, one workgroup per (sample, head) (128 at B = 32; the one-workgroup-per-sample version ran 32): the
// attention backward of head h, wave w owning the 32-key chunks c = w, w + 4, ...: dP' = do1_h V_h^T, the row sums
// sum_j P dP meet in LDS (wave order), dS = P (dP - rowsum), dq1_h = dS K_h (per-wave partials summed in wave
// order), dK1 / dV1 rows of the wave's keys into dqkv[:, 128:384].
// ---------------------------------------------------------------------------------------------
constexpr int G2_KT = 10;  // 16-key tiles of one sample's keys the dkv2 fold reads (Ta <= 160 in G2a's fold)
constexpr int G2_KVLD = 2 * XD + 4;
constexpr int G2B_TLD = 36;

__global__ __launch_bounds__(256) void xh_v2a_pre_bwd_kernel(
    int T, int ntiles, const float* __restrict__ dkv2_part, SplitW WkvT2, const float* __restrict__ demb,
    const float* __restrict__ s_v, const float* __restrict__ mean_v, const float* __restrict__ rstd_v,
    const float* __restrict__ gamma, SplitW WoT1, XhDrop dr, float* __restrict__ dkv2, float* __restrict__ dv2,
    float* __restrict__ dv, float* __restrict__ do1, float* __restrict__ ln_part) {
  __shared__ __attribute__((aligned(16))) float kvL[16 * G2_KVLD];  // dK2 dV2
  __shared__ __attribute__((aligned(16))) float t1[16 * LDA];       // dv1, then ds
  __shared__ __attribute__((aligned(16))) float d2L[16 * LDA];      // dv2
  __shared__ float red[4 * 256];
  const int b = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long row0 = (long)b * T;
  const unsigned long long seed_path = mer_site_seed(dr.seed, dr.site_path);
  const float keep = dropout_scale(seed_path, b, dr.path);
  // both products' weight fragments first (registers): their latency overlaps the fold below
  WRegs<2 * XD / 32, 2> wkv;
  wregs_load(wkv, WkvT2, 2 * XD, 32 * w, 2 * XD / 32);
  WRegs<XD / 32, 2> wo;
  wregs_load(wo, WoT1, XD, 32 * w, XD / 32);
  // dK2 dV2 of this sample: the a2v tiles' partials summed in tile order; thread = one of the 256 columns, rows
  // in groups of 8 with every load of a group in flight at once (T is block-uniform: whole groups are skipped)
  {
    const int c = threadIdx.x;
#pragma unroll
    for (int rb = 0; rb < 16; rb += 8) {
      if (rb < T) {
        float x[8][G2_KT];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int q = 0; q < G2_KT; ++q) {
            const int rc = rb + i < T ? rb + i : T - 1, qc = q < ntiles ? q : ntiles - 1;
            x[i][q] = dkv2_part[(((long)b * ntiles + qc) * 16 + rc) * 2 * XD + c];
          }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int r = rb + i;
          float sum = 0.f;
#pragma unroll
          for (int q = 0; q < G2_KT; ++q) sum += q < ntiles ? x[i][q] : 0.f;
          sum = r < T ? sum : 0.f;
          if (r < T) dkv2[(row0 + r) * 2 * XD + c] = sum;
          kvL[r * G2_KVLD + c] = sum;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) kvL[(rb + i) * G2_KVLD + c] = 0.f;
      }
    }
  }
  lds_sync();
  {  // dv1 (kv2 path) = [dK2 dV2] . Wkv2
    f32x4 acc[1][2];
    zero(acc);
    mm_lw<1, 2, 2 * XD / 32>(acc, kvL, G2_KVLD, wkv);
    store_acc(acc, 32 * w, nullptr, t1, LDA, nullptr, 0, 0, 16);
  }
  lds_sync();
  {  // + v-pool (mean over T); LayerNorm backward; t1 = ds (dv residual), dv2 = keep * ds
    float g0 = 0.f, g1 = 0.f, b0 = 0.f, b1 = 0.f;
    const float pv0 = demb[(long)b * 2 * XD + lane] / T, pv1 = demb[(long)b * 2 * XD + 64 + lane] / T;
    for (int r = w; r < 16; r += 4) {
      float ds0 = 0.f, ds1 = 0.f;
      if (r < T) {
        const long gr = row0 + r;
        ln_row_bwd(t1[r * LDA + lane] + pv0, t1[r * LDA + 64 + lane] + pv1, s_v + gr * XD, mean_v[gr], rstd_v[gr],
                   gamma, ds0, ds1, g0, g1, b0, b1);
        dv2[gr * XD + lane] = keep * ds0;
        dv2[gr * XD + 64 + lane] = keep * ds1;
        dv[gr * XD + lane] = ds0;  // the residual part of dv (G1 adds dq1 . Wq1)
        dv[gr * XD + 64 + lane] = ds1;
      }
      d2L[r * LDA + lane] = keep * ds0;
      d2L[r * LDA + 64 + lane] = keep * ds1;
    }
    ln_part_store(g0, g1, b0, b1, red, ln_part + (long)b * 256);
  }
  lds_sync();
  {  // do1 = dv2 . Wo1
    f32x4 acc[1][2];
    zero(acc);
    mm_lw<1, 2, XD / 32>(acc, d2L, LDA, wo);
    store_acc(acc, 32 * w, nullptr, nullptr, 0, do1, XD, row0, T);
  }
}

// one wave per 32-key chunk (8 waves, Ta <= 256: with 4 waves wave 0 carried two chunks at Ta = 149 and its chunk
// phase -- dS, dq1 partial, the chunk's dK1 / dV1 -- set the block time, tools/xt_phases.py: 5.2 of 10.4 us)
constexpr int G2B_W = 8;

// fixed-order sum of v[0..N) (N a power of two): pairwise, the same tree whatever the wave schedule
template <int N>
__device__ __forceinline__ float tree_sum(const float* v, int stride) {
  if constexpr (N == 1) {
    return v[0];
  } else {
    return tree_sum<N / 2>(v, stride) + tree_sum<N / 2>(v + (N / 2) * stride, stride);
  }
}

__global__ __launch_bounds__(64 * G2B_W) void xh_v2a_attn_bwd_kernel(
    int T, int Ta, const float* __restrict__ do1, const float* __restrict__ P1, const float* __restrict__ kv1,
    const float* __restrict__ q1, XhDrop dr, float scale, float* __restrict__ dq1, float* __restrict__ dqkv,
    float* __restrict__ dS_heads) {
  __shared__ float red[G2B_W][16];
  __shared__ __attribute__((aligned(16))) float dSt[G2B_W][16 * G2B_TLD];  // per-wave dS chunk [query][key]
  __shared__ __attribute__((aligned(16))) float Pdt[G2B_W][16 * G2B_TLD];  // per-wave P' chunk
  __shared__ float oP[G2B_W][16][33];
  XT(2, 0);
  const int b = blockIdx.x >> 2, h = blockIdx.x & 3;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4, fk = fq * 8;
  const long ldkv = 2 * XD, row0 = (long)b * T;
  const float* Kr = kv1 + (long)b * Ta * ldkv + h * XDH;
  const float* Vr = Kr + XD;
  const int c = w;                  // this wave's chunk
  const bool live = 32 * c < Ta;    // (wave-uniform)
  const unsigned long long seed_attn = mer_site_seed(dr.seed, dr.site_attn);
  // every global load first: V fragments (dP), the saved probabilities, K gathers (dq1), the q1 / do1 fragments
  f32x4 vraw[2][2];
  float praw[2][4];
  float kraw[2][8];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int j = 32 * c + 16 * tt + fr, jc = j < Ta ? j : Ta - 1;
    vraw[tt][0] = *reinterpret_cast<const f32x4*>(Vr + (long)jc * ldkv + fk);
    vraw[tt][1] = *reinterpret_cast<const f32x4*>(Vr + (long)jc * ldkv + fk + 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * fq + r;
      praw[tt][r] = P1[(((long)b * XH + h) * T + (i < T ? i : T - 1)) * Ta + jc];  // always in range
    }
  }
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kk = 32 * c + fk + e;
      kraw[jt][e] = Kr[(long)(kk < Ta ? kk : Ta - 1) * ldkv + 16 * jt + fr];
    }
  bf16x8 gh, gl;  // do1_h rows (A of dP)
  frag_row(do1 + (row0 + (fr < T ? fr : T - 1)) * XD + h * XDH + fk, fr < T, gh, gl);
  bf16x8 qch[2], qcl[2], gch[2], gcl[2];  // q1_h / do1_h as [dim][query] B operands of dK / dV
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    frag_col(q1 + (row0 + fk) * XD + h * XDH + 16 * jt + fr, XD, fk, T, qch[jt], qcl[jt]);
    frag_col(do1 + (row0 + fk) * XD + h * XDH + 16 * jt + fr, XD, fk, T, gch[jt], gcl[jt]);
  }
  XT(2, 1);
  f32x4 dp[2];
  float pv[2][4], mk[2][4];
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {  // dP' = do1_h . V_h^T, dP = dP' * mask, rowsum partials of P dP
    const int j = 32 * c + 16 * tt + fr;
    float x[8] = {vraw[tt][0][0], vraw[tt][0][1], vraw[tt][0][2], vraw[tt][0][3],
                  vraw[tt][1][0], vraw[tt][1][1], vraw[tt][1][2], vraw[tt][1][3]};
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = j < Ta ? x[e] : 0.f;
    bf16x8 bh, bl;
    split8(x, bh, bl);
    dp[tt] = mma3(gh, gl, bh, bl, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * fq + r;
      const bool ok = i < T && j < Ta;
      const long pi = (((long)b * XH + h) * T + i) * Ta + j;
      const float m = ok ? dropout_scale(seed_attn, pi, dr.attn) : 0.f;
      const float p = ok ? praw[tt][r] : 0.f;
      pv[tt][r] = p;
      mk[tt][r] = m;
      dp[tt][r] *= m;
      rs[r] += p * dp[tt][r];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) rs[r] += __shfl_xor(rs[r], o, 64);
    if (fr == 0) red[w][4 * fq + r] = rs[r];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) rs[r] = tree_sum<G2B_W>(&red[0][4 * fq + r], 16);
  XT(2, 2);
  f32x4 oq[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  float* st = dSt[w];
  float* pt = Pdt[w];
  if (live) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 4 * fq + r, jj = 16 * tt + fr, j = 32 * c + jj;
        const float ds = pv[tt][r] * (dp[tt][r] - rs[r]);
        st[i * G2B_TLD + jj] = ds;
        pt[i * G2B_TLD + jj] = pv[tt][r] * mk[tt][r];  // P' (zero outside the T x Ta block)
        if (dS_heads && i < T && j < Ta) dS_heads[(((long)b * XH + h) * T + i) * Ta + j] = ds;
      }
    wave_sync_lds();
    {  // dq1_h partial = dS . K_h over this chunk's keys
      bf16x8 ah, al;
      frag_row(st + fr * G2B_TLD + fk, true, ah, al);
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        float x[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = 32 * c + fk + e < Ta ? kraw[jt][e] : 0.f;
        bf16x8 bh, bl;
        split8(x, bh, bl);
        oq[jt] = mma3(ah, al, bh, bl, oq[jt]);
      }
    }
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {  // dK1_h = dS^T q1_h * scale, dV1_h = P'^T do1_h for the chunk's 2 key tiles
      if (32 * c + 16 * tt >= Ta) break;
      bf16x8 sh, sl, ph, pl;
      frag_col(st + (long)fk * G2B_TLD + 16 * tt + fr, G2B_TLD, fk, 16, sh, sl);
      frag_col(pt + (long)fk * G2B_TLD + 16 * tt + fr, G2B_TLD, fk, 16, ph, pl);
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        const f32x4 dk = mma3(sh, sl, qch[jt], qcl[jt], f32x4{0.f, 0.f, 0.f, 0.f});
        const f32x4 dvv = mma3(ph, pl, gch[jt], gcl[jt], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = 32 * c + 16 * tt + 4 * fq + r;
          if (j < Ta) {
            float* drow = dqkv + ((long)b * Ta + j) * 3 * XD;
            drow[XD + h * XDH + 16 * jt + fr] = dk[r] * scale;
            drow[2 * XD + h * XDH + 16 * jt + fr] = dvv[r];
          }
        }
      }
    }
  }
  XT(2, 3);
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) oP[w][4 * fq + r][16 * jt + fr] = oq[jt][r];
  __syncthreads();
  for (int e = threadIdx.x; e < T * XDH; e += 64 * G2B_W) {
    const int i = e / XDH, d = e - i * XDH;
    dq1[(row0 + i) * XD + h * XDH + d] = tree_sum<G2B_W>(&oP[0][i][d], 16 * 33) * scale;
  }
  XT(2, 4);
}

// the prior bias gradient: dbias[b][i][j] = sum over heads of dS (head order, mha_dbias_kernel's order)
__global__ __launch_bounds__(256) void xh_dbias_heads_kernel(long n_per_b, long n, const float* __restrict__ dS_heads,
                                                             float* __restrict__ dbias) {
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const long b = e / n_per_b, k = e - b * n_per_b;
    const float* p = dS_heads + b * XH * n_per_b + k;
    dbias[e] = ((p[0] + p[n_per_b]) + p[2 * n_per_b]) + p[3 * n_per_b];
  }
}

MER_API int mer_xh_v2a_bwd(int B, int T, int Ta, const float* dkv2_part, const void* WkvT2_hi, const void* WkvT2_lo,
                           const float* demb, const float* s_v, const float* mean_v, const float* rstd_v,
                           const float* gamma, const void* WoT1_hi, const void* WoT1_lo, const float* P1,
                           const float* kv1, const float* q1, float attn_p, float path_p, const unsigned long long* seed,
                           unsigned long long site_attn, unsigned long long site_path, float scale, float* dkv2,
                           float* dv2, float* dq1, float* dv, float* dqkv, float* ln_part, float* do1,
                           float* dS_heads, float* dbias, void* stream) {
  if (B <= 0) return 0;
  if (T <= 0 || T > 16 || Ta <= 0 || Ta > 16 * G2_KT || ((attn_p > 0.f || path_p > 0.f) && !seed) || !do1 ||
      (dbias && !dS_heads))
    return (int)hipErrorInvalidValue;
  XhDrop dr{attn_p, path_p, seed, site_attn, site_path};
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(xh_v2a_pre_bwd_kernel, dim3(B), dim3(256), 0, st, T, (Ta + 15) / 16, dkv2_part,
                     SplitW{(const bf16_t*)WkvT2_hi, (const bf16_t*)WkvT2_lo}, demb, s_v, mean_v, rstd_v, gamma,
                     SplitW{(const bf16_t*)WoT1_hi, (const bf16_t*)WoT1_lo}, dr, dkv2, dv2, dv, do1, ln_part);
  hipLaunchKernelGGL(xh_v2a_attn_bwd_kernel, dim3(B * XH), dim3(64 * G2B_W), 0, st, T, Ta, do1, P1, kv1, q1, dr, scale,
                     dq1, dqkv, dbias ? dS_heads : nullptr);
  if (dbias) {
    const long n = (long)B * T * Ta;
    hipLaunchKernelGGL(xh_dbias_heads_kernel, dim3((unsigned)((n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024)),
                       dim3(256), 0, st, (long)T * Ta, n, dS_heads, dbias);
  }
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// G1: audio chain backward, 32 rows per block: da += [dq2 | dK1 dV1] . [Wq2 ; Wkv1], da_s = da . Wa
// Unfused: the dx halves of xattn_head.py:251, 269 and 303-304.  The trailing ceil(B*T/16) blocks: dv += dq1 Wq1,
// dv_feat = dv Wv.  Latency chains like F1: the block's input rows are staged into LDS with one load per
// thread-slot and every weight fragment a wave needs is loaded into registers at block entry (WRegs), so one
// memory latency precedes the products instead of one per k step (phase stamps, B = 32: the 384-deep first
// product took 14.9 us, the video blocks' four 32-column dv_feat passes 12.5 us).
// ---------------------------------------------------------------------------------------------
struct XhVideoBwd {  // G1's video rows: dv += dq1 Wq1 (in place), dvfeat = dv Wv (NULL: not wanted)
  int M, vdim;
  const float* dq1;
  SplitW WqT1, WvT;
  float* dv;
  float* dvfeat;
};

constexpr int G1_WAVES = 8;
constexpr int G1_ALD = 3 * XD + 4;  // LDS row stride of the staged [dq2 | dK1 dV1] rows
constexpr int G1_VROWS = 16;        // video rows per block
constexpr int G1_VK = 512;          // dv_feat width bound (ResNet18: 512)

__global__ __launch_bounds__(64 * G1_WAVES) void xh_audio_bwd_kernel(int M, const float* __restrict__ dqkv,
                                                                     SplitW WcT, SplitW WaT, float* __restrict__ da,
                                                                     float* __restrict__ da_s, XhVideoBwd vid) {
  __shared__ __attribute__((aligned(16))) float inL[32 * G1_ALD];
  __shared__ __attribute__((aligned(16))) float daL[32 * LDA];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
  const int na = (M + 31) / 32;
  constexpr int NT = 64 * G1_WAVES;
  if ((int)blockIdx.x < na) {
    XT(0, 0);
    const long r0 = (long)blockIdx.x * 32;
    const int rmax = (int)(M - r0 < 32 ? M - r0 : 32);
    constexpr int NX = 32 * 3 * XD / 4 / NT;  // float4 slots per thread
    f32x4 x[NX];
#pragma unroll
    for (int q = 0; q < NX; ++q) {
      const int e = threadIdx.x + NT * q, r = e / (3 * XD / 4), c = 4 * (e % (3 * XD / 4));
      x[q] = *reinterpret_cast<const f32x4*>(dqkv + (r0 + (r < rmax ? r : rmax - 1)) * 3 * XD + c);
    }
    WRegs<3 * XD / 32, 1> wc;
    wregs_load(wc, WcT, 3 * XD, 16 * w, 3 * XD / 32);
    WRegs<XD / 32, 1> wa;
    wregs_load(wa, WaT, XD, 16 * w, XD / 32);
    float res[2][4];  // the residual (G3's LayerNorm-backward da), loaded before any store of this block
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * i + 4 * fq + r;
        res[i][r] = da[(r0 + (row < rmax ? row : rmax - 1)) * XD + 16 * w + fr];
      }
#pragma unroll
    for (int q = 0; q < NX; ++q) {
      const int e = threadIdx.x + NT * q, r = e / (3 * XD / 4), c = 4 * (e % (3 * XD / 4));
      *reinterpret_cast<f32x4*>(inL + r * G1_ALD + c) = r < rmax ? x[q] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    lds_sync();
    {
      f32x4 acc[2][1];
      zero(acc);
      mm_lw<2, 1, 3 * XD / 32>(acc, inL, G1_ALD, wc);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * i + 4 * fq + r, col = 16 * w + fr;
          const float v = row < rmax ? acc[i][0][r] + res[i][r] : 0.f;
          if (row < rmax) da[(r0 + row) * XD + col] = v;
          daL[row * LDA + col] = v;
        }
    }
    lds_sync();
    XT(0, 1);
    f32x4 acc[2][1];  // da_s = da . Wa
    zero(acc);
    mm_lw<2, 1, XD / 32>(acc, daL, LDA, wa);
    store_acc(acc, 16 * w, nullptr, nullptr, 0, da_s, XD, r0, rmax);
    XT(0, 2);
    return;
  }
  XT(0, 8);
  const long v0 = (long)(blockIdx.x - na) * G1_VROWS;
  const int vmax = (int)(vid.M - v0 < G1_VROWS ? vid.M - v0 : G1_VROWS), vd = vid.vdim;
  constexpr int NX = G1_VROWS * XD / 4;  // = NT: one float4 per thread
  static_assert(NX == NT, "one staged float4 per thread");
  f32x4 x;
  {
    const int r = threadIdx.x / (XD / 4), c = 4 * (threadIdx.x % (XD / 4));
    x = *reinterpret_cast<const f32x4*>(vid.dq1 + (v0 + (r < vmax ? r : vmax - 1)) * XD + c);
  }
  WRegs<XD / 32, 1> wq;
  wregs_load(wq, vid.WqT1, XD, 16 * w, XD / 32);
  WRegs<XD / 32, G1_VK / 16 / G1_WAVES> wv;  // 64 dv_feat columns per wave
  if (vid.dvfeat) wregs_load(wv, vid.WvT, XD, (G1_VK / G1_WAVES) * w, XD / 32, vd);
  float res[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 4 * fq + r;
    res[r] = vid.dv[(v0 + (row < vmax ? row : vmax - 1)) * XD + 16 * w + fr];
  }
  {
    const int r = threadIdx.x / (XD / 4), c = 4 * (threadIdx.x % (XD / 4));
    *reinterpret_cast<f32x4*>(inL + r * LDA + c) = r < vmax ? x : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  lds_sync();
  {
    f32x4 acc[1][1];
    zero(acc);
    mm_lw<1, 1, XD / 32>(acc, inL, LDA, wq);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * fq + r, col = 16 * w + fr;
      const float v = row < vmax ? acc[0][0][r] + res[r] : 0.f;
      if (row < vmax) vid.dv[(v0 + row) * XD + col] = v;
      daL[row * LDA + col] = v;
    }
  }
  lds_sync();
  XT(0, 9);
  if (vid.dvfeat) {  // dv_feat = dv . Wv
    constexpr int TJ = G1_VK / 16 / G1_WAVES;
    f32x4 acc[1][TJ];
    zero(acc);
    mm_lw<1, TJ, XD / 32>(acc, daL, LDA, wv);
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int col = (G1_VK / G1_WAVES) * w + 16 * j + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 4 * fq + r;
        if (row < vmax && col < vd) vid.dvfeat[(v0 + row) * vd + col] = acc[0][j][r];
      }
    }
  }
  XT(0, 10);
}

MER_API int mer_xh_audio_bwd(int M, const float* dqkv, const void* WcT_hi, const void* WcT_lo, const void* WaT_hi,
                             const void* WaT_lo, float* da, float* da_s, int Mv, int vdim, const float* dq1,
                             const void* WqT1_hi, const void* WqT1_lo, const void* WvT_hi, const void* WvT_lo, float* dv,
                             float* dvfeat, void* stream) {
  // M = 0: the video rows alone (the critical path into the trunk backward); Mv = 0: the audio chain alone
  if (M < 0 || Mv < 0 || M + Mv == 0 ||
      (Mv > 0 && (!dq1 || !dv || (dvfeat && (vdim <= 0 || vdim % 32 || vdim > G1_VK)))))
    return (int)hipErrorInvalidValue;
  const XhVideoBwd vid{Mv, vdim, dq1, SplitW{(const bf16_t*)WqT1_hi, (const bf16_t*)WqT1_lo},
                       SplitW{(const bf16_t*)WvT_hi, (const bf16_t*)WvT_lo}, dv, dvfeat};
  hipLaunchKernelGGL(xh_audio_bwd_kernel, dim3((M + 31) / 32 + (Mv + G1_VROWS - 1) / G1_VROWS), dim3(64 * G1_WAVES), 0,
                     (hipStream_t)stream, M,
                     dqkv, SplitW{(const bf16_t*)WcT_hi, (const bf16_t*)WcT_lo},
                     SplitW{(const bf16_t*)WaT_hi, (const bf16_t*)WaT_lo}, da, da_s, vid);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// W: grouped weight gradients.  Problem p: dW[n][k] (+)= sum_m dY[m][n] X[m][k] and db[n] (+)= sum_m dY[m][n]
// (K = 0: a column-sum-only problem, the LayerNorm dgamma / dbeta partials).  Blocks = (problem, 128 x 128
// output tile, row split); each writes its partial tile to ws, the bias partials (k-tile 0 blocks) after it;
// xh_wfold adds the partials in split order.  The table travels by value in the kernel arguments, so a
// captured graph holds it (no device table to upload).  128 x 128 tiles cover the head's 128 / 256-wide
// Linears with one or two tiles, so each dY / X column block is read once per tile instead of once per 64-wide
// tile of the other operand (the 64 x 64 version re-read dY 12x for audio_seq_proj: 97 MB per step).
// ---------------------------------------------------------------------------------------------
constexpr int WG_MAXP = 32;  // the head's Linears + LayerNorms + classifier + the emotion prior's 10 products
constexpr int WG_HOST_COLS = 11;  // dY ldy X ldx x_dtype M N K splits dW db
constexpr int WG_T = 128;         // output tile (n and k)

struct WgProb {
  const float* dY;
  const void* X;
  float* dW;
  float* db;
  long long ldy, ldx, M, ws_off, ws_b_off;
  int N, K, splits, first_block, xbf, pad;
};

struct WgTab {
  WgProb p[WG_MAXP];
  int nprob;
  int xcd;  // split-major blocks in XCD chunks (xh_wgrad_kernel)
};

// Staging: thread t owns column (t & 127) of the 128-wide dY / X tile and 16 consecutive rows (t >> 7) * 16 ..
// + 15 of the 32-row chunk: 16 wave-coalesced loads per operand, split into bf16 hi / lo once and stored as two
// 16-byte LDS vectors per plane in [column][row] layout, which is exactly the MFMA fragment (8 consecutive m of
// one n / k).  The next chunk's loads are issued before the current chunk's MFMAs.
constexpr int WG_LDM = 32 + 8;  // bf16 row stride of the [128][32] planes (80 bytes: 16-byte aligned)

struct WgChunk {  // raw loads: decoded (dtype, bounds) only when the chunk is consumed
  float y[16];
  uint32_t xw[16];
};

// Branch-free (see mm_aw): unconditional loads from clamped addresses (row m1 - 1, column N - 1 / K - 1); X is
// read as 32-bit words whatever its dtype (a bf16 element is one half of its word), and a K = 0 problem reads a
// valid dummy X (the host points X at dY).  Nothing here uses the loaded values, so the loads stay in flight
// until wg_decode (decoding at load time made every load wait for itself).
__device__ __forceinline__ void wg_load(const WgProb& d, long mc, long m1, int n0, int k0, WgChunk& c) {
  const int col = threadIdx.x & 127, m16 = ((threadIdx.x >> 7) & 1) * 16;  // (each 256-thread group stages a chunk)
  const int nc = n0 + col < d.N ? n0 + col : d.N - 1, kc = k0 + col < d.K ? k0 + col : (d.K > 0 ? d.K - 1 : 0);
  const int esz = d.xbf ? 2 : 4;
  const char* Xb = reinterpret_cast<const char*>(d.X);
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const long m = mc + m16 + e, mm = m < m1 ? m : m1 - 1;
    c.y[e] = d.dY[mm * d.ldy + nc];
    const uintptr_t addr = reinterpret_cast<uintptr_t>(Xb + (mm * d.ldx + kc) * esz);
    // an integer-derived pointer would be a FLAT access (LDS or global: every flat load waits for itself and
    // for LDS traffic); the global address space keeps these ordinary pipelined loads
    c.xw[e] = *(const __attribute__((address_space(1))) uint32_t*)(addr & ~(uintptr_t)3);
  }
}

// zero the out-of-range elements, take the bf16 half of X's words
__device__ __forceinline__ void wg_decode(const WgProb& d, long mc, long m1, int n0, int k0, WgChunk& c,
                                          float (&x)[16]) {
  const int col = threadIdx.x & 127, m16 = ((threadIdx.x >> 7) & 1) * 16;
  const bool okn = n0 + col < d.N, okk = k0 + col < d.K;
  const int kc = okk ? k0 + col : (d.K > 0 ? d.K - 1 : 0);
  const int esz = d.xbf ? 2 : 4;
  const uintptr_t xb = reinterpret_cast<uintptr_t>(d.X);
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const long m = mc + m16 + e, mm = m < m1 ? m : m1 - 1;
    const bool okm = m < m1;
    const uintptr_t addr = xb + (mm * d.ldx + kc) * esz;
    const uint32_t wv = c.xw[e];
    const uint32_t bits = d.xbf ? ((addr & 2) ? (wv & 0xffff0000u) : (wv << 16)) : wv;
    c.y[e] = (okm && okn) ? c.y[e] : 0.f;
    x[e] = (okm && okk) ? __uint_as_float(bits) : 0.f;
  }
}

__device__ __forceinline__ void wg_store_planes(const float (&v)[16], bf16_t* hi, bf16_t* lo) {
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    Frag H, L;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint16_t hb = f2bf(v[8 * half + e]);
      H.h[e] = hb;
      L.h[e] = f2bf(v[8 * half + e] - bf2f(hb));
    }
    *reinterpret_cast<u4*>(hi + 8 * half) = H.u;
    *reinterpret_cast<u4*>(lo + 8 * half) = L.u;
  }
}

// 512 threads = two groups of 4 waves; group g takes the 32-row chunks 2i + g of the block's row range into its own
// LDS planes and accumulators (2 waves per SIMD: twice the loads in flight of a 4-wave block), then group 1 hands
// its 128 x 128 partial to group 0 through LDS, which adds it (fixed order) and writes the block's slab.
constexpr int WG_PLANE = WG_T * WG_LDM;  // bf16 elements per plane

__global__ __launch_bounds__(512) void xh_wgrad_kernel(const WgTab tab, float* __restrict__ ws) {
  __shared__ __attribute__((aligned(16))) bf16_t planes[2][4][WG_PLANE];  // [group][yh, yl, xh, xl]
  __shared__ float bred[4][WG_T];
  // tab.xcd: the tiles of one row split (same dY rows: every tile of a column block tn reads the same dY slice)
  // on consecutive virtual ids of one XCD chunk (xcd_tile's bijective map), so the slice is fetched into one L2
  // once instead of once per XCD the round-robin placement spread them over
  int vb = blockIdx.x, unused;
  if (tab.xcd) xcd_tile(blockIdx.x, 1 << 30, (int)gridDim.x, vb, unused);
  const int pi = table_find(tab.nprob, vb, [&](int i) { return tab.p[i].first_block; });
  const WgProb& d = tab.p[pi];
  const int N = d.N, K = d.K, splits = d.splits;
  const int ntk = K > 0 ? (K + WG_T - 1) / WG_T : 1;
  const int local = vb - d.first_block;
  const int ntiles = ((N + WG_T - 1) / WG_T) * ntk;
  const int split = tab.xcd ? local / ntiles : local % splits, tile = tab.xcd ? local - split * ntiles : local / splits;
  const int tn = tile / ntk, tk = tile - tn * ntk;
  const int n0 = tn * WG_T, k0 = tk * WG_T;
  const long per = (d.M + splits - 1) / splits, m0 = split * per, m1 = m0 + per < d.M ? m0 + per : d.M;
  const int grp = threadIdx.x >> 8, t = threadIdx.x & 255;
  const int w = t >> 6, lane = threadIdx.x & 63, fr = lane & 15, fk = (lane >> 4) * 8;
  const int wn = w >> 1, wk = w & 1;  // this wave's 64 x 64 quadrant of the tile
  const int col = t & 127, m16 = (t >> 7) * 16;
  bf16_t* yh = planes[grp][0];
  bf16_t* yl = planes[grp][1];
  bf16_t* xh_ = planes[grp][2];
  bf16_t* xl = planes[grp][3];
  const bool bias = d.db != nullptr && tk == 0;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;  // column n0 + col, this thread's rows
  const long nchunk = (m1 - m0 + 31) / 32, iters = ((nchunk + 1) / 2 + 1) / 2 * 2;  // even: two buffers
  // chunk i of this group starts at row m0 + 32 * (2i + grp); a chunk past the range loads an empty range
  // (m >= m1 everywhere: zeros), so both groups run the same iterations and barriers.  Two chunks are in
  // flight (buffers c0 / c1, loop unrolled by two so no register copy waits on a load), and the barriers are
  // LDS-only: __syncthreads' release fence would wait for the prefetch at every iteration.
  auto chunk_row = [&](long i) { return m0 + 32 * (2 * i + grp); };
  XT(1, 0);
  auto step = [&](WgChunk& c, long it) {
    lds_sync();  // the previous chunk's fragments are read
    float xv[16];
    wg_decode(d, chunk_row(it), m1, n0, k0, c, xv);
#pragma unroll
    for (int e = 0; e < 16; ++e) bsum += c.y[e];
    wg_store_planes(c.y, yh + col * WG_LDM + m16, yl + col * WG_LDM + m16);
    wg_store_planes(xv, xh_ + col * WG_LDM + m16, xl + col * WG_LDM + m16);
    lds_sync();
    // chunk it + 2 into the buffer just consumed (past the end: an empty range, unused)
    wg_load(d, chunk_row(it + 2 < iters ? it + 2 : iters), m1, n0, k0, c);
    Frag BH[4], BL[4];  // B[k][m] = X[m][k]; the lo plane of bf16 X is zero
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      BH[j].u = *reinterpret_cast<const u4*>(xh_ + (64 * wk + 16 * j + fr) * WG_LDM + fk);
      BL[j].u = *reinterpret_cast<const u4*>(xl + (64 * wk + 16 * j + fr) * WG_LDM + fk);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      Frag AH, AL;  // A[n][m] = dY[m][n]
      AH.u = *reinterpret_cast<const u4*>(yh + (64 * wn + 16 * i + fr) * WG_LDM + fk);
      AL.u = *reinterpret_cast<const u4*>(yl + (64 * wn + 16 * i + fr) * WG_LDM + fk);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] = mma(AH.v, BH[j].v, acc[i][j]);
        acc[i][j] = mma(AL.v, BH[j].v, acc[i][j]);
        acc[i][j] = mma(AH.v, BL[j].v, acc[i][j]);
      }
    }
    if (it < 4) XT(1, 1 + it);
  };
  WgChunk c0, c1;
  wg_load(d, chunk_row(0), m1, n0, k0, c0);
  wg_load(d, chunk_row(1), m1, n0, k0, c1);
  for (long it = 0; it < iters; it += 2) {
    step(c0, it);
    step(c1, it + 1);
  }
  bred[grp * 2 + (t >> 7)][col] = bsum;
  __syncthreads();  // every group is past its last fragment read: the planes take group 1's partial
  float* xch = reinterpret_cast<float*>(&planes[0][0][0]);  // [256 lanes][64] fp32 = 64 KiB of the 80 KiB
  if (grp == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<f32x4*>(xch + ((i * 4 + j) * 256 + t) * 4) = acc[i][j];
  }
  __syncthreads();
  XT(1, 5);
  // group 0 adds group 1's partial (fixed order) and the sum goes back through LDS as a row-major tile, so the
  // slab is written with 16-byte stores of whole row segments: the MFMA-layout stores (4 rows x 64 bytes per
  // instruction) drained at ~1.2 TB/s after the blocks' last phase (~13 us of a 37 us launch at B = 32)
  constexpr int TLD = WG_T + 4;  // [128][132] fp32 = 66 KiB of the 80 KiB planes
  float* tileL = xch;
  f32x4 sum[4][4];
  if (grp == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 o = *reinterpret_cast<const f32x4*>(xch + ((i * 4 + j) * 256 + t) * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) sum[i][j][r] = acc[i][j][r] + o[r];
      }
  }
  __syncthreads();  // the exchange is read: the tile overwrites it
  if (grp == 0 && K > 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          tileL[(64 * wn + 16 * i + 4 * (lane >> 4) + r) * TLD + 64 * wk + 16 * j + fr] = sum[i][j][r];
  }
  if (grp == 0 && bias && t < WG_T && n0 + t < N)
    ws[d.ws_b_off + (long)split * N + n0 + t] = (bred[0][t] + bred[1][t]) + (bred[2][t] + bred[3][t]);
  __syncthreads();
  if (K > 0) {
    float* out = ws + d.ws_off + (long)split * N * K;
    const int c4 = 4 * (threadIdx.x & 31), k = k0 + c4;
#pragma unroll
    for (int q = 0; q < WG_T / 16; ++q) {
      const int rl = (threadIdx.x >> 5) + 16 * q, n = n0 + rl;
      if (n >= N || k >= K) continue;
      const f32x4 v = *reinterpret_cast<const f32x4*>(tileL + rl * TLD + c4);
      float* dst = out + (long)n * K + k;
      if (k + 3 < K && ((uintptr_t)dst & 15) == 0) {
        *reinterpret_cast<f32x4*>(dst) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (k + e < K) dst[e] = v[e];
      }
    }
  }
  XT(1, 6);
}

__global__ __launch_bounds__(256) void xh_wfold_kernel(const WgTab tab, const float* __restrict__ ws) {
  const WgProb& d = tab.p[blockIdx.y];
  const long nk = (long)d.N * d.K, tot = nk + (d.db ? d.N : 0);
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < tot; e += (long)gridDim.x * blockDim.x) {
    // partials in split order, loaded 8 at a time (the sum order stays fixed)
    const bool wpart = e < nk;
    const float* src = wpart ? ws + d.ws_off + e : ws + d.ws_b_off + (e - nk);
    const long stride = wpart ? nk : (long)d.N;
    float s = 0.f;
    for (int q0 = 0; q0 < d.splits; q0 += 32) {  // 32 partials in flight, summed in split order
      float v[32];
#pragma unroll
      for (int q = 0; q < 32; ++q) {
        const float x = src[(long)(q0 + q < d.splits ? q0 + q : d.splits - 1) * stride];
        v[q] = q0 + q < d.splits ? x : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 32; ++q) s += v[q];
    }
    if (wpart)
      d.dW[e] += s;
    else
      d.db[e - nk] += s;
  }
}

// host table rows: {dY, ldy, X, ldx, x_dtype, M, N, K, splits, dW, db} (pointers as int64; X / dW 0 when K = 0,
// db 0 for no bias); returns the workspace floats needed, or -1 for an invalid row
static long long wg_layout(int nprob, const long long* t, WgTab* tab, int* blocks) {
  long long off = 0;
  int fb = 0;
  for (int i = 0; i < nprob; ++i) {
    const long long* r = t + (long)i * WG_HOST_COLS;
    WgProb& p = tab->p[i];
    p.dY = reinterpret_cast<const float*>(r[0]);
    p.ldy = r[1];
    p.X = reinterpret_cast<const void*>(r[2]);
    p.ldx = r[3];
    p.xbf = r[4] == MER_BF16;
    p.M = r[5];
    p.N = (int)r[6];
    p.K = (int)r[7];
    p.splits = (int)r[8];
    p.dW = reinterpret_cast<float*>(r[9]);
    p.db = reinterpret_cast<float*>(r[10]);
    p.pad = 0;
    if (p.K == 0) {  // column sums only: the loader still reads a (valid) X word
      p.X = p.dY;
      p.ldx = 0;
      p.xbf = 0;
    }
    if (p.M <= 0 || p.N <= 0 || p.K < 0 || p.splits <= 0 || p.splits > p.M || !p.dY ||
        (p.K > 0 && (!p.X || !p.dW)) || (p.K == 0 && !p.db))
      return -1;
    p.ws_off = off;
    off += (long long)p.splits * p.N * p.K;
    p.ws_b_off = off;
    if (p.db) off += (long long)p.splits * p.N;
    p.first_block = fb;
    fb += p.splits * ((p.N + WG_T - 1) / WG_T) * (p.K > 0 ? (p.K + WG_T - 1) / WG_T : 1);
  }
  tab->nprob = nprob;
  *blocks = fb;
  return off;
}

#ifdef MER_XH_TIMING
MER_API int mer_xt_read_bwd(long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(mer_xt_buf), sizeof(long long) * 4 * 512 * 16, 0,
                                  hipMemcpyDeviceToHost);
}
#endif

MER_API int mer_xh_wgrad_ws_floats(int nprob, const long long* table, long long* out) {
  if (nprob <= 0 || nprob > WG_MAXP || !out) return (int)hipErrorInvalidValue;
  WgTab tab;
  int blocks = 0;
  const long long n = wg_layout(nprob, table, &tab, &blocks);
  if (n < 0) return (int)hipErrorInvalidValue;
  *out = n;
  return 0;
}

MER_API int mer_xh_wgrad(int nprob, const long long* table, float* ws, long long ws_floats, void* stream) {
  if (nprob <= 0) return 0;
  if (nprob > WG_MAXP) return (int)hipErrorInvalidValue;
  WgTab tab;
  int blocks = 0;
  const long long need = wg_layout(nprob, table, &tab, &blocks);
  if (need < 0 || need > ws_floats) return (int)hipErrorInvalidValue;
  tab.xcd = 1;  // split-major per XCD: the tiles of one row split (same dY slice) share an L2
  hipLaunchKernelGGL(xh_wgrad_kernel, dim3(blocks), dim3(512), 0, (hipStream_t)stream, tab, ws);
  // fold: one element per thread for the largest problem (each thread's split loads are one latency round, not
  // one per element it would otherwise loop over)
  long long most = 0;
  for (int i = 0; i < nprob; ++i) {
    const long long tot = (long long)tab.p[i].N * tab.p[i].K + (tab.p[i].db ? tab.p[i].N : 0);
    most = tot > most ? tot : most;
  }
  const unsigned fold_x = (unsigned)((most + 255) / 256 < 1024 ? (most + 255) / 256 : 1024);
  hipLaunchKernelGGL(xh_wfold_kernel, dim3(fold_x, nprob), dim3(256), 0, (hipStream_t)stream, tab, ws);
  MER_LAUNCH_CHECK();
}
