// Fused xattn head backward: the reverse of xattn_fused.hip (fusion.py:366-411 + the two nn.MultiheadAttention
// blocks, TORCH:6576-6606) on split-bf16 MFMA.  Four data-gradient launches plus one grouped weight-gradient
// launch and its fixed-order fold replace the ~25 backward launches of xattn_head.head_backward:
//   G4 xh_mlp_bwd   (grid 8): classifier head -> demb; the head's own weight gradients (exact fp32 FMA)
//   G3 xh_a2v_bwd   (grid B * ceil(Ta/16)): a-pool / LayerNorm / out-proj / attention backward of 16 query rows
//                   -> da (LN residual part), da2, dq2, per-tile partials of dK2 dV2 and of dgamma / dbeta
//   G2 xh_v2a_bwd   (grid B): dK2 dV2 fold -> dv1 -> LayerNorm / out-proj / attention backward over the
//                   sample's Ta keys -> dq1, dK1 dV1, dv and dv_feat (the ResNet18 trunk's input gradient)
//   G1 xh_audio_bwd (grid B * Ta / 32): da += [dq2 | dK1 dV1] . [Wq2 ; Wkv1], da_s = da . Wa
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
  __syncthreads();
  if (threadIdx.x < 256) {
    float s = 0.f;
    for (int q = 0; q < 4; ++q) s += red[q * 256 + threadIdx.x];
    part[threadIdx.x] = s;
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// G4: classifier head backward, chunks of 32 samples.  Every block recomputes the chunk's dh (B x H1, cheap);
// block k owns dW0 rows [k * H1 / 8, (k + 1) * H1 / 8) and demb of samples b = k (mod 8); block 0 the small
// weights and the biases.  The unfused schedule: xattn_head.py:207-225.
// ---------------------------------------------------------------------------------------------
constexpr int G4_BLOCKS = 8;
constexpr int G4_CHUNK = 32;

__global__ __launch_bounds__(256) void xh_mlp_bwd_kernel(int B, int C, int H1, int gated, const float* __restrict__ dl,
                                                         const float* __restrict__ emb, const float* __restrict__ h,
                                                         const float* __restrict__ gsave,
                                                         const float* __restrict__ fsave, const float* __restrict__ W0,
                                                         const float* __restrict__ W3, const float* __restrict__ Wc,
                                                         float mlp_p, const unsigned long long* __restrict__ seed_ptr,
                                                         unsigned long long site, float* __restrict__ dW0,
                                                         float* __restrict__ db0, float* __restrict__ dW3,
                                                         float* __restrict__ db3, float* __restrict__ dWc,
                                                         float* __restrict__ dbc, float* __restrict__ demb) {
  __shared__ float dh[G4_CHUNK][256];
  __shared__ float dfz[G4_CHUNK][XD + 1];  // gated: dfused (cols 0..127) and dz (col 128)
  const int t = threadIdx.x, k = blockIdx.x;
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  const int rows_per = (H1 + G4_BLOCKS - 1) / G4_BLOCKS;
  for (int c0 = 0; c0 < B; c0 += G4_CHUNK) {
    const int nb = B - c0 < G4_CHUNK ? B - c0 : G4_CHUNK;
    const float* dlc = dl + (long)c0 * C;
    const float* embc = emb + (long)c0 * 2 * XD;
    __syncthreads();
    if (gated) {
      for (int e = t; e < nb * XD; e += 256) {
        const int b = e / XD, c = e - b * XD;
        float acc = 0.f;
        for (int q = 0; q < C; ++q) acc = fmaf(dlc[b * C + q], Wc[q * XD + c], acc);
        dfz[b][c] = acc;
      }
      __syncthreads();
      if (t < nb) {  // dz = sum_c dfused (v - a) g (1 - g)
        float acc = 0.f;
        for (int c = 0; c < XD; ++c) acc += dfz[t][c] * (embc[(long)t * 2 * XD + c] - embc[(long)t * 2 * XD + XD + c]);
        const float g = gsave[c0 + t];
        dfz[t][XD] = acc * g * (1.f - g);
      }
      __syncthreads();
    }
    for (int e = t; e < nb * H1; e += 256) {
      const int b = e / H1, c = e - b * H1;
      float acc;
      if (gated) {
        acc = dfz[b][XD] * W3[c];
      } else {
        acc = 0.f;
        for (int q = 0; q < C; ++q) acc = fmaf(dlc[b * C + q], W3[q * H1 + c], acc);
      }
      const float hv = h[(long)(c0 + b) * H1 + c];  // post-dropout activation: relu' * keep / (1 - p)
      dh[b][c] = hv > 0.f ? acc * dropout_scale(seed, (uint64_t)((long)(c0 + b) * H1 + c), mlp_p) : 0.f;
    }
    __syncthreads();
    for (int r = k * rows_per; r < (k + 1) * rows_per && r < H1; ++r) {  // dW0[r][j] += sum_b dh[b][r] emb[b][j]
      float acc = 0.f;
      for (int b = 0; b < nb; ++b) acc = fmaf(dh[b][r], embc[(long)b * 2 * XD + t], acc);
      dW0[(long)r * 2 * XD + t] += acc;
    }
    if (k == 0) {
      if (t < H1) {
        float acc = 0.f;
        for (int b = 0; b < nb; ++b) acc += dh[b][t];
        db0[t] += acc;
      }
      if (!gated) {
        for (int e = t; e < C * H1; e += 256) {
          const int q = e / H1, c = e - q * H1;
          float acc = 0.f;
          for (int b = 0; b < nb; ++b) acc = fmaf(dlc[b * C + q], h[(long)(c0 + b) * H1 + c], acc);
          dW3[e] += acc;
        }
      } else {
        if (t < H1) {
          float acc = 0.f;
          for (int b = 0; b < nb; ++b) acc = fmaf(dfz[b][XD], h[(long)(c0 + b) * H1 + t], acc);
          dW3[t] += acc;
        }
        if (t == 0) {
          float acc = 0.f;
          for (int b = 0; b < nb; ++b) acc += dfz[b][XD];
          db3[0] += acc;
        }
        for (int e = t; e < C * XD; e += 256) {
          const int q = e / XD, c = e - q * XD;
          float acc = 0.f;
          for (int b = 0; b < nb; ++b) acc = fmaf(dlc[b * C + q], fsave[(long)(c0 + b) * XD + c], acc);
          dWc[e] += acc;
        }
      }
      if (t < C) {  // the classifier bias: xattn_mlp.3 (concat) or xattn_classifier (gated)
        float acc = 0.f;
        for (int b = 0; b < nb; ++b) acc += dlc[b * C + t];
        (gated ? dbc : db3)[t] += acc;
      }
    }
    for (int b = k; b < nb; b += G4_BLOCKS) {  // demb[b][j] = sum_r dh[b][r] W0[r][j] (+ the gate mix)
      float acc = 0.f;
      for (int r = 0; r < H1; ++r) acc = fmaf(dh[b][r], W0[(long)r * 2 * XD + t], acc);
      if (gated) {
        const float g = gsave[c0 + b];
        acc += t < XD ? dfz[b][t] * g : dfz[b][t - XD] * (1.f - g);
      }
      demb[(long)(c0 + b) * 2 * XD + t] = acc;
    }
  }
}

MER_API int mer_xh_mlp_bwd(int B, int C, int H1, int gated, const float* dlogits, const float* emb, const float* h,
                           const float* g, const float* fused, const float* W0, const float* W3, const float* Wc,
                           float mlp_p, const unsigned long long* seed, unsigned long long site, float* dW0, float* db0,
                           float* dW3, float* db3, float* dWc, float* dbc, float* demb, void* stream) {
  if (B <= 0) return 0;
  if (H1 <= 0 || H1 > 256 || C <= 0 || C > 256 || (mlp_p > 0.f && !seed) ||
      (gated && (!Wc || !dWc || !dbc || !g || !fused)))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(xh_mlp_bwd_kernel, dim3(G4_BLOCKS), dim3(256), 0, (hipStream_t)stream, B, C, H1, gated, dlogits,
                     emb, h, g, fused, W0, W3, Wc, mlp_p, seed, site, dW0, db0, dW3, db3, dWc, dbc, demb);
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
    float* __restrict__ dkv2_part, float* __restrict__ ln_part) {
  __shared__ __attribute__((aligned(16))) float d2L[16 * LDA];
  __shared__ __attribute__((aligned(16))) float oL[16 * LDA];
  __shared__ __attribute__((aligned(16))) float tiles[XH * 2 * 16 * G3_TLD];
  __shared__ float red[4 * 256];
  const int b = blockIdx.x / ntiles, tile = blockIdx.x - b * ntiles, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int fr = lane & 15, fq = lane >> 4, fk = fq * 8;
  const int i0 = tile * 16, nr = Ta - i0 < 16 ? Ta - i0 : 16;
  const long row0 = (long)b * Ta + i0;
  const unsigned long long seed_attn = mer_site_seed(dr.seed, dr.site_attn);
  const unsigned long long seed_path = mer_site_seed(dr.seed, dr.site_path);
  const float keep = dropout_scale(seed_path, b, dr.path);
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
  __syncthreads();
  {  // do2 = da2 . Wo2
    f32x4 acc[1][2];
    zero(acc);
    mm_aw(acc, d2L, LDA, 16, XD, WoT2, XD, 32 * w);
    store_acc(acc, 32 * w, nullptr, oL, LDA, nullptr, 0, 0, 16);
  }
  __syncthreads();
  // attention backward of head h = w over the sample's T keys
  const int h = w;
  float* dSt = tiles + (h * 2) * 16 * G3_TLD;
  float* Pdt = dSt + 16 * G3_TLD;
  const float* kb = kv2 + (long)b * T * 2 * XD;
  f32x4 dp = f32x4{0.f, 0.f, 0.f, 0.f};
  {  // dP' = do2_h . V2_h^T
    bf16x8 ah, al, bh, bl;
    frag_row(oL + fr * LDA + h * XDH + fk, true, ah, al);
    frag_row(kb + (long)fr * 2 * XD + XD + h * XDH + fk, fr < T, bh, bl);
    dp = mma3(ah, al, bh, bl, dp);
  }
  float pv[4], rs[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * fq + r, j = fr;
    const bool ok = (4 * fq + r) < nr && j < T;
    const long pi = (((long)b * XH + h) * Ta + i) * T + j;
    const float m = ok ? dropout_scale(seed_attn, pi, dr.attn) : 0.f;
    pv[r] = ok ? P2[pi] : 0.f;
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
      frag_col(kb + (long)fk * 2 * XD + h * XDH + 16 * jt + fr, 2 * XD, fk, T, true, bh, bl);
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
    frag_col(dSt + (long)fk * G3_TLD + fr, G3_TLD, fk, 16, true, sh, sl);
    frag_col(Pdt + (long)fk * G3_TLD + fr, G3_TLD, fk, 16, true, ph, pl);
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      bf16x8 qh, ql, gh, gl;
      frag_col(q2 + (row0 + fk) * XD + h * XDH + 16 * jt + fr, XD, fk, nr, true, qh, ql);
      frag_col(oL + fk * LDA + h * XDH + 16 * jt + fr, LDA, fk, 16, true, gh, gl);
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
}

MER_API int mer_xh_a2v_bwd(int B, int T, int Ta, const float* demb, const float* s_a, const float* mean_a,
                           const float* rstd_a, const float* gamma, const float* P2, const float* kv2, const float* q2,
                           const void* WoT2_hi, const void* WoT2_lo, float attn_p, float path_p,
                           const unsigned long long* seed, unsigned long long site_attn, unsigned long long site_path,
                           float scale, float* da, float* da2, float* dqkv, float* dkv2_part, float* ln_part,
                           void* stream) {
  if (B <= 0) return 0;
  if (T <= 0 || T > 16 || Ta <= 0 || ((attn_p > 0.f || path_p > 0.f) && !seed)) return (int)hipErrorInvalidValue;
  const int ntiles = (Ta + 15) / 16;
  XhDrop dr{attn_p, path_p, seed, site_attn, site_path};
  hipLaunchKernelGGL(xh_a2v_bwd_kernel, dim3(B * ntiles), dim3(256), 0, (hipStream_t)stream, T, Ta, ntiles, demb, s_a,
                     mean_a, rstd_a, gamma, P2, kv2, q2, SplitW{(const bf16_t*)WoT2_hi, (const bf16_t*)WoT2_lo}, dr,
                     scale, da, da2, dqkv, dkv2_part, ln_part);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// G2: v2a block backward, one workgroup per sample (T <= 16 query rows, Ta <= 160 keys), wave = head.
// Unfused: xattn_head.py:252-269 + the v-pool half of 229-231.
// ---------------------------------------------------------------------------------------------
constexpr int G2_KT = 10;               // 16-key tiles (Ta <= 160)
constexpr int G2_SLD = 16 * G2_KT + 4;  // dS / P' tile row stride
constexpr int G2_KVLD = 2 * XD + 4;

__global__ __launch_bounds__(256) void xh_v2a_bwd_kernel(
    int T, int Ta, int ntiles, int vdim, const float* __restrict__ dkv2_part, SplitW WkvT2,
    const float* __restrict__ demb, const float* __restrict__ s_v, const float* __restrict__ mean_v,
    const float* __restrict__ rstd_v, const float* __restrict__ gamma, SplitW WoT1, const float* __restrict__ P1,
    const float* __restrict__ kv1, const float* __restrict__ q1, SplitW WqT1, SplitW WvT, XhDrop dr, float scale,
    float* __restrict__ dkv2, float* __restrict__ dv2, float* __restrict__ dq1, float* __restrict__ dv,
    float* __restrict__ dvfeat, float* __restrict__ dqkv, float* __restrict__ ln_part) {
  extern __shared__ __attribute__((aligned(16))) float g2smem[];
  float* kvL = g2smem;                        // [16][G2_KVLD]  dK2 dV2
  float* t1 = kvL + 16 * G2_KVLD;             // [16][LDA]  dv1, then ds (the residual part of dv)
  float* d2L = t1 + 16 * LDA;                 // [16][LDA]  dv2
  float* oL = d2L + 16 * LDA;                 // [16][LDA]  do1, then dv
  float* dqL = oL + 16 * LDA;                 // [16][LDA]  dq1
  float* tiles = dqL + 16 * LDA;              // [XH][2][16][G2_SLD]  dS, P'
  float* red = tiles + XH * 2 * 16 * G2_SLD;  // [4][256]
  const int b = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int fr = lane & 15, fq = lane >> 4, fk = fq * 8;
  const long row0 = (long)b * T;
  const unsigned long long seed_attn = mer_site_seed(dr.seed, dr.site_attn);
  const unsigned long long seed_path = mer_site_seed(dr.seed, dr.site_path);
  const float keep = dropout_scale(seed_path, b, dr.path);
  // dK2 dV2 of this sample: the a2v tiles' partials summed in tile order
  for (int e = threadIdx.x; e < 16 * 2 * XD; e += 256) {
    const int r = e / (2 * XD), c = e - r * 2 * XD;
    float s = 0.f;
    if (r < T) {
      for (int q = 0; q < ntiles; ++q) s += dkv2_part[(((long)b * ntiles + q) * 16 + r) * 2 * XD + c];
      dkv2[(row0 + r) * 2 * XD + c] = s;
    }
    kvL[r * G2_KVLD + c] = s;
  }
  __syncthreads();
  {  // dv1 (kv2 path) = [dK2 dV2] . Wkv2
    f32x4 acc[1][2];
    zero(acc);
    mm_aw(acc, kvL, G2_KVLD, 16, 2 * XD, WkvT2, 2 * XD, 32 * w);
    store_acc(acc, 32 * w, nullptr, t1, LDA, nullptr, 0, 0, 16);
  }
  __syncthreads();
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
      }
      t1[r * LDA + lane] = ds0;
      t1[r * LDA + 64 + lane] = ds1;
      d2L[r * LDA + lane] = keep * ds0;
      d2L[r * LDA + 64 + lane] = keep * ds1;
    }
    ln_part_store(g0, g1, b0, b1, red, ln_part + (long)b * 256);
  }
  __syncthreads();
  {  // do1 = dv2 . Wo1
    f32x4 acc[1][2];
    zero(acc);
    mm_aw(acc, d2L, LDA, 16, XD, WoT1, XD, 32 * w);
    store_acc(acc, 32 * w, nullptr, oL, LDA, nullptr, 0, 0, 16);
  }
  __syncthreads();
  // attention backward, head h = w, keys = the sample's Ta rows of kv1
  const int h = w;
  float* dSt = tiles + (h * 2) * 16 * G2_SLD;
  float* Pdt = dSt + 16 * G2_SLD;
  const float* kb = kv1 + (long)b * Ta * 2 * XD;
  {
    f32x4 dp[G2_KT];
#pragma unroll
    for (int t = 0; t < G2_KT; ++t) dp[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 ah, al;
    frag_row(oL + fr * LDA + h * XDH + fk, true, ah, al);
#pragma unroll
    for (int t = 0; t < G2_KT; ++t) {  // dP' = do1_h . V1_h^T
      const int j = 16 * t + fr;
      bf16x8 bh, bl;
      frag_row(kb + (long)j * 2 * XD + XD + h * XDH + fk, j < Ta, bh, bl);
      dp[t] = mma3(ah, al, bh, bl, dp[t]);
    }
    float pv[G2_KT][4];
    float rs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < G2_KT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 4 * fq + r, j = 16 * t + fr;
        const bool ok = i < T && j < Ta;
        const long pi = (((long)b * XH + h) * T + i) * Ta + j;
        const float m = ok ? dropout_scale(seed_attn, pi, dr.attn) : 0.f;
        const float p = ok ? P1[pi] : 0.f;
        pv[t][r] = p;
        dp[t][r] *= m;  // dP
        Pdt[i * G2_SLD + j] = p * m;
        rs[r] += p * dp[t][r];
      }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) rs[r] += __shfl_xor(rs[r], o, 64);
#pragma unroll
    for (int t = 0; t < G2_KT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) dSt[(4 * fq + r) * G2_SLD + 16 * t + fr] = pv[t][r] * (dp[t][r] - rs[r]);
  }
  wave_sync_lds();
  {  // dq1_h = dS . K1_h * scale  (keys >= Ta are zero in dS and read as zero from K1)
    f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    for (int k = 0; k < 16 * G2_KT; k += 32) {
      bf16x8 ah, al;
      frag_row(dSt + fr * G2_SLD + k + fk, true, ah, al);
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        bf16x8 bh, bl;
        frag_col(kb + (long)(k + fk) * 2 * XD + h * XDH + 16 * jt + fr, 2 * XD, k + fk, Ta, true, bh, bl);
        o[jt] = mma3(ah, al, bh, bl, o[jt]);
      }
    }
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) dqL[(4 * fq + r) * LDA + h * XDH + 16 * jt + fr] = o[jt][r] * scale;
  }
  {  // dK1_h = dS^T . q1_h * scale, dV1_h = P'^T . do1_h: rows = keys, contraction over the T query rows
    bf16x8 qh[2], ql[2], gh[2], gl[2];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      frag_col(q1 + (row0 + fk) * XD + h * XDH + 16 * jt + fr, XD, fk, T, true, qh[jt], ql[jt]);
      frag_col(oL + fk * LDA + h * XDH + 16 * jt + fr, LDA, fk, 16, true, gh[jt], gl[jt]);
    }
#pragma unroll
    for (int t = 0; t < G2_KT; ++t) {
      if (16 * t >= Ta) break;
      bf16x8 sh, sl, ph, pl;
      frag_col(dSt + (long)fk * G2_SLD + 16 * t + fr, G2_SLD, fk, 16, true, sh, sl);
      frag_col(Pdt + (long)fk * G2_SLD + 16 * t + fr, G2_SLD, fk, 16, true, ph, pl);
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        const f32x4 dk = mma3(sh, sl, qh[jt], ql[jt], f32x4{0.f, 0.f, 0.f, 0.f});
        const f32x4 dvv = mma3(ph, pl, gh[jt], gl[jt], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = 16 * t + 4 * fq + r;
          if (j < Ta) {
            float* drow = dqkv + ((long)b * Ta + j) * 3 * XD;
            drow[XD + h * XDH + 16 * jt + fr] = dk[r] * scale;
            drow[2 * XD + h * XDH + 16 * jt + fr] = dvv[r];
          }
        }
      }
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < T * XD; e += 256) dq1[row0 * XD + e] = dqL[(e / XD) * LDA + e % XD];
  {  // dv = ds + dq1 . Wq1  (rows >= T of dqL are zero: dS is zero there)
    f32x4 acc[1][2];
    zero(acc);
    mm_aw(acc, dqL, LDA, 16, XD, WqT1, XD, 32 * w);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 4 * fq + r, col = 32 * w + 16 * j + fr;
        const float val = row < T ? acc[0][j][r] + t1[row * LDA + col] : 0.f;
        oL[row * LDA + col] = val;
        if (row < T) dv[(row0 + row) * XD + col] = val;
      }
  }
  __syncthreads();
  if (dvfeat) {  // dv_feat = dv . Wv  (16-column tiles round-robin over the waves)
    for (int c0 = 16 * w; c0 < vdim; c0 += 64) {
      f32x4 acc[1][1];
      zero(acc);
      mm_aw(acc, oL, LDA, 16, XD, WvT, XD, c0);
      store_acc(acc, c0, nullptr, nullptr, 0, dvfeat, vdim, row0, T);
    }
  }
}

constexpr size_t G2_LDS_BYTES = sizeof(float) * (16 * G2_KVLD + 4 * 16 * LDA + XH * 2 * 16 * G2_SLD + 4 * 256);

MER_API int mer_xh_v2a_bwd(int B, int T, int Ta, int vdim, const float* dkv2_part, const void* WkvT2_hi,
                           const void* WkvT2_lo, const float* demb, const float* s_v, const float* mean_v,
                           const float* rstd_v, const float* gamma, const void* WoT1_hi, const void* WoT1_lo,
                           const float* P1, const float* kv1, const float* q1, const void* WqT1_hi, const void* WqT1_lo,
                           const void* WvT_hi, const void* WvT_lo, float attn_p, float path_p,
                           const unsigned long long* seed, unsigned long long site_attn, unsigned long long site_path,
                           float scale, float* dkv2, float* dv2, float* dq1, float* dv, float* dvfeat, float* dqkv,
                           float* ln_part, void* stream) {
  if (B <= 0) return 0;
  if (T <= 0 || T > 16 || Ta <= 0 || Ta > 16 * G2_KT || vdim <= 0 || vdim % 16 ||
      ((attn_p > 0.f || path_p > 0.f) && !seed))
    return (int)hipErrorInvalidValue;
  XhDrop dr{attn_p, path_p, seed, site_attn, site_path};
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&xh_v2a_bwd_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)G2_LDS_BYTES) != hipSuccess)
    return (int)hipErrorInvalidConfiguration;
  hipLaunchKernelGGL(xh_v2a_bwd_kernel, dim3(B), dim3(256), G2_LDS_BYTES, (hipStream_t)stream, T, Ta, (Ta + 15) / 16,
                     vdim, dkv2_part, SplitW{(const bf16_t*)WkvT2_hi, (const bf16_t*)WkvT2_lo}, demb, s_v, mean_v,
                     rstd_v, gamma, SplitW{(const bf16_t*)WoT1_hi, (const bf16_t*)WoT1_lo}, P1, kv1, q1,
                     SplitW{(const bf16_t*)WqT1_hi, (const bf16_t*)WqT1_lo},
                     SplitW{(const bf16_t*)WvT_hi, (const bf16_t*)WvT_lo}, dr, scale, dkv2, dv2, dq1, dv, dvfeat, dqkv,
                     ln_part);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// G1: audio chain backward, 32 rows per block: da += [dq2 | dK1 dV1] . [Wq2 ; Wkv1], da_s = da . Wa
// Unfused: the dx halves of xattn_head.py:251, 269 and 303-304.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void xh_audio_bwd_kernel(int M, const float* __restrict__ dqkv, SplitW WcT,
                                                           SplitW WaT, float* __restrict__ da, float* __restrict__ da_s) {
  __shared__ __attribute__((aligned(16))) float daL[32 * LDA];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
  const long r0 = (long)blockIdx.x * 32;
  const int rmax = (int)(M - r0 < 32 ? M - r0 : 32);
  {
    f32x4 acc[2][2];
    zero(acc);
    mm_aw(acc, dqkv + r0 * 3 * XD, 3 * XD, rmax, 3 * XD, WcT, 3 * XD, 32 * w);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * i + 4 * fq + r, col = 32 * w + 16 * j + fr;
          float v = 0.f;
          if (row < rmax) {
            v = acc[i][j][r] + da[(r0 + row) * XD + col];
            da[(r0 + row) * XD + col] = v;
          }
          daL[row * LDA + col] = v;
        }
  }
  __syncthreads();
  f32x4 acc[2][2];
  zero(acc);
  mm_aw(acc, daL, LDA, 32, XD, WaT, XD, 32 * w);
  store_acc(acc, 32 * w, nullptr, nullptr, 0, da_s, XD, r0, rmax);
}

MER_API int mer_xh_audio_bwd(int M, const float* dqkv, const void* WcT_hi, const void* WcT_lo, const void* WaT_hi,
                             const void* WaT_lo, float* da, float* da_s, void* stream) {
  if (M <= 0) return 0;
  hipLaunchKernelGGL(xh_audio_bwd_kernel, dim3((M + 31) / 32), dim3(256), 0, (hipStream_t)stream, M, dqkv,
                     SplitW{(const bf16_t*)WcT_hi, (const bf16_t*)WcT_lo},
                     SplitW{(const bf16_t*)WaT_hi, (const bf16_t*)WaT_lo}, da, da_s);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// W: grouped weight gradients.  Problem p: dW[n][k] (+)= sum_m dY[m][n] X[m][k] and db[n] (+)= sum_m dY[m][n]
// (K = 0: a column-sum-only problem, the LayerNorm dgamma / dbeta partials).  Blocks = (problem, 64 x 64
// output tile, row split); each writes its partial tile to ws, the bias partials (k-tile 0 blocks) after it;
// xh_wfold adds the partials in split order.  The table travels by value in the kernel arguments, so a
// captured graph holds it (no device table to upload).
// ---------------------------------------------------------------------------------------------
constexpr int WG_MAXP = 16;
constexpr int WG_LD = 64 + 4;
constexpr int WG_HOST_COLS = 11;  // dY ldy X ldx x_dtype M N K splits dW db

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
};

__global__ __launch_bounds__(256) void xh_wgrad_kernel(const WgTab tab, float* __restrict__ ws) {
  __shared__ __attribute__((aligned(16))) float yT[32 * WG_LD];
  __shared__ __attribute__((aligned(16))) float xT[32 * WG_LD];
  int pi = 0;
  while (pi + 1 < tab.nprob && tab.p[pi + 1].first_block <= (int)blockIdx.x) ++pi;
  const WgProb& d = tab.p[pi];
  const int N = d.N, K = d.K, splits = d.splits;
  const int ntk = K > 0 ? (K + 63) / 64 : 1;
  const int local = blockIdx.x - d.first_block;
  const int split = local % splits, tile = local / splits;
  const int tn = tile / ntk, tk = tile - tn * ntk;
  const int n0 = tn * 64, k0 = tk * 64;
  const long per = (d.M + splits - 1) / splits, m0 = split * per, m1 = m0 + per < d.M ? m0 + per : d.M;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4, fk = fq * 8;
  const bool bias = d.db != nullptr && tk == 0;
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;  // threads 0..63: column n0 + t of dY summed over the block's rows
  for (long mc = m0; mc < m1; mc += 32) {
    __syncthreads();
    for (int e = threadIdx.x; e < 32 * 64; e += 256) {
      const int r = e >> 6, c = e & 63;
      const long m = mc + r;
      const bool okm = m < m1;
      yT[r * WG_LD + c] = (okm && n0 + c < N) ? d.dY[m * d.ldy + n0 + c] : 0.f;
      float xv = 0.f;
      if (okm && k0 + c < K)
        xv = d.xbf ? bf2f(reinterpret_cast<const bf16_t*>(d.X)[m * d.ldx + k0 + c])
                   : reinterpret_cast<const float*>(d.X)[m * d.ldx + k0 + c];
      xT[r * WG_LD + c] = xv;
    }
    __syncthreads();
    if (bias && threadIdx.x < 64)
      for (int r = 0; r < 32; ++r) bsum += yT[r * WG_LD + threadIdx.x];
    if (K > 0) {
      bf16x8 ah, al;
      frag_col(yT + fk * WG_LD + 16 * w + fr, WG_LD, 0, 32, true, ah, al);  // A[n][m] = dY[m][n]
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bf16x8 bh, bl;
        frag_col(xT + fk * WG_LD + 16 * j + fr, WG_LD, 0, 32, true, bh, bl);  // B[k][m] = X[m][k]
        acc[j] = d.xbf ? mma(al, bh, mma(ah, bh, acc[j])) : mma3(ah, al, bh, bl, acc[j]);
      }
    }
  }
  if (K > 0) {
    float* out = ws + d.ws_off + (long)split * N * K;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + 16 * w + 4 * fq + r, k = k0 + 16 * j + fr;
        if (n < N && k < K) out[(long)n * K + k] = acc[j][r];
      }
  }
  if (bias && threadIdx.x < 64 && n0 + (int)threadIdx.x < N) ws[d.ws_b_off + (long)split * N + n0 + threadIdx.x] = bsum;
}

__global__ __launch_bounds__(256) void xh_wfold_kernel(const WgTab tab, const float* __restrict__ ws) {
  const WgProb& d = tab.p[blockIdx.y];
  const long nk = (long)d.N * d.K, tot = nk + (d.db ? d.N : 0);
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < tot; e += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    if (e < nk) {
      for (int q = 0; q < d.splits; ++q) s += ws[d.ws_off + q * nk + e];
      d.dW[e] += s;
    } else {
      const long n = e - nk;
      for (int q = 0; q < d.splits; ++q) s += ws[d.ws_b_off + (long)q * d.N + n];
      d.db[n] += s;
    }
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
    if (p.M <= 0 || p.N <= 0 || p.K < 0 || p.splits <= 0 || p.splits > p.M || !p.dY ||
        (p.K > 0 && (!p.X || !p.dW)) || (p.K == 0 && !p.db))
      return -1;
    p.ws_off = off;
    off += (long long)p.splits * p.N * p.K;
    p.ws_b_off = off;
    if (p.db) off += (long long)p.splits * p.N;
    p.first_block = fb;
    fb += p.splits * ((p.N + 63) / 64) * (p.K > 0 ? (p.K + 63) / 64 : 1);
  }
  tab->nprob = nprob;
  *blocks = fb;
  return off;
}

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
  hipLaunchKernelGGL(xh_wgrad_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, tab, ws);
  hipLaunchKernelGGL(xh_wfold_kernel, dim3(32, nprob), dim3(256), 0, (hipStream_t)stream, tab, ws);
  MER_LAUNCH_CHECK();
}
