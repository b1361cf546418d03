// Emotion-prior attention bias of the xattn head (EmotionPriorBiasAdapter, fusion.py:153-184, used at fusion.py:390-391)
// as ONE forward and ONE backward launch per batch, one workgroup per sample, exact fp32 FMA.  The unfused schedule
// (xattn_head.prior_forward / prior_backward) is ~14 forward and ~20 backward launches of tiny matvecs: on the fused
// head's dependent chain they cost the step ~6 % (C4 sweep: xattn+prior 180 vs xattn 192 steps/s, round 4).
//
// Forward, sample b (v: [T][d], a: [Ta][d] pre-attention tokens, d = 128):
//   pg = [mean_t v | mean_j a],  h1 = dropout(relu(pg W0^T + b0)),  prior = h1 W3^T + b3
//   token-bias Linears h = 0 v_query, 1 a_key, 2 a_query, 3 v_key over cat([token, prior]) (fusion.py:170-176):
//     tt_h[token] = token . w_h[:d],  tp_h = prior . w_h[d:] + b_h
//   v2a_bias[i][j] = tanh(tt_0[i] + tt_1[j] + (tp_0 + tp_1)) * scale   (query frame i, key audio token j)
//   a2v_bias[j][i] = tanh(tt_2[j] + tt_3[i] + (tp_2 + tp_3)) * scale
// Backward: g = dbias * scale * (1 - tanh^2) -> dtt (row / column sums of g), dtp (sum of g), dscale partial
// (sum dbias * tanh), dprior, dh1 (through the ReLU / dropout mask), dpg, and the token gradients added into dv / da
// (token-bias Linears + the mean pools).  The weight gradients are the grouped weight-gradient launch's problems
// (xattn_fused.py: (dh1, pg), (dprior, h1), (dtt_h, tokens), (dtp_h, prior), column sums of dscale).
// Saved tensors use the unfused schedule's names and layouts, so either backward runs on either forward.
#include "common.h"
#include "mer.h"

namespace {

constexpr int PR_D = 128, PR_MAXT = 16, PR_MAXTA = 160, PR_MAXH1 = 256, PR_MAXPD = 16;

struct PriorHeads {
  const float* w[4];  // [d + PD] each (the Linear's single output row)
  const float* b[4];  // [1]
};

__global__ __launch_bounds__(256) void xh_prior_fwd_kernel(int T, int Ta, int H1, int PD, const float* __restrict__ v,
                                                           const float* __restrict__ a, const float* __restrict__ W0,
                                                           const float* __restrict__ b0, const float* __restrict__ W3,
                                                           const float* __restrict__ b3, PriorHeads hw,
                                                           const float* __restrict__ scale, float p,
                                                           const unsigned long long* __restrict__ seed_ptr,
                                                           unsigned long long site, float* __restrict__ pg,
                                                           float* __restrict__ h1, float* __restrict__ prior,
                                                           float* tt0, float* tt1, float* tt2, float* tt3, float* tp0,
                                                           float* tp1, float* tp2, float* tp3,
                                                           float* __restrict__ v2a_bias, float* __restrict__ a2v_bias) {
  __shared__ float s_pg[2 * PR_D], s_h1[PR_MAXH1], s_pr[PR_MAXPD], s_tt[4][PR_MAXTA], s_tp[4];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  float* const tt[4] = {tt0, tt1, tt2, tt3};
  float* const tp[4] = {tp0, tp1, tp2, tp3};
  // pooled means (temporal.py:108-109 via fusion.py:178-181): thread t < 128 -> v column t, else a column t - 128;
  // two partial sums over alternating rows keep two loads in flight per step
  {
    const bool vside = t < PR_D;
    const int c = vside ? t : t - PR_D, L = vside ? T : Ta;
    const float* x = (vside ? v + (long)b * T * PR_D : a + (long)b * Ta * PR_D) + c;
    float s0 = 0.f, s1 = 0.f;
    int l = 0;
    for (; l + 2 <= L; l += 2) {
      s0 += x[(long)l * PR_D];
      s1 += x[(long)(l + 1) * PR_D];
    }
    if (l < L) s0 += x[(long)l * PR_D];
    const float m = (s0 + s1) / L;
    s_pg[t] = m;
    pg[(long)b * 2 * PR_D + t] = m;
  }
  __syncthreads();
  // prior_net.0 + ReLU + Dropout: one wave per hidden unit, k across the lanes
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  for (int j = w; j < H1; j += 4) {
    float s = 0.f;
    for (int k = lane; k < 2 * PR_D; k += 64) s += W0[(long)j * 2 * PR_D + k] * s_pg[k];
    s = wave_sum(s);
    if (lane == 0) {
      float hv = fmaxf(s + b0[j], 0.f);
      if (p > 0.f) hv *= dropout_scale(seed, (uint64_t)b * H1 + j, p);
      s_h1[j] = hv;
      h1[(long)b * H1 + j] = hv;
    }
  }
  __syncthreads();
  // prior_net.3
  for (int k = w; k < PD; k += 4) {
    float s = 0.f;
    for (int j = lane; j < H1; j += 64) s += W3[(long)k * H1 + j] * s_h1[j];
    s = wave_sum(s);
    if (lane == 0) {
      s_pr[k] = s + b3[k];
      prior[(long)b * PD + k] = s + b3[k];
    }
  }
  __syncthreads();
  // prior halves of the four token-bias Linears: wave h
  {
    float s = lane < PD ? hw.w[w][PR_D + lane] * s_pr[lane] : 0.f;
    s = wave_sum(s);
    if (lane == 0) {
      s_tp[w] = s + hw.b[w][0];
      tp[w][b] = s + hw.b[w][0];
    }
  }
  // token halves: one wave per token row, both heads reading that row (v rows: heads 0, 3; a rows: heads 1, 2)
  for (int r = w; r < T + Ta; r += 4) {
    const bool vrow = r < T;
    const float* x = vrow ? v + ((long)b * T + r) * PR_D : a + ((long)b * Ta + (r - T)) * PR_D;
    const int hA = vrow ? 0 : 1, hB = vrow ? 3 : 2;
    const float x0 = x[lane], x1 = x[lane + 64];
    float sA = x0 * hw.w[hA][lane] + x1 * hw.w[hA][lane + 64];
    float sB = x0 * hw.w[hB][lane] + x1 * hw.w[hB][lane + 64];
    sA = wave_sum(sA);
    sB = wave_sum(sB);
    if (lane == 0) {
      const int i = vrow ? r : r - T;
      const long o = (long)b * (vrow ? T : Ta) + i;
      s_tt[hA][i] = sA;
      s_tt[hB][i] = sB;
      tt[hA][o] = sA;
      tt[hB][o] = sB;
    }
  }
  __syncthreads();
  const float sc = *scale, base1 = s_tp[0] + s_tp[1], base2 = s_tp[2] + s_tp[3];
  for (int e = t; e < T * Ta; e += 256) {
    const int i = e / Ta, j = e - i * Ta;
    v2a_bias[(long)b * T * Ta + e] = tanhf(s_tt[0][i] + s_tt[1][j] + base1) * sc;
  }
  for (int e = t; e < Ta * T; e += 256) {
    const int j = e / T, i = e - j * T;
    a2v_bias[(long)b * Ta * T + e] = tanhf(s_tt[2][j] + s_tt[3][i] + base2) * sc;
  }
}

__global__ __launch_bounds__(256) void xh_prior_bwd_kernel(
    int T, int Ta, int H1, int PD, const float* __restrict__ dbias1, const float* __restrict__ dbias2,
    const float* tt0, const float* tt1, const float* tt2, const float* tt3, const float* tp0, const float* tp1,
    const float* tp2, const float* tp3, const float* __restrict__ scale, PriorHeads hw, const float* __restrict__ W0,
    const float* __restrict__ W3, const float* __restrict__ h1, float p, const unsigned long long* __restrict__ seed_ptr,
    unsigned long long site, float* dtt0, float* dtt1, float* dtt2, float* dtt3, float* dtp0, float* dtp1, float* dtp2,
    float* dtp3, float* __restrict__ dprior, float* __restrict__ dh1, float* __restrict__ dscale_part,
    float* __restrict__ dv, float* __restrict__ da) {
  __shared__ float g1[PR_MAXT * PR_MAXTA], g2[PR_MAXT * PR_MAXTA];  // g of v2a [T][Ta] and a2v [Ta][T]
  __shared__ float s_dtt[4][PR_MAXTA], s_dpr[PR_MAXPD], s_dh1[PR_MAXH1], s_dpg[2 * PR_D], red[3][4];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const float* const tt[4] = {tt0, tt1, tt2, tt3};
  const float* const tp[4] = {tp0, tp1, tp2, tp3};
  float* const dtt[4] = {dtt0, dtt1, dtt2, dtt3};
  float* const dtp[4] = {dtp0, dtp1, dtp2, dtp3};
  const float sc = *scale;
  const float base1 = tp[0][b] + tp[1][b], base2 = tp[2][b] + tp[3][b];
  float dsc = 0.f;
  for (int e = t; e < T * Ta; e += 256) {
    const int i = e / Ta, j = e - i * Ta;
    const float th = tanhf(tt[0][(long)b * T + i] + tt[1][(long)b * Ta + j] + base1);
    const float d = dbias1[(long)b * T * Ta + e];
    g1[e] = d * sc * (1.f - th * th);
    dsc += d * th;
  }
  for (int e = t; e < Ta * T; e += 256) {
    const int j = e / T, i = e - j * T;
    const float th = tanhf(tt[2][(long)b * Ta + j] + tt[3][(long)b * T + i] + base2);
    const float d = dbias2[(long)b * Ta * T + e];
    g2[e] = d * sc * (1.f - th * th);
    dsc += d * th;
  }
  __syncthreads();
  // row / column sums: dtt_0[i] = sum_j g1[i][j], dtt_1[j] = sum_i g1[i][j], dtt_2[j] = sum_i g2[j][i],
  // dtt_3[i] = sum_j g2[j][i]
  float tot1 = 0.f, tot2 = 0.f;
  for (int i = w; i < T; i += 4) {
    float s = 0.f;
    for (int j = lane; j < Ta; j += 64) s += g1[i * Ta + j];
    s = wave_sum(s);
    if (lane == 0) s_dtt[0][i] = s;
    tot1 += lane == 0 ? s : 0.f;
  }
  for (int j = t; j < Ta; j += 256) {
    float s1 = 0.f, s2 = 0.f;
    for (int i = 0; i < T; ++i) {
      s1 += g1[i * Ta + j];
      s2 += g2[j * T + i];
    }
    s_dtt[1][j] = s1;
    s_dtt[2][j] = s2;
    tot2 += s2;
  }
  if (t < T) {
    float s = 0.f;
    for (int j = 0; j < Ta; ++j) s += g2[j * T + t];
    s_dtt[3][t] = s;
  }
  tot1 = wave_sum(tot1);
  tot2 = wave_sum(tot2);
  dsc = wave_sum(dsc);
  if (lane == 0) {
    red[0][w] = tot1;
    red[1][w] = tot2;
    red[2][w] = dsc;
  }
  __syncthreads();
  const float T1 = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  const float T2 = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  if (t == 0) {
    dtp[0][b] = T1;
    dtp[1][b] = T1;
    dtp[2][b] = T2;
    dtp[3][b] = T2;
    dscale_part[b] = (red[2][0] + red[2][1]) + (red[2][2] + red[2][3]);
  }
  for (int i = t; i < T; i += 256) {
    dtt[0][(long)b * T + i] = s_dtt[0][i];
    dtt[3][(long)b * T + i] = s_dtt[3][i];
  }
  for (int j = t; j < Ta; j += 256) {
    dtt[1][(long)b * Ta + j] = s_dtt[1][j];
    dtt[2][(long)b * Ta + j] = s_dtt[2][j];
  }
  // dprior[k] = sum_h dtp_h w_h[d + k]
  if (t < PD) {
    const float dp = ((T1 * hw.w[0][PR_D + t] + T1 * hw.w[1][PR_D + t]) + T2 * hw.w[2][PR_D + t]) + T2 * hw.w[3][PR_D + t];
    s_dpr[t] = dp;
    dprior[(long)b * PD + t] = dp;
  }
  __syncthreads();
  // dh1 = W3^T dprior through ReLU + dropout (relu_dropout_bwd: zero where the saved, dropped-out output is <= 0)
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  for (int j = t; j < H1; j += 256) {
    float s = 0.f;
    for (int k = 0; k < PD; ++k) s += W3[(long)k * H1 + j] * s_dpr[k];
    const float hv = h1[(long)b * H1 + j];
    s = hv > 0.f ? s * dropout_scale(seed, (uint64_t)b * H1 + j, p) : 0.f;
    s_dh1[j] = s;
    dh1[(long)b * H1 + j] = s;
  }
  __syncthreads();
  // dpg = W0^T dh1 (thread t: column t of W0 [H1][2d])
  {
    float s = 0.f;
    for (int j = 0; j < H1; ++j) s += W0[(long)j * 2 * PR_D + t] * s_dh1[j];
    s_dpg[t] = s;
  }
  __syncthreads();
  // token gradients: dv[b, i, c] += dtt_0[i] w_0[c] + dtt_3[i] w_3[c] + dpg[c] / T;
  //                  da[b, j, c] += dtt_1[j] w_1[c] + dtt_2[j] w_2[c] + dpg[d + c] / Ta
  for (int e = t; e < (T + Ta) * PR_D; e += 256) {
    const int r = e / PR_D, c = e - r * PR_D;
    if (r < T) {
      float* o = dv + ((long)b * T + r) * PR_D + c;
      *o += (s_dtt[0][r] * hw.w[0][c] + s_dtt[3][r] * hw.w[3][c]) + s_dpg[c] / T;
    } else {
      const int j = r - T;
      float* o = da + ((long)b * Ta + j) * PR_D + c;
      *o += (s_dtt[1][j] * hw.w[1][c] + s_dtt[2][j] * hw.w[2][c]) + s_dpg[PR_D + c] / Ta;
    }
  }
}

bool prior_dims_ok(int T, int Ta, int d, int H1, int PD) {
  return d == PR_D && T >= 1 && T <= PR_MAXT && Ta >= 1 && Ta <= PR_MAXTA && H1 >= 1 && H1 <= PR_MAXH1 && PD >= 1 &&
         PD <= PR_MAXPD;
}

}  // namespace

MER_API int mer_xh_prior_fwd(int B, int T, int Ta, int d, int H1, int PD, const float* v, const float* a,
                             const float* W0, const float* b0, const float* W3, const float* b3, const float* w_vq,
                             const float* b_vq, const float* w_ak, const float* b_ak, const float* w_aq,
                             const float* b_aq, const float* w_vk, const float* b_vk, const float* scale, float drop_p,
                             const unsigned long long* seed, unsigned long long site, float* pg, float* h1,
                             float* prior, float* tt_vq, float* tt_ak, float* tt_aq, float* tt_vk, float* tp_vq,
                             float* tp_ak, float* tp_aq, float* tp_vk, float* v2a_bias, float* a2v_bias,
                             void* stream) {
  if (B <= 0) return 0;
  if (!prior_dims_ok(T, Ta, d, H1, PD) || drop_p < 0.f || drop_p >= 1.f || (drop_p > 0.f && !seed))
    return (int)hipErrorInvalidValue;
  const PriorHeads hw{{w_vq, w_ak, w_aq, w_vk}, {b_vq, b_ak, b_aq, b_vk}};
  hipLaunchKernelGGL(xh_prior_fwd_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, T, Ta, H1, PD, v, a, W0, b0, W3,
                     b3, hw, scale, drop_p, seed, site, pg, h1, prior, tt_vq, tt_ak, tt_aq, tt_vk, tp_vq, tp_ak, tp_aq,
                     tp_vk, v2a_bias, a2v_bias);
  MER_LAUNCH_CHECK();
}

MER_API int mer_xh_prior_bwd(int B, int T, int Ta, int d, int H1, int PD, const float* dbias_v2a, const float* dbias_a2v,
                             const float* tt_vq, const float* tt_ak, const float* tt_aq, const float* tt_vk,
                             const float* tp_vq, const float* tp_ak, const float* tp_aq, const float* tp_vk,
                             const float* scale, const float* w_vq, const float* w_ak, const float* w_aq,
                             const float* w_vk, const float* W0, const float* W3, const float* h1, float drop_p,
                             const unsigned long long* seed, unsigned long long site, float* dtt_vq, float* dtt_ak,
                             float* dtt_aq, float* dtt_vk, float* dtp_vq, float* dtp_ak, float* dtp_aq, float* dtp_vk,
                             float* dprior, float* dh1, float* dscale_part, float* dv, float* da, void* stream) {
  if (B <= 0) return 0;
  if (!prior_dims_ok(T, Ta, d, H1, PD) || drop_p < 0.f || drop_p >= 1.f || (drop_p > 0.f && !seed))
    return (int)hipErrorInvalidValue;
  const PriorHeads hw{{w_vq, w_ak, w_aq, w_vk}, {nullptr, nullptr, nullptr, nullptr}};
  hipLaunchKernelGGL(xh_prior_bwd_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, T, Ta, H1, PD, dbias_v2a,
                     dbias_a2v, tt_vq, tt_ak, tt_aq, tt_vk, tp_vq, tp_ak, tp_aq, tp_vk, scale, hw, W0, W3, h1, drop_p,
                     seed, site, dtt_vq, dtt_ak, dtt_aq, dtt_vk, dtp_vq, dtp_ak, dtp_aq, dtp_vk, dprior, dh1,
                     dscale_part, dv, da);
  MER_LAUNCH_CHECK();
}
