// CLIP-style audio/video alignment loss (fusion.py:127-150 ClipStyleAlignment.forward after its two
// projections, consumed by train.py:221-225 as loss = cls + w * align):
//
//   a_n = a / max(|a|, 1e-12),  v_n = v / max(|v|, 1e-12)            (F.normalize, dim=-1)
//   s   = min(exp(logit_scale), 100)
//   L   = s * a_n v_n^T                                              [B, B]
//   loss = 0.5 * (CE(L, arange(B)) + CE(L^T, arange(B)))             (mean reductions)
//
// B x B with B <= a few hundred and D = align_dim (256): one workgroup does the whole thing (a latency-
// bound ~10 us launch; the projections around it run on the fp32 GEMM).  Exact fp32, fixed reduction
// order (deterministic).  Backward recomputes the row / column softmaxes from the saved logits.
#include "common.h"
#include "mer.h"

namespace {

constexpr int AL_NT = 256, AL_WAVES = AL_NT / 64;

__global__ __launch_bounds__(AL_NT) void clip_align_fwd_kernel(int B, int D, const float* __restrict__ a,
                                                               const float* __restrict__ v,
                                                               const float* __restrict__ log_scale,
                                                               float* __restrict__ an, float* __restrict__ vn,
                                                               float* __restrict__ norms, float* __restrict__ logits,
                                                               float* __restrict__ loss) {
  __shared__ float red[AL_WAVES];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int r = w; r < 2 * B; r += AL_WAVES) {
    const float* x = r < B ? a + (long)r * D : v + (long)(r - B) * D;
    float* y = r < B ? an + (long)r * D : vn + (long)(r - B) * D;
    float s = 0.f;
    for (int k = lane; k < D; k += 64) s += x[k] * x[k];
    s = wave_sum(s);
    const float n = fmaxf(sqrtf(s), 1e-12f);
    for (int k = lane; k < D; k += 64) y[k] = x[k] / n;
    if (lane == 0) norms[r] = n;
  }
  __syncthreads();
  const float scale = fminf(expf(*log_scale), 100.f);
  for (int e = t; e < B * B; e += AL_NT) {
    const int i = e / B, j = e - i * B;
    const float* x = an + (long)i * D;
    const float* y = vn + (long)j * D;
    float s = 0.f;
    for (int k = 0; k < D; ++k) s = fmaf(x[k], y[k], s);
    logits[e] = scale * s;
  }
  __syncthreads();
  float acc = 0.f;  // wave-local sum of the row (r < B) and column (r >= B) CE terms
  for (int r = w; r < 2 * B; r += AL_WAVES) {
    const bool row = r < B;
    const int i = row ? r : r - B;
    float m = -INFINITY;
    for (int k = lane; k < B; k += 64) m = fmaxf(m, row ? logits[(long)i * B + k] : logits[(long)k * B + i]);
    m = wave_max(m);
    float s = 0.f;
    for (int k = lane; k < B; k += 64) s += __expf((row ? logits[(long)i * B + k] : logits[(long)k * B + i]) - m);
    s = wave_sum(s);
    acc += m + logf(s) - logits[(long)i * B + i];
  }
  if (lane == 0) red[w] = acc;
  __syncthreads();
  if (t == 0) {
    float tot = 0.f;
    for (int q = 0; q < AL_WAVES; ++q) tot += red[q];
    *loss = 0.5f * tot / (float)B;
  }
}

// dlogits[i][j] = g * 0.5 / B * (Prow[i][j] + Pcol[i][j] - 2 [i == j]);  dS = s * dlogits
__global__ __launch_bounds__(AL_NT) void clip_align_bwd_kernel(int B, int D, const float* __restrict__ an,
                                                               const float* __restrict__ vn,
                                                               const float* __restrict__ norms,
                                                               const float* __restrict__ logits,
                                                               const float* __restrict__ log_scale,
                                                               const float* __restrict__ dloss, float* __restrict__ ws,
                                                               float* __restrict__ da, float* __restrict__ dv,
                                                               float* __restrict__ dlog_scale) {
  extern __shared__ float sh[];  // lse_row[B], lse_col[B], red[AL_WAVES]
  float* lse_r = sh;
  float* lse_c = sh + B;
  float* red = sh + 2 * B;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int r = w; r < 2 * B; r += AL_WAVES) {
    const bool row = r < B;
    const int i = row ? r : r - B;
    float m = -INFINITY;
    for (int k = lane; k < B; k += 64) m = fmaxf(m, row ? logits[(long)i * B + k] : logits[(long)k * B + i]);
    m = wave_max(m);
    float s = 0.f;
    for (int k = lane; k < B; k += 64) s += __expf((row ? logits[(long)i * B + k] : logits[(long)k * B + i]) - m);
    s = wave_sum(s);
    if (lane == 0) (row ? lse_r : lse_c)[i] = m + logf(s);
  }
  __syncthreads();
  const float g = *dloss;
  const float scale = fminf(expf(*log_scale), 100.f);
  const float c = g * 0.5f / (float)B;
  float dsc = 0.f;  // sum dlogits * S
  for (int e = t; e < B * B; e += AL_NT) {
    const int i = e / B, j = e - i * B;
    const float l = logits[e];
    const float dl = c * (__expf(l - lse_r[i]) + __expf(l - lse_c[j]) - (i == j ? 2.f : 0.f));
    dsc += dl * (l / scale);
    ws[e] = dl * scale;  // dS
  }
  dsc = wave_sum(dsc);
  if (lane == 0) red[w] = dsc;
  __syncthreads();
  if (t == 0 && dlog_scale) {
    float tot = 0.f;
    for (int q = 0; q < AL_WAVES; ++q) tot += red[q];
    // d/d logit_scale of min(exp(ls), 100): exp(ls) while unclamped (torch clamp passes x <= max)
    *dlog_scale += expf(*log_scale) <= 100.f ? tot * scale : 0.f;
  }
  // da_n[i] = sum_j dS[i][j] vn[j];  dv_n[j] = sum_i dS[i][j] an[i];  then the normalize backward
  for (int r = w; r < 2 * B; r += AL_WAVES) {
    const bool row = r < B;
    const int i = row ? r : r - B;
    const float* y = row ? an + (long)i * D : vn + (long)i * D;
    float* dx = row ? da + (long)i * D : dv + (long)i * D;
    float dot = 0.f;
    for (int k = lane; k < D; k += 64) {
      float s = 0.f;
      for (int q = 0; q < B; ++q)
        s = fmaf(row ? ws[(long)i * B + q] : ws[(long)q * B + i], row ? vn[(long)q * D + k] : an[(long)q * D + k], s);
      dx[k] = s;
      dot = fmaf(s, y[k], dot);
    }
    dot = wave_sum(dot);
    const float n = norms[r];
    const bool clamped = n <= 1e-12f;
    for (int k = lane; k < D; k += 64) dx[k] = clamped ? dx[k] / n : (dx[k] - y[k] * dot) / n;
  }
}

}  // namespace

MER_API int mer_clip_align_fwd(int B, int D, const float* a, const float* v, const float* log_scale, float* an,
                               float* vn, float* norms, float* logits, float* loss, void* stream) {
  if (B <= 0 || D <= 0 || B > 4096) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(clip_align_fwd_kernel, dim3(1), dim3(AL_NT), 0, (hipStream_t)stream, B, D, a, v, log_scale, an,
                     vn, norms, logits, loss);
  MER_LAUNCH_CHECK();
}

MER_API int mer_clip_align_bwd(int B, int D, const float* an, const float* vn, const float* norms, const float* logits,
                               const float* log_scale, const float* dloss, float* ws, float* da, float* dv,
                               float* dlog_scale, void* stream) {
  if (B <= 0 || D <= 0 || B > 4096) return (int)hipErrorInvalidValue;
  const size_t sh = (2 * (size_t)B + AL_WAVES) * sizeof(float);
  hipLaunchKernelGGL(clip_align_bwd_kernel, dim3(1), dim3(AL_NT), sh, (hipStream_t)stream, B, D, an, vn, norms, logits,
                     log_scale, dloss, ws, da, dv, dlog_scale);
  MER_LAUNCH_CHECK();
}

// out = x + w * y over device scalars (train.py:225 loss = cls_loss + fusion_align_weight * align_loss)
__global__ void add_scaled_scalar_kernel(const float* x, const float* y, float w, float* out) { *out = *x + w * *y; }

MER_API int mer_add_scaled_scalar(const float* x, const float* y, float w, float* out, void* stream) {
  hipLaunchKernelGGL(add_scaled_scalar_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, x, y, w, out);
  MER_LAUNCH_CHECK();
}
