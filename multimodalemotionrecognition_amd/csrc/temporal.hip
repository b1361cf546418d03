// Temporal pooling kernels (src/models/temporal.py): the attention pooler (TemporalAttentionPooling,
// temporal.py:9-26) and the pieces of the pre-LN transformer pooler (TemporalTransformerPooling,
// temporal.py:46-75) that the fp32 head kernels (GEMM, LayerNorm, MHA) do not already cover.  fp32.
#include "common.h"
#include "mer.h"

// ---------------------------------------------------------------------------------------
// y = dropout(gelu(z)) (nn.GELU exact erf + nn.Dropout, temporal.py:18-19 and the encoder layer's
// linear1 -> activation -> dropout, TORCH TransformerEncoderLayer._ff_block); and its backward
// dz = dy * mask * gelu'(z).  Row-strided matrices; mask index = row * cols + col.
// ---------------------------------------------------------------------------------------
__global__ void gelu_dropout_fwd_kernel(int rows, int cols, const float* __restrict__ z, long ldz,
                                        float* __restrict__ y, long ldy, float p,
                                        const unsigned long long* __restrict__ seed_ptr, unsigned long long site) {
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  const long n = (long)rows * cols;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int r = (int)(e / cols), c = (int)(e - (long)r * cols);
    y[(long)r * ldy + c] = gelu_erf(z[(long)r * ldz + c]) * dropout_scale(seed, e, p);
  }
}
MER_API int mer_gelu_dropout_fwd(int rows, int cols, const float* z, long ldz, float* y, long ldy, float p,
                                 const unsigned long long* seed, unsigned long long site, void* stream) {
  const long n = (long)rows * cols;
  if (n <= 0) return 0;
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(gelu_dropout_fwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, rows, cols, z, ldz, y,
                     ldy, p, seed, site);
  MER_LAUNCH_CHECK();
}

__global__ void gelu_dropout_bwd_kernel(int rows, int cols, const float* __restrict__ dy, long lddy,
                                        const float* __restrict__ z, long ldz, float* __restrict__ dz, long lddz,
                                        float p, const unsigned long long* __restrict__ seed_ptr,
                                        unsigned long long site) {
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  const long n = (long)rows * cols;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int r = (int)(e / cols), c = (int)(e - (long)r * cols);
    dz[(long)r * lddz + c] = dy[(long)r * lddy + c] * dropout_scale(seed, e, p) * gelu_erf_grad(z[(long)r * ldz + c]);
  }
}
MER_API int mer_gelu_dropout_bwd(int rows, int cols, const float* dy, long lddy, const float* z, long ldz, float* dz,
                                 long lddz, float p, const unsigned long long* seed, unsigned long long site,
                                 void* stream) {
  const long n = (long)rows * cols;
  if (n <= 0) return 0;
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(gelu_dropout_bwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, rows, cols, dy, lddy, z,
                     ldz, dz, lddz, p, seed, site);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// y[i] = x[i] + dropout(r[i % r_period]) over rows of `cols` contiguous floats: the encoder layer's
// residuals x + dropout1(sa) / x + dropout2(ff) (r_period = rows) and the sinusoidal positional
// encoding x + pe[t] (temporal.py:42-43, r_period = L, p = 0).  In-place (y == x) is allowed.
// ---------------------------------------------------------------------------------------
__global__ void add_dropout_kernel(int rows, int cols, const float* x, const float* __restrict__ r, int r_period,
                                   float p, const unsigned long long* __restrict__ seed_ptr, unsigned long long site,
                                   float* y) {
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  const long n = (long)rows * cols;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int row = (int)(e / cols), c = (int)(e - (long)row * cols);
    y[e] = x[e] + r[(long)(row % r_period) * cols + c] * dropout_scale(seed, e, p);
  }
}
MER_API int mer_add_dropout(int rows, int cols, const float* x, const float* r, int r_period, float p,
                            const unsigned long long* seed, unsigned long long site, float* y, void* stream) {
  const long n = (long)rows * cols;
  if (n <= 0) return 0;
  if (r_period <= 0) return (int)hipErrorInvalidValue;
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(add_dropout_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, rows, cols, x, r, r_period, p,
                     seed, site, y);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// Attention pooling tail (temporal.py:23-26): a[b,:] = softmax_L(s[b,:]); y[b] = sum_l a[b,l] x[b,l,:].
// One block per sample; the L scores live in LDS (L <= 4096).  a is saved for backward.
// Backward: dx[b,l,:] (+)= a[b,l] dy[b];  ds[b,l] = a[b,l] (g_l - sum_l' a[b,l'] g_l'),  g_l = dy[b] . x[b,l].
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void attn_pool_fwd_kernel(int L, int D, const float* __restrict__ x,
                                                            const float* __restrict__ s, float* __restrict__ a,
                                                            float* __restrict__ y, long ldy) {
  extern __shared__ float sa[];  // [L]
  __shared__ float red[4];
  const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float mx = -INFINITY;
  for (int l = threadIdx.x; l < L; l += 256) {
    sa[l] = s[(long)b * L + l];
    mx = fmaxf(mx, sa[l]);
  }
  mx = wave_max(mx);
  if (lane == 0) red[w] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int l = threadIdx.x; l < L; l += 256) {
    const float e = __expf(sa[l] - mx);
    sa[l] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  if (lane == 0) red[w] = sum;
  __syncthreads();
  const float inv = 1.f / (red[0] + red[1] + red[2] + red[3]);
  for (int l = threadIdx.x; l < L; l += 256) {
    sa[l] *= inv;
    a[(long)b * L + l] = sa[l];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    float acc = 0.f;
    for (int l = 0; l < L; ++l) acc += sa[l] * x[((long)b * L + l) * D + c];
    y[(long)b * ldy + c] = acc;
  }
}
MER_API int mer_attn_pool_fwd(int B, int L, int D, const float* x, const float* scores, float* attn, float* y,
                              long ldy, void* stream) {
  if (B <= 0) return 0;
  if (L <= 0 || L > 4096 || D <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(attn_pool_fwd_kernel, dim3(B), dim3(256), L * sizeof(float), (hipStream_t)stream, L, D, x, scores,
                     attn, y, ldy);
  MER_LAUNCH_CHECK();
}

__global__ __launch_bounds__(256) void attn_pool_bwd_kernel(int L, int D, const float* __restrict__ x,
                                                            const float* __restrict__ a, const float* __restrict__ dy,
                                                            long lddy, float* __restrict__ dx, int accumulate,
                                                            float* __restrict__ ds) {
  extern __shared__ float g[];  // [L]: dy . x_l
  __shared__ float red[4];
  const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* dyb = dy + (long)b * lddy;
  for (int l = w; l < L; l += 4) {  // one wave per time step: dot over D
    const float* xl = x + ((long)b * L + l) * D;
    float acc = 0.f;
    for (int c = lane; c < D; c += 64) acc += dyb[c] * xl[c];
    acc = wave_sum(acc);
    if (lane == 0) g[l] = acc;
  }
  __syncthreads();
  float dot = 0.f;
  for (int l = threadIdx.x; l < L; l += 256) dot += a[(long)b * L + l] * g[l];
  dot = wave_sum(dot);
  if (lane == 0) red[w] = dot;
  __syncthreads();
  dot = red[0] + red[1] + red[2] + red[3];
  for (int l = threadIdx.x; l < L; l += 256) ds[(long)b * L + l] = a[(long)b * L + l] * (g[l] - dot);
  for (long e = threadIdx.x; e < (long)L * D; e += 256) {
    const int l = (int)(e / D), c = (int)(e - (long)l * D);
    const float v = a[(long)b * L + l] * dyb[c];
    float* o = dx + (long)b * L * D + e;
    *o = accumulate ? *o + v : v;
  }
}
MER_API int mer_attn_pool_bwd(int B, int L, int D, const float* x, const float* attn, const float* dy, long lddy,
                              float* dx, int accumulate, float* dscores, void* stream) {
  if (B <= 0) return 0;
  if (L <= 0 || L > 4096 || D <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(attn_pool_bwd_kernel, dim3(B), dim3(256), L * sizeof(float), (hipStream_t)stream, L, D, x, attn, dy,
                     lddy, dx, accumulate, dscores);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// Softmax backward of one attention head with its dropout mask, for the materialised-attention path of
// long self-attention (the transformer pooler over the audio sequence, where the fused MFMA kernel's
// LDS image does not fit): P [B,H,Lq,Lk] pre-dropout probabilities, dPp = dO V^T for head h [B,Lq,Lk];
//   m = dropout mask (P index);  dS = P (dPp m - sum_j P dPp m);  Pd = P m.
// One wave per (b, i) row.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void softmax_dropout_bwd_kernel(int B, int H, int h, int Lq, int Lk,
                                                                  const float* __restrict__ P,
                                                                  const float* __restrict__ dPp, float* __restrict__ dS,
                                                                  float* __restrict__ Pd, float p,
                                                                  const unsigned long long* __restrict__ seed_ptr,
                                                                  unsigned long long site) {
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B * Lq) return;
  const int b = row / Lq, i = row - b * Lq;
  const long pbase = (((long)b * H + h) * Lq + i) * Lk;
  const long rbase = (long)row * Lk;
  float dot = 0.f;
  for (int j = lane; j < Lk; j += 64) dot += P[pbase + j] * dPp[rbase + j] * dropout_scale(seed, pbase + j, p);
  dot = wave_sum(dot);
  for (int j = lane; j < Lk; j += 64) {
    const float m = dropout_scale(seed, pbase + j, p), pj = P[pbase + j];
    dS[rbase + j] = pj * (dPp[rbase + j] * m - dot);
    Pd[rbase + j] = pj * m;
  }
}
MER_API int mer_softmax_dropout_bwd(int B, int H, int h, int Lq, int Lk, const float* P, const float* dPp, float* dS,
                                    float* Pd, float p, const unsigned long long* seed, unsigned long long site,
                                    void* stream) {
  if (B <= 0 || Lq <= 0) return 0;
  if (h < 0 || h >= H || Lk <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(softmax_dropout_bwd_kernel, dim3((B * Lq + 3) / 4), dim3(256), 0, (hipStream_t)stream, B, H, h, Lq,
                     Lk, P, dPp, dS, Pd, p, seed, site);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------
// Materialised-score attention forward for head widths the fused MFMA MHA kernel does not take (head_dim
// > 64: TemporalPooler('transformer') at the encoders' widths, 512 / 768 with 4 heads, temporal.py:46-75):
// given S_h = Q_h K_h^T of one head ([B][Lq][Lk], from the batched GEMM), P[b,h] = softmax(scale * S_h) (saved,
// pre-dropout, the layout mer_mha_fwd writes) and Pd = dropout(P) (the same mask index as mer_mha_fwd /
// mer_softmax_dropout_bwd: ((b*H + h)*Lq + i)*Lk + j).  One wave per (b, i) row.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void softmax_dropout_fwd_kernel(int B, int H, int h, int Lq, int Lk,
                                                                  const float* __restrict__ S, float scale,
                                                                  float* __restrict__ P, float* __restrict__ Pd, float p,
                                                                  const unsigned long long* __restrict__ seed_ptr,
                                                                  unsigned long long site) {
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B * Lq) return;
  const int b = row / Lq, i = row - b * Lq;
  const long pbase = (((long)b * H + h) * Lq + i) * Lk;
  const long rbase = (long)row * Lk;
  float m = -INFINITY;
  for (int j = lane; j < Lk; j += 64) m = fmaxf(m, S[rbase + j] * scale);
  m = wave_max(m);
  float s = 0.f;
  for (int j = lane; j < Lk; j += 64) s += __expf(S[rbase + j] * scale - m);
  s = wave_sum(s);
  const float inv = 1.f / s;
  for (int j = lane; j < Lk; j += 64) {
    const float pj = __expf(S[rbase + j] * scale - m) * inv;
    P[pbase + j] = pj;
    Pd[rbase + j] = pj * dropout_scale(seed, pbase + j, p);
  }
}
MER_API int mer_softmax_dropout_fwd(int B, int H, int h, int Lq, int Lk, const float* S, float scale, float* P,
                                    float* Pd, float p, const unsigned long long* seed, unsigned long long site,
                                    void* stream) {
  if (B <= 0 || Lq <= 0) return 0;
  if (h < 0 || h >= H || Lk <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(softmax_dropout_fwd_kernel, dim3((B * Lq + 3) / 4), dim3(256), 0, (hipStream_t)stream, B, H, h, Lq,
                     Lk, S, scale, P, Pd, p, seed, site);
  MER_LAUNCH_CHECK();
}
