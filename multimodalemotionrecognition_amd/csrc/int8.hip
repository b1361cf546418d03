// Dynamic-INT8 nn.Linear on CDNA4 matrix cores -- the GPU form of the reference's
// quantize_dynamic({nn.Linear}, qint8) inference path (optimized_runtime.py:95-96), bit-compatible
// with the fbgemm algorithm restated in oracle/int8_ref.py:
//
//   weight (once, at load):  ws = max(amax|W| / 127.5, eps);  qw = clamp(rint(W * (1/ws)), -128, 127)
//   activation (per call):   min/max over the WHOLE input tensor -> (xs, zp) by fbgemm
//                            ChooseQuantizationParams(0, 255, reduce_range) = range [0, 127];
//                            qx = clamp(rint(fma(x, 1/xs, zp)), 0, 255)
//   output:                  y = fma(float(sum_k qx*qw - zp*sum_k qw), xs*ws, bias)  (+ReLU fused)
//
// qx is at most 128 (x <= xmax maps to <= 127.5), so it is held as the signed byte qx - 64 and the
// GEMM runs on v_mfma_i32_16x16x64_i8; the offset folds into the zero-point term
// (64 - zp) * colsum(qw).  Activations are quantized while being staged into LDS (no int8 copy of
// x in HBM); the fp32 input is read exactly once per N-tile.
#include "common.h"
#include "mer.h"

namespace {

typedef __attribute__((ext_vector_type(4))) int i32x4;

constexpr int MM_BLOCKS = 512, MM_THREADS = 256;

template <typename T>
__global__ __launch_bounds__(MM_THREADS) void minmax_partial_kernel(long n, const T* __restrict__ x,
                                                                    float* __restrict__ part) {
  constexpr int V = 16 / sizeof(T);  // elements per 16-byte load
  float lo = INFINITY, hi = -INFINITY;
  const long nv = n / V;
  for (long i = blockIdx.x * (long)MM_THREADS + threadIdx.x; i < nv; i += (long)gridDim.x * MM_THREADS) {
    const uint4 raw = reinterpret_cast<const uint4*>(x)[i];
    const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float v = ldf<T>(e, j);
      lo = fminf(lo, v);
      hi = fmaxf(hi, v);
    }
  }
  for (long i = nv * V + blockIdx.x * (long)MM_THREADS + threadIdx.x; i < n; i += (long)gridDim.x * MM_THREADS) {
    lo = fminf(lo, ldf<T>(x, i));
    hi = fmaxf(hi, ldf<T>(x, i));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, o, 64));
    hi = fmaxf(hi, __shfl_xor(hi, o, 64));
  }
  __shared__ float slo[MM_THREADS / 64], shi[MM_THREADS / 64];
  if ((threadIdx.x & 63) == 0) {
    slo[threadIdx.x >> 6] = lo;
    shi[threadIdx.x >> 6] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < MM_THREADS / 64; ++w) {
      lo = fminf(lo, slo[w]);
      hi = fmaxf(hi, shi[w]);
    }
    part[2 * blockIdx.x] = lo;
    part[2 * blockIdx.x + 1] = hi;
  }
}

// fbgemm ChooseQuantizationParams(min, max, qmin=0, qmax=127) -- double arithmetic as in the CPU code
__device__ void choose_qparams(float fmin, float fmax, float* qp) {
  const int qmin = 0, qmax = 127;
  double mn = fmin < 0.f ? (double)fmin : 0.0, mx = fmax > 0.f ? (double)fmax : 0.0;
  double scale = (mx - mn) / (qmax - qmin);
  if ((float)scale == 0.f || isinf(1.0f / (float)scale)) scale = 0.1;
  const double small = 6.1e-5;
  if (scale < small) {
    const float org = (float)scale;
    scale = small;
    if (mn == 0.0) mx = small * (qmax - qmin);
    else if (mx == 0.0) mn = -small * (qmax - qmin);
    else {
      const float amp = (float)(small / org);
      mn *= amp;
      mx *= amp;
    }
  }
  const double z_min = qmin - mn / scale, z_max = qmax - mx / scale;
  const double e_min = fabs((double)qmin) - fabs(mn / scale), e_max = fabs((double)qmax) - fabs(mx / scale);
  const double z0 = e_min < e_max ? z_min : z_max;
  int zp;
  if (z0 < qmin) zp = qmin;
  else if (z0 > qmax) zp = qmax;
  else zp = (int)rint(z0);
  const float s = (float)scale;
  qp[0] = s;
  qp[1] = 1.0f / s;
  qp[2] = (float)zp;
  qp[3] = 0.f;
}

// mode 0: activation qparams (above); mode 1: symmetric per-tensor weight scale (MinMaxObserver)
__global__ void minmax_final_kernel(int nparts, const float* __restrict__ part, int mode, float* __restrict__ qp) {
  float lo = INFINITY, hi = -INFINITY;
  for (int i = threadIdx.x; i < nparts; i += 64) {
    lo = fminf(lo, part[2 * i]);
    hi = fmaxf(hi, part[2 * i + 1]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, o, 64));
    hi = fmaxf(hi, __shfl_xor(hi, o, 64));
  }
  if (threadIdx.x != 0) return;
  if (mode == 0) {
    choose_qparams(lo, hi, qp);
  } else {
    const float amax = fmaxf(fmaxf(-fminf(lo, 0.f), fmaxf(hi, 0.f)), 0.f);
    float ws = amax / 127.5f;
    ws = fmaxf(ws, 1.1920928955078125e-07f);
    qp[0] = ws;
    qp[1] = 1.0f / ws;
    qp[2] = 0.f;
    qp[3] = 0.f;
  }
}

// one block per output row n: quantize W[n, :] and its integer row sum (the zero-point correction)
// 16 consecutive elements as fp32
template <typename T> __device__ __forceinline__ void load16(const T* p, float4 (&f)[4]);
template <> __device__ __forceinline__ void load16<float>(const float* p, float4 (&f)[4]) {
  const float4* s = reinterpret_cast<const float4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) f[i] = s[i];
}
template <> __device__ __forceinline__ void load16<bf16_t>(const bf16_t* p, float4 (&f)[4]) {
  const uint4* s = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint4 u = s[h];
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 2; ++j)
      f[2 * h + j] = float4{__uint_as_float(w[2 * j] << 16), __uint_as_float(w[2 * j] & 0xffff0000u),
                            __uint_as_float(w[2 * j + 1] << 16), __uint_as_float(w[2 * j + 1] & 0xffff0000u)};
  }
}

__global__ __launch_bounds__(256) void quantize_weight_kernel(int K, const float* __restrict__ w, long ldw,
                                                              const float* __restrict__ qp, int8_t* __restrict__ qw,
                                                              long ldq, int* __restrict__ colsum) {
  const int n = blockIdx.x;
  const float inv = qp[1];
  int s = 0;
  for (int k = threadIdx.x; k < ldq; k += 256) {
    int q = 0;
    if (k < K) q = (int)fminf(fmaxf(rintf(w[(long)n * ldw + k] * inv), -128.f), 127.f);
    qw[(long)n * ldq + k] = (int8_t)q;
    s += q;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  __shared__ int ss[4];
  if ((threadIdx.x & 63) == 0) ss[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) colsum[n] = ss[0] + ss[1] + ss[2] + ss[3];
}

// ---- GEMM: 128x64 output tile, K step 64 bytes, 4 waves each 32 rows x 64 cols ----
constexpr int BM = 128, BN = 64, BK = 64, LDS_ROW = BK + 16;  // 80-byte rows

__device__ __forceinline__ uint32_t pack_q4(float4 v, float inv, float zp) {
  auto q = [&](float x) -> uint32_t {
    const float r = fminf(fmaxf(rintf(fmaf(x, inv, zp)), 0.f), 255.f) - 64.f;
    return (uint32_t)((int)r & 0xff);
  };
  return q(v.x) | (q(v.y) << 8) | (q(v.z) << 16) | (q(v.w) << 24);
}

template <typename T>
__global__ __launch_bounds__(256) void gemm_i8dyn_kernel(int M, int N, int K, const T* __restrict__ x, long ldx,
                                                         const float* __restrict__ xqp, const int8_t* __restrict__ qw,
                                                         long ldq, const float* __restrict__ wqp,
                                                         const int* __restrict__ colsum, const float* __restrict__ bias,
                                                         int act, float* __restrict__ out, long ldo) {
  __shared__ __attribute__((aligned(16))) int8_t la[BM * LDS_ROW];
  __shared__ __attribute__((aligned(16))) int8_t lb[BN * LDS_ROW];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int nx = (N + BN - 1) / BN;
  const int m0 = (blockIdx.x / nx) * BM, n0 = (blockIdx.x % nx) * BN;
  const float inv = xqp[1], zp = xqp[2];

  i32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = i32x4{0, 0, 0, 0};

  // A staging: 128 rows x 64 k = 512 chunks of 16 values, 2 per thread; B: 64 rows x 64 bytes = 256 chunks
  for (int k0 = 0; k0 < K; k0 += BK) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int idx = t + 256 * c, r = idx >> 2, kc = (idx & 3) * 16;
      const int m = m0 + r, k = k0 + kc;
      uint4 pk = {0u, 0u, 0u, 0u};  // zero bytes contribute nothing (W is zero-padded too)
      if (m < M && k < K) {
        float4 f[4];
        load16<T>(x + (long)m * ldx + k, f);
        pk.x = pack_q4(f[0], inv, zp);
        pk.y = pack_q4(f[1], inv, zp);
        pk.z = pack_q4(f[2], inv, zp);
        pk.w = pack_q4(f[3], inv, zp);
      }
      *reinterpret_cast<uint4*>(&la[r * LDS_ROW + kc]) = pk;
    }
    {
      const int r = t >> 2, kc = (t & 3) * 16, n = n0 + r, k = k0 + kc;
      uint4 pk = {0u, 0u, 0u, 0u};
      if (n < N && k < ldq) pk = *reinterpret_cast<const uint4*>(qw + (long)n * ldq + k);
      *reinterpret_cast<uint4*>(&lb[r * LDS_ROW + kc]) = pk;
    }
    __syncthreads();
    const int kof = (lane >> 4) * 16;
    i32x4 af[2], bfr[4];
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = *reinterpret_cast<const i32x4*>(&la[(w * 32 + i * 16 + (lane & 15)) * LDS_ROW + kof]);
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = *reinterpret_cast<const i32x4*>(&lb[(j * 16 + (lane & 15)) * LDS_ROW + kof]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[i], bfr[j], acc[i][j], 0, 0, 0);
    __syncthreads();
  }

  const float s = xqp[0] * wqp[0];
  const int off = 64 - (int)zp;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + j * 16 + (lane & 15);
    if (col >= N) continue;
    const int corr = off * colsum[col];
    const float bv = bias ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + w * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (row >= M) continue;
        float v = fmaf((float)(acc[i][j][r] + corr), s, bv);
        if (act == MER_ACT_RELU) v = fmaxf(v, 0.f);
        out[(long)row * ldo + col] = v;
      }
  }
}

int minmax_qparams(long n, const void* x, int dtype, float* part, int mode, float* qp, hipStream_t st) {
  long blocks = (n / 4 + MM_THREADS - 1) / MM_THREADS;
  blocks = blocks < 1 ? 1 : (blocks > MM_BLOCKS ? MM_BLOCKS : blocks);
  if (dtype == MER_BF16)
    hipLaunchKernelGGL(minmax_partial_kernel<bf16_t>, dim3((unsigned)blocks), dim3(MM_THREADS), 0, st, n,
                       (const bf16_t*)x, part);
  else
    hipLaunchKernelGGL(minmax_partial_kernel<float>, dim3((unsigned)blocks), dim3(MM_THREADS), 0, st, n,
                       (const float*)x, part);
  hipLaunchKernelGGL(minmax_final_kernel, dim3(1), dim3(64), 0, st, (int)blocks, part, mode, qp);
  return (int)hipGetLastError();
}

}  // namespace

MER_API int mer_quant_params(long n, const void* x, int x_dtype, float* partial, int mode, float* qparams,
                             void* stream) {
  if (n <= 0 || (mode != 0 && mode != 1) || (((uintptr_t)x) & 15) || (mode == 1 && x_dtype != MER_F32))
    return (int)hipErrorInvalidValue;
  return minmax_qparams(n, x, x_dtype, partial, mode, qparams, (hipStream_t)stream);
}

MER_API int mer_quantize_weight_s8(int N, int K, const float* w, long ldw, const float* qparams, void* qw, long ldq,
                                   int* colsum, void* stream) {
  if (N <= 0 || K <= 0 || ldq < K || (ldq % 16) != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(quantize_weight_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, K, w, ldw, qparams,
                     (int8_t*)qw, ldq, colsum);
  return (int)hipGetLastError();
}

MER_API int mer_gemm_i8dyn(int M, int N, int K, const void* x, int x_dtype, long ldx, const float* x_qparams,
                           const void* qw, long ldq, const float* w_qparams, const int* colsum, const float* bias,
                           int act, float* out, long ldo, void* stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 16 != 0 || ldx % 8 != 0 || ldq < K || ldq % 16 != 0 || (((uintptr_t)x) & 15) || (((uintptr_t)qw) & 15))
    return (int)hipErrorInvalidValue;
  const long tiles = (long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (x_dtype == MER_BF16)
    hipLaunchKernelGGL(gemm_i8dyn_kernel<bf16_t>, dim3((unsigned)tiles), dim3(256), 0, (hipStream_t)stream, M, N, K,
                       (const bf16_t*)x, ldx, x_qparams, (const int8_t*)qw, ldq, w_qparams, colsum, bias, act, out,
                       ldo);
  else
    hipLaunchKernelGGL(gemm_i8dyn_kernel<float>, dim3((unsigned)tiles), dim3(256), 0, (hipStream_t)stream, M, N, K,
                       (const float*)x, ldx, x_qparams, (const int8_t*)qw, ldq, w_qparams, colsum, bias, act, out,
                       ldo);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Input rows of the emotion-prior token-bias Linears under INT8 (fusion.py:170-176: the Linear sees
// cat([token, prior expanded over L]) and quantize_dynamic quantizes that whole concatenated tensor per call):
// out[(b*L + l), 0:ldo] = [tok[b*L + l, 0:d], prior[b, 0:pd], 0 ...].  The zero tail pads K to a multiple of 16
// (zeros do not move the activation min/max -- the quantization range always contains 0 -- and meet zero weights).
__global__ void concat_prior_rows_kernel(int B, int L, int d, int pd, int ldo, const float* __restrict__ tok,
                                         const float* __restrict__ prior, float* __restrict__ out) {
  const long n = (long)B * L * ldo;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const long r = e / ldo;
    const int k = (int)(e - r * ldo);
    const int b = (int)(r / L);
    out[e] = k < d ? tok[r * d + k] : (k < d + pd ? prior[(long)b * pd + (k - d)] : 0.f);
  }
}

MER_API int mer_concat_prior_rows(int B, int L, int d, int pd, int ldo, const float* tok, const float* prior, float* out,
                                  void* stream) {
  if (B <= 0 || L <= 0 || ldo < d + pd) return (int)hipErrorInvalidValue;
  const long n = (long)B * L * ldo;
  const int grid = (int)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
  hipLaunchKernelGGL(concat_prior_rows_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, B, L, d, pd, ldo, tok,
                     prior, out);
  MER_LAUNCH_CHECK();
}
