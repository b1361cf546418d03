// Shared device helpers of the fused xattn head kernels (xattn_fused.hip, xattn_fused_bwd.hip): split-bf16
// MFMA fragments (fp32 operand = bf16 hi + lo planes), LDS-tile products and stores.
#pragma once
#include "common.h"

namespace xh {

constexpr int XD = 128;      // d_model
constexpr int XH = 4;        // heads
constexpr int XDH = 32;      // head dim
constexpr int LDA = XD + 4;  // LDS row stride (floats) of 128-wide activation tiles

typedef __attribute__((ext_vector_type(4))) uint32_t u4;

union Frag {
  bf16x8 v;
  uint16_t h[8];
  u4 u;
};

__device__ __forceinline__ f32x4 mma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// 8 fp32 -> (hi, lo) bf16 fragments
__device__ __forceinline__ void split8(const float (&x)[8], bf16x8& hi, bf16x8& lo) {
  Frag H, L;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const uint16_t hb = f2bf(x[e]);
    H.h[e] = hb;
    L.h[e] = f2bf(x[e] - bf2f(hb));
  }
  hi = H.v;
  lo = L.v;
}

// fp32 fragment: 8 consecutive k (stride 1) of one row; zero when !valid
__device__ __forceinline__ void frag_row(const float* p, bool valid, bf16x8& hi, bf16x8& lo) {
  float x[8];
  if (valid) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
    x[0] = a[0]; x[1] = a[1]; x[2] = a[2]; x[3] = a[3]; x[4] = b[0]; x[5] = b[1]; x[6] = b[2]; x[7] = b[3];
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = 0.f;
  }
  split8(x, hi, lo);
}

// fp32 fragment gathered with a k stride (transposed operand); element e valid while k0 + e < kmax
__device__ __forceinline__ void frag_col(const float* p, long ks, int k0, int kmax, bool valid, bf16x8& hi,
                                         bf16x8& lo) {
  float x[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) x[e] = (valid && k0 + e < kmax) ? p[(long)e * ks] : 0.f;
  split8(x, hi, lo);
}

// pre-split weight fragment (row n of [N][K] hi / lo planes)
__device__ __forceinline__ void frag_w(const bf16_t* hi_p, const bf16_t* lo_p, bf16x8& hi, bf16x8& lo) {
  Frag H, L;
  H.u = *reinterpret_cast<const u4*>(hi_p);
  L.u = *reinterpret_cast<const u4*>(lo_p);
  hi = H.v;
  lo = L.v;
}

__device__ __forceinline__ f32x4 mma3(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f32x4 c) {
  c = mma(ah, bh, c);
  c = mma(ah, bl, c);
  return mma(al, bh, c);
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

struct XhDrop {  // dropout / drop-path of the head (train mode), sites as xattn_head.py
  float attn, path;
  const unsigned long long* seed;
  unsigned long long site_attn, site_path;
};

struct SplitW {  // one weight's pre-split planes [N][K]
  const bf16_t* hi;
  const bf16_t* lo;
};

// acc[i][j] (+)= A[rows 16i..][0:K] . W[cols c0 + 16j..][0:K]^T with A fp32 rows (row stride lda, 16-byte aligned),
// rows >= rmax read as zero; W pre-split [N][K] (ldw elements)
template <int TI, int TJ>
__device__ __forceinline__ void mm_aw(f32x4 (&acc)[TI][TJ], const float* A, long lda, int rmax, int K, SplitW W,
                                      long ldw, int c0) {
  const int lane = threadIdx.x & 63, fr = lane & 15, fk = (lane >> 4) * 8;
  for (int k = 0; k < K; k += 32) {
    bf16x8 bh[TJ], bl[TJ];
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const long off = (long)(c0 + 16 * j + fr) * ldw + k + fk;
      frag_w(W.hi + off, W.lo + off, bh[j], bl[j]);
    }
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int r = 16 * i + fr;
      bf16x8 ah, al;
      frag_row(A + (long)r * lda + k + fk, r < rmax, ah, al);
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] = mma3(ah, al, bh[j], bl[j], acc[i][j]);
    }
  }
}

template <int TI, int TJ>
__device__ __forceinline__ void zero(f32x4 (&acc)[TI][TJ]) {
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// store acc + bias[col] into an fp32 LDS tile (stride lds_ld) and / or a global matrix (rows < rmax)
template <int TI, int TJ>
__device__ __forceinline__ void store_acc(const f32x4 (&acc)[TI][TJ], int c0, const float* bias, float* lds, int lds_ld,
                                          float* g, long ldg, long grow0, int rmax) {
  const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int col = c0 + 16 * j + fr;
    const float bv = bias ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * i + 4 * fq + r;
        const float v = acc[i][j][r] + bv;
        if (lds) lds[row * lds_ld + col] = row < rmax ? v : 0.f;
        if (g && row < rmax) g[(grow0 + row) * ldg + col] = v;
      }
  }
}

}  // namespace xh
