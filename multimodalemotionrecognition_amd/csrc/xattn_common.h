// Shared device helpers of the fused xattn head kernels (xattn_fused.hip, xattn_fused_bwd.hip): split-bf16
// MFMA fragments (fp32 operand = bf16 hi + lo planes), LDS-tile products and stores.
#pragma once
#include "common.h"

// Phase timestamps for kernel tuning (tools/xt_phases.py builds a separate library with -DMER_XH_TIMING; the
// production library compiles these to nothing): XT(slot, k) stores wall_clock64() of workgroup blockIdx.x's
// thread 0 at phase k into the slot's table.
#ifdef MER_XH_TIMING
static __device__ long long mer_xt_buf[4][512 * 16];  // one table per translation unit
#define XT(slot, k) \
  do { \
    if (threadIdx.x == 0 && blockIdx.x < 512) mer_xt_buf[slot][blockIdx.x * 16 + (k)] = wall_clock64(); \
  } while (0)
#else
#define XT(slot, k) \
  do { \
  } while (0)
#endif

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

typedef __attribute__((ext_vector_type(8))) float f32x8;

// 8 fp32 -> (hi, lo) bf16 fragments: hi = RNE(x), lo = RNE(x - hi), both by the packed hardware conversion
__device__ __forceinline__ void split8(const float (&x)[8], bf16x8& hi, bf16x8& lo) {
  const f32x8 v = {x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]};
  hi = __builtin_convertvector(v, bf16x8);
  lo = __builtin_convertvector(v - __builtin_convertvector(hi, f32x8), bf16x8);
}

// Loads in these helpers are UNCONDITIONAL, and the caller passes an address that is always dereferenceable
// (a clamped row): a load under a per-lane condition compiles to a branch around the load followed by a wait,
// which serialises every load of a loop on the memory latency.  Invalid elements are zeroed by a select.

// the same split from two 4-vectors (no float array in between: an array the compiler does not promote to
// registers ends up in scratch memory)
__device__ __forceinline__ void split8v(f32x4 a, f32x4 b, bf16x8& hi, bf16x8& lo) {
  const f32x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  hi = __builtin_convertvector(v, bf16x8);
  lo = __builtin_convertvector(v - __builtin_convertvector(hi, f32x8), bf16x8);
}

// fp32 fragment: 8 consecutive k (stride 1) of one row; zero when !valid (p must still be dereferenceable)
__device__ __forceinline__ void frag_row(const float* p, bool valid, bf16x8& hi, bf16x8& lo) {
  const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
  split8v(valid ? a : z, valid ? b : z, hi, lo);
}

// fp32 fragment gathered with a k stride (transposed operand) from p = &row k0; element e is row k0 + e, zero
// for rows >= kmax (read from row kmax - 1 instead, so kmax >= 1 and row kmax - 1 must exist)
__device__ __forceinline__ void frag_col(const float* p, long ks, int k0, int kmax, bf16x8& hi, bf16x8& lo) {
  float x[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int kk = k0 + e < kmax ? k0 + e : kmax - 1;
    const float v = p[(long)(kk - k0) * ks];
    x[e] = k0 + e < kmax ? v : 0.f;
  }
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

// workgroup barrier for LDS traffic only: LDS stores / loads before it have retired, global loads and stores
// stay in flight (__syncthreads' release fence waits for every outstanding global access as well).  The empty
// asm statements keep the compiler from moving memory accesses across it.
__device__ __forceinline__ void lds_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  lds_barrier();
  asm volatile("" ::: "memory");
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

// acc[i][j] (+)= A[rows 16i..][0:K] . W[cols c0 + 16j..][0:K]^T with A fp32 rows (row stride lda, 16-byte aligned);
// accumulator rows >= rmax hold junk (a copy of row rmax - 1's product) that callers must not store; W pre-split [N][K] (ldw elements).  Software-pipelined: the A rows and weight
// fragments of the next D 32-wide k steps are in flight while a step's MFMAs run, so a K-long product costs
// ~K / 32 / D memory latencies instead of K / 32 (these kernels are latency-bound: few workgroups, short chains).
template <int TI, int TJ>
struct MmStage {
  f32x4 a0[TI], a1[TI];
  u4 bh[TJ], bl[TJ];
};

template <int TI, int TJ>
__device__ __forceinline__ void mm_load(MmStage<TI, TJ>& st, const float* A, long lda, int rmax, SplitW W, long ldw,
                                        int c0, int k) {
  const int lane = threadIdx.x & 63, fr = lane & 15, fk = (lane >> 4) * 8;
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const long off = (long)(c0 + 16 * j + fr) * ldw + k + fk;
    st.bh[j] = *reinterpret_cast<const u4*>(W.hi + off);
    st.bl[j] = *reinterpret_cast<const u4*>(W.lo + off);
  }
#pragma unroll
  for (int i = 0; i < TI; ++i) {  // rows >= rmax read row rmax - 1: finite junk rows the epilogues never store
    const int r = 16 * i + fr;
    const float* p = A + (long)(r < rmax ? r : rmax - 1) * lda + k + fk;
    st.a0[i] = *reinterpret_cast<const f32x4*>(p);  // no select here: it would wait for the load at issue
    st.a1[i] = *reinterpret_cast<const f32x4*>(p + 4);
  }
}

template <int TI, int TJ>
__device__ __forceinline__ void mm_step(f32x4 (&acc)[TI][TJ], const MmStage<TI, TJ>& st, bool live) {
  bf16x8 bh[TJ], bl[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    Frag H, L;
    H.u = st.bh[j];
    L.u = st.bl[j];
    bh[j] = H.v;
    bl[j] = L.v;
  }
#pragma unroll
  for (int i = 0; i < TI; ++i) {
    const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 a0 = live ? st.a0[i] : z, a1 = live ? st.a1[i] : z;  // a select, not a branch
    bf16x8 ah, al;
    split8v(a0, a1, ah, al);
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = mma3(ah, al, bh[j], bl[j], acc[i][j]);
  }
}

// D k steps in flight: the stage consumed at step s was loaded D steps earlier (one workgroup per CU is common
// here, so there are no other waves to hide a memory latency behind; the depth has to).  The loop body is
// branch-free -- a conditional step or load would make the wait-count pass assume the worst at the merge and
// wait for every load in flight (vmcnt(0)) -- so the tail steps past K load a clamped (valid) k slice and are
// accumulated as zeros.
template <int TI, int TJ, int D = 3, int KS = 0>
__device__ __forceinline__ void mm_aw(f32x4 (&acc)[TI][TJ], const float* A, long lda, int rmax, int K, SplitW W,
                                      long ldw, int c0) {
  // KS > 0: the depth is a compile-time constant (K == KS): the step loop unrolls completely and the stage ring
  // stays in registers (with a run-time trip count the compiler keeps the ring in scratch memory)
  const int nsteps = KS > 0 ? KS / 32 : K / 32;
  MmStage<TI, TJ> st[D];
#pragma unroll
  for (int d = 0; d < D; ++d) mm_load(st[d], A, lda, rmax, W, ldw, c0, 32 * (d < nsteps ? d : nsteps - 1));
#pragma unroll
  for (int s0 = 0; s0 < nsteps; s0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      mm_step(acc, st[d], s0 + d < nsteps);
      const int nx = s0 + d + D;
      mm_load(st[d], A, lda, rmax, W, ldw, c0, 32 * (nx < nsteps ? nx : nsteps - 1));
    }
  }
}

// pre-split weight fragments of NS 32-wide k steps x TJ 16-column tiles, held in registers
template <int NS, int TJ>
struct WRegs {
  u4 h[NS][TJ], l[NS][TJ];
};

// steps >= nvalid load step nvalid - 1 and columns >= nrows row nrows - 1 (valid addresses; the A operand is
// zero past the valid steps, the extra columns are never stored)
template <int NS, int TJ>
__device__ __forceinline__ void wregs_load(WRegs<NS, TJ>& r, SplitW W, long ldw, int c0, int nvalid,
                                           int nrows = 1 << 30) {
  const int lane = threadIdx.x & 63, fr = lane & 15, fk = (lane >> 4) * 8;
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int n = c0 + 16 * j + fr;
      const long off = (long)(n < nrows ? n : nrows - 1) * ldw + 32 * (s < nvalid ? s : nvalid - 1) + fk;
      r.h[s][j] = *reinterpret_cast<const u4*>(W.hi + off);
      r.l[s][j] = *reinterpret_cast<const u4*>(W.lo + off);
    }
}

// acc[i][j] += A[rows 16i..][0 : 32 NS] . W^T: A fp32 rows in LDS (split on the fly), W from registers; the same
// per-step order as mm_aw (hi.hi, hi.lo, lo.hi per k step)
template <int TI, int TJ, int NS>
__device__ __forceinline__ void mm_lw(f32x4 (&acc)[TI][TJ], const float* A, int lda, const WRegs<NS, TJ>& w) {
  const int lane = threadIdx.x & 63, fr = lane & 15, fk = (lane >> 4) * 8;
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      bf16x8 ah, al;
      frag_row(A + (16 * i + fr) * lda + 32 * s + fk, true, ah, al);
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        Frag H, L;
        H.u = w.h[s][j];
        L.u = w.l[s][j];
        acc[i][j] = mma3(ah, al, H.v, L.v, acc[i][j]);
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
