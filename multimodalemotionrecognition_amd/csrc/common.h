// Shared device helpers for the MI355X (gfx950 / CDNA4) fusion-path kernels.
// Wave64 everywhere: every reduction below assumes 64 lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MER_API extern "C" __attribute__((visibility("default")))

typedef uint16_t bf16_t;  // raw bfloat16 storage
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

enum MerDType { MER_F32 = 0, MER_BF16 = 1 };
enum MerAct { MER_ACT_NONE = 0, MER_ACT_RELU = 1, MER_ACT_GELU = 2 };

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// round-to-nearest-even; NaN stays NaN (quiet bit forced)
// f32 -> bf16, round to nearest even, NaN stays NaN: the plain conversion, which gfx950 does in hardware
// (v_cvt_pk_bf16_f32, one instruction per two values; the integer-arithmetic rounding it replaces took ~7 VALU
// instructions per value)
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

template <typename T> __device__ __forceinline__ float ldf(const T* p, long i);
template <> __device__ __forceinline__ float ldf<float>(const float* p, long i) { return p[i]; }
template <> __device__ __forceinline__ float ldf<bf16_t>(const bf16_t* p, long i) { return bf2f(p[i]); }

template <typename T> __device__ __forceinline__ void stf(T* p, long i, float v);
template <> __device__ __forceinline__ void stf<float>(float* p, long i, float v) { p[i] = v; }
template <> __device__ __forceinline__ void stf<bf16_t>(bf16_t* p, long i, float v) { p[i] = f2bf(v); }

// erf for GELU: Abramowitz & Stegun 7.1.26 on |u| (absolute error <= 1.5e-7, far below the bf16 / 1e-3
// parity bars of every caller) -- one v_rcp_f32, one v_exp_f32 and 7 FMAs instead of the library erff's
// branchy polynomial, which made GELU the VALU bound of the WavLM conv0 pass and of the GELU epilogues.
__device__ __forceinline__ float erf_fast(float u) {
  const float a = fabsf(u);
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * a);
  const float p = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  return copysignf(1.0f - p * __expf(-a * a), u);
}
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erf_fast(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143267794f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == MER_ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == MER_ACT_GELU) return gelu_erf(v);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Counter-based RNG over (seed, index): the same mask is regenerated in backward from the same (seed, index) --
// no mask tensor is stored.  32-bit arithmetic only (a 64-bit multiply is four quarter-rate VALU ops on CDNA, and
// the attention / activation dropouts hash every element): the 64-bit seed and index are folded to 32 bits, and
// the word is finalised by the "lowbias32" xorshift-multiply mixer (three 32-bit multiplies).
__device__ __forceinline__ uint32_t mer_hash(uint64_t seed, uint64_t idx) {
  const uint32_t s = (uint32_t)seed ^ ((uint32_t)(seed >> 32) * 0x85EBCA6Bu);
  uint32_t x = ((uint32_t)idx ^ ((uint32_t)(idx >> 32) * 0xC2B2AE35u)) * 0x9E3779B9u + s;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
// Per-call-site dropout seed: the step's RNG base lives in DEVICE memory (so a captured hipGraph replays
// with a fresh base every step, advanced in-graph by mer_rng_advance) and is mixed with a constant site
// id; a NULL base means "no dropout" (p == 0) callers.
__device__ __forceinline__ unsigned long long mer_site_seed(const unsigned long long* base, unsigned long long site) {
  const unsigned long long b = base ? *base : 0ull;
  return b * 0x100000001B3ull + site * 0x9E3779B97F4A7C15ull + 1ull;
}
// keep with probability keep_p; returns 1/keep_p when kept, else 0
__device__ __forceinline__ float dropout_scale(uint64_t seed, uint64_t idx, float p) {
  if (p <= 0.f) return 1.f;
  const float u = (mer_hash(seed, idx) >> 8) * (1.0f / 16777216.0f);
  return u >= p ? 1.0f / (1.0f - p) : 0.0f;
}

// Paired-index dropout (the WavLM encoder's sites: GEMM epilogues, encoder LayerNorm, attention probabilities,
// mer_dropout_rows): one mer_hash word serves two adjacent mask indices -- its low 16 bits decide index 2q, its
// high 16 bits index 2q + 1 -- and an index is kept when its half is >= ceil(p 2^16) (keep rate 1 - 6554 / 65536
// at p = 0.1).  Callers holding adjacent indices hash once per pair: half the VALU work of dropout_scale, which
// was ~40% of a train-mode attention launch.
__device__ __forceinline__ uint32_t drop_thr16(float p) { return (uint32_t)ceilf(p * 65536.0f); }
__device__ __forceinline__ bool pair_keep(uint32_t h, uint64_t idx, uint32_t thr) {
  return ((idx & 1ull) ? (h >> 16) : (h & 0xFFFFu)) >= thr;
}
__device__ __forceinline__ float dropout_scale_pair(uint64_t seed, uint64_t idx, float p) {  // one index
  if (p <= 0.f) return 1.f;
  return pair_keep(mer_hash(seed, idx >> 1), idx, drop_thr16(p)) ? 1.0f / (1.0f - p) : 0.0f;
}
// v[e] *= keep scale of index i0 + e, e < N (N even, i0 even): one hash per pair
template <int N>
__device__ __forceinline__ void dropout_pairs(float* v, uint64_t seed, uint64_t i0, float p) {
  const uint32_t thr = drop_thr16(p);
  const float ks = 1.0f / (1.0f - p);
#pragma unroll
  for (int e = 0; e < N; e += 2) {
    const uint32_t h = mer_hash(seed, (i0 + e) >> 1);
    v[e] *= (h & 0xFFFFu) >= thr ? ks : 0.f;
    v[e + 1] *= (h >> 16) >= thr ? ks : 0.f;
  }
}

// a / d for 0 <= a < 2^22 with inv_d = 1.0f / d (d >= 1): exact, ~3 VALU ops instead of an
// integer-division sequence.  (a + 0.5) / d sits >= 0.5/d away from any integer, far more than the
// float rounding error at these magnitudes.
__device__ __forceinline__ int fdiv(int a, float inv_d) { return (int)(((float)a + 0.5f) * inv_d); }

// XCD-aware tile order (cdna_hip_programming.md T1, bijective form): blocks are dealt round-robin over
// the 8 XCDs, so give each XCD (block-id residue class mod 8) a CONTIGUOUS chunk of the row-major tile
// list.  Tiles that share an A row-panel (same ty, consecutive tx) then run on one XCD and hit its L2
// instead of being fetched once per XCD.  Placement only changes speed, never results.
__device__ __forceinline__ void xcd_tile(int pid, int nx, int ntiles, int& tx, int& ty) {
  const int q = ntiles / 8, r = ntiles % 8, xcd = pid % 8, loc = pid / 8;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  ty = tile / nx;
  tx = tile - ty * nx;
}

// 16-byte global -> LDS DMA (global_load_lds_dwordx4): lane i's 16 bytes land at lds + 16*i (the LDS
// pointer must be wave-uniform).  Wrapped in a non-template function: used directly inside a kernel
// TEMPLATE, hipcc (ROCm 7.2) silently drops the host launch stub (undefined symbol at load time).
// s_waitcnt with only vmcnt constrained (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14])
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
// wait until at most n (runtime, 0..3) tiles of G glds each are still in flight
template <int G>
__device__ __forceinline__ void wait_tiles_in_flight(int n) {
  if (n <= 0) wait_vmcnt<0>();
  else if (n == 1) wait_vmcnt<G>();
  else if (n == 2) wait_vmcnt<2 * G>();
  else wait_vmcnt<3 * G>();
}
// Record of block v in a kernel-argument table sorted by first block (first(0) = 0, non-decreasing, n <= 64):
// each lane loads one record's first block and a ballot counts the records at or before v -- one load latency
// instead of a serial scan whose every step is a dependent scalar load of the argument segment (~0.8 us each,
// paid by every block before its first useful instruction).
template <typename F>
__device__ __forceinline__ int table_find(int n, int v, F first) {
  const int lane = threadIdx.x & 63;
  const int f = lane < n ? first(lane) : 0x7fffffff;
  const unsigned long long m = __ballot(f <= v);
  return __builtin_amdgcn_readfirstlane(__popcll(m) - 1);
}

// lgkmcnt(0) only (LDS reads retired), then a raw s_barrier: glds DMAs stay in flight across it
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void glds16(const void* g, void* lds) { __builtin_amdgcn_global_load_lds(g, lds, 16, 0, 0); }

// xcd_tile plus grouped rasterisation inside each XCD's chunk: consecutive tiles walk a G-row band
// column by column, so the ~64 tiles an XCD runs at once cover ~G x 64/G panels of A and B instead of
// a few full rows (every B panel) -- a smaller working set for that XCD's 4 MB L2.
__device__ __forceinline__ void xcd_tile_grouped(int pid, int nx, int ny, int G, int& tx, int& ty) {
  const int ntiles = nx * ny;
  const int q = ntiles / 8, r = ntiles % 8, xcd = pid % 8, loc = pid / 8;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  G = G < 1 ? 1 : G;
  const int band = G * nx, gid = tile / band, first = gid * G;
  const int gsz = ny - first < G ? ny - first : G;
  const int in = tile - gid * band;
  ty = first + in % gsz;
  tx = in / gsz;
}

#define MER_LAUNCH_CHECK() return (int)hipGetLastError()
