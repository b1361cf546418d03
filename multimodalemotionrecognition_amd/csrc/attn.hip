// Multi-head attention core of the xattn blocks (fusion.py:276-281, 394, 398 -> nn.MultiheadAttention's
// explicit path, TORCH:6576-6606) on the exact-fp32 MFMA (v_mfma_f32_16x16x4_f32: bit-identical to a
// k-ordered fmaf chain, so the head keeps its "logits within 1e-3 of the fp32 CPU reference" bar):
//
//   S_h = scale Q_h K_h^T + bias[b]     P_h = softmax(S_h)     O_h = dropout(P_h) V_h
//
// Rows of Q/K/V/O: X + (b*L + i)*ld + h*dh.  bias: [B, Lq, Lk] per sample, shared by the heads (the
// reference repeat_interleaves it, fusion.py:351-354), or NULL.  P [B,H,Lq,Lk] keeps the pre-dropout
// probabilities for backward; the dropout mask is regenerated from (seed, P index).
//
// Fragment maps of v_mfma_f32_16x16x4_f32 (cdna_hip_programming.md §3): lane l holds A[l&15][k=l>>4],
// B[k=l>>4][l&15]; C/D: col = l&15, row = (l>>4)*4 + r.
//
// LDS strides (floats): an operand read "16 rows x 4 k" (A of any product, or B of Q K^T) uses a row
// stride ST with ST/4 odd, so the 16 rows x 4 columns cover all 64 banks; a read "4 rows x 16 columns"
// (B of P V) uses a stride = 16 or 48 (mod 64) so its 4 rows land on distinct 16-bank groups.
#include "common.h"
#include "mer.h"

namespace {

__host__ __device__ constexpr int st_rows16(int cols) { return (cols + 7) / 8 * 8 + 4; }      // ST/4 odd
__host__ __device__ constexpr int pad16(int n) { return (n + 15) / 16 * 16; }
__host__ __device__ constexpr int st_rows4(int cols16) { return cols16 % 32 == 0 ? cols16 + 16 : cols16; }

constexpr int FWD_MAX_KT = 16;  // key tiles held in registers: Lk <= 256

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Stage rows [0, Lp) x cols [0, cols_p) of head h into LDS (zero outside [0, L) x [0, dh)).
// 16-byte chunks when the rows allow it (dh, ld, st multiples of 4 and a 16-byte aligned source: every
// xattn call site), unrolled so several global loads are in flight per thread -- the element-wise loop was a
// chain of ~80 dependent load -> LDS-store trips per thread for Lk = 149 (v2a forward: 75 us -> ~10 us).
__device__ __forceinline__ void stage_head(float* dst, int st, int Lp, int cols_p, const float* __restrict__ src,
                                           long ld, int b, int L, int h, int dh) {
  const float* base = src + (long)b * L * ld + h * dh;
  if ((dh & 3) == 0 && (ld & 3) == 0 && (st & 3) == 0 && (cols_p & 3) == 0 &&
      (reinterpret_cast<uintptr_t>(base) & 15) == 0) {
    const int cq = cols_p >> 2, n = Lp * cq;
#pragma unroll 4
    for (int e = threadIdx.x; e < n; e += blockDim.x) {
      const int j = e / cq, c = (e - j * cq) * 4;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (j < L && c < dh) v = *reinterpret_cast<const f32x4*>(base + (long)j * ld + c);
      *reinterpret_cast<f32x4*>(dst + j * st + c) = v;
    }
    return;
  }
  for (int e = threadIdx.x; e < Lp * cols_p; e += blockDim.x) {
    const int j = e / cols_p, c = e - j * cols_p;
    dst[j * st + c] = (j < L && c < dh) ? base[(long)j * ld + c] : 0.f;
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// Forward.  Grid (B*H, ceil(Lq / (16*W))), W = waves per block = min(4, ceil(Lq/16)); wave w owns
// 16 query rows.  K_h, V_h staged in LDS once per block; S for the wave's 16 rows x all keys lives in
// registers (Lk <= 256); softmax with 16-lane shuffles; P' = dropout(P) goes through a per-wave LDS
// tile into the P V product.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mha_fwd_kernel(int B, int H, int Lq, int Lk, int dh, const float* __restrict__ Q,
                                                      long ldq, const float* __restrict__ K, long ldk,
                                                      const float* __restrict__ V, long ldv,
                                                      const float* __restrict__ bias, float* __restrict__ O, long ldo,
                                                      float* __restrict__ P, float scale, float drop_p,
                                                      const unsigned long long* __restrict__ seed_ptr,
    unsigned long long site) {
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int LkP = pad16(Lk), dh16 = pad16(dh);
  const int KST = st_rows16(dh), VST = st_rows4(dh16), PST = LkP + 4;
  float* Ks = smem;             // [LkP][KST]
  float* Vs = Ks + LkP * KST;   // [LkP][VST]
  float* Pw = Vs + LkP * VST;   // [waves][16][PST]
  const int b = blockIdx.x / H, h = blockIdx.x - (blockIdx.x / H) * H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  stage_head(Ks, KST, LkP, dh, K, ldk, b, Lk, h, dh);
  stage_head(Vs, VST, LkP, dh16, V, ldv, b, Lk, h, dh);
  __syncthreads();
  const int q0 = (blockIdx.y * nw + w) * 16;
  if (q0 >= Lq) return;  // after the only block-wide barrier
  const int fr = lane & 15, fq = lane >> 4;
  const int NT = LkP / 16;

  // S = Q K^T for rows q0..q0+15 (A fragments straight from global: 16 rows x 4 columns per k-step)
  f32x4 s[FWD_MAX_KT];
#pragma unroll
  for (int ct = 0; ct < FWD_MAX_KT; ++ct) s[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int qa_row = q0 + fr;
  const float* qrow = Q + ((long)b * Lq + (qa_row < Lq ? qa_row : 0)) * ldq + h * dh;
  for (int kk = 0; kk < dh / 4; ++kk) {
    const float a = qa_row < Lq ? qrow[kk * 4 + fq] : 0.f;
#pragma unroll
    for (int ct = 0; ct < FWD_MAX_KT; ++ct)
      if (ct < NT) s[ct] = mfma4(a, Ks[(ct * 16 + fr) * KST + kk * 4 + fq], s[ct]);
  }

  // scale + bias, row max (rows (fq*4 + r) are spread over the 16 lanes of quarter fq)
  float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int ct = 0; ct < FWD_MAX_KT; ++ct) {
    if (ct < NT) {
      const int j = ct * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = q0 + fq * 4 + r;
        float v = -INFINITY;
        if (j < Lk && i < Lq) {
          v = s[ct][r] * scale;
          if (bias) v += bias[((long)b * Lq + i) * Lk + j];
        }
        s[ct][r] = v;
        mx[r] = fmaxf(mx[r], v);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], o, 64));
  float sum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ct = 0; ct < FWD_MAX_KT; ++ct) {
    if (ct < NT) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = (mx[r] == -INFINITY) ? 0.f : __expf(s[ct][r] - mx[r]);
        s[ct][r] = e;
        sum[r] += e;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) sum[r] += __shfl_xor(sum[r], o, 64);

  // P (pre-dropout) to global, P' = dropout(P) to this wave's LDS tile
  float* pw = Pw + w * 16 * PST;
#pragma unroll
  for (int ct = 0; ct < FWD_MAX_KT; ++ct) {
    if (ct < NT) {
      const int j = ct * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = q0 + fq * 4 + r;
        float pd = 0.f;
        if (i < Lq && j < Lk) {
          const float pr = s[ct][r] / sum[r];
          const long pi = (((long)b * H + h) * Lq + i) * Lk + j;
          P[pi] = pr;
          pd = pr * dropout_scale(seed, pi, drop_p);
        }
        pw[(fq * 4 + r) * PST + j] = pd;
      }
    }
  }
  wave_lds_sync();

  // O = P' V  (16 rows x dh16 columns, contraction over LkP keys)
  f32x4 o[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) o[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int NTd = dh16 / 16;
  for (int kk = 0; kk < LkP / 4; ++kk) {
    const float a = pw[fr * PST + kk * 4 + fq];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
      if (nt < NTd) o[nt] = mfma4(a, Vs[(kk * 4 + fq) * VST + nt * 16 + fr], o[nt]);
  }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int c = nt * 16 + fr;
    if (nt < NTd && c < dh)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = q0 + fq * 4 + r;
        if (i < Lq) O[((long)b * Lq + i) * ldo + h * dh + c] = o[nt][r];
      }
  }
}

static size_t mha_fwd_lds(int Lk, int dh, int waves) {
  const int LkP = pad16(Lk), dh16 = pad16(dh);
  return sizeof(float) * ((size_t)LkP * st_rows16(dh) + (size_t)LkP * st_rows4(dh16) + (size_t)waves * 16 * (LkP + 4));
}

MER_API int mer_mha_fwd(int B, int H, int Lq, int Lk, int dh, const float* Q, long ldq, const float* K, long ldk,
                        const float* V, long ldv, const float* bias, float* O, long ldo, float* P, float scale,
                        float drop_p, const unsigned long long* seed, unsigned long long site, void* stream) {
  if (B <= 0 || Lq <= 0) return 0;
  if (dh <= 0 || dh > 64 || (dh % 4) != 0 || Lk <= 0 || Lk > 16 * FWD_MAX_KT) return (int)hipErrorInvalidValue;
  // always 4 waves: all of them stage K/V, waves without query rows retire after the barrier
  const int waves = 4;
  const size_t lds = mha_fwd_lds(Lk, dh, waves);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&mha_fwd_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return (int)hipErrorInvalidConfiguration;
  dim3 grid(B * H, (Lq + 16 * waves - 1) / (16 * waves));
  hipLaunchKernelGGL(mha_fwd_kernel, grid, dim3(64 * waves), lds, (hipStream_t)stream, B, H, Lq, Lk, dh, Q, ldq, K, ldk,
                     V, ldv, bias, O, ldo, P, scale, drop_p, seed, site);
  MER_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// Backward, one block per (b, h):
//   dP'_ij = dO_i . V_j            dP = dP' * m            dS = P (dP - rowsum(P dP))
//   dQ = scale dS K                dK = scale dS^T Q       dV = P'^T dO        (P' = P * m)
// Phase A (waves over 16-row query tiles): dP' on MFMA, dS and P' into LDS (and, when dbias is wanted,
// dS over this head's slice of P, summed over heads by mha_dbias_kernel -- no atomics, deterministic).
// Phase B (waves over 16x16 output tiles of dQ, dK, dV): three MFMA products from LDS.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mha_bwd_kernel(int B, int H, int Lq, int Lk, int dh, const float* __restrict__ Q,
                                                      long ldq, const float* __restrict__ K, long ldk,
                                                      const float* __restrict__ V, long ldv, float* __restrict__ P,
                                                      const float* __restrict__ dO, long lddo, float* __restrict__ dQ,
                                                      long lddq, float* __restrict__ dK, long lddk,
                                                      float* __restrict__ dV, long lddv, int save_ds, float scale,
                                                      float drop_p, const unsigned long long* __restrict__ seed_ptr,
    unsigned long long site) {
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int LqP = pad16(Lq), LkP = pad16(Lk), dh16 = pad16(dh);
  const int ST = st_rows16(dh16), SST = st_rows16(LkP);
  float* Ks = smem;              // [LkP][ST]
  float* Vs = Ks + LkP * ST;     // [LkP][ST]
  float* Qs = Vs + LkP * ST;     // [LqP][ST]
  float* dOs = Qs + LqP * ST;    // [LqP][ST]
  float* dSs = dOs + LqP * ST;   // [LqP][SST]
  float* Pds = dSs + LqP * SST;  // [LqP][SST]  dropped-out probabilities P'
  const int b = blockIdx.x / H, h = blockIdx.x - (blockIdx.x / H) * H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  stage_head(Ks, ST, LkP, dh16, K, ldk, b, Lk, h, dh);
  stage_head(Vs, ST, LkP, dh16, V, ldv, b, Lk, h, dh);
  stage_head(Qs, ST, LqP, dh16, Q, ldq, b, Lq, h, dh);
  stage_head(dOs, ST, LqP, dh16, dO, lddo, b, Lq, h, dh);
  __syncthreads();

  const long pbase = ((long)b * H + h) * Lq * Lk;
  const int NT = LkP / 16;
  for (int it = w; it < LqP / 16; it += nw) {
    const int i0 = it * 16;
    f32x4 dp[FWD_MAX_KT];
#pragma unroll
    for (int ct = 0; ct < FWD_MAX_KT; ++ct) dp[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kk = 0; kk < dh / 4; ++kk) {
      const float a = dOs[(i0 + fr) * ST + kk * 4 + fq];
#pragma unroll
      for (int ct = 0; ct < FWD_MAX_KT; ++ct)
        if (ct < NT) dp[ct] = mfma4(a, Vs[(ct * 16 + fr) * ST + kk * 4 + fq], dp[ct]);
    }
    float pv[FWD_MAX_KT][4];
    float rd[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ct = 0; ct < FWD_MAX_KT; ++ct) {
      if (ct < NT) {
        const int j = ct * 16 + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = i0 + fq * 4 + r;
          float pij = 0.f, g = 0.f, pd = 0.f;
          if (i < Lq && j < Lk) {
            const long pi = pbase + (long)i * Lk + j;
            const float m = dropout_scale(seed, pi, drop_p);
            pij = P[pi];
            g = dp[ct][r] * m;
            pd = pij * m;
          }
          pv[ct][r] = pij;
          dp[ct][r] = g;
          rd[r] += pij * g;
          Pds[(i0 + fq * 4 + r) * SST + j] = pd;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) rd[r] += __shfl_xor(rd[r], o, 64);
#pragma unroll
    for (int ct = 0; ct < FWD_MAX_KT; ++ct) {
      if (ct < NT) {
        const int j = ct * 16 + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = i0 + fq * 4 + r;
          const float ds = pv[ct][r] * (dp[ct][r] - rd[r]);  // 0 outside [0,Lq) x [0,Lk)
          dSs[(i0 + fq * 4 + r) * SST + j] = ds;
          if (save_ds && i < Lq && j < Lk) P[pbase + (long)i * Lk + j] = ds;
        }
      }
    }
  }
  __syncthreads();

  // Phase B: output tiles of dQ [LqP x dh16], dK and dV [LkP x dh16]
  const int NC = dh16 / 16, nq = (LqP / 16) * NC, nk = (LkP / 16) * NC;
  for (int t = w; t < nq + 2 * nk; t += nw) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    if (t < nq) {  // dQ[i][c] = scale * sum_j dS[i][j] K[j][c]
      const int it = t / NC, ct = t - it * NC;
      for (int kk = 0; kk < LkP / 4; ++kk)
        acc = mfma4(dSs[(it * 16 + fr) * SST + kk * 4 + fq], Ks[(kk * 4 + fq) * ST + ct * 16 + fr], acc);
      const int c = ct * 16 + fr;
      if (c < dh)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = it * 16 + fq * 4 + r;
          if (i < Lq) dQ[((long)b * Lq + i) * lddq + h * dh + c] = scale * acc[r];
        }
    } else {
      const bool isk = t < nq + nk;
      const int u = isk ? t - nq : t - nq - nk;
      const int jt = u / NC, ct = u - jt * NC;
      const float* Aimg = isk ? dSs : Pds;  // A[j][i] = X[i][j]
      const float* Bimg = isk ? Qs : dOs;
      for (int kk = 0; kk < LqP / 4; ++kk)
        acc = mfma4(Aimg[(kk * 4 + fq) * SST + jt * 16 + fr], Bimg[(kk * 4 + fq) * ST + ct * 16 + fr], acc);
      const int c = ct * 16 + fr;
      if (c < dh)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = jt * 16 + fq * 4 + r;
          if (j < Lk) {
            if (isk) dK[((long)b * Lk + j) * lddk + h * dh + c] = scale * acc[r];
            else dV[((long)b * Lk + j) * lddv + h * dh + c] = acc[r];
          }
        }
    }
  }
}

// dbias[b][e] = sum_h dS[b][h][e]  (dS left in P by mha_bwd_kernel)
__global__ void mha_dbias_kernel(int B, int H, int LqLk, const float* __restrict__ dS, float* __restrict__ dbias) {
  const long n = (long)B * LqLk;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const long b = e / LqLk, k = e - b * LqLk;
    float s = 0.f;
    for (int h = 0; h < H; ++h) s += dS[(b * H + h) * LqLk + k];
    dbias[e] = s;
  }
}

static size_t mha_bwd_lds(int Lq, int Lk, int dh) {
  const int LqP = pad16(Lq), LkP = pad16(Lk), ST = st_rows16(pad16(dh)), SST = st_rows16(LkP);
  return sizeof(float) * ((size_t)2 * (LkP + LqP) * ST + (size_t)2 * LqP * SST);
}

MER_API int mer_mha_bwd(int B, int H, int Lq, int Lk, int dh, const float* Q, long ldq, const float* K, long ldk,
                        const float* V, long ldv, float* P, const float* dO, long lddo, float* dQ, long lddq,
                        float* dK, long lddk, float* dV, long lddv, float* dbias, float scale, float drop_p,
                        const unsigned long long* seed, unsigned long long site, void* stream) {
  if (B <= 0) return 0;
  if (dh <= 0 || dh > 64 || (dh % 4) != 0 || Lq <= 0 || Lk <= 0 || Lk > 16 * FWD_MAX_KT)
    return (int)hipErrorInvalidValue;
  const size_t lds = mha_bwd_lds(Lq, Lk, dh);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&mha_bwd_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return (int)hipErrorInvalidConfiguration;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(mha_bwd_kernel, dim3(B * H), dim3(256), lds, st, B, H, Lq, Lk, dh, Q, ldq, K, ldk, V, ldv, P, dO,
                     lddo, dQ, lddq, dK, lddk, dV, lddv, dbias ? 1 : 0, scale, drop_p, seed, site);
  if (dbias) {
    const long n = (long)B * Lq * Lk;
    const int grid = (int)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
    hipLaunchKernelGGL(mha_dbias_kernel, dim3(grid), dim3(256), 0, st, B, H, Lq * Lk, P, dbias);
  }
  MER_LAUNCH_CHECK();
}

// LDS bytes mer_mha_bwd needs for these shapes (callers pick the materialised-score path above 160 KiB)
MER_API int mer_mha_bwd_lds_bytes(int Lq, int Lk, int dh, long* bytes) {
  if (Lq <= 0 || Lk <= 0 || dh <= 0 || !bytes) return (int)hipErrorInvalidValue;
  *bytes = (long)mha_bwd_lds(Lq, Lk, dh);
  return 0;
}
