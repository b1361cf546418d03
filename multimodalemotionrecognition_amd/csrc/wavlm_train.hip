// WavLM stage-2 fine-tuning kernels: backward through the last N post-LN encoder layers
// (wavlm_audio.py:70-119 unfreeze_backbone -> train.py:817-829 stage-2 policy; layer math TF:147-336).
//
// Per trainable layer (M = B*L rows, d = 768, dh = 64):
//   forward   x -> qkv GEMM -> gated-rel-pos attention -> out-proj GEMM (+x) = y1 -> LN1 = x1
//             -> FFN1 GEMM = z -> GELU = f -> FFN2 GEMM (+x1) = y2 -> LN2 = out
//   backward  LN2 bwd (mer_ln_bwd) -> FFN2 wgrad / dgrad -> GELU bwd (mer_gelu_bwd) -> FFN1 wgrad / dgrad
//             -> LN1 bwd -> out-proj wgrad / dgrad -> attention bwd (rows + cols kernels, gate grads)
//             -> qkv wgrad / dgrad.  GEMMs run on the bf16 MFMA kernels (gemm_bf16.hip, conv.hip wgrad).
// Every reduction over rows writes per-block partial rows folded in a fixed order (mer_fold_rows):
// the backward is run-to-run deterministic (no float atomics).
#include "common.h"
#include "mer.h"

namespace {

typedef __attribute__((ext_vector_type(2))) float f32x2;

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

// ---------------------------------------------------------------------------------------------
// LayerNorm backward over rows of d (d % 256 == 0, d <= 1024).  g = dy_a (+ dy_b) (+ dy_c), recomputes
// (mean, rstd) from the saved pre-LN fp32 input.  dx = rstd * (g*gamma - mean(g*gamma) - xhat *
// mean(g*gamma*xhat)).  Each block owns LN_ROWS rows; it writes part[blk][0:d] = sum g*xhat (dgamma),
// part[blk][d:2d] = sum g (dbeta), part[blk][2d:3d] = sum dx (the bias gradient of the Linear whose
// output fed this LN through the residual sum).
constexpr int LN_ROWS = 16;
__global__ __launch_bounds__(256) void ln_bwd_kernel(int rows, int d, const float* __restrict__ dya,
                                                     const float* __restrict__ dyb, const float* __restrict__ dyc,
                                                     const float* __restrict__ x, const float* __restrict__ gamma,
                                                     float eps, float* __restrict__ dx32, bf16_t* __restrict__ dx16,
                                                     float* __restrict__ part) {
  __shared__ float red[4][3][1024];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nv = d / 256;  // float4 chunks per lane
  f32x4 adg[4], adb[4], adx[4], gm[4];
  for (int v = 0; v < 4; ++v) {
    adg[v] = adb[v] = adx[v] = f32x4{0.f, 0.f, 0.f, 0.f};
    gm[v] = v < nv ? *reinterpret_cast<const f32x4*>(gamma + v * 256 + lane * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int r0 = blockIdx.x * LN_ROWS;
  for (int rr = w; rr < LN_ROWS; rr += 4) {
    const int r = r0 + rr;
    if (r >= rows) break;
    const long base = (long)r * d;
    f32x4 xv[4], gv[4];
    float s = 0.f, ss = 0.f;
    for (int v = 0; v < nv; ++v) {
      const long o = base + v * 256 + lane * 4;
      xv[v] = *reinterpret_cast<const f32x4*>(x + o);
      f32x4 g = *reinterpret_cast<const f32x4*>(dya + o);
      if (dyb) g += *reinterpret_cast<const f32x4*>(dyb + o);
      if (dyc) g += *reinterpret_cast<const f32x4*>(dyc + o);
      gv[v] = g;
      for (int e = 0; e < 4; ++e) s += xv[v][e];
    }
    const float mean = wave_sum(s) / d;
    for (int v = 0; v < nv; ++v)
      for (int e = 0; e < 4; ++e) { const float t = xv[v][e] - mean; ss += t * t; }
    const float rstd = rsqrtf(wave_sum(ss) / d + eps);
    float a = 0.f, b = 0.f;
    for (int v = 0; v < nv; ++v)
      for (int e = 0; e < 4; ++e) {
        const float xh = (xv[v][e] - mean) * rstd;
        xv[v][e] = xh;
        const float gg = gv[v][e] * gm[v][e];
        a += gg;
        b += gg * xh;
      }
    const float ma = wave_sum(a) / d, mb = wave_sum(b) / d;
    for (int v = 0; v < nv; ++v) {
      f32x4 o;
      for (int e = 0; e < 4; ++e) {
        o[e] = rstd * (gv[v][e] * gm[v][e] - ma - xv[v][e] * mb);
        adg[v][e] += gv[v][e] * xv[v][e];
        adb[v][e] += gv[v][e];
        adx[v][e] += o[e];
      }
      const long off = base + v * 256 + lane * 4;
      if (dx32) *reinterpret_cast<f32x4*>(dx32 + off) = o;
      if (dx16) {
        uint2 pk;
        pk.x = (uint32_t)f2bf(o[0]) | ((uint32_t)f2bf(o[1]) << 16);
        pk.y = (uint32_t)f2bf(o[2]) | ((uint32_t)f2bf(o[3]) << 16);
        *reinterpret_cast<uint2*>(dx16 + off) = pk;
      }
    }
  }
  for (int v = 0; v < nv; ++v)
    for (int e = 0; e < 4; ++e) {
      const int c = v * 256 + lane * 4 + e;
      red[w][0][c] = adg[v][e];
      red[w][1][c] = adb[v][e];
      red[w][2][c] = adx[v][e];
    }
  __syncthreads();
  float* pr = part + (long)blockIdx.x * 3 * d;
  for (int i = threadIdx.x; i < 3 * d; i += 256) {
    const int q = i / d, c = i - q * d;
    pr[i] = ((red[0][q][c] + red[1][q][c]) + red[2][q][c]) + red[3][q][c];
  }
}

// out[k] += sum_p part[p * ldp + k] (fixed order), k < n.
__global__ __launch_bounds__(256) void fold_rows_kernel(int parts, int n, const float* __restrict__ part, long ldp,
                                                        float* __restrict__ out) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int p = 0;
  for (; p + 4 <= parts; p += 4) {
    s0 += part[(long)p * ldp + k];
    s1 += part[(long)(p + 1) * ldp + k];
    s2 += part[(long)(p + 2) * ldp + k];
    s3 += part[(long)(p + 3) * ldp + k];
  }
  for (; p < parts; ++p) s0 += part[(long)p * ldp + k];
  out[k] += (s0 + s1) + (s2 + s3);
}

// First stage of a long fold: split s of gridDim.y sums parts [s*chunk, (s+1)*chunk) of 64 columns, the 4 waves
// taking every 4th part, combined in a fixed order -> tmp[s][k].
__global__ __launch_bounds__(256) void fold_split_kernel(int parts, int n, const float* __restrict__ part, long ldp,
                                                         int chunk, float* __restrict__ tmp) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + lane;
  const int p0 = blockIdx.y * chunk, p1 = min(parts, p0 + chunk);
  float s0 = 0.f, s1 = 0.f;
  if (k < n) {
    int p = p0 + w;
    for (; p + 4 < p1; p += 8) {
      s0 += part[(long)p * ldp + k];
      s1 += part[(long)(p + 4) * ldp + k];
    }
    if (p < p1) s0 += part[(long)p * ldp + k];
  }
  red[w][lane] = s0 + s1;
  __syncthreads();
  if (w == 0 && k < n) tmp[(long)blockIdx.y * n + k] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// Column partial sums of a bf16 / fp32 matrix: part[blockIdx.y][c] = sum over COL_ROWS rows of x[r][c].
constexpr int COL_ROWS = 64;
template <typename T>
__global__ __launch_bounds__(256) void colpart_kernel(int rows, int cols, const T* __restrict__ x, long ldx,
                                                      float* __restrict__ part) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  const int r0 = blockIdx.y * COL_ROWS, r1 = min(rows, r0 + COL_ROWS);
  float s0 = 0.f, s1 = 0.f;
  int r = r0;
  for (; r + 2 <= r1; r += 2) {
    s0 += ldf<T>(x, (long)r * ldx + c);
    s1 += ldf<T>(x, (long)(r + 1) * ldx + c);
  }
  if (r < r1) s0 += ldf<T>(x, (long)r * ldx + c);
  part[(long)blockIdx.y * cols + c] = s0 + s1;
}

// f = gelu(z), bf16 -> bf16, 8 elements per thread.
__global__ __launch_bounds__(256) void gelu_bf16_kernel(long n8, const bf16_t* __restrict__ z, bf16_t* __restrict__ f) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  const uint4 v = reinterpret_cast<const uint4*>(z)[i];
  const uint32_t in[4] = {v.x, v.y, v.z, v.w};
  uint32_t out[4];
  for (int e = 0; e < 4; ++e) {
    const float a = gelu_erf(bf2f((bf16_t)(in[e] & 0xffff))), b = gelu_erf(bf2f((bf16_t)(in[e] >> 16)));
    out[e] = (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
  }
  reinterpret_cast<uint4*>(f)[i] = uint4{out[0], out[1], out[2], out[3]};
}

// dz = df * gelu'(z) (bf16 out) with per-block column partial sums of dz (the FFN1 bias gradient):
// block (column tile of 256, COL_ROWS rows).
__global__ __launch_bounds__(256) void gelu_bwd_kernel(int rows, int cols, const float* __restrict__ df,
                                                       const bf16_t* __restrict__ z, bf16_t* __restrict__ dz,
                                                       float* __restrict__ part) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  const int r0 = blockIdx.y * COL_ROWS, r1 = min(rows, r0 + COL_ROWS);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) {
    const long o = (long)r * cols + c;
    const float g = df[o] * gelu_erf_grad(bf2f(z[o]));
    dz[o] = f2bf(g);
    s += g;
  }
  part[(long)blockIdx.y * cols + c] = s;
}

// ---------------------------------------------------------------------------------------------
// Attention backward, WavLM gated relative position bias (TF:147-186 + F.multi_head_attention_forward).
//   s_ij = scale q_i.k_j + gate_i * tbl[h][j - i + L - 1],  p = softmax_j(s),  o_i = sum_j p_ij v_j
//   dp_ij = do_i.v_j,  ds_ij = p_ij (dp_ij - sum_j p_ij dp_ij)
//   dq_i = scale sum_j ds_ij k_j, dk_j = scale sum_i ds_ij q_i, dv_j = sum_i p_ij do_i
//   dgate_i = sum_j ds_ij tbl[h][j - i + L - 1] -> gate (gru_rel_pos_linear / const) gradients + dx_gate.
// Both kernels run their products on v_mfma_f32_16x16x32_bf16.  bf16 operands (q, k, v, x) are exact; fp32
// operands (dO in dp, dS in dq / dk, P in dv, the gate weight) are split into bf16 hi + lo fragments, so every
// product is fp32-accurate -- dp_ij - sum_j p_ij dp_ij cancels, and the gate-path gradients are held to 1e-4.
// Fragment maps (16x16x32): A lane = (row l & 15, k 8 (l >> 4) .. +7), B lane = (col l & 15, same k),
// C lane = (rows 4 (l >> 4) + r, col l & 15).
constexpr int AB_LMAX = 192;
constexpr int AB_ROWS = 64;       // query rows per rows-kernel block (16 per wave)
constexpr int AB_COLS = 32;       // key columns per cols-kernel block (16 per wave pair)
constexpr int AB_KP = 72;         // bf16 row pitch of K / V in LDS (144 B: 16-byte aligned fragment reads)
constexpr int GATE_PART = 8 * 64 + 8;  // + H (gate const) per partial row

__device__ __forceinline__ f32x4 mma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
union AbFrag {
  bf16x8 v;
  u32x4 u;
  uint16_t h[8];
};
typedef __attribute__((ext_vector_type(8))) float f32x8;
__device__ __forceinline__ void ab_split(f32x4 a, f32x4 b, bf16x8& hi, bf16x8& lo) {
  const f32x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  hi = __builtin_convertvector(v, bf16x8);
  lo = __builtin_convertvector(v - __builtin_convertvector(hi, f32x8), bf16x8);
}
// sum / max over the 16 lanes of a fragment row group (lanes sharing l >> 4)
__device__ __forceinline__ float grp_sum(float v) {
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  return v + __shfl_xor(v, 8);
}
__device__ __forceinline__ float grp_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 1));
  v = fmaxf(v, __shfl_xor(v, 2));
  v = fmaxf(v, __shfl_xor(v, 4));
  return fmaxf(v, __shfl_xor(v, 8));
}

// LDS plan of the rows kernel for NT 16-key tiles (KP = 16 NT padded keys)
template <int NT>
struct RowsLds {
  static constexpr int KP = 16 * NT, KTP = KP + 8, DSP = KP + 4;
  static constexpr int ks = 0;                                   // K [KP][AB_KP] bf16
  static constexpr int vs = ks + KP * AB_KP * 2;                 // V [KP][AB_KP] bf16
  static constexpr int kt = vs + KP * AB_KP * 2;                 // K^T [64][KTP] bf16
  static constexpr int ds = kt + 64 * KTP * 2;                   // per-wave dS tiles [4][16][DSP] fp32
  static constexpr int tb = ds + 4 * 16 * DSP * 4;               // bias row tbl[h] [2 KP] fp32
  static constexpr int bytes = tb + 2 * KP * 4;
  static_assert(16 * DSP >= GATE_PART + 1, "gate partial reduction reuses the dS tiles");
};

// Rows kernel: block = 64 query rows of one (b, h), 4 waves x 16 rows.  Stages K, V (row-major, the B operands of
// S = Q K^T and dP = dO V^T) and K^T (the B operand of dQ = dS K) in LDS with zero rows past L; each wave
// keeps its 16 x KP score / dP tiles in registers (softmax, dS, dgate by 16-lane shuffles), writes P and dS rows
// (fp32 scratch [B*H][L][L]) for the cols kernel, stages its dS tile in LDS for dQ, and folds the gate backward
// into the per-block partial row [8][64] weight, [8] bias, [H] const (this head's entry only).
template <int NT>
__global__ __launch_bounds__(256) void wavlm_attn_bwd_rows_kernel(
    int L, int H, const bf16_t* __restrict__ qkv, long ldqkv, const bf16_t* __restrict__ x, long ldx,
    const float* __restrict__ dout, long ldo, const float* __restrict__ gate_w, const float* __restrict__ gate_b,
    const float* __restrict__ gate_c, const float* __restrict__ tbl, float scale, float* __restrict__ Pbuf,
    float* __restrict__ dSbuf, bf16_t* __restrict__ dqkv, long lddq, float* __restrict__ dxg, long lddxg,
    float* __restrict__ gpart) {
  typedef RowsLds<NT> Ly;
  constexpr int KP = Ly::KP, KTP = Ly::KTP, DSP = Ly::DSP;
  extern __shared__ __attribute__((aligned(16))) unsigned char ab_smem[];
  bf16_t* Ks = reinterpret_cast<bf16_t*>(ab_smem + Ly::ks);
  bf16_t* Vs = reinterpret_cast<bf16_t*>(ab_smem + Ly::vs);
  bf16_t* KsT = reinterpret_cast<bf16_t*>(ab_smem + Ly::kt);
  float* dSw = reinterpret_cast<float*>(ab_smem + Ly::ds);
  float* tbs = reinterpret_cast<float*>(ab_smem + Ly::tb);
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, fr = lane & 15, fq = lane >> 4, fk = 8 * fq;
  const int D = H * 64;
  // stage K, V (16-byte chunks) and K^T; rows L..KP-1 are zero (their products must be finite zeros)
  for (int ch = t; ch < KP * 8; ch += 256) {
    const int j = ch >> 3, c8 = (ch & 7) * 8;
    const long g = (long)(b * L + (j < L ? j : L - 1)) * ldqkv + h * 64 + c8;
    u32x4 kv = *reinterpret_cast<const u32x4*>(qkv + g + D);
    u32x4 vv = *reinterpret_cast<const u32x4*>(qkv + g + 2 * D);
    if (j >= L) kv = vv = u32x4{0u, 0u, 0u, 0u};
    *reinterpret_cast<u32x4*>(Ks + j * AB_KP + c8) = kv;
    *reinterpret_cast<u32x4*>(Vs + j * AB_KP + c8) = vv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      KsT[(c8 + 2 * e) * KTP + j] = (bf16_t)(kv[e] & 0xffff);
      KsT[(c8 + 2 * e + 1) * KTP + j] = (bf16_t)(kv[e] >> 16);
    }
  }
  const float* th = tbl + (long)h * (2 * L - 1);
  for (int k = t; k < 2 * L - 1; k += 256) tbs[k] = th[k];

  // this wave's operand fragments: q, x (bf16, exact), dO split, gate weight split (cols 0..7 valid)
  const int i0 = blockIdx.x * AB_ROWS + w * 16;
  const long rowa = (long)(b * L + (i0 + fr < L ? i0 + fr : L - 1));
  AbFrag qa[2], xa[2];
  bf16x8 oh[2], ol[2], gh[2], gl[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int c = h * 64 + 32 * s + fk;
    qa[s].u = *reinterpret_cast<const u32x4*>(qkv + rowa * ldqkv + c);
    xa[s].u = *reinterpret_cast<const u32x4*>(x + rowa * ldx + c);
    const float* po = dout + rowa * ldo + c;
    ab_split(*reinterpret_cast<const f32x4*>(po), *reinterpret_cast<const f32x4*>(po + 4), oh[s], ol[s]);
    const float* pw = gate_w + (fr & 7) * 64 + 32 * s + fk;
    f32x4 w0 = *reinterpret_cast<const f32x4*>(pw), w1 = *reinterpret_cast<const f32x4*>(pw + 4);
    if (fr >= 8) w0 = w1 = f32x4{0.f, 0.f, 0.f, 0.f};
    ab_split(w0, w1, gh[s], gl[s]);
  }
  // gate (TF:167-177): z[row][n] = x_h . gate_w[n] + gate_b[n]; pa = sum n<4, pb = sum 4<=n<8
  f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    z = mma16(xa[s].v, gh[s], z);
    z = mma16(xa[s].v, gl[s], z);
  }
  const float gbn = fr < 8 ? gate_b[fr & 7] : 0.f, gc = gate_c[h];
  float ga[4], gb[4], gate[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = fr < 8 ? z[r] + gbn : 0.f;
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    ga[r] = sigmoidf_(__shfl(v, fq * 16));
    gb[r] = sigmoidf_(__shfl(v, fq * 16 + 4));
    gate[r] = ga[r] * (gb[r] * gc - 1.f) + 2.f;
  }
  __syncthreads();

  // S = Q K^T (exact), dP = dO V^T (split dO): 16 x KP per wave in registers
  f32x4 s[NT], dp[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    const bf16_t* kr = Ks + (16 * tt + fr) * AB_KP + fk;
    const bf16_t* vr = Vs + (16 * tt + fr) * AB_KP + fk;
    AbFrag k0, k1, v0, v1;
    k0.u = *reinterpret_cast<const u32x4*>(kr);
    k1.u = *reinterpret_cast<const u32x4*>(kr + 32);
    v0.u = *reinterpret_cast<const u32x4*>(vr);
    v1.u = *reinterpret_cast<const u32x4*>(vr + 32);
    const f32x4 zz = f32x4{0.f, 0.f, 0.f, 0.f};
    s[tt] = mma16(qa[1].v, k1.v, mma16(qa[0].v, k0.v, zz));
    f32x4 d = mma16(oh[0], v0.v, zz);
    d = mma16(ol[0], v0.v, d);
    d = mma16(oh[1], v1.v, d);
    dp[tt] = mma16(ol[1], v1.v, d);
  }
  const int ib = i0 + 4 * fq;  // this lane's rows ib + r
  const int tmax = 2 * L - 2;
  float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    const int j = 16 * tt + fr;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = min(max(j - (ib + r) + L - 1, 0), tmax);
      const float v = j < L ? s[tt][r] * scale + gate[r] * tbs[k] : -INFINITY;
      s[tt][r] = v;
      mx[r] = fmaxf(mx[r], v);
    }
  }
  float sum[4], Dr[4], dg[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    mx[r] = grp_max(mx[r]);
    sum[r] = 0.f;
  }
#pragma unroll
  for (int tt = 0; tt < NT; ++tt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[tt][r] = __expf(s[tt][r] - mx[r]);
      sum[r] += s[tt][r];
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    sum[r] = 1.f / grp_sum(sum[r]);
    Dr[r] = 0.f;
  }
#pragma unroll
  for (int tt = 0; tt < NT; ++tt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[tt][r] *= sum[r];
      Dr[r] += s[tt][r] * dp[tt][r];
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    Dr[r] = grp_sum(Dr[r]);
    dg[r] = 0.f;
  }
  float* dsw = dSw + w * 16 * DSP;
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    const int j = 16 * tt + fr;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = ib + r;
      const float ds = s[tt][r] * (dp[tt][r] - Dr[r]);  // 0 for keys past L (p = 0, dp = 0)
      dg[r] += ds * tbs[min(max(j - i + L - 1, 0), tmax)];
      dsw[(4 * fq + r) * DSP + j] = ds;
      if (i < L && j < L) {
        const long o = ((long)bh * L + i) * L + j;
        Pbuf[o] = s[tt][r];
        dSbuf[o] = ds;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");

  // dQ = scale dS K: A = this wave's dS tile (split), B = K^T rows (exact); 4 tiles of 16 dims
  f32x4 dq[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) dq[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KP / 32; ++ks) {
    const float* ap = dsw + fr * DSP + 32 * ks + fk;
    bf16x8 ah, al;
    ab_split(*reinterpret_cast<const f32x4*>(ap), *reinterpret_cast<const f32x4*>(ap + 4), ah, al);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      AbFrag kb;
      kb.u = *reinterpret_cast<const u32x4*>(KsT + (16 * c + fr) * KTP + 32 * ks + fk);
      dq[c] = mma16(ah, kb.v, dq[c]);
      dq[c] = mma16(al, kb.v, dq[c]);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = ib + r;
    if (i < L) {
      bf16_t* o = dqkv + (long)(b * L + i) * lddq + h * 64 + fr;
#pragma unroll
      for (int c = 0; c < 4; ++c) o[16 * c] = f2bf(dq[c][r] * scale);
    }
  }

  // gate backward: gate = ga (gb c - 1) + 2, pa / pb = sums of 4 projections each
  float dpa[4], dpb[4], gcl = 0.f, gal = 0.f, gbl = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float g = ib + r < L ? grp_sum(dg[r]) : 0.f;
    dpa[r] = g * (gb[r] * gc - 1.f) * ga[r] * (1.f - ga[r]);
    dpb[r] = g * ga[r] * gc * gb[r] * (1.f - gb[r]);
    gcl += g * ga[r] * gb[r];
    gal += dpa[r];
    gbl += dpb[r];
  }
  // lane = d: dW[n][d] += dp{a,b} x[row][d] over the wave's 16 rows, dx_gate = dpa wsa + dpb wsb
  float wsa = 0.f, wsb = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    wsa += gate_w[r * 64 + lane];
    wsb += gate_w[(r + 4) * 64 + lane];
  }
  float xd[16];
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) xd[rr] = bf2f(x[(long)(b * L + min(i0 + rr, L - 1)) * ldx + h * 64 + lane]);
  float wa = 0.f, wb = 0.f;
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) {
    const float a = __shfl(dpa[rr & 3], (rr >> 2) * 16), c = __shfl(dpb[rr & 3], (rr >> 2) * 16);
    wa += a * xd[rr];
    wb += c * xd[rr];
    if (dxg && i0 + rr < L) dxg[(long)(b * L + i0 + rr) * lddxg + h * 64 + lane] = a * wsa + c * wsb;
  }
  // one copy per 16-lane group of the row-replicated sums
  gal = __shfl(gal, 0) + __shfl(gal, 16) + __shfl(gal, 32) + __shfl(gal, 48);
  gbl = __shfl(gbl, 0) + __shfl(gbl, 16) + __shfl(gbl, 32) + __shfl(gbl, 48);
  gcl = __shfl(gcl, 0) + __shfl(gcl, 16) + __shfl(gcl, 32) + __shfl(gcl, 48);
  __syncthreads();  // every wave is done with its dS tile: reuse them for the block reduction
  float* red = dSw;  // [4][GATE_PART + 1]
  constexpr int RP = GATE_PART + 1;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[w * RP + r * 64 + lane] = wa;
    red[w * RP + (r + 4) * 64 + lane] = wb;
  }
  if (lane < 8) red[w * RP + 512 + lane] = lane < 4 ? gal : gbl;
  if (lane == 0) red[w * RP + GATE_PART] = gcl;
  __syncthreads();
  float* pr = gpart + ((long)bh * gridDim.x + blockIdx.x) * (GATE_PART + H);
  for (int k = t; k < GATE_PART + H; k += 256) {
    float v;
    if (k < GATE_PART) v = ((red[k] + red[RP + k]) + red[2 * RP + k]) + red[3 * RP + k];
    else
      v = (k - GATE_PART == h)
              ? ((red[GATE_PART] + red[RP + GATE_PART]) + red[2 * RP + GATE_PART]) + red[3 * RP + GATE_PART]
              : 0.f;
    pr[k] = v;
  }
}

// LDS plan of the cols kernel for NI 32-row query steps (IP = 32 NI padded query rows)
template <int NI>
struct ColsLds {
  static constexpr int IP = 32 * NI, TP = IP + 4, BP = IP + 8;
  static constexpr int ps = 0;                      // P^T strip [32][TP] fp32
  static constexpr int ds = ps + 32 * TP * 4;       // dS^T strip [32][TP] fp32
  static constexpr int qt = ds + 32 * TP * 4;       // Q^T [64][BP] bf16
  static constexpr int ot = qt + 64 * BP * 2;       // dO^T [64][BP] bf16
  static constexpr int bytes = ot + 64 * BP * 2;
};

// Cols kernel: block = 32 keys of one (b, h); wave w = (key half w & 1, dim half w >> 1).
//   dK = scale dS^T Q (split dS, exact q), dV = P^T dO (split P; dO rounded to bf16 -- dv has no cancellation).
// The P / dS column strips are staged transposed (contiguous A fragments), Q / dO transposed (contiguous B).
template <int NI>
__global__ __launch_bounds__(256) void wavlm_attn_bwd_cols_kernel(int L, int H, const bf16_t* __restrict__ qkv,
                                                                  long ldqkv, const float* __restrict__ dout, long ldo,
                                                                  const float* __restrict__ Pbuf,
                                                                  const float* __restrict__ dSbuf, float scale,
                                                                  bf16_t* __restrict__ dqkv, long lddq) {
  typedef ColsLds<NI> Ly;
  constexpr int IP = Ly::IP, TP = Ly::TP, BP = Ly::BP;
  extern __shared__ __attribute__((aligned(16))) unsigned char ab_smem[];
  float* PsT = reinterpret_cast<float*>(ab_smem + Ly::ps);
  float* DsT = reinterpret_cast<float*>(ab_smem + Ly::ds);
  bf16_t* QT = reinterpret_cast<bf16_t*>(ab_smem + Ly::qt);
  bf16_t* OT = reinterpret_cast<bf16_t*>(ab_smem + Ly::ot);
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, fr = lane & 15, fq = lane >> 4, fk = 8 * fq;
  const int D = H * 64;
  const int j0 = blockIdx.x * AB_COLS;
  for (int ch = t; ch < IP * 8; ch += 256) {
    const int i = ch >> 3, c8 = (ch & 7) * 8;
    const long row = (long)(b * L + (i < L ? i : L - 1));
    const u32x4 qv = *reinterpret_cast<const u32x4*>(qkv + row * ldqkv + h * 64 + c8);
    const f32x4 o0 = *reinterpret_cast<const f32x4*>(dout + row * ldo + h * 64 + c8);
    const f32x4 o1 = *reinterpret_cast<const f32x4*>(dout + row * ldo + h * 64 + c8 + 4);
    const bool ok = i < L;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      QT[(c8 + 2 * e) * BP + i] = ok ? (bf16_t)(qv[e] & 0xffff) : (bf16_t)0;
      QT[(c8 + 2 * e + 1) * BP + i] = ok ? (bf16_t)(qv[e] >> 16) : (bf16_t)0;
      OT[(c8 + e) * BP + i] = ok ? f2bf(o0[e]) : (bf16_t)0;
      OT[(c8 + 4 + e) * BP + i] = ok ? f2bf(o1[e]) : (bf16_t)0;
    }
  }
  for (int e = t; e < IP * AB_COLS; e += 256) {
    const int i = e >> 5, jc = e & 31, j = j0 + jc;
    const long o = ((long)bh * L + (i < L ? i : L - 1)) * L + (j < L ? j : L - 1);
    const float pv = Pbuf[o], dv = dSbuf[o];
    const bool ok = i < L && j < L;
    PsT[jc * TP + i] = ok ? pv : 0.f;
    DsT[jc * TP + i] = ok ? dv : 0.f;
  }
  __syncthreads();
  const int kt = w & 1, dd = w >> 1;
  f32x4 dk[2], dv[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) dk[c] = dv[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < NI; ++ks) {
    const int a = (16 * kt + fr) * TP + 32 * ks + fk;
    bf16x8 dh, dl, ph, pl;
    ab_split(*reinterpret_cast<const f32x4*>(DsT + a), *reinterpret_cast<const f32x4*>(DsT + a + 4), dh, dl);
    ab_split(*reinterpret_cast<const f32x4*>(PsT + a), *reinterpret_cast<const f32x4*>(PsT + a + 4), ph, pl);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int n = 32 * dd + 16 * c + fr;
      AbFrag qb, ob;
      qb.u = *reinterpret_cast<const u32x4*>(QT + n * BP + 32 * ks + fk);
      ob.u = *reinterpret_cast<const u32x4*>(OT + n * BP + 32 * ks + fk);
      dk[c] = mma16(dh, qb.v, dk[c]);
      dk[c] = mma16(dl, qb.v, dk[c]);
      dv[c] = mma16(ph, ob.v, dv[c]);
      dv[c] = mma16(pl, ob.v, dv[c]);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = j0 + 16 * kt + 4 * fq + r;
    if (j < L) {
      bf16_t* o = dqkv + (long)(b * L + j) * lddq + h * 64 + 32 * dd + fr;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        o[D + 16 * c] = f2bf(dk[c][r] * scale);
        o[2 * D + 16 * c] = f2bf(dv[c][r]);
      }
    }
  }
}

template <int NT>
int wavlm_attention_bwd_launch(int B, int L, int H, const bf16_t* qkv, long ldqkv, const bf16_t* x, long ldx,
                               const float* dout, long ldo, const float* gate_w, const float* gate_b,
                               const float* gate_c, const float* tbl, float scale, float* P, float* dS, bf16_t* dqkv,
                               long lddq, float* dxg, long lddxg, float* gpart, hipStream_t st) {
  constexpr int rb = RowsLds<NT>::bytes, cb = ColsLds<NT / 2>::bytes;
  static_assert(rb <= 160 * 1024 && cb <= 160 * 1024, "LDS");
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&wavlm_attn_bwd_rows_kernel<NT>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, rb) != hipSuccess ||
      hipFuncSetAttribute(reinterpret_cast<const void*>(&wavlm_attn_bwd_cols_kernel<NT / 2>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, cb) != hipSuccess)
    return (int)hipErrorInvalidConfiguration;
  hipLaunchKernelGGL(wavlm_attn_bwd_rows_kernel<NT>, dim3((L + AB_ROWS - 1) / AB_ROWS, B * H), dim3(256), rb, st, L, H,
                     qkv, ldqkv, x, ldx, dout, ldo, gate_w, gate_b, gate_c, tbl, scale, P, dS, dqkv, lddq, dxg, lddxg,
                     gpart);
  hipLaunchKernelGGL(wavlm_attn_bwd_cols_kernel<NT / 2>, dim3((L + AB_COLS - 1) / AB_COLS, B * H), dim3(256), cb, st,
                     L, H, qkv, ldqkv, dout, ldo, P, dS, scale, dqkv, lddq);
  return (int)hipGetLastError();
}

}  // namespace

MER_API int mer_ln_bwd(int rows, int d, const float* dy_a, const float* dy_b, const float* dy_c, const float* x,
                       const float* gamma, float eps, float* dx32, void* dx16, float* part, void* stream) {
  if (d % 256 || d > 1024 || rows <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ln_bwd_kernel, dim3((rows + LN_ROWS - 1) / LN_ROWS), dim3(256), 0, (hipStream_t)stream, rows, d,
                     dy_a, dy_b, dy_c, x, gamma, eps, dx32, (bf16_t*)dx16, part);
  MER_LAUNCH_CHECK();
}

MER_API int mer_fold_rows(int parts, int n, const float* part, long ldp, float* out, float* workspace, void* stream) {
  if (parts <= 0 || n <= 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (parts > 64) {  // two stages: <= 64 split rows of the same fixed-order sum, then the short fold below
    if (!workspace) return (int)hipErrorInvalidValue;
    const int S = min(64, (parts + 63) / 64), chunk = (parts + S - 1) / S;
    hipLaunchKernelGGL(fold_split_kernel, dim3((n + 63) / 64, S), dim3(256), 0, st, parts, n, part, ldp, chunk,
                       workspace);
    part = workspace;
    ldp = n;
    parts = S;
  }
  hipLaunchKernelGGL(fold_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, st, parts, n, part, ldp, out);
  MER_LAUNCH_CHECK();
}

MER_API int mer_colpart(int rows, int cols, const void* x, int x_dtype, long ldx, float* part, void* stream) {
  dim3 grid((cols + 255) / 256, (rows + COL_ROWS - 1) / COL_ROWS);
  if (x_dtype == MER_BF16)
    hipLaunchKernelGGL(colpart_kernel<bf16_t>, grid, dim3(256), 0, (hipStream_t)stream, rows, cols, (const bf16_t*)x,
                       ldx, part);
  else
    hipLaunchKernelGGL(colpart_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, rows, cols, (const float*)x,
                       ldx, part);
  MER_LAUNCH_CHECK();
}

MER_API int mer_gelu_bf16(long n, const void* z, void* f, void* stream) {
  if (n % 8) return (int)hipErrorInvalidValue;
  const long n8 = n / 8;
  hipLaunchKernelGGL(gelu_bf16_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n8,
                     (const bf16_t*)z, (bf16_t*)f);
  MER_LAUNCH_CHECK();
}

MER_API int mer_gelu_bwd(int rows, int cols, const float* df, const void* z, void* dz, float* part, void* stream) {
  dim3 grid((cols + 255) / 256, (rows + COL_ROWS - 1) / COL_ROWS);
  hipLaunchKernelGGL(gelu_bwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, rows, cols, df, (const bf16_t*)z,
                     (bf16_t*)dz, part);
  MER_LAUNCH_CHECK();
}

MER_API int mer_wavlm_attention_bwd(int B, int L, int H, const void* qkv, long ldqkv, const void* x, long ldx,
                                    const void* dout, long ldo, const float* gate_w, const float* gate_b,
                                    const float* gate_const, const float* tbl, float scale, float* P, float* dS,
                                    void* dqkv, long lddq, float* dx_gate, long lddxg, float* gate_part,
                                    void* stream) {
  if (L <= 0 || L > AB_LMAX || ldqkv % 8 || ldx % 8 || ldo % 4 || B <= 0 || H <= 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int nt = (L + 15) / 16;  // 16-key tiles; the kernels are built for 4 / 8 / 10 / 12 (L <= 64 / 128 / 160 / 192)
#define MER_AB_LAUNCH(NT)                                                                                             \
  wavlm_attention_bwd_launch<NT>(B, L, H, (const bf16_t*)qkv, ldqkv, (const bf16_t*)x, ldx, (const float*)dout, ldo, \
                                 gate_w, gate_b, gate_const, tbl, scale, P, dS, (bf16_t*)dqkv, lddq, dx_gate, lddxg,  \
                                 gate_part, st)
  const int rc = nt <= 4 ? MER_AB_LAUNCH(4) : nt <= 8 ? MER_AB_LAUNCH(8) : nt <= 10 ? MER_AB_LAUNCH(10) : MER_AB_LAUNCH(12);
#undef MER_AB_LAUNCH
  return rc;
}

namespace {
// 64x64 tile transpose through LDS (bf16): dst[c][r] = src[r][c].
__global__ __launch_bounds__(256) void transpose_bf16_kernel(int rows, int cols, const bf16_t* __restrict__ src,
                                                             long lds, bf16_t* __restrict__ dst, long ldd) {
  __shared__ bf16_t tile[64][66];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < rows && c < cols) ? src[(long)r * lds + c] : (bf16_t)0;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, r = r0 + tx;
    if (c < cols && r < rows) dst[(long)c * ldd + r] = tile[tx][i];
  }
}
}  // namespace

MER_API int mer_transpose_bf16(int rows, int cols, const void* src, long lds, void* dst, long ldd, void* stream) {
  if (rows <= 0 || cols <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((cols + 63) / 64, (rows + 63) / 64), dim3(256), 0, (hipStream_t)stream,
                     rows, cols, (const bf16_t*)src, lds, (bf16_t*)dst, ldd);
  MER_LAUNCH_CHECK();
}
