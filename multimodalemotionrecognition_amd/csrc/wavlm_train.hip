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
// operands (dO in dp, dS in dq / dk, the gate weight) are split into bf16 hi + lo fragments, so those products
// are fp32-accurate -- dp_ij - sum_j p_ij dp_ij cancels, and the gate-path gradients are held to 1e-4.  Only
// dv = P^T dO runs on single bf16 P and dO (no cancellation there).
// Fragment maps (16x16x32): A lane = (row l & 15, k 8 (l >> 4) .. +7), B lane = (col l & 15, same k),
// C lane = (rows 4 (l >> 4) + r, col l & 15).  Transposed operands come from row-major LDS images through
// ds_read_b64_tr_b16 (lane 4q + p of a 16-lane group addresses row q, columns 4p..4p+3 of a 4-row block and
// receives column (lane & 15) of the 4 rows).
// Scratch between the two kernels (KP = key / query count padded to 16 NT): P, dS hi, dS lo as bf16
// [B*H][KP query rows][KP keys] (rows / keys past L zero), then dO rounded to bf16 [B*H][KP][64].
constexpr int AB_LMAX = 192;
constexpr int AB_ROWS = 64;       // query rows per rows-kernel block (16 per wave)
constexpr int AB_COLS = 32;       // keys per cols-kernel block (16 per wave pair)
constexpr int AB_KP = 72;         // bf16 row pitch of K / V / Q / dO images in LDS (144 B)
constexpr int AB_SP = 40;         // bf16 row pitch of the P / dS strips in LDS (80 B)
constexpr int GATE_PART = 8 * 64 + 8;  // + H (gate const) per partial row

__device__ __forceinline__ f32x4 mma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
typedef __attribute__((ext_vector_type(4))) short s16x4;
union AbFrag {
  bf16x8 v;
  u32x4 u;
};
typedef __attribute__((ext_vector_type(8))) float f32x8;
__device__ __forceinline__ void ab_split8(const f32x8 v, bf16x8& hi, bf16x8& lo) {
  hi = __builtin_convertvector(v, bf16x8);
  lo = __builtin_convertvector(v - __builtin_convertvector(hi, f32x8), bf16x8);
}
__device__ __forceinline__ void ab_split(f32x4 a, f32x4 b, bf16x8& hi, bf16x8& lo) {
  ab_split8(f32x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]}, hi, lo);
}
// 4 bf16 of a 4-row block, transposed (see above); p must be 8-byte aligned, every lane active
__device__ __forceinline__ u32x2 tr_read(const bf16_t* p) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
  return __builtin_bit_cast(u32x2, v);
}
__device__ __forceinline__ bf16x8 tr_frag(const bf16_t* p0, const bf16_t* p1) {
  const u32x2 a = tr_read(p0), b = tr_read(p1);
  AbFrag f;
  f.u = u32x4{a[0], a[1], b[0], b[1]};
  return f.v;
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

template <int NT>
struct RowsLds {
  static constexpr int KP = 16 * NT;
  static constexpr int ks = 0;                    // K [KP][AB_KP] bf16
  static constexpr int vs = ks + KP * AB_KP * 2;  // V [KP][AB_KP] bf16; the gate partial reduction reuses it
  static constexpr int tb = vs + KP * AB_KP * 2;  // bias row tbl[h] [512] fp32 (2L - 1 used)
  static constexpr int bytes = tb + 512 * 4;
  static_assert(KP * AB_KP * 2 >= 4 * (GATE_PART + 1) * 4, "gate partial reduction reuses the V image");
};

// Rows kernel (one-dimensional grid, XCD-aware block -> (row block, b*h)): block = 64 query rows of one (b, h), 4 waves x 16 rows, query row on the lane (l & 15).  Stages K,
// V row-major in LDS (zero rows past L).  Per wave, in registers: S^T = K Q^T and dP^T = V dO^T tiles (keys on
// the accumulator rows), softmax / dS / dgate by register sums + 2 shuffles, dQ^T = K^T dS^T with dS^T taken
// straight from the accumulators (tile pair -> one k step, K^T by transposed LDS reads in the matching k order).
// Writes P / dS hi / dS lo scratch rows, dq, dx_gate and the per-block gate partial row
// [8][64] weight, [8] bias, [H] const (this head's entry only).
template <int NT>
__global__ __launch_bounds__(256) void wavlm_attn_bwd_rows_kernel(
    int L, int H, const bf16_t* __restrict__ qkv, long ldqkv, const bf16_t* __restrict__ x, long ldx,
    const float* __restrict__ dout, long ldo, const float* __restrict__ gate_w, const float* __restrict__ gate_b,
    const float* __restrict__ gate_c, const float* __restrict__ tbl, float scale, int nbh, bf16_t* __restrict__ scr,
    bf16_t* __restrict__ dqkv, long lddq, float* __restrict__ dxg, long lddxg, float* __restrict__ gpart,
    float drop_p, const unsigned long long* __restrict__ seed_ptr, unsigned long long site) {
  typedef RowsLds<NT> Ly;
  constexpr int KP = Ly::KP;
  extern __shared__ __attribute__((aligned(16))) unsigned char ab_smem[];
  bf16_t* Ks = reinterpret_cast<bf16_t*>(ab_smem + Ly::ks);
  bf16_t* Vs = reinterpret_cast<bf16_t*>(ab_smem + Ly::vs);
  float* tbs = reinterpret_cast<float*>(ab_smem + Ly::tb);
  const int nrb = (L + AB_ROWS - 1) / AB_ROWS;
  int rb, bh;  // the row blocks of one (b, h) share its K / V: keep them on one XCD (one L2)
  xcd_tile(blockIdx.x, nrb, nrb * nbh, rb, bh);
  const int b = bh / H, h = bh - b * H;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, fr = lane & 15, fq = lane >> 4, fk = 8 * fq;
  const int D = H * 64;
  // staging loads all issued before the first LDS store (KP * 8 16-byte chunks = NT / 2 per thread)
  u32x4 kv[NT / 2], vv[NT / 2];
#pragma unroll
  for (int it = 0; it < NT / 2; ++it) {
    const int ch = t + 256 * it, j = ch >> 3, c8 = (ch & 7) * 8;
    const long g = (long)(b * L + (j < L ? j : L - 1)) * ldqkv + h * 64 + c8;
    kv[it] = *reinterpret_cast<const u32x4*>(qkv + g + D);
    vv[it] = *reinterpret_cast<const u32x4*>(qkv + g + 2 * D);
  }
  const float* th = tbl + (long)h * (2 * L - 1);
  const float tb_a = th[min(t, 2 * L - 2)], tb_b = th[min(t + 256, 2 * L - 2)];

  // B operands (query row i = i0 + (l & 15) on the lane): q, x exact, dO split; A operand: gate weight rows split
  const int i0 = rb * AB_ROWS + w * 16, i = i0 + fr;
  // gate-backward operands, loaded now so their latency hides behind the staging (lane = d): the wave's 16 x
  // rows, column sums of the gate weight halves
  bf16_t xr[16];
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) xr[rr] = x[(long)(b * L + min(i0 + rr, L - 1)) * ldx + h * 64 + lane];
  float wsa = 0.f, wsb = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    wsa += gate_w[r * 64 + lane];
    wsb += gate_w[(r + 4) * 64 + lane];
  }
  const long rowa = (long)(b * L + (i < L ? i : L - 1));
  AbFrag qb[2], xb[2];
  bf16x8 oh[2], ol[2], gh[2], gl[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int c = h * 64 + 32 * s + fk;
    qb[s].u = *reinterpret_cast<const u32x4*>(qkv + rowa * ldqkv + c);
    xb[s].u = *reinterpret_cast<const u32x4*>(x + rowa * ldx + c);
    const float* po = dout + rowa * ldo + c;
    ab_split(*reinterpret_cast<const f32x4*>(po), *reinterpret_cast<const f32x4*>(po + 4), oh[s], ol[s]);
    const float* pw = gate_w + (fr & 7) * 64 + 32 * s + fk;
    f32x4 w0 = *reinterpret_cast<const f32x4*>(pw), w1 = *reinterpret_cast<const f32x4*>(pw + 4);
    if (fr >= 8) w0 = w1 = f32x4{0.f, 0.f, 0.f, 0.f};
    ab_split(w0, w1, gh[s], gl[s]);
  }
#pragma unroll
  for (int it = 0; it < NT / 2; ++it) {
    const int ch = t + 256 * it, j = ch >> 3, c8 = (ch & 7) * 8;
    const bool jv = j < L;
    *reinterpret_cast<u32x4*>(Ks + j * AB_KP + c8) = jv ? kv[it] : u32x4{0u, 0u, 0u, 0u};
    *reinterpret_cast<u32x4*>(Vs + j * AB_KP + c8) = jv ? vv[it] : u32x4{0u, 0u, 0u, 0u};
  }
  tbs[t] = tb_a;
  tbs[t + 256] = tb_b;
  // dO rounded to bf16 for the cols kernel's dV (scratch plane 3, [B*H][KP][64])
  if (i < KP) {
    bf16_t* od = scr + 3 * (long)nbh * KP * KP + ((long)bh * KP + i) * 64 + fk;
    *reinterpret_cast<bf16x8*>(od) = oh[0];
    *reinterpret_cast<bf16x8*>(od + 32) = oh[1];
  }
  // gate (TF:167-177): z^T[n][i] = gate_w[n] . x_h[i]; pa = sum_{n<4} (z + b), pb = sum_{4<=n<8} (z + b)
  f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    z = mma16(gh[s], xb[s].v, z);
    z = mma16(gl[s], xb[s].v, z);
  }
  float zs = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) zs += z[r] + gate_b[(4 * fq + r) & 7];
  const float ga = sigmoidf_(__shfl(zs, fr)), gb = sigmoidf_(__shfl(zs, 16 + fr));
  const float gc = gate_c[h];
  const float gate = ga * (gb * gc - 1.f) + 2.f;
  __syncthreads();

  // S^T = K Q^T (exact), dP^T = V dO^T (split dO): key rows 16 tt + 4 fq + r in the registers
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
    s[tt] = mma16(k1.v, qb[1].v, mma16(k0.v, qb[0].v, zz));
    f32x4 d = mma16(v0.v, oh[0], zz);
    d = mma16(v0.v, ol[0], d);
    d = mma16(v1.v, oh[1], d);
    dp[tt] = mma16(v1.v, ol[1], d);
  }
  const int tmax = 2 * L - 2;
  const int tb0 = L - 1 - i + 4 * fq;  // tbl index of key 4 fq (+ 16 tt + r)
  float mx = -INFINITY;
#pragma unroll
  for (int tt = 0; tt < NT; ++tt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * tt + 4 * fq + r;
      const float v = j < L ? s[tt][r] * scale + gate * tbs[min(max(tb0 + 16 * tt + r, 0), tmax)] : -INFINITY;
      s[tt][r] = v;
      mx = fmaxf(mx, v);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 16));
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  float sum = 0.f;
#pragma unroll
  for (int tt = 0; tt < NT; ++tt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[tt][r] = __expf(s[tt][r] - mx);
      sum += s[tt][r];
    }
  sum += __shfl_xor(sum, 16);
  sum += __shfl_xor(sum, 32);
  const float inv = 1.f / sum;
  // train mode: attention-probability dropout of the forward (wavlm_attn_kernel, paired mask index
  // ((b*H+h)*L + i)*LE + j, LE = L rounded up to even):
  // O = (P o M) V, so dP = (dO V^T) o M and the cols kernel's dV reads P o M; dS keeps the undropped P
  const unsigned long long dseed = mer_site_seed(seed_ptr, site);
  const long mrow = (((long)b * H + h) * L + (i < L ? i : L - 1)) * (long)(L + (L & 1));
  auto keep = [&](int j) -> float { return dropout_scale_pair(dseed, (uint64_t)(mrow + j), drop_p); };
  float Dr = 0.f;
#pragma unroll
  for (int tt = 0; tt < NT; ++tt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[tt][r] *= inv;
      if (drop_p > 0.f) dp[tt][r] *= keep(16 * tt + 4 * fq + r);
      Dr += s[tt][r] * dp[tt][r];
    }
  Dr += __shfl_xor(Dr, 16);
  Dr += __shfl_xor(Dr, 32);
  // dS (0 for keys past L: p = 0, dp = 0), dgate, scratch rows (zero for query rows past L)
  const bool iv = i < L;
  const long so = ((long)bh * KP + i) * KP + 4 * fq;
  const long plane = (long)nbh * KP * KP;
  float dg = 0.f;
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    float hv[4], lv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float ds = s[tt][r] * (dp[tt][r] - Dr);
      dg += ds * tbs[min(max(tb0 + 16 * tt + r, 0), tmax)];
      dp[tt][r] = ds;
      const float hi = __builtin_bit_cast(float, (uint32_t)f2bf(ds) << 16);
      hv[r] = iv ? hi : 0.f;
      lv[r] = iv ? ds - hi : 0.f;
    }
    if (i < KP) {
      float pm[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) pm[r] = drop_p > 0.f ? s[tt][r] * keep(16 * tt + 4 * fq + r) : s[tt][r];
      const u32x2 pv = iv ? u32x2{pack2(pm[0], pm[1]), pack2(pm[2], pm[3])} : u32x2{0u, 0u};
      *reinterpret_cast<u32x2*>(scr + so + 16 * tt) = pv;
      *reinterpret_cast<u32x2*>(scr + plane + so + 16 * tt) = u32x2{pack2(hv[0], hv[1]), pack2(hv[2], hv[3])};
      *reinterpret_cast<u32x2*>(scr + 2 * plane + so + 16 * tt) = u32x2{pack2(lv[0], lv[1]), pack2(lv[2], lv[3])};
    }
  }
  dg += __shfl_xor(dg, 16);
  dg += __shfl_xor(dg, 32);

  // dQ^T = K^T dS^T: k step ks = key tiles 2ks (elements 0..3) and 2ks + 1 (elements 4..7), split dS; the K^T
  // fragment reads the same keys: rows 32 ks + 4 fq + q (+ 16), columns 16 c + 4 p
  f32x4 dq[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) dq[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int tq = fr >> 2, tp = fr & 3;
#pragma unroll
  for (int ks = 0; ks < NT / 2; ++ks) {
    bf16x8 ah, al;
    ab_split8(f32x8{dp[2 * ks][0], dp[2 * ks][1], dp[2 * ks][2], dp[2 * ks][3], dp[2 * ks + 1][0],
                    dp[2 * ks + 1][1], dp[2 * ks + 1][2], dp[2 * ks + 1][3]},
              ah, al);
    const bf16_t* kp = Ks + (32 * ks + 4 * fq + tq) * AB_KP + 4 * tp;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bf16x8 kt = tr_frag(kp + 16 * c, kp + 16 * AB_KP + 16 * c);
      dq[c] = mma16(kt, ah, dq[c]);
      dq[c] = mma16(kt, al, dq[c]);
    }
  }
  if (iv) {
    bf16_t* o = dqkv + (long)(b * L + i) * lddq + h * 64 + 4 * fq;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      *reinterpret_cast<u32x2*>(o + 16 * c) =
          u32x2{pack2(dq[c][0] * scale, dq[c][1] * scale), pack2(dq[c][2] * scale, dq[c][3] * scale)};
  }

  // gate backward: gate = ga (gb c - 1) + 2, pa / pb sums of 4 projections each (query row i on lane l & 15)
  const float g = iv ? dg : 0.f;
  const float dpa = g * (gb * gc - 1.f) * ga * (1.f - ga);
  const float dpb = g * ga * gc * gb * (1.f - gb);
  // lane = d: dW[n][d] += dp{a,b}(i) x[i][d] over the wave's 16 rows, dx_gate = dpa wsa + dpb wsb
  float wa = 0.f, wb = 0.f;
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) {
    const float a = __shfl(dpa, rr), c = __shfl(dpb, rr);
    wa += a * bf2f(xr[rr]);
    wb += c * bf2f(xr[rr]);
    if (dxg && i0 + rr < L) dxg[(long)(b * L + i0 + rr) * lddxg + h * 64 + lane] = a * wsa + c * wsb;
  }
  // row sums over the wave's 16 rows (lanes 0..15 hold one copy each)
  const float gal = wave_sum(fq == 0 ? dpa : 0.f), gbl = wave_sum(fq == 0 ? dpb : 0.f);
  const float gcl = wave_sum(fq == 0 ? g * ga * gb : 0.f);
  __syncthreads();  // every wave is past dP: the V image becomes the block reduction buffer
  float* red = reinterpret_cast<float*>(Vs);  // [4][GATE_PART + 1]
  constexpr int RP = GATE_PART + 1;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[w * RP + r * 64 + lane] = wa;
    red[w * RP + (r + 4) * 64 + lane] = wb;
  }
  if (lane < 8) red[w * RP + 512 + lane] = lane < 4 ? gal : gbl;
  if (lane == 0) red[w * RP + GATE_PART] = gcl;
  __syncthreads();
  float* pr = gpart + ((long)bh * nrb + rb) * (GATE_PART + H);
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

template <int NT>
struct ColsLds {
  static constexpr int KP = 16 * NT;
  static constexpr int qs = 0;                          // Q [KP][AB_KP] bf16
  static constexpr int os = qs + KP * AB_KP * 2;        // dO (bf16) [KP][AB_KP]
  static constexpr int ps = os + KP * AB_KP * 2;        // P, dS hi, dS lo strips [3][KP][AB_SP] bf16
  static constexpr int bytes = ps + 3 * KP * AB_SP * 2;
};

// Cols kernel: block = 32 keys of one (b, h); wave w = (key half w & 1, dim half w >> 1).
//   dK^T = scale Q^T dS (split dS), dV^T = dO^T P (bf16 dO, P).  Q, dO and the block's P / dS column strips are
// staged row-major (query rows); every fragment (k = query row) is a transposed LDS read.  One-dimensional grid,
// XCD-aware (xcd_tile): block -> (key block, b*h).
template <int NT>
__global__ __launch_bounds__(256) void wavlm_attn_bwd_cols_kernel(int L, int H, const bf16_t* __restrict__ qkv,
                                                                  long ldqkv, int nbh, const bf16_t* __restrict__ scr,
                                                                  float scale, bf16_t* __restrict__ dqkv, long lddq) {
  typedef ColsLds<NT> Ly;
  constexpr int KP = Ly::KP;
  extern __shared__ __attribute__((aligned(16))) unsigned char ab_smem[];
  bf16_t* Qs = reinterpret_cast<bf16_t*>(ab_smem + Ly::qs);
  bf16_t* Os = reinterpret_cast<bf16_t*>(ab_smem + Ly::os);
  bf16_t* Ss = reinterpret_cast<bf16_t*>(ab_smem + Ly::ps);
  constexpr int NKB = KP / AB_COLS;
  int kb, bh;  // the key blocks of one (b, h) share its Q / dO: keep them on one XCD
  xcd_tile(blockIdx.x, NKB, NKB * nbh, kb, bh);
  const int b = bh / H, h = bh - b * H;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, fr = lane & 15, fq = lane >> 4;
  const int D = H * 64;
  const int j0 = kb * AB_COLS;
  const long plane = (long)nbh * KP * KP;
  // all staging loads in flight before the first LDS store.  Query rows past L: any finite values (their P / dS
  // rows are zero).  Q from qkv, dO as the rows kernel's bf16 copy, 4 16-byte chunks per strip row and plane.
  constexpr int NS = (3 * KP * 4 + 255) / 256;
  u32x4 qv[NT / 2], ov[NT / 2], sv[NS];
#pragma unroll
  for (int it = 0; it < NT / 2; ++it) {
    const int ch = t + 256 * it, i = ch >> 3, c8 = (ch & 7) * 8;
    qv[it] = *reinterpret_cast<const u32x4*>(qkv + (long)(b * L + (i < L ? i : L - 1)) * ldqkv + h * 64 + c8);
    ov[it] = *reinterpret_cast<const u32x4*>(scr + 3 * plane + ((long)bh * KP + i) * 64 + c8);
  }
#pragma unroll
  for (int it = 0; it < NS; ++it) {
    const int ch = min(t + 256 * it, 3 * KP * 4 - 1);
    const int pl = ch / (KP * 4), rem = ch - pl * KP * 4, i = rem >> 2, c8 = (rem & 3) * 8;
    sv[it] = *reinterpret_cast<const u32x4*>(scr + pl * plane + ((long)bh * KP + i) * KP + j0 + c8);
  }
#pragma unroll
  for (int it = 0; it < NT / 2; ++it) {
    const int ch = t + 256 * it, i = ch >> 3, c8 = (ch & 7) * 8;
    *reinterpret_cast<u32x4*>(Qs + i * AB_KP + c8) = qv[it];
    *reinterpret_cast<u32x4*>(Os + i * AB_KP + c8) = ov[it];
  }
#pragma unroll
  for (int it = 0; it < NS; ++it) {
    const int ch = t + 256 * it;
    const int pl = ch / (KP * 4), rem = ch - pl * KP * 4, i = rem >> 2, c8 = (rem & 3) * 8;
    if (ch < 3 * KP * 4) *reinterpret_cast<u32x4*>(Ss + (pl * KP + i) * AB_SP + c8) = sv[it];
  }
  __syncthreads();
  const int kt = w & 1, dd = w >> 1, tq = fr >> 2, tp = fr & 3;
  f32x4 dk[2], dv[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) dk[c] = dv[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < NT / 2; ++ks) {
    const int r0 = 32 * ks + 8 * fq + tq;  // rows r0 and r0 + 4 feed elements 0..3 / 4..7
    const bf16_t* sp = Ss + r0 * AB_SP + 16 * kt + 4 * tp;
    const bf16x8 pf = tr_frag(sp, sp + 4 * AB_SP);
    const bf16x8 dh = tr_frag(sp + KP * AB_SP, sp + (KP + 4) * AB_SP);
    const bf16x8 dl = tr_frag(sp + 2 * KP * AB_SP, sp + (2 * KP + 4) * AB_SP);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int n0 = 32 * dd + 16 * c + 4 * tp;
      const bf16x8 qf = tr_frag(Qs + r0 * AB_KP + n0, Qs + (r0 + 4) * AB_KP + n0);
      const bf16x8 of = tr_frag(Os + r0 * AB_KP + n0, Os + (r0 + 4) * AB_KP + n0);
      dk[c] = mma16(qf, dh, dk[c]);
      dk[c] = mma16(qf, dl, dk[c]);
      dv[c] = mma16(of, pf, dv[c]);
    }
  }
  // C: rows d = 32 dd + 16 c + 4 fq + r, column key j0 + 16 kt + (l & 15)
  const int j = j0 + 16 * kt + fr;
  if (j < L) {
    bf16_t* o = dqkv + (long)(b * L + j) * lddq + h * 64 + 32 * dd + 4 * fq;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      *reinterpret_cast<u32x2*>(o + D + 16 * c) =
          u32x2{pack2(dk[c][0] * scale, dk[c][1] * scale), pack2(dk[c][2] * scale, dk[c][3] * scale)};
      *reinterpret_cast<u32x2*>(o + 2 * D + 16 * c) = u32x2{pack2(dv[c][0], dv[c][1]), pack2(dv[c][2], dv[c][3])};
    }
  }
}

template <int NT>
int wavlm_attention_bwd_launch(int B, int L, int H, const bf16_t* qkv, long ldqkv, const bf16_t* x, long ldx,
                               const float* dout, long ldo, const float* gate_w, const float* gate_b,
                               const float* gate_c, const float* tbl, float scale, bf16_t* scr, bf16_t* dqkv,
                               long lddq, float* dxg, long lddxg, float* gpart, float drop_p,
                               const unsigned long long* seed, unsigned long long site, hipStream_t st) {
  constexpr int rb = RowsLds<NT>::bytes, cb = ColsLds<NT>::bytes;
  static_assert(rb <= 160 * 1024 && cb <= 160 * 1024, "LDS");
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&wavlm_attn_bwd_rows_kernel<NT>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, rb) != hipSuccess ||
      hipFuncSetAttribute(reinterpret_cast<const void*>(&wavlm_attn_bwd_cols_kernel<NT>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, cb) != hipSuccess)
    return (int)hipErrorInvalidConfiguration;
  hipLaunchKernelGGL(wavlm_attn_bwd_rows_kernel<NT>, dim3((L + AB_ROWS - 1) / AB_ROWS * B * H), dim3(256), rb, st, L,
                     H, qkv, ldqkv, x, ldx, dout, ldo, gate_w, gate_b, gate_c, tbl, scale, B * H, scr, dqkv, lddq, dxg,
                     lddxg, gpart, drop_p, seed, site);
  hipLaunchKernelGGL(wavlm_attn_bwd_cols_kernel<NT>, dim3(16 * NT / AB_COLS * B * H), dim3(256), cb, st, L, H, qkv,
                     ldqkv, B * H, scr, scale, dqkv, lddq);
  return (int)hipGetLastError();
}

int ab_tiles(int L) {  // 16-key tiles the kernels are built for: 4 / 8 / 10 / 12 (L <= 64 / 128 / 160 / 192)
  const int nt = (L + 15) / 16;
  return nt <= 4 ? 4 : nt <= 8 ? 8 : nt <= 10 ? 10 : 12;
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

namespace {
// y = x * dropout_scale_pair(seed(site), row * cols + col, p): the mask of one dropout call site (the same index as
// the GEMM-epilogue dropout of mer_gemm_bf16_tr), regenerated; 8 columns per thread
template <typename TI>
__global__ __launch_bounds__(256) void dropout_rows_kernel(int rows, int cols, const TI* __restrict__ x, long ldx,
                                                           float* __restrict__ y32, long ldy32, bf16_t* __restrict__ y16,
                                                           long ldy16, float p, const unsigned long long* seed_ptr,
                                                           unsigned long long site) {
  const unsigned long long seed = mer_site_seed(seed_ptr, site);
  const int c8 = cols / 8;
  const long n = (long)rows * c8;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int r = (int)(e / c8), c0 = (int)(e - (long)r * c8) * 8;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = ldf<TI>(x, (long)r * ldx + c0 + k);
    dropout_pairs<8>(v, seed, (uint64_t)((long)r * cols + c0), p);  // cols % 8 == 0: the indices start even
    if (y32) {
      float* o = y32 + (long)r * ldy32 + c0;
      *reinterpret_cast<f32x4*>(o) = f32x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(o + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
    if (y16) {
      *reinterpret_cast<u32x4*>(y16 + (long)r * ldy16 + c0) =
          u32x4{pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7])};
    }
  }
}
}  // namespace

MER_API int mer_dropout_rows(int rows, int cols, const void* x, int x_dtype, long ldx, float* y32, long ldy32,
                             void* y16, long ldy16, float p, const unsigned long long* seed, unsigned long long site,
                             void* stream) {
  if (rows <= 0 || cols <= 0) return 0;
  if (cols % 8 || ldx % 8 || (y32 && ldy32 % 4) || (y16 && ldy16 % 8) || p < 0.f || p >= 1.f || (p > 0.f && !seed))
    return (int)hipErrorInvalidValue;
  const long n = (long)rows * (cols / 8);
  const unsigned grid = (unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  if (x_dtype == MER_BF16)
    hipLaunchKernelGGL(dropout_rows_kernel<bf16_t>, dim3(grid), dim3(256), 0, (hipStream_t)stream, rows, cols,
                       (const bf16_t*)x, ldx, y32, ldy32, (bf16_t*)y16, ldy16, p, seed, site);
  else
    hipLaunchKernelGGL(dropout_rows_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, rows, cols,
                       (const float*)x, ldx, y32, ldy32, (bf16_t*)y16, ldy16, p, seed, site);
  MER_LAUNCH_CHECK();
}

MER_API int mer_wavlm_attention_bwd_kp(int L) { return (L <= 0 || L > AB_LMAX) ? 0 : 16 * ab_tiles(L); }

MER_API int mer_wavlm_attention_bwd(int B, int L, int H, const void* qkv, long ldqkv, const void* x, long ldx,
                                    const void* dout, long ldo, const float* gate_w, const float* gate_b,
                                    const float* gate_const, const float* tbl, float scale, void* scratch,
                                    void* dqkv, long lddq, float* dx_gate, long lddxg, float* gate_part,
                                    void* stream) {
  return mer_wavlm_attention_bwd_tr(B, L, H, qkv, ldqkv, x, ldx, dout, ldo, gate_w, gate_b, gate_const, tbl, scale,
                                    scratch, dqkv, lddq, dx_gate, lddxg, gate_part, 0.f, nullptr, 0ull, stream);
}

MER_API int mer_wavlm_attention_bwd_tr(int B, int L, int H, const void* qkv, long ldqkv, const void* x, long ldx,
                                       const void* dout, long ldo, const float* gate_w, const float* gate_b,
                                       const float* gate_const, const float* tbl, float scale, void* scratch,
                                       void* dqkv, long lddq, float* dx_gate, long lddxg, float* gate_part,
                                       float drop_p, const unsigned long long* seed, unsigned long long site,
                                       void* stream) {
  if (L <= 0 || L > AB_LMAX || ldqkv % 8 || ldx % 8 || ldo % 4 || lddq % 4 || B <= 0 || H <= 0)
    return (int)hipErrorInvalidValue;
  if (drop_p < 0.f || drop_p >= 1.f || (drop_p > 0.f && !seed)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
#define MER_AB_LAUNCH(NT)                                                                                             \
  wavlm_attention_bwd_launch<NT>(B, L, H, (const bf16_t*)qkv, ldqkv, (const bf16_t*)x, ldx, (const float*)dout, ldo, \
                                 gate_w, gate_b, gate_const, tbl, scale, (bf16_t*)scratch, (bf16_t*)dqkv, lddq,       \
                                 dx_gate, lddxg, gate_part, drop_p, seed, site, st)
  const int nt = ab_tiles(L);
  const int rc = nt == 4 ? MER_AB_LAUNCH(4) : nt == 8 ? MER_AB_LAUNCH(8) : nt == 10 ? MER_AB_LAUNCH(10) : MER_AB_LAUNCH(12);
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
