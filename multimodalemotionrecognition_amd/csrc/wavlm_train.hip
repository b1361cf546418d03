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

// make this wave's LDS writes visible to all of its lanes (per-wave row buffers)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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
// Rows kernel: one wave per query row (4 rows per wave, 16 per block); K, V of the (b,h) staged in LDS
// (bf16, 66-element row pitch: odd dword stride, conflict-free per-lane row reads); writes P and dS rows
// (fp32 scratch [B*H][L][L]) for the cols kernel, dq into dqkv, dx_gate, per-block gate-grad partials.
constexpr int AB_LMAX = 192;  // 3 key columns per lane; 2 blocks per CU in LDS (3 s clips: L = 149)
constexpr int AB_PITCH = 68;  // bf16 row pitch: 8-byte aligned rows, 17j mod 32 banks -> conflict-free b64 reads
constexpr int AB_ROWS = 32;  // query rows per block (8 per wave): K/V staged once per 32 rows
constexpr int GATE_PART = 8 * 64 + 8;  // + H (gate const) per partial row

__global__ __launch_bounds__(256) void wavlm_attn_bwd_rows_kernel(
    int L, int H, const bf16_t* __restrict__ qkv, long ldqkv, const bf16_t* __restrict__ x, long ldx,
    const float* __restrict__ dout, long ldo, const float* __restrict__ gate_w, const float* __restrict__ gate_b,
    const float* __restrict__ gate_c, const float* __restrict__ tbl, float scale, float* __restrict__ Pbuf,
    float* __restrict__ dSbuf, bf16_t* __restrict__ dqkv, long lddq, float* __restrict__ dxg, long lddxg,
    float* __restrict__ gpart) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[AB_LMAX * AB_PITCH];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[AB_LMAX * AB_PITCH];
  __shared__ __attribute__((aligned(16))) float qrow[4][64];
  __shared__ __attribute__((aligned(16))) float dorow[4][64];
  __shared__ __attribute__((aligned(16))) float dsrow[4][AB_LMAX];
  __shared__ float gw[8][64];
  __shared__ float red[4][GATE_PART + 1];
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int D = H * 64;
  for (int i = t; i < 8 * 64; i += 256) gw[i >> 6][i & 63] = gate_w[i];
  // stage K and V rows of this (b, h): 8 bf16 per 16-byte chunk, 8 chunks per row
  for (int ch = t; ch < L * 8; ch += 256) {
    const int j = ch >> 3, c8 = (ch & 7) * 8;
    const long g = (long)(b * L + j) * ldqkv + h * 64 + c8;
    const uint4 kv = *reinterpret_cast<const uint4*>(qkv + g + D);
    const uint4 vv = *reinterpret_cast<const uint4*>(qkv + g + 2 * D);
    uint32_t* kd = reinterpret_cast<uint32_t*>(Ks + j * AB_PITCH + c8);
    uint32_t* vd = reinterpret_cast<uint32_t*>(Vs + j * AB_PITCH + c8);
    kd[0] = kv.x; kd[1] = kv.y; kd[2] = kv.z; kd[3] = kv.w;
    vd[0] = vv.x; vd[1] = vv.y; vd[2] = vv.z; vd[3] = vv.w;
  }
  __syncthreads();
  const float* th = tbl + (long)h * (2 * L - 1);
  float wsa = 0.f, wsb = 0.f;  // column sums of the gate weight halves (d(pa)/dx, d(pb)/dx)
  for (int r = 0; r < 4; ++r) { wsa += gw[r][lane]; wsb += gw[r + 4][lane]; }
  float gacc[8], gbacc[8], gcacc = 0.f;
  for (int r = 0; r < 8; ++r) gacc[r] = gbacc[r] = 0.f;
  const float gc = gate_c[h];
  constexpr int NJ = AB_LMAX / 64;
  for (int rr = w; rr < AB_ROWS; rr += 4) {
    const int i = blockIdx.x * AB_ROWS + rr;
    if (i >= L) break;
    const long row = (long)(b * L + i);
    const float qd = bf2f(qkv[row * ldqkv + h * 64 + lane]) * scale;
    const float dod = dout[row * ldo + h * 64 + lane];
    const float xd = bf2f(x[row * ldx + h * 64 + lane]);
    qrow[w][lane] = qd;
    dorow[w][lane] = dod;
    // gate (TF:167-177): 8 projections, pair sums of 4
    float pa = 0.f, pb = 0.f;
    for (int r = 0; r < 4; ++r) pa += wave_sum(xd * gw[r][lane]) + gate_b[r];
    for (int r = 4; r < 8; ++r) pb += wave_sum(xd * gw[r][lane]) + gate_b[r];
    const float ga = sigmoidf_(pa), gb = sigmoidf_(pb);
    const float gate = ga * (gb * gc - 1.f) + 2.f;
    wave_lds_sync();
    float s[NJ], dp[NJ];
    float mx = -INFINITY;
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      const int j = jj * 64 + lane;
      s[jj] = -INFINITY;
      dp[jj] = 0.f;
      if (j < L) {
        // 4 dims per step: one b64 K read, one b64 V read (per lane), one broadcast b128 read each of q and dO
        const uint2* kr = reinterpret_cast<const uint2*>(Ks + j * AB_PITCH);
        const uint2* vr = reinterpret_cast<const uint2*>(Vs + j * AB_PITCH);
        const f32x4* q4 = reinterpret_cast<const f32x4*>(qrow[w]);
        const f32x4* o4 = reinterpret_cast<const f32x4*>(dorow[w]);
        // packed fp32 FMAs (v_pk_fma_f32): two dims per instruction
        f32x2 a = {0.f, 0.f}, c = {0.f, 0.f};
#pragma unroll 4
        for (int e = 0; e < 16; ++e) {
          const uint2 kk = kr[e], vv = vr[e];
          const f32x4 qq = q4[e], oo = o4[e];
          const f32x2 k01 = {__uint_as_float(kk.x << 16), __uint_as_float(kk.x & 0xffff0000u)};
          const f32x2 k23 = {__uint_as_float(kk.y << 16), __uint_as_float(kk.y & 0xffff0000u)};
          const f32x2 v01 = {__uint_as_float(vv.x << 16), __uint_as_float(vv.x & 0xffff0000u)};
          const f32x2 v23 = {__uint_as_float(vv.y << 16), __uint_as_float(vv.y & 0xffff0000u)};
          a = __builtin_elementwise_fma(f32x2{qq[0], qq[1]}, k01, a);
          a = __builtin_elementwise_fma(f32x2{qq[2], qq[3]}, k23, a);
          c = __builtin_elementwise_fma(f32x2{oo[0], oo[1]}, v01, c);
          c = __builtin_elementwise_fma(f32x2{oo[2], oo[3]}, v23, c);
        }
        s[jj] = a[0] + a[1] + gate * th[j - i + L - 1];
        dp[jj] = c[0] + c[1];
      }
      mx = fmaxf(mx, s[jj]);
    }
    mx = wave_max(mx);
    float sum = 0.f;
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      s[jj] = (jj * 64 + lane < L) ? __expf(s[jj] - mx) : 0.f;
      sum += s[jj];
    }
    const float inv = 1.f / wave_sum(sum);
    float pd = 0.f;
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) { s[jj] *= inv; pd += s[jj] * dp[jj]; }
    const float Dsum = wave_sum(pd);
    float dgl = 0.f;
    float* prow = Pbuf + ((long)bh * L + i) * L;
    float* drow = dSbuf + ((long)bh * L + i) * L;
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      const int j = jj * 64 + lane;
      if (j < L) {
        const float ds = s[jj] * (dp[jj] - Dsum);
        dgl += ds * th[j - i + L - 1];
        prow[j] = s[jj];
        drow[j] = ds;
        dsrow[w][j] = ds;
      }
    }
    const float dgate = wave_sum(dgl);
    wave_lds_sync();
    // dq_i[d] = scale * sum_j ds_ij k_j[d]   (lane = d)
    float q0 = 0.f, q1 = 0.f;
    int j = 0;
    for (; j + 4 <= L; j += 4) {
      const f32x4 d4 = *reinterpret_cast<const f32x4*>(&dsrow[w][j]);
      q0 += d4[0] * bf2f(Ks[j * AB_PITCH + lane]);
      q1 += d4[1] * bf2f(Ks[(j + 1) * AB_PITCH + lane]);
      q0 += d4[2] * bf2f(Ks[(j + 2) * AB_PITCH + lane]);
      q1 += d4[3] * bf2f(Ks[(j + 3) * AB_PITCH + lane]);
    }
    for (; j < L; ++j) q0 += dsrow[w][j] * bf2f(Ks[j * AB_PITCH + lane]);
    dqkv[row * lddq + h * 64 + lane] = f2bf((q0 + q1) * scale);
    // gate backward: gate = ga (gb c - 1) + 2
    const float dpa = dgate * (gb * gc - 1.f) * ga * (1.f - ga);
    const float dpb = dgate * ga * gc * gb * (1.f - gb);
    gcacc += dgate * ga * gb;
    for (int r = 0; r < 4; ++r) { gacc[r] += dpa * xd; gacc[r + 4] += dpb * xd; }
    gbacc[0] += dpa;
    gbacc[4] += dpb;
    if (dxg) dxg[row * lddxg + h * 64 + lane] = dpa * wsa + dpb * wsb;
    wave_lds_sync();
  }
  // per-block gate-gradient partial row: [8][64] weight, [8] bias, [H] const (this head only)
  for (int r = 0; r < 8; ++r) red[w][r * 64 + lane] = gacc[r];
  if (lane == 0) {
    for (int r = 0; r < 8; ++r) red[w][512 + r] = gbacc[r < 4 ? 0 : 4];
    red[w][GATE_PART] = gcacc;
  }
  __syncthreads();
  float* pr = gpart + ((long)bh * gridDim.x + blockIdx.x) * (GATE_PART + H);
  for (int k = t; k < GATE_PART + H; k += 256) {
    float v;
    if (k < GATE_PART) v = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
    else v = (k - GATE_PART == h) ? ((red[0][GATE_PART] + red[1][GATE_PART]) + red[2][GATE_PART]) + red[3][GATE_PART] : 0.f;
    pr[k] = v;
  }
}

// Cols kernel: one wave per 4 key columns j (16 per block): dk_j = scale sum_i ds_ij q_i, dv_j = sum_i p_ij do_i
// (lane = d).  Q and dO rows of the (b, h) are staged in LDS (bf16), the block's P / dS column strips [L][16]
// in fp32.
__global__ __launch_bounds__(256) void wavlm_attn_bwd_cols_kernel(int L, int H, const bf16_t* __restrict__ qkv,
                                                                  long ldqkv, const float* __restrict__ dout, long ldo,
                                                                  const float* __restrict__ Pbuf,
                                                                  const float* __restrict__ dSbuf, float scale,
                                                                  bf16_t* __restrict__ dqkv, long lddq) {
  __shared__ __attribute__((aligned(16))) bf16_t Qs[AB_LMAX * AB_PITCH];
  __shared__ __attribute__((aligned(16))) bf16_t Os[AB_LMAX * AB_PITCH];
  __shared__ float Pc[AB_LMAX][17], Dc[AB_LMAX][17];  // 17: keeps the block at 2 per CU in LDS
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int D = H * 64;
  const int j0 = blockIdx.x * 16;
  for (int ch = t; ch < L * 8; ch += 256) {
    const int i = ch >> 3, c8 = (ch & 7) * 8;
    const long row = (long)(b * L + i);
    const uint4 qv = *reinterpret_cast<const uint4*>(qkv + row * ldqkv + h * 64 + c8);
    const f32x4 o0 = *reinterpret_cast<const f32x4*>(dout + row * ldo + h * 64 + c8);
    const f32x4 o1 = *reinterpret_cast<const f32x4*>(dout + row * ldo + h * 64 + c8 + 4);
    uint32_t* qd = reinterpret_cast<uint32_t*>(Qs + i * AB_PITCH + c8);
    uint32_t* od = reinterpret_cast<uint32_t*>(Os + i * AB_PITCH + c8);
    qd[0] = qv.x; qd[1] = qv.y; qd[2] = qv.z; qd[3] = qv.w;
    // dv = sum_i p_ij do_i has no cancellation: dO is staged as bf16 here (it stays fp32 in the rows
    // kernel, where dp_ij - sum_j p_ij dp_ij cancels)
    od[0] = (uint32_t)f2bf(o0[0]) | ((uint32_t)f2bf(o0[1]) << 16);
    od[1] = (uint32_t)f2bf(o0[2]) | ((uint32_t)f2bf(o0[3]) << 16);
    od[2] = (uint32_t)f2bf(o1[0]) | ((uint32_t)f2bf(o1[1]) << 16);
    od[3] = (uint32_t)f2bf(o1[2]) | ((uint32_t)f2bf(o1[3]) << 16);
  }
  for (int e = t; e < L * 16; e += 256) {
    const int i = e >> 4, jc = e & 15, j = j0 + jc;
    const long o = ((long)bh * L + i) * L + j;
    Pc[i][jc] = j < L ? Pbuf[o] : 0.f;
    Dc[i][jc] = j < L ? dSbuf[o] : 0.f;
  }
  __syncthreads();
  float dk[4] = {0.f, 0.f, 0.f, 0.f}, dv[4] = {0.f, 0.f, 0.f, 0.f};
  const int jc0 = w * 4;
  for (int i = 0; i < L; ++i) {
    const float qd = bf2f(Qs[i * AB_PITCH + lane]), od = bf2f(Os[i * AB_PITCH + lane]);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      dk[c] += Dc[i][jc0 + c] * qd;
      dv[c] += Pc[i][jc0 + c] * od;
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int j = j0 + jc0 + c;
    if (j < L) {
      const long row = (long)(b * L + j);
      dqkv[row * lddq + D + h * 64 + lane] = f2bf(dk[c] * scale);
      dqkv[row * lddq + 2 * D + h * 64 + lane] = f2bf(dv[c]);
    }
  }
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
  if (L <= 0 || L > AB_LMAX || ldqkv % 8 || ldo % 4 || B <= 0 || H <= 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int nrb = (L + AB_ROWS - 1) / AB_ROWS;
  hipLaunchKernelGGL(wavlm_attn_bwd_rows_kernel, dim3(nrb, B * H), dim3(256), 0, st, L, H, (const bf16_t*)qkv, ldqkv,
                     (const bf16_t*)x, ldx, (const float*)dout, ldo, gate_w, gate_b, gate_const, tbl, scale, P, dS,
                     (bf16_t*)dqkv, lddq, dx_gate, lddxg, gate_part);
  hipLaunchKernelGGL(wavlm_attn_bwd_cols_kernel, dim3((L + 15) / 16, B * H), dim3(256), 0, st, L, H,
                     (const bf16_t*)qkv, ldqkv, (const float*)dout, ldo, P, dS, scale, (bf16_t*)dqkv, lddq);
  MER_LAUNCH_CHECK();
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
