/*
 * mer.h -- C-ABI of the MI355X-native (gfx950 / CDNA4) multimodal-emotion-recognition hot path.
 *
 * Drop-in boundary for the reference's fusion train/inference path
 * (Wionerlol/MultimodalEmotionRecognition: src/models/{fusion,video,wavlm_audio,temporal}.py,
 * src/train.py:200-228, src/optimized_runtime.py:99-108).  The reference is pure Python over
 * torch / torchvision / transformers; every entry point below replaces the device math of one
 * of its call sites, cited per function.  The Python host layer
 * (multimodalemotionrecognition_amd/ *.py) binds these through ctypes.
 *
 * Conventions (every function):
 *   - returns 0 on success or a hipError_t value (e.g. 1 = hipErrorInvalidValue on bad shapes);
 *   - all tensor arguments are DEVICE pointers; the caller allocates every output/workspace;
 *   - `stream` is a hipStream_t passed as void*; work is enqueued asynchronously on it;
 *   - no internal allocation, no global mutable state; reentrant per stream;
 *   - element strides/leading dimensions are in ELEMENTS; dtype codes: 0 = fp32, 1 = bf16;
 *   - activation codes: 0 none, 1 ReLU, 2 exact-erf GELU.
 * Plain C types only: int = int32, long = int64, unsigned long long = uint64 (RNG seeds).
 * Dropout / drop-path RNG: `seed` points to the step's uint64 RNG base in DEVICE memory (NULL when p == 0),
 * `site` is a constant per call site; masks are hash(base, site, element) and are regenerated in backward.
 */
#ifndef MER_H_
#define MER_H_

/* BatchNorm batch statistics of a conv forward (mer_conv_fwd `stats`): float[MER_BN_STAT_ROWS(M)][C][2]
 * (sum, sum of squares), zeroed by the caller, M = N*Ho*Wo output pixels.  Each output row tile of the
 * conv stores its own row (a single writer per element: deterministic) -- the persistent halo kernels (layer1, stem)
 * instead store one row per workgroup, summed over its tiles in a fixed order -- unused rows stay zero, and the last
 * 64 rows are mer_bn_finalize's scratch.  The backward reductions use the same single-writer rows
 * (MER_BN_RED_ROWS, MER_BN_RED_WS_ROWS below), so the whole trunk step is free of fp32 atomics. */
#define MER_BN_STAT_PARTS 64
#define MER_BN_STAT_ROWS(M) (((M) + 63) / 64 + 64)
/* Backward BatchNorm reductions: per-row-tile rows of mer_conv_dgrad_bnr (+4 for the stride-2 parity classes,
 * +64 fold scratch) and the per-block rows of mer_bn_bwd_reduce (<= 512 blocks + 64 scratch). */
#define MER_BN_RED_ROWS(M) (((M) + 63) / 64 + 4 + 64)
#define MER_BN_RED_WS_ROWS 576

#ifdef __cplusplus
extern "C" {
#endif

/* ============================ fusion head (fp32) ============================ */

/* C[m,n] (+)= act(sum_k A(m,k) B(k,n) + bias[n]), batched over grid z.
 * A(m,k) = A[m*sam + k*sak] (+ batch*bsa), B(k,n) = B[k*sbk + n*sbn]; C row-major (ldc).
 * beta=1 accumulates into C.  splitk>1 (act must be 0, C initialised): each K slice writes its partial
 * into workspace [batch][splitk][M][N] (fp32) and the slices are added into C in slice order -- results
 * are run-to-run reproducible (no atomics).  workspace may be NULL when splitk == 1.
 * Replaces every nn.Linear of the head: fusion.py:269-274 (v_in_proj/a_in_proj/audio_seq_proj),
 * fusion.py:312-326 (xattn_mlp / xattn_gate / xattn_classifier), the MHA in/out projections
 * (TORCH:6576-6606) and their backward GEMMs (dX = dY W, dW = dY^T X). */
int mer_gemm_f32(int M, int N, int K, const void* A, int a_dtype, long sam, long sak, long bsa, const void* B,
                 int b_dtype, long sbk, long sbn, long bsb, float* C, long ldc, long bsc, const float* bias, int beta,
                 int act, int splitk, int batch, float* workspace, void* stream);

/* out[n] += sum_m X[m*ldx + n]  (bias gradients; out must be initialised).  Deterministic: per-block
 * partial rows in workspace (MER_COLSUM_WS_FLOATS(M, N) floats), folded in block order. */
#define MER_COLSUM_WS_FLOATS(M, N) ((long)(((M) + 15) / 16) * (N))
int mer_colsum_f32(int M, int N, const float* X, long ldx, float* out, float* workspace, void* stream);

/* Multi-head attention core of nn.MultiheadAttention (fusion.py:276-281,394,398 -> TORCH:6576-6606):
 * P = softmax(scale * Q_h K_h^T + bias[b]); O_h = dropout(P) V_h.  Rows: X + (b*L+i)*ld + h*dh.
 * bias [B,Lq,Lk] is the per-sample emotion-prior mask repeated over heads (fusion.py:351-354), or NULL.
 * P [B,H,Lq,Lk] receives the pre-dropout probabilities (saved for backward).  QK^T and PV on the exact-f32
 * MFMA (v_mfma_f32_16x16x4_f32).  Limits: dh % 4 == 0, dh <= 64, Lk <= 256 (hipErrorInvalidValue else). */
int mer_mha_fwd(int B, int H, int Lq, int Lk, int dh, const float* Q, long ldq, const float* K, long ldk,
                const float* V, long ldv, const float* bias, float* O, long ldo, float* P, float scale, float drop_p,
                const unsigned long long* seed, unsigned long long site, void* stream);

/* Backward of mer_mha_fwd: writes dQ, dK, dV (not accumulated) and dbias[b] = sum_h dS (if non-NULL).
 * One workgroup per (b, h), all four products on the f32 MFMA.  When dbias is requested, P is overwritten
 * with dS (the per-head scratch of the deterministic head sum).  Same limits as mer_mha_fwd, plus the
 * LDS image 4*(Lq+Lk)*dh + 2*Lq*Lk floats (padded) must fit in 160 KiB. */
int mer_mha_bwd(int B, int H, int Lq, int Lk, int dh, const float* Q, long ldq, const float* K, long ldk,
                const float* V, long ldv, float* P, const float* dO, long lddo, float* dQ, long lddq, float* dK,
                long lddk, float* dV, long lddv, float* dbias, float scale, float drop_p, const unsigned long long* seed, unsigned long long site,
                void* stream);

/* Host-side query (no launch): the LDS bytes mer_mha_bwd needs for (Lq, Lk, dh), written to *bytes. */
int mer_mha_bwd_lds_bytes(int Lq, int Lk, int dh, long* bytes);

/* y = LayerNorm(x + s_b * r) with StochasticDepth scale s_b regenerated from (seed, row/rows_per_sample)
 * (fusion.py:11-26, 284-285, 395, 399).  r may be NULL.  Saves sum/mean/rstd when non-NULL. */
int mer_add_ln_fwd(int rows, int d, int rows_per_sample, const float* x, const float* r, float dp_p,
                   const unsigned long long* seed, unsigned long long site, const float* gamma, const float* beta, float eps, float* y, float* sum_out,
                   float* mean_out, float* rstd_out, void* stream);

/* Backward of mer_add_ln_fwd: dx = dsum, dr = s_b*dsum (dr may be NULL); dgamma/dbeta accumulate (+=),
 * deterministically: per-16-row-block partials in workspace (MER_ADD_LN_WS_FLOATS(rows, d) floats). */
#define MER_ADD_LN_WS_FLOATS(rows, d) ((long)(((rows) + 15) / 16) * 2 * (d))
int mer_add_ln_bwd(int rows, int d, int rows_per_sample, const float* dy, const float* s, const float* mean,
                   const float* rstd, const float* gamma, float dp_p, const unsigned long long* seed, unsigned long long site, float* dx, float* dr,
                   float* dgamma, float* dbeta, float* workspace, void* stream);

/* TemporalPooler 'mean' (temporal.py:108-109): y[b*ldy + c] = mean_l x[b,l,c]; and its backward. */
int mer_mean_pool_fwd(int B, int L, int D, const float* x, float* y, long ldy, void* stream);
int mer_mean_pool_bwd(int B, int L, int D, const float* dy, long lddy, float* dx, int accumulate, void* stream);

/* ---- temporal pooling (TemporalPooler 'attn' / 'transformer', temporal.py:9-75), fp32 ---- */

/* y = dropout(gelu(z)) (exact erf GELU; temporal.py:18-19, the encoder layer's FFN) and its backward
 * dz = dy * mask * gelu'(z); row-strided; mask index = row * cols + col. */
int mer_gelu_dropout_fwd(int rows, int cols, const float* z, long ldz, float* y, long ldy, float p,
                         const unsigned long long* seed, unsigned long long site, void* stream);
int mer_gelu_dropout_bwd(int rows, int cols, const float* dy, long lddy, const float* z, long ldz, float* dz,
                         long lddz, float p, const unsigned long long* seed, unsigned long long site, void* stream);

/* y = x + dropout(r[row % r_period]) over contiguous rows (encoder residuals; r_period = L, p = 0 adds the
 * sinusoidal positional encoding, temporal.py:42-43).  y may alias x. */
int mer_add_dropout(int rows, int cols, const float* x, const float* r, int r_period, float p,
                    const unsigned long long* seed, unsigned long long site, float* y, void* stream);

/* Attention pooling (temporal.py:23-26): attn = softmax_L(scores [B,L]); y[b*ldy + c] = sum_l attn x[b,l,c];
 * backward: dx (+)= attn dy, dscores = attn (dy.x_l - sum attn dy.x).  L <= 4096. */
int mer_attn_pool_fwd(int B, int L, int D, const float* x, const float* scores, float* attn, float* y, long ldy,
                      void* stream);
int mer_attn_pool_bwd(int B, int L, int D, const float* x, const float* attn, const float* dy, long lddy, float* dx,
                      int accumulate, float* dscores, void* stream);

/* Softmax + dropout backward of head h for materialised attention (long self-attention whose fused kernel
 * image exceeds LDS): dS = P (dPp m - rowsum(P dPp m)), Pd = P m; P [B,H,Lq,Lk], dPp/dS/Pd [B,Lq,Lk]. */
int mer_softmax_dropout_bwd(int B, int H, int h, int Lq, int Lk, const float* P, const float* dPp, float* dS,
                            float* Pd, float p, const unsigned long long* seed, unsigned long long site, void* stream);
/* Its forward for head widths the fused mer_mha_fwd does not take (head_dim > 64, the encoders' transformer
 * pooling at 512 / 768 wide, temporal.py:46-75): S = Q_h K_h^T of head h [B,Lq,Lk] -> P[b,h] = softmax(scale*S)
 * (pre-dropout, mer_mha_fwd's layout) and Pd = dropout(P) [B,Lq,Lk] with the same mask index. */
int mer_softmax_dropout_fwd(int B, int H, int h, int Lq, int Lk, const float* S, float scale, float* P, float* Pd,
                            float p, const unsigned long long* seed, unsigned long long site, void* stream);

/* nn.CrossEntropyLoss(label_smoothing) (train.py:1033) or, late=1, NLLLoss(log(p+1e-8)) (train.py:212-214),
 * mean over the batch, fused with dloss/dlogits (for dloss = 1).  labels are int64.  preds (nullable): the
 * per-row top-1 index, first maximum as torch.argmax (train.py:216,220 ``outputs.argmax(dim=1)``). */
int mer_cross_entropy(int B, int C, const float* logits, const long long* labels, float label_smoothing, int late,
                      float* loss, float* dlogits, long long* preds, void* stream);

/* state = splitmix64(state + golden): the next step's RNG base, computed on the device (graph-capturable). */
int mer_rng_advance(unsigned long long* state, void* stream);

/* y = x * s[0] with s a device scalar (autograd grad_output of the loss). */
int mer_scale_dev(long n, const float* x, const float* s, float* y, void* stream);

/* In-place nn.Dropout(p) (train mode) over a row-strided matrix; mask regenerated from (seed, index). */
int mer_dropout_inplace(int rows, int cols, float* x, long ldx, float p, const unsigned long long* seed, unsigned long long site, void* stream);

/* Backward of dropout(relu(z)) given y: dy <- dy * (y > 0) * keep/(1-p), in place. */
int mer_relu_dropout_bwd(int rows, int cols, float* dy, long lddy, const float* y, long ldy, float p,
                         const unsigned long long* seed, unsigned long long site, void* stream);

/* Gated xattn head (fusion.py:318-327, 408-411): g = sigmoid(z[b]); out = g*v + (1-g)*a; and backward
 * (dv/da ACCUMULATE, dz written). */
int mer_gate_mix_fwd(int B, int D, const float* z, const float* v, long ldv, const float* a, long lda, float* out,
                     float* g_out, void* stream);
int mer_gate_mix_bwd(int B, int D, const float* g, const float* v, long ldv, const float* a, long lda,
                     const float* dout, float* dz, float* dv, long lddv, float* da, long ldda, void* stream);

/* EmotionPriorBiasAdapter._token_bias (fusion.py:170-176):
 * bias[b,i,j] = tanh(qt[b,i] + qp[b] + kt[b,j] + kp[b]) * scale[0]; and backward
 * (dqp == dkp == row-total; dscale_part[b] = per-sample partial of dscale). */
int mer_token_bias_fwd(int B, int Lq, int Lk, const float* qt, const float* qp, const float* kt, const float* kp,
                       const float* scale, float* out, void* stream);
int mer_token_bias_bwd(int B, int Lq, int Lk, const float* qt, const float* qp, const float* kt, const float* kp,
                       const float* scale, const float* dbias, float* dqt, float* dkt, float* dqp, float* dkp,
                       float* dscale_part, void* stream);

/* late fusion (fusion.py:358-363): out = (softmax(za) + softmax(zv)) / 2 (row-wise, [B,C]), saving both
 * softmaxes; and its backward (da, dv written). */
int mer_softmax_avg_fwd(int B, int C, const float* za, const float* zv, float* out, float* pa, float* pv, void* stream);
int mer_softmax_avg_bwd(int B, int C, const float* pa, const float* pv, const float* dout, float* da, float* dv,
                        void* stream);

/* out (+)= sum_i x[i]  (single-block deterministic reduce). */
int mer_vec_sum(int n, const float* x, float* out, int accumulate, void* stream);

/* torch.optim.Adam step (train.py:872,902; L2 weight decay added to the gradient) over one flat fp32
 * buffer; `step` is the 1-based step count used for bias correction; the gradient is multiplied by
 * grad_scale first (1/world_size after a SUM all-reduce).  16-byte aligned buffers. */
int mer_adam_step(long n, float* p, const float* g, float* m, float* v, float lr, float b1, float b2, float eps,
                  float wd, int step, float grad_scale, void* stream);

/* ============================ encoders (bf16 MFMA) ============================ */

/* C[m,n] = act(sum_k A(m,k) W[n,k] + bias[n]) (+ R[m,n]), bf16 operands, fp32 accumulate, C bf16 (c_dtype=1)
 * or fp32 (0).  Row m of A starts at A + (m / a_rpg)*a_gstride + (m % a_rpg)*a_rstride (K contiguous):
 * a_rpg = M, a_rstride = lda is a plain GEMM (WavLM projections/FFN, TF:108-296); a_rpg = L_out,
 * a_rstride = stride*C_in, a_gstride = L_in*C_in is a channel-last Conv1d (WavLM conv1-6, TF:675-745).
 * W is [N][K] (ldw).  K, strides multiple of 8; A, W 16-byte aligned.  bias / R may be NULL. */
int mer_gemm_bf16(int M, int N, int K, const void* A, long a_gstride, long a_rstride, int a_rpg, const void* W,
                  long ldw, void* C, int c_dtype, long ldc, const float* bias, const void* R, long ldr, int act,
                  void* stream);

/* mer_gemm_bf16 with an explicit kernel variant: -1 the wall-time pick (what mer_gemm_bf16 does), -2 the
 * CU-time pick (every shape on the 256x256 split ring: the train step's side-stream encoder forward), 0 the
 * 128x128 register-staged kernel (any K % 8 == 0), and the global_load_lds pipelined kernel as 7 (128x64 tiles,
 * 3-deep ring), 9 (128x128, 8 waves, 2-deep), 13 (256x256, 16 waves, 2-deep), 18 (256x256, 16 waves, split
 * rings: A 3-deep, B 2-deep), 22 (v18 with the LDS-DMA issued between the MFMA rows) and 23 (v22 on operand-
 * swapped MFMA: a bf16 output without residual or dropout is rounded before the LDS staging).  The automatic picks
 * send the split-ring shapes to v23 / v22 (v23 where its epilogue applies): -1 wherever it picks the split ring,
 * -2 for N <= 512 (the feature-extractor convs; the encoder layers keep v18).  K % 64 == 0 for 7-23, otherwise
 * variant 0 runs.  Every variant gives the same bits.  Other values: hipErrorInvalidValue. */
int mer_gemm_bf16_ex(int M, int N, int K, const void* A, long a_gstride, long a_rstride, int a_rpg, const void* W,
                     long ldw, void* C, int c_dtype, long ldc, const float* bias, const void* R, long ldr, int act,
                     int variant, void* stream);

/* Grouped positional Conv1d of WavLM (TF:48-90): out[b,t,g*Cg+n] = act(sum_{tap,c} X[b,t+tap-pad,g*Cg+c]
 * Wp[g][n][tap][c] + bias) (+ R), rows t in [0, L) (the SamePad crop).  Wp is the weight-normed, bf16
 * repacked kernel (mer_weightnorm_scale + mer_permute3_bf16).  variant -1: the Toeplitz strip kernel where it
 * applies (48 channels per group, L <= 160), else the gather GEMM; 0: the gather GEMM (bit-identical). */
int mer_posconv_gemm_bf16(int B, int L, int C_total, int groups, int taps, int pad, const void* X, long ldx,
                          const void* Wp, void* out, int out_dtype, long ldo, const float* bias, const void* R,
                          long ldr, int act, int variant, void* stream);

/* WavLM feature-extractor layer 0 (TF:723-745): Conv1d(1,512,k=10,s=5,no bias) of wav [B,S] fp32 ->
 * GroupNorm(512,512) (per (clip, channel) statistics over time of the bf16-rounded conv output) -> GELU,
 * written once as bf16 [B,Lout,512].  Two passes over the (cheap: 10 taps, on split-bf16 MFMA at fp32-class
 * accuracy) conv: statistics into per-tile partial rows, reduced in a fixed order (deterministic, no atomics),
 * then conv recompute + normalise + GELU.  workspace (16-byte aligned): float[B * (ceil(Lout/128) + 1) * 1024
 * + 16384] (the last 64 KB hold the split weight fragments). */
int mer_wavlm_conv0_gn_gelu(int B, int S, int Lout, const float* wav, const float* w0, const float* gamma,
                            const float* beta, float eps, float* workspace, void* out, void* stream);

/* Row LayerNorm (nn.LayerNorm(d), TF:93-105, 314-336, 418): x (x_dtype) -> y (y_dtype), d <= 1024. */
int mer_layernorm(int rows, int d, const void* x, int x_dtype, long ldx, const float* gamma, const float* beta,
                  float eps, void* y, int y_dtype, long ldy, void* stream);

/* WavLM self-attention with gated relative position bias (TF:147-271), one workgroup per (b,h):
 * qkv bf16 [B*L, 3*H*64] (q|k|v), x bf16 layer input (gate source), gate_w [8][64], gate_b [8],
 * gate_const [H], rel_emb [320][H], bucket int32 [2L-1] (bucket of relative position j-i), out bf16. L <= 256.
 * bucket == NULL: rel_emb is instead the per-head bias table [H][2L-1] = rel_emb[bucket].T (precomputed once
 * per forward: the position bias is shared by all 12 layers, TF:380-385). */
int mer_wavlm_attention(int B, int L, int H, const void* qkv, long ldqkv, const void* x, long ldx, const float* gate_w,
                        const float* gate_b, const float* gate_const, const float* rel_emb, const int* bucket,
                        void* out, long ldo, float scale, void* stream);

/* dst[i0][i1][i2] = bf16(src[i0*s0 + i1*s1 + i2*s2] * (scale ? scale[i1] : 1))  (weight repacking). */
int mer_permute3_bf16(int n0, int n1, int n2, const float* src, long s0, long s1, long s2, const float* scale,
                      void* dst, void* stream);

/* weight_norm(dim=2) factors of the positional conv: scale[k] = g[k] / ||v[:,:,k]||_2, v [n01][taps]. */
int mer_weightnorm_scale(int n01, int taps, const float* v, const float* g, float* scale, void* stream);

/* y = bf16(x), contiguous. */
int mer_cast_bf16(long n, const float* x, void* y, void* stream);

/* ---- WavLM train-mode semantics (the reference runs the frozen WavLM in train mode under no_grad,
 * train.py:194 + wavlm_audio.py:177-182): dropout, LayerDrop, SpecAugment time masking ----
 * Common train-mode arguments: drop_p / seed / site = dropout probability, the step's device RNG base and a
 * constant call-site id (mask = hash(base, site, element), regenerated by backward kernels); skip_mask /
 * skip_bit = LayerDrop (TF:417-419): the launch is a no-op when bit skip_bit of the device int64 *skip_mask is
 * set (one host-drawn bitmask per forward, so a captured hipGraph replays any layer subset). */

/* mer_gemm_bf16_ex + dropout after the activation and before the residual (attention output dropout TF:323,
 * FFN intermediate / output dropout TF:286-294; mask index row*N + col) + LayerDrop skip. */
int mer_gemm_bf16_tr(int M, int N, int K, const void* A, long a_gstride, long a_rstride, int a_rpg, const void* W,
                     long ldw, void* C, int c_dtype, long ldc, const float* bias, const void* R, long ldr, int act,
                     float drop_p, const unsigned long long* seed, unsigned long long site, const long long* skip_mask,
                     int skip_bit, int variant, void* stream);

/* mer_layernorm + dropout of the OUTPUT (WavLMEncoder.dropout after the encoder LayerNorm, TF:406-407; mask index
 * row*d + c) + LayerDrop skip (the post-LN layers' norms). */
int mer_layernorm_tr(int rows, int d, const void* x, int x_dtype, long ldx, const float* gamma, const float* beta,
                     float eps, void* y, int y_dtype, long ldy, float drop_p, const unsigned long long* seed,
                     unsigned long long site, const long long* skip_mask, int skip_bit, void* stream);

/* mer_wavlm_attention + attention-probability dropout (F.multi_head_attention_forward dropout_p, TF:206-228;
 * mask index ((b*H + h)*L + i)*L + j) + LayerDrop skip. */
int mer_wavlm_attention_tr(int B, int L, int H, const void* qkv, long ldqkv, const void* x, long ldx,
                           const float* gate_w, const float* gate_b, const float* gate_const, const float* rel_emb,
                           const int* bucket, void* out, long ldo, float scale, float drop_p,
                           const unsigned long long* seed, unsigned long long site, const long long* skip_mask,
                           int skip_bit, void* stream);

/* SpecAugment time masking (WavLMModel._mask_hidden_states TF:985-1015, _compute_mask_indices TF:834-950):
 * in the projected features h bf16 [B*L, D] (ldh), n spans of mask_len frames per sample are replaced by
 * masked_spec_embed (fp32 [D]); n = max(int(mask_prob * L / mask_len + eps), min_masks) (capped as TF), eps
 * shared by the batch, span starts distinct and uniform in [0, L - mask_len] (device hash RNG).  mask_out
 * (optional, uint8 [B, L]) receives the masked-frame indicator. */
int mer_wavlm_time_mask(int B, int L, int D, void* h, long ldh, const float* embed, float mask_prob, int mask_len,
                        int min_masks, const unsigned long long* seed, unsigned long long site, unsigned char* mask_out,
                        void* stream);

/* y = x for a contiguous bf16 x, y bf16 (y_dtype 1) or fp32 (0). */
int mer_bf16_convert(long n, const void* x, void* y, int y_dtype, void* stream);

/* ============================ WavLM stage-2 fine-tuning (backward of the last N layers) ============================
 * The reference unfreezes the last N encoder layers (wavlm_audio.py:70-88 _unfreeze_last_n_layers, called by
 * train.py:817-822 _apply_two_stage_freeze_policy); these entry points are the backward of those layers
 * (post-LN WavLMEncoderLayer TF:314-336, attention TF:147-186).  Deterministic: row reductions are stored as
 * per-block partial rows and folded in a fixed order by mer_fold_rows. */

/* LayerNorm backward (nn.LayerNorm(d), TF:326,329): g = dy_a (+ dy_b) (+ dy_c) (NULL addends skipped), x = the saved
 * fp32 LN input; dx written fp32 (dx32) and/or bf16 (dx16) (either may be NULL).  part: float[ceil(rows/16)][3][d]
 * = per-block (sum g*xhat, sum g, sum dx) -- fold with mer_fold_rows for dgamma, dbeta and the upstream bias.
 * d % 256 == 0, d <= 1024. */
int mer_ln_bwd(int rows, int d, const float* dy_a, const float* dy_b, const float* dy_c, const float* x,
               const float* gamma, float eps, float* dx32, void* dx16, float* part, void* stream);

/* out[k] += sum_{p < parts} part[p * ldp + k] for k < n, summed in a fixed order (deterministic).  parts > 64 runs
 * two stages through workspace float[64 * n] (may be NULL when parts <= 64). */
int mer_fold_rows(int parts, int n, const float* part, long ldp, float* out, float* workspace, void* stream);

/* part[p][c] = sum of rows [64p, 64p+64) of x[:, c] (x_dtype 0 fp32 / 1 bf16): part is float[ceil(rows/64)][cols]. */
int mer_colpart(int rows, int cols, const void* x, int x_dtype, long ldx, float* part, void* stream);

/* f = gelu(z) elementwise, bf16 -> bf16, n % 8 == 0 (the FFN activation of a trainable layer, TF:286-296). */
int mer_gelu_bf16(long n, const void* z, void* f, void* stream);

/* dz = df * gelu'(z) -> bf16 [rows][cols]; part float[ceil(rows/64)][cols] column partial sums of dz (bias grad). */
int mer_gelu_bwd(int rows, int cols, const float* df, const void* z, void* dz, float* part, void* stream);

/* Linear weight gradient dw[n][k] += sum_m dy[m][n] x[m][k] (bf16 operands, fp32 dw), x [M][K] contiguous, dy rows
 * of stride ldy (a column slice of a wider gradient works); bf16 MFMA (the 1x1 case of mer_conv_wgrad).
 * workspace: splits * N * K floats.  K, N, ldy multiples of 8. */
int mer_linear_wgrad(int M, int N, int K, const void* x, const void* dy, long ldy, float* dw, int splits,
                     float* workspace, void* stream);

/* Backward of mer_wavlm_attention (tbl form: per-head bias table [H][2L-1]), L <= 192, on bf16 MFMA (fp32
 * operands split hi + lo).  dout fp32 [B*L][>=H*64] (gradient of the attention output; fp32 because
 * dp_ij - sum_j p_ij dp_ij cancels for peaked rows), qkv / x as in the forward (ldqkv, ldx multiples of 8, ldo and
 * lddq of 4).  Writes dqkv bf16 [B*L][3*H*64] (dq | dk | dv), dx_gate fp32 (the gate path's gradient of the layer
 * input x; may be NULL), gate_part float[B*H*ceil(L/64)][8*64 + 8 + H] per-block partials of
 * (d gru_rel_pos_linear.weight [8][64], .bias [8], d gru_rel_pos_const [H]) -- fold with mer_fold_rows.
 * scratch: B*H * KP * (3 KP + 64) bf16 (P, dS hi, dS lo, bf16 dO between the two kernels),
 * KP = mer_wavlm_attention_bwd_kp(L). */
int mer_wavlm_attention_bwd(int B, int L, int H, const void* qkv, long ldqkv, const void* x, long ldx,
                            const void* dout, long ldo, const float* gate_w, const float* gate_b,
                            const float* gate_const, const float* tbl, float scale, void* scratch,
                            void* dqkv, long lddq, float* dx_gate, long lddxg, float* gate_part, void* stream);
/* Train mode (stage-2 fine-tuning with the reference's attention dropout, TF:206-228): the same backward for a forward
 * run with mer_wavlm_attention_tr(drop_p, seed, site): the probability mask (index ((b*H+h)*L + i)*L + j) is
 * regenerated, dP = (dO V^T) o M and dV = (P o M)^T dO.  drop_p = 0 is mer_wavlm_attention_bwd.
 * Replaces: the backward of F.multi_head_attention_forward's dropout_p inside WavLMAttention (TF:206-228). */
int mer_wavlm_attention_bwd_tr(int B, int L, int H, const void* qkv, long ldqkv, const void* x, long ldx,
                               const void* dout, long ldo, const float* gate_w, const float* gate_b,
                               const float* gate_const, const float* tbl, float scale, void* scratch,
                               void* dqkv, long lddq, float* dx_gate, long lddxg, float* gate_part, float drop_p,
                               const unsigned long long* seed, unsigned long long site, void* stream);
/* y = x o M / (1 - p) for the dropout call site `site` (mask index row * cols + col, the index of the GEMM-epilogue
 * dropout of mer_gemm_bf16_tr), regenerated from the step's RNG base: x fp32 or bf16 [rows][ldx], y32 (fp32) and /
 * or y16 (bf16) outputs (either may be NULL).  cols and the strides multiples of 8 (ldy32 of 4).  Stage-2 uses: the
 * FFN activation dropout in the forward, and every dropout's backward (the same mask on the gradient).
 * Replaces: nn.Dropout / F.dropout of WavLMFeedForward and WavLMAttention's output (TF:286-294, 323) in backward. */
int mer_dropout_rows(int rows, int cols, const void* x, int x_dtype, long ldx, float* y32, long ldy32, void* y16,
                     long ldy16, float p, const unsigned long long* seed, unsigned long long site, void* stream);
/* Padded key / query count of mer_wavlm_attention_bwd's scratch (16 * 4 / 8 / 10 / 12 for L <= 64 / 128 / 160 /
 * 192; 0 when L is out of range). */
int mer_wavlm_attention_bwd_kp(int L);

/* dst[c][r] = src[r][c], bf16 (the transposed weight operands of the stage-2 data-gradient GEMMs). */
int mer_transpose_bf16(int rows, int cols, const void* src, long lds, void* dst, long ldd, void* stream);

/* ============================ clip assembly (first step) ============================ */

/* Post-decode frame preprocessing of load_video_frames (ravdess.py:352 cv2.resize(frame, (S, S), INTER_LINEAR),
 * :363 /255, :386-389 (x - mean) / std, HWC -> CHW): frames = N decoded RGB uint8 [H0][W0][3] images, frame_stride
 * bytes apart -> out fp32 [N][3][S][S].  OpenCV's scalar fixed-point linear path (11-bit weights, exact 2x
 * downscale = INTER_AREA 2x2 average). */
int mer_frames_resize_normalize(int N, int H0, int W0, const void* frames, long frame_stride, int S, float mean0,
                                float mean1, float mean2, float std0, float std1, float std2, float* out, void* stream);

/* cv2.resize(frame, (S, S), INTER_LINEAR) alone (ravdess.py:352): out uint8 [N][S][S][3] (the augmentation's input). */
int mer_frames_resize_u8(int N, int H0, int W0, const void* frames, long frame_stride, int S, void* out, void* stream);
/* Train-split video augmentation + normalisation of load_video_frames (ravdess.py:363-389) on resized frames
 * frames_u8 [N][S][S][3] (N = clips * T): per clip c, clip_params[c] = (factor, noise_scale, ksize) and a noise seed
 * clip_seeds[c] (DEVICE arrays): uint8 round trip, cv2.GaussianBlur(k, sigma 0) in OpenCV's exact 8U fixed-point form
 * (BORDER_REFLECT_101), /255, * factor, + noise_scale * ztable[hash(seed, element) >> 16] (ztable: DEVICE fp32
 * [65536], the inverse normal CDF at (i + 0.5) / 65536), clip to [0, 1], (x - mean) / std -> out fp32 [N][3][S][S].
 * Replaces: the `if augment:` block of ravdess.py:366-384. */
int mer_frames_augment_normalize(int N, int S, int T, const void* frames_u8, const float* clip_params,
                                 const unsigned long long* clip_seeds, const float* ztable, float mean0, float mean1,
                                 float mean2, float std0, float std1, float std2, float* out, void* stream);

/* load_audio_wav pad / crop (ravdess.py:505-513): out[b][t] = t < lengths[b] ? packed[offsets[b] + t] : 0,
 * out fp32 [B][target]; offsets / lengths are DEVICE int64 arrays (a ragged batch of decoded waveforms). */
int mer_wav_pad_crop(int B, int target, const float* packed, const long long* offsets, const long long* lengths,
                     float* out, void* stream);

/* ============================ ResNet18 frame trunk (bf16 MFMA, NHWC) ============================
 * VideoNet.backbone (video.py:21-23 -> torchvision resnet18 children[:-1]).  Activations are NHWC bf16
 * with channels padded to a multiple of 8. */

/* y[n,oh,ow,k] = sum_{r,s,c} x[n,oh*st-pad+r,ow*st-pad+s,c] w[k][r][s][c]  (bf16 out); if stats != NULL,
 * stats (zeroed float[MER_BN_STAT_ROWS(M)][K][2]) receives, per output row tile, the (sum, sum of squares) of the
 * stored outputs (BatchNorm batch statistics; deterministic, see MER_BN_STAT_ROWS). */
int mer_conv_fwd(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* x,
                 const void* w_packed, void* y, float* stats, void* stream);

/* mer_conv_fwd / mer_conv_dgrad with an explicit kernel: -1 auto, 0 the register-staged implicit GEMM,
 * 1 the global_load_lds pipelined one (zero padding served from a zero chunk), 2 the same with 8-wave tiles
 * (the default), 3 with 256-row tiles (8 or 16 waves) on large-M layers. */
int mer_conv_fwd_ex(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* x,
                    const void* w_packed, void* y, float* stats, int variant, void* stream);

/* dx[n,h,w,c] = sum_{r,s,k} dy[n,(h+pad-r)/st,(w+pad-s)/st,k] wt[c][r][s][k] (+ residual where mask > 0). */
int mer_conv_dgrad(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* dy,
                   const void* wt_packed, void* dx, const void* residual, const void* residual_mask, void* stream);
int mer_conv_dgrad_ex(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* dy,
                      const void* wt_packed, void* dx, const void* residual, const void* residual_mask, int variant,
                      void* stream);

/* mer_conv_dgrad_ex (pipelined kernel only) with the BatchNorm-backward reduction of the BN the gradient
 * flows into fused into the epilogue: g = (bn_mask > 0) * dx (after the residual), each output row tile
 * STORES its (sum g, sum g * (bn_x - mean) * rstd) row with (mean, rstd) = bn_ms[c] into bn_red, and bn_red2
 * likewise for bn_x2 / bn_ms2 (may be NULL).  bn_red / bn_red2 are zeroed float[MER_BN_RED_ROWS(M)][C][2]
 * (M = N*H*W gradient pixels); fold them with mer_partials_sum(C, MER_BN_RED_ROWS(M) - 64, ...) before
 * mer_bn_bwd_apply (fixed-order sums: deterministic).  Replaces mer_bn_bwd_reduce after a conv backward. */
int mer_conv_dgrad_bnr(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* dy,
                       const void* wt_packed, void* dx, const void* residual, const void* residual_mask,
                       const void* bn_mask, const void* bn_x, const float* bn_ms, float* bn_red, const void* bn_x2,
                       const float* bn_ms2, float* bn_red2, int variant, void* stream);
/* mer_conv_dgrad_bnr of a 3x3 / stride-2 / pad-1 conv with the input gradient of a 1x1 / stride-2 / pad-0
 * downsample of the SAME input fused in (the first BasicBlock of layers 2-4, video.py:21-23 -> torchvision
 * BasicBlock.downsample): dx += conv-transpose(ds_dy [N][Ho][Wo][ds_K], ds_wt_packed [C][ds_K]) as an extra
 * reduction segment of parity class (0, 0), the only pixels its taps reach -- one launch and one fp32 accumulator
 * instead of a separate dgrad whose bf16 output the 3x3 dgrad read back as its residual.  ds_K, K multiples of
 * 64; ds_dy NULL = mer_conv_dgrad_bnr. */
int mer_conv_dgrad_ds(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* dy,
                      const void* wt_packed, void* dx, const void* residual, const void* residual_mask,
                      const void* bn_mask, const void* bn_x, const float* bn_ms, float* bn_red, const void* bn_x2,
                      const float* bn_ms2, float* bn_red2, const void* ds_dy, const void* ds_wt_packed, int ds_K,
                      int variant, void* stream);

/* The number of leading partial rows (BatchNorm statistics rows of mer_conv_fwd_ex / BN-backward reduction rows of
 * mer_conv_dgrad_ds) the call with these arguments writes: one per output row tile (MER_BN_STAT_ROWS(M) - 64,
 * MER_BN_RED_ROWS(M) - 64), or one per workgroup where the persistent halo kernel runs (layer1, the stem: 256 / 512
 * at B = 32 instead of 3,136 / 12,544), whose rows past these stay zero.  For mer_conv_fwd_ex with variant -1 the
 * count is exact (every row below it is written: one per BM-row tile of the default tile choice), so a statistics
 * buffer of such a call needs no zeroing; for an explicit variant it is an upper bound (zero the buffer).  Likewise
 * mer_conv_dgrad_rows for a stride-1 / stride-2 dgrad with variant -1 (one row per BM-row tile, per parity class).   The same geometry test as the launch; a
 * negative hipError_t on invalid arguments.  Pass the count to mer_bn_finalize_rows / mer_partials_sum so the
 * fold reads only written rows (one launch instead of two past 1,024 tile rows). */
int mer_conv_fwd_rows(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* x,
                      const void* w_packed, int variant);
int mer_conv_dgrad_rows(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* dy,
                        const void* wt_packed, const void* ds_dy, int variant);

/* out[c][0:2] = sum_p in[p][c][0:2] over `parts` partial rows, in a fixed order.  parts > 64 needs 64 more
 * rows after them in `in` (fold scratch, overwritten). */
int mer_partials_sum(int C, int parts, float* in, float* out, void* stream);
/* Two mer_partials_sum folds of the same shape (C, parts) in one launch (in, out) and (in2, out2): a stride-2
 * BasicBlock's bn2 and downsample-BN backward sums, which one fused dgrad epilogue wrote. */
int mer_partials_sum2(int C, int parts, float* in, float* out, float* in2, float* out2, void* stream);

/* dw[k][c][r][s] += sum_p dy[p][k] x(p; r,s,c) for c < Creal, fp32 PyTorch layout (dw initialised).  The
 * pixel reduction is split `splits` ways; each split writes an fp32 slab [K][R*S*C] into `workspace`
 * (splits*K*R*S*C floats), then a reduce pass sums the slabs into dw (deterministic, no atomics). */
int mer_conv_wgrad(int N, int H, int W, int C, int Creal, int K, int R, int S, int stride, int pad, const void* x,
                   const void* dy, float* dw, int splits, float* workspace, void* stream);
/* mer_conv_wgrad with an explicit kernel: -1 auto, 1 4-wave tiles, 2 8-wave tiles (the default). */
int mer_conv_wgrad_ex(int N, int H, int W, int C, int Creal, int K, int R, int S, int stride, int pad, const void* x,
                      const void* dy, float* dw, int splits, float* workspace, int variant, void* stream);
/* The split-K pass of mer_conv_wgrad alone: workspace = splits x [K][R*S*C] fp32 partial slabs, folded later by
 * mer_wgrad_fold_batch (one launch for all weight gradients of a backward segment). */
int mer_conv_wgrad_partials(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, const void* x,
                            const void* dy, int splits, float* workspace, int variant, void* stream);
/* Fold n <= 32 deferred slab sets in one launch.  rows: n x 8 int64 {ws, dw, map, K, C, Creal, R*S, splits}:
 * dw[k][c][r][s] += sum_z ws[z][k][(r*S+s)*C + c] for c < Creal (fixed split order), or, with map != NULL
 * (int32 [R*S*C], -1 = dropped), dw[k][map[j]] += sum_z ws[z][k][j] with Creal = dw floats per k. */
int mer_wgrad_fold_batch(int n, const long long* rows, void* stream);

/* NCHW fp32 frames -> NHWC bf16 with channels zero-padded to Cp (<= 16). */
int mer_pack_input_nhwc(int N, int C, int H, int W, int Cp, const float* x, void* y, void* stream);
/* Space-to-depth stem input: fp32 NCHW [N][C<=4][H][W] (H, W even) -> bf16 [N][H/2+3][W/2+3][16].
 * ResNet conv1 (7x7, stride 2, pad 3) then runs as a 4x4, stride-1, unpadded conv on 16 channels
 * (K = 256 instead of 392), weights packed by mer_pack_conv_weights mode 2 (video.py:21-23 stem). */
int mer_pack_input_s2d(int N, int C, int H, int W, const float* x, void* y, void* stream);

/* PyTorch conv weight [K][C][R][S] fp32 -> bf16 [K][R][S][Cp] (transpose=0, forward) or [Cp][R][S][K]
 * (transpose=1, data-gradient operand); channels >= C are zero. */
int mer_pack_conv_weight(int K, int C, int R, int S, int Cp, int transpose, const float* w, void* out, void* stream);

/* n (<= 64) mer_pack_conv_weight layouts in one launch (the trunk's per-step re-pack).  desc: DEVICE table of
 * n records of 9 int64 {w, out, K, C, R, S, Cp, transpose, first element} (transpose 2: space-to-depth stem
 * layout [K][(R+2)/2][(S+2)/2][Cp], see mer_pack_input_s2d), records in output order, first
 * elements the prefix sums of K*R*S*Cp; total = the sum. */
int mer_pack_conv_weights(int n, const long long* desc, long total, void* stream);
/* The same packs on a 1-D grid with no idle blocks: column 8 of each record is instead its first block, a record
 * taking K blocks (transpose 0 / 2) or Cp * ceil(K / 64) blocks (transpose 1); total_blocks = the sum.  Output is
 * bit-identical to mer_pack_conv_weights (the per-step re-pack in video.py uses this form). */
int mer_pack_conv_weights_flat(int n, const long long* desc, long total_blocks, void* stream);

/* BatchNorm2d finalize: ms[c] = (mean, rstd) from the MER_BN_STAT_ROWS(M) stats rows of a conv forward (summed in a
 * fixed order, through the buffer's 64 scratch rows) over M values and, when non-NULL, updates
 * running_mean / running_var (unbiased) with `momentum` and increments num_batches_tracked (train mode).
 * stats == NULL is eval mode: ms = (running_mean, 1/sqrt(running_var + eps)), nothing updated. */
int mer_bn_finalize(int C, long M, const float* stats, float eps, float momentum, float* ms, float* rmean,
                    float* rvar, long long* num_batches_tracked, void* stream);
/* mer_bn_finalize summing only the first data_rows (<= MER_BN_STAT_ROWS(M) - 64) statistics rows -- the count
 * mer_conv_fwd_rows returned for the conv that filled them; the scratch rows stay at the buffer's end. */
int mer_bn_finalize_rows(int C, long M, int data_rows, const float* stats, float eps, float momentum, float* ms,
                         float* rmean, float* rvar, long long* num_batches_tracked, void* stream);
/* Two train-mode mer_bn_finalize_rows in one launch (both stats non-NULL; shared eps / momentum): a stride-2
 * BasicBlock's bn2 and downsample BN, both convs done before either BatchNorm is applied. */
int mer_bn_finalize_rows2(int C, long M, int data_rows, const float* stats, float* ms, float* rmean, float* rvar,
                          long long* nbt, int C2, long M2, int data_rows2, const float* stats2, float* ms2,
                          float* rmean2, float* rvar2, long long* nbt2, float eps, float momentum, void* stream);

/* y = [relu](bn(x) + (ms2 ? bn2(res) : res)), ms = (mean, rstd) pairs; res may be NULL. */
int mer_bn_apply(long M, int C, const void* x, const float* ms, const float* gamma, const float* beta, const void* res,
                 const float* ms2, const float* gamma2, const float* beta2, int relu, void* y, void* stream);

/* BN backward reduction: red[c] = (sum g, sum g*xhat), g = dy * (mask > 0) (mask = ReLU output or NULL);
 * per-block partial rows in workspace (float[MER_BN_RED_WS_ROWS][C][2]) folded in a fixed order. */
int mer_bn_bwd_reduce(long M, int C, const void* dy, const void* mask, const void* x, const float* ms, float* red,
                      float* workspace, void* stream);

/* BN backward apply: dx = gamma*rstd*(g - s1/M - xhat*s2/M) with batch statistics (batch_stats=1, train
 * mode) or dx = gamma*rstd*g with running statistics (batch_stats=0, eval mode); dgamma += s2, dbeta += s1. */
int mer_bn_bwd_apply(long M, int C, const void* dy, const void* mask, const void* x, const float* ms,
                     const float* gamma, const float* red, int batch_stats, void* dx, float* dgamma, float* dbeta,
                     void* stream);
/* Two mer_bn_bwd_apply passes over the same dy and ReLU mask (non-NULL) in one launch -- a stride-2 BasicBlock's
 * bn2 (x, ms, gamma, red -> dx) and downsample BN (x2, ms2, gamma2, red2 -> dx2), video.py:21-23 -> torchvision
 * BasicBlock: g and the mask are read once; each output bit-identical to its own mer_bn_bwd_apply (dx, dx2 must not
 * alias dy). */
int mer_bn_bwd_apply2(long M, int C, const void* dy, const void* mask, const void* x, const float* ms,
                      const float* gamma, const float* red, const void* x2, const float* ms2, const float* gamma2,
                      const float* red2, int batch_stats, void* dx, void* dx2, float* dgamma, float* dbeta,
                      float* dgamma2, float* dbeta2, void* stream);

/* Fused stem tail (C % 8 == 0, C <= 512, N*H*W < 2^22; x = the stem conv output [N][H][W][C] bf16):
 * y = maxpool3x3s2p1(bf16(relu(bn(x)))) with argmax taps, the BN/ReLU activation never stored.
 * Replaces bn_apply + maxpool_fwd for torchvision's conv1 -> bn1 -> relu -> maxpool (video.py:21-23). */
int mer_stem_bnrelu_maxpool_fwd(int N, int H, int W, int C, const void* x, const float* ms, const float* gamma,
                                const float* beta, void* y, void* argmax, void* stream);
/* Its backward to the conv output: the maxpool gather of dy is written to dx, then g = dx * relu'(bn(x)) (mask
 * recomputed from x, no activation tensor) feeds a BatchNorm reduction (red[C][2] = (sum g, sum g*xhat), through
 * workspace float[MER_BN_RED_WS_ROWS][C][2] as mer_bn_bwd_reduce) and an in-place apply pass
 * dx = gamma*rstd*(g - [batch_stats] (sum g + xhat * sum g*xhat)/M); dgamma += sum g*xhat, dbeta += sum g. */
int mer_stem_pool_bn_bwd(int N, int H, int W, int C, const void* dy, const void* argmax, const void* x,
                         const float* ms, const float* gamma, const float* beta, float* red, int batch_stats,
                         void* dx, float* dgamma, float* dbeta, float* workspace, void* stream);

/* MaxPool2d(3, 2, 1) forward (argmax tap saved as uint8) and gather backward. */
int mer_maxpool_fwd(int N, int H, int W, int C, const void* x, void* y, void* argmax, void* stream);
int mer_maxpool_bwd(int N, int H, int W, int C, const void* dy, const void* argmax, void* dx, void* stream);

/* AdaptiveAvgPool2d(1): NHWC bf16 -> [N,C] fp32, and backward (dx = dy / HW, bf16). */
int mer_avgpool_fwd(int N, int HW, int C, const void* x, float* y, void* stream);
int mer_avgpool_bwd(int N, int HW, int C, const float* dy, void* dx, void* stream);

/* ============================ dynamic INT8 Linear (inference) ============================
 * TorchModelRunner(enable_dynamic_quant=True): optimized_runtime.py:95-96
 * (torch.quantization.quantize_dynamic(model, {nn.Linear}, qint8), fbgemm semantics -- oracle/int8_ref.py).
 * qparams are 4 floats on the device: {scale, 1/scale, zero_point, 0}. */

/* min/max over x[0:n] (fp32 or bf16; partial = 2*512 floats of workspace) -> qparams.  mode 0: activation
 * (fbgemm ChooseQuantizationParams, range [0,127] = reduce_range); mode 1: symmetric weight scale
 * max(amax/127.5, FLT_EPSILON), zero point 0. */
int mer_quant_params(long n, const void* x, int x_dtype, float* partial, int mode, float* qparams, void* stream);

/* qw[n, 0:ldq] = int8 clamp(rint(W[n,k] / ws)) (zero for k >= K); colsum[n] = sum_k qw[n,k].
 * ldq % 16 == 0.  Run once per Linear when the model is quantized. */
int mer_quantize_weight_s8(int N, int K, const float* w, long ldw, const float* qparams, void* qw, long ldq,
                           int* colsum, void* stream);

/* out[m,n] = act(fma(sum_k qx[m,k] qw[n,k] - zp * colsum[n], xs*ws, bias[n])) with
 * qx = clamp(rint(fma(x, 1/xs, zp)), 0, 255) computed on the fly from fp32 / bf16 x (K % 16 == 0;
 * act 0 or 1).  The quantized Linear forward (torch.ao.nn.quantized.dynamic.Linear). */
int mer_gemm_i8dyn(int M, int N, int K, const void* x, int x_dtype, long ldx, const float* x_qparams, const void* qw,
                   long ldq, const float* w_qparams, const int* colsum, const float* bias, int act, float* out, long ldo,
                   void* stream);

/* INT8 emotion-prior token-bias input rows (fusion.py:170-176): out[b*L + l] = [tok[b*L + l, :d], prior[b, :pd],
 * zeros up to ldo] (ldo >= d + pd, a multiple of 16 for mer_gemm_i8dyn). */
int mer_concat_prior_rows(int B, int L, int d, int pd, int ldo, const float* tok, const float* prior, float* out,
                          void* stream);

/* ============================ fused xattn head (csrc/xattn_fused.hip) ============================
 * The xattn branch after the encoders (fusion.py:372-411: projections, v2a / a2v nn.MultiheadAttention with
 * residual + StochasticDepth + LayerNorm, mean TemporalPooler, concat / gated head) in four launches, every
 * product on split-bf16 MFMA (fp32 operands as bf16 hi + lo planes, fp32 accumulation).  d_model 128, 4 heads.
 * Dropout / drop-path: attention-probability masks index ((b*H + h)*Lq + i)*Lk + j, drop-path one draw per
 * sample, MLP dropout row*H1 + col -- the conventions of mer_mha_fwd / mer_add_ln_fwd / mer_dropout_inplace,
 * so mer_mha_bwd / mer_add_ln_bwd and the rest of the unfused backward regenerate the same masks. */

/* Split fp32 weights into bf16 hi / lo planes, one descriptor row (src, hi, lo, rows, cols, trans, dst_ld) of
 * the device int64 table desc[n_items][7] per [rows][cols] weight: trans 0 writes the planes in the source layout,
 * trans 1 transposed (dst[c * dst_ld + r], the [in][out] planes the fused backward's data-gradient products read). */
int mer_xh_split(int n_items, const long long* desc, void* stream);

/* F1 from a precomputed first product: pair [M][ldp] fp32 holds aseq Ws_hi^T in columns 0..127 and aseq Ws_lo^T in
 * 128..255 (one mer_gemm_bf16 of the bf16 WavLM features with the stacked [hi; lo] planes of audio_seq_proj);
 * a_s = pair[:, :128] + pair[:, 128:] + bs, then a, q2, kv1 and the video rows as mer_xh_audio_fwd does.  The two
 * halves are summed after their K loops, where mer_xh_audio_fwd folds hi and lo into one running sum per k step, so
 * the two entries agree to fp32 rounding, not bit for bit (tests/test_xattn_fused_gpu.py::test_f1_pair_matches_in_kernel). */
int mer_xh_audio_fwd_pair(int M, const float* pair, long ldp, const float* bs, const void* Wa_hi, const void* Wa_lo,
                          const float* ba, const void* Wc_hi, const void* Wc_lo, const float* bq2, const float* bkv1,
                          float* a_s, float* a, float* q2, float* kv1, int Mv, int vdim, const float* vfeat,
                          const void* Wv_hi, const void* Wv_lo, const float* bv, const void* Wq1_hi, const void* Wq1_lo,
                          const float* bq1, float* v, float* q1, void* stream);

/* F1: a_s = aseq Ws^T + bs (aseq [M][S] bf16 -- the WavLM features, exact -- or fp32), a = a_s Wa^T + ba,
 * [q2 | kv1] = a Wc^T + [bq2 | bkv1] (Wc = [a2v in_proj q rows; v2a in_proj k, v rows], 384 x 128).  Outputs
 * fp32: a_s, a, q2 [M][128], kv1 [M][256].  S % 32 == 0.  The same launch projects the Mv video rows:
 * v = vfeat Wv^T + bv, q1 = v Wq1^T + bq1 ([Mv][128]; vdim % 32 == 0). */
int mer_xh_audio_fwd(int M, int S, const void* aseq, int aseq_dtype, long ldas, const void* Ws_hi, const void* Ws_lo,
                     const float* bs, const void* Wa_hi, const void* Wa_lo, const float* ba, const void* Wc_hi,
                     const void* Wc_lo, const float* bq2, const float* bkv1, float* a_s, float* a, float* q2,
                     float* kv1, int Mv, int vdim, const float* vfeat, const void* Wv_hi, const void* Wv_lo,
                     const float* bv, const void* Wq1_hi, const void* Wq1_lo, const float* bq1, float* v, float* q1,
                     void* stream);

/* F2 (two launches: the attention per (sample, head), then the rest per sample; T <= 16, Ta <= 256): v2a attention
 * of q1 over kv1, o1 Wo1^T + bo1,
 * v1 = LayerNorm(v + keep_b * v2) (saving the pre-LN sum, mean, rstd), kv2 = v1 Wkv2^T + bkv2,
 * emb[b][0:128] = mean_t v1.  P1 [B][4][T][Ta] receives the pre-dropout probabilities.  bias (nullable): the
 * emotion-prior attention bias [B][T][Ta] added to every head's scaled scores (fusion.py:390-394 attn_mask). */
int mer_xh_v2a_fwd(int B, int T, int Ta, const float* v, const float* q1, const float* kv1, const void* Wo1_hi,
                   const void* Wo1_lo, const float* bo1, const float* gamma, const float* beta, const void* Wkv2_hi,
                   const void* Wkv2_lo, const float* bkv2, float attn_p, float path_p, const unsigned long long* seed,
                   unsigned long long site_attn, unsigned long long site_path, float scale, float* P1, float* o1,
                   float* s_v, float* mean_v, float* rstd_v, float* v1, float* kv2, float* emb, long ld_emb,
                   const float* bias, void* stream);

/* F3 (one workgroup per (sample, 16 query rows)): a2v attention of q2 over kv2 (T keys), o2 Wo2^T + bo2,
 * a1 = LayerNorm(a + keep_b * a2) (pre-LN sum / mean / rstd saved), part[b][tile][128] = column sums of a1 over the
 * tile's rows.  P2 [B][4][Ta][T].  bias (nullable): the emotion-prior a2v bias [B][Ta][T] (fusion.py:391,398). */
int mer_xh_a2v_fwd(int B, int T, int Ta, const float* q2, const float* kv2, const float* a, const void* Wo2_hi,
                   const void* Wo2_lo, const float* bo2, const float* gamma, const float* beta, float attn_p,
                   float path_p, const unsigned long long* seed, unsigned long long site_attn,
                   unsigned long long site_path, float scale, float* P2, float* o2, float* s_a, float* mean_a,
                   float* rstd_a, float* part, const float* bias, void* stream);

/* Emotion-prior attention bias forward (EmotionPriorBiasAdapter, fusion.py:153-184, used at fusion.py:390-391;
 * replaces xattn_head.prior_forward's ~14 launches), one workgroup per sample, exact fp32: pg = [mean_t v | mean_j a]
 * [B][2d], h1 = dropout(relu(pg W0^T + b0)) [B][H1] (mask index b*H1 + j at `site`), prior = h1 W3^T + b3 [B][PD];
 * the four token-bias Linears (w_*: [d + PD] rows, b_*: [1]) as token halves tt_* = token . w[:d] ([B*T] for vq / vk,
 * [B*Ta] for ak / aq) and prior halves tp_* = prior . w[d:] + b ([B]); v2a_bias[b][i][j] = tanh(tt_vq + tt_ak + tp_vq
 * + tp_ak) * scale [B][T][Ta], a2v_bias[b][j][i] = tanh(tt_aq + tt_vk + tp_aq + tp_vk) * scale [B][Ta][T].
 * v [B*T][d], a [B*Ta][d] fp32 pre-attention tokens; d = 128, T <= 16, Ta <= 160, H1 <= 256, PD <= 16. */
int mer_xh_prior_fwd(int B, int T, int Ta, int d, int H1, int PD, const float* v, const float* a, const float* W0,
                     const float* b0, const float* W3, const float* b3, const float* w_vq, const float* b_vq,
                     const float* w_ak, const float* b_ak, const float* w_aq, const float* b_aq, const float* w_vk,
                     const float* b_vk, const float* scale, float drop_p, const unsigned long long* seed,
                     unsigned long long site, float* pg, float* h1, float* prior, float* tt_vq, float* tt_ak,
                     float* tt_aq, float* tt_vk, float* tp_vq, float* tp_ak, float* tp_aq, float* tp_vk,
                     float* v2a_bias, float* a2v_bias, void* stream);

/* Its backward (xattn_head.prior_backward's ~20 launches), one workgroup per sample: from dbias_v2a [B][T][Ta] and
 * dbias_a2v [B][Ta][T], the token-half gradients dtt_* (layouts of tt_*), the prior-half gradients dtp_* [B], dprior
 * [B][PD], dh1 [B][H1] (through the ReLU / dropout mask of the saved h1), dscale_part [B] (this sample's sum of
 * dbias * tanh over both biases), and the token gradients ADDED into dv [B*T][d] / da [B*Ta][d] (token-bias Linears
 * + mean pools).  The weight gradients are products of these with the saved tensors (grouped wgrad problems). */
int mer_xh_prior_bwd(int B, int T, int Ta, int d, int H1, int PD, const float* dbias_v2a, const float* dbias_a2v,
                     const float* tt_vq, const float* tt_ak, const float* tt_aq, const float* tt_vk,
                     const float* tp_vq, const float* tp_ak, const float* tp_aq, const float* tp_vk,
                     const float* scale, const float* w_vq, const float* w_ak, const float* w_aq, const float* w_vk,
                     const float* W0, const float* W3, const float* h1, float drop_p, const unsigned long long* seed,
                     unsigned long long site, float* dtt_vq, float* dtt_ak, float* dtt_aq, float* dtt_vk,
                     float* dtp_vq, float* dtp_ak, float* dtp_aq, float* dtp_vk, float* dprior, float* dh1,
                     float* dscale_part, float* dv, float* da, void* stream);

/* F4: emb[b][128:256] = sum_tiles part / Ta (tile order), then the classifier: concat (gated = 0):
 * h = dropout(relu(emb W0^T + b0)) [B][H1], logits = h W3^T + b3; gated: h [B][H1 = 128], g = sigmoid(h W3^T + b3),
 * fused = g emb_v + (1 - g) emb_a (gsave [B], fsave [B][128]), logits = fused Wc^T + bc.  Exact fp32 FMA. */
int mer_xh_mlp_fwd(int B, int Ta, int gated, int H1, int C, const float* part, float* emb, const float* W0,
                   const float* b0, const float* W3, const float* b3, const float* Wc, const float* bc, float mlp_p,
                   const unsigned long long* seed, unsigned long long site, float* hsave, float* gsave, float* fsave,
                   float* logits, void* stream);

/* ---- fused xattn head backward (csrc/xattn_fused_bwd.hip; the unfused schedule is xattn_head.head_backward,
 * xattn_head.py:191-315).  W*T_hi / _lo are the TRANSPOSED split planes ([in][out]).  Gradient buffers are
 * accumulated into (+=); data gradients are written. ---- */

/* G4: the classifier head's data gradients (fusion.py:404-411 backward; concat: h W3 / gated: gate + classifier),
 * one workgroup per sample: dh [B][H1] (the gradient at the hidden pre-activation), dz [B] (gated: at the gate
 * logit) and demb [B][256].  The head's weight / bias gradients (dW0 = dh^T emb, dW3 = dl^T h; gated
 * dWg3 = dz^T h, dWc = dl^T fused) are problems of mer_xh_wgrad.  Exact fp32 FMA. */
int mer_xh_mlp_bwd(int B, int C, int H1, int gated, const float* dlogits, const float* emb, const float* h,
                   const float* g, const float* W0, const float* W3, const float* Wc, float mlp_p,
                   const unsigned long long* seed, unsigned long long site, float* dh, float* dz, float* demb,
                   void* stream);

/* G3 (one workgroup per (sample, 16 query rows)): a-pool + LayerNorm backward -> da (the residual part, [B*Ta][128])
 * and da2 = keep_b * ds; do2 = da2 Wo2; attention backward -> dq2 into dqkv[:, 0:128] ([B*Ta][384]), per-tile
 * dK2 dV2 partials dkv2_part [B][ceil(Ta/16)][16][256], LayerNorm dgamma / dbeta partials ln_part [B*tiles][256].
 * dbias (nullable): the prior bias gradient [B][Ta][T] = sum over heads of dS (head order). */
int mer_xh_a2v_bwd(int B, int T, int Ta, const float* demb, const float* s_a, const float* mean_a, const float* rstd_a,
                   const float* gamma, const float* P2, const float* kv2, const float* q2, const void* WoT2_hi,
                   const void* WoT2_lo, float attn_p, float path_p, const unsigned long long* seed,
                   unsigned long long site_attn, unsigned long long site_path, float scale, float* da, float* da2,
                   float* dqkv, float* dkv2_part, float* ln_part, float* dbias, void* stream);

/* G2 (two launches: one workgroup per sample, then the attention backward per (sample, head); T <= 16,
 * Ta <= 160): dkv2 = fold(dkv2_part) [B*T][256], dv1 = demb_v / T + dkv2 Wkv2, LayerNorm backward (dv2, ln_part
 * [B][256]), do1 = dv2 Wo1 ([B*T][128] scratch), attention backward -> dq1 [B*T][128], dK1 dV1 into
 * dqkv[:, 128:384], dv [B*T][128] = the LayerNorm-residual part of dv (G1 adds dq1 Wq1).  dbias (nullable): the
 * prior bias gradient [B][T][Ta] = sum over heads of dS (head order), through the dS_heads scratch [B][4][T][Ta]. */
int mer_xh_v2a_bwd(int B, int T, int Ta, const float* dkv2_part, const void* WkvT2_hi, const void* WkvT2_lo,
                   const float* demb, const float* s_v, const float* mean_v, const float* rstd_v, const float* gamma,
                   const void* WoT1_hi, const void* WoT1_lo, const float* P1, const float* kv1, const float* q1,
                   float attn_p, float path_p, const unsigned long long* seed, unsigned long long site_attn,
                   unsigned long long site_path, float scale, float* dkv2, float* dv2, float* dq1, float* dv,
                   float* dqkv, float* ln_part, float* do1, float* dS_heads, float* dbias, void* stream);

/* G1 (32 rows per workgroup): da += dqkv [Wq2 ; Wkv1] (in place), da_s = da Wa; the trailing ceil(Mv/32)
 * workgroups: dv += dq1 Wq1 (in place), dvfeat = dv Wv [Mv][vdim] (NULL: not wanted). */
int mer_xh_audio_bwd(int M, const float* dqkv, const void* WcT_hi, const void* WcT_lo, const void* WaT_hi,
                     const void* WaT_lo, float* da, float* da_s, int Mv, int vdim, const float* dq1,
                     const void* WqT1_hi, const void* WqT1_lo, const void* WvT_hi, const void* WvT_lo, float* dv,
                     float* dvfeat, void* stream);

/* Grouped weight gradients: host table [nprob <= 16][11] rows {dY, ldy, X, ldx, x_dtype, M, N, K, splits, dW, db}:
 * dW [N][K] += dY^T X and db [N] += column sums of dY (K = 0: column sums only).  Row splits write partials to ws
 * (mer_xh_wgrad_ws_floats floats), added in split order by a second launch -- deterministic, no atomics. */
int mer_xh_wgrad_ws_floats(int nprob, const long long* table, long long* out);
int mer_xh_wgrad(int nprob, const long long* table, float* ws, long long ws_floats, void* stream);

/* ============================ CLIP-style alignment (concat / gated, fusion_align_mode="clip") ============
 * ClipStyleAlignment.forward after its two projections (fusion.py:137-150): a_n / v_n = F.normalize rows,
 * logits = min(exp(logit_scale), 100) * a_n v_n^T, loss = (CE(logits, arange) + CE(logits^T, arange)) / 2.
 * a, v fp32 [B, D]; outputs an, vn [B, D], norms [2B] (max(|x|, 1e-12)), logits [B, B], loss [1]. */
int mer_clip_align_fwd(int B, int D, const float* a, const float* v, const float* log_scale, float* an, float* vn,
                       float* norms, float* logits, float* loss, void* stream);
/* Backward given the device scalar dloss: da, dv [B, D] (written), dlog_scale[0] += dL/dlogit_scale
 * (NULL: not wanted); ws = B*B floats of workspace. */
int mer_clip_align_bwd(int B, int D, const float* an, const float* vn, const float* norms, const float* logits,
                       const float* log_scale, const float* dloss, float* ws, float* da, float* dv, float* dlog_scale,
                       void* stream);
/* out[0] = x[0] + w * y[0] (device scalars): train.py:225 loss = cls_loss + fusion_align_weight * align_loss. */
int mer_add_scaled_scalar(const float* x, const float* y, float w, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MER_H_ */
