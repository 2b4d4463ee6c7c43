/*
 * dfk.h — C ABI of the DeepFake MI355X (gfx950) hot-path library libdfk.so.
 *
 * The reference (Polarisjame/DeepFake @ 2024_10_08) has no FFI: its hot path
 * is plain nn.Module code on stock PyTorch ops.  These entry points are the
 * native layer below the same nn.Module surface; each cites
 * the reference op(s) it replaces.  Conventions for every entry point:
 *   - plain device pointers + sizes; the caller owns every buffer (no
 *     allocation inside, no host synchronisation: graph-capturable);
 *   - work is enqueued on the given hipStream_t;
 *   - returns 0 on success, a hipError_t value on a launch error, or
 *     DFK_EINVAL (-1) when arguments violate the documented contract;
 *   - dtype: DFK_F32 (0) or DFK_BF16 (1) for activations / weights; all
 *     reductions and statistics are fp32.
 */
#ifndef DFK_H
#define DFK_H
#include <stdint.h>
#include <hip/hip_runtime.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DFK_F32 0
#define DFK_BF16 1
#define DFK_EINVAL (-1)
#define DFK_ENOTSUP (-2)   /* a size the entry point does not take (documented per entry point) */

/* Training-mode dropout / DropPath / LayerDrop masks, drawn by a counter-based hash inside the kernels
 * that apply them, so the backward regenerates the forward's mask and a captured HIP graph draws new
 * masks at every replay (the seed and step counter live in device memory; the step is advanced once per
 * training micro-step).  Replaces nn.Dropout / F.dropout (src/utils.py:253-258, HF modeling_wav2vec2.py
 * :434,:458,:568,:572,:604,:692), timm DropPath (video_swin_transformer.py:214,272,276;
 * swin_transformer2d.py:240,301,304) and the LayerDrop coin (HF :700-706).
 *   keep(draw) <=> uniform(draw) >= p; kept values are scaled by 1/(1-p).
 *   mode 1: one draw per element (row, col); mode 2: one draw per group of group_rows rows (DropPath: the
 *   tokens of one clip).  shared: draw from the rank-independent seed (LayerDrop flags, identical on every
 *   data-parallel rank) instead of the per-rank one.  rng == NULL or mode == 0: no dropout. */
typedef struct {
  const int64_t* rng;   /* device int64[4]: per-rank seed, step, shared seed, unused */
  int32_t mode;
  int32_t site;         /* distinct per dropout site of the model */
  float p;
  int32_t group_rows;
  int32_t shared;
} dfk_drop;

/* A 2-D operand view V(r, c), contiguous along c.
 *  plain: V(r,c) = ptr[r*ld + c]
 *  conv : V(r,c) = ptr[(r*conv_stride + c/conv_cg - conv_pad)*ld + c%conv_cg]   (0 outside [0,conv_rows))
 *         an implicit-GEMM view of a channels-last 1-D convolution input.
 * Batched launches index z = z0*nz1 + z1 and add z0*bs0 + z1*bs1 elements. */
typedef struct {
  const void* ptr;
  int64_t ld;
  int64_t bs0;
  int64_t bs1;
  int32_t conv_cg;      /* 0 = plain view */
  int32_t conv_stride;
  int32_t conv_pad;
  int32_t conv_rows;
} dfk_view;

/* C[i,j] (+)= sum_k A(i,k) B(k,j) with fused prologue/epilogue.
 *  A(i,k) = a_kmajor ? a.V(k,i) : a.V(i,k);   B(k,j) = b_kmajor ? b.V(k,j) : b.V(j,k)
 * Replaces every nn.Linear forward (y = x W^T + b) and its two backward GEMMs
 * (dx = dy W, dW = dy^T x), and the wav2vec2 Conv1d stack as implicit GEMM:
 *   video_swin_transformer.py:134,136 (qkv/proj), src/utils.py:249-251 (Mlp),
 *   :291 (PatchMerging.reduction), ModalFusion.py:16-25, HF modeling_wav2vec2.py
 *   :258-272 (conv1..6), :326-368 (pos-conv), :495-498,:556-561 (encoder linears).
 * Epilogue, in order: +bias[j]; act==1: aux<-v (if aux), v=gelu(v);
 *   act==2: v *= gelu'(aux[i,j]); v *= drop mask (row i + z*M, col j); v *= alpha (0 reads as 1);
 *   +residual[i,j]; act==3: v = relu(v) (Inception-ResNet blocks: relu(x + scale*conv(x_res)),
 *   InceptionResV2.py:95,117,164); then store
 *   (beta: v += beta*C_old) or fp32 atomicAdd (atomic=1, for split-K / batch-summed weight grads).
 * Contract: the contiguous extent and ld of each view are multiples of 8 (bf16) / 4 (f32). */
typedef struct {
  dfk_view a;
  dfk_view b;
  void* c;
  const void* bias;
  const void* residual;
  void* aux;
  int64_t ldc, cbs0, cbs1;
  int64_t ldr, rbs0, rbs1;
  int64_t ldaux;        /* aux shares C's batch strides (cbs0, cbs1) */
  int64_t bias_bs1;     /* bias offset per z1 (grouped convs) */
  int32_t M, N, K;
  int32_t dtype;        /* of A, B, bias, residual, aux (and C unless c_f32) */
  int32_t a_kmajor, b_kmajor;
  int32_t c_f32;
  int32_t nz0, nz1;
  int32_t splitk;
  int32_t act;
  int32_t atomic;
  float beta;
  void* ws;             /* fp32 split-K slabs, dfk_gemm_workspace(g) bytes (NULL: no automatic split) */
  float* rowsum;        /* optional, nz0 = nz1 = 1: rowsum[i] += sum_k A(i,k) (fp32) — the bias gradient
                           of a Linear when A = dy^T, computed by one extra MFMA against a ones operand */
  dfk_drop drop;        /* dropout / DropPath of the output before the residual add (bf16/f32 C only) */
  float alpha;          /* scale of the product (+bias) before the residual add; 0 = 1 */
  uint8_t* mx_q;        /* dfk_gemm_mx only (NULL elsewhere): also write the bf16 C, quantised along N, as an MX
                           operand (see dfk_mx_operand below; N % 128 == 0) — the next MX GEMM's input */
  uint32_t* mx_s;
  int64_t mx_ldq, mx_lds;
} dfk_gemm_args;
int dfk_gemm(const dfk_gemm_args* g, hipStream_t stream);
/* Bytes of scratch dfk_gemm wants in g->ws: grids too small to fill the chip (the
 * wav2vec2 / SwinV2-stage-3 Linears, M ~ 1.6k rows) are split along K into fp32
 * slabs that a second kernel sums before the epilogue.  0 = no split. */
int64_t dfk_gemm_workspace(const dfk_gemm_args* g);

/* ---- MX-fp8 (OCP microscaling) GEMM path of the C4 Swin-B video trunk (BASELINE configs[3]: "fp8 MFMA
 * attention/QKV path"): the qkv / proj / fc1 / fc2 Linears of video_swin_transformer.py:134-136 (WindowAttention3D)
 * and src/utils.py:249-251 (Mlp) — forward y = x W^T and input gradient dx = dy W — on the block-scaled
 * v_mfma_scale_f32_16x16x128_f8f6f4 (2x the bf16 MFMA rate).  The weight gradient stays bf16.
 * An MX operand holds a [rows][K] matrix, K contiguous: OCP e4m3 (e4m3fn) values q (row stride ld bytes) and one
 * E8M0 scale per 32 consecutive k; the four scales of k-tile t (k in [128t, 128t+128)) of row r are the bytes of
 * the dword s[t*lds + r] (byte j: k-block 4t + j).  Element value = e4m3(q) * 2^(scale - 127).  K % 128 == 0. */
typedef struct {
  const uint8_t* q;
  const uint32_t* s;
  int64_t ld;           /* bytes between rows of q (multiple of 16) */
  int64_t lds;          /* dwords between k-tiles of s (>= rows) */
} dfk_mx_operand;
/* Quantise x [rows][cols] (dtype bf16 or f32, row stride ldx elements) to an MX operand along cols (transpose = 0:
 * q [rows][cols], s [cols/128][lds = rows]; cols % 128 == 0), or x^T along rows (transpose = 1: q [cols][rows],
 * s [rows/128][lds = cols]; rows % 128 == 0) — the dx GEMM's weight operand W^T.  Per 32-element block: scale
 * exponent e = the smallest with amax / 2^e <= 448 (e4m3's largest finite value, so nothing saturates), values
 * x / 2^e rounded to nearest even (v_cvt_pk_fp8_f32); an all-zero block gets scale 2^0. */
int dfk_mx_quant(const void* x, int dtype, int64_t rows, int64_t cols, int64_t ldx, int transpose, uint8_t* q,
                 int64_t ldq, uint32_t* s, hipStream_t stream);
/* C [M][N] = A B^T (+ g's epilogue: bias / GELU with aux / dGELU / dropout / residual, bf16 output) with A [M][K]
 * and B [N][K] MX operands.  g supplies M, N, K and the epilogue fields only: dtype DFK_BF16, no split-K, no atomic,
 * no fp32 C, no rowsum, no batching; g->a / g->b are ignored.  K % 128 == 0. */
int dfk_gemm_mx(const dfk_gemm_args* g, const dfk_mx_operand* a, const dfk_mx_operand* b, hipStream_t stream);

/* out[j] (+)= sum_i x[i*ld + j] (fp32 atomics).  Linear bias gradients. */
int dfk_colsum(const void* x, int dtype, int64_t rows, int64_t cols, int64_t ld, float* out, hipStream_t stream);

/* LayerNorm over the last dim C of `rows` rows (nn.LayerNorm / F.layer_norm,
 * video_swin_transformer.py:209,215,292,548,678; HF :424,:586-588,:661).
 * y = (x-mean)*rstd*w + b; saves mean/rstd (fp32) for the backward.
 * Optional: y = residual + drop(LN(x)) — the SwinV2 post-norm residual x + DropPath(LN(a))
 * (swin_transformer2d.py:301,304) and LN -> dropout of the wav2vec2 encoder input (HF :691-692);
 * residual / drop may be NULL. */
int dfk_layernorm_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
                      int64_t rows, int32_t C, float eps, int dtype, const void* residual, const dfk_drop* drop,
                      hipStream_t stream);
/* dx = LN'(dy) (+ addend when addend != NULL, else + dx when accumulate); dw, db accumulate (+=); drop (may be
 * NULL): the forward's mask applied to dy first (the gradient of drop(LN(x))).  addend ([rows][C], dtype): the
 * gradient of a skip alias of x (the block's residual path), summed in the same pass without writing into the
 * caller's gradient buffer.  ws: fp32 scratch of
 * dfk_layernorm_bwd_workspace(rows, C) bytes for per-workgroup dw/db partials,
 * column-summed by a second pass; NULL: fp32 atomics per workgroup and channel
 * (same-address contention: slow when many workgroups share few channels). */
int dfk_layernorm_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                      void* dx, float* dw, float* db, int64_t rows, int32_t C, int accumulate, int dtype,
                      float* ws, const dfk_drop* drop, const void* addend, hipStream_t stream);
int64_t dfk_layernorm_bwd_workspace(int64_t rows, int32_t C);

/* Windowed multi-head attention core on token-major buffers (no window
 * partition / roll copies: both are index arithmetic inside the kernel).
 * Replaces WindowAttention3D.forward (video_swin_transformer.py:148-170) with
 * forward_part1's pad/roll/window_partition/window_reverse/roll/crop (:224-252),
 * and eager_attention_forward of wav2vec2 (HF :438-463) as a single window.
 *   q/k/v: element (b, d, h, w, head, e) at ptr[((b*D+d)*H+h)*W+w)*ld + head*hd + e]
 *   out  : same indexing with ld_out.
 *   window (wd,wh,ww) = clamped window; full_window = RPB decode geometry (Q3);
 *   shift along each dim (0 = none); positions padded up to the window grid
 *   read the qkv bias (`pad_q/k/v`, zero input after LN, :229) .
 *   rpb: [L, nH] fp32 table or NULL;  shifted-window 0/-100 mask (Q4) from
 *   arithmetic region labels, applied iff any shift > 0.  Alternatively an
 *   explicit additive mask [mask_nw, N, N] fp32 (WindowAttention3D.forward's
 *   `mask` argument, :160-163) indexed by (clip-window index) % mask_nw.
 *   scale multiplies q before q k^T (Q5).
 *   lse (fp32 [B*nW, nH, Np]) saved for the backward.
 *   tab: bf16 path only (NULL = table-free kernels): device scratch of
 *   dfk_wattn_table_workspace() bytes holding the per-(shift class, head)
 *   score-bias tables (RPB + shift mask, fp32, in MFMA accumulator order) that
 *   dfk_wattn_table builds from rpb; dfk_wattn_fwd and dfk_wattn_bwd read them,
 *   so both must get the buffer built with the same geometry and rpb. */
typedef struct {
  const void* q; const void* k; const void* v;
  void* out;
  const float* rpb;
  const void* pad_q; const void* pad_k; const void* pad_v;
  float* lse;
  const float* mask;
  int64_t mask_nw;
  int64_t ld_qkv, ld_out;
  int32_t B, D, H, W;
  int32_t wd, wh, ww;
  int32_t fd, fh, fw;
  int32_t sd, sh, sw;
  int32_t heads, hd;
  int32_t dtype;
  float scale;
  void* tab;
  dfk_drop drop;        /* attention-probability dropout (mode 1, bf16 table path only; row = query,
                           col = key of the (clip, window, head) unit): HF eager_attention_forward's
                           nn.functional.dropout(attn_weights, p=attention_dropout) (HF :458) */
} dfk_wattn_args;
int dfk_wattn_fwd(const dfk_wattn_args* a, hipStream_t stream);
/* kernel-selection policy of dfk_wattn_fwd's hd-32 table path (process-wide; tests and A/B runs only — the
 * defaults are the product's choice): version 6 = no-running-max forward on 16x16x32 tiles (default), 5 = the
 * same on 32x32x16 tiles, 4 = the max-subtracted forward; bal_min_units = smallest launch (units = clips x windows
 * x heads) that runs the key-split balanced schedule (default: 512 for version 5, never for version 6).  -1
 * leaves a setting unchanged, bal_min_units -2 restores its default.  Returns 0.  dfk_wattn_table builds its forward bias tiles in
 * the layout of the version in force, so a table must come from the same policy as the forward that reads it. */
int dfk_wattn_fwd_policy(int32_t version, int64_t bal_min_units);
/* backward policy (process-wide; tests and A/B runs only).  group: the bf16 table backward runs `group` windows of
 * one (shift class, head) per workgroup and sums their dS^T into one dRPB scratch slab (0 = automatic: enough
 * groups for about three rounds of one workgroup per CU, at most 8).  version: 4 = the two-pass kernel (dK/dV
 * pass with keys on the lane, dQ pass with queries on the lane; hd 32 windows of >= 4 query blocks, the default),
 * 3 = the staggered single-pass kernel everywhere, -1 leaves it.  dfk_wattn_bwd_workspace sizes for the setting
 * in force, so set it before asking for the workspace.  Returns 0, or DFK_EINVAL. */
int dfk_wattn_bwd_policy(int32_t group, int32_t version);
int64_t dfk_wattn_table_workspace(const dfk_wattn_args* a);
/* builds a->tab (fwd and bwd layouts) from a->rpb, the shift and the window geometry
 * (replaces the RPB gather + mask add of WindowAttention3D.forward, :152-163) */
int dfk_wattn_table(const dfk_wattn_args* a, hipStream_t stream);
/* backward: f is the forward's argument block (f.out = the forward output O,
 * f.lse its log-sum-exp).  dq/dk/dv are written (=) at the q/k/v layout with
 * row stride ld_dqkv; drpb [L,nH] fp32 (+=); gradients of padded positions
 * (which read the qkv bias in the forward) are summed into dpad_q/k/v
 * [heads*hd] fp32 (+=, may be NULL when the volume needs no padding).
 * ws: fp32 scratch of dfk_wattn_bwd_workspace(&f) bytes for the per-window
 * dRPB partials (reduced deterministically by a second kernel; NULL falls back
 * to device-scope atomics on the [L,nH] table, which contend heavily). */
typedef struct {
  dfk_wattn_args f;
  const void* dout;
  void* dq; void* dk; void* dv;
  float* drpb;
  float* dpad_q; float* dpad_k; float* dpad_v;
  int64_t ld_dqkv, ld_dout;
  float* ws;
  float* dscore;        /* NULL, or [heads] fp32 (+=): sum over rows and keys of dS * score (the score before
                           the bias, scale q.k) = the gradient of a per-head multiplier of the scores — SwinV2's
                           logit_scale (swin_transformer2d.py:155-157: attn = cos(q,k) * exp(logit_scale)), taken in
                           fp32 inside the backward with the exact softmax-backward row constant.  bf16 bias-table
                           path without dropout only (else DFK_EINVAL) */
} dfk_wattn_bwd_args;
int dfk_wattn_bwd(const dfk_wattn_bwd_args* a, hipStream_t stream);
int64_t dfk_wattn_bwd_workspace(const dfk_wattn_args* f);

/* Patch im2col for Conv3d/Conv2d with kernel == stride (PatchEmbed3D,
 * video_swin_transformer.py:436,446-453; SwinV2 PatchEmbed swin_transformer2d.py:461,477):
 * out[((b*Do+d)*Ho+h)*Wo+w][((c*pd+kd)*ph+kh)*pw+kw] = x[b,c,d*pd+kd,h*ph+kh,w*pw+kw]
 * (element strides sb..sw, so [B,T,C,H,W] clips need no permute; zero past T/H/W = F.pad). */
typedef struct {
  int64_t sb, sc, st, sh, sw;
  int32_t B, cin, T, H, W;
  int32_t pd, ph, pw;
  int32_t Do, Ho, Wo;
} dfk_im2col_args;
int dfk_patch_im2col(const void* x, int x_dtype, void* out, int out_dtype, const dfk_im2col_args* a,
                     hipStream_t stream);

/* Fused PatchEmbed3D (video_swin_transformer.py:420-460: pad + Conv3d(3->C, k = s = 2x4x4) + LayerNorm(C)),
 * bf16 compute, one pass over the clip.  x fp32 clip, element strides sb..sw (sw == 1, others multiples of 4:
 * [B,T,3,H,W] clips are read in place); w [C][96] bf16 (the Conv3d weight flattened), b, ln_w, ln_b [C] bf16;
 * C in {96, 128}.  fwd: out [B*Do*Ho*Wo][C] bf16 normalised tokens, mean/rstd [tokens] fp32 (LN statistics of
 * the fp32 conv output).  bwd (dy = d out, bf16): recomputes the conv from the clip and accumulates (+=, fp32)
 * dw [C][96], db, dln_w, dln_b [C]; no input gradient. */
typedef struct {
  const void* x;
  int64_t sb, sc, st, sh, sw;
  int32_t B, T, H, W, C;
  const void* w;
  const void* b;
  const void* ln_w;
  const void* ln_b;
  float eps;
  void* out;
  float* mean;
  float* rstd;
  float* dw;
  float* db;
  float* dln_w;
  float* dln_b;
} dfk_patch_embed_args;
int dfk_patch_embed_fwd(const dfk_patch_embed_args* a, hipStream_t stream);
int dfk_patch_embed_bwd(const dfk_patch_embed_args* a, const void* dy, hipStream_t stream);

/* PatchMerging 2x2 gather (reverse=0) / its gradient scatter (reverse=1) on
 * channels-last [B*D, H, W, C] <-> [B*D*ceil(H/2)*ceil(W/2), 4C], order x0,x1,x2,x3 (Q7),
 * zero padding of odd H/W (video_swin_transformer.py:300-311). */
int dfk_patch_merge(const void* src, void* dst, int B, int D, int H, int W, int C, int reverse, int dtype,
                    hipStream_t stream);

/* out[g][c] = mean_r x[g*R+r][c]: per-clip token means (VST mean(dim=[2,3,4]) Q8,
 * Audio2D AdaptiveAvgPool audioTransformer.py:13,23, SwinV2 avgpool swin_transformer2d.py:614). */
int dfk_rowmean(const void* x, void* out, int groups, int R, int C, int dtype, int out_f32, hipStream_t stream);

int dfk_cast(const void* x, int x_dtype, void* y, int y_dtype, int64_t n, hipStream_t stream);

/* wav2vec2 feature-encoder layer 0 (HF modeling_wav2vec2.py:302-323,
 * Wav2Vec2GroupNormConvLayer): Conv1d(1->512,k10,s5,no bias) -> GroupNorm(512,512)
 * (per clip and channel over all T0=(S-10)/5+1 frames) -> GELU, output
 * channels-last [B, T0, 512] (dtype).  wave [B,S] fp32, w [512,10], gamma/beta
 * [512] fp32; stats [B,512,2] fp32 (sum, sumsq of the conv output) saved for
 * the backward.  The conv output is recomputed, never stored. */
int dfk_w2v_conv0_fwd(const float* wave, int64_t B, int64_t S, const float* w, const float* gamma,
                      const float* beta, float eps, float* stats, void* out, int dtype, float* ws, hipStream_t stream);
/* ws: fp32 scratch of dfk_w2v_conv0_fwd_workspace(B, S) bytes for the per-time-block GroupNorm partial sums,
 * summed into stats in a fixed order (the forward is bitwise reproducible: no atomics). */
int64_t dfk_w2v_conv0_fwd_workspace(int64_t B, int64_t S);
/* backward: dw [512,10], dgamma, dbeta fp32 (+=); scratch: fp32 buffer of scratch_bytes >=
 * dfk_w2v_conv0_bwd_workspace(B, S) bytes (the [B,512,2] GroupNorm reductions, then per-workgroup dw partials
 * summed without atomics); a smaller buffer returns DFK_EINVAL. */
int64_t dfk_w2v_conv0_bwd_workspace(int64_t B, int64_t S);
int dfk_w2v_conv0_bwd(const float* wave, int64_t B, int64_t S, const float* w, const float* gamma,
                      const float* beta, float eps, const float* stats, const void* dout, int dtype,
                      float* scratch, int64_t scratch_bytes, float* dw, float* dgamma, float* dbeta,
                      hipStream_t stream);

/* SwinV2 cosine-attention prologue (swin_transformer2d.py:154-157) on a [rows, 3C]
 * qkv buffer: q' = normalize(q)*scale[h], k' = normalize(k), v' = v, so the window
 * attention kernel then runs with scale 1; scale[h] = exp(min(logit_scale[h], max_log))
 * (torch.clamp(logit_scale, max=log(1/0.01)).exp(), :156) from the fp32 parameter itself.
 * The backward writes dqkv and accumulates the logit_scale gradient dlogit_scale[h] (fp32 +=). */
int dfk_cosine_qk_fwd(const void* qkv, void* out, const float* logit_scale, float max_log, int64_t rows, int heads,
                      int hd, int dtype, hipStream_t stream);
/* dscore: NULL (the logit_scale gradient from q-hat . dq' here), or the [heads] fp32 sum of dS * score that
 * dfk_wattn_bwd accumulated (dfk_wattn_bwd_args.dscore): then dlogit_scale[h] += dscore[h] where logit_scale[h]
 * <= max_log, and dscore is set back to zero for the next step. */
int dfk_cosine_qk_bwd(const void* qkv, const void* dout, void* dqkv, const float* logit_scale, float max_log,
                      float* dlogit_scale, int64_t rows, int heads, int hd, int dtype, float* dscore,
                      hipStream_t stream);

/* SwinV2 continuous position bias (swin_transformer2d.py:99-100,159-162): out[l][h] =
 * 16 * sigmoid(sum_j W2[h][j] * relu(W1[j][0]*c[l][0] + W1[j][1]*c[l][1] + b1[j])) for the L = (2Wh-1)(2Ww-1)
 * relative coordinates c (relative_coords_table), cpb_mlp = Linear(2,hidden) -> ReLU -> Linear(hidden,heads,no
 * bias); all fp32 (the parameters' own dtype).  bwd: dout [L, heads] -> dW1 [hidden,2], db1 [hidden],
 * dW2 [heads,hidden] (fp32 +=), recomputing the hidden layer. */
int dfk_cpb_bias_fwd(const float* coords, const float* w1, const float* b1, const float* w2, float* out, int32_t L,
                     int32_t hidden, int32_t heads, hipStream_t stream);
int dfk_cpb_bias_bwd(const float* coords, const float* w1, const float* b1, const float* w2, const float* out,
                     const float* dout, float* dw1, float* db1, float* dw2, int32_t L, int32_t hidden, int32_t heads,
                     hipStream_t stream);
/* every SwinV2 block's table in one launch each way (the 24 blocks of SwinV2-B: 48 launches -> 2).  desc: DEVICE
 * array of n records of 12 int64 {coords, w1, b1, w2, dw1, db1, dw2 (device pointers; the gradients are
 * accumulated with fp32 atomics), off (float offset of the block's [L, heads] table in out / dout), L, hidden,
 * heads (<= 32), 0}; max_L >= every record's L.  Same arithmetic per table as dfk_cpb_bias_fwd / _bwd. */
int dfk_cpb_bias_fwd_many(const int64_t* desc, int32_t n, int32_t max_L, float* out, hipStream_t stream);
int dfk_cpb_bias_bwd_many(const int64_t* desc, int32_t n, int32_t max_L, const float* out, const float* dout,
                          hipStream_t stream);

/* dx = dy * gelu'(pre) (exact-erf GELU backward, torch nn.GELU / HF ACT2FN["gelu"]). */
int dfk_gelu_bwd(const void* dy, const void* pre, void* dx, int64_t n, int dtype, hipStream_t stream);

/* wav2vec2 positional-conv weight norm, HF weight_norm(conv, dim=2) (transformers modeling_wav2vec2.py:336-350;
 * replaces its g * v / ||v|| parametrization): v [C][Cg][k] fp32 (weight_v), g [k] fp32 (weight_g).
 * fwd: norm[k] = ||v[:, :, k]||; w = g v / norm written as the two operands of the grouped conv's implicit GEMMs
 * (dtype DFK_BF16 / DFK_F32): w2 [C][k*Cg], w2[o][kk*Cg+i] = w[o][i][kk] (forward), and w3 [C][k*Cg],
 * w3[gr*Cg+ci][u*Cg+co] = w[gr*Cg+co][ci][k-1-u] (the transposed conv of the input gradient).
 * bwd: from dw2 [C][k*Cg] fp32 (the weight-gradient GEMM's output in w2's layout), dg += (dw . v) / norm and
 * dv += g / norm dw - g (dw . v) / norm^3 v.  ws: C*k floats; Cg*k*4 bytes <= 64 KB; fixed summation order. */
int dfk_posconv_wnorm_fwd(const float* v, const float* g, int32_t C, int32_t Cg, int32_t k, float* norm, float* ws,
                          void* w2, void* w3, int dtype, hipStream_t stream);
int dfk_posconv_wnorm_bwd(const float* v, const float* g, const float* norm, const float* dw2, int32_t C, int32_t Cg,
                          int32_t k, float* ws, float* dv, float* dg, hipStream_t stream);

/* torch.optim.SGD(momentum, weight_decay) step over a flat fp32 parameter
 * buffer (src/trainer.py:80-84,295), optionally writing the bf16 compute
 * shadow of the updated parameters in the same pass; lr read from device
 * memory when lr_dev != NULL (graph-replay safe CosineAnnealingLR). */
int dfk_sgd_step(float* param, const float* grad, float* momentum_buf, void* bf16_shadow, int64_t n,
                 const float* lr_dev, float lr, float momentum, float weight_decay, int first_step,
                 const float* gate, float grad_scale, const void* grad_bf16, hipStream_t stream);
/* Every run of one optimizer step in one launch (replaces the per-run dfk_sgd_step loop of optim.FusedSGD.step;
 * same arithmetic per element).  runs: HOST int64 [nruns][4] = {start element, n, gate device pointer (0: none),
 * first_step}, copied into the launch's arguments (so a captured graph holds no table pointer); nruns <= 64
 * (DFK_ENOTSUP beyond that: the caller loops dfk_sgd_step).  Run starts are multiples of 4 elements (param / grad /
 * momentum 16-B, grad_bf16 / shadow 8-B aligned). */
int dfk_sgd_step_runs(float* param, const float* grad, float* momentum_buf, void* bf16_shadow, const int64_t* runs,
                      int32_t nruns, const float* lr_dev, float lr, float momentum, float weight_decay,
                      float grad_scale, const void* grad_bf16, hipStream_t stream);
/* gate (above; may be NULL): device flag, the step is skipped when *gate == 0 — the parameters of a
 * LayerDrop-skipped wav2vec2 layer have grad None in the reference and torch's SGD leaves them (and
 * their momentum) untouched.
 * grad_scale multiplies the gradient read (1 / world: the data-parallel mean of the all-reduced sum,
 * DataParallel's averaging of src/trainer.py:74-75 folded into the step); grad_bf16 (NULL, or 8-B aligned):
 * read the gradient from this bf16 buffer (the all-reduced bf16 bucket copy) instead of `grad`. */

/* y = x * mask / (1 - p) over [rows, cols] (row stride ld; y may alias x): nn.Dropout / DropPath as a
 * standalone pass, and the backward of every fused dropout site (the same mask applied to the gradient). */
int dfk_dropout(const void* x, void* y, int64_t rows, int32_t cols, int64_t ld, const dfk_drop* drop, int dtype,
                hipStream_t stream);
/* out[i] = keep(draw i) ? 1 : 0 for i < n (fp32): the per-layer LayerDrop coins of the wav2vec2 encoder
 * (HF :700-706: skip layer when rand < layerdrop), drawn on the device so a replayed graph re-draws them. */
int dfk_bernoulli_flags(const dfk_drop* drop, int32_t n, float* out, hipStream_t stream);
/* The same coins for one micro-step of an accumulation window: keep[i] = coin i, and used[i] = max(used[i],
 * keep[i]) — the SGD gate of layer i is the OR of its coins over the window (the caller zeroes `used` with the
 * gradients): torch's SGD steps a parameter whose accumulated .grad is not None, i.e. whose layer ran in ANY
 * micro-step of the window (src/trainer.py:280-297 with HF :700-706). */
int dfk_layerdrop_flags(const dfk_drop* drop, int32_t n, float* keep, float* used, hipStream_t stream);
/* LayerDrop output select (HF wav2vec2 encoder :700-706, the skipped layer returns its input):
 * forward (out2 == NULL): out = *keep > 0 ? y : x; backward (x == NULL, y = the output gradient):
 * out = *keep > 0 ? y : 0 (the layer's), out2 = *keep > 0 ? 0 : y (the skip path's).  nbytes % 16 == 0,
 * 16-B aligned buffers. */
int dfk_layer_select(const void* y, const void* x, const float* keep, void* out, void* out2, int64_t nbytes,
                     hipStream_t stream);
/* SpecAugment time masking (HF Wav2Vec2Model._mask_hidden_states :1272-1317 with _compute_mask_indices
 * :101-218, no attention mask): per clip, num = max(min_masks, int(mask_prob*T/mask_length + eps)) (eps one
 * uniform draw per call, num clamped as HF does) distinct span starts drawn uniformly from [0, T-mask_length],
 * frames [start, start+mask_length) masked; out = h with masked frames replaced by embed [C].  mask [B,T] uint8
 * is written for the backward.  bwd: dx = dy with masked frames zeroed, dembed [C] fp32 += sum of their dy. */
int dfk_spec_augment_fwd(const void* h, void* out, uint8_t* mask, const void* embed, int32_t B, int32_t T,
                         int32_t C, float mask_prob, int32_t mask_length, int32_t min_masks, const dfk_drop* drop,
                         int dtype, hipStream_t stream);
int dfk_spec_augment_bwd(const void* dy, void* dx, const uint8_t* mask, float* dembed, int32_t B, int32_t T,
                         int32_t C, int dtype, hipStream_t stream);

/* Frame normalisation on the device: T.ToTensor() + T.Normalize(mean, std) of
 * data/data_process.py:55-69 on decoded RGB frames (src/utils.py:22-39): src uint8 [frames, H, W, 3]
 * -> dst fp32 [frames, 3, H, W], (x/255 - mean[c]) / std[c] in fp32 (bit-exact to torchvision).
 * mean3 / std3 are HOST arrays of 3 floats.  Requires H*W % 4 == 0, dst 16-B aligned. */
int dfk_frame_normalize(const uint8_t* src, float* dst, int64_t frames, int32_t H, int32_t W, const float* mean3,
                        const float* std3, hipStream_t stream);
/* Waveform normalisation on the device: Wav2Vec2FeatureExtractor zero_mean_unit_var_norm
 * (transformers feature_extraction_wav2vec2.py:94-95, called at src/trainer.py:258) of every row of a
 * zero-padded [B, S] batch (no attention mask, Q13): y = (x - mean) / sqrt(var + eps), eps = 1e-7. */
int dfk_wave_normalize(const float* x, float* y, int64_t B, int64_t S, float eps, hipStream_t stream);

/* ---- media front end on the device (csrc/media.hip) ----
 * Mel-spectrogram image of generate_mel_spectrogram (src/utils.py:63-87): librosa.feature.melspectrogram(y, sr,
 * n_mels) with its defaults (periodic Hann window of n_fft, hop, center=True zero padding, power 2) ->
 * power_to_db(ref=max, amin 1e-10, top_db 80) -> cv2.normalize(NORM_MINMAX, 0, 255) -> uint8 (truncation) ->
 * cv2.resize(out_w x out_h, INTER_LINEAR, uint8 fixed point).  wave fp32 [B, S] at the filterbank's sample rate
 * (S % 4 == 0 for the vector path); basis fp32 [n_fft][ld] with ld = 2*(n_fft/2+1) rounded up to 4: the
 * window-folded cos | -sin DFT basis; fbank fp32 [n_mels][n_fft/2+1] (Slaney); ws of dfk_mel_workspace bytes;
 * out uint8 [B, out_h, out_w].  The STFT runs on dfk_gemm (fp32 MFMA). */
int64_t dfk_mel_workspace(int64_t B, int64_t S, int32_t n_fft, int32_t hop, int32_t n_mels);
int dfk_mel_image(const float* wave, int64_t B, int64_t S, const float* basis, const float* fbank, int32_t n_fft,
                  int32_t hop, int32_t n_mels, int32_t out_h, int32_t out_w, void* ws, int64_t ws_bytes, uint8_t* out,
                  hipStream_t stream);
/* Gray uint8 [n, H, W] -> fp32 [n, 3, H, W]: Image.convert('RGB') + T.ToTensor() + T.Normalize(mean, std)
 * (data_process.py:55-69,162); mean3 / std3 are HOST arrays of 3 floats. */
int dfk_gray_normalize(const uint8_t* src, float* dst, int64_t n_img, int32_t H, int32_t W, const float* mean3,
                       const float* std3, hipStream_t stream);
/* Frame transform of data_process.py:55-69 as the reference runs it — torchvision transforms on PIL images
 * (src/utils.py:32-33 Image.fromarray; the mel JPEG at :162 through the same transform):
 *   T.Resize -> PIL Image.resize(BILINEAR): separable, width pass then height pass, each into uint8 — a triangle
 *     filter whose support scales with the downscale factor (antialiased), per-output-pixel coefficients in PIL's
 *     22-bit fixed point (bounds [out][2] = first source index, tap count; coefficients [out][k]), built on the host
 *     by deepfake_amd.media.pil_bilinear_coeffs exactly as PIL's precompute_coeffs / normalize_coeffs_8bpc;
 *   T.RandomHorizontalFlip (flips[f] bit 0), T.RandomVerticalFlip (bit 1): Image.transpose;
 *   T.RandomRotation -> Image.rotate(angle, NEAREST, fill 0): affine[f] = 8 int32 {on, a0, a1, a2, a3, a4, a5, 0},
 *     PIL affine_fixed's 16.16 inverse map (source x = (a2 + x a0 + y a1) >> 16, y = (a5 + x a3 + y a4) >> 16) of
 *     the matrix PIL builds (media.pil_rotate_fixed); on = 0: no rotation;
 *   T.ToTensor + T.Normalize.
 * src uint8 [frames][H][W][cin] (cin 3: decoded RGB; cin 1: a grey image converted to RGB); tmp uint8 scratch of
 * frames*H*out_w*cin bytes (the width pass); dst fp32 [frames][3][out_h][out_w].  flips / affine: DEVICE arrays
 * (NULL: none); mean3 / std3: HOST arrays of 3 floats. */
typedef struct {
  int32_t H, W, cin;
  int32_t out_h, out_w;
  const int32_t* xb; const int32_t* xk; int32_t kx;
  const int32_t* yb; const int32_t* yk; int32_t ky;
} dfk_pil_resize;
int dfk_frame_augment(const uint8_t* src, int64_t frames, const dfk_pil_resize* rs, const int32_t* flips,
                      const int32_t* affine, const float* mean3, const float* std3, uint8_t* tmp, float* dst,
                      hipStream_t stream);

/* ---- 2-D convolution family of the Inception-ResNet-v2 video branch (SURVEY.md §8f f4:
 * src/models/InceptionResV2.py:6-190, IResNet.py:331-393).  Activations are channels-last [N*H*W, C] rows with
 * a row stride ld (>= C), so a branch reads / writes a channel slice of a torch.cat buffer in place. */
typedef struct {
  int32_t N, H, W, C;       /* input */
  int32_t kh, kw, sh, sw, ph, pw;
  int32_t Ho, Wo;           /* output */
} dfk_conv2d_geo;
/* im2col of nn.Conv2d (InceptionResV2.py:9): out [N*Ho*Wo][(ky*kw + kx)*C + c] (zero padding); the conv is
 * then the GEMM out . W'^T with W' = weight.permute(0,2,3,1) [Cout][kh*kw*C].  col2im2d: the input gradient
 * dx (=, or += when accumulate) from dcols of the same layout (a gather: no atomics). */
int dfk_im2col2d(const void* x, int64_t ldx, void* out, const dfk_conv2d_geo* g, int dtype, hipStream_t stream);
int dfk_col2im2d(const void* dcols, void* dx, int64_t ldx, const dfk_conv2d_geo* g, int accumulate, int dtype,
                 hipStream_t stream);
/* BatchNorm2d in training mode (+ the ReLU of the reference's Conv2d block, InceptionResV2.py:10-15): batch
 * statistics per channel over all rows (fp32), running_mean / running_var updated with momentum (unbiased
 * variance; may both be NULL); mean / rstd [C] saved for the backward; ws [2C] fp32 scratch.
 * bn2d_apply: y = (x - mean) * rstd * gamma + beta (+ReLU) from given statistics (eval mode: the running ones). */
int dfk_bn2d_fwd(const void* x, int64_t ldx, void* y, int64_t ldy, int64_t rows, int32_t C, const float* gamma,
                 const float* beta, float eps, float momentum, int relu, float* mean, float* rstd,
                 float* running_mean, float* running_var, float* ws, int dtype, hipStream_t stream);
int dfk_bn2d_apply(const void* x, int64_t ldx, void* y, int64_t ldy, int64_t rows, int32_t C, const float* mean,
                   const float* rstd, const float* gamma, const float* beta, int relu, int dtype, hipStream_t stream);
/* backward of y = relu?(BN(x)): dx (=), dgamma / dbeta (fp32 +=, may be NULL); y is read for the ReLU mask. */
int dfk_bn2d_bwd(const void* dy, int64_t lddy, const void* y, int64_t ldy, const void* x, int64_t ldx, void* dx,
                 int64_t lddx, int64_t rows, int32_t C, const float* mean, const float* rstd, const float* gamma,
                 int relu, float* dgamma, float* dbeta, float* ws, int dtype, hipStream_t stream);
/* MaxPool2d(k, s, p) (mode 0; backward routes to the first maximum of each window, as torch) and AvgPool2d(k, s, p,
 * count_include_pad=False) (mode 1): InceptionResV2.py:27,43,47,61,122.  bwd: dx (=, or += when accumulate). */
int dfk_pool2d_fwd(const void* x, int64_t ldx, void* y, int64_t ldy, const dfk_conv2d_geo* g, int mode, int dtype,
                   hipStream_t stream);
int dfk_pool2d_bwd(const void* x, int64_t ldx, const void* dy, int64_t lddy, void* dx, int64_t lddx,
                   const dfk_conv2d_geo* g, int mode, int accumulate, int dtype, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif
