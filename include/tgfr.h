/* tgfr.h -- C ABI of libtgfr_hip.so, the MI355X (gfx950) kernels of the TGFR
 * FCAM/FCFM training hot path.
 *
 * The reference (Mahedi-61/Text_Guided_Face_Recognition) is pure Python with
 * no FFI layer; its boundary for this path is the Python call surface of
 * models/losses.py, models/attention.py and models/fusion_nets.py.  Each entry
 * point below replaces the arithmetic behind one of those calls (cited per
 * function).  The Python mirror in text_guided_face_recognition_amd/models
 * keeps the reference signatures and binds these with ctypes
 * (text_guided_face_recognition_amd/_hip.py).
 *
 * Conventions
 *   - All pointers are device pointers owned by the caller; all buffers and
 *     workspaces are allocated by the caller.  Strides are in elements.
 *   - `stream` is a hipStream_t passed as void*; every call only enqueues
 *     work on it (no host synchronisation, no allocation) so calls can be
 *     captured into a HIP graph.
 *   - Return 0 on success, a hipError_t from the launch, or
 *     1001 (bad shape/argument) / 1002 (bad precision mode).
 *   - mode: 0 = bf16 MFMA operands, 1 = fp32 operands carried as bf16 hi/lo
 *     pairs (three MFMAs per product; the fp32-parity mode); the word-region
 *     entry points (tgfr_wr_fwd / tgfr_wr_bwd, general kernels) also take
 *     2 = fp16 operands (v_mfma_f32_32x32x16_f16, fp32 accumulation;
 *     BASELINE config 5's precision), with operands from tgfr_prep_rows_f16.
 *   - bf16 buffers are uint16_t bit patterns.
 *   - Feature dim D is 256 (aux_feat_dim_per_granularity, cfg/train_bert.yml:28);
 *     regions R = 196 (14x14, padded to 224 in the split images); words per
 *     caption T <= t_pad, t_pad = 32 or 64 (64-token captions, T = 62): the
 *     token stride of every words / stats / C / token-table buffer.  t_pad =
 *     64 (modes 0 / 2): two waves per caption; bounded = 1 drops the running
 *     max both ways (scores bounded as below; Rnorm unused).
 *   - ABI 600: the max-free t_pad-32 kernels (pipelined forward, two-role
 *     backward) run in mode 2 as well as mode 0; in mode 2 the forward
 *     stores C-hat scaled by 2^-8 and the token-table calls take bounded = 2.
 *   - ABI 610: tgfr_imim_dw_ln; tgfr_ln_tail_bwd / _att accept dlnw = dlnb =
 *     NULL (the LayerNorm's dw / db partials stay in ws for it).
 *   - ABI 620: tgfr_ln_tail_bwd_att keeps dZ in bf16 (half the scratch).
 */
#ifndef TGFR_H
#define TGFR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version (major*100 + minor). */
int tgfr_version(void);

/* fp32 rows (element (item,row,col) at x[item*s_item + row*s_row + col*s_col])
 * -> bf16 hi/lo of scale*x [n_items][rows_pad][256] with rows >=
 * min(n_rows, lens[item]) zeroed, plus optional fp32 L2 norms of the unscaled
 * rows [n_items][rows_pad].  Feeds the word<->region kernels with R (image
 * regions, models/models.py:401-404) and W (words, models/models.py:231). */
int tgfr_prep_rows(const float* x, long long s_item, long long s_row, long long s_col,
                   int n_items, int n_rows, int n_cols, int rows_pad, const int* lens,
                   float scale, uint16_t* hi, uint16_t* lo, float* norms, void* stream);
/* tgfr_prep_rows for the fp16 operand mode (mode 2 of tgfr_wr_fwd / _bwd):
 * hi receives fp16 bits of scale * x (no lo plane). */
int tgfr_prep_rows_f16(const float* x, long long s_item, long long s_row, long long s_col,
                       int n_items, int n_rows, int n_cols, int rows_pad, const int* lens,
                       float scale, uint16_t* hi, float* norms, void* stream);

/* Forward of words_loss's similarity matrix for all (image b, caption i) pairs:
 * replaces the per-caption loop of models/losses.py:73-122 together with
 * func_attention (models/attention.py:10-43):
 *   logits[b*ld + i] = gamma3 * log sum_{t<lens[i]} exp(gamma2 * cos_t)
 * Also writes per-token stats [B_img][B_cap][32] float4 {Z_t, n_t, |C_t|, cos_t}
 * and the weighted context C (attention.py:41) as bf16 hi (Chi) and, in
 * mode 1, lo (Clo) in chunk-major order [pair][32 chunks of 8 d][32 t][8],
 * for the backward; att (nullable) receives A2 [b][t][196] for the matching
 * pair i == b + img_offset (the att_maps of losses.py:97).  Wnorm: |W_t|
 * [B_cap][32].  Mode 0 keeps the image's R resident in LDS (Rlo/Wlo unused, may
 * be NULL) and takes the words scaled by log2(e) (Whi = bf16(log2(e) W),
 * tgfr_prep_rows scale).  bounded = 1 (with Rnorm = |R_r| [B_img][224]) lets
 * the mode-0 / mode-2 forward run without a running max (mode 2: fp16
 * operands, words scaled as in mode 0, C-hat stored x 2^-8).  t_pad 32 (with Sp): the
 * max-free pipelined kernel, exact for ANY input -- each caption whose
 * score bound max|W| max|R| exceeds 84.5 takes its running-max variant on
 * the device (the unit-norm BERT-path features have ~1) -- which also
 * writes the scores S' = log2(e) R.W of every (pair, 32-region tile) for the
 * backward into Sp (uint16 [B_img][B_cap][7][1088]: per record 64 lanes x 16
 * fp16 scores in MFMA accumulator order, then 32 fp32 region maxima; a
 * caption past the bound stores S' - max and the maxima); Sp NULL runs the
 * exact-max kernel instead.
 * t_pad 64: exact while the bound is <= 85.9 (unshifted up to 84.5, shifted
 * by the bound beyond).  For inputs not known to be unit rows pass a guard
 * (tgfr_wr_guard, below; NULL: none): the max-free kernel and its exact
 * running-max twin are then both launched and the guard picks one on the
 * device.  Otherwise the exact-max kernel runs.  C is stored unnormalised
 * (C-hat = Z C); tgfr_wr_bwd_tok folds the 1/Z back in. */
int tgfr_wr_fwd(const uint16_t* Rhi, const uint16_t* Rlo, const uint16_t* Whi,
                const uint16_t* Wlo, const float* Wnorm, const float* Rnorm, const int* lens,
                int B_img, int B_cap,
                int img_offset, float gamma1, float gamma2, float gamma3, float eps,
                float* logits, int ld_logits, float* stats, uint16_t* Chi, uint16_t* Clo,
                uint16_t* Sp, float* att, int att_T, int bounded, int t_pad, int mode,
                const int* guard, void* stream);

/* Device-side choice of the 64-token bounded path (ABI 510):
 * *guard = !(max Wnorm[0..n_w) * max Rnorm[0..n_r) <= 85.9), one 1024-thread
 * workgroup.  With the guard, tgfr_wr_fwd / tgfr_wr_bwd_tok(_ce) /
 * tgfr_wr_bwd (bounded = 1, t_pad 64, modes 0 / 2) launch the max-free
 * kernels and their exact twins, each exiting at once unless the guard
 * selects it -- so a call captured into a HIP graph stays exact for any
 * input, as the reference's softmaxes (models/attention.py:28-36) are, with
 * no host read.  Replaces the host-side norm check of round 4. */
int tgfr_wr_guard(const float* Wnorm, int n_w, const float* Rnorm, int n_r, int* guard,
                  void* stream);

/* Backward of tgfr_wr_fwd w.r.t. the image regions given dL/dlogits, in two
 * calls.  tgfr_wr_bwd_tok: per-(pair, token) scalars from the forward stats
 * and dlogits into tok_ws (B_img*B_cap*t_pad*8 floats).  tgfr_wr_bwd: the
 * fused recompute + both softmax backwards + dR GEMM, writing
 * dR[b][r][d] (r < 196) at dR[b*s_b + r*s_r + d*s_d] -- overwritten, not
 * accumulated.  ws: tgfr_wr_bwd_ws floats of workspace: caption-chunk partial
 * slabs, added in chunk order into dR by a reduction launch inside the call.
 * Rnorm (bounded only; the forward's |R_r| [B_img][224]): the pair's score
 * bound c = max|W| max|R| is formed again here, giving the same per-caption
 * variant (t_pad 32) / score shift (t_pad 64) as the forward's.
 * The text side is detached in the reference (utils/dataset_utils.py:42).
 * bounded = 1 (modes 0 / 2 with t_pad 32 after a bounded forward, or modes
 * 0 / 2 with t_pad 64; scores bounded as for tgfr_wr_fwd): both calls must
 * pass it -- tgfr_wr_bwd_tok(_ce) as 2 in mode 2 with t_pad 32 (its table
 * then folds the forward's 2^-8 C-hat scale back in) -- Whi is the forward's log2(e)-scaled words, and the max-free kernels
 * run (t_pad 32: the two-role one, wr_bwd_duo_kernel, which reads the
 * forward's stored scores Sp instead of recomputing them -- required then;
 * NULL otherwise).  guard: the forward's (tgfr_wr_guard; NULL: none); with
 * it tgfr_wr_bwd also takes Wplain, the plain (unscaled) word rows of the
 * exact twin (tgfr_prep_rows with scale 1). */
int tgfr_wr_bwd_tok(const float* stats, const float* Wnorm, const float* Rnorm, const int* lens,
                    int B_img, int B_cap, float gamma1, float gamma2, float gamma3, float eps,
                    const float* dlogits, int ld, int bounded, int t_pad, float* tok_ws,
                    const int* guard, void* stream);
/* tgfr_wr_bwd_tok with the contrastive CE's gradient formed in the same
 * launch instead of read from dlogits (tgfr_ce_grad's formula: logits [B_img]
 * [ld] from tgfr_wr_fwd, row_lse / col_lse from tgfr_ce_stats, row_offset,
 * inv_n = 1 / n_global, upstream gradients g0 / g1 (device scalars, nullable:
 * 1) weighted by w0 / w1 (0: that loss has no gradient)); kernels.WordRegionCE,
 * one launch fewer per step. */
int tgfr_wr_bwd_tok_ce(const float* stats, const float* Wnorm, const float* Rnorm,
                       const int* lens, int B_img, int B_cap, float gamma1, float gamma2,
                       float gamma3, float eps, const float* logits, int ld, int row_offset,
                       float inv_n, const float* row_lse, const float* col_lse, const float* g0,
                       const float* g1, float w0, float w1, int bounded, int t_pad,
                       float* tok_ws, const int* guard, void* stream);
int tgfr_wr_bwd_ws(int B_img, int B_cap, int bounded, int t_pad, int mode, long long* floats);
int tgfr_wr_bwd(const uint16_t* Rhi, const uint16_t* Rlo, const uint16_t* Whi,
                const uint16_t* Wlo, int B_img, int B_cap, float gamma1, const float* tok_ws,
                const uint16_t* Chi, const uint16_t* Clo, const uint16_t* Sp, float* dR,
                long long s_b, long long s_r, long long s_d, float* ws, int bounded, int t_pad,
                int mode, const uint16_t* Wplain, const int* guard, void* stream);

/* Verification pair scores (utils/modules.py:152-153): out[i] = x_i.y_i /
 * max(|x_i| |y_i|, eps) for matched rows of x [rows][d] (ldx) and y (ldy). */
int tgfr_pair_cosine(const float* x, long long ldx, const float* y, long long ldy, int rows,
                     int d, float eps, float* out, void* stream);

/* Standalone func_attention (models/attention.py:10-43), exact fp32, one
 * workgroup per sample (R = ih*iw <= 256, T <= 64, D <= 256):
 *   S = ctx^T q, A1 = softmax_T(S), A2 = softmax_R(gamma1 A1^T), C = ctx A2^T.
 * query element (b, d, t) at q[b*qsb + d*qsd + t*qst]; context (b, d, r) at
 * ctx[b*csb + d*csd + r*csr]; C at the given strides; A1 [B][R][T] (kept for
 * the backward) and attn = A2 [B][T][R] dense.  The backward takes dC (any
 * strides) and dattn ([B][T][R] dense, nullable) and overwrites dq [B][D][T]
 * and dctx [B][D][R] (dense).  The trainers reach this arithmetic through
 * tgfr_wr_fwd/_bwd; this is the per-call API. */
int tgfr_func_attention_fwd(const float* q, long long qsb, long long qsd, long long qst,
                            const float* ctx, long long csb, long long csd, long long csr, int B,
                            int D, int T, int R, float gamma1, float* C, long long Csb,
                            long long Csd, long long Cst, float* A1, float* attn, void* stream);
int tgfr_func_attention_bwd(const float* q, long long qsb, long long qsd, long long qst,
                            const float* ctx, long long csb, long long csd, long long csr,
                            const float* dC, long long dsb, long long dsd, long long dst,
                            const float* dattn, int B, int D, int T, int R, float gamma1,
                            const float* A1, const float* attn, float* dq, float* dctx,
                            void* stream);

/* Dynamic LDS bytes of the streaming forward (which = 0), the fp32-mode
 * backward (1) and the resident-R bf16 forward (2). */
int tgfr_wr_lds_bytes(int which);

/* logits[b*ldo + i] = scale * x_b.y_i / max(|x_b||y_i|, eps) (normalize = 1;
 * sent_loss models/losses.py:38-43, global_loss :338-343) or scale * x_b.y_i
 * (normalize = 0; ClipLoss :292-296).  masked = 1 applies the same-class
 * off-diagonal -inf mask of sent_loss (:21-30, :48) with global class ids
 * cls[] and this rank's first global row row_offset. */
int tgfr_cos_logits(const float* x, long long ldx, const float* y, long long ldy, int n_x,
                    int n_y, int d, int normalize, float scale, float eps, int masked,
                    const long long* cls, int row_offset, float* out, long long ldo,
                    void* stream);

/* dx_b = sum_i g[b*gs0 + i*gs1] d logits[b][i] / d x_b for tgfr_cos_logits
 * (swap x/y and the g strides for dy). */
int tgfr_cos_logits_bwd(const float* g, long long gs0, long long gs1, const float* x,
                        long long ldx, const float* y, long long ldy, int n_x, int n_y, int d,
                        int normalize, float scale, float eps, float* dx, long long lddx,
                        void* stream);

/* Row log-sum-exp and column (max, sum exp) partials of a [n_r x n_c] block;
 * col_lse (nullable) also receives the column LSE of this block alone (the
 * single-process case, where no exchange is needed).  With loss set (needs
 * col_lse and one zeroed counters word, left zeroed) the launch also computes
 * what tgfr_ce_loss would (row_offset, inv_n as there). */
int tgfr_ce_stats(const float* L, long long ld, int n_r, int n_c, float* row_lse,
                  float* col_max, float* col_sum, float* col_lse, int row_offset, float inv_n,
                  float* loss, unsigned* counters, void* stream);

/* sent_loss + global_loss of one process holding the whole batch (n <= 64,
 * models/losses.py:19-57 and :329-351): x = img [n][256], y = sent [n][256]
 * (16-byte aligned rows), cls [n] class ids; logits s_sent * cos with the
 * same-class off-diagonal mask and s_glob * cos without.  loss [3] = (sent
 * loss0, sent loss1, global loss0 + loss1); saves cosv [n][n], stats [4][n]
 * (row / column log-sum-exps of both logit sets) and nrm [2][n] for the
 * backward, which writes dx [n][256] (row stride lddx) from the upstream
 * gradients gs0, gs1, ggl (device scalars, each nullable = 0). */
int tgfr_sent_global(const float* x, long long ldx, const float* y, long long ldy, int n,
                     const long long* cls, float s_sent, float s_glob, float eps, float* cosv,
                     float* stats, float* nrm, float* loss, void* stream);
int tgfr_sent_global_bwd(const float* gs0, const float* gs1, const float* ggl, const float* x,
                         long long ldx, const float* y, long long ldy, int n,
                         const long long* cls, float s_sent, float s_glob, float eps,
                         const float* cosv, const float* stats, const float* nrm, float* dx,
                         long long lddx, void* stream);

/* The same two losses for n_r <= 64 local images (global rows row_offset ..)
 * against n_c <= 8192 all-gathered captions -- one process per GPU, or one
 * process with more than 64 rows.  _fwd (grid over 64-column tiles): cosv
 * [n_r][n_c], row partials, this rank's column partials colpart [2][2][n_c]
 * (sets sent / global x (max, sum exp)) and norms nrm [n_r + n_c]; the caller
 * all-gathers colpart rank-major (ONE collective for both losses) and _loss
 * (one workgroup) forms the column and row log-sum-exps into stats
 * [2 (n_r + n_c)] and this rank's contributions loss[3] = {sent loss0, sent
 * loss1, global loss} (each / N_global via inv_n); _bwd: dx [n_r][256] from
 * the losses' upstream gradients (device scalars, nullable).  Workspace sizes
 * (floats): tgfr_sent_global_dist_ws. */
int tgfr_sent_global_dist_ws(int n_r, int n_c, long long* rowpart, long long* colpart,
                             long long* stats);
int tgfr_sent_global_dist_fwd(const float* x, long long ldx, int n_r, const float* y,
                              long long ldy, int n_c, const long long* cls, int row_offset,
                              float s_sent, float s_glob, float eps, float* cosv, float* rowpart,
                              float* colpart, float* nrm, void* stream);
int tgfr_sent_global_dist_loss(const float* cosv, int n_r, int n_c, int row_offset, float s_sent,
                               float s_glob, const float* rowpart, const float* colparts,
                               int world, long long ld_parts, float inv_n, float* stats,
                               float* loss, void* stream);
int tgfr_sent_global_dist_bwd(const float* gs0, const float* gs1, const float* ggl,
                              const float* x, long long ldx, int n_r, const float* y,
                              long long ldy, int n_c, const long long* cls, int row_offset,
                              float s_sent, float s_glob, float eps, float inv_n,
                              const float* cosv, const float* stats, const float* nrm, float* dx,
                              long long lddx, void* stream);

/* Data-parallel glue (one rank's step; no host work between collectives):
 * tgfr_col_lse_combine: the global column log-sum-exp col_lse [n_c] from the
 * ranks' gathered column partials -- rank w's [2][n_c] = (max, sum exp(x -
 * max)) of tgfr_ce_stats at parts + w * ld (ld >= 2 n_c: the partials may
 * ride in a merged exchange buffer) -- combined in rank order.
 * tgfr_focal_global: the focal identity losses on the GLOBAL mean CE
 * (models/losses.py:313-325 on the gathered batch) for 1 or 2 heads whose
 * tgfr_focal_ce / tgfr_focal_ce2 workspaces ws0 / ws1 hold the local mean CE
 * at [rows]: phase 0 writes sums[k] = rows * that mean (the input of the one
 * collective); phase 1 adds the world ranks' sums (rank w's at sums + w * ld;
 * world 1: already all-reduced), writes logp = total * inv_n back into
 * ws_k[rows] (the backward's factor) and loss_k[0] = (1 - exp(-logp))^gamma
 * logp.  tgfr_sent_global_dist_loss reads rank r's column partials at
 * colparts + r * ld_parts (0: 4 n_c, the plain gathered layout). */
int tgfr_col_lse_combine(const float* parts, int world, long long ld, int n_c, float* col_lse,
                         void* stream);
int tgfr_focal_global(int phase, float* sums, int world, long long ld, int n_heads, int rows,
                      float inv_n, float gamma, float* ws0, float* ws1, float* loss0,
                      float* loss1, void* stream);

/* loss[0] = inv_n * sum_b (row_lse[b] - L[b][b+off]), loss[1] = inv_n * sum_b
 * (col_lse[b+off] - L[b][b+off]): this rank's share of nn.CrossEntropyLoss on
 * the rows and on the transposed matrix (models/losses.py:52-53, 131-132). */
int tgfr_ce_loss(const float* L, long long ld, int n_r, int row_offset, float inv_n,
                 const float* row_lse, const float* col_lse, float* loss, void* stream);

/* dL = w0*g0*inv_n (softmax_row - onehot) + w1*g1*inv_n (softmax_col - onehot),
 * with the upstream gradients g0, g1 read on the device (nullable: 1). */
int tgfr_ce_grad(const float* L, long long ld, int n_r, int n_c, int row_offset, float inv_n,
                 const float* row_lse, const float* col_lse, const float* g0, const float* g1,
                 float w0, float w1, float* dL, long long ldd, void* stream);

/* Batched C[b] = epi(alpha * A[b] B[b] (+ C[b] when accumulate) + bias) with
 * arbitrary element strides (transposes are stride swaps): the QK^T and PV
 * products of SelfAttention (models/fusion_nets.py:103, :115), the 1x1-conv /
 * Linear projections of IMIM and FCFM (models/models.py:386-404), and their
 * backward.  bias (nullable, per column) and relu form the epilogue.  With
 * ksplit > 1 the K range is split over ksplit blocks per output tile; each
 * stores its partial tile to slab (at least ksplit * batch * ceil(M/128)*128 *
 * ceil(N/128)*128 floats) and the partials are summed in slice order
 * (deterministic) before the epilogue, by the tile's last-arriving block
 * (ksplit <= 4) or by a second, chip-wide launch (ksplit > 4).
 * counters: >= batch * ceil(M/64) * ceil(N/64) zeroed uint32 words, left
 * zeroed on return. */
/* C = A W^T + bias with a bf16 output (IMIM's packed q/k/v projection in bf16
 * mode, models/models.py:397-398 -> fusion_nets.py:99-111): A [M][K] fp32 rows
 * (K = 128 or 256), W [N][K] fp32 (row stride sWn), C [M][N] bf16 (sCm). */
int tgfr_linear_bf16out(const float* A, long long sAm, int M, int K, const float* W,
                        long long sWn, const float* bias, int N, uint16_t* C, long long sCm,
                        void* stream);
/* The same with a bf16 A (rows 16-B aligned, sAm % 8 == 0): the BatchNorm'd
 * map of tgfr_bn_fwd_cl_bf16; identical products (the fp32 path rounds A to
 * bf16 at fragment read). */
int tgfr_linear_bf16io(const uint16_t* A, long long sAm, int M, int K, const float* W,
                       long long sWn, const float* bias, int N, uint16_t* C, long long sCm,
                       void* stream);

int tgfr_bgemm(const float* A, long long sAb, long long sAm, long long sAk, const float* B,
               long long sBb, long long sBk, long long sBn, float* C, long long sCb,
               long long sCm, long long sCn, int batch, int M, int N, int K, float alpha,
               int accumulate, const float* bias, int relu, int ksplit, float* slab,
               unsigned* counters, int mode, void* stream);

/* P = softmax(scale * S) per row (models/fusion_nets.py:103-106), optional LSE. */
int tgfr_attn_softmax(const float* S, float* P, float* lse, long long rows, int n, long long ld,
                      float scale, void* stream);

/* dS = scale * P * (dP - rowsum(P * dP)). */
int tgfr_attn_softmax_bwd(const float* P, const float* dP, float* dS, long long rows, int n,
                          long long ld, float scale, void* stream);

/* Fused self-attention for IMIM (fusion_nets.py:93-118 with C' = C = 256,
 * HW <= 224), bf16 operands / fp32 accumulation, no HW x HW matrix in HBM:
 *   O = softmax(scale * Q K^T) V  per sample; lse = row log-sum-exp of the
 *   scaled scores (saved for the backward).
 * Q, K, V: [B][hw][256] bf16 views (row stride ld, sample stride sb, both
 * multiples of 8), e.g. the column slices of the packed projection
 * [B][hw][768] written by tgfr_linear_bf16out.  O: [B][hw][256] fp32 (ldo,
 * sbo).  The backward recomputes P from lse and writes dQ, dK, dV in bf16
 * (ldg, sbg; overwritten: the operand of tgfr_dw_bf16); dO and O must be
 * dense [B][hw][256] fp32; ws: tgfr_attn_bwd_ws bytes. */
int tgfr_attn_fwd(const uint16_t* Q, const uint16_t* K, const uint16_t* V, long long ld,
                  long long sb, int B, int hw, float scale, float* O, long long ldo,
                  long long sbo, float* lse, void* stream);
int tgfr_attn_bwd_ws(int B, int hw, long long* bytes);
int tgfr_attn_bwd(const uint16_t* Q, const uint16_t* K, const uint16_t* V, long long ld,
                  long long sb, int B, int hw, float scale, const float* O, const float* dO,
                  long long ldo, long long sbo, const float* lse, uint16_t* dQ, uint16_t* dK,
                  uint16_t* dV, long long ldg, long long sbg, void* ws, void* stream);

/* Fused small attention for FCFM's cross-attention (fusion_nets.py:93-118 as
 * called at :248 with SelfAttention(36, scale=1): HW = C' = C = 36), one
 * workgroup per sample, exact fp32.  Replaces the composed QK^T / softmax /
 * PV (tgfr_bgemm + tgfr_attn_softmax) for HW, C', C <= 64.
 * X [B][hw][*] fp32 rows (sample stride sxn, row stride sxr) hold Qr at
 * columns [0, cq) and V at [cv, cv + c); Y (NULL = X) holds Kr at
 * [ck, ck + cq).  O [B][hw][c] (son, sor) = softmax(scale Qr Kr^T) V;
 * P [B][hw][hw] dense, saved for the backward.
 * The backward overwrites dQr / dV in dX's columns [0, cq) / [cv, cv + c)
 * and dKr in dY's [ck, ck + cq) (dY NULL = dX; the three ranges must then
 * be disjoint).  1001 on a shape that does not fit. */
int tgfr_attn_small_fwd(const float* X, long long sxn, long long sxr, const float* Y,
                        long long syn, long long syr, int B, int hw, int cq, int ck, int cv,
                        int c, float scale, float* O, long long son, long long sor, float* P,
                        void* stream);
int tgfr_attn_small_bwd(const float* X, long long sxn, long long sxr, const float* Y,
                        long long syn, long long syr, int B, int hw, int cq, int ck, int cv,
                        int c, float scale, const float* P, const float* dO, long long sdn,
                        long long sdr, float* dX, long long sgn, long long sgr, float* dY,
                        long long skn, long long skr, void* stream);

/* y = x / max(|x|, eps) per row (F.normalize; ProjectionHead models/models.py:119,
 * ArcMarginProduct models/metrics.py:44); inv_norm[row] = 1 / max(|x|, eps). */
int tgfr_l2norm_rows(const float* x, long long ldx, int rows, int d, float eps, float* y,
                     long long ldy, float* inv_norm, void* stream);

/* dx = (dy - y (y.dy)) * inv_norm (rows with |x| <= eps: dx = dy / eps). */
int tgfr_l2norm_rows_bwd(const float* dy, long long lddy, const float* y, long long ldy,
                         const float* inv_norm, int rows, int d, float eps, float* dx,
                         long long lddx, void* stream);

/* ArcMarginProduct margin (models/metrics.py:45-57) on a [rows x cols] cosine
 * matrix: out = s * (label column ? phi(cos) : cos). */
int tgfr_arc_margin(const float* cosv, const long long* label, int rows, int cols, float s,
                    float m, int easy, float* out, void* stream);

/* d cos from d out for tgfr_arc_margin. */
int tgfr_arc_margin_bwd(const float* cosv, const long long* label, const float* dout, int rows,
                        int cols, float s, float m, int easy, float* dcos, void* stream);

/* FocalLoss (models/losses.py:313-325): logp = mean_b CE(L_b, label_b),
 * loss[0] = (1 - exp(-logp))^gamma * logp; ws receives 2 * rows + 1 floats
 * (row LSE [rows], logp, row NLL [rows]) for the backward; counters: 1 zeroed
 * word (left zeroed). */
int tgfr_focal_ce(const float* L, int rows, int cols, const long long* label, float gamma,
                  float* ws, unsigned* counters, float* loss, void* stream);
/* Two focal losses on the same labels in one launch (the trainer's text and
 * image identity heads): (L, ws, loss) and (L2, ws2, loss2); counters: 2
 * zeroed words (left zeroed). */
int tgfr_focal_ce2(const float* L, const float* L2, int rows, int cols, const long long* label,
                   float gamma, float* ws, float* ws2, unsigned* counters, float* loss,
                   float* loss2, void* stream);

/* dL = gscale[0] * dloss/dlogp * (softmax(L_b) - onehot) / rows. */
int tgfr_focal_ce_bwd(const float* L, int rows, int cols, const long long* label, float gamma,
                      const float* ws, const float* gscale, float* dL, void* stream);

/* ---- per-sample LayerNorm (IMIM ln, models/models.py:388 / :401) -----------
 * x [rows][E] (row-contiguous, E % 4 == 0, 16-B aligned), affine w, b of E
 * elements: indexed like a row (ch == 0), or stored channel-major [ch][E/ch]
 * for rows laid out [E/ch][ch] (ch > 0, ch % 4 == 0): LayerNorm([C, H, W])
 * weights applied to channels-last rows (read in place, no transposed copy).
 * y = (x - mean_r) / sqrt(var_r + eps) * w + b with biased var_r, as
 * nn.LayerNorm.  ws: tgfr_ln_ws_floats(rows, E, ch, 1) floats; the forward
 * leaves mean/rstd in it for the backward (pass the same ws). */
int tgfr_ln_ws_floats(int rows, long long E, int ch, int backward, long long* out);
int tgfr_ln_fwd(const float* x, int rows, long long E, const float* w, const float* b, float eps,
                int ch, float* y, float* ws, void* stream);
/* dx, dw = sum_r dy xhat, db = sum_r dy (fixed-order reductions). */
int tgfr_ln_bwd(const float* dy, const float* x, int rows, long long E, const float* w, int ch,
                float* ws, float* dx, float* dw, float* db, void* stream);

/* ---- IMIM tail (models/models.py:399-405 + ProjectionHead :98-120), bf16 ----
 * Replaces, after IMIM's LayerNorm: conv1x1_1 + ReLU (:399-400), conv1x1_2 +
 * ReLU (:402), project_local (Linear 256->256, :403/:116) and F.normalize
 * (:117), over channels-last rows Z [rows][256] (rows = B*196), and their
 * backward.  One fused launch each way; weight gradients in one launch + a
 * deterministic slice reduce.
 *   tail_pack: W1 [128][256], W2 [256][128], Wp [256][256] (fp32, as the
 *     reference's conv/linear weights) -> pk, tgfr_tail_pack_elems() uint16
 *     (bf16 weights and their transposes); re-pack after every update.
 *   tail_fwd: R [rows][256] (ld ldr) = normalize(...); saves for the backward
 *     Zb [rows][256], H1b [rows][128], H2b [rows][256] (bf16) and
 *     inv [rows] = 1 / max(|P|, eps).  Optional (Rrows / Rnorm non-NULL, rows
 *     a multiple of rows_per_item): R again in the word<->region kernels'
 *     operand layout, Rrows [rows / rows_per_item][rows_pad][256] bf16 (fp16
 *     when rows_f16) with rows rows_per_item .. rows_pad - 1 zero, and
 *     Rnorm [..][rows_pad] = |R_row| -- what tgfr_prep_rows makes of R, so the
 *     step needs no separate pass over it (models/models.py:399-405 ->
 *     models/losses.py:96).
 *   tail_bwd: dZ [rows][256] (fp32, ld lddz) from dR; writes dPb [rows][256],
 *     dH2b [rows][256], dH1b [rows][128] (bf16, the ReLU masks applied).
 *   tail_dw: dWp = dP^T H2, dW2 = dH2^T H1, dW1 = dH1^T Z ([out][in], fp32,
 *     overwritten) and dbp/db2/db1 = column sums; ws: tgfr_tail_dw_ws floats. */
int tgfr_tail_pack_elems(void);
int tgfr_tail_pack(const float* W1, const float* W2, const float* Wp, uint16_t* pk,
                   void* stream);
int tgfr_tail_fwd(const float* Z, long long ldz, int rows, const uint16_t* pk, const float* b1,
                  const float* b2, const float* bp, float eps, float* R, long long ldr,
                  uint16_t* Zb, uint16_t* H1b, uint16_t* H2b, float* inv, uint16_t* Rrows,
                  float* Rnorm, int rows_per_item, int rows_pad, int rows_f16, void* stream);
int tgfr_tail_bwd(const float* dR, long long lddr, const float* R, long long ldr,
                  const float* inv, int rows, float eps, const uint16_t* pk, const uint16_t* H1b,
                  const uint16_t* H2b, float* dZ, long long lddz, uint16_t* dPb, uint16_t* dH2b,
                  uint16_t* dH1b, void* stream);
int tgfr_tail_dw_ws(int rows, long long* floats);
/* The tail with IMIM's LayerNorm([C, H, W]) (models/models.py:401) fused in,
 * on the attention output X [rows][256] (channels-last, rows = n * hw, hw >=
 * 32): Z = LayerNorm(X) is formed on the tail's load and never stored, and the
 * LayerNorm backward's per-sample sums run in the tail backward's epilogue.
 * Replaces tgfr_ln_fwd + tgfr_tail_pack + tgfr_tail_fwd (forward) and
 * tgfr_tail_bwd + tgfr_ln_bwd (backward): 3 + 3 launches instead of 4 + 4.
 *   ws: tgfr_ln_tail_ws floats, one buffer for the pair (LayerNorm moments and
 *     statistics, the backward's partial sums, the affine maps as
 *     channels-last rows); the forward's contents are read by the backward.
 *   tail_pack_ln: tail_pack plus the affine maps lnw, lnb ([256][hw], as the
 *     reference stores them) transposed into ws.
 *   ln_tail_fwd: LayerNorm slice moments of X, then tail_fwd on the
 *     normalised rows (ln_eps: nn.LayerNorm eps); outputs as tgfr_tail_fwd.
 *   ln_tail_bwd: tail_bwd (dZ [rows][256] fp32, dPb, dH2b, dH1b) plus the
 *     LayerNorm backward: dX [rows][256], dlnw / dlnb [256][hw] (reference
 *     layout, overwritten).  tgfr_tail_dw then takes the same saved operands. */
int tgfr_ln_tail_ws(int rows, int hw, long long* floats);
int tgfr_tail_pack_ln(const float* W1, const float* W2, const float* Wp, const float* lnw,
                      const float* lnb, int rows, int hw, uint16_t* pk, float* ws, void* stream);
int tgfr_ln_tail_fwd(const float* X, int rows, int hw, float ln_eps, float* ws,
                     const uint16_t* pk, const float* b1, const float* b2, const float* bp,
                     float eps, float* R, long long ldr, uint16_t* Zb, uint16_t* H1b,
                     uint16_t* H2b, float* inv, uint16_t* Rrows, float* Rnorm,
                     int rows_per_item, int rows_pad, int rows_f16, void* stream);
int tgfr_ln_tail_bwd(const float* dR, const float* R, const float* inv, int rows, float eps,
                     const uint16_t* pk, const uint16_t* H1b, const uint16_t* H2b,
                     const float* X, int hw, float* ws, float* dZ, uint16_t* dPb,
                     uint16_t* dH2b, uint16_t* dH1b, float* dX, float* dlnw, float* dlnb,
                     void* stream);
/* IMIM as one node (kernels.ImimFused): tgfr_imim_pack = tgfr_bn_fold3 (the
 * q/k/v weights Wqkv[3] / biases bqkv[3] (nullable), rows_qkv rows of C each,
 * folded with gamma / beta into Wf, bf) + tgfr_tail_pack_ln, one launch;
 * tgfr_ln_tail_bwd_att = tgfr_ln_tail_bwd writing, instead of dX, the
 * attention backward's operands into att_ws (tgfr_attn_bwd's workspace: D
 * [rows] = rowsum(dX * X), then dX [rows][256] in bf16), with dZ a scratch of
 * rows x 256 bf16 values (ABI 620: the LayerNorm backward reads dZ in bf16;
 * a float* of rows x 128 suffices); tgfr_attn_bwd_prepped
 * = tgfr_attn_bwd without its prep pass, reading them from ws. */
int tgfr_imim_pack(const float* const* Wqkv, const float* const* bqkv, int rows_qkv, int C,
                   const float* gamma, const float* beta, float* Wf, float* bf, const float* W1,
                   const float* W2, const float* Wp, const float* lnw, const float* lnb,
                   int rows, int hw, uint16_t* pk, float* ws, void* stream);
/* tgfr_imim_pack with IMIM's BatchNorm batch statistics (tgfr_bn_stats of
 * x [N][C][HW]; eps, momentum, training and the running buffers as there) as
 * the same launch's first C workgroups (ABI 600): the head's whole per-step
 * preparation before tgfr_bn_qkv_bf16 in one launch; Wfb (nullable) also
 * receives the folded q/k/v weights in bf16 [O][C]. */
int tgfr_imim_prep(const float* x, int N, int HW, float bn_eps, float momentum, int training,
                   float* running_mean, float* running_var, long long* nbt, float* mean,
                   float* rstd, const float* const* Wqkv, const float* const* bqkv, int rows_qkv,
                   int C, const float* gamma, const float* beta, float* Wf, uint16_t* Wfb,
                   float* bf, const float* W1, const float* W2, const float* Wp,
                   const float* lnw, const float* lnb, int rows, int hw, uint16_t* pk, float* ws,
                   void* stream);
int tgfr_ln_tail_bwd_att(const float* dR, const float* R, const float* inv, int rows, float eps,
                         const uint16_t* pk, const uint16_t* H1b, const uint16_t* H2b,
                         const float* X, int hw, float* ws, float* dZ, uint16_t* dPb,
                         uint16_t* dH2b, uint16_t* dH1b, void* att_ws, float* dlnw, float* dlnb,
                         void* stream);
/* tgfr_attn_fwd_ln: tgfr_attn_fwd (O dense [B][hw][256]) that also writes
 * each 32-query tile's LayerNorm moments (mean, M2) into ln_ws (the
 * tgfr_ln_tail_ws buffer); tgfr_ln_tail_fwd_att: tgfr_ln_tail_fwd taking those
 * moments instead of running its statistics pass. */
int tgfr_attn_fwd_ln(const uint16_t* Q, const uint16_t* K, const uint16_t* V, long long ld,
                     long long sb, int B, int hw, float scale, float* O, float* lse,
                     float* ln_ws, void* stream);
int tgfr_ln_tail_fwd_att(const float* X, int rows, int hw, float ln_eps, float* ws,
                         const uint16_t* pk, const float* b1, const float* b2, const float* bp,
                         float eps, float* R, long long ldr, uint16_t* Zb, uint16_t* H1b,
                         uint16_t* H2b, float* inv, uint16_t* Rrows, float* Rnorm,
                         int rows_per_item, int rows_pad, int rows_f16, void* stream);
/* tgfr_imim_dw: tgfr_tail_dw and tgfr_dw_bf16 (bf16 Y: the q/k/v projection's
 * dWq = Xq^T Yq [Nq][Kq], dbq = colsum Xq) in one launch + one reduce; ws:
 * tgfr_imim_dw_ws floats. */
int tgfr_imim_dw_ws(int rows, int Nq, int Kq, long long* floats);
int tgfr_imim_dw(const uint16_t* dPb, const uint16_t* H2b, const uint16_t* dH2b,
                 const uint16_t* H1b, const uint16_t* dH1b, const uint16_t* Zb, int rows,
                 float* dWp, float* dbp, float* dW2, float* db2, float* dW1, float* db1,
                 const uint16_t* Xq, const uint16_t* Yq, int Nq, int Kq, float* dWq, float* dbq,
                 float* ws, void* stream);
/* tgfr_imim_dw + the IMIM LayerNorm's dw / db [256][hw] (ABI 610): with
 * dlnw = dlnb = NULL, tgfr_ln_tail_bwd_att leaves the LayerNorm's per-group
 * partials in its tail workspace lnws, and this launch's reduce sums them
 * (same order, same values as the separate reduce) -- one kernel less on the
 * step's critical path.  Same ws as tgfr_imim_dw. */
int tgfr_imim_dw_ln(const uint16_t* dPb, const uint16_t* H2b, const uint16_t* dH2b,
                    const uint16_t* H1b, const uint16_t* dH1b, const uint16_t* Zb, int rows,
                    float* dWp, float* dbp, float* dW2, float* db2, float* dW1, float* db1,
                    const uint16_t* Xq, const uint16_t* Yq, int Nq, int Kq, float* dWq,
                    float* dbq, const float* lnws, int hw, float* dlnw, float* dlnb, float* ws,
                    void* stream);
int tgfr_attn_bwd_prepped(const uint16_t* Q, const uint16_t* K, const uint16_t* V, long long ld,
                          long long sb, int B, int hw, float scale, const float* lse,
                          uint16_t* dQ, uint16_t* dK, uint16_t* dV, long long ldg, long long sbg,
                          void* ws, void* stream);
/* Generic bf16 weight gradient of a row-wise linear map: dW [N][K] = X^T Y,
 * db [N] = column sums of X, for dense X [rows][N] bf16 and Y [rows][K]
 * (bf16, or fp32 when y_f32); N, K multiples of 128; fp32 outputs
 * overwritten; ws: tgfr_dw_bf16_ws floats (row-slice partials, summed in
 * slice order by a second launch). */
int tgfr_dw_bf16_ws(int rows, int N, int K, long long* floats);
int tgfr_dw_bf16(const uint16_t* X, const void* Y, int y_f32, int rows, int N, int K, float* dW,
                 float* db, float* ws, void* stream);
int tgfr_tail_dw(const uint16_t* dPb, const uint16_t* H2b, const uint16_t* dH2b,
                 const uint16_t* H1b, const uint16_t* dH1b, const uint16_t* Zb, int rows,
                 float* dWp, float* dbp, float* dW2, float* db2, float* dW1, float* db1, float* ws,
                 void* stream);

/* Bias gradient of a row-wise linear map: db[c] = sum_r dy[r][c].  With y
 * (the ReLU output) the ReLU mask is applied first and the masked gradient is
 * written to dym (both set or both NULL).  ws: ceil(rows / 128) * cols floats;
 * counters: ceil(cols / 64) zeroed words (left zeroed). */
int tgfr_bias_grad(const float* dy, long long lddy, int rows, int cols, const float* y,
                   long long ldy, float* dym, long long lddm, float* db, float* ws,
                   unsigned* counters, void* stream);

/* Weighted sums of scalar device losses: out[j] = sum_i W[j][i] * *losses[i]
 * (losses: host array of n <= 16 device pointers; W: host [m][n], m <= 4).
 * Row 0 is the training objective; tgfr_loss_mix_bwd gives its gradient
 * dloss[i] = g[0] * W[0][i].  Replaces the trainer's chain of scalar ops
 * (src/train_encoders_bert.py:279-323). */
int tgfr_loss_mix(int n, const float* const* losses, int m, const float* W, float* out,
                  void* stream);
int tgfr_loss_mix_bwd(const float* g, int n, const float* W, float* dloss, void* stream);

/* ---- IMIM input BatchNorm folded into the q/k/v projection --------------
 * (models/models.py:397-398 -> models/fusion_nets.py:97-99)
 * tgfr_bn_fwd_cl: x [N][C][HW] -> xhat [N][HW][C] = (x - mean) * rstd with
 * batch statistics (training: biased var for the normalisation, unbiased for
 * running_var, momentum update, *nbt += 1; each buffer nullable) or running
 * statistics (training == 0).  mean, rstd [C] are outputs. */
int tgfr_bn_fwd_cl(const float* x, int N, int C, int HW, float eps, float momentum,
                   int training, float* running_mean, float* running_var, long long* nbt,
                   float* mean, float* rstd, float* xhat, void* stream);
/* tgfr_bn_fwd_cl with xhat written in bf16 (bf16 mode without a BN input
 * gradient: its consumers, tgfr_linear_bf16io and tgfr_dw_bf16, read bf16). */
int tgfr_bn_fwd_cl_bf16(const float* x, int N, int C, int HW, float eps, float momentum,
                        int training, float* running_mean, float* running_var, long long* nbt,
                        float* mean, float* rstd, uint16_t* xhat, void* stream);
/* The batch statistics of tgfr_bn_fwd_cl alone (mean, rstd [C]; running
 * statistics updated as there), for tgfr_bn_qkv_bf16. */
int tgfr_bn_stats(const float* x, int N, int C, int HW, float eps, float momentum, int training,
                  float* running_mean, float* running_var, long long* nbt, float* mean,
                  float* rstd, void* stream);
/* IMIM's bf16 front end in one launch (ABI 600; models/models.py:394,
 * models/fusion_nets.py:97-109): px [N][HW][O] bf16 = bf16((x - mean) rstd)
 * W'^T + b' straight from the NCHW map x [N][C][HW] with the BN-folded
 * weights in bf16, Wfb [O][C] (tgfr_imim_prep), and bf [O], and the
 * channels-last bf16 xhat [N][HW][C] for the weight gradient.  Replaces
 * tgfr_bn_fwd_cl_bf16's normalisation pass + tgfr_linear_bf16io.  C = 256,
 * 128 < HW <= 224, HW % 4 == 0, O % 256 == 0, O <= 2048; x, Wfb, xhat 16-B
 * aligned, px 8-B aligned. */
int tgfr_bn_qkv_bf16(const float* x, int N, int C, int HW, const float* mean, const float* rstd,
                     const uint16_t* Wfb, const float* bf, int O, uint16_t* px, uint16_t* xhat,
                     void* stream);
/* BatchNorm2d input gradient: dx [N][C][HW] from the channels-last gradient
 * of xhat, dxh [N][HW][C], xhat and rstd of tgfr_bn_fwd_cl; training = batch
 * statistics (rstd (dxh - mean dxh - xhat mean(dxh xhat))), else rstd dxh. */
int tgfr_bn_bwd_cl(const float* dxh, const float* xhat, const float* rstd, int N, int C, int HW,
                   int training, float* dx, void* stream);
/* Wf = W diag(gamma), bf = b + W beta (W [O][C]; b nullable). */
int tgfr_bn_fold(const float* W, const float* b, int O, int C, const float* gamma,
                 const float* beta, float* Wf, float* bf, void* stream);
/* From G = dY^T xhat [O][C] and s = colsum(dY) [O]: dW = G diag(gamma) +
 * s beta^T, dgamma = sum_o W .* G, dbeta = sum_o W .* s (fixed-order sums).
 * ws: 2 * ceil(O / 16) * C floats; counters: ceil(C / 64) zeroed words. */
int tgfr_bn_unfold(const float* G, const float* s, const float* W, int O, int C,
                   const float* gamma, const float* beta, float* dW, float* dgamma, float* dbeta,
                   float* ws, unsigned* counters, void* stream);
/* tgfr_bn_fold / tgfr_bn_unfold with W (and b) given as 3 row blocks of
 * `rows` rows each (host arrays of 3 device pointers; b nullable, and each
 * of its entries nullable): the three 1x1 projections of a self-attention
 * (key, query, value) read in place.  Wf, bf, dW are the packed [3 rows][C]. */
int tgfr_bn_fold3(const float* const* W, const float* const* b, int rows, int C,
                  const float* gamma, const float* beta, float* Wf, float* bf, void* stream);
int tgfr_bn_unfold3(const float* G, const float* s, const float* const* W, int rows, int C,
                    const float* gamma, const float* beta, float* dW, float* dgamma,
                    float* dbeta, float* ws, unsigned* counters, void* stream);

/* ---- ArcMarginProduct (models/metrics.py:17-60), fused --------------------
 * tgfr_arc_fwd: logits[b][c] = s * margin(cos[b][c]) with cos = normalize(x_b)
 * . normalize(W_c) (F.normalize eps), the additive angular margin on column
 * label[b] (easy_margin or the th / mm fallback, :45-57); also writes cos
 * [B][C], xn = normalize(x) [B][D] and the inverse norms inv_nx [B], inv_nw
 * [C] for the backward.  fp32 FMA.  D % 4 == 0, D <= 1024, 16-B aligned rows.
 * tgfr_arc_bwd: from dlogits, dW = the gradient w.r.t. W (margin backward and
 * the l2-norm backward fused) and, when dcs is non-NULL, dcs[b][c] = dcos[b][c]
 * * inv_nw[c], so that d normalize(x) = dcs W (a GEMM) feeds
 * tgfr_l2norm_rows_bwd for dx.  B <= 1024.  ws: tgfr_arc_bwd_ws floats (0 for
 * B <= 64; NULL is accepted and runs the single-block-row path): for B > 64
 * the batch is split over block rows of <= 64 rows whose partial dW sums are
 * added in fixed order by a second launch. */
int tgfr_arc_fwd(const float* x, long long ldx, int B, int D, const float* W, long long ldw,
                 int C, const long long* label, float s, float m, int easy, float eps,
                 float* logits, float* cosv, float* xn, float* inv_nx, float* inv_nw,
                 void* stream);
int tgfr_arc_bwd(const float* dlogits, const float* cosv, const long long* label,
                 const float* xn, const float* W, long long ldw, const float* inv_nw, int B,
                 int D, int C, float s, float m, int easy, float eps, float* dW, long long lddw,
                 float* dcs, float* ws, void* stream);
int tgfr_arc_bwd_ws(int B, int D, int C, long long* floats);
/* Several ArcMarginProduct heads of the same (B, D, C) (the trainer's text and
 * image identity classifiers, src/train_encoders_bert.py:293-306) in one
 * launch each way, n_heads <= 2.  Per head: x [B][D], W [C][D] (dense rows,
 * 16-byte aligned), label, scale s; outputs as tgfr_arc_fwd.  The backward
 * (B <= 64) takes the head's focal loss (tgfr_focal_ce_heads) instead of
 * dlogits: its logit gradient g f'(logp) / B (softmax - onehot) is formed in
 * place from logits, focal_ws and the upstream gradient g (device scalar,
 * nullable = 1); writes dW and, when dcs is non-NULL, dcs as tgfr_arc_bwd. */
typedef struct {
  const float* x;
  const float* W;
  const long long* label;
  float s;
  float* logits;
  float* cosv;
  float* xn;
  float* inv_nx;
  float* inv_nw;
  const float* focal_ws;
  const float* g;
  float* dW;
  float* dcs;
} tgfr_arc_head;
int tgfr_arc_fwd_heads(const tgfr_arc_head* heads, int n_heads, int B, int D, int C, float m,
                       int easy, float eps, void* stream);
int tgfr_arc_focal_bwd_heads(const tgfr_arc_head* heads, int n_heads, int B, int D, int C,
                             float m, int easy, float eps, float gamma, void* stream);

/* ---- small-batch fp32 heads (csrc/tgfr_proj.hip) ---------------------------
 * tgfr_proj_l2norm_fwd: g = normalize(x W^T + b) per row, F.normalize(dim = 1,
 * eps) after nn.Linear -- ImageHeading.project_global (models/models.py:98-120,
 * :336) -- in one launch, exact fp32 (VALU FMA).  x [B][K] (ldx), W [N][K]
 * (ldw), bias [N] (nullable); g [B][N] (ldg), inv_norm [B] = 1 / max(|y|, eps)
 * for the backward.  N % 32 == 0, N <= 1024, K % 4 == 0, K <= 612, 16-B
 * aligned x / W.
 * ws: tgfr_proj_l2norm_ws floats.  counters: zeroed words (ceil(B / 8) used,
 * left zero).  Replaces tgfr_bgemm + tgfr_l2norm_rows.
 * tgfr_proj_dw: the Linear's weight gradient from dy (the l2-norm backward's
 * output, tgfr_l2norm_rows_bwd): dW = dy^T x [N][K] (lddw), db = colsum dy
 * (nullable); B <= 64.  Replaces tgfr_bias_grad + tgfr_bgemm.  Both: fixed
 * summation order (deterministic). */
int tgfr_proj_l2norm_ws(int B, int N, long long* floats);
int tgfr_proj_l2norm_fwd(const float* x, long long ldx, int B, int K, const float* W,
                         long long ldw, const float* bias, int N, float eps, float* ws,
                         float* g, long long ldg, float* inv_norm, unsigned* counters,
                         void* stream);
int tgfr_proj_dw(const float* dy, long long lddy, const float* x, long long ldx, int B, int K,
                 int N, float* dW, long long lddw, float* db, void* stream);
/* tgfr_arc_dx: an ArcMarginProduct head's input gradient from the dcs its
 * backward wrote (tgfr_arc_bwd / tgfr_arc_focal_bwd_heads): dxn = dcs W over
 * class chunks (partials in ws, tgfr_arc_dx_ws floats), summed in chunk order,
 * then dx = (dxn - xn (xn . dxn)) inv_nx (models/metrics.py:43, F.normalize
 * backward).  dcs [B][C], W [C][D] (16-B aligned, ldw % 4 == 0), xn [B][D],
 * D % 4 == 0, D <= 768.
 * Replaces tgfr_bgemm (+ its k-split reduce) + tgfr_l2norm_rows_bwd. */
int tgfr_arc_dx_ws(int B, int C, int D, long long* floats);
int tgfr_arc_dx(const float* dcs, const float* W, long long ldw, int B, int C, int D,
                const float* xn, const float* inv_nx, float eps, float* ws, float* dx,
                void* stream);

/* ---- optimiser step ------------------------------------------------------
 * Every trainable tensor of a trainer in one launch (replaces the two torch
 * optimiser steps of src/train_encoders_bert.py:212-222 / :323-330 and
 * src/fusion_bert.py:119-139).  Per group:
 *   Adam (torch.optim.Adam, amsgrad off):  g += wd p;  m = b1 m + (1-b1) g;
 *     v = b2 v + (1-b2) g^2;  p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
 *   SGD (torch.optim.SGD, nesterov off):  g += wd p;  buf = g at t = 1, else
 *     momentum buf + (1-dampening) g;  p -= lr buf  (no buf when momentum = 0)
 * state0 = m / buf, state1 = v (Adam only).  lr_scale (device, nullable):
 * one float per group multiplying that group's lr, read at launch time, so
 * an lr schedule applies to a captured step without re-capture.
 * counters: 2 ints, [0] = steps
 * taken so far (t - 1; the launch increments it), [1] = 0 (left 0).  The
 * segment table travels in the kernel arguments, so a captured launch
 * replays with the pointers it was captured with.  n_segs <= 48,
 * n_groups <= 4. */
#define TGFR_OPTIM_ADAM 0
#define TGFR_OPTIM_SGD 1
typedef struct {
  int kind;
  float lr, beta1, beta2, eps, weight_decay, momentum, dampening;
} tgfr_optim_group;
typedef struct {
  float* param;
  const float* grad;
  float* state0;
  float* state1;
  long long n;
  int group;
  int reserved;
} tgfr_optim_seg;
int tgfr_optim_step(const tgfr_optim_seg* segs, int n_segs, const tgfr_optim_group* groups,
                    int n_groups, const float* lr_scale, int* counters, void* stream);

/* TextHeading / Bert_Word_Mapping forward (models/models.py:170-232; run under
 * no_grad by utils/dataset_utils.py:42-45).
 *   tgfr_text_pack: conv_w, a host array of 3 device pointers to the
 *     Conv2d(1, 256, (K, 768)) weights [256][K*768] for K = 2, 3, 4 -> taps,
 *     tgfr_text_pack_bytes(mode) bytes of bf16 planes [9 taps][256][768] in
 *     the kernel's staging order (opaque to the caller)
 *     (hi, plus lo in mode 1).  Run once per weight update (the module
 *     caches it; the reference never updates these weights, no gradient
 *     reaches them).
 *   tgfr_text_heading: X [B][L1][768] fp32 BERT hidden states without [CLS]
 *     (L1 = bert_words_num - 1 >= 4), conv_b host array of 3 device pointers
 *     to the biases [256].  Writes words [B][L1-1][256] (row stride s_wt,
 *     caption stride s_wb; unit rows, the storage behind the reference's
 *     transposed [B, 256, L-2] view, :231) and sent [B][256] (row stride s_sb;
 *     unit rows, :215-220).  ws: tgfr_text_heading_ws floats (the three relu'd
 *     conv maps).  X, taps and the weights 16-byte aligned.  Optional (Wrows
 *     non-NULL): the words again as the word<->region kernels' operand rows,
 *     Wrows [B][t_pad][256] = bf16 (fp16 when rows_f16) of scale * word with
 *     rows L1-1 .. t_pad-1 zero, and Wnorm [B][t_pad] = |word| -- what
 *     tgfr_prep_rows makes of the words (scale log2(e) for the bf16 / fp16
 *     forward), so the step needs no separate pass over them.
 * Replaces the conv stack and the per-token Python loop of
 * get_each_word_feature / get_word_feature. */
int tgfr_text_pack_bytes(int mode, long long* bytes);
int tgfr_text_pack(const float* const* conv_w, uint16_t* taps, int mode, void* stream);
int tgfr_text_heading_ws(int B, int L1, long long* floats);
int tgfr_text_heading(const float* X, int B, int L1, const uint16_t* taps,
                      const float* const* conv_b, float* ws, float* words, long long s_wb,
                      long long s_wt, float* sent, long long s_sb, uint16_t* Wrows, float* Wnorm,
                      int t_pad, float scale, int rows_f16, int mode, void* stream);

/* ---- FCFM image branch (models/fusion_nets.py:236-237) ----------------------
 * relu(Conv2d(256, 36, 3, padding=0)(x)) -> MaxPool2d(2), fused, and its
 * backward.  x: the [B, 256, 14, 14] input read as channels-last rows
 * [B][196][256] (sample stride s_b, row stride s_p, channels contiguous,
 * 16-byte aligned; ImageHeading's physical layout).  mode 0 = bf16, 1 = fp32
 * (split bf16 pairs).
 *   tgfr_fcfm_pack: the Conv2d weight [36][256][3][3] fp32 -> pk,
 *     tgfr_fcfm_pack_elems() uint16 (bf16 MFMA fragments of both directions,
 *     opaque); re-pack after every update.
 *   tgfr_fcfm_conv_fwd: pooled [B][36][6][6] fp32 and code [B][36][6][6]
 *     (argmax 0..3 = dy*2+dx of the 2x2 window, -1 when the max is <= 0).
 *   tgfr_fcfm_conv_dx: dX rows [B][196][256] (strides s_b, s_p; overwritten)
 *     from gpool [B][36][6][6] (contiguous) and code.
 *   tgfr_fcfm_conv_dw: dW [36][256][3][3], db [36] (overwritten); ws:
 *     tgfr_fcfm_conv_dw_ws floats (sample-group partials summed in group
 *     order by a second launch). */
/* Working's second MaxPool2d(2) (fusion_nets.py:252) on a channels-last map:
 * x [B][H*W][C] -> y [B][C][H/2][W/2] (NCHW) and idx (argmax 0..3 = dy*2+dx,
 * first maximum); the backward writes every element of dx [B][H*W][C]. */
int tgfr_maxpool2_cl(const float* x, int B, int H, int W, int C, float* y, uint8_t* idx,
                     void* stream);
int tgfr_maxpool2_cl_bwd(const float* dy, const uint8_t* idx, int B, int H, int W, int C,
                         float* dx, void* stream);
int tgfr_fcfm_pack_elems(void);
int tgfr_fcfm_pack(const float* W, uint16_t* pk, void* stream);
int tgfr_fcfm_conv_fwd(const float* x, long long s_b, long long s_p, int B, const uint16_t* pk,
                       const float* bias, float* pooled, int8_t* code, int mode, void* stream);
int tgfr_fcfm_conv_dx(const float* gpool, const int8_t* code, int B, const uint16_t* pk,
                      float* dx, long long s_b, long long s_p, int mode, void* stream);
int tgfr_fcfm_conv_dw_ws(int B, long long* floats);
int tgfr_fcfm_conv_dw(const float* x, long long s_b, long long s_p, const float* gpool,
                      const int8_t* code, int B, float* dW, float* db, float* ws, int mode,
                      void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TGFR_H */
