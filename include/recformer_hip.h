/*
 * librecformer_hip — C ABI of the MI355X-native Recformer encoder + scorer.
 *
 * The reference exposes no C ABI: its boundary is the Python class API of
 * recformer/models.py (RecformerModel.forward models.py:274-356,
 * RecformerForSeqRec.forward models.py:547-599). These entry points are what the
 * build's autograd Functions (recformer_amd/ops.py) bind with ctypes; each one names
 * the reference computation it replaces. See INTEGRATION.md for the bindings.
 *
 * Conventions:
 *  - all pointers are DEVICE pointers owned by the caller (PyTorch's caching
 *    allocator); the library never allocates, frees or synchronises;
 *  - `stream` is the caller's hipStream_t (torch.cuda.current_stream().cuda_stream);
 *    every call is asynchronous on it and safe to capture in a hipGraph;
 *  - matrices are row-major with explicit leading dimensions in ELEMENTS;
 *  - `dtype` selects the storage/compute type of activations and weights:
 *    RF_F32 (fp32 storage, exact-fp32 MFMA), RF_BF16 or RF_F16 (16-bit storage, fp32
 *    accumulate; RF_F16 = the fp16 autocast of the reference's drivers);
 *    biases, LayerNorm affine parameters, norms and scores are always fp32;
 *  - return 0 on success; otherwise rf_last_error() holds a thread-local message.
 */
#ifndef RECFORMER_HIP_H
#define RECFORMER_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* rf_stream_t;

enum { RF_OK = 0, RF_ERR_ARG = 1, RF_ERR_HIP = 2 };
enum { RF_F32 = 0, RF_BF16 = 1, RF_F16 = 2 };
enum { RF_IO_C_F32 = 1, RF_IO_R_F32 = 2 }; /* rf_gemm io_flags (bf16 GEMMs): C / residual in fp32 */
enum {
  RF_EPI_NONE = 0,       /* C = A.W^T                                   */
  RF_EPI_BIAS = 1,       /* C = A.W^T + b              (nn.Linear)      */
  RF_EPI_BIAS_GELU = 2,  /* C = gelu_erf(A.W^T + b)    (TF:1113-1116)   */
  RF_EPI_BIAS_RESID = 3, /* C = A.W^T + b + R          (TF:1068-1071 / 1127-1130, pre-LN) */
  RF_EPI_COS = 4,        /* C(f32) = A.W^T * ra[m] * rw[n] * scale (Similarity, models.py:358-369) */
  RF_EPI_BIAS_RESID_LN = 5, /* C(f32) = A.W^T + b + LN(R): rf_gemm_resid_ln only */
  RF_EPI_BIAS_GELU_AUX = 6, /* C = gelu_erf(A.W^T + b) and R (bf16, written) = A.W^T + b: the
                               pre-activation the training path's GELU backward reads */
  RF_EPI_DGELU = 7          /* C = (A.W^T) * gelu_erf'(R), R the 16-bit pre-activation, no bias: the
                               GELU backward fused into the dA GEMM of the next Linear (TF:1113-1116) */
};

const char* rf_last_error(void);
/* Device-side dropout seeds for captured (hipGraph) training steps: registers a device uint64 step
 * counter (NULL: none, the default). Every dropout launch made while one is registered uses
 * seed + counter * 0x9E3779B97F4A7C15 (read on the device at kernel start), so a captured step whose
 * graph advances the counter draws new masks on each replay while its backward regenerates the
 * forward's. Returns the previous counter. Process-wide; not thread-safe. */
const uint64_t* rf_set_seed_source(const uint64_t* step_counter);
/* ABI version of this header (2): bumped whenever an entry point's arguments change; a binding
 * refuses a library that reports another (recformer_amd/_lib.py ABI_VERSION). */
int rf_abi_version(void);
/* Diagnostics (A/B tools; the product never sets them): set a launch-path tuning knob ("gemm_gn",
 * "gemm_variant", "band_qpb", "band_path", "gfold_path", "gfold_qsplit", "gemm_pf", "gemm_mfma32",
 * "rank_w32", "gfold_chunk", "gemm_skinny", "epi_tile", "tn_wgs", "mid_tile", "colsum_slices", "gemm_n192", "adam_nt", "gemm_w8", "gemm_w4p") for the process;
 * returns the previous value
 * (INT32_MIN and rf_last_error() for an unknown name). The compiled defaults are the measured choices;
 * no launch reads the environment. */
int rf_debug_set_knob(const char* name, int value);
/* the knob's current value (INT32_MIN and rf_last_error for an unknown name) */
int rf_debug_get_knob(const char* name);

/* A2 — RecformerModel.forward prologue, models.py:306-329 (_merge_to_attention_mask
 * 262-272, _pad_to_window_size 210-260) + create_position_ids_from_input_ids 68-79.
 * Inputs (B,L) int64 (attention_mask / global_attention_mask / token_type_ids /
 * position_ids may be NULL = reference defaults). Outputs (B,Lp) int32 ids/pos/type/
 * item-pos, uint8 flags {0 pad, 1 local, 2 global}, and gidx (B,gmax) int32 = the
 * positions of each row's global tokens in order, -1 padded (replaces the nonzero()
 * bookkeeping of TF:869-896 without a host sync). gstat (B,2) int32, optional (NULL: not
 * written): per sequence its number of global tokens and whether position 0 (the CLS) is one —
 * what the caller reads back once to size gidx (the global-slot count) and to pick the
 * CLS-only last layer, instead of reducing the masks with separate device ops. */
int rf_prepare_inputs(const int64_t* input_ids, const int64_t* attention_mask,
                      const int64_t* global_attention_mask, const int64_t* token_type_ids,
                      const int64_t* item_position_ids, const int64_t* position_ids,
                      int B, int L, int Lp, int pad_id, int gmax,
                      int32_t* ids, int32_t* pos, int32_t* tt, int32_t* ip, uint8_t* flags,
                      int32_t* gidx, int32_t* gstat, rf_stream_t stream);

/* A3 — RecformerEmbeddings.forward, models.py:108-138: LN(Ew[id] + Ep[pos] + Et[tt] +
 * Ei[ip]) for M tokens, one fused pass. Tables in table_dtype, LN params fp32, output in
 * out_dtype plus an optional fp32 copy out32 (M x D; the bf16 path's residual stream). */
int rf_embed_ln_fwd(int table_dtype, int out_dtype, int M, int D, const int32_t* ids,
                    const int32_t* pos, const int32_t* tt, const int32_t* ip,
                    const void* word_emb, const void* pos_emb, const void* type_emb,
                    const void* ipos_emb, const float* ln_w, const float* ln_b, float eps,
                    void* out, float* out32, rf_stream_t stream);

/* A4 linears — nn.Linear / the 9 addmm per layer (TF:504-506, 982-984, 1064-1071,
 * 1107, 1123) on MFMA: C[M,N] = epi(A[M,K] . W[N,K]^T). The first `scale_cols`
 * output columns are multiplied by `col_scale` after the bias (the q/sqrt(hd) of
 * TF:514). C and the residual R are stored in `dtype`, or in fp32 when io_flags has
 * RF_IO_C_F32 / RF_IO_R_F32 (the bf16 path keeps the residual stream and the pre-LayerNorm
 * sums in fp32, as the reference's autocast does: LayerNorm outputs fp32 there).
 * EPI_COS always writes fp32 C and needs ra (M) / rw (N) inverse norms. */
int rf_gemm(int dtype, int M, int N, int K, const void* A, int lda, const void* W, int ldw,
            const float* bias, const void* resid, int ldr, void* C, int ldc, int io_flags,
            int epilogue, int scale_cols, float col_scale, const float* ra, const float* rw,
            rf_stream_t stream);

/* The residual-add linears (attention output TF:1068-1071, FFN output TF:1127-1130) with the
 * residual given as the PREVIOUS LayerNorm's fp32 input rows R and its row statistics:
 * C(f32) = A.W^T + b + ((R - mean) * rstd * gamma + beta) — the same expression the LayerNorm
 * kernel evaluates, so the LN output never needs an fp32 copy in HBM. */
int rf_gemm_resid_ln(int dtype, int M, int N, int K, const void* A, int lda, const void* W,
                     int ldw, const float* bias, const float* resid_pre, int ldr,
                     const float* r_mean, const float* r_rstd, const float* r_gamma,
                     const float* r_beta, float* C, int ldc, rf_stream_t stream);

/* LayerNorm over rows of D (TF:1071, 1130; nn.LayerNorm eps); x in x_dtype, y in y_dtype,
 * optional fp32 copy y32 (M x D, contiguous); mean/rstd (M) optional. */
int rf_layernorm_fwd(int x_dtype, int y_dtype, int M, int D, const void* x, int ldx,
                     const float* w, const float* b, float eps, void* y, int ldy, float* y32,
                     float* mean, float* rstd, rf_stream_t stream);

/* Residual add + LayerNorm, the reference's LayerNorm(dense(h) + input_tensor) (TF:1064-1071
 * LongformerSelfOutput, TF:1123-1130 LongformerOutput): y = LN(x + res) with x the dense
 * output (x_dtype, the bf16 GEMM output under autocast) and res the fp32 residual stream
 * (M x D, contiguous). y32 (fp32 copy, M x D) may alias res: the stream is updated in place. */
int rf_add_layernorm_fwd(int x_dtype, int y_dtype, int M, int D, const void* x, int ldx, const float* res,
                         const float* w, const float* b, float eps, void* y, int ldy, float* y32,
                         float* mean, float* rstd, rf_stream_t stream);

/* The bf16 path's fp32 residual stream, stored split: plane hi (bf16, M x D) =
 * the top half of each fp32 value rounded half-up — also the next GEMM's bf16 operand — and
 * plane lo (uint16, M x D) = its low 16 bits; together they decode to the fp32 value exactly.
 * rf_embed_ln_split_fwd: rf_embed_ln_fwd writing the stream as planes (models.py:108-138).
 * rf_add_layernorm_split_fwd: rf_add_layernorm_fwd on planes: y = LN(x + join(res_hi, res_lo))
 * (TF:1064-1071, 1123-1130) with x bf16; writes planes (y_hi, y_lo; may alias res_hi, res_lo)
 * and/or an fp32 copy y32 (M x D). res planes NULL = plain LayerNorm of x. */
int rf_embed_ln_split_fwd(int table_dtype, int M, int D, const int32_t* ids, const int32_t* pos,
                          const int32_t* tt, const int32_t* ip, const void* word_emb, const void* pos_emb,
                          const void* type_emb, const void* ipos_emb, const float* ln_w, const float* ln_b,
                          float eps, uint16_t* out_hi, uint16_t* out_lo, rf_stream_t stream);
int rf_add_layernorm_split_fwd(int M, int D, const void* x, int ldx, const uint16_t* res_hi,
                               const uint16_t* res_lo, const float* w, const float* b, float eps,
                               uint16_t* y_hi, uint16_t* y_lo, float* y32, rf_stream_t stream);

/* LayerNorm backward for the training path (autograd of TF:1071, 1130 / models.py:136):
 * dy, x (the fp32 LayerNorm input rows, leading dim ldx), the forward's row mean / rstd and
 * gamma w -> dx (M x D fp32), dw = sum_rows dy * xhat, db = sum_rows dy (fp32 [D]); column sums
 * are reduced deterministically through rf_layernorm_bwd_workspace(M, D) bytes of workspace. */
size_t rf_layernorm_bwd_workspace(int M, int D);
/* Training path, hidden dropout + residual + LayerNorm (TF:1068-1071, 1127-1130 with
 * nn.Dropout(hidden_dropout_prob)): x = dropout_p(t) + res (t bf16 dense output, ld ldt; res fp32
 * M x D), y = LN(x); writes x (fp32, the backward's input), y (fp32) and the row stats. The keep
 * mask is a counter hash of (seed, row * D + col), regenerated by rf_drop_add_ln_bwd, which
 * writes dres = dx (fp32), dt = dx * mask / (1 - p) (bf16) and dw / db (workspace as
 * rf_layernorm_bwd). p = 0: plain residual add. */
int rf_drop_add_ln_fwd(int M, int D, const void* t, int ldt, const float* res, float p, uint64_t seed,
                       const float* w, const float* b, float eps, float* x, float* y, float* mean, float* rstd,
                       rf_stream_t stream);
int rf_drop_add_ln_bwd(int M, int D, const float* dy, const float* x, const float* mean, const float* rstd,
                       const float* w, float p, uint64_t seed, float* dres, void* dt, float* dw, float* db,
                       void* workspace, rf_stream_t stream);
/* The same pair for an output with two consumers (training: the next residual add in fp32 and
 * the next GEMM in bf16): _dual forward also writes y16 = bf16(y) (null: not written); _dual
 * backward takes both consumers' gradients, dy (fp32) and dy16 (bf16), either may be null, and
 * sums them in the kernel (dy + float(dy16), as autograd would). */
int rf_drop_add_ln_fwd_dual(int M, int D, const void* t, int ldt, const float* res, float p, uint64_t seed,
                            const float* w, const float* b, float eps, float* x, float* y, float* mean,
                            float* rstd, void* y16, rf_stream_t stream);
int rf_drop_add_ln_bwd_dual(int M, int D, const float* dy, const void* dy16, const float* x, const float* mean,
                            const float* rstd, const float* w, float p, uint64_t seed, float* dres, void* dt,
                            float* dw, float* db, void* workspace, rf_stream_t stream);
/* The same pair with the dense output t / y16 / dt / dy16 in dtype (RF_BF16 or RF_F16: the fp16
 * autocast path, finetune.py:106-110). mask_row_mul (>= 1): the keep mask of row r is that of row
 * r * mask_row_mul, i.e. the hash index is (r * mask_row_mul * D + col) — the training path's CLS-only
 * last layer runs the B CLS rows compacted and passes Lp, so each draws the mask of its full-layer row
 * b * Lp (1: the plain row-major index). */
int rf_drop_add_ln_fwd_t(int dtype, int M, int D, const void* t, int ldt, const float* res, float p, uint64_t seed,
                         const float* w, const float* b, float eps, float* x, float* y, float* mean, float* rstd,
                         void* y16, int mask_row_mul, rf_stream_t stream);
int rf_drop_add_ln_bwd_t(int dtype, int M, int D, const float* dy, const void* dy16, const float* x,
                         const float* mean, const float* rstd, const float* w, float p, uint64_t seed, float* dres,
                         void* dt, float* dw, float* db, void* workspace, int mask_row_mul, rf_stream_t stream);
/* rf_drop_add_ln_bwd_t that also writes dbias_t (D fp32) = the column sums of dt as stored (16-bit):
 * the bias gradient of the Linear whose output t is (TF:1064-1071, 1123-1130), from the same pass (no
 * separate read of dt for it). */
int rf_drop_add_ln_bwd_tb(int dtype, int M, int D, const float* dy, const void* dy16, const float* x,
                          const float* mean, const float* rstd, const float* w, float p, uint64_t seed, float* dres,
                          void* dt, float* dw, float* db, float* dbias_t, void* workspace, int mask_row_mul,
                          rf_stream_t stream);
/* Weight gradient of an nn.Linear, C (=|+=) X^T Y: C[n][k] = sum_m X[m][n] Y[m][k] over the M token
 * rows (X = dC (M x N), Y = A (M x K), 16-bit row-major; C fp32 N x K, the master weight's dtype) —
 * the dW = dC^T A of autograd through TF:504-514, 1064-1130 and the LM head (models.py:499-510).
 * MFMA with transposed LDS reads; the rows split over workgroups into fp32 slabs reduced in a fixed
 * order (deterministic); accumulate != 0 adds into C. Rows n < scale_rows of the product are
 * multiplied by row_scale before they are stored / added (a Linear whose first outputs carry a column
 * scale: the query's 1/sqrt(head_dim), TF:504-514; 0 = none). Workspace: rf_weight_grad_workspace bytes. */
size_t rf_weight_grad_workspace(int M, int N, int K);
int rf_weight_grad(int dtype, int M, int N, int K, const void* X, int ldx, const void* Y, int ldy, float* C, int ldc,
                   int accumulate, int scale_rows, float row_scale, void* workspace, size_t ws_bytes,
                   rf_stream_t stream);
/* Backward of the fused embedding + LayerNorm (RecformerEmbeddings, models.py:108-138): from dh (M x D
 * fp32) the row gradient dx = dL/d(Ew[id] + Ep[pos] + Et[tt] + Ei[ip]) (M x D fp32; the pre-LN sum is
 * regathered from the fp32 tables, not stored) and dgamma / dbeta (deterministic, fixed-order sums).
 * Workspace: rf_embed_ln_bwd_workspace bytes. */
size_t rf_embed_ln_bwd_workspace(int M, int D);
int rf_embed_ln_bwd(int M, int D, const int32_t* ids, const int32_t* pos, const int32_t* tt, const int32_t* ip,
                    const float* word_emb, const float* pos_emb, const float* type_emb, const float* ipos_emb,
                    const float* ln_w, float eps, const float* dh, float* dx, float* dgamma, float* dbeta,
                    void* workspace, rf_stream_t stream);
/* An embedding table's gradient without atomics (nn.Embedding backward, models.py:82-138):
 * dst[keys_sorted[j]] = sum of src[perm[j']] over the run of equal keys containing j, summed in the
 * sorted order (perm / keys_sorted: a stable sort of the token indices); rows of key `pad`
 * (padding_idx) and untouched rows are left as they are (the caller zero-fills dst).
 * Workspace: rf_segment_rows_sum_workspace bytes. */
size_t rf_segment_rows_sum_workspace(int M, int D);
int rf_segment_rows_sum(int M, int D, const float* src, const int32_t* perm, const int32_t* keys_sorted, int pad,
                        float* dst, int V, void* workspace, rf_stream_t stream);
/* Column sums out[n] = sum_m x[m][n] (fp32 out; x in dtype, row-major, leading dim ldx), two
 * deterministic stages through rf_colsum_workspace(M, N) bytes — the bias gradient of the
 * training path's linears (db = sum_rows dC, the autograd of TF:504-1130's nn.Linear bias); columns
 * n < scale_cols multiplied by col_scale (the query's bias under its 1/sqrt(head_dim) scale; 0 = none). */
size_t rf_colsum_workspace(int M, int N);
int rf_colsum(int dtype, int M, int N, const void* x, int64_t ldx, float* out, int scale_cols, float col_scale,
              void* workspace, rf_stream_t stream);
/* dst[rows[r]] += src[r] (r < R; rows[r] < 0 skipped) for one or two (src, dst) pairs of the
 * same shape (src1 = dst1 = null: one); repeated rows add in row order. The training path's
 * global-key gradient columns added into dk / dv at the global positions (the reduction of
 * TF:898-926's gradient, train.py). */
int rf_scatter_add_rows(int dtype, int R, int D, const int32_t* rows, const void* src0, const void* src1,
                        int ld_src, void* dst0, void* dst1, int ld_dst, rf_stream_t stream);
int rf_layernorm_bwd(int M, int D, const float* dy, const float* x, int ldx, const float* mean,
                     const float* rstd, const float* w, float* dx, float* dw, float* db, void* workspace,
                     rf_stream_t stream);

/* A5 — LongformerSelfAttention local branch (TF:482-604 with _sliding_chunks_* 759-867,
 * _mask_invalid_locations 743-757, _concat_with_global_key_attn_probs 898-926,
 * _compute_attn_output_with_global_indices 928-962). q (pre-scaled), k, v are
 * (B*Lp, *) row-major with leading dim ld_qkv, head h at column h*hd. hd must be 64.
 * Output ctx (B*Lp, H*hd), ld_out; padded query rows are written as 0. */
int rf_band_attn_fwd(int dtype, int B, int Lp, int H, int hd, int half_w, const void* q,
                     const void* k, const void* v, int ld_qkv, const uint8_t* flags,
                     const int32_t* gidx, int gmax, void* out, int ld_out, rf_stream_t stream);



/* Training form with attention-probability dropout (TF:585-586, nn.functional.dropout on the
 * softmax probabilities, p_drop in [0, 1)): the probabilities entering P.V are multiplied by a keep
 * mask / (1 - p_drop); the mask is a counter hash of (seed, ((b*H + h)*Lp + i)*Lp + j) for query i
 * and key j (never stored; rf_band_attn_bwd_drop regenerates it). p_drop = 0: rf_band_attn_fwd. */
int rf_band_attn_fwd_drop(int dtype, int B, int Lp, int H, int hd, int half_w, const void* q,
                          const void* k, const void* v, int ld_qkv, const uint8_t* flags,
                          const int32_t* gidx, int gmax, void* out, int ld_out, float p_drop,
                          uint64_t seed, rf_stream_t stream);

/* Backward of the local branch (A5/A9: gradient of LongformerSelfAttention's sliding-window
 * attention TF:482-604 incl. its global-key columns TF:898-962), bf16 q/k/v/o/dout (q
 * pre-scaled, as the forward), fp32 gradients (B*Lp, ld_grad) dq, dk, dv. Workspace outputs:
 * lse2, delta (B*H*Lp fp32: row log2-sum-exp and dO.O), gds, gpr (B*H*Lp*gmax fp32: dS and P
 * of the global-key columns; the caller reduces them into dk/dv at the global positions).
 * Query rows with flag != 1 (padding, or global rows whose local output is overwritten) carry
 * no gradient. Window 64 (half 32), head_dim 64, gmax <= 32. */
int rf_band_attn_bwd(int B, int Lp, int H, int hd, int half_w, const void* q, const void* k,
                     const void* v, int ld_qkv, const void* o, int ld_o, const void* dout, int ld_do,
                     const uint8_t* flags, const int32_t* gidx, int gmax, float* dq, float* dk,
                     float* dv, int ld_grad, float* lse2, float* delta, float* gds, float* gpr,
                     rf_stream_t stream);
/* The same with the gradients dq, dk, dv written in grad_dtype (RF_F32 or RF_BF16: what the
 * bf16 q|k|v projection's backward consumes, as under the reference's autocast). */
int rf_band_attn_bwd_dt(int grad_dtype, int B, int Lp, int H, int hd, int half_w, const void* q,
                        const void* k, const void* v, int ld_qkv, const void* o, int ld_o,
                        const void* dout, int ld_do, const uint8_t* flags, const int32_t* gidx,
                        int gmax, void* dq, void* dk, void* dv, int ld_grad, float* lse2,
                        float* delta, float* gds, float* gpr, rf_stream_t stream);
/* rf_band_attn_bwd_dt for a forward run with attention-probability dropout (same p_drop, seed):
 * dP = mask/(1-p) o dO V^T, dS = P o (dP - dO.O); gpr holds the dropped probabilities. Operands
 * q/k/v/o/dout in dtype (RF_BF16 or RF_F16), gradients in grad_dtype (RF_F32 or dtype). */
int rf_band_attn_bwd_drop(int dtype, int grad_dtype, int B, int Lp, int H, int hd, int half_w, const void* q,
                          const void* k, const void* v, int ld_qkv, const void* o, int ld_o,
                          const void* dout, int ld_do, const uint8_t* flags, const int32_t* gidx,
                          int gmax, void* dq, void* dk, void* dv, int ld_grad, float* lse2,
                          float* delta, float* gds, float* gpr, float p_drop, uint64_t seed,
                          rf_stream_t stream);
/* A6 — global query rows, _compute_global_attn_output_from_hidden TF:964-1057 + the
 * overwrite TF:612-629: for every (b, g < count_b): ctx[gidx[b,g], h] =
 * softmax(qg[b*gmax+g, h] . kg[b, :, h]^T over valid keys) . vg[b, :, h]. */
int rf_global_attn_fwd(int dtype, int B, int Lp, int H, int hd, const void* qg, int ld_qg,
                       const void* kg, const void* vg, int ld_kv, const uint8_t* flags,
                       const int32_t* gidx, int gmax, void* out, int ld_out,
                       rf_stream_t stream);

/* A6, production form — the same global rows through the key/value-projection fold
 * (exact algebra, different rounding; SURVEY.md §7 'Global-path algebra'):
 *   s_j = (Wkg_h^T qg_h) . h_j + qg_h . bkg_h over valid keys j,
 *   ctx[gidx[b,g], h] = Wvg_h (sum_j softmax(s)_j h_j) + bvg_h.
 * h is the layer input (B*Lp, D) (leading dim ldh), wkg/wvg (D, D) nn.Linear weights in
 * dtype, bkg/bvg fp32. Replaces key_global/value_global over all L tokens (TF:983-984).
 * workspace: rf_global_fold_workspace(B, Lp, D, H, gmax) bytes of device memory. */
size_t rf_global_fold_workspace(int B, int Lp, int D, int H, int gmax);
int rf_global_attn_fold_fwd(int dtype, int B, int Lp, int D, int H, const void* qg, int ld_qg,
                            const void* h, int ldh, const void* wkg, const float* bkg,
                            const void* wvg, const float* bvg, const uint8_t* flags,
                            const int32_t* gidx, int gmax, void* workspace, void* out,
                            int ld_out, rf_stream_t stream);
/* The same with attention-probability dropout on the global rows (training; TF:1036-1037):
 * w_h = sum_j z_j p_j h_j and the value bias weighted by sum_j z_j p_j, with z the keep mask x
 * 1/(1-p) of row (b*H + h)*Lp + gidx[b,g], key j (rf_common.h drop_keep). 16-bit dtypes only;
 * p_drop = 0 is rf_global_attn_fold_fwd. */
int rf_global_attn_fold_fwd_drop(int dtype, int B, int Lp, int D, int H, const void* qg, int ld_qg,
                                 const void* h, int ldh, const void* wkg, const float* bkg,
                                 const void* wvg, const float* bvg, const uint8_t* flags,
                                 const int32_t* gidx, int gmax, void* workspace, void* out,
                                 int ld_out, float p_drop, uint64_t seed, rf_stream_t stream);
/* rf_global_attn_fold_fwd_drop in two stages on the same workspace: stage 1 = u and the pass over h
 * (reads qg, h, wkg; `out` unused), stage 2 = the chunk merge and Wvg, written into out's global rows;
 * 3 = both. Stage 1 does not touch `out`, so a training forward runs it beside the local attention that
 * writes out, and stage 2 after it. */
int rf_global_attn_fold_fwd_stage(int stage, int dtype, int B, int Lp, int D, int H, const void* qg, int ld_qg,
                                  const void* h, int ldh, const void* wkg, const float* bkg,
                                  const void* wvg, const float* bvg, const uint8_t* flags,
                                  const int32_t* gidx, int gmax, void* workspace, void* out,
                                  int ld_out, float p_drop, uint64_t seed, rf_stream_t stream);
/* That mask for the backward: z (B, H, gmax, Lp) fp32, z[b,h,g,l] = keep x 1/(1-p) of row
 * (b*H + h)*Lp + max(gidx[b,g], 0), key l. */
int rf_attn_global_keep(int B, int H, int Lp, const int32_t* gidx, int gmax, float p_drop,
                        uint64_t seed, float* z, rf_stream_t stream);

/* The same, starting from the layer input: qg_h = (Wqg_h h_g + bqg_h) * q_scale for each global
 * row's hidden vector h_g (query_global, TF:972-982, rounded to dtype like a GEMM output), then
 * the fold as above — one entry point for the whole global path of a layer (no separate gather
 * and qg GEMM). D <= 1024. */
int rf_global_attn_fold_h_fwd(int dtype, int B, int Lp, int D, int H, const void* h, int ldh,
                              const void* wqg, const float* bqg, float q_scale, const void* wkg,
                              const float* bkg, const void* wvg, const float* bvg, const uint8_t* flags,
                              const int32_t* gidx, int gmax, void* workspace, void* out, int ld_out,
                              rf_stream_t stream);

/* rf_global_attn_fold_h_fwd in two halves on one workspace: stage 1 = the query_global
 * projection + the partial softmax over h (reads h, writes only the workspace), stage 2 = the
 * merge + value fold (reads only the workspace, writes the global rows of out); 3 = both. Lets
 * the caller read h while it is still cache-resident (right after the LayerNorm that wrote it)
 * and write out after the local attention has filled the other rows. */
int rf_global_attn_fold_h_stage(int stage, int dtype, int B, int Lp, int D, int H, const void* h, int ldh,
                                const void* wqg, const float* bqg, float q_scale, const void* wkg,
                                const float* bkg, const void* wvg, const float* bvg, const uint8_t* flags,
                                const int32_t* gidx, int gmax, void* workspace, void* out, int ld_out,
                                rf_stream_t stream);

/* Row gather: out[r] = x[b*Lp + gidx[b, g]] for r = b*gmax + g (zero rows for -1). Feeds
 * the query_global projection of the global rows (TF:972-982). */
int rf_gather_global_rows(int dtype, int B, int Lp, int D, int gmax, const void* x, int ldx,
                          const int32_t* gidx, void* out, rf_stream_t stream);

/* A8 helpers — 1 / max(||x_m||, eps) per row (torch cosine_similarity clamp, models.py:366). */
int rf_row_inv_norm(int dtype, int M, int D, const void* x, int ldx, float eps, float* out,
                    rf_stream_t stream);

/* A8 sampled candidates — similarity_score with candidates (models.py:539-545):
 * s[b,c] = <z_b, E[cand[b,c]]> * rz[b] * re[cand[b,c]] * inv_temp. */
int rf_cos_score_cand(int dtype, int B, int C, int D, const void* z, int ldz, const float* rz,
                      const void* items, int ldi, const float* ri, const int64_t* cand,
                      float inv_temp, float* scores, rf_stream_t stream);

/* A9/A10 losses — torch CrossEntropyLoss rows (models.py:494-510 contrastive + MLM, :589-597
 * SeqRec): loss[m] = logsumexp(x[m, :N]) - x[m, label[m]] in fp32 (0 where label == ignore_index;
 * the caller divides the sum by the non-ignored count, as mean reduction does); optional
 * argmax[m] (first maximum, torch.argmax) for cl_correct_num (models.py:497). ldx in elements. */
/* Backward of the cosine scoring head (Similarity, models.py:358-369; the CrossEntropyLoss over
 * it, models.py:583-599): for logits s[b, c] = inv_temp (z_b . t_n) rz_b ri_n, n = c (cand == NULL,
 * the full catalog) or n = cand[b * C + c] (sampled softmax), and their gradient g = dL/ds (B x C
 * fp32), writes
 *   dz_b = rz_b (inv_temp sum_c g_bc ri_n t_n - (sum_c g_bc s_bc) rz_b z_b)      (B x D fp32).
 * z / items in dtype (fp32, bf16, fp16), rz / ri the inverse norms the forward used; ws holds
 * rf_cos_score_bwd_workspace(B, C, D) bytes. Two launches, fixed-order sums (deterministic). */
size_t rf_cos_score_bwd_workspace(int B, int C, int D);
int rf_cos_score_bwd(int dtype, int B, int C, int D, const void* z, int ldz, const float* rz, const void* items,
                     int ldi, const float* ri, const int64_t* cand, float inv_temp, const float* g, int64_t ldg,
                     const float* s, int64_t lds, void* ws, float* dz, int64_t lddz, rf_stream_t stream);
int rf_cross_entropy_fwd(int dtype, int M, int N, const void* logits, int64_t ldx, const int64_t* labels,
                         int64_t ignore_index, float* loss, int32_t* argmax, rf_stream_t stream);
/* Its gradient w.r.t. the logits for the mean loss (the LM-head decoder's backward, models.py:499-510):
 * dlogits[m, c] = (softmax(x_m)[c] - [c == labels[m]]) * grad_scale[0] (device scalar: upstream
 * gradient / counted rows), 0 for rows labelled ignore_index; dlogits in the logits' dtype. */
int rf_cross_entropy_bwd(int dtype, int M, int N, const void* logits, int64_t ldx, const int64_t* labels,
                         int64_t ignore_index, const float* grad_scale, void* dlogits, int64_t ldd,
                         rf_stream_t stream);

/* Ranker (utils.py:76-108) counts over a block of fp32 scores (M rows x N columns, ld):
 * gt[m] += #{n: s[m,n] > s_label[m]} (the strict rank), valid[m] += #{n: s[m,n] > -max_val}
 * (valid_length), and, if sexp != NULL, sexp[m] += sum_n exp(s[m,n] - shift) (log-sum-exp of
 * cosine/temp rows with |s| <= shift, for the CE without a row max). Accumulates with atomics,
 * so a catalog can be scored in column blocks (never the whole (B, N) matrix) — §8f row 1. */
int rf_rank_accum(int M, int N, const float* scores, int64_t ld, const float* s_label, float max_val,
                  float shift, int32_t* gt, int32_t* valid, float* sexp, rf_stream_t stream);

/* C5 catalog retrieval with a fused ranking epilogue (Ranker utils.py:76-108
 * over Similarity(z, E) / temp, models.py:358-369): the (B, N) score matrix is never written.
 * dtype RF_BF16 or RF_F16 (fp32 scores); q (B, D) queries and items (Nshard, D) one catalog shard,
 * D % 32 == 0, with fp32 inverse norms rq / ri (rf_row_inv_norm); item ids are idx_base + shard row.
 *
 * rf_label_scores: s_label[b] = cos(q_b, items[labels[b] - label_base]) * inv_temp for labels inside
 * the shard, 0 otherwise (sum over shards = the label score) — bit-identical to the score
 * rf_score_rank computes for that column.
 * rf_score_rank: shard rows [col0, col0 + ncols) in 256 x 256 tiles (rf_score_rank_tiles(ncols) tile
 * columns); per tile column t and row b writes part_cnt[(tn0 + t) * B + b] = #{s > s_label[b]} |
 * #{s > -max_val} << 16 and part_sexp[...] = sum exp(s - shift) (shift >= max |s|). mode 0 also
 * writes the scores to dense (B x ncols, ldd); mode 1 appends the scores s >= tau[b] with their item
 * ids to the row's list cval / cidx[b * capr + j], j < rcnt[b] (rcnt zeroed by the caller; it exceeds
 * capr when the list or a tile's 32-entry stage overflowed); mode 2 writes only the partials.
 * D % 64 == 0 (D >= 128) with the knob rank_w32 on: both entry points run the 32x32x16 four-wave
 * kernels (items as the MFMA A operand; k_rank_w32 / k_label_score32, still bit-identical to each
 * other); then mode 0 needs ldd >= ncols rounded up to 256, and mode 1 appends each candidate straight
 * to its row's list with one atomic (no per-tile stage): a row overflows only when its list passes
 * capr (rcnt > capr).
 * rf_rank_reduce: gt / valid / sexp per row = the partials summed over ntiles tile columns in order.
 * rf_topk_dense: top-k (k <= 256) of each row of a dense (B, n <= 2048) block, value descending, ties
 * by lower id (ids from idx (B, n) or idx_base + column).
 * rf_topk_merge: top-k of each row over a seed list (v0 / i0, B x k0; id < 0 skipped) and the row's
 * candidate list (mode 1); a row whose list overflowed keeps its seed list and gets overflow[b] = 1
 * (never cleared: re-rank such rows densely). */
int rf_label_scores(int dtype, int B, int D, const void* q, int ldq, const float* rq, const void* items, int ldi,
                    const float* ri, int nshard, const int64_t* labels, int64_t label_base, float inv_temp,
                    float* s_label, rf_stream_t stream);
int rf_score_rank(int dtype, int mode, int B, int D, const void* q, int ldq, const float* rq, const void* items,
                  int ldi, const float* ri, int col0, int ncols, float inv_temp, const float* s_label,
                  float max_val, float shift, const float* tau, float* dense, int64_t ldd, float* cval,
                  int32_t* cidx, int32_t* rcnt, int capr, int32_t idx_base, int32_t* part_cnt, float* part_sexp,
                  int tn0, rf_stream_t stream);
int rf_score_rank_tiles(int ncols);
int rf_rank_reduce(int B, int ntiles, const int32_t* part_cnt, const float* part_sexp, int32_t* gt,
                   int32_t* valid, float* sexp, rf_stream_t stream);
int rf_topk_dense(int B, int n, const float* vals, int64_t ldv, const int32_t* idx, int64_t ldi, int32_t idx_base,
                  int k, float* out_v, int32_t* out_i, rf_stream_t stream);
int rf_topk_merge(int B, int k0, const float* v0, const int32_t* i0, const float* cval, const int32_t* cidx,
                  const int32_t* rcnt, int capr, int k, float* out_v, int32_t* out_i, int32_t* overflow,
                  rf_stream_t stream);

/* AdamW over all of an optimizer's parameter tensors in one launch (torch.optim.AdamW as the
 * reference's drivers use it: optimization.py:28-32, litmodels.py:42-56). One descriptor per fp32
 * tensor (device memory); block_tensor[b] names the descriptor workgroup b updates — a tensor of n
 * elements owns ceil(n / rf_adamw_chunk()) consecutive workgroups starting at its first_block.
 *   p <- p decay;  m <- lerp(m, g, w1);  v <- beta2 v + w2 g^2;
 *   p <- p - step_size m / (sqrt(v) / bias_correction2_sqrt + eps)
 * with decay = 1 - lr weight_decay, w1 = 1 - beta1, w2 = 1 - beta2 (rounded from double on the host,
 * as torch passes them). step == NULL: step_size = lr / (1 - beta1^t) and bias_correction2_sqrt
 * are the host's (torch's non-capturable AdamW); otherwise both are computed on the device from the
 * step count *step (already advanced), so a captured optimizer step needs no host values.
 * hyper != NULL (capturable groups): lr = hyper[0] and decay = hyper[1] are read on the device — the
 * group's learning rate lives in device memory the host updates between graph replays (an LR
 * scheduler's value reaches a captured step, as torch's capturable AdamW with a Tensor lr). */
typedef struct rf_adamw_tensor {
  float* param;
  float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  const float* step;
  const float* hyper;
  int64_t numel;
  int64_t first_block;
  float decay, beta1, w1, beta2, w2, eps, lr, step_size, bias_correction2_sqrt;
  int32_t maximize;
} rf_adamw_tensor; /* 104 bytes */
int rf_adamw_chunk(void);
int rf_adamw_step(const rf_adamw_tensor* tensors, int ntensors, const int32_t* block_tensor, int nblocks,
                  rf_stream_t stream);
/* The same under a gradient scaler (torch.amp.GradScaler driving an optimizer with
 * _step_supports_amp_scaling, finetune.py:116-126 / lightning precision=16): grad_scale != NULL
 * divides every gradient by *grad_scale before the update (the scaler's unscale, fused); found_inf
 * != NULL and *found_inf != 0 skips the whole step — no parameter or moment is written, as
 * GradScaler skips optimizer.step() on an inf/NaN gradient. Both are device scalars, so the step
 * needs no host read and can be captured. */
int rf_adamw_step_amp(const rf_adamw_tensor* tensors, int ntensors, const int32_t* block_tensor, int nblocks,
                      const float* grad_scale, const float* found_inf, rf_stream_t stream);

/* Training-step weight packing (autocast's per-op weight casts, finetune.py:106-110): every
 * descriptor's fp32 source (rows x cols, row-major, lda) rounded to the compute dtype (RF_BF16 /
 * RF_F16) at row row_off of dst (ld_dst elements, may be NULL) and, if dstT is not NULL, transposed
 * at column row_off of dstT (ld_T), the first scale_n source rows of the transposed copy multiplied
 * by t_scale after rounding. One launch: workgroup b packs 64 x 64 tile b - first_tile of
 * descriptor block_entry[b] (a descriptor owns ceil(rows/64) * ceil(cols/64) consecutive blocks). */
typedef struct rf_pack_entry {
  const float* src;
  void* dst;
  void* dstT;
  int64_t lda, ld_dst, ld_T;
  int64_t first_tile;
  int32_t rows, cols, row_off, scale_n;
  float t_scale;
  int32_t pad_;
} rf_pack_entry; /* 80 bytes */
int rf_pack_weights(int dtype, const rf_pack_entry* entries, int nentries, const int32_t* block_entry, int nblocks,
                    rf_stream_t stream);

/* Training backward of the global rows through the fold (autograd of TF:964-1057; closed form of
 * train._global_bwd) in one pass over h, from the forward's fold workspace (rf_global_attn_fold_fwd_drop
 * with the same arguments; kept between forward and backward). dw: (B*gmax, 16, D) fp32 = Wvg_h^T do_h
 * per head (heads >= H zero); cb: (B*gmax, 16) fp32 = do_h . bvg_h (attention dropout only, else NULL).
 * Outputs: dh (B*Lp rows, lddh, 16-bit) = the global branch's gradient of h; du (B*gmax, 16, D) fp32
 * (dq = Wkg du, dWkg = q du^T per head); w (B*gmax, 16, D) fp32 = sum_j p'_j h_j (dWvg = do w^T);
 * stats (B*gmax, 16, 4) fp32 = (M, 1/L, Delta, S'), S' = sum_j p'_j (dbvg = do S'). 16-bit, D a multiple
 * of 128 up to 768, gmax <= 4. Workspace: rf_global_fold_bwd_workspace bytes. */
size_t rf_global_fold_bwd_workspace(int B, int Lp, int D, int gmax);
int rf_global_fold_bwd(int dtype, int B, int Lp, int D, int H, const void* h, int ldh, const uint8_t* flags,
                       const int32_t* gidx, int gmax, const void* fwd_workspace, const float* dw, const float* cb,
                       float p_drop, uint64_t seed, void* dh, int lddh, float* du, float* w, float* stats,
                       void* workspace, rf_stream_t stream);

/* The whole global-branch backward of one attention layer (the autograd of TF:964-1057 for the global
 * query rows and the key_global / value_global weights), from the attention output gradient: do_h is
 * read at the global rows of dout (B*Lp rows, lddout, 16-bit; empty slots contribute 0), dw_h = Wvg_h^T
 * do_h and c_h = do_h . bvg_h are formed inside, then rf_global_fold_bwd's pass over h (dh written),
 * then dqg (B*gmax, D) fp32 = per head Wkg_h du_h, dWkg = sum_r qg_r du_r^T and dWvg = sum_r do_r w_r^T
 * (D x D fp32, written, not accumulated), dbvg = sum_r do_r S'_r (D fp32) and dbkg = 0 (D fp32, may be
 * NULL; softmax-invariant). qg: the forward's scaled query_global rows (B*gmax, ldqg, 16-bit); wkg / wvg:
 * the (D x D) key_global / value_global weights in the compute dtype. Same shapes and limits as
 * rf_global_fold_bwd, B*gmax <= 1024. Workspace: rf_global_fold_bwd_full_workspace bytes. */
size_t rf_global_fold_bwd_full_workspace(int B, int Lp, int D, int gmax);
int rf_global_fold_bwd_full(int dtype, int B, int Lp, int D, int H, const void* h, int ldh, const uint8_t* flags,
                            const int32_t* gidx, int gmax, const void* fwd_workspace, const void* dout, int lddout,
                            const void* qg, int ldqg, const void* wkg, const void* wvg, const float* bvg, float p_drop,
                            uint64_t seed, void* dh, int lddh, float* dqg, float* dwkg, float* dwvg, float* dbvg,
                            float* dbkg, void* workspace, rf_stream_t stream);

/* Gradient of the global-key / global-value rows of the local branch (the key / value projections at
 * the global positions, TF:562-575 under autograd): with gds / gpr the band backward's (B, H, Lp, gmax)
 * fp32 dS / P columns of the global keys (rf_band_attn_bwd_drop),
 *   dk[b*Lp + gidx[b][g]][h*64+d] += sum_i gds[b][h][i][g] q[b*Lp+i][h*64+d]
 *   dv[b*Lp + gidx[b][g]][h*64+d] += sum_i gpr[b][h][i][g] dout[b*Lp+i][h*64+d]
 * in place (16-bit dk / dv, e.g. column views of the fused dqkv), fp32 accumulation in a fixed order;
 * empty slots (gidx < 0) skipped. Replaces the reference's gather of the global key / value rows'
 * gradients through autograd (and a batched product plus a scatter). */
int rf_global_kv_grad(int dtype, int B, int Lp, int H, int gmax, const float* gds, const float* gpr, const void* q,
                      int ldq, const void* dout, int lddout, const int32_t* gidx, void* dk, int ldk, void* dv,
                      int ldv, rf_stream_t stream);

/* Backward of the query_global projection of the global rows, qg = (h_g Wqg^T + bqg) * q_scale
 * (TF:966-967 under autograd), from dqg (B*gmax, D) fp32 (rf_global_fold_bwd_full; rows of empty slots
 * ignored): dWqg (D x D) and dbqg (D) fp32 written, and dh (B*Lp rows, lddh, 16-bit) += dqg . Wqg * q_scale
 * at the global rows, in place. wqgT: the (D x D) transposed weight Wqg^T * q_scale in the compute dtype
 * (the training path's packed copy); h: the layer input (B*Lp rows, ldh). B*gmax <= 1024. */
int rf_global_query_bwd(int dtype, int B, int Lp, int D, int gmax, const int32_t* gidx, const float* dqg,
                        float q_scale, const void* h, int ldh, const void* wqgT, float* dwqg, float* dbqg, void* dh,
                        int lddh, rf_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* RECFORMER_HIP_H */
