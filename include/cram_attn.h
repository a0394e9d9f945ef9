/*
 * cram_attn.h — C-ABI of the MI355X (gfx950) credibility-biased attention library.
 *
 * This is the drop-in boundary for CrAM's credibility re-weighting hot path.
 * In the reference the path is a Python forward-pre-hook that rewrites the
 * dense attention mask of every selected (layer, head):
 *
 *   /root/reference/utils/re_weighting.py:36-61   Re_Weighting_Strategy.edit_attention_mask
 *       mask[0,h,i,j] = dtype(log_fp16(w_j))  for causal-allowed (i, j), j < W, h in head_idx
 *   /root/reference/utils/re_weighting.py:118-124 hook registration (generate path)
 *   /root/reference/utils/re_weighting.py:163-168 hook registration (IE sweep path)
 *
 * and the attention op the mask then flows into (transformers 5.15
 * sdpa_attention_forward -> F.scaled_dot_product_attention).  Here the mask is
 * never materialised: the kernels take an O(S) per-key bias vector plus an O(Hq)
 * per-head enable mask and add  enable[b,h] * bias[b,j]  (for j < W) to the
 * scaled QK^T scores inline.
 *
 * Conventions
 *   - all tensor pointers are DEVICE pointers owned by the caller; no entry
 *     point allocates, frees or synchronises;
 *   - q/k/v/o (and every other 16-bit tensor) are bf16 or fp16, named by the
 *     `dtype` argument (CRAM_DTYPE_*: the model's torch_dtype, which the
 *     reference loads with dtype="auto" -> bf16 for Llama-3 / Qwen2, fp16 for
 *     Llama-2, re_weighting.py:22); last dimension contiguous, every stride
 *     given in ELEMENTS and a multiple of 8, every base pointer 16-byte aligned;
 *   - bias is fp32 [B][bias_sb] in natural-log units (the hook's
 *     dtype(log_fp16(w)) already widened to fp32); enable is uint8 [B][en_sb];
 *     a NULL bias or NULL enable means "no re-weighting" (plain causal);
 *   - work is enqueued on `stream` (a hipStream_t; NULL = default stream);
 *   - every entry point returns CRAM_OK (0) or a negative CRAM_ERR_* code and
 *     never aborts; cram_strerror() names the code.
 */
#ifndef CRAM_ATTN_H
#define CRAM_ATTN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRAM_OK 0
#define CRAM_ERR_INVALID_ARG -1   /* null pointer, non-positive size, Hq % Hkv != 0 ... */
#define CRAM_ERR_UNSUPPORTED -2   /* head dim not in {64,128}, GQA group size or dtype not supported */
#define CRAM_ERR_ALIGNMENT -3     /* stride not a multiple of 8 elements / pointer not 16-B aligned */
#define CRAM_ERR_LAUNCH -4        /* hipLaunchKernel failed */
#define CRAM_ERR_WORKSPACE -5     /* split-S workspace missing or too small */

#define CRAM_ABI_VERSION 8        /* 2: dtype argument on every tensor entry point; 3: kernel-selection knobs;
                                     4: cram_get_knob(which, *value), decode projection GEMM;
                                     5: cram_gemm_residual, cram_gemm_rope, cram_gemm_splitk_residual;
                                     6: cram_gemm_small; 7: cram_attn_prefill_varlen_cached;
                                     8: cram_attn_decode_shared */

#define CRAM_DTYPE_BF16 0
#define CRAM_DTYPE_F16 1

typedef void* cram_stream_t; /* hipStream_t */

const char* cram_strerror(int code);
int cram_abi_version(void);

/*
 * Process-wide kernel-selection knobs (A/B runs and tests; the product default is automatic = -1).
 * The initial values are read once from the environment (CRAM_PREFILL_VARIANT, CRAM_DECODE_U, CRAM_DECODE_MFMA,
 * CRAM_GEMM_VARIANT) at
 * the first query (once per process, thread-safe); no launch reads the environment.  Knob values are atomics:
 * a value set from one thread is seen by launches issued afterwards from any thread.
 *   CRAM_KNOB_PREFILL_VARIANT  -1 = automatic: 64-key tiles, 4 waves, except GQA-7 groups with sequences <= 2048
 *                              (7-wave workgroups) and bf16 d = 128 GQA groups of 4k with >= 256 query rows (variant 4);
 *                              0 = always 4 waves; 3 = 32-key tiles; 8 = 8-wave workgroups;
 *                              7 = 7-wave workgroups for GQA-7 groups; 4 = two workgroups per CU, 32 rows per wave,
 *                              hand-ordered stream (bf16, d = 128, GQA groups of 4k; otherwise as 0).  (6, round 2's
 *                              one-wave-per-SIMD kernel, was removed in round 4: CRAM_ERR_INVALID_ARG)
 *   CRAM_KNOB_DECODE_U         -1 = by grid size; 1, 2, 4 = keys per lane group per iteration (VALU decode body)
 *   CRAM_KNOB_DECODE_MFMA      -1 / 1 = GQA groups of >= 4 heads at d = 128 decode on the matrix cores; 0 = VALU body
 *   CRAM_KNOB_GEMM_VARIANT     -1 = automatic: cram_gemm calls with >= 2 K-tiles and 16-byte output rows on the
 *                              4-wave 128 x 128-per-wave kernel (tile order by shape), others on the 8-wave kernel;
 *                              0 = the 8-wave kernel; 1 / 2 = the 4-wave kernel with weight-tile / activation-tile
 *                              groups (where it applies; otherwise as 0); cram_gemm_rope always runs the 4-wave
 *                              kernel
 * cram_set_knob returns CRAM_ERR_INVALID_ARG for an unknown knob or value; cram_get_knob stores the value in
 * *value and returns CRAM_OK, or CRAM_ERR_INVALID_ARG for an unknown knob / null pointer (ABI 4: the value -1,
 * "automatic", is never an error code).
 */
#define CRAM_KNOB_PREFILL_VARIANT 0
#define CRAM_KNOB_DECODE_U 1
#define CRAM_KNOB_DECODE_MFMA 2
#define CRAM_KNOB_GEMM_VARIANT 3
#define CRAM_KNOB_COUNT 4
int cram_set_knob(int which, int value);
int cram_get_knob(int which, int* value);

/*
 * Prefill / multi-token attention (replaces the hooked SDPA call for
 * q_len > 1; reference: re_weighting.py:39-59 mask build + sdpa_attention.py:154).
 *
 *   q : [B][Hq][Tq][d]   strides (q_sb, q_sh, q_st)
 *   k : [B][Hkv][S][d]   strides (k_sb, k_sh, k_st)
 *   v : [B][Hkv][S][d]   strides (v_sb, v_sh, v_st)
 *   o : [B][Hq][Tq][d]   strides (o_sb, o_sh, o_st)   (o[b,h,i,:] may alias a [B,Tq,Hq,d] buffer)
 *   query i sits at absolute position q_pos0 + i and attends keys j <= q_pos0 + i, j < S
 *   score(i,j) = scale * q_i . k_j + (enable[b*en_sb+h] ? bias[b*bias_sb+j] : 0 for j < W)
 */
int cram_attn_prefill(const void* q, int64_t q_sb, int64_t q_sh, int64_t q_st,
                      const void* k, int64_t k_sb, int64_t k_sh, int64_t k_st,
                      const void* v, int64_t v_sb, int64_t v_sh, int64_t v_st,
                      void* o, int64_t o_sb, int64_t o_sh, int64_t o_st,
                      int B, int Hq, int Hkv, int Tq, int S, int d, int q_pos0, float scale,
                      const float* bias, int64_t bias_sb, const uint8_t* enable, int64_t en_sb, int W,
                      int dtype, cram_stream_t stream);

/*
 * Packed variable-length prefill (batched reweighted decode: many prompts in one GEMM pass).
 * Sequence b occupies tokens [cu_seqlens[b], cu_seqlens[b+1]) of q/k/v/o, all laid out
 * [token][head][d] with strides (x_st per token, x_sh per head); each sequence is causal from 0;
 * bias row b applies to its own tokens.  max_len >= every sequence length.
 */
int cram_attn_prefill_varlen(const void* q, int64_t q_sh, int64_t q_st, const void* k, int64_t k_sh, int64_t k_st,
                             const void* v, int64_t v_sh, int64_t v_st, void* o, int64_t o_sh, int64_t o_st,
                             const int32_t* cu_seqlens, int B, int max_len, int Hq, int Hkv, int d, float scale,
                             const float* bias, int64_t bias_sb, const uint8_t* enable, int64_t en_sb, int W,
                             int dtype, cram_stream_t stream);

/*
 * (ABI 7) Packed prefill of prompt SUFFIXES whose keys sit in a KV cache behind a shared prefix (the batched decode's
 * prefill when every prompt starts with the same `prefix` tokens, computed once): sequence b's queries are tokens
 * [cu_seqlens[b], cu_seqlens[b+1]) of q / o ([token][head][d]) at absolute positions prefix + i; its keys / values
 * are rows 0 .. prefix + len_b - 1 of cache row b: k + b k_sb + j k_st + h k_sh (the prefix's rows, then its own,
 * already written).  Causal from the row's position; bias row b indexes absolute key positions.  max_len >= every
 * suffix length.  Same arithmetic as cram_attn_prefill_varlen over the whole prompts.
 */
int cram_attn_prefill_varlen_cached(const void* q, int64_t q_sh, int64_t q_st, const void* k, int64_t k_sb,
                                    int64_t k_sh, int64_t k_st, const void* v, int64_t v_sb, int64_t v_sh,
                                    int64_t v_st, void* o, int64_t o_sh, int64_t o_st, const int32_t* cu_seqlens,
                                    int B, int max_len, int prefix, int Hq, int Hkv, int d, float scale,
                                    const float* bias, int64_t bias_sb, const uint8_t* enable, int64_t en_sb, int W,
                                    int dtype, cram_stream_t stream);

/*
 * Single-token decode attention (replaces the hooked SDPA call for q_len == 1;
 * reference: re_weighting.py:42-44 decode mask + :57-59 bias fill).
 *
 *   q : [B][Hq][d] (q_sb, q_sh);  o : [B][Hq][d] (o_sb, o_sh)
 *   k, v : [B][Hkv][S_max][d] (k_sb, k_sh, k_st) / (v_sb, v_sh, v_st)
 *   seq_lens : device int32 [B] keys per batch row, or NULL -> every row has S keys
 *   num_splits > 1 splits the keys of each (b, kv head) over that many workgroups;
 *   it needs `workspace` of cram_attn_decode_workspace_size(B, Hq, d, num_splits) bytes.
 */
size_t cram_attn_decode_workspace_size(int B, int Hq, int d, int num_splits);
int cram_attn_decode(const void* q, int64_t q_sb, int64_t q_sh,
                     const void* k, int64_t k_sb, int64_t k_sh, int64_t k_st,
                     const void* v, int64_t v_sb, int64_t v_sh, int64_t v_st,
                     void* o, int64_t o_sb, int64_t o_sh,
                     int B, int Hq, int Hkv, int S, const int32_t* seq_lens, int d, float scale,
                     const float* bias, int64_t bias_sb, const uint8_t* enable, int64_t en_sb, int W,
                     int num_splits, void* workspace, size_t workspace_bytes,
                     int dtype, cram_stream_t stream);

/*
 * (ABI 8) cram_attn_decode for a batch whose rows share their first `shared_rows` keys (the prompt opening prefilled
 * once and copied into every cache row, cram_attn_prefill_varlen_cached): the caller guarantees keys / values
 * [0, shared_rows) are equal in every batch row; the matrix-core body then reads them (in whole 32-key blocks) from
 * batch row 0, one HBM stream for the batch instead of one per row.  Results are bit-identical to cram_attn_decode.
 * shared_rows = 0 is cram_attn_decode.
 */
int cram_attn_decode_shared(const void* q, int64_t q_sb, int64_t q_sh,
                            const void* k, int64_t k_sb, int64_t k_sh, int64_t k_st,
                            const void* v, int64_t v_sb, int64_t v_sh, int64_t v_st,
                            void* o, int64_t o_sb, int64_t o_sh,
                            int B, int Hq, int Hkv, int S, const int32_t* seq_lens, int d, float scale,
                            const float* bias, int64_t bias_sb, const uint8_t* enable, int64_t en_sb, int W,
                            int shared_rows, int num_splits, void* workspace, size_t workspace_bytes,
                            int dtype, cram_stream_t stream);

/*
 * Answer-token logits (replaces the full-vocab lm_head + gather of
 * re_weighting.py:159-160,169-170):  out[i] = sum_d hidden[i][d] * w_lm[ids[i]][d]
 * in fp32; round_logits != 0 rounds each logit to `dtype` first (transformers 5.15 returns
 * logits in the model dtype).
 *   hidden : [n][D] row stride h_rs;  w_lm : [V][D] row stride w_rs;  ids : int32 [n]
 */
int cram_answer_logits(const void* hidden, int64_t h_rs, const void* w_lm, int64_t w_rs,
                       const int32_t* ids, int n, int D, int round_logits, float* out,
                       int dtype, cram_stream_t stream);

/*
 * Fused elementwise kernels of the engine (cram_fused.hip), bf16 or fp16 (`dtype`), rows of 16-byte
 * aligned vectors; below, rnd() rounds to that dtype.
 * They keep transformers' rounding points (LlamaRMSNorm, apply_rotary_pos_emb, LlamaMLP), i.e. the
 * arithmetic the reference's hooked model runs between its GEMMs (re_weighting.py:127 -> generate,
 * :159/:169 -> model forward).
 *
 * cram_rmsnorm       y = rnd(w * rnd(h * rsqrt(mean(h^2) + eps))) per row; if residual != NULL then
 *                    h = rnd(x + residual) is also written to h_out, else h = x.
 * cram_rope_inplace  rotates the first `heads` heads (q then k) of every row of a fused QKV buffer in
 *                    place; row r uses position pos[r] (int64) or r % T when pos == NULL; cos/sin are
 *                    [P][d] tables of the same dtype (row stride tab_rs).
 * cram_rope_split    the same rotation over a q | k | v row (hq, hkv, hkv heads): q in place, k rotated into
 *                    kout (and also in place when keep_k) and v copied into vout.  Buffer row r goes to row
 *                    kv_row0 + r % T of sequence r / T (rows % T == 0), or, when dst_b is given, to row
 *                    kv_row0 + pos[r] of sequence dst_b[r] (int64); element strides kv_bs (sequence), kv_hs
 *                    (head), kv_rs (row).  Replaces the copies / index_put that placed the IE sweep's suffix K/V
 *                    behind their prefix and the packed decode prefill's K/V into the cache (cram_amd/engine.py)
 * cram_silu_mul      y[r, :F] = rnd(rnd(silu(gu[r, :F])) * gu[r, F:2F])
 */
int cram_rmsnorm(const void* x, int64_t x_rs, const void* residual, int64_t r_rs, void* h_out, int64_t h_rs,
                 const void* w, void* y, int64_t y_rs, int rows, int D, float eps, int dtype,
                 cram_stream_t stream);
int cram_rope_inplace(void* qkv, int64_t row_stride, int rows, int T, int heads, int d, const void* cos_t,
                      const void* sin_t, int64_t tab_rs, const int64_t* pos, int dtype, cram_stream_t stream);
int cram_rope_split(void* qkv, int64_t row_stride, int rows, int T, int hq, int hkv, int d, const void* cos_t,
                    const void* sin_t, int64_t tab_rs, const int64_t* pos, void* kout, void* vout, int64_t kv_bs,
                    int64_t kv_hs, int64_t kv_rs, int kv_row0, const int64_t* dst_b, int keep_k, int dtype,
                    cram_stream_t stream);
int cram_silu_mul(const void* gu, int64_t gu_rs, void* y, int64_t y_rs, int rows, int F, int dtype,
                  cram_stream_t stream);

/*
 * Projection GEMM of the engine (cram_gemm.hip; replaces F.linear / hipBLASLt for the sweep's and the packed
 * prefill's projections and the elementwise op next to each -- the MLP activation here, the residual add and RoPE
 * in cram_gemm_residual / cram_gemm_rope below: re_weighting.py:158,170 run them as nn.Linear inside every hooked
 * forward).
 *   out[m, n] = sum_k y[m, k] * x[n, k]      y: activations [M][K] (row stride ldy), x: weights [N][K] (ldx),
 *   fp32 accumulation, bf16 / fp16 in and out; N % 256 == 0, K % 64 == 0, 16-byte aligned rows, any M >= 1.
 *   CRAM_GEMM_STORE      out [M][N] (ldo) = rnd(acc)
 *   CRAM_GEMM_SILU_MUL   x is a gate/up weight with rows interleaved in blocks of 32 (rows 64j..64j+31 = gate rows
 *                        32j.., rows 64j+32..64j+63 = up rows 32j..); out [M][N/2] (ldo):
 *                        out[m, f] = rnd(rnd(silu(rnd(gate))) * rnd(up)), cram_silu_mul's arithmetic
 */
#define CRAM_GEMM_STORE 0
#define CRAM_GEMM_SILU_MUL 1
#define CRAM_GEMM_SILU_MUL_CAT 2
int cram_gemm(const void* y, int64_t ldy, const void* x, int64_t ldx, void* out, int64_t ldo, int M, int N, int K,
              int epilogue, int dtype, cram_stream_t stream);

/*
 * The q | k | v projection with RoPE in its epilogue (LlamaAttention.forward's q_proj / k_proj / v_proj followed by
 * apply_rotary_pos_emb, re_weighting.py:158,170 via the hooked forward): cram_gemm with N = (hq + 2 hkv) * d, then
 * on the rounded projection exactly cram_rope_split's arithmetic, table row pos[m] (or pos0 + m % T: the IE
 * sweep's suffix rows, whose positions continue a shared prefix of pos0 tokens, need no position array):
 *   kout == vout == NULL: cram_rope_inplace over the q and k heads (v heads stored as computed), all in out;
 *   otherwise cram_rope_split: q rotated into out, k rotated into kout, v copied into vout; buffer row m < rows goes
 *   to sequence m / T, row kv_row0 + m % T, or with dst_b to dst_b[m], kv_row0 + pos[m] (strides kv_bs / kv_hs /
 *   kv_rs, elements); the k / v columns of out hold the rotated k and v if keep_k, else they are not written.
 * Rows in [rows, M) are GEMM padding: out rows written (q), nothing else.  bf16 / fp16, d = 128, K % 64 == 0,
 * K >= 128 (the 4-wave kernel), ldo % 8 == 0; pos / dst_b int64 device arrays of >= rows entries.  bias [N]
 * (16-byte aligned; Qwen2's q / k / v) or NULL: the projection is rnd(acc + bias), F.linear's rounding, before RoPE.
 * Part of the fused weight: hq = 0 (y = the k | v rows: K / V only) or hkv = 0 (y = the q rows; no kout).
 */
int cram_gemm_rope(const void* y, int64_t ldy, const void* x, int64_t ldx, const void* bias, void* out, int64_t ldo,
                   int M, int K, int rows, int T, int hq, int hkv, int d, const void* cos_t, const void* sin_t,
                   int64_t tab_rs, const int64_t* pos, int pos0, void* kout, void* vout, int64_t kv_bs, int64_t kv_hs,
                   int64_t kv_rs, int kv_row0, const int64_t* dst_b, int keep_k, int dtype, cram_stream_t stream);

/*
 * The same GEMM with the decoder layer's residual add in its epilogue (o_proj and down_proj: the residual
 * stream h = h + o_proj(a), h = h + down(act) of LlamaDecoderLayer.forward, re_weighting.py:158,170 via the hooked
 * forward): out[m, n] = rnd(res[m, n] + rnd(sum_k y[m, k] * x[n, k])) -- the bf16 add HF runs after the projection.
 * res [M][N] (row stride ldr) may be out itself (same pointer and stride); any other overlap is CRAM_ERR_INVALID_ARG.
 * Requirements of cram_gemm plus ldo % 8 == 0, ldr % 8 == 0 and a 16-byte aligned res.
 */
int cram_gemm_residual(const void* y, int64_t ldy, const void* x, int64_t ldx, const void* res, int64_t ldr, void* out,
                       int64_t ldo, int M, int N, int K, int dtype, cram_stream_t stream);

/*
 * Split-K form of the same GEMM for the decode step's projections (few activation rows, M = the batch: 256 at
 * config 2, 16 at config 5; re_weighting.py:127-132 runs them inside generate, one token per step).  K is cut into
 * `splits` equal ranges (K % (64 * splits) == 0), every (256 x 256 output tile, K range) is one workgroup writing
 * fp32 partial sums to the caller's workspace [splits][M][N] (cram_gemm_splitk_workspace_size bytes, 16-B
 * aligned), and a combine pass adds the ranges in range order (deterministic: no atomics) and applies
 *   CRAM_GEMM_STORE         out [M][N] (ldo) = rnd(sum + bias[n])   (bias [N] or NULL: nn.Linear with bias)
 *   CRAM_GEMM_SILU_MUL_CAT  x = [gate; up] rows as the checkpoint stores them ([2F][K], F = N / 2);
 *                           out [M][F] (ldo) = rnd(rnd(silu(rnd(g))) * rnd(u)), cram_silu_mul's arithmetic
 * Same requirements as cram_gemm plus ldo % 8 == 0; returns CRAM_ERR_WORKSPACE for a missing / short workspace.
 */
size_t cram_gemm_splitk_workspace_size(int M, int N, int splits);
int cram_gemm_splitk(const void* y, int64_t ldy, const void* x, int64_t ldx, void* out, int64_t ldo, int M, int N,
                     int K, int splits, int epilogue, const void* bias, void* workspace, size_t ws_bytes, int dtype,
                     cram_stream_t stream);

/*
 * The decode step's projections (ABI 6): the same GEMM on 128 x 128 output tiles for few activation rows (M = the
 * decode batch, ~128-512: re_weighting.py:127-132 runs q/k/v, o_proj, the MLP and lm_head inside generate, one token
 * per row per step), where 256 x 256 tiles leave most CUs idle; a four-deep LDS ring keeps three K-tiles of the
 * weights (streamed from HBM once per step) in flight.  K is cut into `splits` equal ranges (K % (64 * splits) == 0);
 * splits > 1 writes fp32 partial sums to the workspace ([splits][M][N], cram_gemm_splitk_workspace_size bytes,
 * 16-B aligned) and combines them in range order (deterministic).
 *   CRAM_GEMM_STORE      out [M][N] (ldo) = rnd(acc + bias[n])   (bias [N], 16-B aligned, or NULL)
 *   CRAM_GEMM_SILU_MUL   x = the interleaved gate/up weight of cram_gemm; out [M][N/2] = the MLP activation
 * N % 128 == 0, 16-byte aligned rows, any M >= 1; ldo % 8 == 0 when splits > 1.
 */
int cram_gemm_small(const void* y, int64_t ldy, const void* x, int64_t ldx, const void* bias, void* out, int64_t ldo,
                    int M, int N, int K, int splits, int epilogue, void* workspace, size_t ws_bytes, int dtype,
                    cram_stream_t stream);

/*
 * Split-K with cram_gemm_residual's epilogue: out = rnd(res + rnd(sum)) (res may be out itself).  The engine runs the
 * sparse last wave of the sweep's o_proj / down_proj tiles through it (rows past the last whole wave of 256 x 256
 * tiles on the 256 CUs, cut into K ranges so they fill the chip) instead of leaving most CUs idle for one tile time.
 * Requirements of cram_gemm_splitk plus those of cram_gemm_residual on res / ldr.
 */
int cram_gemm_splitk_residual(const void* y, int64_t ldy, const void* x, int64_t ldx, const void* res, int64_t ldr,
                              void* out, int64_t ldo, int M, int N, int K, int splits, void* workspace,
                              size_t ws_bytes, int dtype, cram_stream_t stream);

/*
 * Host-side prompt -> credibility weights (cram_spans.cpp; no device, no stream), batched over B prompts.
 * Replaces the per-passage offset-mapping scan of re_weighting.py:100-111.
 *
 *   tok_start [cu_tok[B]]  character start of every token (offset_mapping[:, 0]), prompt b's tokens at
 *                          [cu_tok[b], cu_tok[b+1])
 *   char_lo/char_hi/score [cu_par[B]]  passage p of prompt b (p in [cu_par[b], cu_par[b+1])): index of
 *                          "Passage-i: " in the prompt (prompt.find, re_weighting.py:102) and of its
 *                          trailing '\n' (:103); the passage's score as fp32
 *   span_lo/span_hi [cu_par[B]]  out: max{t : tok_start[t] <= char_lo} and max{t : tok_start[t] <= char_hi}
 *                          (token indices within the prompt, inclusive span, :105-109)
 *   w16 [cu_tok[B]]        out: fp16 bits, fp16(score) over each span (later passages overwrite), 1.0 elsewhere
 * Returns CRAM_ERR_INVALID_ARG for a passage that was not found (char_lo < 0) or precedes every token.
 */
int cram_passage_weights(int B, const int64_t* cu_tok, const int64_t* tok_start, const int64_t* cu_par,
                         const int64_t* char_lo, const int64_t* char_hi, const float* score,
                         int32_t* span_lo, int32_t* span_hi, uint16_t* w16);

#ifdef __cplusplus
}
#endif

#endif /* CRAM_ATTN_H */
