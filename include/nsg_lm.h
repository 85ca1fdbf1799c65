/*
 * nsg_lm.h -- batch-invariant decode-step kernels of the batched GPT-2 forward (row a19 of SURVEY.md §8),
 * part of `libnsgcoder.so`.
 *
 * Replace, for the decode steps of the reference's per-token forward
 * `model(prev, past_key_values=past, position_ids=...)` (code_base/arithmetic.py:115-122, Hugging Face
 * GPT2Block: ln_1 -> c_attn -> attention -> c_proj (+ residual) -> ln_2 -> c_fc -> gelu_new -> c_proj
 * (+ residual); ln_f; lm_head), the PyTorch/hipBLASLt ops whose per-row results depend on the batch size (the
 * library picks a GEMM kernel per M).  The arithmetic coder needs the DECODER to see bit-identical logits to
 * the ENCODER, and a cover made in a batch of B streams is often revealed alone (B = 1): every kernel here
 * computes a row's result in an order that does not depend on M, on the row's position in the batch or on the
 * tile shape chosen for M:
 *
 *   ns_lm_gemm       Y = epilogue(X . Wt^T + bias): one MFMA instruction (v_mfma_f32_16x16x32_f16) for every
 *                    shape, output element (m, n) at MFMA position (n mod 16, m mod 16); K cut by K ALONE
 *                    into 1, 2 or 4 consecutive ranges (K <= 1024 / <= 2048 / larger), each accumulated in
 *                    ascending 32-wide steps into one fp32 chain from zero, the chains added in order; the
 *                    tile (16 x 16..64 direct loads for small M, 64x64 .. 256x128 LDS tiles for large M)
 *                    changes only WHICH wave computes an element, never how.
 *   ns_lm_layernorm  one wavefront per row, fixed per-lane order + xor butterfly for mean and variance.
 *   ns_lm_embed_ln   h = wte[token] + wpe[pos] (fp16) and ln_1(h) in one pass (pos = L mod n_positions,
 *                    code_base/arithmetic.py:44-48; L from the host or from device memory for graph replays).
 *
 * fp16 operands, fp32 accumulation; no allocation; stream-ordered on the caller's hipStream_t.  Returns 0 or a
 * negative NS_ERR_* code of nsg_coder.h.
 */
#ifndef NSG_LM_H
#define NSG_LM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NS_LM_EPI_STORE 0    /* y = fp16(acc + bias)                                   */
#define NS_LM_EPI_GELU 1     /* y = fp16(gelu_tanh(acc + bias))   (GPT-2 "gelu_new")   */
#define NS_LM_EPI_RESIDUAL 2 /* y = fp16(y + (acc + bias)), in place (the residual add) */
#define NS_LM_EPI_STORE_F32 3 /* y (fp32) = acc + bias                                   */

/* d_x fp16 [M, ldx] (rows = streams), d_wt fp16 [N, ldw] (the weight TRANSPOSED: row n holds output column
 * n's K coefficients), d_bias fp16 [N] or NULL, d_y [M, ldy] fp16 (fp32 for NS_LM_EPI_STORE_F32).  K must be a
 * multiple of 64 and N a multiple of 16; rows 16-byte aligned (ldx, ldw multiples of 8 elements, ldy of 4). */
int ns_lm_gemm(const void* d_x, int64_t ldx, const void* d_wt, int64_t ldw, const void* d_bias, void* d_y,
               int64_t ldy, int M, int N, int K, int epilogue, void* hip_stream);

/* ns_lm_gemm with a forced tile configuration 0 <= config < ns_lm_gemm_configs() (-1 = the automatic choice):
 * direct 16/32/64-row waves, 64x64 / 128x128 / 256x128 / 128x256 LDS tiles with 2-4 stages.  Every
 * configuration produces the same bits (the batch-invariance contract); the choice is speed only (tuning and
 * tests). */
int ns_lm_gemm_config(const void* d_x, int64_t ldx, const void* d_wt, int64_t ldw, const void* d_bias, void* d_y,
                      int64_t ldy, int M, int N, int K, int epilogue, int config, void* hip_stream);
int ns_lm_gemm_configs(void);

/* d_x fp16 [M, ldx] -> d_y fp16 [M, ldy] = (x - mean) / sqrt(var + eps) * w + b per row; C % 4 == 0,
 * C <= 2048. */
int ns_lm_layernorm(const void* d_x, int64_t ldx, const void* d_w, const void* d_b, void* d_y, int64_t ldy, int M,
                    int C, float eps, void* hip_stream);

/* ns_lm_layernorm that also advances the int32 *d_counter by one (when not NULL) in the same launch: the decode
 * step's final layer norm moves the device-side cache length (ns_lm_embed_ln / attention d_L) to the next step
 * without a launch of its own.  Round 5. */
int ns_lm_layernorm_count(const void* d_x, int64_t ldx, const void* d_w, const void* d_b, void* d_y, int64_t ldy,
                          int M, int C, float eps, int32_t* d_counter, void* hip_stream);

/* ns_lm_layernorm of d_x (C = K; ln_w, ln_b) followed by ns_lm_gemm of the normalised rows, in ONE launch when
 * the GEMM is a small-batch one (M <= 16, K <= 1024: every workgroup normalises the M rows into LDS with the
 * layernorm kernel's arithmetic, bit-identical), else the two kernels with d_a fp16 [M, lda] as the normalised
 * rows.  Same bits either way (the decode step at B = 1 is bound by launch latency: 24 launches fewer). */
int ns_lm_ln_gemm(const void* d_x, int64_t ldx, const void* d_ln_w, const void* d_ln_b, float eps, const void* d_wt,
                  int64_t ldw, const void* d_bias, void* d_y, int64_t ldy, int M, int N, int K, int epilogue,
                  void* d_a, int64_t lda, void* hip_stream);

/* d_tokens int32 [M]; d_wte fp16 [V, C]; d_wpe fp16 [n_positions, C]; position = L mod n_positions with
 * L = *d_L (int32, device) when d_L is not NULL, else the host value.  Writes d_h fp16 [M, ldh] = wte + wpe
 * and d_a fp16 [M, lda] = layernorm(h; w, b, eps).  Token ids outside [0, V) write NaN rows (the caller
 * validates ids on the host; the kernel never reads outside the table). */
int ns_lm_embed_ln(const int32_t* d_tokens, const void* d_wte, const void* d_wpe, int V, int n_positions, int L,
                   const int32_t* d_L, void* d_h, int64_t ldh, const void* d_w, const void* d_b, void* d_a,
                   int64_t lda, int M, int C, float eps, void* hip_stream);

/* ns_lm_embed_ln with a cache length PER ROW: row b takes position d_lens[b] mod n_positions (int32 [M], device;
 * code_base/arithmetic.py:44-48 per message).  The paged decode step with slot refill (round 6). */
int ns_lm_embed_ln_rows(const int32_t* d_tokens, const void* d_wte, const void* d_wpe, int V, int n_positions,
                        const int32_t* d_lens, void* d_h, int64_t ldh, const void* d_w, const void* d_b, void* d_a,
                        int64_t lda, int M, int C, float eps, void* hip_stream);

/* ns_lm_layernorm that also advances d_lens[row] by one for every row (int32 [M]) in the same launch: the paged
 * decode step's ln_f moves every stream's cache length after all its attention layers have read it. */
int ns_lm_layernorm_rows(const void* d_x, int64_t ldx, const void* d_w, const void* d_b, void* d_y, int64_t ldy,
                         int M, int C, float eps, int32_t* d_lens, void* hip_stream);

/* ns_lm_embed_ln for M = B*T rows of whole sequences: row b*T + t takes position t mod n_positions (the default
 * positions of a first forward call: the context prefill, the guard's scoring forward, the max_context window). */
int ns_lm_embed_seq_ln(const int32_t* d_tokens, const void* d_wte, const void* d_wpe, int V, int n_positions, int T,
                       void* d_h, int64_t ldh, const void* d_w, const void* d_b, void* d_a, int64_t lda, int M, int C,
                       float eps, void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* NSG_LM_H */
