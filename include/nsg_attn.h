/*
 * nsg_attn.h -- decode-step attention of the batched GPT-2 forward (row a19 of SURVEY.md §8), part of
 * `libnsgcoder.so`.
 *
 * Replaces, for one new token per stream, the attention of the reference's per-token forward
 * `model(prev, past_key_values=past, position_ids=...)` (code_base/arithmetic.py:115-122, the Hugging Face
 * GPT2Attention over the whole unbounded cache: softmax(q k^T / sqrt(D)) v).  It fuses the KV append of
 * the new token with the attention over the cache: one wavefront per (stream, head) streams the K and V rows
 * of that head once from HBM (online softmax in fp32), so the step is HBM-bound at B*(L+1)*2*D*2 bytes per
 * layer.  A pair's rows are split over 1, 2, 4 or 8 waves by the key count alone (one wave up to 256 keys, eight
 * beyond 1,024), partials merged in wave order: the summation order -- and every output bit -- does not depend on
 * the batch size, so the decoder of a cover reproduces the encoder's logits at any B.  fp16 in and out, fp32
 * accumulation; no allocation, stream-ordered on the caller's hipStream_t.
 */
#ifndef NSG_ATTN_H
#define NSG_ATTN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One layer, one decode position.
 *   d_qkv     fp16 [B, qkv_stride]: q at columns [0, H*D), k at [H*D, 2*H*D), v at [2*H*D, 3*H*D) (the c_attn
 *             output of GPT-2, head h at columns h*D..h*D+D-1 of each part).
 *   d_k_cache, d_v_cache  fp16, element (b, h, j, d) at b*cache_b_stride + h*cache_h_stride + j*D + d.
 *   L0        positions already cached; the call writes the new k/v at position L0 and attends to
 *             positions 0..L0 (L0 + 1 keys).  The caller guarantees L0 < the cache's capacity.
 *   d_out     fp16 [B, out_stride]: head h of stream b at columns h*D..h*D+D-1.
 *   scale     the score scale (1/sqrt(D) for GPT-2).
 * D must be 64.  Returns 0, or a negative NS_ERR_* code of nsg_coder.h on bad arguments / launch failure. */
int ns_decode_attention(const void* d_qkv, int64_t qkv_stride, void* d_k_cache, void* d_v_cache,
                        int64_t cache_b_stride, int64_t cache_h_stride, int B, int H, int D, int L0, void* d_out,
                        int64_t out_stride, float scale, void* hip_stream);

/* The same with the cache length read from device memory (*d_L0, int32) when the kernel runs, so one captured
 * hipGraph serves every decode step; `cap` = the cache capacity in positions (a step with *d_L0 >= cap writes
 * and reads nothing). */
int ns_decode_attention_dev(const void* d_qkv, int64_t qkv_stride, void* d_k_cache, void* d_v_cache,
                            int64_t cache_b_stride, int64_t cache_h_stride, int B, int H, int D, const int32_t* d_L0,
                            int cap, void* d_out, int64_t out_stride, float scale, void* hip_stream);

/* The general form: positions [0, T0) are a prefix SHARED by all B streams (the common context, stored once:
 * element (h, j, d) at h*prefix_h_stride + j*D + d, j < T0), positions [T0, L0] are the stream's own rows at
 * index r = j - T0 of d_k_cache / d_v_cache, grouped in 32-row chunks: element (b, h, r, d) at
 * b*cache_b_stride + h*cache_h_stride + (r/32)*cache_chunk_stride + (r%32)*D + d.  cache_chunk_stride = 0 (or
 * 32*D) is the plain per-pair row-contiguous layout; a chunk-plane layout (cache_chunk_stride = B*H*32*D,
 * cache_b_stride = H*32*D, cache_h_stride = 32*D) keeps the rows every step reads dense in memory whatever
 * the cache's capacity (fewer pages touched).  `cap` = total positions (prefix + the stream cache's rows); the
 * new token is written at stream index L0 - T0.  L0 comes from *d_L0 when d_L0 is not NULL (graph replays),
 * else from the argument.  T0 = 0 is ns_decode_attention(_dev).  The output bits do not depend on where a
 * row is stored (same values, same order).  window > 0 (opt-in; 0 = the reference's unbounded attention) attends
 * to the last `window` positions only, [max(0, L0 + 1 - window), L0]: a sliding-window approximation that bounds
 * the per-step KV traffic (NOT the reference's max_context, which re-runs a trimmed context). */
int ns_decode_attention_prefix(const void* d_qkv, int64_t qkv_stride, void* d_k_cache, void* d_v_cache,
                               int64_t cache_b_stride, int64_t cache_h_stride, int64_t cache_chunk_stride,
                               const void* d_k_prefix, const void* d_v_prefix, int64_t prefix_h_stride, int T0, int B,
                               int H, int D, int L0, const int32_t* d_L0, int cap, int window, void* d_out,
                               int64_t out_stride, float scale, void* hip_stream);

/* ns_decode_attention_prefix over an fp8 KV cache (OCP e4m3fn bytes, element layout as above with 1-byte
 * elements): half the HBM bytes of the fp16 cache.  The new token's k/v are quantised (saturated to +-448,
 * round to nearest even) before they are stored and used.  q, scores and the softmax stay fp16/fp32; rows
 * are split by key count only (64-row chunks), so the output is batch-invariant too.  An opt-in numerics
 * mode: logits differ from the fp16 cache's at the fp8 quantisation level. */
int ns_decode_attention_fp8(const void* d_qkv, int64_t qkv_stride, void* d_k_cache, void* d_v_cache,
                            int64_t cache_b_stride, int64_t cache_h_stride, int64_t cache_chunk_stride,
                            const void* d_k_prefix, const void* d_v_prefix, int64_t prefix_h_stride, int T0, int B,
                            int H, int D, int L0, const int32_t* d_L0, int cap, int window, void* d_out,
                            int64_t out_stride, float scale, void* hip_stream);

/* KV element formats of ns_decode_attention_ex */
#define NS_KV_FP16 0
#define NS_KV_FP8 1

/* ns_decode_attention_prefix (kv_format NS_KV_FP16) / ns_decode_attention_fp8 (NS_KV_FP8) with an optional
 * per-stream end: stream b is skipped if d_done is not NULL and bit 0 of d_done[b * done_stride] is set (uint32
 * words; e.g. the flags word of the coder state, NS_ST_DONE -- encode), or if d_stop is not NULL and the cache
 * length L0 >= d_stop[b] (int32; the position after which a decode needs no more logits): no KV append, no cache
 * read, its output row left as it was.  Both are read when the kernel runs (L0 from d_L0 on graph replays), so one
 * captured hipGraph serves every step while streams finish.  The other streams' outputs are the same bits with or without the flags (a stream's row split depends
 * on its key count only): a lockstep batch whose covers differ in length (peaked, trained-LM rows) stops paying
 * the finished streams' cache reads. */
int ns_decode_attention_ex(const void* d_qkv, int64_t qkv_stride, void* d_k_cache, void* d_v_cache,
                           int64_t cache_b_stride, int64_t cache_h_stride, int64_t cache_chunk_stride,
                           const void* d_k_prefix, const void* d_v_prefix, int64_t prefix_h_stride, int T0, int B,
                           int H, int D, int L0, const int32_t* d_L0, int cap, int window, int kv_format,
                           const uint32_t* d_done, int64_t done_stride, const int32_t* d_stop, void* d_out,
                           int64_t out_stride, float scale, void* hip_stream);

/* ns_decode_attention_ex over a PAGED cache with a cache length PER STREAM (round 6: slot refill and growth
 * without a copy).  Stream b's rows live in 32-position pages: d_page_table[b * table_stride + c] (uint64; the table
 * 8-byte aligned, so a row range of a larger table is a table too) is the
 * device address (16-byte aligned; 0 = none) of the page holding its stream rows 32c .. 32c + 31, i.e. positions
 * T0 + 32c ...; this layer's block of the page starts `layer_offset` elements after that address and holds
 * [K|V][H][32][D] in the kv_format's element type (K at +0, V at +H*32*D; the pool decides where the layers of a page
 * live: layer * 2*H*32*D for pages holding every layer back to back, layer * SEG * 2*H*32*D for segments of SEG pages
 * stored layer-major).  d_lens[b] (int32) = positions already cached for stream b
 * (the new token is written at position d_lens[b] and attended with positions 0 .. d_lens[b]); positions < T0 come
 * from the shared prefix as in ns_decode_attention_prefix.  Only table entries 0 .. max_chunks-1 are read; a stream
 * whose new-token page is missing gets NaN output rows (the coder rejects them) and writes nothing.  d_done / d_stop
 * skip finished streams as in ns_decode_attention_ex (the stop test compares d_lens[b]).  A pair's rows are split
 * by its own key count and merged in the same order as the lockstep kernels: for the same cache contents the output
 * bits equal ns_decode_attention_ex's, whatever the batch, the other streams' lengths or where the pages live.
 * Replaces the reference's per-message cache of code_base/arithmetic.py:96-122 (each message its own loop). */
int ns_decode_attention_paged(const void* d_qkv, int64_t qkv_stride, const uint64_t* d_page_table,
                              int64_t table_stride, int max_chunks, int64_t layer_offset, const void* d_k_prefix,
                              const void* d_v_prefix, int64_t prefix_h_stride, int T0, int B, int H, int D,
                              const int32_t* d_lens, int window, int kv_format, const uint32_t* d_done,
                              int64_t done_stride, const int32_t* d_stop, void* d_out, int64_t out_stride, float scale,
                              void* hip_stream);

/* Causal attention over B whole sequences of T tokens (positions 0..T-1, no cache): the prefill of the shared
 * context (code_base/arithmetic.py:115-122, the first call), the guard's scoring forward
 * (src/neuralstego/metrics/lm_scorer.py:121-131) and the src provider's max_context window forward
 * (src/neuralstego/lm/arithmetic.py:45-74).  d_qkv fp16 [B*T, qkv_stride] (row b*T + t; q, k, v column blocks as in
 * ns_decode_attention), d_out fp16 [B*T, out_stride].  Flash attention on the 16x16x32 f16 MFMA with an fp32
 * online softmax and P rounded to fp16 for the PV product; each output row depends on its own sequence only
 * (batch-invariant).  D must be 64. */
int ns_seq_attention(const void* d_qkv, int64_t qkv_stride, void* d_out, int64_t out_stride, int B, int T, int H,
                     int D, float scale, void* hip_stream);

/* fp16 [n] -> fp8 e4m3fn [n] with the attention's conversion (n % 4 == 0, 8-byte aligned). */
int ns_quantize_fp8(const void* d_src, void* d_dst, int64_t n, void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* NSG_ATTN_H */
