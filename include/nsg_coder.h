/*
 * nsg_coder.h -- C ABI of the MI355X (gfx950) batched arithmetic-coding step library `libnsgcoder.so`.
 *
 * One call runs ONE coder step for B independent message streams on a [B, ld] logit matrix that is
 * already resident in HBM.  The work is stream-ordered on the caller's hipStream_t (passed as void*);
 * no call allocates, synchronises or copies except ns_create / ns_destroy / ns_read_counters.
 *
 * What each entry point replaces in the reference (nobkagit/NeuralSteganography):
 *
 *   ns_encode_step  -- one iteration of the `while i < len(message)` loop body of
 *                      code_base/arithmetic.py:124-203 (ban, sort, float64 softmax, cutoff k
 *                      (_select_cutoff_k :51-75), integer CDF :143-165, bit consume :167-190, token
 *                      append :202), batched over B streams.  The Python loop that calls it replaces
 *                      encode_arithmetic (code_base/arithmetic.py:78-217) and, behind the provider
 *                      protocol, src/neuralstego/lm/arithmetic.py:162-191 (ArithmeticLM.encode_arithmetic).
 *   ns_decode_step  -- one iteration of code_base/arithmetic.py:255-371 (same CDF, rank lookup :298,
 *                      bit emit :354-360), batched; replaces decode_arithmetic (:220-373) and
 *                      src/neuralstego/lm/arithmetic.py:193-226.  A received token outside the kept top-k
 *                      is reported per stream (NS_ST_ERR_DIVERGE) instead of running the BPE-repair
 *                      heuristics of :300-342 (those need the tokenizer; the host applies them).
 *   ns_init_state   -- `cur_interval = [0, 2**precision]`, `i = 0` (code_base/arithmetic.py:96-98,112).
 *
 * Bit conventions: payload bytes are read LSB-first (bit j = byte[j>>3] >> (j&7)), the order in which
 * src/neuralstego/api.py:153-157 turns bytes into the bit list the coder consumes; within a step the
 * next `precision` bits form an MSB-first integer (code_base/arithmetic.py:168-171).  Decoded bits are
 * written back in the same LSB-first packing.
 *
 * Errors: return NS_OK (0) or a negative NS_ERR_*; ns_last_error() gives a message.  Per-stream coder
 * failures (the reference's ArithmeticRangeError / DecodeDivergenceError, src/neuralstego/codec/errors.py:10-15)
 * are flags in ns_stream_state.flags; the Python host raises them.
 */
#ifndef NSG_CODER_H
#define NSG_CODER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NS_OK 0
#define NS_ERR_CONFIG -1      /* bad argument: maps to ConfigurationError / ValueError          */
#define NS_ERR_UNSUPPORTED -2 /* valid for the reference, not (yet) for this kernel (topk too large) */
#define NS_ERR_HIP -3         /* HIP runtime error (launch failure)                             */

#define NS_DTYPE_F32 0
#define NS_DTYPE_F16 1
#define NS_DTYPE_F64 2 /* rank coder only: rows are a provider's float64 probabilities (ns_set_rank_rows) */

/* per-stream flags */
#define NS_ST_DONE 1u         /* encode: all payload bits consumed; no further tokens are produced */
#define NS_ST_ERR_RANGE 2u    /* no CDF bucket above the payload index (ArithmeticRangeError)      */
#define NS_ST_ERR_DIVERGE 4u  /* decode: received token not in the kept top-k (DecodeDivergenceError) */
#define NS_ST_EXACT_SUM 8u    /* the last step needed the exact float64 row sum (slow path taken)   */

/* step flags */
#define NS_STEP_FORCE_EXACT_SUM 1u /* always take the exact-sum path (parity testing) */
#define NS_STEP_FINISH_SENT 16u /* encode: after the payload, emit top-1 tokens until a sentence end
                                   (code_base/arithmetic.py:114,134-137); needs ns_set_sentence_end   */
/* diagnostic flags for phase timing only: the step does NOT advance any state when one is set */
#define NS_STEP_DIAG_STREAM_ONLY 2u    /* stop after the streaming pass                           */
#define NS_STEP_DIAG_NO_CANDIDATES 4u  /* streaming pass without candidate collection, then stop  */
#define NS_STEP_DIAG_SKIP_CDF 8u       /* stop after the exact top-K ranking                      */

#define NS_MAX_BANNED 8

typedef struct ns_stream_state {
    uint64_t lo;      /* interval bottom (inclusive)                                    */
    uint64_t hi;      /* interval top (exclusive)                                       */
    int64_t bit_pos;  /* encode: payload bits fixed so far (`i`); decode: bits emitted  */
    int32_t ntokens;  /* tokens produced (encode) / consumed (decode)                   */
    uint32_t flags;   /* NS_ST_*                                                        */
} ns_stream_state;

typedef struct ns_step_trace { /* optional per-stream record of the last step (tests, debugging) */
    int32_t k;      /* kept candidates after the 1/R cutoff and topk                   */
    int32_t kprime; /* after the overfill trim                                         */
    int32_t sel;    /* selected rank                                                   */
    int32_t n;      /* bits fixed (encode) / emitted before the last-token rule (decode) */
    int32_t token;  /* token id emitted / consumed                                     */
    int32_t exact;  /* 1 if the exact float64 row sum was computed                     */
    double S;       /* row sum used for the cutoff (fast estimate or exact)            */
} ns_step_trace;

typedef struct ns_ctx ns_ctx;

/* Create a context on `device` for logits rows of `vocab` entries of `logits_dtype` (NS_DTYPE_*),
 * at most `max_batch` streams per call, interval precision `precision` (1..60 bits) and top-k up to
 * `max_k`.  max_k <= ns_max_topk(dtype) uses the single-pass kernel only; a larger max_k also allocates
 * the wide path (stats pass, collect, segmented radix sort, workgroup CDF; 16 B x max_batch x vocab of
 * scratch, vocab < 131072).  Returns NULL on failure (see ns_last_error(NULL)). */
ns_ctx* ns_create(int device, int max_batch, int vocab, int max_k, int precision, int logits_dtype);
void ns_destroy(ns_ctx* ctx);
const char* ns_last_error(const ns_ctx* ctx);
const char* ns_version(void);

/* Largest topk the single-pass kernel handles for a logits dtype (larger topk takes the wide path). */
int ns_max_topk(int logits_dtype);

/* Single-pass steps of at most `max_batch` streams run the split form (one workgroup of 16 fp32 / 8 fp16 waves per
 * stream) instead of one wave per stream; 0 disables it, a negative value restores the automatic limit (B * waves
 * per stream <= 6144: fp32 B <= 384, fp16 B <= 768; environment NSG_SPLIT_MAX_B sets an explicit one).
 * Process-wide; speed only -- both forms emit the same tokens and bits.  Returns the previous setting (-1:
 * automatic). */
int ns_set_split_max_batch(int max_batch);

/* Reset B stream states to [0, 2^precision), bit_pos 0. */
int ns_init_state(ns_ctx* ctx, ns_stream_state* d_state, int B, void* hip_stream);

/* One encode step for streams [0,B).  d_logits: [B, ld] row-major, 16-byte aligned, ld a multiple of
 * 16/sizeof(dtype) and >= vocab.  d_payload: [B, payload_stride] bytes, d_payload_nbits: [B] int64.
 * d_out_token: [B] (written for every stream that produced a token this step).  d_token_hist: optional
 * [B, hist_stride] history, token t of stream b at b*hist_stride+t.  banned: HOST array of nbanned ids
 * (<= NS_MAX_BANNED), the reference bans {vocab-1, 628}.  d_trace: optional [B].  temp > 0. */
int ns_encode_step(ns_ctx* ctx, const void* d_logits, int64_t ld, int B, const uint8_t* d_payload,
                   int64_t payload_stride, const int64_t* d_payload_nbits, ns_stream_state* d_state,
                   int32_t* d_out_token, int32_t* d_token_hist, int64_t hist_stride, double temp, int topk,
                   const int32_t* banned, int nbanned, ns_step_trace* d_trace, uint32_t step_flags,
                   void* hip_stream);

/* One decode step.  d_in_token: [B] received token of this step; d_is_last: [B] nonzero when it is the
 * stream's last token (then all `precision` bits of the new bottom are emitted, arithmetic.py:356-357).
 * d_out_bits: [B, out_stride] bytes, bits appended LSB-first at ns_stream_state.bit_pos.
 * d_active: optional [B] mask; streams with 0 are skipped (ragged token counts). */
int ns_decode_step(ns_ctx* ctx, const void* d_logits, int64_t ld, int B, const int32_t* d_in_token,
                   const uint8_t* d_is_last, const uint8_t* d_active, ns_stream_state* d_state,
                   uint8_t* d_out_bits, int64_t out_stride, double temp, int topk, const int32_t* banned,
                   int nbanned, ns_step_trace* d_trace, uint32_t step_flags, void* hip_stream);

/* Register the sentence-end table used by NS_STEP_FINISH_SENT: d_table is a DEVICE array of `vocab`
 * bytes, nonzero for ids whose text contains '.', '!' or '?' (code_base/utils.py:55-57,
 * is_sent_finish).  The caller keeps it alive; NULL clears it. */
int ns_set_sentence_end(ns_ctx* ctx, const uint8_t* d_table);

/* Rank export for decode repair: when a later ns_decode_step finds stream b's received token outside the
 * kept top-k' (NS_ST_ERR_DIVERGE; the state is left unchanged so the step can be re-issued), the kernel
 * writes the kept ids in rank order to d_ranked[b*stride + i], i < k', followed by -1 (truncated at
 * stride).  The host runs the reference's BPE-repair heuristics on them (code_base/arithmetic.py:300-342)
 * and re-issues the step with the repaired token.  d_ranked is a DEVICE int32 array; NULL switches it off. */
int ns_set_rank_export(ns_ctx* ctx, int32_t* d_ranked, int stride);

/* Statistics of the encode steps (code_base/arithmetic.py:193-199, returned by encode_arithmetic :217):
 * d_stats is a DEVICE array [B][4] of doubles that every later ns_encode_step accumulates into, per
 * stream: [0] sum of log p(selected) under the untempered softmax, [1] sum of KL(q || p) in bits over the
 * kept CDF entries, [2] sum of the tempered softmax's entropy over V in bits, [3] message-phase steps.
 * avg_NLL = -[0]/[3], avg_KL = [1]/[3], avg_Hq = [2]/[3], words_per_bit = [3]/bit_pos.  Float64 values
 * computed from fp32 streaming sums: within 1e-5 relative of the float64 reference (not bit-exact).
 * NULL switches statistics off (the default, and the fast kernel). */
int ns_set_stats(ns_ctx* ctx, double* d_stats);

/* One sampler step (code_base/sample.py:22-48, the non-stego token loop) for streams [0,B): top-k of the
 * banned-masked row (topk <= 0: every id, which the reference's sample.py:39 cannot run), temperature
 * softmax, one draw.  The draw is counter based: u = splitmix64(seed, stream_offset + b, ntokens of the
 * stream), the token is the first rank whose 2^48-scaled integer CDF exceeds (u * total) >> 64 -- bit-exact
 * against oracle/nsg_oracle.c or_sample_step, and distributed as torch.multinomial (sample.py:44).
 * d_state: only ntokens is used (set it to 0 with ns_init_state); d_stats: optional [B][4] as in
 * ns_set_stats with [1] = KL(p_tau,k || p) and [2] = entropy of p_tau,k over the top-k set. */
int ns_sample_step(ns_ctx* ctx, const void* d_logits, int64_t ld, int B, uint64_t seed, int64_t stream_offset,
                   ns_stream_state* d_state, int32_t* d_out_token, int32_t* d_token_hist, int64_t hist_stride,
                   double temp, int topk, const int32_t* banned, int nbanned, double* d_stats,
                   ns_step_trace* d_trace, uint32_t step_flags, void* hip_stream);

/* Quality policies of the src rank coder (src/neuralstego/codec/quality.py:57-141 apply_quality /
 * cap_bits_per_token, keys as codec/arithmetic.py:345-362 reads them).  Off: top_k <= 0, cap_bits <= 0,
 * top_p <= 0, min_prob < 0, prob_temp <= 0.
 * prob_temp > 0 selects the crypto quality LM instead (src/neuralstego/crypto/arithmetic.py:20-40 +
 * crypto/quality.py:15-89): the temperature acts on the PROBABILITIES, p' = normalise(exp(log(p + 1e-12)/T
 * - max)), which gives every id nonzero mass, and top_k / top_p then filter p' (min_prob and cap_bits are
 * not part of that policy and must be off).  prob_temp == 1 (math.isclose) leaves p unchanged. */
typedef struct ns_rank_quality {
    int32_t top_k;
    int32_t cap_bits;
    double top_p;
    double min_prob;
    double prob_temp;
} ns_rank_quality;

/* One step of the src package's own coder, the uniform rank coder of encode_with_lm
 * (src/neuralstego/codec/arithmetic.py:122-168) over the softmax of logits/temp (lm/arithmetic.py:45-74): the
 * n tokens left with nonzero probability by the quality policies are ranked (value desc, id asc), c =
 * floor(log2 n) payload bits (read MSB-first per payload byte, zero padded) select the token of that rank.
 * d_payload holds the packet BYTES (the api bit list packed LSB-first, i.e. the bytes themselves),
 * d_payload_nbits their bit count; d_consumed_hist [B, hist_stride] receives the bits each token actually
 * consumed (the reference's state["history"]).  No ids are banned on this path.  NS_ST_ERR_RANGE: no capacity
 * (n < 2).  Runs on the wide path (every id sorted per step). */
int ns_rank_encode_step(ns_ctx* ctx, const void* d_logits, int64_t ld, int B, const uint8_t* d_payload,
                        int64_t payload_stride, const int64_t* d_payload_nbits, ns_stream_state* d_state,
                        int32_t* d_out_token, int32_t* d_token_hist, int32_t* d_consumed_hist, int64_t hist_stride,
                        double temp, const ns_rank_quality* quality, ns_step_trace* d_trace, uint32_t step_flags,
                        void* hip_stream);

/* Decode step of the rank coder (codec/arithmetic.py:171-231): the received token's rank among the first 2^c,
 * the first d_keep_bits[b] of its c bits (the consumption history) appended MSB-first into d_out_bits bytes.
 * A token outside the first 2^c ranks: NS_ST_ERR_DIVERGE. */
int ns_rank_decode_step(ns_ctx* ctx, const void* d_logits, int64_t ld, int B, const int32_t* d_in_token,
                        const int32_t* d_keep_bits, const uint8_t* d_active, ns_stream_state* d_state,
                        uint8_t* d_out_bits, int64_t out_stride, double temp, const ns_rank_quality* quality,
                        ns_step_trace* d_trace, uint32_t step_flags, void* hip_stream);

/* Rank coder over a GENERIC next_token_probs provider (codec/types.py:41-45; codec/arithmetic.py:337-385): a
 * context created with NS_DTYPE_F64 takes, in ns_rank_encode_step / ns_rank_decode_step, d_logits = [B, ld]
 * float64 rows holding the provider's own ProbDist values (not logits; temp must be 1): an ndarray ProbDist by
 * id, or a dict ProbDist's items sorted by id.  The values are ranked (value desc, position asc), filtered by
 * the quality policy and renormalised in float64 exactly as codec/quality.py:57-105 does (numpy's own sum
 * restated for the normalisations, crypto/quality.py:57-89 when prob_temp > 0), replacing the round-3 float32
 * log-probability staging.  d_count: [B] entries per row (NULL: every row has `vocab` = ld-capacity entries);
 * d_idmap: [B, idmap_stride] token id of each entry (NULL: the position is the id); dict_rows: the rows are
 * dict ProbDists (then cap_bits runs over the kept entries only, as _arrays_to_dist drops zeros).  The pointers
 * stay registered for later steps; vocab (the row capacity) must be < 131072, ids are any int32. */
int ns_set_rank_rows(ns_ctx* ctx, const int32_t* d_count, const int32_t* d_idmap, int64_t idmap_stride,
                     int dict_rows);

/* next_token_probs of the src distribution providers (codec/distribution.py:107-142, lm/arithmetic.py:45-74):
 * d_probs [B, probs_stride] float64 receives, by token id, softmax(logits / temp) restricted to the
 * quality support (top_k / top_p / min_prob of `quality`, cap_bits ignored) and renormalised, zeros
 * elsewhere.  d_scratch_state: [B] states the call may overwrite. */
int ns_token_probs(ns_ctx* ctx, const void* d_logits, int64_t ld, int B, double temp, const ns_rank_quality* quality,
                   double* d_probs, int64_t probs_stride, ns_stream_state* d_scratch_state, void* hip_stream);

/* Rare-event diagnostics, cumulative since ns_create: counters[0] = stream-steps that took the exact-sum
 * path, counters[1] = candidate-buffer overflow compactions, counters[2] = speculative-threshold misses
 * (row re-read), counters[3] = top-K selections that left the histogram fast path (value ties or a skewed
 * row: bisection compaction or full-count ranking; on the wide path, LDS sorts that fell back to bitonic
 * order).  Synchronises the device. */
int ns_read_counters(ns_ctx* ctx, uint64_t* host_counters4);

#ifdef __cplusplus
}
#endif

#endif /* NSG_CODER_H */
