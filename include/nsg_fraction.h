/*
 * nsg_fraction.h -- the src package's exact-rational arithmetic coder as a batched device kernel (SURVEY.md §8
 * row a12, "Fraction coder ... as selectable kernels", §8(f) 4), part of `libnsgcoder.so`.
 *
 * Replaces, for B independent messages at once:
 *   - encode_bits / _encode_step   (src/neuralstego/codec/arithmetic.py:234-270, 408-434)
 *   - decode_bits / _decode_step   (src/neuralstego/codec/arithmetic.py:273-325, 437-466)
 *   - _cumulative_distribution, _to_fraction, _prefix_interval, _prefix_from_interval (:469-550)
 * The interval [lo, hi) is kept exactly as three integers (lo = PL / Q, hi = PH / Q) in device memory; every
 * comparison the reference makes on fractions.Fraction values is made on integers, so tokens, the per-token
 * bit counts (the state "history") and decoded bits are identical to the reference's.  One wavefront per
 * stream: the lanes convert the distribution's float64 values to fractions (limit_denominator(2^30)) and build
 * the cumulative numerators; lane 0 runs the interval arithmetic.  Host-side (Python, codec/fraction.py):
 * iterating the ProbDist iterables, type / sign / NaN checks, the state dict and the exceptions.
 *
 * Status per stream (d_status) after a step: NS_FRAC_OK, NS_FRAC_SKIPPED (no work for this stream), or an
 * error -- the state is left unchanged on every error, so a step can be re-run with a larger table.  A skipped
 * stream's d_token / d_used entries are not written, so streams can be run in several launches that share the
 * output buffers (e.g. a re-run of the NS_FRAC_ERR_TABLE streams only).
 *
 * Supported envelope: D = lcm of a step's limit_denominator(2^30) denominators must fit cap_limbs 32-bit limbs;
 * V unrelated 30-bit denominators make D about 30 V bits, so with the default 4,096 limbs a step holds up to
 * ~4,000 entries with unrelated denominators (dyadic / shared denominators cost nothing), and the interval
 * integers grow by about the size of D per token.  Real GPT-2 rows (V = 50,257) exceed it on the first step
 * (NS_FRAC_ERR_CAPACITY): that is the reference's own arithmetic, whose fractions grow the same way.
 */
#ifndef NSG_FRACTION_H
#define NSG_FRACTION_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ns_frac_ctx ns_frac_ctx;

#define NS_FRAC_OK 0
#define NS_FRAC_SKIPPED 1
#define NS_FRAC_ERR_NO_MASS (-1)     /* "Probability distribution must have positive mass" (:473-475)          */
#define NS_FRAC_ERR_UNRESOLVED (-2)  /* "Unable to resolve token interval with available bits" (:434-435)      */
#define NS_FRAC_ERR_NOT_PRESENT (-3) /* "Token {id} not present in distribution" (:460-461)                    */
#define NS_FRAC_ERR_NO_PREFIX (-4)   /* "No binary prefix fits within the interval" (:531-532)                 */
#define NS_FRAC_ERR_CAPACITY (-5)    /* an integer outgrew cap_limbs (no larger table can help)               */
#define NS_FRAC_ERR_TABLE (-6)       /* the step's cumulative table needs more than table_limbs per stream:
                                        re-run that stream with a larger table (its state is unchanged)       */

/* Context for up to max_batch streams whose interval integers may grow to cap_limbs 32-bit limbs each. */
ns_frac_ctx* ns_frac_create(int max_batch, int cap_limbs, int device);
void ns_frac_destroy(ns_frac_ctx* ctx);
const char* ns_frac_last_error(const ns_frac_ctx* ctx);

/* Start B streams: [lo, hi) = [0, 1), nothing consumed; h_nbits[b] = payload bits of stream b (host array). */
int ns_frac_init(ns_frac_ctx* ctx, int B, const int64_t* h_nbits, void* hip_stream);

/* Scratch slots: with d_slot set (device int32[B], until reset with NULL), stream b uses scratch slot d_slot[b]
 * (< nslots) and a stream whose slot is negative is skipped, so a launch that runs R of B streams needs scratch
 * for R streams only.  d_slot must stay valid while steps run.  Default (NULL): slot b for stream b. */
int ns_frac_set_slots(ns_frac_ctx* ctx, const int32_t* d_slot, int nslots);

/* Device scratch bytes one step allocates for nslots streams (the context keeps the largest so far). */
int64_t ns_frac_scratch_bytes(const ns_frac_ctx* ctx, int nslots, int64_t ld, int64_t max_bits, int64_t table_limbs);

/* One encode step for every stream b with d_count[b] >= 0 and payload bits left (else NS_FRAC_SKIPPED):
 *   d_probs [B, ld] float64 values and d_ids [B, ld] int32 token ids of the stream's distribution in the
 *   reference's order (array: 0..V-1; dict: sorted keys), d_count[b] = V entries (<= ld);
 *   d_bits [B, bits_stride] the payload, one bit per byte, MSB-first (zero-padded past the payload by the step);
 *   table_limbs: per-stream room for the V + 1 cumulative numerators (NS_FRAC_ERR_TABLE if short);
 *   max_bits: the largest payload length of the batch (sizes the scratch; at most 2^20 -- NS_ERR_CONFIG above: a
 *   failing step searches one depth per payload bit, each linear in the integers' growing size).
 * Outputs d_token[b] (the token id), d_used[b] (bits consumed = the depth, the reference's history entry). */
int ns_frac_encode_step(ns_frac_ctx* ctx, int B, const double* d_probs, const int32_t* d_ids, int64_t ld,
                        const int32_t* d_count, const uint8_t* d_bits, int64_t bits_stride, int64_t max_bits,
                        int64_t table_limbs, int32_t* d_token, int32_t* d_used, int32_t* d_status, void* hip_stream);

/* One decode step for every stream b with d_count[b] >= 0 (else NS_FRAC_SKIPPED): narrows [lo, hi) to token
 * d_token[b] of the distribution and, if d_used[b] > 0, writes the d_used[b] bits of the dyadic interval it
 * holds (MSB first, one bit per byte) at d_out_bits[b * out_stride + d_out_pos[b]] and advances d_out_pos[b].
 * max_used = max over b of d_used[b] (sizes the scratch). */
int ns_frac_decode_step(ns_frac_ctx* ctx, int B, const double* d_probs, const int32_t* d_ids, int64_t ld,
                        const int32_t* d_count, const int32_t* d_token, const int32_t* d_used, int64_t max_used,
                        int64_t table_limbs, uint8_t* d_out_bits, int64_t out_stride, int64_t* d_out_pos,
                        int32_t* d_status, void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* NSG_FRACTION_H */
