/*
 * nsg_score.h -- per-position language-model scores for the cover-text quality guard,
 * part of `libnsgcoder.so`.
 *
 * Replaces the two Hugging Face reductions the reference's guard metrics run over a text's logits:
 *   - LMScorer.score (src/neuralstego/metrics/lm_scorer.py:121-131): `model(**inputs, labels=ids).loss`, the
 *     mean over positions t < T-1 of  -log softmax(logits[t])[ids[t+1]];
 *   - avg_entropy (src/neuralstego/metrics/entropy.py:36-46): the mean over positions t < T-1 of
 *     -sum_j p_j log(p_j + 1e-12), p = softmax(logits[t]).
 * One wavefront streams one row of V logits once (HBM-bound), keeping an online max, sum of exponentials and
 * sum of p-weighted logits per lane; nll = lse - x[label] and entropy = lse - sum_j p_j x_j are produced in
 * float64 from fp32 partials (the 1e-12 inside the reference's log changes the entropy by < 1e-9 nats).
 */
#ifndef NSG_SCORE_H
#define NSG_SCORE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* d_logits: [nrows, ld] rows of dtype (0 = fp32, 1 = fp16, NS_DTYPE_*), V <= ld valid columns, 16-byte aligned
 * rows.  d_labels: [nrows] int32 target id per row, or a negative value for "no label" (nll written as 0).
 * d_nll, d_entropy: [nrows] float64 outputs (either may be NULL).  Returns 0 or a negative NS_ERR_* code. */
int ns_score_rows(const void* d_logits, int64_t ld, int64_t nrows, int V, int dtype, const int32_t* d_labels,
                  double* d_nll, double* d_entropy, void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* NSG_SCORE_H */
