"""CPU: the host-side next_token_probs providers (codec/distribution.py MockLM, CachedLM); the reference's
tests/codec/test_distribution_mock.py checks the same properties."""

import numpy as np
import pytest

from neuralsteganography_amd.codec.distribution import CachedLM, MockLM


def test_mock_lm_zipf_prior():
    lm = MockLM(vocab_size=16, alpha=1.5)
    p = lm.next_token_probs([1, 2, 3])
    assert p.shape == (16,)
    assert p.sum() == pytest.approx(1.0)
    assert np.all(np.diff(p) < 0)
    assert p[0] / p[1] == pytest.approx(2 ** 1.5)
    np.testing.assert_array_equal(lm.next_token_probs([]), p)  # context is ignored
    with pytest.raises(ValueError):
        MockLM(vocab_size=0)


def test_cached_lm_memoises_and_copies():
    calls = []

    class Counting:
        def next_token_probs(self, ctx):
            calls.append(tuple(ctx))
            return np.full(4, 0.25)

    lm = CachedLM(Counting(), maxsize=2)
    a = lm.next_token_probs([1])
    a[0] = 9.0  # callers get copies
    assert lm.next_token_probs([1])[0] == 0.25
    lm.next_token_probs([2])
    lm.next_token_probs([3])  # evicts (1,)
    lm.next_token_probs([1])
    assert calls == [(1,), (2,), (3,), (1,)]
