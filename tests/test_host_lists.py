"""CPU: the session helpers that turn device token / bit rows into the Python lists the codec API returns
(coder.py ``_rows_to_lists`` / ``_bit_rows_to_lists``): ragged lengths, empty rows, only the used columns read."""

import numpy as np
import torch

from neuralsteganography_amd.coder import _bit_rows_to_lists, _rows_to_lists


def test_rows_to_lists_ragged():
    h = torch.arange(5 * 40, dtype=torch.int32).reshape(5, 40)
    n = np.array([0, 3, 17, 17, 1], dtype=np.int32)
    got = _rows_to_lists(h, n)
    assert got == [h[i, :k].tolist() for i, k in enumerate(n)]
    assert all(type(v) is int for r in got for v in r)
    assert _rows_to_lists(h, np.zeros(5, dtype=np.int64)) == [[]] * 5


def test_bit_rows_to_lists_ragged():
    rng = np.random.default_rng(1)
    ob = torch.from_numpy(rng.integers(0, 256, size=(4, 20), dtype=np.uint8))
    nb = np.array([0, 5, 64, 13], dtype=np.int64)
    got = _bit_rows_to_lists(ob, nb)
    want = [np.unpackbits(ob[i].numpy(), bitorder="little")[:k].tolist() for i, k in enumerate(nb)]
    assert got == want


def test_bit_array_matches_numpy_conversion():
    from neuralsteganography_amd.coder import _bit_array

    for bits in ([0, 1, 1, 0, 1], (1, 0), [True, False, True], np.array([1, 0, 1], dtype=np.int64), [0, 2, 1]):
        assert np.array_equal(_bit_array(bits), np.asarray(bits, dtype=np.uint8))
