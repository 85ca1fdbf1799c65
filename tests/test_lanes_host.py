"""Host logic of the decode-step lanes (``BatchedGPT2._lanes``): the row ranges cover the batch exactly, each lane
non-empty, at every batch size the slot scheduler can compact to (a lane past the batch would read and write outside
the step's buffers)."""
import types

from neuralsteganography_amd.lm.gpt2 import BatchedGPT2


def test_lane_ranges_partition_the_batch():
    for lanes, min_b in ((2, 2), (2, 1024), (1, 2)):
        o = types.SimpleNamespace(decode_lanes=lanes, decode_lanes_min_batch=min_b)
        for B in list(range(1, 70)) + [1023, 1024, 1025, 4095, 4096]:
            r = BatchedGPT2._lanes(o, B)
            assert r[0][0] == 0 and sum(n for _, n in r) == B and all(n > 0 for _, n in r), (B, r)
            assert all(r[k][0] + r[k][1] == r[k + 1][0] for k in range(len(r) - 1)), (B, r)
            assert len(r) == (2 if lanes == 2 and B >= max(2, min_b) else 1), (B, r)
