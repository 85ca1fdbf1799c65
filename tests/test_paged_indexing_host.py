"""CPU: a restatement of ``paged_attn_kernel``'s row / page indexing (``csrc/nsg_attn.hip``), checking that every row
a task loads comes from the shared prefix or from a MAPPED page of its stream, and the right one.

The host maps a stream's pages through the chunk of its new token (``lens[b] - T0``) before a step; the kernel
reads the rows of 32-row iterations ``j0 = s0 + 32 * (w + k * S)`` (split w of S), clamped to the last cached row,
with the page addresses of an iteration prefetched per lane (first and last stream row it reads).  An address
computed for an unmapped chunk would fault the GPU; this test walks the same arithmetic for every split, iteration
and row over a grid of (T0, L0, window) and fails on any such row."""

import pytest


def att_split(lk, rows1=256):
    return 1 if lk <= rows1 else 2 if lk <= 2 * rows1 else 4 if lk <= 4 * rows1 else 8


def check(T0, L0, window):
    Lk = L0 + 1
    s0 = max(0, Lk - window) if window > 0 else 0
    S = att_split(Lk - s0)
    last_cached = L0 - 1 if L0 > 0 else 0
    hi_row = last_cached - T0
    mapped = set(range(((L0 - T0) >> 5) + 1))  # the host invariant: pages through the new token's chunk
    step = 32 * S
    for wv in range(S):
        j0 = s0 + 32 * wv
        while j0 < Lk:
            jj = j0 - T0
            lo, hi = max(min(jj, hi_row), 0), min(jj + 31, hi_row)
            any_ = hi >= 0 and jj <= L0 - T0
            pa = lo >> 5 if any_ else None
            pb = hi >> 5 if any_ and (hi >> 5) != (lo >> 5) else pa
            for p in (pa, pb):
                assert p is None or p in mapped, (T0, L0, window, wv, j0, p)
            interior = j0 >= T0 and j0 + 32 <= L0
            for r in range(32):
                row = j0 + r
                if interior:
                    jr = row - T0
                    page = pa if (jr >> 5) == (jj >> 5) else pb
                    assert page == jr >> 5, (T0, L0, window, row)
                    continue
                rc = min(row, last_cached)
                if rc < T0:
                    assert 0 <= rc < T0, (T0, L0, window, row)  # a prefix row
                    continue
                jr = rc - T0
                ca = max(min(jj, hi_row), 0) >> 5
                page = pa if (jr >> 5) == ca else pb
                assert page is not None and page == jr >> 5 and page in mapped, (T0, L0, window, row, page)
            j0 += step


@pytest.mark.parametrize("T0", [0, 1, 7, 31, 32, 33])
@pytest.mark.parametrize("window", [0, 1, 16, 100, 256])
def test_every_loaded_row_has_a_mapped_page(T0, window):
    for L0 in list(range(T0, T0 + 200)) + [T0 + n for n in (255, 256, 257, 511, 512, 513, 1023, 1024, 1025, 2049)]:
        check(T0, L0, window)
