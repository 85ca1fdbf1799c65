"""CPU: host logic of the paged KV cache (``lm/kvpages.py``), driven with CPU tensors (page addresses are real
addresses of the CPU segments).  The device side (``ns_decode_attention_paged``) is covered by the GPU tests."""

import numpy as np
import pytest
import torch

from neuralsteganography_amd.lm.kvpages import PAGE_ROWS, KVPagePool, PagedKV


def _pool(budget_pages=None, seg_pages=4):
    holder = {}
    budget = None
    if budget_pages is not None:
        def budget():
            return (budget_pages - holder["pool"].total) * holder["pool"].page_bytes
    pool = KVPagePool(n_layer=2, n_head=2, head_dim=64, dtype=torch.float16, device="cpu", budget_bytes=budget,
                      seg_pages=seg_pages)
    holder["pool"] = pool
    return pool


def test_page_geometry_and_addresses():
    pool = _pool(seg_pages=8)
    assert pool.block_elems == 2 * 2 * PAGE_ROWS * 64 and pool.page_elems == 2 * pool.block_elems
    assert pool.page_bytes == 2 * pool.page_elems
    pages = pool.take(5)
    assert pages.size == 5 and len(set(pages.tolist())) == 5
    seg = pool.segments[0]
    assert tuple(seg.shape) == (2, 8, pool.block_elems)  # layer-major: [layer][page][block]
    base = seg.data_ptr()
    for a in pages.tolist():  # every address is a layer-0 block inside the segment
        assert (a - base) % pool.block_bytes == 0 and 0 <= (a - base) // pool.block_bytes < 8
        assert a % 16 == 0
    # layer 1 of a page is layer_offset(1) elements after its address: the same page index in the second layer plane
    i = (int(pages[2]) - base) // pool.block_bytes
    flat = seg.view(-1)
    off = (int(pages[2]) - base) // pool.esize + pool.layer_offset(1)
    flat[off] = 7.0
    assert seg[1, i, 0].item() == 7.0


def test_take_give_reuses_pages_and_grows_by_segments():
    pool = _pool(seg_pages=4)
    a = pool.take(3)
    assert pool.total == 4 and pool.free_pages == 1
    b = pool.take(6)  # grows by whole segments: max(short, total/4) pages, rounded up
    assert pool.total >= 9 and pool.total % 4 == 0 and len(pool.segments) >= 2
    pool.give(a)
    c = pool.take(3)
    assert set(c.tolist()) == set(a.tolist())  # freed pages come back first
    assert not set(c.tolist()) & set(b.tolist())


def test_budget_limits_growth_and_failure_takes_nothing():
    pool = _pool(budget_pages=10, seg_pages=1)
    assert pool.take(8) is not None
    free_before = pool.free_pages
    assert pool.take(5) is None  # 8 used + 5 > 10
    assert pool.free_pages == free_before
    assert pool.take(2) is not None
    assert pool.total <= 10
    seg4 = _pool(budget_pages=10, seg_pages=4)
    assert seg4.take(8) is not None and seg4.take(1) is None  # a third segment of 4 would pass the budget


def test_ensure_maps_pages_in_order_and_mirrors_the_device_table():
    pool = _pool()
    kv = PagedKV(pool, B=3, T0=5, width=1)
    assert kv.ensure([0, 1, 2], [5, 5 + 1, 5 + 70]).size == 0  # 0, 1 and 3 pages
    assert kv.nch.tolist() == [0, 1, 3]
    assert kv.width >= 3  # grown for slot 2
    assert np.array_equal(kv.table.numpy(), kv.host)
    assert (kv.host[2, :3] != 0).all() and (kv.host[0] == 0).all()
    before = kv.host[2, :3].copy()
    assert kv.ensure([2], 5 + 96).size == 0  # positions up to T0 + 96: no new page
    assert kv.ensure([2], 5 + 97).size == 0  # one more page appended, the first three unchanged
    assert kv.nch[2] == 4 and np.array_equal(kv.host[2, :3], before)


def test_release_reset_and_steps_reserved():
    pool = _pool()
    kv = PagedKV(pool, B=2, T0=4, width=4)
    kv.ensure([0, 1], 4 + 40)
    assert kv.steps_reserved([0, 1]) == 64 - 0
    kv.advance(10)
    assert kv.steps_reserved([0, 1]) == 54
    free = pool.free_pages
    kv.reset([1])
    assert pool.free_pages == free + 2 and kv.nch[1] == 0 and (kv.table[1] == 0).all()
    assert kv.lens[1].item() == 4 and kv.lens_host[1] == 4 and kv.lens_host[0] == 14


def test_ensure_reports_slots_the_pool_cannot_serve():
    pool = _pool(budget_pages=5, seg_pages=1)
    kv = PagedKV(pool, B=3, T0=0, width=8)
    failed = kv.ensure([0, 1, 2], [64, 64, 64])  # 2 pages each, 5 available: slot 2 fails, nothing half-mapped
    assert failed.tolist() == [2]
    assert kv.nch.tolist() == [2, 2, 0]
    kv.release([0])
    assert kv.ensure([2], 64).size == 0


def test_compact_moves_rows_without_touching_pages():
    pool = _pool()
    kv = PagedKV(pool, B=4, T0=1, width=2)
    kv.ensure([0, 1, 2, 3], [33, 40, 1, 60])
    kv.lens[:] = torch.tensor([9, 8, 7, 6], dtype=torch.int32)
    kv.lens_host[:] = [9, 8, 7, 6]
    rows = {s: kv.host[s].copy() for s in range(4)}
    kv.release([0, 2])
    v = kv.version
    kv.compact([3, 1])
    assert kv.B == 2 and kv.version == v + 1
    assert np.array_equal(kv.host[0], rows[3]) and np.array_equal(kv.host[1], rows[1])
    assert np.array_equal(kv.table.numpy(), kv.host)
    assert kv.lens.tolist() == [6, 8] and kv.lens_host.tolist() == [6, 8]
    with pytest.raises(RuntimeError):
        kv.compact([0])  # slot 1 still holds pages


def test_pool_reset_frees_every_page():
    pool = _pool()
    kv = PagedKV(pool, B=2, T0=0, width=4)
    kv.ensure([0, 1], 100)
    assert pool.free_pages < pool.total
    pool.reset()
    assert pool.free_pages == pool.total
