"""GPU: the paged KV cache and the slot schedulers (round 6; ``lm/kvpages.py``, ``lm/slots.py``,
``ns_decode_attention_paged``).

* the paged attention (pages anywhere in a pool, a cache length per stream, P = 1 and P = 8 workgroup forms, fp16
  and fp8, prefix, window, done / stop skips) gives the SAME BITS as the lockstep kernel over the same rows, and a
  stream whose new-token page is missing gets NaN rows and writes nothing;
* slot refill: messages queued through fewer slots than messages give the same tokens as all at once and as each
  message alone, and the CPU oracle replays a message's tokens from its logits (reference:
  ``code_base/arithmetic.py:96-122``, every message its own loop and cache);
* eviction: a pool too small for every live stream re-queues the youngest messages and still gives the same tokens;
* the provider accepts the reference's usual ``device="cuda"``.
"""

import math

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from neuralsteganography_amd import _lib, synthetic  # noqa: E402
from neuralsteganography_amd.coder import _stream_handle  # noqa: E402
from oracle import oracle  # noqa: E402

pytestmark = pytest.mark.gpu

H, D = 12, 64


def _q8(t):
    out = torch.empty(t.shape, dtype=torch.uint8, device="cuda")
    assert _lib.lib().ns_quantize_fp8(t.contiguous().data_ptr(), out.data_ptr(), t.numel(), _stream_handle()) == 0
    return out


def _paged_case(B, T0, kv, seed, n_layer=2, layer=1, maxlen=420):
    """B streams with their own lengths: dense per-stream rows [B, H, rows, D] and the same rows scattered over a
    page pool in random order (layer ``layer`` of ``n_layer``-layer pages)."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    rng = np.random.default_rng(seed)
    lens = rng.integers(T0, T0 + maxlen, size=B)
    lens[0] = T0  # a stream at the shared context only
    rows = int(lens.max() - T0 + 1)
    nch = (rows + 31) // 32
    qkv = torch.randn((B, 3 * H * D), generator=g, device="cuda").half()
    dk = torch.randn((B, H, nch * 32, D), generator=g, device="cuda").half()
    dv = torch.randn((B, H, nch * 32, D), generator=g, device="cuda").half()
    kp = torch.randn((H, max(T0, 1), D), generator=g, device="cuda").half()
    vp = torch.randn((H, max(T0, 1), D), generator=g, device="cuda").half()
    if kv == "fp8":
        dk, dv, kp, vp = _q8(dk), _q8(dv), _q8(kp), _q8(vp)
    need = [(int(L) - T0) // 32 + 1 for L in lens]  # pages through the new token's row
    npages = sum(need) + 3
    pool = torch.zeros((npages, n_layer, 2, H, 32, D), dtype=dk.dtype, device="cuda")
    perm = rng.permutation(npages)
    table = np.zeros((B, nch + 2), dtype=np.int64)
    k = 0
    esz = pool.element_size()
    page_bytes = pool[0].numel() * esz
    for b in range(B):
        for c in range(need[b]):
            pg = int(perm[k])
            k += 1
            pool[pg, layer, 0] = dk[b, :, 32 * c: 32 * c + 32]
            pool[pg, layer, 1] = dv[b, :, 32 * c: 32 * c + 32]
            table[b, c] = pool.data_ptr() + pg * page_bytes
    return dict(qkv=qkv, dk=dk, dv=dv, kp=kp, vp=vp, pool=pool, table=torch.from_numpy(table).cuda(),
                lens=torch.from_numpy(lens.astype(np.int32)).cuda(), lens_np=lens, nch=nch, layer=layer, T0=T0,
                fmt=_lib.NS_KV_FP8 if kv == "fp8" else _lib.NS_KV_FP16)


def _run_paged(c, B, window=0, done=None, stop=None, table=None):
    out = torch.full((B, H * D), 7.0, device="cuda").half()
    tab = c["table"] if table is None else table
    T0 = c["T0"]
    rc = _lib.lib().ns_decode_attention_paged(
        c["qkv"].data_ptr(), c["qkv"].stride(0), tab.data_ptr(), tab.stride(0), tab.shape[1],
        c["layer"] * 2 * H * 32 * D,
        c["kp"].data_ptr() if T0 else None, c["vp"].data_ptr() if T0 else None, c["kp"].stride(0) if T0 else 0, T0, B,
        H, D, c["lens"].data_ptr(), window, c["fmt"], done.data_ptr() if done is not None else None,
        done.stride(0) if done is not None else 0, stop.data_ptr() if stop is not None else None, out.data_ptr(),
        out.stride(0), D ** -0.5, _stream_handle())
    assert rc == 0
    torch.cuda.synchronize()
    return out


def _run_dense_one(c, b, window=0):
    """The lockstep kernel on stream b alone (plain layout) at its own length: batch-invariant, so it is the
    reference for that stream inside any batch."""
    T0, L0 = c["T0"], int(c["lens_np"][b])
    k, v = c["dk"][b:b + 1].clone(), c["dv"][b:b + 1].clone()
    out = torch.empty((1, H * D), device="cuda").half()
    cap = T0 + k.shape[2]
    rc = _lib.lib().ns_decode_attention_ex(
        c["qkv"][b:].data_ptr(), c["qkv"].stride(0), k.data_ptr(), v.data_ptr(), k.stride(0), k.stride(1), 0,
        c["kp"].data_ptr() if T0 else None, c["vp"].data_ptr() if T0 else None, c["kp"].stride(0) if T0 else 0, T0, 1,
        H, D, L0, None, cap, window, c["fmt"], None, 0, None, out.data_ptr(), out.stride(0), D ** -0.5,
        _stream_handle())
    assert rc == 0
    torch.cuda.synchronize()
    return out[0], k[0], v[0]


@pytest.mark.parametrize("kv", ["fp16", "fp8"])
@pytest.mark.parametrize("B,T0,window", [(5, 32, 0), (5, 0, 0), (300, 32, 0), (300, 7, 0), (300, 32, 100),
                                         (90, 32, 40)])
def test_paged_attention_equals_lockstep_kernel(kv, B, T0, window):
    c = _paged_case(B, T0, kv, seed=B + T0 + window)
    out = _run_paged(c, B, window)
    esz_rows = c["pool"]
    page_bytes = c["pool"][0].numel() * c["pool"].element_size()
    base = c["pool"].data_ptr()
    for b in range(B) if B <= 5 else list(range(0, B, 37)) + [B - 1]:
        ref, kref, vref = _run_dense_one(c, b, window)
        assert torch.equal(out[b], ref), b
        r = int(c["lens_np"][b]) - T0  # the appended row landed in the stream's page
        pg = (int(c["table"][b, r // 32].item()) - base) // page_bytes
        assert torch.equal(esz_rows[pg, c["layer"], 0, :, r % 32], kref[:, r])
        assert torch.equal(esz_rows[pg, c["layer"], 1, :, r % 32], vref[:, r])
        assert not esz_rows[pg, 1 - c["layer"]].any()  # the other layer's block untouched


@pytest.mark.parametrize("B", [4, 200])
def test_paged_attention_skips_and_poisons(B):
    """done flags / stop lengths skip a stream (output untouched, nothing written); a stream whose new-token page
    is missing gets NaN rows (the coder rejects them) and writes nothing; the others' bits do not change."""
    c = _paged_case(B, 32, "fp16", seed=99 + B)
    ref = _run_paged(c, B)
    flags = torch.zeros((B, 8), dtype=torch.int32, device="cuda")
    flags[1::3, 7] = 1
    pool0 = c["pool"].clone()
    got = _run_paged(c, B, done=flags[:, 7])
    skip = (flags[:, 7] & 1) == 1
    assert torch.equal(got[~skip], ref[~skip]) and (got[skip] == 7.0).all()
    stop = c["lens"].clone()
    stop[::2] += 1  # even streams run, odd ones are at their stop
    got = _run_paged(c, B, stop=stop)
    run = torch.arange(B, device="cuda") % 2 == 0
    assert torch.equal(got[run], ref[run]) and (got[~run] == 7.0).all()
    # missing page for stream 2's new token
    tab = c["table"].clone()
    r = int(c["lens_np"][2]) - 32
    tab[2, r // 32] = 0
    c["pool"].copy_(pool0)
    got = _run_paged(c, B, table=tab)
    assert torch.isnan(got[2]).all()
    keep = torch.ones(B, dtype=torch.bool, device="cuda")
    keep[2] = False
    assert torch.equal(got[keep], ref[keep])


# ----------------------------------------------------------------------------------------------- slot schedulers
Q = {"temp": 0.9, "precision": 26, "topk": 300}


def _provider(scale=6.0, seed=41, **kw):
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2

    return HipArithmeticLM(random_gpt2("gpt2", seed=seed), None, logits_dtype="f16", logit_scale=scale, **kw)


def _record_alone(lm, bits, ctx):
    """One message alone through one slot, eager, with every step's logits copied to the host."""
    seen = []
    orig_prefill, orig_static = lm.lm.prefill, lm.lm.step_static

    def rec_prefill(*a, **k):
        out = orig_prefill(*a, **k)
        seen.append(out[0, : lm.vocab].float().cpu().numpy())
        return out

    def rec_static(tok):
        out = orig_static(tok)
        seen.append(out[0, : lm.vocab].float().cpu().numpy())
        return out

    lm.lm.prefill, lm.lm.step_static = rec_prefill, rec_static
    try:
        toks = lm.encode_batch([bits], ctx, quality=Q, graphs=False)[0]
    finally:
        lm.lm.prefill, lm.lm.step_static = orig_prefill, orig_static
    return toks, seen


def test_slot_refill_same_tokens_as_lockstep_and_alone_and_oracle():
    lm = _provider()
    ctx = [lm.vocab - 1] + list(synthetic.DEFAULT_CONTEXT[1:])
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, n)) for s, n in
            enumerate([24, 3, 40, 16, 1, 31, 24, 8, 48, 12, 20, 5])]
    lock = lm.encode_batch(bits, ctx, quality=Q)  # 12 slots at once (compaction at the tail)
    lens = sorted(map(len, lock))
    assert lens[-1] > 2 * lens[len(lens) // 2], lens  # peaked rows: uneven covers
    assert lm.last_schedule["compactions"] >= 1
    refill = lm.encode_batch(bits, ctx, quality=Q, slots=4)  # 12 messages through 4 slots
    assert refill == lock
    eager = lm.encode_batch(bits, ctx, quality=Q, slots=5, graphs=False)
    assert eager == lock
    for s in (2, 9):
        alone, seen = _record_alone(lm, bits[s], ctx)
        assert alone == lock[s]
        o, _ = oracle.encode_stream(lambda t: seen[t], bits[s], banned=[lm.vocab - 1, 628], temp=Q["temp"],
                                    precision=Q["precision"], topk=Q["topk"])
        assert o == lock[s], s
    for slots in (3, 12):
        for graphs in (True, False):
            out = lm.decode_batch(lock, ctx, quality=Q, slots=slots, graphs=graphs)
            assert all(o[: len(b)] == b for o, b in zip(out, bits)), (slots, graphs)


def test_eviction_when_the_pool_is_small_gives_the_same_tokens():
    ctx = [50256] + list(synthetic.DEFAULT_CONTEXT[1:])
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(100 + s, 40)) for s in range(8)]
    ref_lm = _provider(seed=43)
    ref = ref_lm.encode_batch(bits, ctx, quality=Q)
    del ref_lm
    lm = _provider(seed=43)
    lm.lm.kv_segment_pages = 1  # a page-exact budget
    pool = lm.lm.page_pool()
    cap_pages = 14  # far fewer than 8 live covers of ~80-150 tokens need at their peak
    pool.budget_bytes = lambda: (cap_pages - pool.total) * pool.page_bytes
    got = lm.encode_batch(bits, ctx, quality=Q)
    assert got == ref
    assert lm.last_schedule["evictions"] > 0, lm.last_schedule
    assert pool.total <= cap_pages
    out = lm.decode_batch(got, ctx, quality=Q)  # admission maps a message's pages up front: fewer at once
    assert all(o[: len(b)] == b for o, b in zip(out, bits))


def test_kv_capacity_error_not_torch_oom():
    from neuralsteganography_amd.exceptions import KVCapacityError

    lm = _provider(seed=44)
    lm.lm.kv_segment_pages = 1  # a page-exact budget
    pool = lm.lm.page_pool()
    pool.budget_bytes = lambda: (2 - pool.total) * pool.page_bytes  # 2 pages: 64 positions per message at most
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(5, 200))]
    with pytest.raises(KVCapacityError):
        lm.encode_batch(bits, synthetic.DEFAULT_CONTEXT, quality=Q)


def test_device_string_cuda_round_trip():
    """``device="cuda"`` (no index) -- the reference's usual string -- encodes and decodes."""
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2

    lm = HipArithmeticLM(random_gpt2("gpt2", seed=3), None, device="cuda", logits_dtype="f16")
    assert lm.lm.device.index is not None
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, 10)) for s in range(3)]
    for graphs in (True, False):
        toks = lm.encode_batch(bits, synthetic.DEFAULT_CONTEXT, quality=Q, graphs=graphs)
        out = lm.decode_batch(toks, synthetic.DEFAULT_CONTEXT, quality=Q, graphs=graphs)
        assert all(o[: len(b)] == b for o, b in zip(out, bits))


def test_slots_keep_statistics_and_stop_text():
    """Refilled slots carry the per-message features of the lockstep batch: the statistics accumulators (reset per
    message) and the '<eos>'-style stop text (the eager, per-step checked loop) -- the same tokens and statistics
    through 3-4 slots as all at once."""
    lm = _provider(scale=4.0, seed=47)
    ctx = [lm.vocab - 1] + list(synthetic.DEFAULT_CONTEXT[1:])
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(200 + s, n)) for s, n in
            enumerate([40, 10, 90, 30, 70, 20, 60, 50, 80, 35])]
    a, sa = lm.encode_batch(bits, ctx, quality=Q, return_stats=True)
    b, sb = lm.encode_batch(bits, ctx, quality=Q, return_stats=True, slots=3)
    assert a == b
    assert sa == sb  # per-message float64 accumulators, reset when a slot takes a message
    c = lm.encode_batch(bits, ctx, quality=Q, stop_text="e", slots=4)
    d = lm.encode_batch(bits, ctx, quality=Q, stop_text="e")
    assert c == d
    stopped = [i for i, t in enumerate(d) if len(t) < len(a[i])]
    assert stopped, "no cover reached the stop text: pick another one"
    for i in stopped:
        assert lm.tokenizer.decode(d[i]).endswith("e") and d[i] == a[i][: len(d[i])]


def test_history_and_table_growth_inside_the_pipelined_loop():
    """A tiny initial token history and page-table width (8 tokens) make the pipelined loop grow both several times
    (each a re-captured graph): the tokens equal the eager loop's and the default budget's."""
    lm = _provider(seed=48)
    ctx = synthetic.DEFAULT_CONTEXT
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(300 + s, n)) for s, n in enumerate([20, 5, 30, 12])]
    ref = lm.encode_batch(bits, ctx, quality=Q)
    lm.slot_budget_tokens = 8
    try:
        assert lm.encode_batch(bits, ctx, quality=Q) == ref
        assert lm.encode_batch(bits, ctx, quality=Q, graphs=False, slots=2) == ref
    finally:
        lm.slot_budget_tokens = None
    assert max(map(len, ref)) > 64  # several growths of the 8-token start


@pytest.mark.parametrize("order,cu_split", [("alternate", None), ("free", None), ("split", None), ("split", 0.5)])
def test_two_decode_lanes_give_the_same_tokens(order, cu_split):
    """The decode step as two row halves on two streams (``decode_lanes = 2``, one half's GEMMs beside the other's
    attention): the same tokens as one launch chain -- graph-replayed with refilled slots and compaction, eager -- and
    the decode round-trips through the lanes too."""
    lm = _provider(seed=49)
    ctx = [lm.vocab - 1] + list(synthetic.DEFAULT_CONTEXT[1:])
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(400 + s, n)) for s, n in
            enumerate([24, 3, 40, 16, 1, 31, 24, 8, 48, 12, 20, 5, 33, 9, 17, 26, 2, 44, 11, 30])]
    ref = lm.encode_batch(bits, ctx, quality=Q)
    lm.lm.decode_lanes, lm.lm.decode_lanes_min_batch, lm.lm.decode_lanes_order = 2, 2, order
    lm.lm.decode_lane_cu_split = cu_split
    graphs = order != "split"  # the split form runs eagerly only
    try:
        assert lm.encode_batch(bits, ctx, quality=Q, graphs=graphs) == ref
        assert lm.encode_batch(bits, ctx, quality=Q, slots=7, graphs=graphs) == ref
        assert lm.encode_batch(bits, ctx, quality=Q, graphs=False) == ref
        out = lm.decode_batch(ref, ctx, quality=Q, graphs=graphs)
        assert all(o[: len(b)] == b for o, b in zip(out, bits))
    finally:
        lm.lm.decode_lanes = 1
