"""GPU: the batch-invariant decode-step kernels (include/nsg_lm.h, csrc/nsg_lm.hip; fixed-split attention of
csrc/nsg_attn.hip).

* numerics vs plain PyTorch fp32 references of the same ops (fp16 outputs: tolerances in each test);
* batch invariance: a row's result is BIT-identical whatever M (and hence whichever kernel variant / tile and
  position in the tile) computes it -- the property the arithmetic decoder needs (a cover encoded
  among B streams is revealed alone);
* end to end: fp16 GPT-2 logits of a stream equal bit for bit across batch sizes, and covers made with
  cover_generate_batch at B > 1 in fp16 reveal one by one with cover_reveal.
"""

import math

import pytest

torch = pytest.importorskip("torch")

from neuralsteganography_amd import _lib, synthetic  # noqa: E402
from neuralsteganography_amd.coder import _stream_handle  # noqa: E402

pytestmark = pytest.mark.gpu

EPIS = {"store": _lib.NS_LM_EPI_STORE, "gelu": _lib.NS_LM_EPI_GELU, "residual": _lib.NS_LM_EPI_RESIDUAL,
        "f32": _lib.NS_LM_EPI_STORE_F32}


def _gemm(x, wt, bias, y, epi):
    M, K = x.shape
    N = wt.shape[0]
    rc = _lib.lib().ns_lm_gemm(x.data_ptr(), x.stride(0), wt.data_ptr(), wt.stride(0),
                               bias.data_ptr() if bias is not None else None, y.data_ptr(), y.stride(0), M, N, K,
                               EPIS[epi], _stream_handle())
    assert rc == 0
    return y


def _ref(x, wt, bias, y0, epi):
    acc = x.double() @ wt.double().t()
    if bias is not None:
        acc = acc + bias.double()
    if epi == "gelu":
        acc = 0.5 * acc * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (acc + 0.044715 * acc ** 3)))
    if epi == "residual":
        acc = y0.double() + acc
    return acc


def _operands(M, N, K, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn((M, K), generator=g, device="cuda").half()
    wt = (torch.randn((N, K), generator=g, device="cuda") / math.sqrt(K)).half()
    bias = (0.5 * torch.randn((N,), generator=g, device="cuda")).half()
    return x, wt, bias


@pytest.mark.parametrize("M,N,K", [(1, 768, 768), (5, 2304, 768), (16, 64, 128), (17, 768, 3072), (33, 1024, 1024),
                                   (64, 3072, 768), (65, 768, 768), (200, 2304, 768), (1000, 768, 3072),
                                   (2048, 2048, 768), (4096, 2304, 768)])
@pytest.mark.parametrize("epi", ["store", "gelu", "residual", "f32"])
def test_gemm_matches_fp64_reference(M, N, K, epi):
    """ns_lm_gemm vs float64 torch: fp32 accumulation of exact fp16 products, one fp16 rounding of the result
    (2^-11 relative) -> |err| <= 2e-3 |ref| + 2e-3 on O(1) outputs."""
    x, wt, bias = _operands(M, N, K, seed=M * 7 + N)
    if epi == "f32":
        y = torch.full((M, N), float("nan"), device="cuda")
    elif epi == "residual":
        y = torch.randn((M, N), device="cuda").half()
    else:
        y = torch.full((M, N), float("nan"), device="cuda").half()
    y0 = y.clone()
    use_bias = bias if (M + N) % 2 == 0 or epi != "store" else None
    _gemm(x, wt, use_bias, y, epi)
    torch.cuda.synchronize()
    want = _ref(x, wt, use_bias, y0, epi)
    err = (y.double() - want).abs()
    assert torch.isfinite(y).all()
    assert (err <= 2e-3 * want.abs() + 2e-3).all(), err.max().item()


def test_gemm_ragged_leading_dims_and_rejections():
    """Strided rows (ld > K / N) read and write only their own columns; bad shapes are refused, not launched."""
    M, N, K = 70, 192, 256
    x, wt, bias = _operands(M, N, K, seed=3)
    xs = torch.zeros((M, K + 64), device="cuda").half()
    xs[:, :K] = x
    ys = torch.full((M, N + 8), 7.0, device="cuda").half()
    _gemm(xs[:, :K], wt, bias, ys[:, :N], "store")
    torch.cuda.synchronize()
    assert torch.equal(ys[:, N:], torch.full((M, 8), 7.0, device="cuda").half())
    want = _ref(x, wt, bias, None, "store")
    assert ((ys[:, :N].double() - want).abs() <= 2e-3 * want.abs() + 2e-3).all()
    f = _lib.lib().ns_lm_gemm
    y = torch.empty((M, N), device="cuda").half()
    assert f(x.data_ptr(), K, wt.data_ptr(), K, None, y.data_ptr(), N, M, N, 96, 0, None) == _lib.NS_ERR_UNSUPPORTED
    assert f(x.data_ptr(), K, wt.data_ptr(), K, None, y.data_ptr(), N, M, 100, K, 0, None) == _lib.NS_ERR_UNSUPPORTED
    assert f(x.data_ptr(), K, wt.data_ptr(), K, None, y.data_ptr(), N, M, N, K, 9, None) == _lib.NS_ERR_CONFIG
    assert f(x.data_ptr(), K - 8, wt.data_ptr(), K, None, y.data_ptr(), N, M, N, K, 0, None) == _lib.NS_ERR_CONFIG


@pytest.mark.parametrize("N,K,epi", [(2304, 768, "store"), (768, 3072, "residual"), (3072, 768, "gelu"),
                                     (1024, 1024, "f32")])
def test_gemm_rows_are_batch_invariant(N, K, epi):
    """The same activation row gives the same output bits for every M (direct kernels M <= 16/32/64, 64x64 and
    128x128 LDS tiles above) and every position of the row in its tile."""
    Mbig = 4096
    x, wt, bias = _operands(Mbig, N, K, seed=N + K)
    ydt = torch.float32 if epi == "f32" else torch.float16
    y0 = torch.randn((Mbig, N), device="cuda").to(ydt)
    full = y0.clone()
    _gemm(x, wt, bias, full, epi)
    for M, off in [(1, 0), (1, 1234), (3, 7), (16, 100), (17, 31), (32, 5), (40, 2000), (64, 64), (65, 9),
                   (300, 1), (1000, 1111), (2000, 3), (4000, 90)]:
        y = y0[off:off + M].clone()
        _gemm(x[off:off + M], wt, bias, y, epi)
        torch.cuda.synchronize()
        assert torch.equal(y, full[off:off + M]), (M, off)


@pytest.mark.parametrize("M,N,K,epi", [(1, 768, 768, "store"), (70, 2304, 768, "gelu"), (300, 768, 3072, "residual"),
                                       (129, 1024, 1024, "f32")])
def test_gemm_tile_configurations_agree_bitwise(M, N, K, epi):
    """Every tile configuration (direct 16/32/64-row waves, 64x64 .. 256x128 LDS tiles, 2-4 stages) produces
    the same bits: the configuration is a speed choice only."""
    x, wt, bias = _operands(M, N, K, seed=M + 2 * N)
    ydt = torch.float32 if epi == "f32" else torch.float16
    y0 = torch.randn((M, N), device="cuda").to(ydt)
    ref = y0.clone()
    _gemm(x, wt, bias, ref, epi)
    n = _lib.lib().ns_lm_gemm_configs()
    assert n >= 8
    for cfg in range(n):
        y = y0.clone()
        rc = _lib.lib().ns_lm_gemm_config(x.data_ptr(), K, wt.data_ptr(), K, bias.data_ptr(), y.data_ptr(), N, M, N, K,
                                          EPIS[epi], cfg, _stream_handle())
        assert rc == 0
        torch.cuda.synchronize()
        assert torch.equal(y, ref), cfg
    assert _lib.lib().ns_lm_gemm_config(x.data_ptr(), K, wt.data_ptr(), K, None, y0.data_ptr(), N, M, N, K, 0, n,
                                        None) == _lib.NS_ERR_CONFIG


@pytest.mark.parametrize("M,N,K,epi,with_bias", [(1100, 8192, 768, "f32", False), (4096, 3072, 768, "gelu", True),
                                                  (777, 2304, 768, "store", True), (300, 1024, 3072, "gelu", True),
                                                  (129, 1536, 2048, "f32", True), (5000, 768, 64, "store", False),
                                                  (333, 2176, 768, "f32", False)])
def test_gemm_persistent_configurations_agree_bitwise(M, N, K, epi, with_bias):
    """The 256 x 256 (plain and ping-pong) and persistent 128 x 128 kernels (one workgroup per CU looping over
    several tiles): ragged last row / column blocks, K-chain splits, one-K-tile tiles, with and without bias) give the tiled kernel's bits and the fp64 result."""
    x, wt, bias = _operands(M, N, K, seed=M + 3 * N + K)
    b = bias if with_bias else None
    ydt = torch.float32 if epi == "f32" else torch.float16
    y0 = torch.full((M + 1, N), 7.0, device="cuda").to(ydt)  # one guard row past M: never written
    L = _lib.lib()
    n = L.ns_lm_gemm_configs()

    def run(cfg):
        y = y0.clone()
        rc = L.ns_lm_gemm_config(x.data_ptr(), K, wt.data_ptr(), K, b.data_ptr() if b is not None else None,
                                 y.data_ptr(), N, M, N, K, EPIS[epi], cfg, _stream_handle())
        assert rc == 0
        torch.cuda.synchronize()
        return y

    ref = run(6)  # CFG_T128_3
    assert torch.equal(ref[M], y0[M])
    want = _ref(x, wt, b, None, epi)
    assert ((ref[:M].double() - want).abs() <= 2e-3 * want.abs() + 2e-3).all()
    for cfg in range(13, n):  # from CFG_B256 on: the 256 x 256, persistent and ping-pong kernels
        y = run(cfg)
        assert torch.equal(y, ref), cfg


@pytest.mark.parametrize("M,C", [(1, 768), (7, 1024), (300, 768), (5, 64), (33, 1600)])
def test_layernorm_matches_torch(M, C):
    g = torch.Generator(device="cuda").manual_seed(M + C)
    x = (3 * torch.randn((M, C), generator=g, device="cuda") + 1).half()
    w = torch.randn((C,), generator=g, device="cuda").half()
    b = torch.randn((C,), generator=g, device="cuda").half()
    y = torch.full((M, C), float("nan"), device="cuda").half()
    rc = _lib.lib().ns_lm_layernorm(x.data_ptr(), C, w.data_ptr(), b.data_ptr(), y.data_ptr(), C, M, C, 1e-5,
                                    _stream_handle())
    assert rc == 0
    want = torch.nn.functional.layer_norm(x.float(), (C,), w.float(), b.float(), 1e-5)
    assert ((y.float() - want).abs() <= 2e-3 * want.abs() + 4e-3).all()
    # batch invariance: row 0 alone equals row 0 of the batch
    y1 = torch.empty((1, C), device="cuda").half()
    _lib.lib().ns_lm_layernorm(x.data_ptr(), C, w.data_ptr(), b.data_ptr(), y1.data_ptr(), C, 1, C, 1e-5,
                               _stream_handle())
    torch.cuda.synchronize()
    assert torch.equal(y1[0], y[0])


@pytest.mark.parametrize("M", [1, 9, 4096])
def test_layernorm_count_advances_the_counter_once(M):
    """ns_lm_layernorm_count (the decode step's ln_f in a captured graph) writes the same rows as
    ns_lm_layernorm and adds exactly one to the device counter, whatever the grid size."""
    C = 768
    g = torch.Generator(device="cuda").manual_seed(M)
    x = torch.randn((M, C), generator=g, device="cuda").half()
    w = torch.randn((C,), generator=g, device="cuda").half()
    b = torch.randn((C,), generator=g, device="cuda").half()
    y0 = torch.empty((M, C), device="cuda").half()
    y1 = torch.empty((M, C), device="cuda").half()
    ctr = torch.tensor([41], dtype=torch.int32, device="cuda")
    L = _lib.lib()
    assert L.ns_lm_layernorm(x.data_ptr(), C, w.data_ptr(), b.data_ptr(), y0.data_ptr(), C, M, C, 1e-5,
                             _stream_handle()) == 0
    for _ in range(3):
        assert L.ns_lm_layernorm_count(x.data_ptr(), C, w.data_ptr(), b.data_ptr(), y1.data_ptr(), C, M, C, 1e-5,
                                       ctr.data_ptr(), _stream_handle()) == 0
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    assert int(ctr.item()) == 44
    # no counter: plain layer norm
    assert L.ns_lm_layernorm_count(x.data_ptr(), C, w.data_ptr(), b.data_ptr(), y1.data_ptr(), C, M, C, 1e-5,
                                   None, _stream_handle()) == 0
    torch.cuda.synchronize()
    assert int(ctr.item()) == 44


@pytest.mark.parametrize("dev_len", [False, True])
def test_embed_ln_matches_torch(dev_len):
    V, P, C, M, L = 1000, 64, 256, 9, 70  # position = 70 % 64 = 6
    g = torch.Generator(device="cuda").manual_seed(5)
    wte = torch.randn((V, C), generator=g, device="cuda").half()
    wpe = torch.randn((P, C), generator=g, device="cuda").half()
    w = torch.randn((C,), generator=g, device="cuda").half()
    b = torch.randn((C,), generator=g, device="cuda").half()
    tok = torch.randint(0, V, (M,), generator=g, device="cuda", dtype=torch.int32)
    h = torch.empty((M, C), device="cuda").half()
    a = torch.empty((M, C), device="cuda").half()
    dL = torch.tensor([L], dtype=torch.int32, device="cuda")
    rc = _lib.lib().ns_lm_embed_ln(tok.data_ptr(), wte.data_ptr(), wpe.data_ptr(), V, P, -1 if dev_len else L,
                                   dL.data_ptr() if dev_len else None, h.data_ptr(), C, w.data_ptr(), b.data_ptr(),
                                   a.data_ptr(), C, M, C, 1e-5, _stream_handle())
    assert rc == 0
    want_h = wte[tok.long()] + wpe[L % P]
    assert torch.equal(h, want_h)
    want_a = torch.nn.functional.layer_norm(want_h.float(), (C,), w.float(), b.float(), 1e-5)
    assert ((a.float() - want_a).abs() <= 2e-3 * want_a.abs() + 4e-3).all()


@pytest.mark.parametrize("L0", [0, 5, 255, 256, 511, 700, 1100])  # one, two, four and eight waves per pair
def test_decode_attention_is_batch_invariant(L0):
    """The attention output of one (stream, head) is bit-identical at B = 1 (one pair per workgroup) and inside
    B = 700 (eight pairs per workgroup): the split of a pair's rows over waves depends on the key count only."""
    B, H, D = 700, 12, 64
    g = torch.Generator(device="cuda").manual_seed(9)
    qkv = torch.randn((B, 3 * H * D), generator=g, device="cuda").half()
    kc = torch.randn((B, H, L0 + 8, D), generator=g, device="cuda").half()
    vc = torch.randn((B, H, L0 + 8, D), generator=g, device="cuda").half()
    f = _lib.lib().ns_decode_attention
    out = torch.empty((B, H * D), device="cuda").half()
    assert f(qkv.data_ptr(), qkv.stride(0), kc.data_ptr(), vc.data_ptr(), kc.stride(0), kc.stride(1), B, H, D, L0,
             out.data_ptr(), out.stride(0), D ** -0.5, _stream_handle()) == 0
    # a small batch (one-wave workgroups, partials merged across workgroups) twice in a row: same rows
    for _ in range(2):
        o80 = torch.empty((80, H * D), device="cuda").half()
        assert f(qkv[300:].data_ptr(), qkv.stride(0), kc[300:].data_ptr(), vc[300:].data_ptr(), kc.stride(0),
                 kc.stride(1), 80, H, D, L0, o80.data_ptr(), o80.stride(0), D ** -0.5, _stream_handle()) == 0
        torch.cuda.synchronize()
        assert torch.equal(o80, out[300:380])
    for b in (0, 1, 399, 699):
        o1 = torch.empty((1, H * D), device="cuda").half()
        assert f(qkv[b:].data_ptr(), qkv.stride(0), kc[b:].data_ptr(), vc[b:].data_ptr(), kc.stride(0),
                 kc.stride(1), 1, H, D, L0, o1.data_ptr(), o1.stride(0), D ** -0.5, _stream_handle()) == 0
        torch.cuda.synchronize()
        assert torch.equal(o1[0], out[b]), b


@pytest.mark.parametrize("T0,L0,dev", [(32, 40, False), (32, 40, True), (1, 1, False), (100, 350, True),
                                       (7, 7, False)])
def test_prefix_attention_equals_full_cache(T0, L0, dev):
    """ns_decode_attention_prefix (context rows stored once, shared by every stream) gives the same bits as
    ns_decode_attention over a per-stream cache holding the same rows, and appends the new k/v at stream index
    L0 - T0."""
    B, H, D = 40, 12, 64
    cap = L0 + 3
    g = torch.Generator(device="cuda").manual_seed(T0 + L0)
    qkv = torch.randn((B, 3 * H * D), generator=g, device="cuda").half()
    kp = torch.randn((H, T0, D), generator=g, device="cuda").half()
    vp = torch.randn((H, T0, D), generator=g, device="cuda").half()
    ks = torch.randn((B, H, cap - T0, D), generator=g, device="cuda").half()
    vs = torch.randn((B, H, cap - T0, D), generator=g, device="cuda").half()
    full_k = torch.cat([kp[None].expand(B, -1, -1, -1), ks], dim=2).contiguous()
    full_v = torch.cat([vp[None].expand(B, -1, -1, -1), vs], dim=2).contiguous()
    want = torch.empty((B, H * D), device="cuda").half()
    lib = _lib.lib()
    assert lib.ns_decode_attention(qkv.data_ptr(), qkv.stride(0), full_k.data_ptr(), full_v.data_ptr(),
                                   full_k.stride(0), full_k.stride(1), B, H, D, L0, want.data_ptr(), want.stride(0),
                                   D ** -0.5, _stream_handle()) == 0
    got = torch.empty((B, H * D), device="cuda").half()
    dL = torch.tensor([L0], dtype=torch.int32, device="cuda")
    assert lib.ns_decode_attention_prefix(qkv.data_ptr(), qkv.stride(0), ks.data_ptr(), vs.data_ptr(), ks.stride(0),
                                          ks.stride(1), 0, kp.data_ptr(), vp.data_ptr(), kp.stride(0), T0, B, H, D,
                                          -1 if dev else L0, dL.data_ptr() if dev else None, cap, 0, got.data_ptr(),
                                          got.stride(0), D ** -0.5, _stream_handle()) == 0
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    assert torch.equal(ks[:, :, L0 - T0], full_k[:, :, L0]) and torch.equal(vs[:, :, L0 - T0], full_v[:, :, L0])
    # a position inside the prefix cannot be appended
    assert lib.ns_decode_attention_prefix(qkv.data_ptr(), qkv.stride(0), ks.data_ptr(), vs.data_ptr(), ks.stride(0),
                                          ks.stride(1), 0, kp.data_ptr(), vp.data_ptr(), kp.stride(0), T0, B, H, D,
                                          T0 - 1, None, cap, 0, got.data_ptr(), got.stride(0), D ** -0.5,
                                          None) == _lib.NS_ERR_CONFIG


@pytest.mark.parametrize("kv", ["fp16", "fp8"])
@pytest.mark.parametrize("T0,L0", [(0, 100), (32, 32), (32, 300), (5, 1000)])
def test_chunk_plane_layout_equals_plain(kv, T0, L0):
    """The chunk-plane cache layout ([chunk][B][H][32][D]: the rows a step reads stay dense whatever the
    capacity) gives the same bits as the plain [B][H][rows][D] layout holding the same rows, and appends the
    new token at the same logical position."""
    B, H, D = 24, 12, 64
    rows = L0 - T0 + 5
    nch = (rows + 31) // 32
    g = torch.Generator(device="cuda").manual_seed(L0 + T0)
    qkv = torch.randn((B, 3 * H * D), generator=g, device="cuda").half()
    plain_k = torch.randn((B, H, nch * 32, D), generator=g, device="cuda").half()
    plain_v = torch.randn((B, H, nch * 32, D), generator=g, device="cuda").half()
    kp = torch.randn((H, max(T0, 1), D), generator=g, device="cuda").half()
    vp = torch.randn((H, max(T0, 1), D), generator=g, device="cuda").half()
    if kv == "fp8":
        plain_k, plain_v, kp, vp = _q8(plain_k), _q8(plain_v), _q8(kp), _q8(vp)
        f = _lib.lib().ns_decode_attention_fp8
    else:
        f = _lib.lib().ns_decode_attention_prefix
    chunk_k = plain_k.view(B, H, nch, 32, D).permute(2, 0, 1, 3, 4).contiguous()  # [nch, B, H, 32, D]
    chunk_v = plain_v.view(B, H, nch, 32, D).permute(2, 0, 1, 3, 4).contiguous()
    cap = T0 + rows
    outs = []
    for k, v, strides in ((plain_k, plain_v, (plain_k.stride(0), plain_k.stride(1), 0)),
                          (chunk_k, chunk_v, (chunk_k.stride(1), chunk_k.stride(2), chunk_k.stride(0)))):
        o = torch.empty((B, H * D), device="cuda").half()
        assert f(qkv.data_ptr(), qkv.stride(0), k.data_ptr(), v.data_ptr(), *strides, kp.data_ptr() if T0 else None,
                 vp.data_ptr() if T0 else None, kp.stride(0) if T0 else 0, T0, B, H, D, L0, None, cap, 0, o.data_ptr(),
                 o.stride(0), D ** -0.5, _stream_handle()) == 0
        outs.append(o)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    r = L0 - T0
    assert torch.equal(chunk_k[r // 32, :, :, r % 32], plain_k[:, :, r]) and torch.equal(
        chunk_v[r // 32, :, :, r % 32], plain_v[:, :, r])


@pytest.mark.parametrize("logits", ["f16", "f32"])
def test_gpt2_fp16_logits_are_batch_invariant(logits):
    """GPT-2-small fp16 decode steps on the native kernels: every stream's logits at B = 37 equal, bit for bit,
    the logits of the same stream run alone (B = 1) and inside a B = 5 batch, over several steps."""
    from neuralsteganography_amd.lm.gpt2 import BatchedGPT2, random_gpt2

    m = random_gpt2("gpt2", seed=8)
    ldt = torch.float16 if logits == "f16" else torch.float32
    ctx = synthetic.DEFAULT_CONTEXT
    g = torch.Generator().manual_seed(1)
    steps = 4
    toks = torch.randint(0, 50257, (steps, 37), generator=g)
    big = BatchedGPT2(m, device="cuda", compute_dtype=torch.float16, logits_dtype=ldt)
    out_big = [big.prefill(ctx, 37, steps + 1)]
    for t in range(steps):
        out_big.append(big.step(toks[t].cuda()))
    for rows in ([0], [36], [3, 10, 11, 20, 30]):
        small = BatchedGPT2(m, device="cuda", compute_dtype=torch.float16, logits_dtype=ldt)
        out = [small.prefill(ctx, len(rows), steps + 1)]
        for t in range(steps):
            out.append(small.step(toks[t, rows].cuda()))
        for t in range(steps + 1):
            assert torch.equal(out[t], out_big[t][rows]), (rows, t)


def test_fp16_cover_batch_reveals_alone():
    """covers encoded with cover_generate_batch at B > 1 in fp16 -- the default on the GPU --
    reveal one at a time with cover_reveal (B = 1), and the spans of a stego_encode_batch decode per message."""
    from neuralsteganography_amd.cover import cover_generate_batch, cover_reveal
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2
    from test_gpu_guard import IdTokenizer

    m = random_gpt2("tiny", vocab_size=2000, n_positions=1024, n_embd=128, n_head=2, seed=23)
    lm = HipArithmeticLM(m, IdTokenizer(2000), compute_dtype=torch.float16, logits_dtype="f16")
    assert lm.lm.native
    q = {"temp": 0.9, "precision": 26, "topk": 300, "finish_sent": False}
    secrets = [b"first secret", bytes(range(60)), b"z", b"another one, a little longer than the rest"]
    seed = "w5. w6. w3"
    texts = cover_generate_batch(secrets, seed_text=seed, quality=q, ecc="none", lm=lm, quality_gate=False,
                                 chunk_bytes=24)
    for text, secret in zip(texts, secrets):
        assert cover_reveal(text, seed_text=seed, quality=q, ecc="none", lm=lm) == secret


# ------------------------------------------------------------------------------------------ fp8 KV cache (opt-in)
def _q8(t):
    out = torch.empty(t.shape, dtype=torch.uint8, device="cuda")
    assert _lib.lib().ns_quantize_fp8(t.contiguous().data_ptr(), out.data_ptr(), t.numel(), _stream_handle()) == 0
    return out


def _dq8(u):
    return u.view(torch.float8_e4m3fn).float()


def test_fp8_quantizer_matches_torch_e4m3fn():
    """ns_quantize_fp8 = round-to-nearest-even OCP e4m3fn with saturation to +-448 (torch's float8_e4m3fn cast
    of the clamped value)."""
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.cat([torch.randn(4096, generator=g, device="cuda") * s for s in (1e-3, 0.1, 1.0, 30.0, 600.0)]).half()
    got = _q8(x)
    want = x.float().clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    torch.cuda.synchronize()
    assert torch.equal(got, want)


@pytest.mark.parametrize("B,L0,T0", [(3, 0, 0), (5, 77, 0), (40, 300, 32), (700, 1030, 32), (2, 2000, 1)])
def test_fp8_attention_matches_fp32_reference(B, L0, T0):
    """ns_decode_attention_fp8 vs softmax(q k^T / sqrt(D)) v in fp32 over the DEQUANTISED fp8 rows (the new
    token's k/v quantised the same way); the new k/v land in the cache as fp8.  2e-3 absolute (fp16 output)."""
    H, D = 12, 64
    cap = L0 + 4
    g = torch.Generator(device="cuda").manual_seed(L0 + B)
    qkv = torch.randn((B, 3 * H * D), generator=g, device="cuda").half()
    kf = torch.randn((B, H, cap, D), generator=g, device="cuda").half()
    vf = torch.randn((B, H, cap, D), generator=g, device="cuda").half()
    k8, v8 = _q8(kf), _q8(vf)
    kp, vp = k8[0, :, :T0].contiguous(), v8[0, :, :T0].contiguous()
    ks, vs = k8[:, :, T0:].contiguous(), v8[:, :, T0:].contiguous()
    out = torch.empty((B, H * D), device="cuda").half()
    rc = _lib.lib().ns_decode_attention_fp8(qkv.data_ptr(), qkv.stride(0), ks.data_ptr(), vs.data_ptr(), ks.stride(0),
                                            ks.stride(1), 0, kp.data_ptr() if T0 else None,
                                            vp.data_ptr() if T0 else None, kp.stride(0) if T0 else 0, T0, B, H, D, L0,
                                            None, cap, 0, out.data_ptr(), out.stride(0), D ** -0.5, _stream_handle())
    assert rc == 0
    torch.cuda.synchronize()
    q, k, v = qkv.view(B, 3, H, D).unbind(1)
    kk = torch.cat([kp[None].expand(B, -1, -1, -1), ks], dim=2) if T0 else ks.clone()
    vv = torch.cat([vp[None].expand(B, -1, -1, -1), vs], dim=2) if T0 else vs.clone()
    kk, vv = _dq8(kk.contiguous()), _dq8(vv.contiguous())
    kk[:, :, L0] = _dq8(_q8(k))
    vv[:, :, L0] = _dq8(_q8(v))
    s = torch.einsum("bhd,bhjd->bhj", q.float(), kk[:, :, : L0 + 1]) * D ** -0.5
    want = torch.einsum("bhj,bhjd->bhd", torch.softmax(s, -1), vv[:, :, : L0 + 1]).reshape(B, H * D)
    assert (out.float() - want).abs().max().item() < 2e-3
    assert torch.equal(ks[:, :, L0 - T0], _q8(k)) and torch.equal(vs[:, :, L0 - T0], _q8(v))


def test_fp8_attention_is_batch_invariant():
    B, H, D, L0 = 300, 12, 64, 700
    g = torch.Generator(device="cuda").manual_seed(2)
    qkv = torch.randn((B, 3 * H * D), generator=g, device="cuda").half()
    kc = _q8(torch.randn((B, H, L0 + 2, D), generator=g, device="cuda").half())
    vc = _q8(torch.randn((B, H, L0 + 2, D), generator=g, device="cuda").half())
    f = _lib.lib().ns_decode_attention_fp8
    out = torch.empty((B, H * D), device="cuda").half()
    assert f(qkv.data_ptr(), qkv.stride(0), kc.data_ptr(), vc.data_ptr(), kc.stride(0), kc.stride(1), 0, None, None,
             0, 0, B, H, D, L0, None, L0 + 2, 0, out.data_ptr(), out.stride(0), D ** -0.5, _stream_handle()) == 0
    for b in (0, 150, 299):
        o1 = torch.empty((1, H * D), device="cuda").half()
        assert f(qkv[b:].data_ptr(), qkv.stride(0), kc[b:].data_ptr(), vc[b:].data_ptr(), kc.stride(0), kc.stride(1),
                 0, None, None, 0, 0, 1, H, D, L0, None, L0 + 2, 0, o1.data_ptr(), o1.stride(0), D ** -0.5,
                 _stream_handle()) == 0
        torch.cuda.synchronize()
        assert torch.equal(o1[0], out[b]), b


def test_gpt2_fp8_kv_logits_close_and_batch_invariant():
    """GPT-2-small with the fp8 KV cache: logits within the fp8 quantisation error of the fp16 cache's
    (random-init weights), and bit-identical for a stream at B = 1 and B = 9."""
    from neuralsteganography_amd.lm.gpt2 import BatchedGPT2, random_gpt2

    m = random_gpt2("gpt2", seed=8)
    ctx = synthetic.DEFAULT_CONTEXT
    toks = torch.randint(0, 50257, (5, 9), generator=torch.Generator().manual_seed(3))
    outs = {}
    for kvd, B in (("fp16", 9), ("fp8", 9), ("fp8", 1)):
        lm = BatchedGPT2(m, device="cuda", compute_dtype=torch.float16, logits_dtype=torch.float32, kv_dtype=kvd)
        lo = [lm.prefill(ctx, B, 8)]
        for t in range(5):
            lo.append(lm.step(toks[t, :B].cuda()))
        outs[(kvd, B)] = lo
    for t in range(6):
        assert torch.equal(outs[("fp8", 1)][t][0], outs[("fp8", 9)][t][0]), t
        assert (outs[("fp8", 9)][t] - outs[("fp16", 9)][t]).abs().max().item() < 0.1


def test_fp8_kv_cover_batch_reveals_alone():
    from neuralsteganography_amd.cover import cover_generate_batch, cover_reveal
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2
    from test_gpu_guard import IdTokenizer

    m = random_gpt2("tiny", vocab_size=2000, n_positions=1024, n_embd=128, n_head=2, seed=29)
    lm = HipArithmeticLM(m, IdTokenizer(2000), compute_dtype=torch.float16, logits_dtype="f16", kv_dtype="fp8")
    q = {"temp": 0.9, "precision": 26, "topk": 300, "finish_sent": False}
    secrets = [b"fp8 cache", bytes(range(40)), b"x"]
    seed = "w5. w6. w3"
    texts = cover_generate_batch(secrets, seed_text=seed, quality=q, ecc="none", lm=lm, quality_gate=False,
                                 chunk_bytes=24)
    for text, secret in zip(texts, secrets):
        assert cover_reveal(text, seed_text=seed, quality=q, ecc="none", lm=lm) == secret


# --------------------------------------------------------------------------------- attention window (opt-in)
@pytest.mark.parametrize("kv", ["fp16", "fp8"])
@pytest.mark.parametrize("T0,L0,W", [(32, 40, 16), (32, 300, 64), (32, 300, 290), (5, 1000, 200), (0, 77, 1),
                                     (32, 31 + 5, 100)])
def test_window_attention_matches_reference(kv, T0, L0, W):
    """window > 0: softmax over the last W positions [max(0, L0 + 1 - W), L0] only (prefix rows included while
    inside the window), vs fp32 torch; the output is batch-invariant (B = 1 vs B = 30)."""
    B, H, D = 30, 12, 64
    cap = L0 + 3
    g = torch.Generator(device="cuda").manual_seed(T0 + L0 + W)
    qkv = torch.randn((B, 3 * H * D), generator=g, device="cuda").half()
    kf = torch.randn((B, H, cap, D), generator=g, device="cuda").half()
    vf = torch.randn((B, H, cap, D), generator=g, device="cuda").half()
    if kv == "fp8":
        kq, vq = _q8(kf), _q8(vf)
        deq = _dq8
        f = _lib.lib().ns_decode_attention_fp8
        knew, vnew = _dq8(_q8(qkv.view(B, 3, H, D)[:, 1])), _dq8(_q8(qkv.view(B, 3, H, D)[:, 2]))
    else:
        kq, vq = kf, vf
        deq = lambda t: t.float()  # noqa: E731
        f = _lib.lib().ns_decode_attention_prefix
        knew, vnew = qkv.view(B, 3, H, D)[:, 1].float(), qkv.view(B, 3, H, D)[:, 2].float()
    kp, vp = kq[0, :, :T0].contiguous(), vq[0, :, :T0].contiguous()
    ks, vs = kq[:, :, T0:].contiguous(), vq[:, :, T0:].contiguous()

    def run(b0, nb):
        o = torch.empty((nb, H * D), device="cuda").half()
        assert f(qkv[b0:].data_ptr(), qkv.stride(0), ks[b0:].data_ptr(), vs[b0:].data_ptr(), ks.stride(0), ks.stride(1),
                 0, kp.data_ptr() if T0 else None, vp.data_ptr() if T0 else None, kp.stride(0) if T0 else 0, T0, nb, H,
                 D, L0, None, cap, W, o.data_ptr(), o.stride(0), D ** -0.5, _stream_handle()) == 0
        return o

    out = run(0, B)
    one = run(7, 1)
    torch.cuda.synchronize()
    assert torch.equal(one[0], out[7])
    kk = torch.cat([kp[None].expand(B, -1, -1, -1), ks], dim=2) if T0 else ks
    vv = torch.cat([vp[None].expand(B, -1, -1, -1), vs], dim=2) if T0 else vs
    kk, vv = deq(kk.contiguous()).clone(), deq(vv.contiguous()).clone()
    kk[:, :, L0], vv[:, :, L0] = knew, vnew
    s0 = max(0, L0 + 1 - W)
    q = qkv.view(B, 3, H, D)[:, 0].float()
    sc = torch.einsum("bhd,bhjd->bhj", q, kk[:, :, s0: L0 + 1]) * D ** -0.5
    want = torch.einsum("bhj,bhjd->bhd", torch.softmax(sc, -1), vv[:, :, s0: L0 + 1]).reshape(B, H * D)
    assert (out.float() - want).abs().max().item() < 2e-3


def test_window_cover_batch_reveals_alone():
    """The opt-in modes together (fp8 KV cache + a 24-position attention window, shorter than the covers): covers
    from cover_generate_batch reveal one by one."""
    from neuralsteganography_amd.cover import cover_generate_batch, cover_reveal
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2
    from test_gpu_guard import IdTokenizer

    m = random_gpt2("tiny", vocab_size=2000, n_positions=1024, n_embd=128, n_head=2, seed=31)
    lm = HipArithmeticLM(m, IdTokenizer(2000), compute_dtype=torch.float16, logits_dtype="f16", kv_dtype="fp8",
                         attention_window=24)
    q = {"temp": 0.9, "precision": 26, "topk": 300, "finish_sent": False}
    secrets = [b"windowed attention", bytes(range(50)), b"w"]
    seed = "w5. w6. w3"
    texts = cover_generate_batch(secrets, seed_text=seed, quality=q, ecc="none", lm=lm, quality_gate=False,
                                 chunk_bytes=24)
    for text, secret in zip(texts, secrets):
        assert cover_reveal(text, seed_text=seed, quality=q, ecc="none", lm=lm) == secret


def _seq_attn(qkv, B, T, H, D=64):
    o = torch.empty((B * T, H * D), device="cuda", dtype=torch.float16)
    rc = _lib.lib().ns_seq_attention(qkv.data_ptr(), qkv.stride(0), o.data_ptr(), o.stride(0), B, T, H, D, D ** -0.5,
                                     _stream_handle())
    assert rc == 0
    return o


@pytest.mark.parametrize("B,T,H", [(1, 1, 12), (3, 5, 12), (2, 64, 4), (2, 100, 12), (1, 300, 16), (2, 1024, 2)])
def test_seq_attention_matches_fp32_reference(B, T, H):
    """Causal MFMA flash attention over whole sequences (prefill, guard scoring, max_context windows) vs a plain
    fp32 PyTorch softmax(q k^T / sqrt(D) + causal mask) v of the same fp16 inputs (P is rounded to fp16 for the
    PV product: 2e-3 absolute on unit-scale values)."""
    D = 64
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + T)
    qkv = torch.randn((B * T, 3 * H * D), generator=g, device="cuda").half()
    o = _seq_attn(qkv, B, T, H)
    x = qkv.float().view(B, T, 3, H, D)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    s = (q @ k.transpose(-1, -2)) * D ** -0.5
    s = s.masked_fill(torch.triu(torch.ones(T, T, device="cuda", dtype=torch.bool), 1), float("-inf"))
    ref = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B * T, H * D)
    assert (o.float() - ref).abs().max().item() < 2e-3


def test_seq_attention_rows_depend_on_their_sequence_only():
    """Batch and length invariance of the sequence attention: a sequence's output rows are bit-identical run
    alone, inside a batch of 5, and right-padded to a longer T (causality keeps padding out of real rows)."""
    H, D = 12, 64
    g = torch.Generator(device="cuda").manual_seed(3)
    T = 150
    seqs = torch.randn((5, T, 3 * H * D), generator=g, device="cuda").half()
    big = _seq_attn(seqs.reshape(5 * T, -1).contiguous(), 5, T, H).view(5, T, -1)
    for b in (0, 4):
        alone = _seq_attn(seqs[b].contiguous(), 1, T, H)
        assert torch.equal(alone, big[b])
        pad = torch.cat([seqs[b], torch.randn((70, 3 * H * D), generator=g, device="cuda").half()]).contiguous()
        padded = _seq_attn(pad, 1, T + 70, H)
        assert torch.equal(padded[:T], big[b])


def test_native_prefill_and_scoring_use_no_torch_attention_or_blas(monkeypatch):
    """in fp16 on the GPU the context prefill, the scoring forward and the max_context window
    forward run on the library's own kernels -- PyTorch's SDPA (AOTriton attn_fwd) and addmm / matmul (hipBLASLt)
    are never called -- and their logits match Hugging Face's fp32 forward within fp16 tolerance."""
    import torch.nn.functional as F

    from neuralsteganography_amd.lm.gpt2 import BatchedGPT2, random_gpt2

    m = random_gpt2("gpt2", seed=14)
    lm = BatchedGPT2(m, device="cuda", compute_dtype=torch.float16, logits_dtype=torch.float32)

    def banned(*a, **k):
        raise AssertionError("PyTorch attention / BLAS called on the native path")

    monkeypatch.setattr(F, "scaled_dot_product_attention", banned)
    monkeypatch.setattr(torch, "addmm", banned)
    monkeypatch.setattr(torch, "matmul", banned)
    ctx = list(synthetic.DEFAULT_CONTEXT)
    lg = lm.prefill(ctx, 3, 8)
    seqs = torch.tensor([ctx, ctx[::-1]], device="cuda")
    fs = lm.forward_sequences(seqs)
    wl = lm.window_logits(seqs[:, -9:].contiguous())
    monkeypatch.undo()
    with torch.no_grad():
        ref = m(torch.tensor([ctx])).logits[0].double()
        ref_rev = m(torch.tensor([ctx[::-1]])).logits[0].double()
        ref_w = m(torch.tensor([ctx[-9:]])).logits[0, -1].double()
    V = 50257
    assert (lg[:, :V].double().cpu() - ref[-1]).abs().max() < 3e-2
    assert torch.equal(lg[0], lg[2])
    assert (fs[0, :, :V].double().cpu() - ref).abs().max() < 3e-2
    assert (fs[1, :, :V].double().cpu() - ref_rev).abs().max() < 3e-2
    assert (wl[0, :V].double().cpu() - ref_w).abs().max() < 3e-2


@pytest.mark.parametrize("B,L", [(3, 40), (700, 300)])
def test_decode_attention_done_flags_skip_finished_streams(B, L):
    """ns_decode_attention_ex with done flags (round 5): streams whose flag bit 0 is set are skipped -- no KV
    append, their output rows untouched -- and every other stream's output is bit-identical to the unflagged call
    (P = 1 and P = 8 workgroup forms)."""
    H, D, T0 = 12, 64, 8
    C = H * D
    g = torch.Generator(device="cuda").manual_seed(B + L)
    cap = L + 1
    nch = (cap - T0 + 31) // 32
    kc = torch.randn((nch, B, H, 32, D), generator=g, device="cuda").half()
    vc = torch.randn((nch, B, H, 32, D), generator=g, device="cuda").half()
    kp = torch.randn((H, T0, D), generator=g, device="cuda").half()
    vp = torch.randn((H, T0, D), generator=g, device="cuda").half()
    qkv = torch.randn((B, 3 * C), generator=g, device="cuda").half()
    flags = torch.zeros((B, 8), dtype=torch.int32, device="cuda")
    flags[::3, 7] = 1  # every third stream finished
    flags[1::3, 7] = 2  # other bits do not count
    L_ = _lib.lib()

    def run(done, stop=None):
        k2, v2 = kc.clone(), vc.clone()
        out = torch.full((B, C), 5.0, device="cuda").half()
        rc = L_.ns_decode_attention_ex(qkv.data_ptr(), qkv.stride(0), k2.data_ptr(), v2.data_ptr(), k2.stride(1),
                                       k2.stride(2), k2.stride(0), kp.data_ptr(), vp.data_ptr(), kp.stride(0), T0, B, H,
                                       D, L, None, cap, 0, _lib.NS_KV_FP16,
                                       done.data_ptr() if done is not None else None, done.stride(0) if done is not None
                                       else 0, stop.data_ptr() if stop is not None else None, out.data_ptr(),
                                       out.stride(0), 1.0 / math.sqrt(D), _stream_handle())
        assert rc == 0
        torch.cuda.synchronize()
        return out, k2, v2

    ref, kr, vr = run(None)
    got, kg, vg = run(flags[:, 7])
    live = (flags[:, 7] & 1) == 0
    assert torch.equal(got[live], ref[live])
    assert (got[~live] == 5.0).all()  # skipped: untouched
    r = L - T0  # the appended row of every stream
    assert torch.equal(kg[r // 32, live, :, r % 32], kr[r // 32, live, :, r % 32])
    assert torch.equal(kg[r // 32, ~live, :, r % 32], kc[r // 32, ~live, :, r % 32])  # no append when skipped
    # stop positions: streams whose stop <= L are skipped the same way
    stop = torch.full((B,), L + 1, dtype=torch.int32, device="cuda")
    stop[::2] = L
    got2, _, _ = run(None, stop)
    run_s = torch.arange(B, device="cuda") % 2 == 1
    assert torch.equal(got2[run_s], ref[run_s]) and (got2[~run_s] == 5.0).all()


def test_encode_skip_done_streams_gives_the_same_tokens():
    """The encode loop hands the coder state's flags to the attention (finished streams skip their cache reads):
    ragged payloads give the same tokens with and without it, graph-replayed and eager."""
    from neuralsteganography_amd import synthetic
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2

    lm = HipArithmeticLM(random_gpt2("gpt2", seed=3), None, logits_dtype="f16", max_batch=6)
    ctx = synthetic.DEFAULT_CONTEXT
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, n)) for s, n in enumerate((1, 40, 7, 64, 2, 30))]
    q = {"temp": 0.9, "precision": 26, "topk": 300}
    for graphs in (True, False):
        lm.skip_done = True
        a = lm.encode_batch(bits, ctx, quality=q, graphs=graphs)
        lm.skip_done = False
        b = lm.encode_batch(bits, ctx, quality=q, graphs=graphs)
        assert a == b
        assert lm.decode_batch(a, ctx, quality=q, graphs=graphs) == [o for o in lm.decode_batch(b, ctx, quality=q,
                                                                                              graphs=graphs)]
    lm.skip_done = True
    out = lm.decode_batch(a, ctx, quality=q)
    assert all(o[: len(x)] == x for o, x in zip(out, bits))
