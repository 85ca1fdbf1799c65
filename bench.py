"""Benchmark of the batched arithmetic-coding stego path (BASELINE.json metric).

Headline (config C3, one MI355X per rank): GPT-2-small (random-init weights of that architecture, fp16 compute,
fp16 logits) + the HIP coder, B = 4096 independent streams per GPU, each encoding a 1 KiB random payload from
the shared 32-token context to completion (temp 0.9, precision 26, topk 300, banned {V-1, 628}).  A *step* is
one lockstep token step over all B streams: the coder step on the current logits, then the batch-invariant GPT-2
decode step that turns its tokens into the next logits (captured once as a hipGraph and replayed).  The whole
job is timed: ``value`` = payload bits encoded per second over all ranks, ``ms_per_step`` = job time / lockstep
steps.  The covers are then decoded (timed separately) and ``roundtrip_exact_fraction`` = share of streams whose
payload came back bit for bit.

``coder``: the coder hot path alone (SURVEY §8(d)'s roofline unit): ``--steps K`` launches of ``ns_encode_step``
over B resident [B, ld] synthetic 3*N(0,1) logit batches after ``--warmup W``, the K launches captured as one
hipGraph and replayed; ``roofline`` is that kernel's (HBM-bound).  ``cpu_baseline``: the oracle port on the host
cores (rank 0, N = 1).

Multi-GPU: one process per GPU, each with its own B streams (weak scaling, no collective on the data path; the
only collectives are the end-of-job reductions).  Launch: python bench.py [--gpus N --steps K --warmup W]; N>1
under torch.distributed.run.
"""

from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "payload bits/sec + cover tokens/sec, GPT-2 arithmetic stego at batch, 1-8 GPUs"


def log(msg: str) -> None:
    """Progress on stderr (the JSON line alone goes to stdout)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200, help="coder sub-benchmark: timed launches")
    ap.add_argument("--warmup", type=int, default=20, help="coder sub-benchmark: untimed launches")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--vocab", type=int, default=50257)
    ap.add_argument("--dtype", default="f32", choices=["f32", "f16"])
    ap.add_argument("--precision", type=int, default=26)
    ap.add_argument("--topk", type=int, default=300)
    ap.add_argument("--temp", type=float, default=0.9)
    ap.add_argument("--payload-bytes", type=int, default=1024)
    ap.add_argument("--pool", type=int, default=6, help="distinct logit batches cycled over the coder steps")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-e2e-seconds", type=float, default=10.0,
                    help="end-to-end CPU baseline (HF GPT-2 forward + oracle coder per core); 0 = skip")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip every end-to-end GPT-2 leg (the headline is then the coder sub-benchmark)")
    ap.add_argument("--no-decode", action="store_true", help="headline: skip the decode / round-trip check")
    ap.add_argument("--no-wide", action="store_true", help="skip the api-default (wide path) side line")
    ap.add_argument("--no-c4", action="store_true",
                    help="skip the gpt2-fa geometry leg (config C4's per-GPU share: 4096 streams, V = 42,001)")
    ap.add_argument("--no-c5", action="store_true",
                    help="skip the C5 per-GPU share: GPT-2-medium fp16, topk 100, temp 0.9, 1024 streams")
    ap.add_argument("--no-c5-guard", action="store_true",
                    help="skip the C5 quality-guard-on leg (gated cover generation, pass rate, reveal)")
    ap.add_argument("--no-f16-coder", action="store_true",
                    help="skip the fp16 coder sub-benchmark (the headline's coder kernel: roofline_f16)")
    ap.add_argument("--fp8kv", action="store_true", help="add the fp8-KV-cache end-to-end side line (opt-in mode)")
    ap.add_argument("--optin-window", type=int, default=256,
                    help="side line with the opt-in modes: fp8 KV cache + this attention window (0: skip)")
    ap.add_argument("--no-pcie", action="store_true", help="skip the host-logits (PCIe-inclusive) side figure")
    ap.add_argument("--no-attention-bench", action="store_true",
                    help="skip the decode-attention roofline (roofline_attention)")
    ap.add_argument("--no-fraction", action="store_true", help="skip the src Fraction-coder side line (row a12)")
    ap.add_argument("--fraction-batch", type=int, default=1024)
    ap.add_argument("--fraction-vocab", type=int, default=16)
    ap.add_argument("--fraction-bytes", type=int, default=32)
    ap.add_argument("--no-trained", action="store_true",
                    help="skip the trained-entropy side line (GPT-2-small head scaled so rows carry a few bits/token)")
    ap.add_argument("--trained-scale", type=float, default=6.0, help="head scale (6: ~4.2 bits/token)")
    ap.add_argument("--trained-payload-bytes", type=int, default=512)
    ap.add_argument("--trained-messages", type=int, default=16384,
                    help="trained-entropy leg: messages per GPU, queued through --trained-batch slots")
    ap.add_argument("--trained-batch", type=int, default=4096,
                    help="slots of the trained-entropy leg (covers ~2x as long as C3's on average, a few far longer: "
                         "finished slots take the next queued message)")
    ap.add_argument("--no-c2", action="store_true",
                    help="skip the batch-1 end-to-end side line (BASELINE config C2: GPT-2-small, B = 1, 1 KiB payload)")
    ap.add_argument("--e2e-batch", type=int, default=4096)
    ap.add_argument("--e2e-model", default="gpt2", choices=["gpt2", "gpt2-medium", "gpt2-fa"])
    ap.add_argument("--e2e-payload-bytes", type=int, default=1024)
    ap.add_argument("--e2e-eager", action="store_true", help="per-token launches instead of the captured hipGraph")
    ap.add_argument("--blas", default=None, choices=["rocblas", "hipblaslt"],
                    help="GEMM library for the GPT-2 forward (torch.backends.cuda.preferred_blas_library)")
    ap.add_argument("--e2e-logits", default="f16", choices=["f32", "f16"],
                    help="logits handed to the coder; the fp16 head GEMM's output either way (f32 = upcast copy)")
    ap.add_argument("--eager", action="store_true",
                    help="coder: time eager launches (one event pair each) instead of the replayed hipGraph")
    ap.add_argument("--traffic-bytes", type=float, default=None,
                    help="HBM bytes per coder launch measured by a rocprofv3 --pmc pass (corrected), if known")
    return ap.parse_args(argv)


def _cpu_workers(module, argv, seconds, max_workers=16):
    """One child process per host core (the affinity mask, capped at the box's 16-CPU share and at
    ``max_workers``), each running ``python -m <module> <argv...>`` on one thread with the GPU hidden; returns
    (cores, parsed JSON results)."""
    import subprocess

    cores = max(1, min(16, max_workers, len(os.sched_getaffinity(0))))
    env = dict(os.environ, OMP_NUM_THREADS="1", HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="",
               CUDA_VISIBLE_DEVICES="")
    procs = []
    for c in range(cores):
        cmd = [sys.executable, "-m", module] + [str(a) for a in argv(c)]
        procs.append(subprocess.Popen(cmd, cwd=str(ROOT), env=env, stdout=subprocess.PIPE, text=True))
    res = []
    for pr in procs:
        text, _ = pr.communicate(timeout=seconds * 4 + 180)
        if pr.returncode != 0:
            raise RuntimeError(f"{module} worker failed ({pr.returncode})")
        res.append(json.loads(text.strip().splitlines()[-1]))
    return cores, res


def cpu_baseline(args, seconds, streams_per_core=16):
    """The oracle port timed on the host cores on a bounded sample of the same workload (one
    process per core, the core count from the affinity mask, capped at the box's 16-CPU share).  Each worker is
    a child process (``python -m oracle.cpu_baseline``) that never touches the GPU and encodes its own streams
    of 3·N(0,1) fp32 rows for ``seconds``; bits and stream-steps are summed, the time is the slowest worker's.
    ``end_to_end`` adds BASELINE.md's second number: the reference's token loop (batch 1, Hugging Face GPT-2-small
    forward with the KV cache, random-init fp32) + the oracle coder per core (``oracle/cpu_e2e.py``)."""
    cores, res = _cpu_workers("oracle.cpu_baseline", lambda c: [seconds, streams_per_core, 1000 + c, args.vocab,
                                                                args.temp, args.precision, args.topk,
                                                                args.payload_bytes], seconds)
    dt = max(r["seconds"] for r in res)
    bits = sum(r["bits"] for r in res)
    ss = sum(r["stream_steps"] for r in res)
    out = {"value": bits / dt, "unit": "payload bits/s", "cores": cores, "kind": "port",
           "cover_tokens_per_s": ss / dt, "per_core_bits_per_s": bits / dt / cores,
           "sample": f"oracle/nsg_oracle.c or_encode_batch: {cores} worker processes (1 core each) x "
                     f"{streams_per_core} streams of 3N(0,1) fp32 rows, V {args.vocab}, topk {args.topk}, "
                     f"{args.payload_bytes}-byte payloads, {dt:.1f} s"}
    if args.cpu_e2e_seconds > 0:
        cores, res = _cpu_workers("oracle.cpu_e2e", lambda c: [args.cpu_e2e_seconds, 2000 + c, args.vocab,
                                                               args.temp, args.precision, args.topk,
                                                               args.payload_bytes], args.cpu_e2e_seconds,
                                  max_workers=8)  # torch workers: keep the box's GPU-process count bounded
        dt = max(r["seconds"] for r in res)
        bits = sum(r["bits"] for r in res)
        tok = sum(r["tokens"] for r in res)
        out["end_to_end"] = {
            "value": bits / dt, "unit": "payload bits/s", "cores": cores, "cover_tokens_per_s": tok / dt,
            "cover_tokens_per_s_per_core": tok / dt / cores, "bits_per_token": bits / max(tok, 1),
            "sample": f"{cores} worker processes (1 thread each), each the reference's batch-1 token loop: HF "
                      f"GPT2LMHeadModel (random-init GPT-2-small, fp32, KV cache) + oracle or_encode_batch, "
                      f"{args.payload_bytes}-byte payloads, {dt:.1f} s; model construction excluded"}
    if not args.no_fraction:
        out["fraction_coder"] = _fraction_cpu(args)
    return out


def _fraction_dists(V: int, n_steps: int, n_msgs: int):
    """Per-step float64 distributions of the Fraction-coder leg: 97 random rows, message b's step t = row (b + t) % 97."""
    import numpy as np

    rng = np.random.default_rng(0)
    base = rng.random((97, V))
    base /= base.sum(axis=1, keepdims=True)
    return [[base[(b + t) % 97] for t in range(n_steps)] for b in range(n_msgs)]


def _fraction_cpu(args, seconds=4.0):
    """The src Fraction coder's own arithmetic (fractions.Fraction, restated in oracle/fraction_coder.py) on one
    core, over the fraction_coder leg's messages until ``seconds`` have passed."""
    import time

    from oracle import fraction_coder as fc

    streams = _fraction_dists(args.fraction_vocab, 64, 256)
    payload = bytes(args.fraction_bytes)
    t0, tok, msgs = time.perf_counter(), 0, 0
    while time.perf_counter() - t0 < seconds and msgs < len(streams):
        toks, _ = fc.encode(payload, streams[msgs])
        tok += len(toks)
        msgs += 1
    dt = time.perf_counter() - t0
    return {"value": 8 * args.fraction_bytes * msgs / dt, "unit": "payload bits/s", "cores": 1, "kind": "port",
            "cover_tokens_per_s": tok / dt,
            "sample": f"oracle/fraction_coder.py encode (fractions.Fraction), {msgs} messages of "
                      f"{args.fraction_bytes} zero bytes over V = {args.fraction_vocab} rows, {dt:.1f} s"}


def fraction_coder(args, rank, world, dev):
    """Row a12, the src package's exact-rational coder (``codec/arithmetic.py:234-325``) as the device kernel:
    ``--fraction-batch`` messages per GPU of ``--fraction-bytes`` zero bytes (the payloads this coder carries:
    DESIGN.md §4) over per-step V-token float64 distributions, encoded in lockstep (timed, host-inclusive: the host
    gathers each step's rows from the ProbDist iterables), then decoded and compared.  A side line."""
    import torch
    import torch.distributed as dist

    from neuralsteganography_amd.codec import fraction as F
    from neuralsteganography_amd.dist import reduce_job, shard_range

    mine = shard_range(args.fraction_batch * world, world, rank)
    streams = _fraction_dists(args.fraction_vocab, 64, len(mine))
    payloads = [bytes(args.fraction_bytes)] * len(mine)
    F.encode_bits_batch(payloads[:8], [iter(s) for s in streams[:8]], [{} for _ in range(8)])  # warm-up
    states = [{} for _ in payloads]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    toks = F.encode_bits_batch(payloads, [iter(s) for s in streams], states)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    dec = F.decode_bits_batch(toks, [iter(s) for s in streams], [dict(st) for st in states])
    ok = sum(d == p for d, p in zip(dec, payloads))
    ntok = sum(len(t) for t in toks)
    bits, tok, T, _ = reduce_job(8 * args.fraction_bytes * len(payloads), ntok, dt, 0.0, dev)
    good = reduce_job(ok, 0, 0.0, 0.0, dev)[0]
    return {"value": bits / T, "unit": "payload bits/s", "cover_tokens_per_s": tok / T, "seconds": T,
            "messages": args.fraction_batch * world, "lockstep_steps": max(len(t) for t in toks),
            "roundtrip_exact_fraction": good / (args.fraction_batch * world),
            "workload": f"src Fraction coder (ns_frac_encode_step), {args.fraction_batch} messages/GPU x "
                        f"{args.fraction_bytes} zero bytes, V = {args.fraction_vocab} float64 rows per step, "
                        "host-inclusive lockstep encode"}


def _wide_traffic(B):
    """HBM bytes per wide_onepass_kernel launch from a committed PMC record of THIS library build
    (profiles/r05/pmc_traffic_wide_onepass_*.json: FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction), scaled to
    batch B, or None."""
    import glob

    from neuralsteganography_amd import _lib

    ver = _lib.version()
    for path in sorted(glob.glob(str(ROOT / "profiles" / "r0[56]" / "pmc_traffic_wide_onepass_*.json"))):
        try:
            rec = json.load(open(path))
        except (OSError, ValueError):
            continue
        if rec.get("library_version") == ver:
            return rec["traffic_bytes_per_launch"] * B / rec["batch"], "from " + str(Path(path).relative_to(ROOT))
    return None, None


def wide_path(args, rank, world, dev, steps=10, warmup=3):
    """The api default quality (precision 16, topk 50,000: api.py:81-86) at the coder batch: the wide path
    (csrc/nsg_wide.hip) on resident 3*N(0,1) fp32 logits, 1-KiB payloads, whole steps timed with HIP events on
    the launch stream.  A side line."""
    import torch
    import torch.distributed as dist

    from neuralsteganography_amd import synthetic
    from neuralsteganography_amd.coder import CoderContext, CoderParams, EncodeSession, row_stride
    from neuralsteganography_amd.dist import reduce_job, shard_range

    V, B = args.vocab, args.batch
    params = CoderParams(vocab=V, precision=16, temp=1.0, topk=50000, dtype="f32")
    ctx = CoderContext(params, max_batch=B)
    ld = row_stride(V, "f32")
    g = torch.Generator(device=dev)
    pool = []
    for i in range(3):
        g.manual_seed(1000 * rank + i)
        pool.append(3.0 * torch.randn((B, ld), generator=g, device=dev))
    mine = shard_range(B * world, world, rank)
    sess = EncodeSession(ctx, [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, args.payload_bytes))
                               for s in mine])
    for t in range(warmup):
        sess.step(pool[t % 3])
    bp0 = sess.fields()["bit_pos"].astype("int64").sum()
    nt0 = sess.fields()["ntokens"].astype("int64").sum()
    c0 = ctx.counters()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record()
    for t in range(steps):
        sess.step(pool[t % 3])
    end.record()
    torch.cuda.synchronize()
    elapsed = start.elapsed_time(end) / 1e3
    sess.raise_errors()
    f = sess.fields()
    c1 = ctx.counters()
    nbits = int(f["bit_pos"].astype("int64").sum() - bp0)
    ntok = int(f["ntokens"].astype("int64").sum() - nt0)
    bits_all, tok_all, el_max, _ = reduce_job(nbits, ntok, elapsed, 0.0, device=dev)
    alg = B * (V * 4 + 76)  # the row read once + state/token/payload window, per step
    wtr = _wide_traffic(B)
    del pool, sess, ctx
    torch.cuda.empty_cache()
    return {"value": bits_all / el_max, "unit": "payload bits/s", "cover_tokens_per_s": tok_all / el_max,
            "ms_per_step": 1e3 * el_max / steps, "steps": steps,
            "achieved_gbs": alg / (el_max / steps) / 1e9, "peak_gbs": HBM_PEAK_GBS,
            "frac": alg / (el_max / steps) / 1e9 / HBM_PEAK_GBS,
            "listed_stream_step_fraction": (c1[0] - c0[0]) / max(ntok, 1),
            "traffic": wtr[0], "traffic_source": wtr[1],
            "workload": f"api default quality: {B} streams/GPU x ns_encode_step, precision 16, topk 50000, temp 1.0, "
                        f"resident [{B},{ld}] f32 3N(0,1) logits, {args.payload_bytes}-byte payloads"}


def attention_bench(args, rank, world, dev, L=None, steps=20, warmup=3, T0=32):
    """The decode attention of the headline's step alone (``ns_decode_attention_paged``, ``paged_attn_kernel``:
    ~80 % of the C3 step): one GPT-2-small layer at the e2e batch, the shared 32-position context stored once and
    each stream's own rows in 32-position pages of a layer-major pool segment, mapped chunk by chunk over the streams
    as the slot scheduler maps them, every stream at cache length ``L`` (default: the C3 job's mean attended
    length), random fp16 K/V/q.  K launches timed with HIP events on the launch stream.  Algorithmic bytes per launch
    (DESIGN §4b): B·H·(L+1−T0)·2·D·2 (each stream's K and V rows, the new one included) + H·T0·2·D·2 (the shared
    prefix) + B·3C·2 (qkv) + B·C·2 (out).  Returns the ``roofline_attention`` object."""
    import math

    import numpy as np
    import torch

    from neuralsteganography_amd import _lib
    from neuralsteganography_amd.coder import _stream_handle

    B, H, D = args.e2e_batch, 12, 64
    C = H * D
    L = int(L or 544)
    rows = L + 1 - T0
    nch = (rows + 31) // 32
    blk = 2 * H * 32 * D  # one layer's [K|V][H][32][D] block of a page
    npages = B * nch
    g = torch.Generator(device=dev)
    g.manual_seed(77 + rank)
    pool = torch.randn((npages, blk), generator=g, device=dev, dtype=torch.float16)  # one layer plane of a segment
    kp = torch.randn((H, T0, D), generator=g, device=dev, dtype=torch.float16)
    vp = torch.randn((H, T0, D), generator=g, device=dev, dtype=torch.float16)
    qkv = torch.randn((B, 3 * C), generator=g, device=dev, dtype=torch.float16)
    out = torch.empty((B, C), device=dev, dtype=torch.float16)
    order = np.arange(npages, dtype=np.int64).reshape(nch, B).T  # page of (stream b, chunk c) = c * B + b
    table = torch.from_numpy(np.ascontiguousarray(pool.data_ptr() + 2 * blk * order)).to(dev)
    lens = torch.full((B,), L, dtype=torch.int32, device=dev)
    lib = _lib.lib()
    st = _stream_handle()
    stream = torch.cuda.current_stream()

    def launch():
        rc = lib.ns_decode_attention_paged(qkv.data_ptr(), qkv.stride(0), table.data_ptr(), table.stride(0), nch, 0,
                                           kp.data_ptr(), vp.data_ptr(), kp.stride(0), T0, B, H, D, lens.data_ptr(), 0,
                                           _lib.NS_KV_FP16, None, 0, None, out.data_ptr(), out.stride(0),
                                           1.0 / math.sqrt(D), st)
        if rc != 0:
            raise RuntimeError(f"ns_decode_attention_paged failed ({rc})")

    for _ in range(warmup):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        launch()
    e1.record(stream)
    torch.cuda.synchronize()
    kern_ms = e0.elapsed_time(e1) / steps
    if not torch.isfinite(out.float()).all():
        raise RuntimeError("attention bench: non-finite output")
    alg = B * H * rows * 2 * D * 2 + H * T0 * 2 * D * 2 + B * 3 * C * 2 + B * C * 2
    achieved = alg / (kern_ms / 1e3) / 1e9
    del pool, kp, vp, qkv, out, table
    torch.cuda.empty_cache()
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
            "traffic": None, "kernel": "paged_attn_kernel<FmtF16,8> (ns_decode_attention_paged)",
            "kernel_ms_avg": kern_ms, "launches": steps, "alg_bytes_per_launch": alg,
            "workload": f"one GPT-2-small layer, {B} streams x {H} heads, cache length L = {L} (T0 = {T0} shared "
                        f"context positions + {rows} own rows incl. the new one, 32-position pages of a layer-major "
                        "segment), fp16",
            "alg_bytes_formula": "B*H*(L+1-T0)*2*D*2 + H*T0*2*D*2 + B*3C*2 + B*C*2",
            "timing": "K eager launches between two HIP events on the launch stream"}


def rank_payloads(total, world, rank, nbytes):
    """This rank's payload bit lists: streams ``shard_range(total, world, rank)`` (contiguous slices), stream s
    carrying ``synthetic.payload_bytes(s, nbytes)`` as LSB-first bits, so the union over ranks is
    the same stream set whatever the world size."""
    from neuralsteganography_amd import synthetic
    from neuralsteganography_amd.dist import shard_range

    return [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, nbytes)) for s in shard_range(total, world, rank)]


def e2e_job(lm, bit_lists, context, quality, *, dev, world, decode=True, graphs=None, slots=None):
    """One timed whole job on this rank: ``lm.encode_batch`` of the rank's streams to completion, bracketed by a
    barrier and a device synchronisation on both sides; then (``decode``) ``lm.decode_batch`` of the covers,
    timed the same way, and the share of streams whose payload came back bit for bit.  Totals are summed over
    ranks and times maxed (``dist.reduce_job``); ``per_rank_*`` expose load imbalance.  Works on
    any provider with ``encode_batch`` / ``decode_batch`` (the gloo test drives it with a CPU stand-in)."""
    import torch
    import torch.distributed as dist

    from neuralsteganography_amd.dist import per_rank, reduce_job

    def sync():
        if getattr(dev, "type", "cpu") == "cuda":
            torch.cuda.synchronize(dev)

    def timed(fn):
        if world > 1:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        res = fn()
        sync()
        dt = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
        return res, dt

    kw = {"slots": slots} if slots else {}
    toks, elapsed = timed(lambda: lm.encode_batch(bit_lists, context, quality=quality, graphs=graphs, **kw))
    nbits = sum(len(b) for b in bit_lists)
    ntok = sum(len(t) for t in toks)
    steps = max((len(t) for t in toks), default=0)
    bits_all, tok_all, el_max, steps_max = reduce_job(nbits, ntok, elapsed, float(steps), device=dev)
    out = {"value": bits_all / el_max, "unit": "payload bits/s", "cover_tokens_per_s": tok_all / el_max,
           "cover_tokens_per_s_per_gpu": tok_all / el_max / world, "seconds": el_max, "payload_bits": bits_all,
           "cover_tokens": tok_all, "streams": int(round(reduce_job(len(bit_lists), 0, 0, 0, device=dev)[0])),
           "per_rank_seconds": per_rank(elapsed, device=dev),
           "per_rank_lockstep_steps": [int(v) for v in per_rank(steps, device=dev)],
           "lockstep_steps": int(steps_max), "ms_per_step": 1e3 * el_max / max(steps_max, 1),
           "bits_per_token": bits_all / max(tok_all, 1)}
    if decode:
        dec, dt = timed(lambda: lm.decode_batch(toks, context, quality=quality, graphs=graphs, **kw))
        exact = sum(1 for d, b in zip(dec, bit_lists) if list(d[: len(b)]) == list(b))
        ex_all, n_all, dt_max, _ = reduce_job(exact, len(bit_lists), dt, 0.0, device=dev)
        out["roundtrip_exact_fraction"] = ex_all / max(n_all, 1)
        out["roundtrip_exact_streams"] = int(ex_all)
        out["decode"] = {"seconds": dt_max, "value": bits_all / dt_max, "unit": "payload bits/s",
                         "cover_tokens_per_s": tok_all / dt_max, "ms_per_step": 1e3 * dt_max / max(steps_max, 1),
                         "per_rank_seconds": per_rank(dt, device=dev)}
    return out


def end_to_end(args, rank, world, dev, kv_dtype="fp16", window=0, batch=None, model=None, topk=None,
               decode=False, logit_scale=1.0, payload_bytes=None, messages=None, slots=None):
    """The whole stego encode at batch: GPT-2 forward (random-init weights of the named architecture, fp16
    compute, HIP decode step) + HIP coder step per token, every stream encoding its full payload from the shared
    32-token context until the last stream is done (lockstep, like the reference's per-message loop run for all
    messages at once); ``decode`` adds the decode and the round-trip check (:func:`e2e_job`)."""
    import torch

    from neuralsteganography_amd import synthetic
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2

    B = batch or args.e2e_batch
    model = model or args.e2e_model
    topk = topk or args.topk
    nbytes = payload_bytes or args.e2e_payload_bytes
    if args.blas:
        torch.backends.cuda.preferred_blas_library({"rocblas": "cublas", "hipblaslt": "cublaslt"}[args.blas])
    lm = HipArithmeticLM(random_gpt2(model), None, device=str(dev), logits_dtype=args.e2e_logits,
                         max_batch=B, kv_dtype=kv_dtype, attention_window=window, logit_scale=logit_scale)
    quality = {"temp": args.temp, "precision": args.precision, "topk": topk}
    # [<|endoftext|>] + 31 ids; the end-of-text id is the vocabulary's last (gpt2-fa: 42,000)
    context = [lm.vocab - 1] + list(synthetic.DEFAULT_CONTEXT[1:])
    graphs = False if args.e2e_eager else None
    # warm-up: kernels and the coder context at the same batch, short payloads; then the KV page pool is grown to
    # what the device allows and written once (a fresh process's first pass over ~250 GB of new allocations
    # measured up to 12 % slower per step than later ones): the timed job maps warm pages, allocates none
    S = min(B, slots or B)
    lm.encode_batch([[1, 0, 1, 1] * 8] * S, context, quality=quality, graphs=graphs)
    msgs = messages or B
    bits = rank_payloads(msgs * world, world, rank, nbytes)
    pool_pages = lm.lm.warm_pool(B=S)
    torch.cuda.synchronize()
    out = e2e_job(lm, bits, context, quality, dev=dev, world=world, decode=decode, graphs=graphs, slots=S)
    out.update({"kv_pages_pool": pool_pages, "kv_page_bytes": lm.lm.pool.page_bytes, "schedule": lm.last_schedule,
                "kv_dtype": kv_dtype, "attention_window": window or None,
                "workload": f"{model} (random-init weights, fp16 compute, {args.e2e_logits} logits, {kv_dtype} KV "
                            f"cache, batch-invariant native decode step) + ns_encode_step (temp {args.temp}, "
                            f"precision {args.precision}, topk {topk}), {msgs} messages/GPU x {nbytes}-"
                            f"byte payloads through {S} slots (paged KV cache, slot refill), encoded to completion "
                            f"from a 32-token context, "
                            + (f"head scaled x{logit_scale} (trained-entropy rows), " if logit_scale != 1.0 else "")
                            + (f"attention window {window} (opt-in)" if window else "unbounded KV cache")})
    lm.lm.release_cache()
    del lm
    gc.collect()
    torch.cuda.empty_cache()
    return out


def c5_guard(args, rank, world, dev, n=1024, max_bytes=256):
    """C5's quality guard ON (``cover_generate_batch``, api.py:565-662): GPT-2-medium (random-init, fp16), topk 100,
    temp 0.9, finish_sent, the reference's regeneration schedule (2 more attempts: next seed, top_k 80 / 70,
    temp 0.8 / 0.7), n secrets of 0 .. max_bytes - 1 bytes per GPU (one packet each; the default guard's unigram
    metrics reject long covers outright -- a text of a few hundred distinct ids has a unigram entropy above the
    5.5 limit -- so the secrets span short to long covers).  Random-init weights give no meaningful perplexity,
    so the gate's max_ppl is the median of an ungated first pass over the same secrets (the schedule runs for the
    rejected ones).  Timed: the gated generation (every attempt's
    encode + guard scoring); then every passed cover is revealed from its text.  Reports the pass rate per
    attempt and the reveal's exact fraction."""
    import torch

    from neuralsteganography_amd import synthetic
    from neuralsteganography_amd.cover import (_ensure_guard, cover_generate_batch, cover_reveal_batch,
                                               iter_attempts, prepare_gate_thresholds)
    from neuralsteganography_amd.dist import reduce_job
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2
    from neuralsteganography_amd.stego import normalise_quality

    lm = HipArithmeticLM(random_gpt2("gpt2-medium", seed=77), synthetic.IdTokenizer(50257), device=str(dev),
                         logits_dtype="f16", max_batch=2 * n)
    q = {"temp": 0.9, "precision": args.precision, "topk": 100, "finish_sent": True}
    secrets = [synthetic.payload_bytes(n * rank + s, s % max_bytes) for s in range(n)]
    seed = "w11. w12. w13"
    strategy = {"seed_pool": ["w21. w22. w23", "w31. w32. w33"]}
    first = cover_generate_batch(secrets, seed_text=seed, quality=q, ecc="rs", lm=lm, quality_gate=False)
    guard = _ensure_guard(None)
    ppl = sorted(v.metrics["ppl"] for v in guard.evaluate_batch(first, prepare_gate_thresholds(None)))
    gate = {"max_ppl": float(ppl[n // 2])}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = cover_generate_batch(secrets, seed_text=seed, quality=q, ecc="rs", lm=lm, quality_gate=True,
                               gate_thresholds=gate, regen_attempts=2, regen_strategy=strategy, return_errors=True)
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    passed = [i for i, t in enumerate(out) if isinstance(t, str)]
    attempts = list(iter_attempts(seed, 2, strategy))
    by_attempt = {}
    for i in passed:
        a = next(j for j, att in enumerate(attempts) if out[i].startswith(att.seed_text))
        by_attempt.setdefault(a, []).append(i)
    exact = 0
    t1 = time.perf_counter()
    for a, idx in sorted(by_attempt.items()):
        aq = dict(normalise_quality(q), **attempts[a].overrides)
        got = cover_reveal_batch([out[i] for i in idx], seed_text=attempts[a].seed_text, quality=aq, ecc="rs", lm=lm)
        exact += sum(1 for i, g in zip(idx, got) if g == secrets[i])
    torch.cuda.synchronize()
    rev_s = time.perf_counter() - t1
    npass_all, n_all, gen_max, _ = reduce_job(len(passed), n, gen_s, 0.0, device=dev)
    ex_all, _, rev_max, _ = reduce_job(exact, 0, rev_s, 0.0, device=dev)
    lm.lm.release_cache()
    del lm
    gc.collect()
    torch.cuda.empty_cache()
    return {"secrets": int(n_all), "secret_bytes": f"0..{max_bytes - 1}", "gate": gate, "seconds": gen_max,
            "covers_per_s": npass_all / gen_max, "secrets_per_s": n_all / gen_max,
            "pass_rate": npass_all / max(n_all, 1),
            "passed_per_attempt": {str(a + 1): len(v) for a, v in sorted(by_attempt.items())},
            "reveal_exact_fraction": ex_all / max(npass_all, 1), "reveal_seconds": rev_max,
            "workload": f"gpt2-medium (random-init, fp16) cover_generate_batch, quality guard ON (api default guard, "
                        f"regeneration schedule api.py:496-523), topk 100, temp 0.9, finish_sent, {n} secrets/GPU of "
                        f"0-{max_bytes - 1} B; gate max_ppl = median of an ungated pass (random weights)"}


def host_logits_rate(args, sess, logits, stream, steps=5):
    """PCIe-inclusive side figure (never `value`): the same coder step when the caller hands over the logit
    batch in pinned host memory, i.e. one H2D copy of [B, ld] per step before ns_encode_step (this GPU only)."""
    import torch

    host = logits.cpu().pin_memory()
    dev_buf = torch.empty_like(logits)
    f0 = sess.fields()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    start.record(stream)
    for _ in range(steps):
        dev_buf.copy_(host, non_blocking=True)
        sess.step(dev_buf)
    end.record(stream)
    torch.cuda.synchronize()
    sec = start.elapsed_time(end) / 1e3 / steps
    bits = int(sess.fields()["bit_pos"].sum() - f0["bit_pos"].sum())
    nbytes = host.numel() * host.element_size()
    del host, dev_buf
    return {"ms_per_step": sec * 1e3, "value": bits / steps / sec, "unit": "payload bits/s",
            "h2d_bytes_per_step": nbytes, "h2d_gbs": nbytes / sec / 1e9,
            "note": "logits copied from pinned host memory each step, this GPU only; not the headline"}


def measured_traffic(args, version):
    """Per-launch HBM bytes from a committed rocprofv3 PMC record (tools/pmc_traffic.py) of THIS library
    build and workload, else None."""
    import glob

    best = None
    for path in sorted(glob.glob(str(ROOT / "profiles" / "pmc_traffic_*.json")) +
                       glob.glob(str(ROOT / "profiles" / "r0[56]" / "pmc_traffic_*.json"))):
        try:
            rec = json.load(open(path))
        except (OSError, ValueError):
            continue
        if (rec.get("library_version") == version and rec.get("batch") == args.batch and rec.get("vocab") == args.vocab
                and rec.get("dtype") == args.dtype and rec.get("topk") == args.topk
                and rec.get("kernel", "coder_step_kernel") == "coder_step_kernel"):
            best = (rec["traffic_bytes_per_launch"], "from " + str(Path(path).relative_to(ROOT)) +
                    " (committed rocprofv3 PMC record of this library build; not measured in this run)")
    return best


def _attn_traffic(args, L):
    """Per-launch HBM bytes of the attention microbenchmark from a committed PMC record of this library build
    (tools/pmc_traffic.py --kernel decode_attn_kernel), scaled from its cache length to ``L`` by the per-row bytes."""
    import glob

    from neuralsteganography_amd import _lib

    ver = _lib.version()
    for path in sorted(glob.glob(str(ROOT / "profiles" / "r0[56]" / "pmc_traffic_attn*.json"))):
        try:
            rec = json.load(open(path))
        except (OSError, ValueError):
            continue
        if rec.get("library_version") == ver and rec.get("batch") == args.e2e_batch and rec.get("L"):
            per_row = rec["traffic_bytes_per_launch"] / rec["alg_bytes_per_launch"]
            B, H, D, T0 = args.e2e_batch, 12, 64, 32
            alg = B * H * (L + 1 - T0) * 2 * D * 2 + H * T0 * 2 * D * 2 + B * 3 * H * D * 2 + B * H * D * 2
            return per_row * alg, (f"from {Path(path).relative_to(ROOT)} (committed rocprofv3 PMC record of this "
                                   f"library build, traffic/alg ratio {per_row:.3f} at L = {rec['L']}; not measured in "
                                   "this run)")
    return None, None


def _coder_kernel_name(dtype, topk, B):
    """The coder_step_kernel instantiation ns_encode_step launches (launch_one in csrc/nsg_coder.hip): NSK rank
    slots per lane from K, one wave per stream above the split form's batch limit."""
    nsk = 2 if topk <= 128 else 5 if topk <= 320 else (8 if dtype == "f32" and topk <= 512 else 12 if dtype == "f32"
                                                         else 8)
    nsplit = 16 if dtype == "f32" else 8
    form = 1 if B > 6144 // nsplit else nsplit
    return f"coder_step_kernel<{'_Float16' if dtype == 'f16' else 'float'},false,{nsk},false,{form}>"


def coder_bench(args, rank, world, dev, dtype=None, topk=None, pcie=True):
    """The coder hot path alone: K launches of ns_encode_step over B resident synthetic logit rows (a pool of
    distinct batches, far larger than the 256 MiB Infinity Cache, cycled step by step; every stream's payload
    cursor advances for real).  Returns the sub-object, its ``roofline`` included.  ``dtype`` / ``topk``
    override the command line (the fp16 run is the coder the headline's end-to-end step launches)."""
    import copy

    args = copy.copy(args)
    args.dtype = dtype or args.dtype
    args.topk = topk or args.topk
    import torch
    import torch.distributed as dist

    from neuralsteganography_amd import _lib, synthetic
    from neuralsteganography_amd.coder import CoderContext, CoderParams, EncodeSession, row_stride
    from neuralsteganography_amd.dist import per_rank, reduce_job, shard_range

    B, V = args.batch, args.vocab
    params = CoderParams(vocab=V, precision=args.precision, temp=args.temp, topk=args.topk, dtype=args.dtype)
    ctx = CoderContext(params, max_batch=B, device=dev.index)
    ld = row_stride(V, args.dtype)
    tdt = params.torch_dtype
    gen = torch.Generator(device=dev)
    pool = []
    for i in range(args.pool):
        gen.manual_seed(1000 * rank + i)
        x = torch.randn((B, ld), generator=gen, device=dev, dtype=torch.float32).mul_(3.0)
        pool.append(x.to(tdt))
        del x
    mine = shard_range(B * world, world, rank)  # weak scaling: B streams per rank, disjoint payload seeds
    payload_bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, args.payload_bytes)) for s in mine]
    sess = EncodeSession(ctx, payload_bits)
    stream = torch.cuda.current_stream()

    for t in range(args.warmup):
        sess.step(pool[t % args.pool])
    torch.cuda.synchronize()
    # side figure: eager launches with one HIP event pair per launch (the per-launch kernel time rocprofv3 sees)
    n_eager = 0 if args.eager else min(args.steps, 50)
    eager = None
    if n_eager:
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_eager)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(n_eager):
            ev[t][0].record(stream)
            sess.step(pool[(args.warmup + t) % args.pool])
            ev[t][1].record(stream)
        torch.cuda.synchronize()
        eager = {"ms_per_step": 1e3 * (time.perf_counter() - t0) / n_eager,
                 "kernel_ms_avg": float(np.mean([a.elapsed_time(b) for a, b in ev])), "steps": n_eager}
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    graph = None
    if not args.eager:
        # the K timed steps captured once as a hipGraph and replayed (as the product's token loop replays its
        # captured step), so the step time is the launches' own, without host launch gaps
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for t in range(args.steps):
                sess.step(pool[(args.warmup + n_eager + t) % args.pool])
    torch.cuda.synchronize()
    f0 = sess.fields()
    c0 = ctx.counters()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if graph is not None:
        g0.record(stream)
        graph.replay()
        g1.record(stream)
    else:
        for t in range(args.steps):
            ev[t][0].record(stream)
            sess.step(pool[(args.warmup + t) % args.pool])
            ev[t][1].record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()

    f1 = sess.fields()
    c1 = ctx.counters()
    if graph is not None:  # per-launch average over the replay (launch gaps of a graph included)
        kern_ms = g0.elapsed_time(g1) / args.steps
        del graph
    else:
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    stream_steps = int(f1["ntokens"].sum() - f0["ntokens"].sum())
    bits = int(f1["bit_pos"].sum() - f0["bit_pos"].sum())
    sess.raise_errors()
    pcie = None if (args.no_pcie or not pcie) else host_logits_rate(args, sess, pool[0], stream)

    bits_all, ss_all, elapsed_max, kern_ms_max = reduce_job(bits, stream_steps, elapsed, kern_ms, device=dev)
    rank_s = per_rank(elapsed, device=dev)
    traffic = measured_traffic(args, _lib.version())
    if args.traffic_bytes is not None:
        traffic = (args.traffic_bytes, "command line")
    esz = 2 if args.dtype == "f16" else 4
    per_stream_step = V * esz + 76  # logit row + state r/w (64) + token (4) + history (4) + payload window (~4)
    alg_bytes = B * per_stream_step
    achieved = alg_bytes / (kern_ms / 1e3) / 1e9
    out = {
        "value": bits_all / elapsed_max, "unit": "payload bits/s", "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed_max / args.steps, "per_rank_seconds": rank_s,
        "cover_tokens_per_s": ss_all / elapsed_max, "bits_per_token": bits_all / max(ss_all, 1.0),
        "kernel_ms_avg": kern_ms,
        "timing": ("K launches captured in one hipGraph, replayed once; kernel_ms_avg = replay time / K (HIP "
                   "events on the launch stream)") if not args.eager else "eager launches, one event pair each",
        "eager_launches": eager,  # the first min(K, 50) steps after the warm-up, launched one by one
        "exact_sum_fraction": (c1[0] - c0[0]) / max(stream_steps, 1),
        "overflow_compactions_per_stream_step": (c1[1] - c0[1]) / max(stream_steps, 1),
        "speculation_miss_fraction": (c1[2] - c0[2]) / max(stream_steps, 1),
        "workload": f"C3 coder hot path: {B} streams/GPU x 1 step of ns_encode_step on resident [{B},{ld}] "
                    f"{args.dtype} 3N(0,1) logits (GPT-2-small vocab {V}), temp {args.temp}, precision "
                    f"{args.precision}, topk {args.topk}, {args.payload_bytes}-byte payloads",
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic[0] if traffic else None,
                     "traffic_source": traffic[1] if traffic else None,
                     "kernel": _coder_kernel_name(args.dtype, args.topk, B),
                     "alg_bytes_per_launch": alg_bytes,
                     "alg_bytes_per_stream_step": per_stream_step, "stream_steps_per_launch": B},
    }
    if pcie is not None:
        out["host_logits_pcie"] = pcie
    del pool, sess, ctx
    torch.cuda.empty_cache()
    return out


def _side_leg(fn):
    """A side line's result, or {"error": ...} if it fails: on one GPU a side line never takes the headline down with
    it (device memory is released before the next leg).  With several ranks a failure propagates: a rank that
    skipped a leg's collectives would leave the others waiting in them."""
    import torch

    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return fn()
    try:
        return fn()
    except Exception as exc:  # noqa: BLE001 - reported in the JSON line, the run goes on
        log(f"side line failed: {type(exc).__name__}: {exc}")
        torch.cuda.empty_cache()
        return {"error": f"{type(exc).__name__}: {str(exc)[:300]}"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    log("coder sub-benchmark")
    coder = coder_bench(args, rank, world, dev)
    roofline_f32 = coder.pop("roofline")
    side = {}
    roofline_f16 = None
    if not args.no_f16_coder:  # the coder the headline's end-to-end step runs: fp16 rows from the head GEMM
        log("fp16 coder sub-benchmark")
        side["coder_f16"] = coder_bench(args, rank, world, dev, dtype="f16", topk=args.topk, pcie=False)
        roofline_f16 = side["coder_f16"].pop("roofline")
    if not args.no_wide:
        log("wide path")
        side["wide_path"] = _side_leg(lambda: wide_path(args, rank, world, dev))
    if not args.no_fraction:
        log("src Fraction coder")
        side["fraction_coder"] = _side_leg(lambda: fraction_coder(args, rank, world, dev))
    head = None
    if not args.no_e2e:
        # headline: config C3 end to end, encoded then decoded and checked
        log("C3 end to end (encode + decode)")
        head = end_to_end(args, rank, world, dev, decode=not args.no_decode)
        if not args.no_c2:  # C2: one message per GPU -- per-token latency of the whole step (small-batch coder form)
            log("C2 end to end")
            side["end_to_end_c2"] = _side_leg(lambda: end_to_end(args, rank, world, dev, batch=1, decode=True))
        if not args.no_c4:  # C4's per-GPU share: gpt2-fa geometry (V = 42,001), 4096 streams
            log("C4 share end to end")
            side["end_to_end_c4"] = _side_leg(lambda: end_to_end(args, rank, world, dev, model="gpt2-fa", decode=True))
        if not args.no_c5:  # C5's per-GPU share: GPT-2-medium fp16, topk 100, temp 0.9, 1024 streams
            log("C5 share end to end")
            side["end_to_end_c5"] = _side_leg(lambda: end_to_end(args, rank, world, dev, model="gpt2-medium",
                                                                 batch=1024, topk=100, decode=True))
        if not args.no_c5_guard:  # C5 with the quality guard ON: gated covers, pass rate, reveal from text
            log("C5 guard on")
            side["c5_guard"] = _side_leg(lambda: c5_guard(args, rank, world, dev))
        if args.fp8kv:  # opt-in numerics mode, reported beside (never as) the fp16 reference configuration
            log("fp8 KV end to end")
            side["end_to_end_fp8kv"] = _side_leg(lambda: end_to_end(args, rank, world, dev, kv_dtype="fp8"))
        if args.optin_window:  # opt-in: fp8 KV + sliding attention window (bounded per-step KV traffic)
            log("opt-in end to end")
            side["end_to_end_optin"] = _side_leg(lambda: end_to_end(args, rank, world, dev, kv_dtype="fp8",
                                                                    window=args.optin_window))

    if not args.no_e2e and not args.no_trained:
        # peaked (trained-LM-like) rows: longer, uneven covers and the 1/R cutoff path at scale; last, because a
        # stream stuck in a low-entropy loop grows its cover (and the KV cache) far beyond the mean
        log("trained-entropy end to end")
        side["end_to_end_trained"] = _side_leg(lambda: end_to_end(
            args, rank, world, dev, decode=True, logit_scale=args.trained_scale, batch=args.trained_batch,
            payload_bytes=args.trained_payload_bytes, messages=args.trained_messages, slots=args.trained_batch))
    roofline_attn = None
    if not args.no_e2e and not args.no_attention_bench:
        # the decode attention at the C3 job's mean attended length: T0 + (lockstep steps + 1) / 2 keys
        L_mean = 32 + (head["lockstep_steps"] + 1) // 2 if head is not None else 544
        log(f"decode attention at L = {L_mean}")
        roofline_attn = attention_bench(args, rank, world, dev, L=L_mean)
        roofline_attn["traffic"], roofline_attn["traffic_source"] = _attn_traffic(args, L_mean)
    # the headline's roofline is the coder kernel its timed region runs (fp16 rows, topk 300); the fp32 coder's
    # figure is a side key
    if args.no_e2e or roofline_f16 is None or args.e2e_logits != "f16":
        roofline, roofline_side = roofline_f32, roofline_f16
    else:
        roofline, roofline_side = roofline_f16, roofline_f32
    cfg = {"global_batch": args.batch * world, "vocab": args.vocab, "precision": args.precision, "topk": args.topk,
           "temp": args.temp, "parallelism": f"dp{world} (independent streams, no collective)"}
    if head is not None:
        out = {"metric": METRIC, "value": head["value"], "unit": "payload bits/s", "n_gpus": world,
               "steps": head["lockstep_steps"], "warmup": args.warmup, "ms_per_step": head["ms_per_step"],
               "per_rank_seconds": head["per_rank_seconds"], "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "f64", "data": "synthetic",
               "config": dict(cfg, workload="C3 end to end: " + head["workload"], global_batch=args.e2e_batch * world,
                              model=f"{args.e2e_model} (random-init)", lm_dtype="fp16",
                              logits_dtype=args.e2e_logits, payload_bytes=args.e2e_payload_bytes),
               "steps_note": ("steps = lockstep token steps of the timed job (every stream's payload encoded to "
                              "completion); --steps/--warmup set the coder sub-benchmark"),
               "cover_tokens_per_s": head["cover_tokens_per_s"],
               "cover_tokens_per_s_per_gpu": head["cover_tokens_per_s_per_gpu"],
               "bits_per_token": head["bits_per_token"],
               "roundtrip_exact_fraction": head.get("roundtrip_exact_fraction"),
               "roofline": roofline, "end_to_end": head, "coder": coder}
    else:
        out = {"metric": METRIC, "value": coder["value"], "unit": "payload bits/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": coder["ms_per_step"],
               "per_rank_seconds": coder["per_rank_seconds"], "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "f64", "data": "synthetic",
               "config": dict(cfg, workload=coder["workload"], logits_dtype=args.dtype,
                              payload_bytes=args.payload_bytes),
               "cover_tokens_per_s": coder["cover_tokens_per_s"], "roofline": roofline, "coder": coder}
    out.update(side)
    if roofline_side is not None:
        out["roofline_coder_f32" if roofline is roofline_f16 else "roofline_f16"] = roofline_side
    if roofline_attn is not None:
        out["roofline_attention"] = roofline_attn
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("CPU baselines")
        out["cpu_baseline"] = cpu_baseline(args, args.cpu_baseline_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
