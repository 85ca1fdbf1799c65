"""CPU, world size 2 over gloo: stream sharding, whole-job reductions and result gathering of the
multi-GPU path (neuralsteganography_amd/dist.py), with a deterministic CPU stand-in provider (the coder
itself needs a GPU; what is tested here is the partitioning and the collectives around it)."""

import os
import socket

import pytest
import torch.multiprocessing as mp

from neuralsteganography_amd.dist import shard_range


def test_shard_range_partitions_exactly():
    for total in (0, 1, 7, 4096, 32768, 8191):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                rg = shard_range(total, world, r)
                seen.extend(rg)
            assert seen == list(range(total))
            sizes = [len(shard_range(total, world, r)) for r in range(world)]
            assert max(sizes) - min(sizes) <= 1


class _EchoProvider:
    """encode_batch returns per-stream tokens derived from the bits (identity-like, deterministic)."""

    def encode_batch(self, bit_lists, context, *, quality):
        return [[len(context)] + [sum(b[i:i + 8]) for i in range(0, len(b), 8)] for b in bit_lists]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from neuralsteganography_amd import dist as nd

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bits = [[(s >> k) & 1 for k in range(16)] for s in range(11)]
        toks = nd.encode_sharded(_EchoProvider(), bits, [1, 2, 3], quality={})
        b, ss, el, km = nd.reduce_job(100.0 * (rank + 1), 10.0, 1.0 + rank, 0.5 * (rank + 1))
        q.put((rank, toks, (b, ss, el, km), nd.per_rank(1.5 * rank + 0.25)))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_world2_gloo_sharded_encode_and_reductions():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = _EchoProvider().encode_batch([[(s >> k) & 1 for k in range(16)] for s in range(11)], [1, 2, 3],
                                          quality={})
    for rank, toks, red, times in res:
        assert toks == expect  # every rank sees all 11 streams, in stream order
        assert red == (300.0, 20.0, 2.0, 1.0)  # bits summed, stream-steps summed, times max
        assert times == [0.25, 1.75]  # per-rank values in rank order on every rank


class _CpuCoder:
    """CPU stand-in with the provider's batched protocol (``encode_batch`` / ``decode_batch``): one token per
    4-bit group plus a stream-dependent tail of filler tokens, so streams need different lockstep step counts."""

    def encode_batch(self, bit_lists, context, *, quality, graphs=None):
        out = []
        for b in bit_lists:
            toks = [int("".join(str(x) for x in b[i:i + 4]).ljust(4, "0"), 2) for i in range(0, len(b), 4)]
            out.append(toks + [16] * (sum(b) % 7))
        return out

    def decode_batch(self, token_lists, context, *, quality, graphs=None):
        return [[int(c) for t in toks if t < 16 for c in format(t, "04b")] for toks in token_lists]


def _bench_worker(rank, world, port, q, total, nbytes):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bits = bench.rank_payloads(total, world, rank, nbytes)
        res = bench.e2e_job(_CpuCoder(), bits, [1, 2, 3], {}, dev=torch.device("cpu"), world=world)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_world2_gloo_bench_e2e_job_matches_single_rank():
    """bench.py's end-to-end job (rank_payloads -> e2e_job: barrier-bracketed encode + decode, reduce_job sums
    and maxes, per_rank gathers) on world 2 over gloo equals the single-rank run over the same global stream set:
    streams, payload bits and cover tokens summed, the lockstep step count the max of the per-rank counts, every
    payload recovered."""
    import torch

    import bench

    total, nbytes = 13, 5
    single = bench.e2e_job(_CpuCoder(), bench.rank_payloads(total, 1, 0, nbytes), [1, 2, 3], {},
                           dev=torch.device("cpu"), world=1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, q, total, nbytes)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shard_steps = []
    for r in range(2):
        mine = bench.rank_payloads(total, 2, r, nbytes)
        shard_steps.append(max(len(t) for t in _CpuCoder().encode_batch(mine, [1, 2, 3], quality={})))
    for r, got in res.items():
        for key in ("streams", "payload_bits", "cover_tokens", "lockstep_steps", "roundtrip_exact_fraction",
                    "roundtrip_exact_streams", "bits_per_token"):
            assert got[key] == single[key], (r, key, got[key], single[key])
        assert got["roundtrip_exact_fraction"] == 1.0
        assert got["per_rank_lockstep_steps"] == shard_steps
        assert max(shard_steps) == single["lockstep_steps"]
        assert len(got["per_rank_seconds"]) == 2 and got["seconds"] == max(got["per_rank_seconds"])
        assert got["value"] == got["payload_bits"] / got["seconds"]
