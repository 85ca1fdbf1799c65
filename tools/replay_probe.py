"""Host cost of one hipGraph replay of the lockstep step vs its GPU time: B streams, the captured step replayed
64 times (host enqueue time without a sync, then wall time to completion, then HIP events on the stream).
usage: python tools/replay_probe.py [--batch 4096] [--kv fp16] [--window 0] [--reps 64] [--lanes 2 --order free]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--kv", default="fp16")
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--reps", type=int, default=64)
    ap.add_argument("--skip", type=int, default=300, help="replays before timing (cache length ~ mid-job)")
    ap.add_argument("--blocks", type=int, default=0, help="then this many more blocks of --reps replays, timed")
    ap.add_argument("--lanes", type=int, default=1, help="decode-step lanes (BatchedGPT2.decode_lanes)")
    ap.add_argument("--order", default="alternate", help="lane order: alternate | free")
    ap.add_argument("--cu-split", type=float, default=None, help="split order: CU fraction of the attention stream")
    ap.add_argument("--eager", action="store_true", help="launch every step eagerly instead of replaying the graph")
    args = ap.parse_args()
    import torch

    from neuralsteganography_amd import coder as coder_mod
    from neuralsteganography_amd import synthetic
    from neuralsteganography_amd.lm import arithmetic as A
    from neuralsteganography_amd.lm.gpt2 import random_gpt2

    B = args.batch
    lm = A.HipArithmeticLM(random_gpt2("gpt2", seed=1234), None, logits_dtype="f16", max_batch=B, kv_dtype=args.kv,
                           attention_window=args.window)
    lm.lm.decode_lanes, lm.lm.decode_lanes_order = args.lanes, args.order
    lm.lm.decode_lane_cu_split = args.cu_split
    q = {"temp": 0.9, "precision": 26, "topk": 300}
    ctx_ids = [lm.vocab - 1] + list(synthetic.DEFAULT_CONTEXT[1:])
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, 1024)) for s in range(B)]
    params = A.coder_params_from_quality(q, lm.vocab, lm.logits_dtype, lm.banned)
    ctx = lm._coder(params, B)
    budget = 2 * 8192 + 64 if not args.blocks else 2 * 8192 + 64 + args.blocks * args.reps
    lm.lm.warm_pool(B=B)
    logits = lm.lm.prefill(ctx_ids, B, budget)
    if not lm.lm.reserve(args.skip + args.reps * (2 + args.blocks) + 8):  # the paged cache: map every page ahead
        raise SystemExit("no device memory for the pages")
    sess = coder_mod.EncodeSession(ctx, bits, max_tokens=budget)
    if args.eager:  # no graph at all (a captured graph does not keep CU-masked streams)
        import types

        buf = logits.clone()
        lm.lm.begin_static(buf)

        def eager():
            lm.lm.step_static(sess.step(buf))
            lm.lm.L += 1

        g = types.SimpleNamespace(replay=eager)
    else:
        g = A._StepGraph(lm.lm, lambda lg: sess.step(lg), logits)
    for _ in range(args.skip):
        g.replay()
    torch.cuda.synchronize()
    out = {"batch": B, "lanes": args.lanes, "order": args.order, "cu_split": args.cu_split, "eager": args.eager, "kv": args.kv, "window": args.window, "reps": args.reps, "L": lm.lm.L}
    t0 = time.perf_counter()
    for _ in range(args.reps):
        g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out["host_enqueue_ms_per_replay"] = 1e3 * (t1 - t0) / args.reps
    out["wall_ms_per_step"] = 1e3 * (t2 - t0) / args.reps
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    out["event_ms_per_step"] = e0.elapsed_time(e1) / args.reps
    if args.blocks:  # sustained load: ms per step of consecutive blocks of --reps replays
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.blocks + 1)]
        ev[0].record()
        for k in range(args.blocks):
            for _ in range(args.reps):
                g.replay()
            ev[k + 1].record()
        torch.cuda.synchronize()
        out["block_ms_per_step"] = [round(ev[k].elapsed_time(ev[k + 1]) / args.reps, 4) for k in range(args.blocks)]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
