"""CPU: the two bench.py CPU-baseline workers run and report consistent numbers (BASELINE.md "CPU baseline plan":
the coder-only oracle port and the reference's batch-1 end-to-end token loop).  Small samples; no GPU."""

import numpy as np
import pytest


def test_coder_only_worker_reports_bits_and_steps():
    from oracle.cpu_baseline import run

    r = run(0.5, 2, 7, 50257, 0.9, 26, 300, 64)
    assert r["stream_steps"] > 0 and r["stream_steps"] % 2 == 0
    assert 0 < r["bits"] <= 2 * 64 * 8
    assert r["seconds"] >= 0.5


def test_end_to_end_worker_runs_the_reference_token_loop():
    pytest.importorskip("transformers")
    from oracle.cpu_e2e import run

    r = run(1.0, 3, 50257, 0.9, 26, 300, 16)
    assert r["tokens"] > 0 and r["messages"] >= 1
    # random-init GPT-2 logits are near-uniform: every token fixes several payload bits
    assert 2.0 < r["bits"] / r["tokens"] <= 26.0
    assert np.isfinite(r["seconds"])
