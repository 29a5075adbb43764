"""The driver's multi-rank bench command, rehearsed on the CPU (gloo + the ops' CPU reference
paths): ``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`` must print
exactly one JSON line from rank 0 with the contract's fields — through the Fleet API for sharded DP,
TP × DP, PP × DP (1F1B), interleaved PP, a sharding axis × DP, and ZeRO-3."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n,extra,par,gb", [
    (2, [], "dp2_zero1", 4),
    (4, ["--tp", "2"], "tp2dp2_zero1", 4),
    (4, ["--pp", "2"], "pp2dp2_zero1", 4),
    (2, ["--pp", "2", "--vpp", "2", "--accumulate", "2", "--num-layers", "4"], "pp2v2dp1", 2),
    (4, ["--sharding-degree", "2"], "sh2dp2_zero1", 8),
    (2, ["--sharding", "3"], "dp2_zero3", 4),
    (4, ["--pp", "2", "--sharding-degree", "2", "--sharding", "3"], "pp2sh2dp1_zero3", 4),
])
def test_bench_multirank_contract(n, extra, par, gb):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--steps", "2", "--warmup", "1", "--device", "cpu", "--model", "gpt3-tiny",
           "--seq", "64", "--micro-batch", "2"] + extra
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert KEYS <= set(out)
    assert out["n_gpus"] == n and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["parallelism"] == par
    assert out["config"]["global_batch"] == gb
    assert out["value"] > 0 and out["final_loss"] == out["final_loss"]


def test_bench_gpt13b_pp2_sharding3_rehearsal():
    """BASELINE config 5's shape (GPT-3 13B, sharding stage 3 x pp 2) through the driver command,
    4 of its 40 layers at seq 64 so it fits a CPU rehearsal: real 13B widths (hidden 5120, 40
    heads, vocab 50304)."""
    n = 4
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--steps", "1", "--warmup", "0", "--device", "cpu", "--model", "gpt3-13b",
           "--num-layers", "4", "--pp", "2", "--sharding-degree", "2", "--sharding", "3",
           "--seq", "64", "--micro-batch", "2"]
    env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=ROOT)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["config"]["parallelism"] == "pp2sh2dp1_zero3"
    assert out["config"]["params"] > 1.7e9 and out["final_loss"] == out["final_loss"]
