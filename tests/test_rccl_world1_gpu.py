"""The multi-GPU code paths on real HIP / RCCL at world size 1 (`tests/gpu_scripts/rccl_world1.py`,
run in its own process so its "nccl" process group — created before any other GPU call — does
not leak into the other tests): with PIAMD_FORCE_COLLECTIVES=1 the flat-engine ZeRO-1
reduce-scatter / all-gather, DataParallel's bucketed all-reduce, the TP layers' all-reduces and the
static GradBuckets all run on RCCL, and every loss / gradient matches the run without a group."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_paths_world1_match_no_group():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    here = os.path.dirname(os.path.abspath(__file__))
    p = subprocess.run([sys.executable, os.path.join(here, "gpu_scripts", "rccl_world1.py")], env=env,
                       cwd=os.path.dirname(here), capture_output=True, text=True, timeout=110)
    line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")]
    assert p.returncode == 0 and line, (p.returncode, p.stdout[-3000:], p.stderr[-3000:])
    res = json.loads(line[0][len("RESULT "):])
    for key in ("flat", "dp", "tp", "static"):
        forced, plain = res[key]
        assert len(forced) == len(plain) and len(forced) >= 2, (key, res[key])
        for a, b in zip(forced, plain):
            assert abs(a - b) <= 1e-4 * max(1.0, abs(b)), (key, forced, plain)
    assert res["static_bucket_plans"] == 1, res
    assert res["flat_sharding_forced"] == 1, res  # the ZeRO-1 reduce-scatter / all-gather path ran
