"""Elastic launcher (reference `fleet/elastic` + launch `--np min:max`): membership kept in a
TCPStore; a node joining scales the job out (every worker relaunched with the larger world), a
node leaving scales it in."""
import os
import signal
import socket
import subprocess
import sys
import time

import pytest

WORKER = """
import os, time
d = os.environ["OUT_DIR"]
tag = f"{os.environ['NODE']}-{os.environ['PADDLE_RESTART_COUNT']}-{os.environ['WORLD_SIZE']}-{os.environ['RANK']}"
open(os.path.join(d, tag), "w").close()
time.sleep(120)
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launcher(tmp, node, server, master):
    env = dict(os.environ, OUT_DIR=str(tmp), NODE=node, PYTHONPATH=os.getcwd())
    cmd = [sys.executable, "-m", "paddle_infer_amd.distributed.launch", "--nproc_per_node", "1",
           "--elastic_server", server, "--np", "1:3", "--job_id", "t", "--node_id", node,
           "--elastic_heartbeat", "0.3", "--elastic_ttl", "1.5", "--elastic_settle", "0.5",
           "--log_dir", str(tmp / f"log_{node}")]
    if master:
        cmd.append("--elastic_master")
    cmd.append(str(tmp / "worker.py"))
    return subprocess.Popen(cmd, env=env, start_new_session=True)


def _wait_for(tmp, pred, timeout=40):
    t0 = time.time()
    while time.time() - t0 < timeout:
        names = set(os.listdir(tmp))
        if pred(names):
            return names
        time.sleep(0.2)
    raise AssertionError(f"timed out; files: {sorted(os.listdir(tmp))}")


@pytest.mark.timeout(120)
def test_elastic_scale_out_and_in(tmp_path):
    (tmp_path / "worker.py").write_text(WORKER)
    server = f"127.0.0.1:{_port()}"
    a = _launcher(tmp_path, "a", server, True)
    b = None
    try:
        _wait_for(tmp_path, lambda n: any(x.startswith("a-0-1-0") for x in n))
        b = _launcher(tmp_path, "b", server, False)
        # scale out: both nodes relaunch with world 2 (a rank 0, b rank 1)
        _wait_for(tmp_path, lambda n: any(x.startswith("a-") and x.endswith("-2-0") for x in n)
                  and any(x.startswith("b-") and x.endswith("-2-1") for x in n))
        os.killpg(b.pid, signal.SIGTERM)
        b.wait(20)
        # scale in: a relaunches alone with world 1 (restart count > 1)
        _wait_for(tmp_path, lambda n: any(x.startswith("a-") and x.endswith("-1-0") and not x.startswith("a-0-")
                                          for x in n))
    finally:
        for p in (a, b):
            if p is not None and p.poll() is None:
                os.killpg(p.pid, signal.SIGTERM)
                try:
                    p.wait(20)
                except subprocess.TimeoutExpired:
                    os.killpg(p.pid, signal.SIGKILL)
