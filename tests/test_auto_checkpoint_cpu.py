"""Auto checkpoint (reference `fluid/incubate/checkpoint/auto_checkpoint.py` train_epoch_range):
a job killed mid-range resumes after its last checkpointed epoch with the saved parameters and
optimizer state, and ends bitwise where an uninterrupted job ends — for a static program (registered
by Executor.run) and for dygraph objects (register())."""
import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import static
from paddle_infer_amd.incubate.checkpoint import auto_checkpoint as acp


@pytest.fixture
def acp_env(tmp_path, monkeypatch):
    monkeypatch.setenv("PADDLE_RUNNING_ENV", "PADDLE_EDL_AUTO_CHECKPOINT")
    monkeypatch.setenv("PADDLE_JOB_ID", "job_1")
    monkeypatch.setenv("PADDLE_EDL_HDFS_CHECKPOINT_PATH", str(tmp_path / "ckpt"))
    monkeypatch.setenv("PADDLE_TRAINER_ID", "0")
    return tmp_path


class Crash(Exception):
    pass


def _data(e):
    r = np.random.RandomState(e)
    return r.randn(6, 4).astype("float32"), r.randn(6, 1).astype("float32")


def _static_job(crash_at=None, epochs=5):
    torch.manual_seed(0)
    paddle.enable_static()
    try:
        main = static.Program()
        with static.program_guard(main):
            x = static.data("x", [None, 4], "float32")
            y = static.data("y", [None, 1], "float32")
            loss = paddle.mean((static.nn.fc(x, 1) - y) ** 2)
            paddle.optimizer.Adam(learning_rate=0.05).minimize(loss)
        seen = []
        with static.scope_guard(static.Scope()):
            exe = static.Executor(paddle.CPUPlace())
            for epoch in acp.train_epoch_range(epochs, save_checkpoint_inter=0):
                if epoch == crash_at:
                    raise Crash()
                X, Y = _data(epoch)
                seen.append(epoch)
                out = exe.run(main, feed={"x": X, "y": Y}, fetch_list=[loss])
            w = {n: static.global_scope().get(n).detach().clone() for n in main.params}
        return seen, float(out[0]), w
    finally:
        paddle.disable_static()


def test_static_program_resumes(acp_env):
    ref_seen, ref_loss, ref_w = _static_job()
    import shutil
    shutil.rmtree(acp_env / "ckpt")
    with pytest.raises(Crash):
        _static_job(crash_at=3)
    seen, loss, w = _static_job()
    assert seen == [3, 4] and ref_seen == [0, 1, 2, 3, 4]
    assert loss == ref_loss
    assert len(w) == len(ref_w)
    for a, b in zip(w.values(), ref_w.values()):  # same program, names generated per build
        assert torch.equal(a, b)


_DYGRAPH_JOB = r"""
import sys, json, numpy as np, torch
sys.path.insert(0, sys.argv[1])
import paddle_infer_amd as paddle
from paddle_infer_amd.incubate.checkpoint import auto_checkpoint as acp
crash_at = int(sys.argv[2])
torch.manual_seed(0)
net = paddle.nn.Linear(4, 1)
opt = paddle.optimizer.Momentum(learning_rate=0.05, momentum=0.9, parameters=net.parameters())
seen = []
for epoch in acp.train_epoch_range(4, save_checkpoint_inter=0):
    acp.register(net, opt, keys=["net", "opt"])
    if epoch == crash_at:
        sys.exit(17)  # the job dies here
    r = np.random.RandomState(epoch)
    X, Y = torch.as_tensor(r.randn(6, 4).astype("float32")), torch.as_tensor(r.randn(6, 1).astype("float32"))
    loss = torch.mean((net(X) - Y) ** 2)
    loss.backward()
    opt.step()
    opt.clear_grad()
    seen.append(epoch)
print(json.dumps({"seen": seen, "w": net.weight.detach().flatten().tolist(), "b": net.bias.detach().tolist()}))
"""


def _dygraph_job(root, crash_at=-1):
    """One job process (a restart is a new process, as on a cluster)."""
    import json
    import os
    import subprocess
    import sys
    r = subprocess.run([sys.executable, "-c", _DYGRAPH_JOB, root, str(crash_at)], capture_output=True,
                       text=True, env=dict(os.environ), timeout=300)
    if crash_at >= 0:
        assert r.returncode == 17, r.stderr[-2000:]
        return None
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_dygraph_objects_resume(acp_env):
    import os
    import shutil
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ref = _dygraph_job(root)
    shutil.rmtree(acp_env / "ckpt")
    _dygraph_job(root, crash_at=2)
    got = _dygraph_job(root)
    assert ref["seen"] == [0, 1, 2, 3] and got["seen"] == [2, 3]
    assert got["w"] == ref["w"] and got["b"] == ref["b"]  # bitwise: params + momentum restored


def test_off_without_env(tmp_path, monkeypatch):
    monkeypatch.delenv("PADDLE_RUNNING_ENV", raising=False)
    assert list(acp.train_epoch_range(3)) == [0, 1, 2]


def test_keeps_last_checkpoints_only(acp_env):
    _static_job(epochs=6)
    import os
    rng = acp_env / "ckpt" / "job_1" / "range" / "range_0"
    assert sorted(os.listdir(rng)) == ["checkpoint.3", "checkpoint.4"]
