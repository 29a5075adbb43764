"""CompiledProgram / BuildStrategy (reference `python/paddle/fluid/compiler.py`): fusion passes
applied to a Paddle-typed inference program (outputs unchanged), and ``with_data_parallel``
static training over 2 gloo ranks (gradients averaged before the optimizer ops) matching a
single process on the full batch."""
import os

import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import static

from dist_utils import run_distributed


def _mlp_program(seed=0):
    torch.manual_seed(seed)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data("x", [None, 8], "float32")
        y = static.data("y", [None, 1], "float32")
        h = static.nn.fc(x, 16, activation="relu")
        pred = static.nn.fc(h, 1)
        loss = paddle.mean((pred - y) ** 2)
        paddle.optimizer.SGD(learning_rate=0.1).minimize(loss)
    return main, loss


def _feeds(n=4, B=8, seed=1):
    r = np.random.RandomState(seed)
    return [(r.randn(B, 8).astype("float32"), r.randn(B, 1).astype("float32")) for _ in range(n)]


def _train(compiled_dp, rank=0, world=1):
    paddle.enable_static()
    try:
        main, loss = _mlp_program()
        exe = static.Executor("cpu")
        scope = static.Scope()
        prog = static.CompiledProgram(main).with_data_parallel(loss_name=loss.var_name) if compiled_dp else main
        losses = []
        with static.scope_guard(scope):
            for X, Y in _feeds():
                xs, ys = np.split(X, world)[rank], np.split(Y, world)[rank]
                (lv,) = exe.run(prog, feed={"x": xs, "y": ys}, fetch_list=[loss])
                losses.append(float(lv))
            params = [scope.get(n).detach().clone() for n in main.params
                      if not n.startswith("learning_rate")]
        return params, losses
    finally:
        paddle.disable_static()


def _dp_worker(rank, world):
    return _train(True, rank, world)


def test_with_data_parallel_matches_single_process():
    ref_params, ref_losses = _train(False)
    res = run_distributed(_dp_worker, 2)
    for r in range(2):
        params, losses = res[r]
        assert len(params) == len(ref_params) == 4
        for a, b in zip(params, ref_params):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    # the full-batch loss is the mean of the two half-batch losses
    for i, l0 in enumerate(ref_losses):
        assert (res[0][1][i] + res[1][1][i]) / 2 == pytest.approx(l0, rel=1e-5)


def test_build_strategy_fusion_on_inference_program(tmp_path):
    import paddle_infer_amd.nn as nn
    from paddle_infer_amd import jit
    from paddle_infer_amd.static import InputSpec

    class M(nn.Layer):
        def __init__(self):
            super().__init__()
            self.a = nn.Linear(8, 16)
            self.b = nn.Linear(16, 4)

        def forward(self, x):
            return self.b(paddle.nn.functional.relu(self.a(x)))

    torch.manual_seed(0)
    m = M()
    m.eval()
    path = os.path.join(tmp_path, "m")
    jit.save(m, path, input_spec=[InputSpec([None, 8], "float32", "x")])
    x = np.random.RandomState(0).randn(3, 8).astype("float32")
    with torch.no_grad():
        ref = m(torch.from_numpy(x)).numpy()
    paddle.enable_static()
    try:
        exe = static.Executor("cpu")
        prog, feeds, fetches = static.load_inference_model(path, exe)
        bs = static.BuildStrategy()
        bs.fuse_elewise_add_act_ops = True
        cp = static.CompiledProgram(prog, build_strategy=bs)
        (out,) = exe.run(cp, feed={feeds[0]: x}, fetch_list=fetches)
        types = [op.type for op in cp._program.global_block().ops]
    finally:
        paddle.disable_static()
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-5)
    assert "fc" in types and "matmul_v2" not in types
    assert [op.type for op in prog.global_block().ops].count("matmul_v2") == 2  # source untouched
