"""Static autodiff (CPU): per-op grad ops, renamed-gradient sums, the optimizer pass (sgd / momentum /
adam / adamw ops + grad clip), static-vs-dygraph training parity, and a saved TRAINING program
(reference op types only) that reloads and keeps training to the same losses.

Parity: reference `python/paddle/fluid/backward.py:1569` (append_backward), `optimizer.py`
(_create_optimization_pass), `python/paddle/static/io.py` (save / load of a training program);
test style after `unittests/test_backward.py` and `test_imperative_*` static-vs-dygraph checks."""
import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import static
from paddle_infer_amd.static.backward import op_role, BACKWARD, OPTIMIZE


@pytest.fixture(autouse=True)
def _static_mode():
    paddle.enable_static()
    yield
    paddle.disable_static()


def _mlp_program(opt_fn, seed=0):
    torch.manual_seed(seed)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data("x", [None, 8], "float32")
        y = static.data("y", [None, 1], "float32")
        h = static.nn.fc(x, 16, activation="relu")
        pred = static.nn.fc(h, 1)
        loss = paddle.mean((pred - y) ** 2)
        opt_fn().minimize(loss)
    return main, loss


def _dygraph_losses(main, opt_fn, feeds):
    """Same network in dygraph, initialised from the static program's initial parameters."""
    paddle.disable_static()
    try:
        names = [n for n, t in main.params.items() if t.requires_grad]
        ws = {n: main.params[n].detach().clone().requires_grad_(True) for n in names}
        w1, b1, w2, b2 = [ws[n] for n in names]
        opt = opt_fn(list(ws.values()))
        out = []
        for X, Y in feeds:
            X, Y = torch.as_tensor(X), torch.as_tensor(Y)
            h = torch.relu(X @ w1 + b1)
            loss = torch.mean((h @ w2 + b2 - Y) ** 2)
            loss.backward()
            opt.step()
            opt.clear_grad()
            out.append(float(loss))
        return out
    finally:
        paddle.enable_static()


def _feeds(n=6, seed=1):
    r = np.random.RandomState(seed)
    return [(r.randn(5, 8).astype("float32"), r.randn(5, 1).astype("float32")) for _ in range(n)]


def test_grad_ops_per_forward_op():
    main, loss = _mlp_program(lambda: paddle.optimizer.SGD(learning_rate=0.1))
    types = [op.type for op in main.global_block().ops]
    bwd = [op for op in main.global_block().ops if op_role(op) == BACKWARD]
    assert any(t.endswith("_grad") for t in types)
    assert all(op.type.endswith("_grad") or op.type in ("fill_any_like", "sum") for op in bwd)
    fwd_n = len([op for op in main.global_block().ops if op_role(op) == 0])
    assert len([op for op in bwd if op.type.endswith("_grad")]) == fwd_n
    assert sum(op.type == "sgd" and op_role(op) == OPTIMIZE for op in main.global_block().ops) == 4
    # grad op slots: forward inputs/outputs + Out@GRAD -> X@GRAD
    g = [op for op in bwd if op.type.endswith("_grad")][0]
    assert any(k.endswith("@GRAD") for k in g.paddle_inputs) and all(k.endswith("@GRAD") for k in g.paddle_outputs)


def test_repeated_use_is_summed():
    main = static.Program()
    with static.program_guard(main):
        x = static.data("x", [3, 3], "float32")
        w = static.create_parameter([3, 3], "float32")
        y = x @ w
        loss = paddle.sum(y * w + w)  # w feeds three ops
        pg = static.append_backward(loss)
    ops = main.global_block().ops
    assert any(op.type == "sum" for op in ops)
    exe = static.Executor(paddle.CPUPlace())
    X = np.random.RandomState(0).randn(3, 3).astype("float32")
    g, = exe.run(main, feed={"x": X}, fetch_list=[pg[0][1].var_name])
    W = static.global_scope().get(pg[0][0].var_name).detach().clone().requires_grad_(True)
    ref = torch.autograd.grad(torch.sum((torch.as_tensor(X) @ W) * W + W), W)[0]
    np.testing.assert_allclose(g, ref.numpy(), rtol=1e-5, atol=1e-6)


def test_gradients_wrt_data():
    main = static.Program()
    with static.program_guard(main):
        x = static.data("x", [2, 4], "float32")
        y = paddle.sum(paddle.tanh(x) * 3.0)
        gx, = static.gradients(y, [x])
    exe = static.Executor(paddle.CPUPlace())
    X = np.random.RandomState(2).randn(2, 4).astype("float32")
    g, = exe.run(main, feed={"x": X}, fetch_list=[gx.var_name])
    np.testing.assert_allclose(g, 3.0 * (1 - np.tanh(X) ** 2), rtol=1e-5)


@pytest.mark.parametrize("kind", ["sgd", "momentum", "adam", "adamw_clip"])
def test_static_training_matches_dygraph(kind):
    O = paddle.optimizer

    def mk(params=None):
        if kind == "sgd":
            return O.SGD(learning_rate=0.05, parameters=params)
        if kind == "momentum":
            return O.Momentum(learning_rate=0.05, momentum=0.9, parameters=params)
        if kind == "adam":
            return O.Adam(learning_rate=0.01, parameters=params)
        return O.AdamW(learning_rate=0.01, weight_decay=0.05, parameters=params,
                       grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    main, loss = _mlp_program(mk)
    feeds = _feeds()
    ref = _dygraph_losses(main, mk, feeds)
    with static.scope_guard(static.Scope()):
        exe = static.Executor(paddle.CPUPlace())
        got = [float(exe.run(main, feed={"x": X, "y": Y}, fetch_list=[loss])[0]) for X, Y in feeds]
    np.testing.assert_allclose(got, ref, rtol=2e-4, atol=1e-6)
    assert got[-1] < got[0]


def test_saved_training_program_reloads_and_trains(tmp_path):
    O = paddle.optimizer
    mk = lambda p=None: O.Adam(learning_rate=0.01, parameters=p,  # noqa: E731
                               grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    main, loss = _mlp_program(mk)
    feeds = _feeds(8)
    with static.scope_guard(static.Scope()):
        exe = static.Executor(paddle.CPUPlace())
        ref = [float(exe.run(main, feed={"x": X, "y": Y}, fetch_list=[loss])[0]) for X, Y in feeds]
    with static.scope_guard(static.Scope()):
        exe = static.Executor(paddle.CPUPlace())
        for X, Y in feeds[:3]:
            exe.run(main, feed={"x": X, "y": Y}, fetch_list=[loss])
        static.save(main, str(tmp_path / "train"))
    prog = static.deserialize_program(open(tmp_path / "train.pdmodel", "rb").read())
    types = {op.type for op in prog.global_block().ops}
    assert {"matmul_v2_grad", "adam", "fill_any_like"} <= types, types
    assert all(op.func is None for op in prog.global_block().ops)  # reference op types only
    assert not any("op_callable" in op.attrs for op in prog.global_block().ops)
    with static.scope_guard(static.Scope()):
        exe = static.Executor(paddle.CPUPlace())
        static.load(prog, str(tmp_path / "train"), exe)
        got = [float(exe.run(prog, feed={"x": X, "y": Y}, fetch_list=[loss.var_name])[0]) for X, Y in feeds[3:]]
    np.testing.assert_allclose(got, ref[3:], rtol=2e-4, atol=1e-6)


def test_recompute_vjp_path_matches(monkeypatch):
    """Grad ops without an op-local graph re-run their forward op on leaves: same gradients."""
    from paddle_infer_amd.static import executor as E
    main = static.Program()
    with static.program_guard(main):
        x = static.data("x", [4, 6], "float32")
        w = static.create_parameter([6, 5], "float32")
        h = paddle.nn.functional.gelu(x @ w)
        loss = paddle.mean(paddle.nn.functional.softmax(h, -1) * h)
        pg = static.append_backward(loss)
    X = np.random.RandomState(3).randn(4, 6).astype("float32")
    exe = static.Executor(paddle.CPUPlace())
    g_fast, = exe.run(main, feed={"x": X}, fetch_list=[pg[0][1].var_name])
    orig = E.Executor._run_grad_op

    def no_graph(self, op, sub, env):
        self._leafmap = {}
        return orig(self, op, sub, env)
    monkeypatch.setattr(E.Executor, "_run_grad_op", no_graph)
    g_re, = exe.run(main, feed={"x": X}, fetch_list=[pg[0][1].var_name])
    np.testing.assert_allclose(g_re, g_fast, rtol=1e-6, atol=1e-7)


def test_static_training_through_cond_and_while_matches_dygraph(tmp_path):
    """append_backward through control flow (reference while_grad / conditional_block_grad,
    `while_op.cc:586`, `conditional_block_op.cc:423`): a data-dependent branch and a
    data-dependent loop between two fc layers train to the same losses as dygraph."""
    torch.manual_seed(3)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data("x", [None, 8], "float32")
        y = static.data("y", [None, 1], "float32")
        h = static.nn.fc(x, 8, activation="relu")
        h2 = static.nn.cond(paddle.mean(h) > 0.3, lambda: h * 2.0, lambda: h - 1.0)
        k0 = paddle.zeros([1], "float32")
        h3, _ = static.nn.while_loop(lambda a, k: paddle.sum(paddle.abs(a)) < 40.0,
                                     lambda a, k: [a * 1.5 + 0.1, k + 1.0], [h2, k0])
        pred = static.nn.fc(h3, 1)
        loss = paddle.mean((pred - y) ** 2)
        paddle.optimizer.SGD(learning_rate=0.001).minimize(loss)
    types = {op.type for op in main.global_block().ops}
    assert {"cond_grad", "while_grad"} <= types
    names = [n for n, t in main.params.items() if t.requires_grad]
    init = {n: main.params[n].detach().clone() for n in names}
    feeds = _feeds(5, seed=4)
    exe = static.Executor()
    got = [float(exe.run(main, feed={"x": X, "y": Y}, fetch_list=[loss])[0]) for X, Y in feeds]
    paddle.disable_static()
    try:
        w1, b1, w2, b2 = [init[n].clone().requires_grad_(True) for n in names]
        opt = paddle.optimizer.SGD(learning_rate=0.001, parameters=[w1, b1, w2, b2])
        ref = []
        for X, Y in feeds:
            X, Y = torch.as_tensor(X), torch.as_tensor(Y)
            h = torch.relu(X @ w1 + b1)
            h = h * 2.0 if float(h.mean()) > 0.3 else h - 1.0
            while float(h.abs().sum()) < 40.0:
                h = h * 1.5 + 0.1
            loss_d = torch.mean((h @ w2 + b2 - Y) ** 2)
            loss_d.backward()
            opt.step()
            opt.clear_grad()
            ref.append(float(loss_d))
    finally:
        paddle.enable_static()
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)
    # the trained program saves as a Paddle program (conditional_block / while sub-blocks) and the
    # reloaded inference model reproduces the dygraph forward with the trained weights
    path = str(tmp_path / "cf")
    static.save_inference_model(path, [x], [pred], exe, program=main)
    lp, lfeeds, lfetch = static.load_inference_model(path, exe)
    assert {"conditional_block", "while", "select_input"} <= {op.type for b in lp.blocks for op in b.ops}
    for X, _ in feeds[:3]:
        out = exe.run(lp, feed={lfeeds[0]: X}, fetch_list=lfetch)[0]
        with torch.no_grad():
            h = torch.relu(torch.as_tensor(X) @ w1 + b1)
            h = h * 2.0 if float(h.mean()) > 0.3 else h - 1.0
            while float(h.abs().sum()) < 40.0:
                h = h * 1.5 + 0.1
            np.testing.assert_allclose(out, (h @ w2 + b2).numpy(), rtol=1e-4, atol=1e-5)
