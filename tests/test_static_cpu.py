"""Static-graph tests (CPU): Program recording, Executor training, dynamic batch dims,
inference-model save/load round trip, and execution of a Paddle-wire ProgramDesc built from raw
Paddle op types (the path used for `.pdmodel` files produced by the reference).

Parity model: reference `python/paddle/fluid/tests/unittests/test_executor_and_mul.py`,
`test_inference_model_io.py`, `test_program.py` (same APIs exercised).
"""
import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import static
from paddle_infer_amd.static import proto


@pytest.fixture(autouse=True)
def _static_mode():
    paddle.enable_static()
    yield
    paddle.disable_static()


def _mlp_program():
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data("x", [None, 8], "float32")
        y = static.data("y", [None, 1], "float32")
        h = static.nn.fc(x, 16, activation="relu")
        pred = static.nn.fc(h, 1)
        loss = paddle.mean((pred - y) ** 2)
        paddle.optimizer.Adam(learning_rate=0.01).minimize(loss)
    return main, startup, x, y, pred, loss


def test_executor_trains_and_dynamic_batch(tmp_path):
    paddle.seed(1)
    main, startup, x, y, pred, loss = _mlp_program()
    exe = static.Executor(paddle.CPUPlace())
    exe.run(startup)
    rng = np.random.RandomState(0)
    X = rng.randn(64, 8).astype("float32")
    Y = X.sum(1, keepdims=True).astype("float32")
    losses = [float(exe.run(main, feed={"x": X, "y": Y}, fetch_list=[loss])[0]) for _ in range(60)]
    assert losses[-1] < 0.2 * losses[0]
    test = main.clone(for_test=True)
    # a different batch size than the one fed during training
    out, = exe.run(test, feed={"x": X[:5], "y": Y[:5]}, fetch_list=[pred])
    assert out.shape == (5, 1)


def test_inference_model_round_trip(tmp_path):
    main, startup, x, y, pred, loss = _mlp_program()
    exe = static.Executor(paddle.CPUPlace())
    exe.run(startup)
    X = np.random.RandomState(1).randn(7, 8).astype("float32")
    exe.run(main, feed={"x": X, "y": X[:, :1]}, fetch_list=[loss])
    ref, = exe.run(main.clone(for_test=True), feed={"x": X, "y": X[:, :1]}, fetch_list=[pred])
    prefix = str(tmp_path / "m" / "model")
    static.save_inference_model(prefix, [x], [pred], exe, program=main)
    with static.scope_guard(static.Scope()):
        exe2 = static.Executor(paddle.CPUPlace())
        prog, feeds, fetches = static.load_inference_model(prefix, exe2)
        assert feeds == ["x"]
        got, = exe2.run(prog, feed={"x": X}, fetch_list=fetches)
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-6)
    # the pdmodel is a valid framework.proto ProgramDesc with feed/fetch ops
    desc = proto.decode("ProgramDesc", open(prefix + ".pdmodel", "rb").read())
    types = [o["type"] for o in desc["blocks"][0]["ops"]]
    assert types[0] == "feed" and types[-1] == "fetch"


def _op(type_, ins, outs, attrs=()):
    return {"type": type_, "inputs": [{"parameter": k, "arguments": v} for k, v in ins.items()],
            "outputs": [{"parameter": k, "arguments": v} for k, v in outs.items()],
            "attrs": list(attrs)}


def _var(name, dims, persistable=False):
    return {"name": name, "persistable": persistable,
            "type": {"type": proto.VT_LOD_TENSOR,
                     "lod_tensor": {"tensor": {"data_type": proto.VT["float32"], "dims": dims}}}}


def test_paddle_wire_program_executes(tmp_path):
    """A ProgramDesc written with Paddle's own op types and slots (as Paddle's
    save_inference_model emits them) loads and runs through the op registry."""
    A = proto.ATTR
    rng = np.random.RandomState(3)
    w = rng.randn(6, 4).astype("float32")
    b = rng.randn(4).astype("float32")
    g = rng.rand(4).astype("float32") + 0.5
    be = rng.randn(4).astype("float32")
    ops = [
        _op("feed", {"X": ["feed"]}, {"Out": ["x"]}, [{"name": "col", "type": A["INT"], "i": 0}]),
        _op("matmul_v2", {"X": ["x"], "Y": ["fc.w"]}, {"Out": ["t0"]},
            [{"name": "trans_x", "type": A["BOOLEAN"], "b": False},
             {"name": "trans_y", "type": A["BOOLEAN"], "b": False}]),
        _op("elementwise_add", {"X": ["t0"], "Y": ["fc.b"]}, {"Out": ["t1"]},
            [{"name": "axis", "type": A["INT"], "i": -1}]),
        _op("relu", {"X": ["t1"]}, {"Out": ["t2"]}),
        _op("layer_norm", {"X": ["t2"], "Scale": ["ln.g"], "Bias": ["ln.b"]},
            {"Y": ["t3"], "Mean": ["m"], "Variance": ["v"]},
            [{"name": "epsilon", "type": A["FLOAT"], "f": 1e-5},
             {"name": "begin_norm_axis", "type": A["INT"], "i": 1}]),
        _op("scale", {"X": ["t3"]}, {"Out": ["t4"]},
            [{"name": "scale", "type": A["FLOAT"], "f": 2.0}, {"name": "bias", "type": A["FLOAT"], "f": 0.5},
             {"name": "bias_after_scale", "type": A["BOOLEAN"], "b": True}]),
        _op("softmax", {"X": ["t4"]}, {"Out": ["out"]}, [{"name": "axis", "type": A["INT"], "i": -1}]),
        _op("fetch", {"X": ["out"]}, {"Out": ["fetch"]}, [{"name": "col", "type": A["INT"], "i": 0}]),
    ]
    vars_ = [_var("x", [-1, 6]), _var("fc.w", [6, 4], True), _var("fc.b", [4], True),
             _var("ln.g", [4], True), _var("ln.b", [4], True)] + \
        [_var(n, [-1, 4]) for n in ("t0", "t1", "t2", "t3", "t4", "out")]
    desc = {"blocks": [{"idx": 0, "parent_idx": -1, "vars": vars_, "ops": ops}]}
    prefix = str(tmp_path / "wire")
    open(prefix + ".pdmodel", "wb").write(proto.encode("ProgramDesc", desc))
    params = {"fc.b": b, "fc.w": w, "ln.b": be, "ln.g": g}
    with open(prefix + ".pdiparams", "wb") as f:
        for n in sorted(params):
            f.write(proto.tensor_to_stream(params[n], proto.VT["float32"]))
    with static.scope_guard(static.Scope()):
        exe = static.Executor(paddle.CPUPlace())
        prog, feeds, fetches = static.load_inference_model(prefix, exe)
        X = rng.randn(3, 6).astype("float32")
        got, = exe.run(prog, feed={"x": X}, fetch_list=fetches)
    t = torch.relu(torch.from_numpy(X) @ torch.from_numpy(w) + torch.from_numpy(b))
    t = torch.nn.functional.layer_norm(t, (4,), torch.from_numpy(g), torch.from_numpy(be), 1e-5)
    ref = torch.softmax(t * 2.0 + 0.5, -1).numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)


def test_append_backward_and_gradients():
    main = static.Program()
    with static.program_guard(main):
        x = static.data("x", [4, 3], "float32")
        w = static.create_parameter([3, 2], "float32")
        loss = paddle.sum(paddle.matmul(x, w) ** 2)
        pg = static.append_backward(loss)
    assert len(pg) == 1
    exe = static.Executor(paddle.CPUPlace())
    X = np.ones((4, 3), "float32")
    gname = pg[0][1].var_name if hasattr(pg[0][1], "var_name") else pg[0][1]
    g, = exe.run(main, feed={"x": X}, fetch_list=[gname])
    W = static.global_scope().get(pg[0][0].var_name if hasattr(pg[0][0], "var_name") else pg[0][0])
    W = W.detach().numpy()
    ref = 2 * X.T @ (X @ W)
    np.testing.assert_allclose(g, ref, rtol=1e-5)


def test_native_plan_frees_intermediates():
    from paddle_infer_amd.static.executor import build_plan
    main = static.Program()
    with static.program_guard(main):
        x = static.data("x", [2, 2], "float32")
        a = x + 1
        b = a * 2
        c = b - 3
    order, frees, levels = build_plan(main.global_block().ops, {c.var_name})
    assert order == [0, 1, 2]
    freed = [n for f in frees for n in f]
    assert a.var_name in freed and b.var_name in freed and c.var_name not in freed
