"""dy2static (reference `fluid/dygraph/dygraph_to_static/`): Python control flow on tensors in a
to_static function becomes cond / while ops with sub-blocks; the recorded Program then takes the
branch / iteration count the FED data selects (the trace alone would freeze the first one)."""
import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import jit, static
from paddle_infer_amd.jit import dy2static


def f_if(x):
    if paddle.mean(x) > 0:
        y = x * 2.0
    else:
        y = x - 1.0
    return y + 1.0


def f_while(x):
    s = x
    while paddle.sum(paddle.abs(s)) < 100.0:
        s = s * 2.0
    return s


def f_for_and(x, n: int = 3):
    acc = paddle.zeros_like(x)
    for i in range(n):
        acc = acc + x * float(i + 1)
    if paddle.max(acc) > 0 and paddle.min(acc) > -100:
        acc = acc / 2.0
    return acc


def _run_program(fn, X):
    prog, feeds, fetch = jit.trace_program(fn, [static.InputSpec([None, 4], "float32", "x")])
    exe = static.Executor(paddle.CPUPlace())
    return prog, exe.run(prog, feed={"x": X}, fetch_list=[f.var_name for f in fetch])[0]


@pytest.mark.parametrize("fn", [f_if, f_while, f_for_and])
def test_program_follows_fed_data(fn):
    conv = dy2static.convert_to_static(fn)
    for seed, sign in [(0, 1.0), (1, -1.0)]:
        X = (np.abs(np.random.RandomState(seed).randn(3, 4)) * sign + 0.1 * sign).astype("float32")
        ref = fn(torch.as_tensor(X)).numpy()
        np.testing.assert_allclose(conv(torch.as_tensor(X)).numpy(), ref, rtol=1e-6)  # eager: same semantics
        prog, got = _run_program(fn, X)
        np.testing.assert_allclose(got, ref, rtol=1e-6)
    types = {op.type for b in prog.blocks for op in b.ops}
    if fn is f_if:
        assert "cond" in types
    if fn is f_while:
        assert "while" in types


def test_branch_assigns_new_name_and_closure():
    scale = 3.0

    def f(x):
        if paddle.sum(x) > 0:
            z = x * scale
        else:
            z = -x
        return z

    for X in (np.ones((2, 4), "float32"), -np.ones((2, 4), "float32")):
        _, got = _run_program(f, X)
        np.testing.assert_allclose(got, f(torch.as_tensor(X)).numpy())


def test_python_values_stay_python():
    def f(x, flag=True):
        if flag:
            x = x + 1
        k = 0
        while k < 3:
            k = k + 1
        return x * k
    conv = dy2static.convert_to_static(f)
    x = torch.ones(2)
    assert torch.equal(conv(x), f(x))
    assert "convert_ifelse" in conv._dy2static_source


def test_return_inside_branch_left_as_python():
    def f(x):
        if x.sum() > 0:
            return x
        return -x
    conv = dy2static.convert_to_static(f)
    assert torch.equal(conv(torch.ones(2)), torch.ones(2))
    assert "convert_ifelse" not in conv._dy2static_source


@pytest.mark.parametrize("fn", [f_if, f_while, f_for_and])
def test_control_flow_saves_as_paddle_program(fn, tmp_path):
    """cond / while serialise as Paddle ``conditional_block`` + ``select_input`` / ``while`` ops
    with sub-blocks (reference `layers/control_flow.py`), and the reloaded .pdmodel still follows
    the fed data."""
    from paddle_infer_amd.static import io as sio
    prog, feeds, fetch = jit.trace_program(fn, [static.InputSpec([None, 4], "float32", "x")])
    exe = static.Executor(paddle.CPUPlace())
    path = str(tmp_path / "m")
    static.save_inference_model(path, feeds, fetch, exe, program=prog)
    with open(path + ".pdmodel", "rb") as f:
        desc = sio.proto.decode("ProgramDesc", f.read())
    types = {od["type"] for bd in desc["blocks"] for od in bd.get("ops", [])}
    assert not types & {"cond"}
    if fn in (f_if, f_for_and):
        assert {"conditional_block", "select_input"} <= types and len(desc["blocks"]) >= 3
    if fn is f_while:
        assert "while" in types and len(desc["blocks"]) >= 2
    lp, lfeeds, lfetch = static.load_inference_model(path, exe)
    for seed, sign in [(0, 1.0), (1, -1.0), (2, 0.01)]:
        X = (np.abs(np.random.RandomState(seed).randn(3, 4)) * sign + 0.1 * sign).astype("float32")
        ref = fn(torch.as_tensor(X)).numpy()
        got = exe.run(lp, feed={lfeeds[0]: X}, fetch_list=lfetch)[0]
        np.testing.assert_allclose(got, ref, rtol=1e-6)
