"""The long-tail program op types (`static/ops_registry_tail.py`): each op runs from a hand-built
Paddle-wire ProgramDesc (feed → op → fetch, reference slot / attribute names) through the static
Executor and is compared with an independent numpy / fp32 composition of the reference kernel's
formula. Optimizer ops are stepped twice against literal transcriptions of the reference
kernels; collectives run on 2 gloo ranks."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from paddle_infer_amd import static
from paddle_infer_amd.static import proto
from paddle_infer_amd.static.io import deserialize_program
from paddle_infer_amd.static.ops_registry import REGISTRY

A = proto.ATTR
R = np.random.RandomState(0)


def _attr(k, v):
    if isinstance(v, bool):
        return {"name": k, "type": A["BOOLEAN"], "b": v}
    if isinstance(v, int):
        return {"name": k, "type": A["INT"], "i": v}
    if isinstance(v, float):
        return {"name": k, "type": A["FLOAT"], "f": v}
    if isinstance(v, str):
        return {"name": k, "type": A["STRING"], "s": v}
    if isinstance(v, (list, tuple)):
        if all(isinstance(t, str) for t in v) and v:
            return {"name": k, "type": A["STRINGS"], "strings": list(v)}
        if any(isinstance(t, float) for t in v):
            return {"name": k, "type": A["FLOATS"], "floats": [float(t) for t in v]}
        return {"name": k, "type": A["INTS"], "ints": [int(t) for t in v]}
    raise TypeError(k)


def _dt(a):
    return {np.float32: "float32", np.float64: "float64", np.int64: "int64", np.int32: "int32",
            np.bool_: "bool", np.uint8: "uint8", np.int8: "int8"}[a.dtype.type]


def run_op(op_type, inputs, outputs, attrs=None):
    """inputs: {slot: ndarray or [ndarray, ...]}; outputs: {slot: n_vars}. Returns {slot: [ndarray]}."""
    vars_, ops, feed, fetch = [], [], {}, []
    ins = {}
    col = 0
    for slot, vals in inputs.items():
        vals = vals if isinstance(vals, list) else [vals]
        names = []
        for i, v in enumerate(vals):
            n = f"{slot}_{i}"
            vars_.append({"name": n, "type": {"type": proto.VT_LOD_TENSOR, "lod_tensor": {
                "tensor": {"data_type": proto.VT[_dt(v)], "dims": list(v.shape)}, "lod_level": 0}},
                "persistable": False})
            ops.append({"type": "feed", "inputs": [{"parameter": "X", "arguments": ["feed"]}],
                        "outputs": [{"parameter": "Out", "arguments": [n]}], "attrs": [_attr("col", col)]})
            col += 1
            feed[n] = v.copy()  # in-place optimizer ops must not touch the test's arrays
            names.append(n)
        ins[slot] = names
    outs = {}
    for slot, k in outputs.items():
        names = [f"o_{slot}_{i}" for i in range(k)]
        for n in names:
            vars_.append({"name": n, "type": {"type": proto.VT_LOD_TENSOR, "lod_tensor": {
                "tensor": {"data_type": proto.VT["float32"], "dims": [-1]}, "lod_level": 0}},
                "persistable": False})
        outs[slot] = names
    ops.append({"type": op_type, "inputs": [{"parameter": k, "arguments": v} for k, v in ins.items()],
                "outputs": [{"parameter": k, "arguments": v} for k, v in outs.items()],
                "attrs": [_attr(k, v) for k, v in (attrs or {}).items()]})
    for slot, names in outs.items():
        for n in names:
            ops.append({"type": "fetch", "inputs": [{"parameter": "X", "arguments": [n]}],
                        "outputs": [{"parameter": "Out", "arguments": ["fetch"]}],
                        "attrs": [_attr("col", len(fetch))]})
            fetch.append(n)
    desc = {"blocks": [{"idx": 0, "parent_idx": -1, "vars": vars_, "ops": ops}]}
    prog = deserialize_program(proto.encode("ProgramDesc", desc))
    exe = static.Executor("cpu")
    with static.scope_guard(static.Scope()):
        res = exe.run(prog, feed=feed, fetch_list=fetch)
    out, i = {}, 0
    for slot, names in outs.items():
        out[slot] = res[i:i + len(names)]
        i += len(names)
    return out


def f32(*s, lo=-1.0, hi=1.0):
    return R.uniform(lo, hi, s).astype("float32")


# --------------------------------------------------------------------------- elementwise / math
UNARY = [
    ("acos", lambda x: np.arccos(x), {}), ("asinh", np.arcsinh, {}), ("atan", np.arctan, {}),
    ("cosh", np.cosh, {}), ("tan", np.tan, {}), ("expm1", np.expm1, {}), ("log2", lambda x: np.log2(x + 2), "shift"),
    ("celu", lambda x: np.where(x > 0, x, 0.7 * (np.exp(x / 0.7) - 1)), {"alpha": 0.7}),
    ("hard_shrink", lambda x: np.where(np.abs(x) > 0.3, x, 0), {"threshold": 0.3}),
    ("thresholded_relu", lambda x: np.where(x > 0.2, x, 0), {"threshold": 0.2}),
    ("brelu", lambda x: np.clip(x, -0.5, 0.4), {"t_min": -0.5, "t_max": 0.4}),
    ("selu", lambda x: 1.05 * np.where(x > 0, x, 1.6 * (np.exp(x) - 1)), {"scale": 1.05, "alpha": 1.6}),
]


@pytest.mark.parametrize("op,ref,attrs", UNARY, ids=[u[0] for u in UNARY])
def test_unary_ops(op, ref, attrs):
    x = f32(3, 5)
    if attrs == "shift":
        out = run_op(op, {"X": x + 2}, {"Out": 1}, {})["Out"][0]
        np.testing.assert_allclose(out, ref(x), rtol=1e-5, atol=1e-5)
        return
    out = run_op(op, {"X": x}, {"Out": 1}, attrs)["Out"][0]
    np.testing.assert_allclose(out, ref(x), rtol=1e-4, atol=1e-5)


def test_reductions_and_norms():
    x = f32(4, 6)
    np.testing.assert_allclose(run_op("reduce_amax", {"X": x}, {"Out": 1}, {"dim": [1]})["Out"][0], x.max(1))
    np.testing.assert_allclose(run_op("frobenius_norm", {"X": x}, {"Out": 1}, {"dim": [0, 1]})["Out"][0],
                               np.sqrt((x * x).sum()), rtol=1e-5)
    np.testing.assert_allclose(run_op("squared_l2_norm", {"X": x}, {"Out": 1})["Out"][0], [(x * x).sum()], rtol=1e-5)
    y = run_op("clip_by_norm", {"X": x}, {"Out": 1}, {"max_norm": 1.0})["Out"][0]
    np.testing.assert_allclose(y, x / np.sqrt((x * x).sum()), rtol=1e-5)
    y = run_op("clip_by_norm", {"X": x * 0.01}, {"Out": 1}, {"max_norm": 10.0})["Out"][0]
    np.testing.assert_allclose(y, x * 0.01, rtol=1e-6)
    r = run_op("norm", {"X": x}, {"Out": 1, "Norm": 1}, {"axis": 1, "epsilon": 1e-10})
    np.testing.assert_allclose(r["Out"][0], x / np.sqrt((x * x).sum(1, keepdims=True) + 1e-10), rtol=1e-5)
    np.testing.assert_allclose(run_op("logsumexp", {"X": x}, {"Out": 1}, {"axis": [1], "keepdim": False})["Out"][0],
                               np.log(np.exp(x).sum(1)), rtol=1e-5)


def test_binary_and_linalg():
    x, y = f32(4, 4), f32(4, 4)
    np.testing.assert_allclose(run_op("atan2", {"X1": x, "X2": y}, {"Out": 1})["Out"][0], np.arctan2(x, y), rtol=1e-5)
    np.testing.assert_allclose(run_op("elementwise_fmax", {"X": x, "Y": y}, {"Out": 1})["Out"][0], np.fmax(x, y))
    np.testing.assert_allclose(run_op("kron", {"X": x[:2, :2], "Y": y}, {"Out": 1})["Out"][0], np.kron(x[:2, :2], y),
                               rtol=1e-5)
    spd = x @ x.T + 4 * np.eye(4, dtype="float32")
    np.testing.assert_allclose(run_op("inverse", {"Input": spd}, {"Output": 1})["Output"][0], np.linalg.inv(spd),
                               rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(run_op("determinant", {"Input": spd}, {"Out": 1})["Out"][0], np.linalg.det(spd),
                               rtol=1e-4)
    np.testing.assert_allclose(run_op("cholesky", {"X": spd}, {"Out": 1}, {"upper": False})["Out"][0],
                               np.linalg.cholesky(spd), rtol=1e-4, atol=1e-5)
    b = f32(4, 2)
    np.testing.assert_allclose(run_op("solve", {"X": spd, "Y": b}, {"Out": 1})["Out"][0], np.linalg.solve(spd, b),
                               rtol=1e-4, atol=1e-5)
    inp = f32(4, 4)
    np.testing.assert_allclose(run_op("addmm", {"Input": inp, "X": x, "Y": y}, {"Out": 1},
                                      {"Alpha": 0.5, "Beta": 2.0})["Out"][0], 2 * inp + 0.5 * x @ y, rtol=1e-5)
    np.testing.assert_allclose(run_op("trace", {"Input": x}, {"Out": 1}, {"offset": 1})["Out"][0],
                               np.trace(x, 1), rtol=1e-5)
    np.testing.assert_allclose(run_op("lerp", {"X": x, "Y": y, "Weight": np.float32([0.25]).reshape(1)},
                                      {"Out": 1})["Out"][0], x + 0.25 * (y - x), rtol=1e-5)


def test_manipulation_ops():
    x = f32(2, 8, 4, 4)
    np.testing.assert_allclose(run_op("pixel_shuffle", {"X": x}, {"Out": 1}, {"upscale_factor": 2})["Out"][0],
                               F.pixel_shuffle(torch.from_numpy(x), 2).numpy())
    np.testing.assert_allclose(run_op("pixel_unshuffle", {"X": x}, {"Out": 1}, {"downscale_factor": 2})["Out"][0],
                               F.pixel_unshuffle(torch.from_numpy(x), 2).numpy())
    ts = run_op("temporal_shift", {"X": x}, {"Out": 1}, {"seg_num": 2, "shift_ratio": 0.25})["Out"][0]
    ref = np.zeros_like(x).reshape(1, 2, 8, 4, 4)
    xr = x.reshape(1, 2, 8, 4, 4)
    ref[:, :-1, :2] = xr[:, 1:, :2]
    ref[:, 1:, 2:4] = xr[:, :-1, 2:4]
    ref[:, :, 4:] = xr[:, :, 4:]
    np.testing.assert_allclose(ts, ref.reshape(x.shape))
    u = np.array([3, 1, 3, 2, 1, 7], dtype="int64")
    r = run_op("unique", {"X": u}, {"Out": 1, "Index": 1, "Indices": 1, "Counts": 1},
               {"return_index": True, "return_inverse": True, "return_counts": True, "is_sorted": True, "dtype": 3})
    np.testing.assert_array_equal(r["Out"][0], [1, 2, 3, 7])
    np.testing.assert_array_equal(r["Indices"][0], [1, 3, 0, 5])
    np.testing.assert_array_equal(r["Index"][0], [2, 0, 2, 1, 0, 3])
    np.testing.assert_array_equal(r["Counts"][0], [2, 1, 2, 1])
    arr, idx, val = f32(3, 4), np.array([[0], [2], [1]], dtype="int64"), f32(3, 1)
    out = run_op("put_along_axis", {"Input": arr, "Index": idx, "Value": val}, {"Result": 1},
                 {"Axis": 1, "Reduce": "add"})["Result"][0]
    ref = arr.copy()
    for i in range(3):
        ref[i, idx[i, 0]] += val[i, 0]
    np.testing.assert_allclose(out, ref, rtol=1e-6)
    y = run_op("space_to_depth", {"X": x}, {"Out": 1}, {"blocksize": 2})["Out"][0]
    assert y.shape == (2, 32, 2, 2)
    np.testing.assert_allclose(y[0, 0], x[0, 0, ::2, ::2])
    np.testing.assert_allclose(y[0, 8], x[0, 0, ::2, 1::2])  # (by, bx) = (0, 1) → channel block 1
    seg = run_op("segment_pool", {"X": f32(5, 3), "SegmentIds": np.array([0, 0, 1, 1, 1], "int64")},
                 {"Out": 1, "SummedIds": 1}, {"pooltype": "MEAN"})
    assert seg["Out"][0].shape == (2, 3)


@pytest.mark.parametrize("op,nd", [("linear_interp_v2", 1), ("trilinear_interp_v2", 3)])
@pytest.mark.parametrize("align_corners,align_mode", [(True, 1), (False, 0), (False, 1)])
def test_linear_trilinear_interp(op, nd, align_corners, align_mode):
    shape = (2, 3) + (5,) * nd
    x = f32(*shape)
    outsz = [7] * nd
    keys = {1: ["out_w"], 3: ["out_d", "out_h", "out_w"]}[nd]
    attrs = {k: 7 for k in keys}
    attrs.update(align_corners=align_corners, align_mode=align_mode, interp_method="linear" if nd == 1 else "trilinear",
                 data_layout="NCHW")
    y = run_op(op, {"X": x}, {"Out": 1}, attrs)["Out"][0]

    def axis_ref(a, ax, O):  # reference interpolate_v2 coordinate map, literal
        I = a.shape[ax]
        out = np.zeros(a.shape[:ax] + (O,) + a.shape[ax + 1:], np.float64)
        for o in range(O):
            if align_corners:
                src = o * (I - 1) / (O - 1)
            elif align_mode == 0:
                src = max((o + 0.5) * I / O - 0.5, 0.0)
            else:
                src = o * I / O
            lo = min(int(math.floor(src)), I - 1)
            hi = min(lo + 1, I - 1)
            w = src - lo
            out.take(0, ax)  # noqa: B018
            sl = [slice(None)] * a.ndim
            sl[ax] = o
            out[tuple(sl)] = np.take(a, lo, ax) * (1 - w) + np.take(a, hi, ax) * w
        return out
    ref = x.astype(np.float64)
    for i in range(nd):
        ref = axis_ref(ref, 2 + i, outsz[i])
    np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-5)
    if align_corners and nd == 1:
        torch.testing.assert_close(torch.from_numpy(y), F.interpolate(torch.from_numpy(x), 7, mode="linear",
                                                                      align_corners=True))


# ------------------------------------------------------------------------------------ losses
def test_losses():
    x, lab = f32(6, 4, lo=-3, hi=3), R.randint(0, 2, (6, 4)).astype("float32")
    lab[0, 0] = -100
    out = run_op("sigmoid_cross_entropy_with_logits", {"X": x, "Label": lab}, {"Out": 1},
                 {"normalize": True, "ignore_index": -100})["Out"][0]
    l = np.maximum(x, 0) - x * lab + np.log1p(np.exp(-np.abs(x)))
    l[0, 0] = 0
    np.testing.assert_allclose(out, l / 23, rtol=1e-5, atol=1e-6)
    p, y = f32(5, 1, lo=0.05, hi=0.95), R.randint(0, 2, (5, 1)).astype("float32")
    np.testing.assert_allclose(run_op("bce_loss", {"X": p, "Label": y}, {"Out": 1})["Out"][0],
                               -(y * np.log(p) + (1 - y) * np.log(1 - p)), rtol=1e-5)
    a_, b_ = f32(5, 3), f32(5, 3)
    r = run_op("huber_loss", {"X": a_, "Y": b_}, {"Out": 1, "Residual": 1}, {"delta": 0.5})
    d = b_ - a_
    np.testing.assert_allclose(r["Out"][0], np.where(np.abs(d) <= 0.5, 0.5 * d * d, 0.5 * (np.abs(d) - 0.25)),
                               rtol=1e-5, atol=1e-7)
    r = run_op("smooth_l1_loss", {"X": a_, "Y": b_}, {"Out": 1, "Diff": 1}, {"sigma": 2.0})
    ad = np.abs(a_ - b_)
    np.testing.assert_allclose(r["Out"][0], np.where(ad < 0.25, 2 * (a_ - b_) ** 2, ad - 0.125).sum(1, keepdims=True),
                               rtol=1e-5)
    logp = np.log(np.random.RandomState(1).dirichlet(np.ones(4), 5)).astype("float32")
    lb = np.array([0, 3, 1, 2, 3], "int64")
    out = run_op("nll_loss", {"X": logp, "Label": lb}, {"Out": 1, "Total_weight": 1}, {"reduction": "mean"})["Out"][0]
    np.testing.assert_allclose(out, -logp[np.arange(5), lb].mean(), rtol=1e-5)
    pr = np.random.RandomState(2).dirichlet(np.ones(4), 5).astype("float32")
    out = run_op("cross_entropy2", {"X": pr, "Label": lb.reshape(5, 1)}, {"Y": 1, "MatchX": 1}, {})["Y"][0]
    np.testing.assert_allclose(out.reshape(-1), -np.log(pr[np.arange(5), lb]), rtol=1e-5)


# -------------------------------------------------------------------------------- optimizers
def _opt_inputs(shape=(3, 4)):
    return f32(*shape), f32(*shape), np.float32([0.01])


def test_adagrad_adadelta_adamax_rmsprop():
    p, g, lr = _opt_inputs()
    m = np.abs(f32(3, 4)) * 0.1
    r = run_op("adagrad", {"Param": p, "Grad": g, "Moment": m, "LearningRate": lr}, {"ParamOut": 1, "MomentOut": 1},
               {"epsilon": 1e-6})
    m2 = m + g * g
    np.testing.assert_allclose(r["ParamOut"][0], p - 0.01 * g / (np.sqrt(m2) + 1e-6), rtol=1e-5)
    sg, su = np.abs(f32(3, 4)), np.abs(f32(3, 4))
    r = run_op("adadelta", {"Param": p, "Grad": g, "AvgSquaredGrad": sg, "AvgSquaredUpdate": su},
               {"ParamOut": 1, "AvgSquaredGradOut": 1, "AvgSquaredUpdateOut": 1}, {"rho": 0.9, "epsilon": 1e-6})
    sg2 = 0.9 * sg + 0.1 * g * g
    upd = -np.sqrt((su + 1e-6) / (sg2 + 1e-6)) * g
    np.testing.assert_allclose(r["ParamOut"][0], p + upd, rtol=1e-5)
    np.testing.assert_allclose(r["AvgSquaredUpdateOut"][0], 0.9 * su + 0.1 * upd * upd, rtol=1e-5)
    mo, inf, b1p = f32(3, 4), np.abs(f32(3, 4)), np.float32([0.9 ** 3])
    r = run_op("adamax", {"Param": p, "Grad": g, "LearningRate": lr, "Moment": mo, "InfNorm": inf, "Beta1Pow": b1p},
               {"ParamOut": 1, "MomentOut": 1, "InfNormOut": 1}, {"beta1": 0.9, "beta2": 0.999, "epsilon": 1e-8})
    mo2 = 0.9 * mo + 0.1 * g
    inf2 = np.maximum(np.abs(g), 0.999 * inf + 1e-8)
    np.testing.assert_allclose(r["ParamOut"][0], p - 0.01 / (1 - 0.9 ** 3) * mo2 / inf2, rtol=1e-5)
    ms, mom, mg = np.abs(f32(3, 4)), f32(3, 4), f32(3, 4) * 0.1
    for centered in (False, True):
        r = run_op("rmsprop", {"Param": p, "MeanSquare": ms, "Grad": g, "Moment": mom, "LearningRate": lr,
                               "MeanGrad": mg}, {"ParamOut": 1, "MomentOut": 1, "MeanSquareOut": 1, "MeanGradOut": 1},
                   {"epsilon": 1e-6, "decay": 0.9, "momentum": 0.5, "centered": centered})
        ms2 = 0.9 * ms + 0.1 * g * g
        den = np.sqrt(ms2 - (0.9 * mg + 0.1 * g) ** 2 + 1e-6) if centered else np.sqrt(ms2 + 1e-6)
        mom2 = 0.5 * mom + 0.01 * g / den
        np.testing.assert_allclose(r["ParamOut"][0], p - mom2, rtol=1e-5)


def test_lamb():
    p, g, lr = _opt_inputs()
    m1, m2 = f32(3, 4) * 0.1, np.abs(f32(3, 4)) * 0.1
    b1p, b2p = np.float32([0.9]), np.float32([0.999])
    r = run_op("lamb", {"Param": p, "Grad": g, "LearningRate": lr, "Moment1": m1, "Moment2": m2, "Beta1Pow": b1p,
                        "Beta2Pow": b2p}, {"ParamOut": 1, "Moment1Out": 1, "Moment2Out": 1, "Beta1PowOut": 1,
                                           "Beta2PowOut": 1}, {"weight_decay": 0.01, "beta1": 0.9, "beta2": 0.999,
                                                               "epsilon": 1e-6})
    n1, n2 = 0.9 * m1 + 0.1 * g, 0.999 * m2 + 0.001 * g * g
    rr = (n1 / (1 - 0.9)) / (np.sqrt(n2 / (1 - 0.999)) + 1e-6) + 0.01 * p
    trust = np.linalg.norm(p) / np.linalg.norm(rr)
    np.testing.assert_allclose(r["ParamOut"][0], p - 0.01 * trust * rr, rtol=1e-5)
    np.testing.assert_allclose(r["Beta1PowOut"][0], [0.81], rtol=1e-6)


def test_merged_adam_and_momentum_match_per_param():
    ps = [f32(3, 2), f32(4)]
    gs = [f32(3, 2), f32(4)]
    lr = np.float32([0.1])
    m1 = [np.zeros_like(p) for p in ps]
    m2 = [np.zeros_like(p) for p in ps]
    b1 = [np.float32([0.9]), np.float32([0.9])]
    b2 = [np.float32([0.999]), np.float32([0.999])]
    r = run_op("merged_adam", {"Param": ps, "Grad": gs, "LearningRate": [lr], "Moment1": m1, "Moment2": m2,
                               "Beta1Pow": b1, "Beta2Pow": b2},
               {"ParamOut": 2, "Moment1Out": 2, "Moment2Out": 2, "Beta1PowOut": 2, "Beta2PowOut": 2},
               {"beta1": 0.9, "beta2": 0.999, "epsilon": 1e-8})
    for i in range(2):
        mm1, mm2 = 0.1 * gs[i], 0.001 * gs[i] ** 2
        step = 0.1 * np.sqrt(1 - 0.999) / (1 - 0.9)
        ref = ps[i] - step * mm1 / (np.sqrt(mm2) + 1e-8 * np.sqrt(1 - 0.999))
        np.testing.assert_allclose(r["ParamOut"][i], ref, rtol=1e-5)
    vs = [np.zeros_like(p) for p in ps]
    r = run_op("merged_momentum", {"Param": ps, "Grad": gs, "Velocity": vs, "LearningRate": [lr]},
               {"ParamOut": 2, "VelocityOut": 2}, {"mu": 0.9})
    for i in range(2):
        np.testing.assert_allclose(r["ParamOut"][i], ps[i] - 0.1 * gs[i], rtol=1e-5)


# ------------------------------------------------------------------------------------ RNN ops
def test_lstm_unit_gru_unit_and_cudnn_lstm():
    x, cp = f32(3, 16), f32(3, 4)
    r = run_op("lstm_unit", {"X": x, "C_prev": cp}, {"C": 1, "H": 1}, {"forget_bias": 0.5})
    sig = lambda t: 1 / (1 + np.exp(-t))  # noqa: E731
    i, f, o, g = np.split(x, 4, 1)
    c = sig(f + 0.5) * cp + sig(i) * np.tanh(g)
    np.testing.assert_allclose(r["C"][0], c, rtol=1e-5)
    np.testing.assert_allclose(r["H"][0], sig(o) * np.tanh(c), rtol=1e-5)
    D = 4
    xi, hp, w, b = f32(3, 3 * D), f32(3, D), f32(D, 3 * D), f32(1, 3 * D)
    r = run_op("gru_unit", {"Input": xi, "HiddenPrev": hp, "Weight": w, "Bias": b}, {"Gate": 1, "ResetHiddenPrev": 1,
                                                                                       "Hidden": 1},
               {"gate_activation": 1, "activation": 2, "origin_mode": False})
    flat = w.reshape(-1)
    wur, wc = flat[:2 * D * D].reshape(D, 2 * D), flat[2 * D * D:].reshape(D, D)
    g = xi + b
    ur = sig(g[:, :2 * D] + hp @ wur)
    u, rr = ur[:, :D], ur[:, D:]
    cc = np.tanh(g[:, 2 * D:] + (rr * hp) @ wc)
    np.testing.assert_allclose(r["Hidden"][0], u * cc + (1 - u) * hp, rtol=1e-5, atol=1e-6)
    T, B, I, H = 5, 2, 3, 4
    xs = f32(T, B, I)
    lstm = torch.nn.LSTM(I, H)
    wl = [lstm.weight_ih_l0.detach().numpy(), lstm.weight_hh_l0.detach().numpy(),
          lstm.bias_ih_l0.detach().numpy(), lstm.bias_hh_l0.detach().numpy()]
    h0, c0 = f32(1, B, H), f32(1, B, H)
    r = run_op("cudnn_lstm", {"Input": xs, "InitH": h0, "InitC": c0, "WeightList": wl},
               {"Out": 1, "LastH": 1, "LastC": 1}, {"hidden_size": H, "num_layers": 1, "is_bidirec": False,
                                                    "is_test": True})
    ref, (hn, cn) = lstm(torch.from_numpy(xs), (torch.from_numpy(h0), torch.from_numpy(c0)))
    np.testing.assert_allclose(r["Out"][0], ref.detach().numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(r["LastC"][0], cn.detach().numpy(), rtol=1e-4, atol=1e-5)


def test_lstm_and_gru_ops_sequence():
    T, D = 6, 3
    sig = lambda t: 1 / (1 + np.exp(-t))  # noqa: E731
    xg, w, b = f32(T, 4 * D), f32(D, 4 * D), f32(1, 7 * D)
    r = run_op("lstm", {"Input": xg, "Weight": w, "Bias": b}, {"Hidden": 1, "Cell": 1},
               {"use_peepholes": True, "is_reverse": False, "gate_activation": "sigmoid", "cell_activation": "tanh",
                "candidate_activation": "tanh"})
    h, c = np.zeros((1, D)), np.zeros((1, D))
    bb = b.reshape(-1)
    for t in range(T):
        gg = xg[t:t + 1] + h @ w + bb[:4 * D]
        gc, gi, gf, go = np.split(gg, 4, 1)
        i = sig(gi + c * bb[4 * D:5 * D])
        f = sig(gf + c * bb[5 * D:6 * D])
        c = np.tanh(gc) * i + c * f
        o = sig(go + c * bb[6 * D:7 * D])
        h = o * np.tanh(c)
        np.testing.assert_allclose(r["Hidden"][0][t], h[0], rtol=1e-4, atol=1e-5)
    xg3, w3 = f32(T, 3 * D), f32(D, 3 * D)
    r = run_op("gru", {"Input": xg3, "Weight": w3}, {"Hidden": 1}, {"is_reverse": True, "origin_mode": True,
                                                                    "gate_activation": "sigmoid",
                                                                    "activation": "tanh"})
    flat = w3.reshape(-1)
    wur, wc = flat[:2 * D * D].reshape(D, 2 * D), flat[2 * D * D:].reshape(D, D)
    h = np.zeros((1, D))
    for t in reversed(range(T)):
        ur = sig(xg3[t:t + 1, :2 * D] + h @ wur)
        u, rr = ur[:, :D], ur[:, D:]
        cc = np.tanh(xg3[t:t + 1, 2 * D:] + (rr * h) @ wc)
        h = u * h + (1 - u) * cc
        np.testing.assert_allclose(r["Hidden"][0][t], h[0], rtol=1e-4, atol=1e-5)


# ----------------------------------------------------------------------------- fork serving ops
def test_weight_quantize_dequantize_linear2_number_count():
    w = f32(64, 32)
    r = run_op("weight_quantize", {"x": w}, {"out": 1, "scale": 1}, {"algo": "weight_only_int8"})
    q, s = r["out"][0], r["scale"][0]
    assert q.shape == (32, 64) and s.shape == (32,)
    deq = run_op("weight_dequantize", {"x": q, "scale": s}, {"out": 1}, {"algo": "weight_only_int8", "out_dtype": 5})
    np.testing.assert_allclose(deq["out"][0], w, atol=float(s.max()) * 0.51)
    x = f32(3, 64)
    y = run_op("weight_only_linear2", {"x": x, "weight": q, "weight_scale": s}, {"out": 1},
               {"m": 3, "n": 32, "k": 64, "weight_dtype": "int8", "act_method": "none"})["out"][0]
    np.testing.assert_allclose(y, x @ deq["out"][0], rtol=1e-4, atol=1e-4)
    ids = np.array([[0, 3], [3, -1], [7, 1]], "int64")
    np.testing.assert_array_equal(run_op("number_count_v2", {"numbers": ids}, {"out": 1}, {"upper_range": 4})["out"][0],
                                  [1, 1, 0, 2])


def test_flash_attn_unpadded_matches_dense_per_sequence():
    H, D = 2, 8
    lens = [3, 5]
    cu = np.array([0, 3, 8], "int32")
    q, k, v = f32(8, H, D), f32(8, H, D), f32(8, H, D)
    out = run_op("flash_attn_unpadded", {"q": q, "k": k, "v": v, "cu_seqlens_q": cu, "cu_seqlens_k": cu},
                 {"out": 1}, {"max_seqlen_q": 5, "max_seqlen_k": 5, "scale": 0.3, "causal": True,
                              "is_test": True})["out"][0]
    for b, (s0, s1) in enumerate([(0, 3), (3, 8)]):
        qs, ks, vs = (torch.from_numpy(t[s0:s1]).transpose(0, 1) for t in (q, k, v))
        sc = qs @ ks.transpose(-1, -2) * 0.3
        n = s1 - s0
        sc = sc.masked_fill(torch.triu(torch.ones(n, n, dtype=torch.bool), 1), -1e30)
        ref = (torch.softmax(sc, -1) @ vs).transpose(0, 1).numpy()
        np.testing.assert_allclose(out[s0:s1], ref, rtol=1e-4, atol=1e-5)
    del lens


def test_fused_moe_kernel_matches_composition():
    torch.manual_seed(0)
    B, S, Dm, Fd, E, k = 2, 3, 8, 16, 4, 2
    x = f32(B, S, Dm)
    gw, gb = f32(Dm, E), f32(E)
    lns, lnb = 1 + f32(Dm) * 0.1, f32(Dm) * 0.1
    w1 = [f32(Dm, Fd) for _ in range(E)]
    b1 = [f32(Fd) for _ in range(E)]
    w2 = [f32(Fd, Dm) for _ in range(E)]
    b2 = [f32(Dm) for _ in range(E)]
    for pre in (True, False):
        out = run_op("fused_moe_kernel", {"x": x, "gate_weight": gw, "gate_bias": gb, "ln_scale": lns, "ln_bias": lnb,
                                          "experts_weight1": w1, "experts_bias1": b1, "experts_weight2": w2,
                                          "experts_bias2": b2}, {"out": 1},
                     {"pre_layer_norm": pre, "ln_epsilon": 1e-5, "topk": k, "mp_size": 1, "mp_rank": 0,
                      "num_expert": E, "world_size": 1, "moe_ring_id": -1, "approximate": False})["out"][0]
        xt = torch.from_numpy(x).reshape(-1, Dm)
        h = F.layer_norm(xt, (Dm,), torch.from_numpy(lns), torch.from_numpy(lnb), 1e-5) if pre else xt
        lg = h @ torch.from_numpy(gw) + torch.from_numpy(gb)
        val, idx = torch.topk(lg, k, -1)
        y = torch.zeros_like(h)
        for t in range(h.shape[0]):
            for j in range(k):
                e = int(idx[t, j])
                ex = F.gelu(h[t] @ torch.from_numpy(w1[e]) + torch.from_numpy(b1[e])) @ torch.from_numpy(w2[e]) + \
                    torch.from_numpy(b2[e])
                y[t] += val[t, j] * ex
        ref = xt + y
        if not pre:
            ref = F.layer_norm(ref, (Dm,), torch.from_numpy(lns), torch.from_numpy(lnb), 1e-5)
        np.testing.assert_allclose(out, ref.reshape(B, S, Dm).numpy(), rtol=1e-4, atol=1e-5)


# --------------------------------------------------------------------------------- detection
def test_detection_ops_through_programs():
    from paddle_infer_amd.vision import ops as V
    bb = np.stack([np.concatenate([R.rand(10, 2) * 0.5, R.rand(10, 2) * 0.5 + 0.5], 1) for _ in range(2)]).astype("float32")
    sc = R.rand(2, 3, 10).astype("float32")
    r = run_op("matrix_nms", {"BBoxes": bb, "Scores": sc}, {"Out": 1, "Index": 1, "RoisNum": 1},
               {"score_threshold": 0.1, "post_threshold": 0.05, "nms_top_k": 5, "keep_top_k": 6,
                "background_label": 0, "normalized": True, "use_gaussian": False, "gaussian_sigma": 2.0})
    ref, num = V.matrix_nms(torch.from_numpy(bb), torch.from_numpy(sc), 0.1, 0.05, 5, 6)
    np.testing.assert_allclose(r["Out"][0], ref.numpy())
    np.testing.assert_array_equal(r["RoisNum"][0], num.numpy())
    x = f32(1, 8, 6, 6)
    rois = np.array([[0, 0, 4, 4], [1, 1, 5, 3]], "float32")
    out = run_op("psroi_pool", {"X": x, "ROIs": rois, "RoisNum": np.array([2], "int32")}, {"Out": 1},
                 {"output_channels": 2, "spatial_scale": 1.0, "pooled_height": 2, "pooled_width": 2})["Out"][0]
    np.testing.assert_allclose(out, V.psroi_pool(torch.from_numpy(x), torch.from_numpy(rois), torch.tensor([2]), 2).numpy())


# ------------------------------------------------------------------------- static collectives
def _coll_worker(rank, world):
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_program_ops_tail_cpu import run_op as run
    x = (np.arange(12, dtype="float32").reshape(4, 3) + 100 * rank)
    ag = run("c_allgather", {"X": x}, {"Out": 1}, {"ring_id": 0, "nranks": world})["Out"][0]
    rs = run("c_reducescatter", {"X": x}, {"Out": 1}, {"ring_id": 0, "nranks": world})["Out"][0]
    a2a = run("alltoall", {"X": x}, {"Out": 1}, {"ring_id": 0})["Out"][0]
    xb = (np.random.RandomState(rank).randn(4, 3, 2, 2) * 2 + 3).astype("float32")
    bn = run("sync_batch_norm", {"X": xb, "Scale": np.ones(3, "float32"), "Bias": np.zeros(3, "float32"),
                                 "Mean": np.zeros(3, "float32"), "Variance": np.ones(3, "float32")},
             {"Y": 1, "MeanOut": 1, "VarianceOut": 1}, {"is_test": False, "momentum": 0.9, "epsilon": 1e-5,
                                                        "data_layout": "NCHW", "ring_id": 0})
    return ag, rs, a2a, bn["Y"][0], xb


def test_static_collectives_on_two_ranks():
    from dist_utils import run_distributed
    res = run_distributed(_coll_worker, 2)
    xs = [np.arange(12, dtype="float32").reshape(4, 3) + 100 * r for r in range(2)]
    for r in range(2):
        ag, rs, a2a, y, _ = (np.asarray(t) for t in res[r])
        np.testing.assert_allclose(ag, np.concatenate(xs, 0))
        np.testing.assert_allclose(rs, (xs[0] + xs[1])[2 * r:2 * r + 2])
        np.testing.assert_allclose(a2a, np.concatenate([xs[0][2 * r:2 * r + 2], xs[1][2 * r:2 * r + 2]], 0))
    full = np.concatenate([np.asarray(res[r][4]) for r in range(2)], 0)
    mean = full.mean((0, 2, 3), keepdims=True)
    var = full.var((0, 2, 3), keepdims=True)
    ref = (full - mean) / np.sqrt(var + 1e-5)
    got = np.concatenate([np.asarray(res[r][3]) for r in range(2)], 0)
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4)
