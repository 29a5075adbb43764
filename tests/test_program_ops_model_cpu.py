"""Program op types of exported / static-training models (`static/ops_registry_model.py`) against
literal transcriptions of the reference kernels, fp32 compositions and the reference's own unit-test
fixtures: quantize_linear / dequantize_linear (+ a QAT-style program through create_predictor, with
and without the weight-dequant fold onto the int8 weight-only GEMM), the fake-quant family,
fused_batch_norm_act, c_softmax_with_cross_entropy (+ grad, single rank and 2-rank gloo),
fused_gate_attention, beam_search (`test_beam_search_op.py` cases) and beam_search_decode
(`test_beam_search_decode_op.py`)."""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from paddle_infer_amd.static.grad_kernels import GRAD_KERNELS
from paddle_infer_amd.static.ops_registry import REGISTRY
from paddle_infer_amd.static import proto

torch.manual_seed(0)


# ----------------------------------------------------------------------------- quantization
def _np_quant(x, s, bits, round_type):
    b = 2 ** (bits - 1) - 1
    if round_type == 0:
        q = np.round(b * x / s)  # numpy rounds half to even
        return np.clip(q, -b - 1, b)
    v = np.clip(x, -s, s) * b / s
    return np.sign(v) * np.floor(np.abs(v) + 0.5)


@pytest.mark.parametrize("round_type", [0, 1])
@pytest.mark.parametrize("axis", [-1, 0, 1])
def test_quantize_dequantize_linear(round_type, axis):
    x = torch.randn(6, 8) * 3
    x[0, 0] = 2.5 * (4.0 / 127)  # a tie on the grid
    if axis < 0:
        s = torch.tensor([4.0])
        sv = 4.0
    else:
        s = x.abs().amax(dim=1 - axis) * 0.8
        sv = s.numpy().reshape([-1 if d == axis else 1 for d in range(2)])
    a = {"quant_axis": axis, "bit_length": 8, "round_type": round_type, "is_test": True}
    y = REGISTRY["quantize_linear"]({"X": [x], "Scale": [s]}, a)["Y"]
    ref = _np_quant(x.numpy(), sv, 8, round_type)
    np.testing.assert_array_equal(y.numpy(), ref)
    d = REGISTRY["dequantize_linear"]({"X": [y.to(torch.int8)], "Scale": [s]}, a)["Y"]
    np.testing.assert_allclose(d.numpy(), ref * sv / 127.0, rtol=1e-6, atol=1e-7)


def test_quantize_linear_training_scales():
    x = torch.randn(4, 5)
    a = {"quant_axis": -1, "bit_length": 8, "is_test": False, "moving_rate": 0.9}
    st, ac = torch.tensor([2.0]), torch.tensor([3.0])
    out = REGISTRY["quantize_linear"]({"X": [x], "Scale": [torch.tensor([1.0])], "InState": [st],
                                       "InAccum": [ac]}, a)
    state = 0.9 * 2.0 + 1
    accum = 0.9 * 3.0 + x.abs().max().item()
    assert out["OutState"].item() == pytest.approx(state)
    assert out["OutAccum"].item() == pytest.approx(accum)
    assert out["OutScale"].item() == pytest.approx(accum / state)
    ch = REGISTRY["quantize_linear"]({"X": [x], "Scale": [torch.ones(4)]},
                                     {"quant_axis": 0, "is_test": False})
    torch.testing.assert_close(ch["OutScale"], x.abs().amax(1))


def test_fake_quant_family():
    x = torch.randn(3, 7)
    s = x.abs().max()
    out = REGISTRY["fake_quantize_dequantize_abs_max"]({"X": [x]}, {"bit_length": 8})
    q = _np_quant(x.numpy(), s.item(), 8, 1)
    np.testing.assert_allclose(out["Out"].numpy(), q * s.item() / 127, rtol=1e-6, atol=1e-7)
    out = REGISTRY["fake_channel_wise_quantize_dequantize_abs_max"]({"X": [x]}, {"quant_axis": 0})
    sc = x.abs().amax(1, keepdim=True).numpy()
    np.testing.assert_allclose(out["Out"].numpy(), _np_quant(x.numpy(), sc, 8, 1) * sc / 127, rtol=1e-6,
                               atol=1e-7)
    w = torch.randint(-127, 128, (4, 6)).float()
    sc = torch.rand(4) + 0.5
    o = REGISTRY["fake_channel_wise_dequantize_max_abs"]({"X": [w], "Scales": [sc]},
                                                         {"quant_bits": [8], "quant_axis": 0})["Out"]
    torch.testing.assert_close(o, w * sc[:, None] / 127)


def _op(t, ins, outs, attrs=()):
    return {"type": t, "inputs": [{"parameter": k, "arguments": v} for k, v in ins.items()],
            "outputs": [{"parameter": k, "arguments": v} for k, v in outs.items()], "attrs": list(attrs)}


def _var(n, dims, persistable=False, dt="float32"):
    return {"name": n, "type": {"type": proto.VT_LOD_TENSOR, "lod_tensor": {
        "tensor": {"data_type": proto.VT[dt], "dims": dims}, "lod_level": 0}}, "persistable": persistable}


def write_qat_program(prefix, K=128, N=96, fc=False, seed=0):
    """feed x [-1, K] → quantize_linear / dequantize_linear (activation, per tensor) → matmul_v2 (or
    fc + bias + relu) with Y = dequantize_linear(int8 W [K, N], per-output-channel scales) → fetch."""
    A = proto.ATTR
    rs = np.random.RandomState(seed)
    w_q = rs.randint(-127, 128, size=(K, N)).astype(np.int8)
    w_s = (rs.rand(N).astype(np.float32) + 0.5) * 0.2
    x_s = np.array([3.0], np.float32)
    bias = (rs.randn(N) * 0.1).astype(np.float32)
    params = {"w": (w_q, "int8"), "w_scale": (w_s, "float32"), "x_scale": (x_s, "float32")}
    if fc:
        params["b"] = (bias, "float32")
    q_attr = [{"name": "quant_axis", "type": A["INT"], "i": -1}, {"name": "bit_length", "type": A["INT"], "i": 8},
              {"name": "round_type", "type": A["INT"], "i": 0}, {"name": "is_test", "type": A["BOOLEAN"], "b": True}]
    w_attr = [{"name": "quant_axis", "type": A["INT"], "i": 1}, {"name": "bit_length", "type": A["INT"], "i": 8}]
    vars_ = [_var("x", [-1, K]), _var("xq", [-1, K]), _var("xd", [-1, K]), _var("wd", [K, N]), _var("y", [-1, N]),
             _var("w", [K, N], True, "int8"), _var("w_scale", [N], True), _var("x_scale", [1], True)]
    ops = [_op("feed", {"X": ["feed"]}, {"Out": ["x"]}, [{"name": "col", "type": A["INT"], "i": 0}]),
           _op("quantize_linear", {"X": ["x"], "Scale": ["x_scale"]}, {"Y": ["xq"]}, q_attr),
           _op("dequantize_linear", {"X": ["xq"], "Scale": ["x_scale"]}, {"Y": ["xd"]}, q_attr),
           _op("dequantize_linear", {"X": ["w"], "Scale": ["w_scale"]}, {"Y": ["wd"]}, w_attr)]
    if fc:
        vars_.append(_var("b", [N], True))
        ops.append(_op("fc", {"Input": ["xd"], "W": ["wd"], "Bias": ["b"]}, {"Out": ["y"]},
                       [{"name": "in_num_col_dims", "type": A["INT"], "i": 1},
                        {"name": "activation_type", "type": A["STRING"], "s": "relu"}]))
    else:
        ops.append(_op("matmul_v2", {"X": ["xd"], "Y": ["wd"]}, {"Out": ["y"]},
                       [{"name": "trans_x", "type": A["BOOLEAN"], "b": False},
                        {"name": "trans_y", "type": A["BOOLEAN"], "b": False}]))
    ops.append(_op("fetch", {"X": ["y"]}, {"Out": ["fetch"]}, [{"name": "col", "type": A["INT"], "i": 0}]))
    desc = {"blocks": [{"idx": 0, "parent_idx": -1, "vars": vars_, "ops": ops}]}
    with open(prefix + ".pdmodel", "wb") as f:
        f.write(proto.encode("ProgramDesc", desc))
    with open(prefix + ".pdiparams", "wb") as f:
        for n in sorted(params):
            arr, dt = params[n]
            f.write(proto.tensor_to_stream(np.ascontiguousarray(arr), proto.VT[dt]))

    def ref(x):
        xq = np.clip(np.round(127 * x / x_s[0]), -128, 127) * x_s[0] / 127
        y = xq @ (w_q.astype(np.float32) * w_s[None, :] / 127)
        if fc:
            y = np.maximum(y + bias, 0)
        return y
    return ref


@pytest.mark.parametrize("fc", [False, True])
@pytest.mark.parametrize("ir_optim", [False, True])
def test_qat_program_through_predictor(tmp_path, fc, ir_optim):
    from paddle_infer_amd import inference as pinf
    prefix = str(tmp_path / "qat")
    ref = write_qat_program(prefix, fc=fc)
    c = pinf.Config(prefix + ".pdmodel", prefix + ".pdiparams")
    c.disable_gpu()
    c.switch_ir_optim(ir_optim)
    p = pinf.create_predictor(c)
    x = np.random.RandomState(1).randn(5, 128).astype(np.float32)
    p.get_input_handle(p.get_input_names()[0]).copy_from_cpu(x)
    p.run()
    y = p.get_output_handle(p.get_output_names()[0]).copy_to_cpu()
    np.testing.assert_allclose(y, ref(x), rtol=1e-4, atol=1e-4)
    if ir_optim:
        types = [o.type for o in p._program.global_block().ops]
        assert "weight_only_linear" in types and "matmul_v2" not in types and "fc" not in types, types
        assert types.count("dequantize_linear") == 1  # the activation's stays


def test_weight_dequant_fold_conv(tmp_path):
    """A non-matmul consumer gets the dequantized float weight as a folded parameter."""
    from paddle_infer_amd.inference.passes import Graph
    from paddle_infer_amd.inference.passes_quant import delete_weight_dequant_linear_op_pass
    from paddle_infer_amd.static.framework import Program
    from paddle_infer_amd.inference.passes import _new
    prog = Program()
    b = prog.global_block()
    prog.params["w"] = torch.randint(-127, 128, (4, 3, 3, 3)).to(torch.int8)
    prog.params["s"] = torch.rand(4) + 0.5
    b.ops.append(_new(b, "dequantize_linear", {"X": ["w"], "Scale": ["s"]}, {"Y": ["wd"]},
                      {"quant_axis": 0, "bit_length": 8}))
    b.ops.append(_new(b, "conv2d", {"Input": ["x"], "Filter": ["wd"]}, {"Output": ["y"]}, {}))
    n = delete_weight_dequant_linear_op_pass(Graph(prog, ["y"]))
    assert n == 1 and [o.type for o in b.ops] == ["conv2d"]
    fold = b.ops[0].paddle_inputs["Filter"][0]
    torch.testing.assert_close(prog.params[fold], prog.params["w"].float() * prog.params["s"][:, None, None, None] / 127)


# ----------------------------------------------------------------------------- fused BN + act
def test_fused_batch_norm_act():
    x = torch.randn(4, 5, 6, 8)  # NHWC
    g, b = 1 + 0.1 * torch.randn(8), 0.1 * torch.randn(8)
    rm, rv = torch.zeros(8), torch.ones(8)
    out = REGISTRY["fused_batch_norm_act"]({"X": [x], "Scale": [g], "Bias": [b], "Mean": [rm], "Variance": [rv]},
                                           {"momentum": 0.9, "epsilon": 1e-5, "act_type": "relu"})
    xc = x.permute(0, 3, 1, 2)
    mu = xc.mean((0, 2, 3))
    var = xc.var((0, 2, 3), unbiased=False)
    ref = F.relu((x - mu) / torch.sqrt(var + 1e-5) * g + b)
    torch.testing.assert_close(out["Y"], ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out["SavedMean"], mu, rtol=1e-5, atol=1e-6)
    n = x.numel() // 8
    torch.testing.assert_close(out["MeanOut"], 0.1 * mu, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(out["VarianceOut"], 0.9 + 0.1 * var * n / (n - 1), rtol=1e-4, atol=1e-5)


# ----------------------------------------------------------------------------- vocab-parallel CE
def test_c_softmax_with_cross_entropy_single_rank():
    lg = torch.randn(6, 11)
    lab = torch.tensor([[1], [4], [10], [0], [-100], [7]])
    out = REGISTRY["c_softmax_with_cross_entropy"]({"Logits": [lg], "Label": [lab]},
                                                   {"ring_id": 0, "rank": 0, "nranks": 1, "ignore_index": -100})
    ref = F.cross_entropy(lg, lab.reshape(-1), ignore_index=-100, reduction="none")
    torch.testing.assert_close(out["Loss"].reshape(-1), ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(out["Softmax"], torch.softmax(lg, -1), rtol=1e-5, atol=1e-6)
    dl = torch.rand(6, 1)
    g = GRAD_KERNELS["c_softmax_with_cross_entropy_grad"](
        {"Softmax": [out["Softmax"]], "Label": [lab], "Loss@GRAD": [dl]},
        {"rank": 0, "nranks": 1, "ignore_index": -100})["Logits@GRAD"]
    x = lg.clone().requires_grad_()
    r = F.cross_entropy(x, lab.reshape(-1), ignore_index=-100, reduction="none")
    (rg,) = torch.autograd.grad(r, x, dl.reshape(-1))
    torch.testing.assert_close(g, rg, rtol=1e-5, atol=1e-6)


def _c_xent_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        lg = torch.randn(5, 12)
        lab = torch.tensor([[0], [5], [6], [11], [3]])
        V = 12 // world
        out = REGISTRY["c_softmax_with_cross_entropy"](
            {"Logits": [lg[:, rank * V:(rank + 1) * V].contiguous()], "Label": [lab]},
            {"ring_id": 0, "rank": rank, "nranks": world, "ignore_index": -100})
        g = GRAD_KERNELS["c_softmax_with_cross_entropy_grad"](
            {"Softmax": [out["Softmax"]], "Label": [lab], "Loss@GRAD": [torch.ones(5, 1)]},
            {"rank": rank, "nranks": world, "ignore_index": -100})["Logits@GRAD"]
        q.put((rank, out["Loss"].reshape(-1).numpy(), out["Softmax"].numpy(), g.numpy()))
    finally:
        dist.destroy_process_group()


def test_c_softmax_with_cross_entropy_two_ranks():
    import torch.multiprocessing as mp
    from dist_utils import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_c_xent_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (l, s, g)) for r, l, s, g in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(60)
    torch.manual_seed(0)
    lg = torch.randn(5, 12)
    lab = torch.tensor([0, 5, 6, 11, 3])
    ref = F.cross_entropy(lg, lab, reduction="none").numpy()
    x = lg.clone().requires_grad_()
    (rg,) = torch.autograd.grad(F.cross_entropy(x, lab, reduction="sum"), x)
    sm = torch.softmax(lg, -1).numpy()
    for r in range(2):
        np.testing.assert_allclose(res[r][0], ref, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(res[r][1], sm[:, r * 6:(r + 1) * 6], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(res[r][2], rg.numpy()[:, r * 6:(r + 1) * 6], rtol=1e-5, atol=1e-6)


# ----------------------------------------------------------------------------- gate attention
@pytest.mark.parametrize("merge_qkv", [True, False])
@pytest.mark.parametrize("has_gating", [True, False])
def test_fused_gate_attention(merge_qkv, has_gating):
    B, M, R, Qd, H, D = 1, 3, 5, 6, 2, 4
    rs = np.random.RandomState(123)
    t = lambda *s: torch.from_numpy(rs.random_sample(s).astype(np.float32))  # noqa: E731
    query = t(B, M, R, Qd)
    qw, kw, vw = t(Qd, H, D), t(Qd, H, D), t(Qd, H, D)
    key = query if merge_qkv else t(B, M, 7, Qd)
    mask = t(B, M, 1, 1, key.shape[2])
    nbias = t(B, 1, H, R, key.shape[2])
    gw, gb = t(Qd, H, D), t(H, D)
    ow, ob = t(H, D, Qd), t(Qd)
    ins = {"Query": [query], "SrcMask": [mask], "NonbatchedBias": [nbias], "OutLinearWeight": [ow],
           "OutLinearBias": [ob]}
    if merge_qkv:
        ins["QKVWeight"] = [torch.stack([w.permute(1, 2, 0) for w in (qw, kw, vw)])]
    else:
        ins.update(Key=[key], QueryWeight=[qw], KeyWeight=[kw], ValueWeight=[vw])
    if has_gating:
        ins.update(GateWeight=[gw], GateBias=[gb])
    out = REGISTRY["fused_gate_attention"](ins, {"merge_qkv": merge_qkv, "has_gating": has_gating})["Out"]
    # the reference test's composition (test_fused_gate_attention_op.py get_reference_out)
    q = torch.einsum("nbqa,ahc->nbqhc", query, qw) * D ** -0.5
    k = torch.einsum("nbka,ahc->nbkhc", key, kw)
    v = torch.einsum("nbka,ahc->nbkhc", key, vw)
    logits = torch.einsum("nbqhc,nbkhc->nbhqk", q, k) + mask + nbias
    fmha = torch.matmul(torch.softmax(logits, -1), v.permute(0, 1, 3, 2, 4)).permute(0, 1, 3, 2, 4)
    if has_gating:
        fmha = fmha * torch.sigmoid(torch.einsum("nbqc,chv->nbqhv", query, gw) + gb)
    ref = torch.einsum("nbqhc,hco->nbqo", fmha, ow) + ob
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)


# ----------------------------------------------------------------------------- beam search
def _lodt(arr, lod, dtype):
    t = torch.tensor(np.array(arr), dtype=dtype)
    t.lod = lod
    return t


_BS_CASES = [  # (pre_ids, pre_scores, ids, scores, lod, beam, accumulated, out_ids, out_scores, out_lod, parent)
    ([[1, 2, 3, 4]], [[0.1, 0.2, 0.3, 0.4]], [[4, 2, 5], [2, 1, 3], [3, 5, 2], [8, 2, 1]],
     [[0.5, 0.3, 0.2], [0.6, 0.3, 0.1], [0.9, 0.5, 0.1], [0.7, 0.5, 0.1]], [[0, 2, 4], [0, 1, 2, 3, 4]], 2, True,
     [4, 2, 3, 8], [0.5, 0.6, 0.9, 0.7], [[0, 2, 4], [0, 1, 2, 3, 4]], [0, 1, 2, 3]),
    ([[1], [2], [3], [4]], [[0.1, 0.2, 0.3, 0.4]], [[4, 2], [7, 3], [3, 5], [8, 1]],
     [[0.6, 0.9], [0.5, 0.3], [0.9, 0.5], [0.1, 0.7]], [[0, 2, 4], [0, 1, 2, 3, 4]], 2, True,
     [2, 4, 3, 1], [0.9, 0.6, 0.9, 0.7], [[0, 2, 4], [0, 2, 2, 3, 4]], [0, 0, 2, 3]),
    ([[1], [0], [0], [4]], [[0.1], [1.2], [0.5], [0.4]], [[4, 2], [7, 3], [3, 5], [8, 1]],
     [[0.6, 0.9], [0.5, 0.3], [0.9, 0.5], [0.6, 0.7]], [[0, 2, 4], [0, 1, 2, 3, 4]], 2, True,
     [2, 0, 1, 8], [0.9, 1.2, 0.7, 0.6], [[0, 2, 4], [0, 1, 2, 2, 4]], [0, 1, 3, 3]),
    ([[0], [0], [0], [4]], [[0.1], [1.2], [0.5], [0.4]], [[4, 2], [7, 3], [3, 5], [8, 1]],
     [[0.6, 0.9], [0.5, 0.3], [0.9, 0.5], [0.6, 0.7]], [[0, 2, 4], [0, 1, 2, 3, 4]], 2, True,
     [1, 8], [0.7, 0.6], [[0, 2, 4], [0, 0, 0, 0, 2]], [3, 3]),
    ([[1], [2], [3], [4]], [[0.1, 2.2, 0.3, 0.4]], [[4, 2], [7, 3], [3, 5], [8, 1]],
     [[0.6, 0.9], [0.5, 0.3], [0.9, 0.5], [0.1, 0.7]], [[0, 2, 4], [0, 1, 2, 3, 4]], 2, False,
     [7, 3, 3, 1], [1.50685, 0.996027, 0.194639, 0.043325], [[0, 2, 4], [0, 0, 2, 3, 4]], [1, 1, 2, 3]),
    ([[1], [2], [3], [4]], [[0.1, 0.2, 0.3, 0.4]], [[4, 2], [7, 3], [3, 5], [8, 1]],
     [[0.6, 0.9], [0.5, 0.3], [0.9, 0.5], [0.1, 0.7]], [[0, 1, 2, 3, 4], [0, 1, 2, 3, 4]], 1, True,
     [2, 7, 3, 1], [0.9, 0.5, 0.9, 0.7], [[0, 1, 2, 3, 4], [0, 1, 2, 3, 4]], [0, 1, 2, 3]),
]


@pytest.mark.parametrize("case", range(len(_BS_CASES)))
def test_beam_search_reference_cases(case):
    pi, ps, ids, sc, lod, beam, acc, oid, osc, olod, opar = _BS_CASES[case]
    out = REGISTRY["beam_search"]({"pre_ids": [_lodt(pi, None, torch.int64)],
                                   "pre_scores": [_lodt(ps, None, torch.float32)],
                                   "ids": [_lodt(ids, lod, torch.int64)], "scores": [_lodt(sc, lod, torch.float32)]},
                                  {"level": 0, "beam_size": beam, "end_id": 0, "is_accumulated": acc})
    np.testing.assert_array_equal(out["selected_ids"].numpy().reshape(-1), oid)
    np.testing.assert_allclose(out["selected_scores"].numpy().reshape(-1), osc, rtol=1e-5)
    assert out["selected_ids"].lod == olod and out["selected_scores"].lod == olod
    np.testing.assert_array_equal(out["parent_idx"].numpy(), opar)


def test_beam_search_decode_reference_case():
    steps = [([[0, 1, 2], [0, 1, 2]], [0, 0]), ([[0, 1, 2], [0, 2, 4]], [2, 3, 4, 5]),
             ([[0, 2, 4], [0, 2, 2, 4, 4]], [3, 1, 5, 4]), ([[0, 2, 4], [0, 1, 2, 3, 4]], [1, 1, 3, 5]),
             ([[0, 2, 4], [0, 0, 0, 2, 2]], [5, 1])]
    ids = [_lodt(v, lod, torch.int64) for lod, v in steps]
    scores = [_lodt(v, lod, torch.float32) for lod, v in steps]
    out = REGISTRY["beam_search_decode"]({"Ids": ids, "Scores": scores}, {"beam_size": 2, "end_id": 1})
    exp = np.array([0, 2, 3, 1, 0, 2, 1, 0, 4, 5, 3, 5, 0, 4, 5, 3, 1])
    assert out["SentenceIds"].lod == [[0, 2, 4], [0, 4, 7, 12, 17]]
    assert out["SentenceScores"].lod == [[0, 2, 4], [0, 4, 7, 12, 17]]
    np.testing.assert_array_equal(out["SentenceIds"].numpy(), exp)
    np.testing.assert_array_equal(out["SentenceScores"].numpy(), exp.astype(np.float32))


math  # noqa
