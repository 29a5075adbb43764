"""Extended Paddle op set (`static/ops_registry_ext.py`) against NumPy / PyTorch references, Paddle
control flow (`while` / `conditional_block` sub-blocks) from a hand-built ProgramDesc, load-time
rejection of unknown op types, and the fork's LLM ops in program form vs their dygraph layers."""
import os
import sys

import numpy as np
import pytest
import torch

from paddle_infer_amd.static import proto
from paddle_infer_amd.static.ops_registry import REGISTRY

sys.path.insert(0, os.path.dirname(__file__))
from fmt_wire import _op, _var  # noqa: E402

A = proto.ATTR


def run(op, ins, attrs=None):
    return REGISTRY[op](ins, attrs or {})


def test_indexing_ops():
    x = torch.arange(24.).reshape(4, 6)
    torch.testing.assert_close(run("gather", {"X": [x], "Index": [torch.tensor([2, 0])]})["Out"], x[[2, 0]])
    torch.testing.assert_close(run("gather", {"X": [x], "Index": [torch.tensor([5, 1])]}, {"axis": 1})["Out"], x[:, [5, 1]])
    idx = torch.tensor([[1, 2], [3, 0]])
    torch.testing.assert_close(run("gather_nd", {"X": [x], "Index": [idx]})["Out"], x[[1, 3], [2, 0]])
    torch.testing.assert_close(run("gather_nd", {"X": [x], "Index": [torch.tensor([[2]])]})["Out"], x[[2]])
    torch.testing.assert_close(run("index_select", {"X": [x], "Index": [torch.tensor([4, 4])]}, {"dim": 1})["Out"], x[:, [4, 4]])
    torch.testing.assert_close(run("tril_triu", {"X": [x]}, {"diagonal": 1, "lower": False})["Out"], torch.triu(x, 1))
    torch.testing.assert_close(run("tril_triu", {"X": [x]}, {"diagonal": -1, "lower": True})["Out"], torch.tril(x, -1))


def test_set_value_variants():
    x = torch.zeros(4, 5)
    out = run("set_value", {"Input": [x]}, {"axes": [0, 1], "starts": [1, 0], "ends": [3, 5], "steps": [1, 2],
                                            "fp32_values": [7.0], "shape": [1]})["Out"]
    ref = x.clone()
    ref[1:3, 0:5:2] = 7.0
    torch.testing.assert_close(out, ref)
    v = torch.arange(5.)
    out = run("set_value", {"Input": [x], "ValueTensor": [v]}, {"axes": [0], "starts": [-1], "ends": [4],
                                                               "steps": [1], "decrease_axes": [0]})["Out"]
    ref = x.clone()
    ref[3] = v
    torch.testing.assert_close(out, ref)
    out = run("set_value", {"Input": [x], "StartsTensorList": [torch.tensor([4])],
                            "EndsTensorList": [torch.tensor([0])], "StepsTensorList": [torch.tensor([-2])]},
              {"axes": [1], "fp32_values": [1.0], "shape": [1]})["Out"]
    ref = x.clone()
    ref[:, [4, 2]] = 1.0  # columns 4:0:-2
    torch.testing.assert_close(out, ref)


def test_creation_and_math_ops():
    r = run("range", {"Start": [torch.tensor([2])], "End": [torch.tensor([11])], "Step": [torch.tensor([3])]})["Out"]
    assert r.tolist() == [2, 5, 8]
    x = torch.randn(3, 7)
    f = run("fill_constant_batch_size_like", {"Input": [x]}, {"shape": [-1, 4], "value": 2.5, "dtype": 5,
                                                              "input_dim_idx": 0, "output_dim_idx": 0})["Out"]
    assert f.shape == (3, 4) and float(f[0, 0]) == 2.5
    c = run("cumsum", {"X": [x]}, {"axis": 1, "exclusive": True, "reverse": True})["Out"]
    ref = torch.flip(torch.cumsum(torch.flip(x, [1]), 1), [1]) - x
    torch.testing.assert_close(c, ref)
    oh = run("one_hot_v2", {"X": [torch.tensor([[1], [3]])]}, {"depth": 4, "dtype": 5})["Out"]
    assert oh.shape == (2, 1, 4) and oh[1, 0, 3] == 1
    rs = run("reduce_sum", {"X": [x]}, {"dim": [1], "keep_dim": True})["Out"]
    torch.testing.assert_close(rs, x.sum(1, keepdim=True))
    rm = run("reduce_mean", {"X": [x]}, {"reduce_all": True})["Out"]
    torch.testing.assert_close(rm, x.mean())


def test_norm_and_interp_ops():
    x = torch.randn(2, 6, 5, 4)
    g, b = torch.rand(6) + 0.5, torch.randn(6)
    out = run("group_norm", {"X": [x], "Scale": [g], "Bias": [b]}, {"groups": 3, "epsilon": 1e-5})
    torch.testing.assert_close(out["Y"], torch.nn.functional.group_norm(x, 3, g, b, 1e-5))
    assert out["Mean"].shape == (2, 3)
    out = run("instance_norm", {"X": [x], "Scale": [g], "Bias": [b]}, {"epsilon": 1e-5})
    torch.testing.assert_close(out["Y"], torch.nn.functional.instance_norm(x, weight=g, bias=b, eps=1e-5))
    y = run("bilinear_interp_v2", {"X": [x]}, {"out_h": 10, "out_w": 8, "align_corners": False,
                                               "align_mode": 0})["Out"]
    torch.testing.assert_close(y, torch.nn.functional.interpolate(x, (10, 8), mode="bilinear", align_corners=False))
    y = run("nearest_interp_v2", {"X": [x]}, {"scale": [2.0, 2.0]})["Out"]
    assert y.shape == (2, 6, 10, 8)


def test_c_embedding_vocab_shard():
    w = torch.randn(5, 3)
    ids = torch.tensor([[4, 5, 9, 7]])
    out = run("c_embedding", {"W": [w], "Ids": [ids]}, {"start_index": 5})["Out"]
    ref = torch.zeros(1, 4, 3)
    ref[0, 1], ref[0, 2], ref[0, 3] = w[0], w[4], w[2]
    torch.testing.assert_close(out, ref)


def test_top_p_sampling_stays_in_nucleus():
    probs = torch.tensor([[0.5, 0.3, 0.15, 0.05]] * 64)
    out = run("top_p_sampling", {"x": [probs], "ps": [torch.full((64,), 0.7)]}, {"seed": 3})
    assert set(out["ids"].reshape(-1).tolist()) <= {0, 1}
    torch.testing.assert_close(out["out"], probs.gather(1, out["ids"]))


def test_fused_gemm_epilogue_cpu():
    x, y, b = torch.randn(4, 3, 8), torch.randn(16, 8), torch.randn(16)
    out = run("fused_gemm_epilogue", {"X": [x], "Y": [y], "Bias": [b]}, {"trans_y": True, "activation": "relu"})
    torch.testing.assert_close(out["Out"], torch.relu(x @ y.t() + b))


def _prog(blocks):
    return proto.encode("ProgramDesc", {"blocks": blocks, "version": {"version": 0}})


def test_paddle_while_and_conditional_block_programs():
    """i = 0; s = 0; while i < n: s += x; i += 1  — then  y = flag ? s * 2 : s + 1 (two
    conditional_blocks + select_input, the reference's lowering of ``cond``)."""
    from paddle_infer_amd import static
    from paddle_infer_amd.static.io import deserialize_program
    F, I64 = proto.VT["float32"], proto.VT["int64"]

    def fill(out, v, dt):
        return _op("fill_constant", {}, {"Out": [out]},
                   [{"name": "shape", "type": A["LONGS"], "longs": [1]},
                    {"name": "value", "type": A["FLOAT"], "f": float(v)},
                    {"name": "dtype", "type": A["INT"], "i": dt}])
    g_ops = [
        _op("feed", {"X": ["feed"]}, {"Out": ["x"]}, [{"name": "col", "type": A["INT"], "i": 0}]),
        _op("feed", {"X": ["feed"]}, {"Out": ["flag"]}, [{"name": "col", "type": A["INT"], "i": 1}]),
        fill("i", 0, I64), fill("n", 3, I64), fill("s", 0, F),
        _op("less_than", {"X": ["i"], "Y": ["n"]}, {"Out": ["c"]}),
        _op("while", {"X": ["x", "i", "n", "s"], "Condition": ["c"]}, {"Out": ["i", "s"], "StepScopes": ["ss"]},
            [{"name": "sub_block", "type": A["BLOCK"], "block_idx": 1},
             {"name": "is_test", "type": A["BOOLEAN"], "b": True}]),
        _op("logical_not", {"X": ["flag"]}, {"Out": ["nflag"]}),
        _op("conditional_block", {"Cond": ["flag"], "Input": ["s"]}, {"Out": ["ya"], "Scope": ["sa"]},
            [{"name": "sub_block", "type": A["BLOCK"], "block_idx": 2},
             {"name": "is_scalar_condition", "type": A["BOOLEAN"], "b": True}]),
        _op("conditional_block", {"Cond": ["nflag"], "Input": ["s"]}, {"Out": ["yb"], "Scope": ["sb"]},
            [{"name": "sub_block", "type": A["BLOCK"], "block_idx": 3},
             {"name": "is_scalar_condition", "type": A["BOOLEAN"], "b": True}]),
        _op("cast", {"X": ["flag"]}, {"Out": ["fi"]}, [{"name": "in_dtype", "type": A["INT"], "i": 0},
                                                      {"name": "out_dtype", "type": A["INT"], "i": 2}]),
        _op("select_input", {"X": ["yb", "ya"], "Mask": ["fi"]}, {"Out": ["y"]}),
        _op("fetch", {"X": ["y"]}, {"Out": ["fetch"]}, [{"name": "col", "type": A["INT"], "i": 0}]),
    ]
    body = [_op("elementwise_add", {"X": ["s"], "Y": ["x"]}, {"Out": ["s"]}, [{"name": "axis", "type": A["INT"], "i": -1}]),
            _op("increment", {"X": ["i"]}, {"Out": ["i"]}, [{"name": "step", "type": A["FLOAT"], "f": 1.0}]),
            _op("less_than", {"X": ["i"], "Y": ["n"]}, {"Out": ["c"]})]
    ba = [_op("scale", {"X": ["s"]}, {"Out": ["ya"]}, [{"name": "scale", "type": A["FLOAT"], "f": 2.0},
                                                       {"name": "bias", "type": A["FLOAT"], "f": 0.0}])]
    bb = [_op("scale", {"X": ["s"]}, {"Out": ["yb"]}, [{"name": "scale", "type": A["FLOAT"], "f": 1.0},
                                                       {"name": "bias", "type": A["FLOAT"], "f": 1.0}])]
    vars0 = [_var("x", [4]), _var("flag", [1], dt="bool"), _var("s", [1]), _var("i", [1], dt="int64")]
    data = _prog([{"idx": 0, "parent_idx": -1, "vars": vars0, "ops": g_ops},
                  {"idx": 1, "parent_idx": 0, "vars": [], "ops": body},
                  {"idx": 2, "parent_idx": 0, "vars": [], "ops": ba},
                  {"idx": 3, "parent_idx": 0, "vars": [], "ops": bb}])
    prog = deserialize_program(data)
    exe = static.Executor()
    x = np.arange(4, dtype=np.float32)
    for flag, ref in ((True, 3 * x * 2), (False, 3 * x + 1)):
        (y,) = exe.run(prog, feed={"x": x, "flag": np.array([flag])}, fetch_list=["y"])
        np.testing.assert_allclose(y, ref)


def test_unknown_op_rejected_at_load():
    from paddle_infer_amd.static.io import deserialize_program
    ops = [_op("feed", {"X": ["feed"]}, {"Out": ["x"]}, [{"name": "col", "type": A["INT"], "i": 0}]),
           _op("frobnicate_v9", {"X": ["x"]}, {"Out": ["y"]}),
           _op("fetch", {"X": ["y"]}, {"Out": ["fetch"]}, [{"name": "col", "type": A["INT"], "i": 0}])]
    with pytest.raises(NotImplementedError, match="frobnicate_v9"):
        deserialize_program(_prog([{"idx": 0, "parent_idx": -1, "vars": [_var("x", [1])], "ops": ops}]))


def test_beam_search_softmax_program_op_slots():
    from paddle_infer_amd.ops.search import beam_search_softmax
    torch.manual_seed(0)
    bs, beam, V, maxd = 2, 2, 11, 4
    logits = torch.randn(bs * beam, V)
    ins = {"logits": [logits], "cum_scores": [torch.zeros(bs * beam)],
           "sequence_lengths": [torch.zeros(bs * beam, dtype=torch.int32)],
           "stop_flags": [torch.zeros(bs * beam, dtype=torch.bool)],
           "end_ids": [torch.tensor([10], dtype=torch.int32)],
           "step_ids": [torch.zeros(bs * beam, dtype=torch.int32)],
           "last_cache_ids": [torch.zeros(bs * beam, maxd, dtype=torch.int32)],
           "last_beam_offsets": [torch.zeros(bs * beam, maxd, dtype=torch.int32)]}
    out = run("beam_search_softmax", ins, {"beam_size": beam, "max_seq_len": 0, "max_dec_len": maxd,
                                           "fuse_softmax": True, "early_stop": False})
    ref = beam_search_softmax(*(v[0] for v in ins.values()), beam, 0, maxd, True, False)
    for k, r in zip(("ids_this_time", "out_cum_scores", "parent_idx"), (ref[0], ref[1], ref[4])):
        torch.testing.assert_close(out[k], r)


def _fmt_layer_slots(layer, i, names):
    return {slot: [getattr(layer, attr)[i]] for slot, attr in names.items()}


def test_fused_multi_transformer_moe_program_op_matches_layer():
    from paddle_infer_amd.incubate.nn.layer.fused_transformer import FusedMultiTransformerMoe
    torch.manual_seed(0)
    E, H, Fd, ne, L = 32, 4, 64, 4, 2
    layer = FusedMultiTransformerMoe(E, E, H, Fd, num_expert=ne, top_k=2, num_layers=L)
    for p in layer.parameters():
        if p.dim() > 1:
            p.data.normal_(0, 0.05)
    x = torch.randn(2, 5, E)
    ref = layer(x, causal=True)
    ins = {"X": [x], "LnScale": list(layer.ln_scales), "LnBias": list(layer.ln_biases),
           "QKVW": list(layer.qkv_weights), "QKVBias": list(layer.qkv_biases),
           "OutLinearW": list(layer.linear_weights), "OutLinearBias": list(layer.linear_biases),
           "GateWeight": list(layer.gate_weights), "GateBias": list(layer.gate_biases),
           "FFNLnScale": list(layer.ffn_ln_scales), "FFNLnBias": list(layer.ffn_ln_biases),
           "ExpertWeight1": list(layer.expert_weights1), "ExpertBias1": list(layer.expert_biases1),
           "ExpertWeight2": list(layer.expert_weights2), "ExpertBias2": list(layer.expert_biases2)}
    out = run("fused_multi_transformer_moe", ins, {"num_expert": ne, "topk": 2, "approximate": True,
                                                   "pre_layer_norm": True, "epsilon": 1e-5,
                                                   "trans_qkvw": True, "causal": True,
                                                   "act_method": "gelu", "num_head": H})["Out"]
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)


def test_fused_multi_transformer_int8_program_op_matches_layer():
    from paddle_infer_amd.incubate.nn.layer.fused_transformer import (FusedMultiTransformer,
                                                                      FusedMultiTransformerINT8)
    torch.manual_seed(1)
    E, H, Fd, L = 64, 4, 128, 2
    fmt = FusedMultiTransformer(E, H, Fd, num_layers=L)
    for p in fmt.parameters():
        if p.dim() > 1:
            p.data.normal_(0, 0.05)
    q = FusedMultiTransformerINT8(E, H, Fd, num_layers=L).load_from_float(fmt)
    x = torch.randn(2, 6, E)
    ref = q(x, causal=True)
    ins = {"X": [x], "LnScale": list(q.ln_scales), "LnBias": list(q.ln_biases),
           "QKVW": list(q.qkv_weights), "QKVBias": list(q.qkv_biases),
           "OutLinearW": list(q.linear_weights), "OutLinearBias": list(q.linear_biases),
           "FFNLnScale": list(q.ffn_ln_scales), "FFNLnBias": list(q.ffn_ln_biases),
           "FFN1Weight": list(q.ffn1_weights), "FFN1Bias": list(q.ffn1_biases),
           "FFN2Weight": list(q.ffn2_weights), "FFN2Bias": list(q.ffn2_biases),
           "QKVOutScale": list(q.qkv_scales), "OutLinearOutScale": list(q.linear_scales),
           "FFN1OutScale": list(q.ffn1_scales), "FFN2OutScale": list(q.ffn2_scales)}
    out = run("fused_multi_transformer_int8", ins, {"pre_layer_norm": True, "epsilon": 1e-5,
                                                    "trans_qkvw": True, "causal": True, "num_head": H,
                                                    "act_method": "gelu"})["Out"]
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
