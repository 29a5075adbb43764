"""Paddle-wire programs (CPU): jit.save writes only Paddle op types; loading refuses callables off
the allowlist; fused_multi_transformer / multihead_matmul / fused_fc_elementwise_layernorm run
from their reference slots; the fused_multi_transformer encoder pass rewrites a plain-op GPT."""
import os
import sys

import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import inference as pinf
from paddle_infer_amd import jit
from paddle_infer_amd.static import InputSpec, proto
from paddle_infer_amd.static.io import deserialize_program

sys.path.insert(0, os.path.dirname(__file__))
from fmt_wire import _op, _var, write_fmt_program  # noqa: E402


@pytest.mark.parametrize("callable_name", ["os.system", "builtins.eval", "subprocess.call",
                                           "torch.load", "torch.hub.load", "pickle.loads",
                                           "paddle_infer_amd.framework.io.load"])
def test_pdmodel_rejects_callables_off_the_allowlist(callable_name):
    A = proto.ATTR
    ops = [_op("feed", {"X": ["feed"]}, {"Out": ["x"]}, [{"name": "col", "type": A["INT"], "i": 0}]),
           _op("torch_op", {"X": ["x"]}, {"Out": ["y"]},
               [{"name": "op_callable", "type": A["STRING"], "s": callable_name},
                {"name": "op_spec", "type": A["STRING"],
                 "s": '{"args": ["echo pwned"], "kwargs": {"$d": {}}, "outputs": {"$v": "y"}}'}]),
           _op("fetch", {"X": ["y"]}, {"Out": ["fetch"]}, [{"name": "col", "type": A["INT"], "i": 0}])]
    desc = {"blocks": [{"idx": 0, "parent_idx": -1, "vars": [_var("x", [1]), _var("y", [1])], "ops": ops}]}
    with pytest.raises(ValueError, match="not an allowed operator"):
        deserialize_program(proto.encode("ProgramDesc", desc))


def test_allowlisted_callable_still_loads():
    A = proto.ATTR
    ops = [_op("feed", {"X": ["feed"]}, {"Out": ["x"]}, [{"name": "col", "type": A["INT"], "i": 0}]),
           _op("relu", {"X": ["x"]}, {"Out": ["y"]},
               [{"name": "op_callable", "type": A["STRING"], "s": "torch.relu"},
                {"name": "op_spec", "type": A["STRING"],
                 "s": '{"args": [{"$v": "x"}], "kwargs": {"$d": {}}, "outputs": {"$v": "y"}}'}]),
           _op("fetch", {"X": ["y"]}, {"Out": ["fetch"]}, [{"name": "col", "type": A["INT"], "i": 0}])]
    desc = {"blocks": [{"idx": 0, "parent_idx": -1, "vars": [_var("x", [3]), _var("y", [3])], "ops": ops}]}
    prog = deserialize_program(proto.encode("ProgramDesc", desc))
    assert prog.global_block().ops[0].func is torch.relu


def test_jit_save_refuses_unlowerable_op_unless_allowed(tmp_path):
    class Net(paddle.nn.Layer):
        def forward(self, x):
            return torch.special.erfcx(x)  # no Paddle op
    with pytest.raises(ValueError, match="no Paddle op lowering"):
        jit.save(Net(), str(tmp_path / "a"), input_spec=[InputSpec([None, 4], "float32", "x")])
    jit.save(Net(), str(tmp_path / "b"), input_spec=[InputSpec([None, 4], "float32", "x")],
             allow_custom_ops=True)
    loaded = jit.load(str(tmp_path / "b"))
    x = torch.rand(2, 4)
    torch.testing.assert_close(loaded(x), torch.special.erfcx(x))


def test_gpt_export_rewritten_by_fused_multi_transformer_pass(tmp_path):
    """Plain-op GPT program (jit.save lowering) → fused_multi_transformer_encoder_traced_pass rewrites each
    pre-LN causal layer, fuse_multi_transformer_layer_pass merges them into ONE op; logits match."""
    from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config
    torch.manual_seed(0)
    m = GPTForPretraining(gpt_config("gpt3-tiny", hidden_size=64, num_heads=2, num_layers=3,
                                     vocab_size=128))
    m.eval()
    path = str(tmp_path / "gpt")
    jit.save(jit.to_static(m, input_spec=[InputSpec([None, 16], "int64", "ids")]), path)
    pred = pinf.create_predictor(pinf.Config(path + ".pdmodel", path + ".pdiparams"))
    st = pred.pass_stats
    assert st["fused_multi_transformer_encoder_traced_pass"] == 3, st
    assert st["fuse_multi_transformer_layer_pass"] == 2, st
    fmt = [o for o in pred.program.global_block().ops if o.type == "fused_multi_transformer"]
    assert len(fmt) == 1 and len(fmt[0].paddle_inputs["QKVW"]) == 3
    ids = torch.randint(0, 128, (2, 16))
    ref = m(ids)
    ref = ref[0] if isinstance(ref, (tuple, list)) else ref
    pred.get_input_handle("ids").copy_from_cpu(ids.numpy())
    assert pred.run()
    got = pred.get_output_handle(pred.get_output_names()[0]).to_torch().float()
    tol = 2e-4 if ref.dtype == torch.float32 else 3e-2
    torch.testing.assert_close(got, ref.detach().float(), rtol=tol, atol=tol)


def run_fmt_wire(tmp_path, device):
    """Context (prompt) + two decode steps of a hand-built fused_multi_transformer ProgramDesc via
    create_predictor vs the dygraph FusedMultiTransformer with the same weights and caches."""
    from paddle_infer_amd.incubate.nn import FusedMultiTransformer
    torch.manual_seed(0)
    E, H, L, B, S, MAXS = (64, 4, 2, 2, 8, 16) if device == "cpu" else (256, 4, 2, 2, 8, 16)
    layer = FusedMultiTransformer(E, H, 2 * E, num_layers=L)
    layer.eval()
    ctx_p, dec_p = str(tmp_path / "ctx"), str(tmp_path / "dec")
    write_fmt_program(layer, ctx_p, False, L, E)
    write_fmt_program(layer, dec_p, True, L, E)
    dt = torch.float32 if device == "cpu" else torch.bfloat16

    def make(prefix):
        c = pinf.Config(prefix + ".pdmodel", prefix + ".pdiparams")
        if device != "cpu":
            c.enable_use_gpu(256, 0)
            c.exp_enable_mixed_precision(pinf.PrecisionType.Bfloat16)
        return pinf.create_predictor(c)
    pc, pd = make(ctx_p), make(dec_p)
    dev = torch.device(device)
    ref_layer = layer.to(dev)
    if dt != torch.float32:
        ref_layer._amp_decorate("bfloat16")
        for lst in (ref_layer.ln_scales, ref_layer.ln_biases, ref_layer.ffn_ln_scales, ref_layer.ffn_ln_biases):
            for p in lst:
                p.data = p.data.to(dt)
    caches = ref_layer.gen_cache(B, MAXS, dtype=dt, device=dev)
    caches_p = [torch.zeros_like(c) for c in caches]
    x = torch.randn(B, S, E, device=dev).to(dt)
    ref, _ = ref_layer(x, caches=caches, causal=True)
    h = pc.get_input_handle("x")
    h.share_external_data(x)
    for i, c in enumerate(caches_p):
        pc.get_input_handle(f"cache_kv.{i}").share_external_data(c)
    assert pc.run()
    got = pc.get_output_handle("out").to_torch()
    tol = 2e-4 if dt == torch.float32 else 6e-2
    torch.testing.assert_close(got.float(), ref.float(), rtol=tol, atol=tol)
    for c, cp in zip(caches, caches_p):
        torch.testing.assert_close(cp[:, :, :, :S].float(), c[:, :, :, :S].float(), rtol=tol, atol=tol)
    for t in range(S, S + 2):
        xt = torch.randn(B, 1, E, device=dev).to(dt)
        ts = torch.tensor([t], dtype=torch.int32)
        ref_t, _ = ref_layer(xt, caches=caches, time_step=ts)
        pd.get_input_handle("x").share_external_data(xt)
        for i, c in enumerate(caches_p):
            pd.get_input_handle(f"cache_kv.{i}").share_external_data(c)
        pd.get_input_handle("time_step").copy_from_cpu(ts.numpy())
        assert pd.run()
        torch.testing.assert_close(pd.get_output_handle("out").to_torch().float(), ref_t.float(),
                                   rtol=tol, atol=tol)


def test_fused_multi_transformer_wire_program_context_and_decode(tmp_path):
    run_fmt_wire(tmp_path, "cpu")


def test_multihead_matmul_and_fc_eltwise_ln_ops_match_reference():
    from paddle_infer_amd.static.ops_registry import REGISTRY
    torch.manual_seed(0)
    B, S, E, H = 2, 5, 32, 4
    x = torch.randn(B, S, E)
    w = torch.randn(E, 3, E) * 0.1
    b = torch.randn(3, E) * 0.1
    mask = torch.randn(B, 1, S, S)
    out = REGISTRY["multihead_matmul"]({"Input": [x], "W": [w], "Bias": [b], "BiasQK": [mask]},
                                       {"head_number": H, "alpha": 0.25})["Out"]
    qkv = (x @ w.reshape(E, 3 * E) + b.reshape(-1)).reshape(B, S, 3, H, E // H)
    q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))
    p = torch.softmax(q @ k.transpose(-1, -2) * 0.25 + mask, -1)
    ref = (p @ v).transpose(1, 2).reshape(B, S, E)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
    W, b0, y = torch.randn(E, E) * 0.1, torch.randn(E), torch.randn(B, S, E)
    g, b1 = torch.rand(E) + 0.5, torch.randn(E)
    out = REGISTRY["fused_fc_elementwise_layernorm"](
        {"X": [x], "W": [W], "Bias0": [b0], "Y": [y], "Scale": [g], "Bias1": [b1]},
        {"x_num_col_dims": 2, "epsilon": 1e-5})["Out"]
    ref = torch.nn.functional.layer_norm(x @ W + b0 + y, (E,), g, b1, 1e-5)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
