"""Inference API tests (CPU): Config / create_predictor / handles, IR fusion passes on a
Paddle-wire program (each pass rewrites and the output is unchanged), a Predictor over a model
saved by our own static graph, mixed-precision conversion, PredictorPool/clone.

Parity model: reference `python/paddle/fluid/tests/unittests/ir/inference/test_*_fuse_pass.py`
(each pass: build program, run with and without the pass, compare outputs) and
`test_inference_api.py`."""
import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import inference as pinf
from paddle_infer_amd import static
from paddle_infer_amd.static import proto

A = proto.ATTR


def _op(t, ins, outs, attrs=()):
    return {"type": t, "inputs": [{"parameter": k, "arguments": v} for k, v in ins.items()],
            "outputs": [{"parameter": k, "arguments": v} for k, v in outs.items()], "attrs": list(attrs)}


def _var(name, dims, persistable=False, dt="float32"):
    return {"name": name, "persistable": persistable,
            "type": {"type": proto.VT_LOD_TENSOR,
                     "lod_tensor": {"tensor": {"data_type": proto.VT[dt], "dims": dims}}}}


def _i(n, v):
    return {"name": n, "type": A["INT"], "i": v}


def _f(n, v):
    return {"name": n, "type": A["FLOAT"], "f": v}


def _b(n, v):
    return {"name": n, "type": A["BOOLEAN"], "b": v}


def _s(n, v):
    return {"name": n, "type": A["STRING"], "s": v}


def _ints(n, v):
    return {"name": n, "type": A["INTS"], "ints": list(v)}


def _build_bert_block(path):
    """emb(word)+emb(pos) → LN → fc(+gelu) → fc → residual add → LN → self-attention core
    → dropout(is_test) → scale(1) ; written with Paddle op types and slots."""
    E, F, V, P, H = 32, 64, 50, 16, 4
    D = E // H
    rng = np.random.RandomState(0)
    params = {
        "word_emb": rng.randn(V, E) * 0.1, "pos_emb": rng.randn(P, E) * 0.1,
        "ln0.g": 1 + rng.randn(E) * 0.1, "ln0.b": rng.randn(E) * 0.1,
        "fc1.w": rng.randn(E, F) * 0.1, "fc1.b": rng.randn(F) * 0.1,
        "fc2.w": rng.randn(F, E) * 0.1, "fc2.b": rng.randn(E) * 0.1,
        "ln1.g": 1 + rng.randn(E) * 0.1, "ln1.b": rng.randn(E) * 0.1,
    }
    ops = [
        _op("feed", {"X": ["feed"]}, {"Out": ["ids"]}, [_i("col", 0)]),
        _op("feed", {"X": ["feed"]}, {"Out": ["pos"]}, [_i("col", 1)]),
        _op("lookup_table_v2", {"Ids": ["ids"], "W": ["word_emb"]}, {"Out": ["e0"]}),
        _op("lookup_table_v2", {"Ids": ["pos"], "W": ["pos_emb"]}, {"Out": ["e1"]}),
        _op("elementwise_add", {"X": ["e0"], "Y": ["e1"]}, {"Out": ["e2"]}, [_i("axis", -1)]),
        _op("layer_norm", {"X": ["e2"], "Scale": ["ln0.g"], "Bias": ["ln0.b"]},
            {"Y": ["h0"], "Mean": ["m0"], "Variance": ["v0"]}, [_f("epsilon", 1e-5), _i("begin_norm_axis", 2)]),
        _op("matmul_v2", {"X": ["h0"], "Y": ["fc1.w"]}, {"Out": ["t0"]}, [_b("trans_x", False), _b("trans_y", False)]),
        _op("elementwise_add", {"X": ["t0"], "Y": ["fc1.b"]}, {"Out": ["t1"]}, [_i("axis", -1)]),
        _op("gelu", {"X": ["t1"]}, {"Out": ["t2"]}, [_b("approximate", False)]),
        _op("matmul_v2", {"X": ["t2"], "Y": ["fc2.w"]}, {"Out": ["t3"]}, [_b("trans_x", False), _b("trans_y", False)]),
        _op("elementwise_add", {"X": ["t3"], "Y": ["fc2.b"]}, {"Out": ["t4"]}, [_i("axis", -1)]),
        _op("elementwise_add", {"X": ["t4"], "Y": ["h0"]}, {"Out": ["t5"]}, [_i("axis", -1)]),
        _op("layer_norm", {"X": ["t5"], "Scale": ["ln1.g"], "Bias": ["ln1.b"]},
            {"Y": ["h1"], "Mean": ["m1"], "Variance": ["v1"]}, [_f("epsilon", 1e-5), _i("begin_norm_axis", 2)]),
        _op("reshape2", {"X": ["h1"]}, {"Out": ["r0"], "XShape": ["xs0"]}, [_ints("shape", [0, 0, H, D])]),
        _op("transpose2", {"X": ["r0"]}, {"Out": ["q"], "XShape": ["xs1"]}, [_ints("axis", [0, 2, 1, 3])]),
        _op("matmul_v2", {"X": ["q"], "Y": ["q"]}, {"Out": ["s0"]}, [_b("trans_x", False), _b("trans_y", True)]),
        _op("scale", {"X": ["s0"]}, {"Out": ["s1"]}, [_f("scale", D ** -0.5), _f("bias", 0.0), _b("bias_after_scale", True)]),
        _op("softmax", {"X": ["s1"]}, {"Out": ["p"]}, [_i("axis", -1)]),
        _op("matmul_v2", {"X": ["p"], "Y": ["q"]}, {"Out": ["o0"]}, [_b("trans_x", False), _b("trans_y", False)]),
        _op("dropout", {"X": ["o0"]}, {"Out": ["o1"], "Mask": ["mk"]},
            [_f("dropout_prob", 0.1), _b("is_test", True), _s("dropout_implementation", "upscale_in_train")]),
        _op("scale", {"X": ["o1"]}, {"Out": ["out"]}, [_f("scale", 1.0), _f("bias", 0.0), _b("bias_after_scale", True)]),
        _op("fetch", {"X": ["out"]}, {"Out": ["fetch"]}, [_i("col", 0)]),
    ]
    vars_ = [_var("ids", [-1, -1], dt="int64"), _var("pos", [-1, -1], dt="int64")]
    vars_ += [_var(n, list(v.shape), True) for n, v in params.items()]
    for n, s in [("e0", 3), ("e1", 3), ("e2", 3), ("h0", 3), ("t0", 3), ("t1", 3), ("t2", 3), ("t3", 3),
                 ("t4", 3), ("t5", 3), ("h1", 3), ("r0", 4), ("q", 4), ("s0", 4), ("s1", 4), ("p", 4),
                 ("o0", 4), ("o1", 4), ("out", 4)]:
        vars_.append(_var(n, [-1] * s))
    desc = {"blocks": [{"idx": 0, "parent_idx": -1, "vars": vars_, "ops": ops}]}
    open(path + ".pdmodel", "wb").write(proto.encode("ProgramDesc", desc))
    with open(path + ".pdiparams", "wb") as f:
        for n in sorted(params):
            f.write(proto.tensor_to_stream(params[n].astype("float32"), proto.VT["float32"]))


def _run(cfg, ids, pos):
    pred = pinf.create_predictor(cfg)
    names = pred.get_input_names()
    assert names == ["ids", "pos"]
    h = pred.get_input_handle("ids")
    h.reshape(ids.shape)
    h.copy_from_cpu(ids)
    pred.get_input_handle("pos").copy_from_cpu(pos)
    assert pred.run()
    out = pred.get_output_handle(pred.get_output_names()[0]).copy_to_cpu()
    return pred, out


def test_passes_rewrite_and_preserve_output(tmp_path):
    path = str(tmp_path / "bert")
    _build_bert_block(path)
    ids = np.random.RandomState(1).randint(0, 50, (2, 6)).astype("int64")
    pos = np.tile(np.arange(6), (2, 1)).astype("int64")
    cfg = pinf.Config(path + ".pdmodel", path + ".pdiparams")
    cfg.switch_ir_optim(False)
    _, ref = _run(cfg, ids, pos)
    cfg2 = pinf.Config(path + ".pdmodel", path + ".pdiparams")
    pred, got = _run(cfg2, ids, pos)
    st = pred.pass_stats
    for name in ("embedding_eltwise_layernorm_fuse_pass", "fc_fuse_pass", "fc_act_fuse_pass",
                 "self_attention_fuse_pass", "identity_scale_op_clean_pass"):
        assert st[name] >= 1, (name, st)
    # dropout(is_test) goes in simplify_with_basic_ops_pass (reference order), before delete_dropout
    assert st["simplify_with_basic_ops_pass"] + st["delete_dropout_op_pass"] >= 1, st
    # residual + LN after an fc: the reference's fc_elementwise_layernorm_fuse_pass takes it
    assert st["skip_layernorm_fuse_pass"] + st["fc_elementwise_layernorm_fuse_pass"] >= 1, st
    types = [o.type for o in pred.program.global_block().ops]
    assert "fused_embedding_eltwise_layernorm" in types and "fc" in types and \
        ("skip_layernorm" in types or "fused_fc_elementwise_layernorm" in types)
    assert "flash_attn" in types and "dropout" not in types
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)


def test_conv_bn_fuse_pass(tmp_path):
    rng = np.random.RandomState(2)
    params = {"w": rng.randn(4, 3, 3, 3).astype("float32"), "g": (1 + rng.rand(4)).astype("float32"),
              "b": rng.randn(4).astype("float32"), "m": rng.randn(4).astype("float32"),
              "v": (rng.rand(4) + 0.5).astype("float32")}
    ops = [_op("feed", {"X": ["feed"]}, {"Out": ["x"]}, [_i("col", 0)]),
           _op("conv2d", {"Input": ["x"], "Filter": ["w"]}, {"Output": ["c"]},
               [_ints("strides", [1, 1]), _ints("paddings", [1, 1]), _ints("dilations", [1, 1]), _i("groups", 1)]),
           _op("batch_norm", {"X": ["c"], "Scale": ["g"], "Bias": ["b"], "Mean": ["m"], "Variance": ["v"]},
               {"Y": ["y"]}, [_f("epsilon", 1e-5), _b("is_test", True)]),
           _op("relu", {"X": ["y"]}, {"Out": ["out"]}),
           _op("fetch", {"X": ["out"]}, {"Out": ["fetch"]}, [_i("col", 0)])]
    vars_ = [_var("x", [-1, 3, 8, 8])] + [_var(n, list(v.shape), True) for n, v in params.items()] + \
        [_var(n, [-1, 4, 8, 8]) for n in ("c", "y", "out")]
    path = str(tmp_path / "cbn")
    open(path + ".pdmodel", "wb").write(proto.encode("ProgramDesc", {"blocks": [{"idx": 0, "parent_idx": -1, "vars": vars_, "ops": ops}]}))
    with open(path + ".pdiparams", "wb") as f:
        for n in sorted(params):
            f.write(proto.tensor_to_stream(params[n], proto.VT["float32"]))
    x = rng.randn(2, 3, 8, 8).astype("float32")
    outs = []
    for opt in (False, True):
        cfg = pinf.Config(path + ".pdmodel", path + ".pdiparams")
        cfg.switch_ir_optim(opt)
        pred = pinf.create_predictor(cfg)
        outs.append(pred.run([torch.from_numpy(x)])[0].numpy())
        if opt:
            assert pred.pass_stats["conv_bn_fuse_pass"] == 1
            assert "batch_norm" not in [o.type for o in pred.program.global_block().ops]
    np.testing.assert_allclose(outs[1], outs[0], rtol=1e-4, atol=1e-5)


def test_predictor_on_static_saved_model_and_clone(tmp_path):
    paddle.enable_static()
    try:
        main, startup = static.Program(), static.Program()
        with static.program_guard(main, startup):
            x = static.data("x", [None, 8], "float32")
            h = static.nn.fc(x, 16, activation="relu")
            y = static.nn.fc(h, 4)
        exe = static.Executor(paddle.CPUPlace())
        exe.run(startup)
        X = np.random.RandomState(0).randn(3, 8).astype("float32")
        ref, = exe.run(main, feed={"x": X}, fetch_list=[y])
        prefix = str(tmp_path / "mlp" / "inference")
        static.save_inference_model(prefix, [x], [y], exe, program=main)
    finally:
        paddle.disable_static()
    cfg = pinf.Config(str(tmp_path / "mlp"))
    assert cfg.prog_file().endswith("inference.pdmodel")
    pred = pinf.create_predictor(cfg)
    out = pred.run([torch.from_numpy(X)])[0]
    np.testing.assert_allclose(out.numpy(), ref, rtol=1e-6)
    c = pred.clone()
    np.testing.assert_allclose(c.run([torch.from_numpy(X)])[0].numpy(), ref, rtol=1e-6)
    pool = pinf.PredictorPool(cfg, 2)
    np.testing.assert_allclose(pool.retrive(1).run([torch.from_numpy(X)])[0].numpy(), ref, rtol=1e-6)
    assert "hip_graph" in cfg.summary()


def test_convert_to_mixed_precision(tmp_path):
    path = str(tmp_path / "bert")
    _build_bert_block(path)
    pinf.convert_to_mixed_precision(path + ".pdmodel", path + ".pdiparams", path + "_bf16.pdmodel",
                                    path + "_bf16.pdiparams", pinf.PrecisionType.Bfloat16)
    prog = static.deserialize_program(open(path + "_bf16.pdmodel", "rb").read())
    with static.scope_guard(static.Scope()):
        static.deserialize_persistables(prog, open(path + "_bf16.pdiparams", "rb").read())
        assert prog.params["fc1.w"].dtype == torch.bfloat16


def _tiny_gpt(dtype="float32"):
    from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config
    paddle.seed(5)
    cfg = gpt_config("gpt3-tiny", dtype=dtype, hidden_dropout_prob=0.0, vocab_size=128,
                     max_position_embeddings=64)
    return GPTForPretraining(cfg).eval()


def test_gpt_generation_greedy_matches_full_recompute():
    from paddle_infer_amd.inference.generation import GPTGenerator
    m = _tiny_gpt()
    ids = torch.randint(0, 128, (2, 7))
    gen = GPTGenerator(m, max_batch=4, max_seq_len=32)
    out = gen.generate(ids, max_new_tokens=5)
    # reference: recompute the whole sequence each step, argmax of the last logits
    seq = ids.clone()
    with torch.no_grad():
        for _ in range(5):
            nxt = m(seq)[:, -1].argmax(-1)
            seq = torch.cat([seq, nxt[:, None]], 1)
    assert torch.equal(out, seq[:, 7:])


def test_gpt_generation_ragged_prompts_and_sampling_and_beam():
    from paddle_infer_amd.inference.generation import GPTGenerator
    m = _tiny_gpt()
    gen = GPTGenerator(m, max_batch=8, max_seq_len=32)
    ids = torch.randint(0, 128, (2, 6))
    lens = torch.tensor([6, 3])
    out = gen.generate(ids, lengths=lens, max_new_tokens=4)
    # the short prompt alone gives the same continuation
    solo = gen.generate(ids[1:2, :3], max_new_tokens=4)
    assert torch.equal(out[1], solo[0])
    s = gen.generate(ids, max_new_tokens=4, decode_strategy="sampling", top_k=5, top_p=0.9, seed=1)
    assert s.shape == (2, 4) and int(s.max()) < 128
    b = gen.generate(ids, max_new_tokens=4, num_beams=3)
    assert b.shape == (2, 4)
    # beam search's best beam scores at least as well as greedy
    g = gen.generate(ids, max_new_tokens=4)

    def logp(cont):
        seq = torch.cat([ids, cont], 1)
        with torch.no_grad():
            lp = torch.log_softmax(m(seq).float(), -1)
        return lp[:, 5:-1].gather(-1, seq[:, 6:, None]).sum((1, 2))
    assert bool((logp(b) >= logp(g) - 1e-4).all())


def test_traced_bert_predictor_symbolic_batch_and_epilogue_pass(tmp_path):
    """dygraph BERT → jit.save → Predictor: the export holds ONLY Paddle op types (recorded ops
    lowered to matmul_v2 / elementwise_add / layer_norm / split / flash_attn ...) with a symbolic
    batch dim; at load the IR passes fuse it back (fc + gelu epilogue GEMMs, skip_layernorm,
    packed flash attention); outputs match the dygraph model at two batch sizes."""
    from paddle_infer_amd import jit
    from paddle_infer_amd.models.bert import BertModel, bert_config
    from paddle_infer_amd.static import InputSpec
    torch.manual_seed(0)
    m = BertModel(bert_config("bert-tiny"))
    m.eval()
    st = jit.to_static(m, input_spec=[InputSpec([None, 16], "int64", "input_ids")])
    path = str(tmp_path / "bert")
    jit.save(st, path)
    from paddle_infer_amd.static.io import deserialize_program
    from paddle_infer_amd.static.ops_registry import REGISTRY
    with open(path + ".pdmodel", "rb") as f:
        saved = deserialize_program(f.read())
    saved_types = {o.type for o in saved.global_block().ops}
    assert all(o.func is None for o in saved.global_block().ops)  # no callables in the file
    assert saved_types <= set(REGISTRY), saved_types - set(REGISTRY)
    assert {"matmul_v2", "layer_norm", "flash_attn", "lookup_table_v2"} <= saved_types
    pred = pinf.create_predictor(pinf.Config(path + ".pdmodel", path + ".pdiparams"))
    st_ = pred.pass_stats
    assert st_["fc_act_fuse_pass"] >= 2 and st_["fc_fuse_pass"] >= 8
    assert st_["multihead_matmul_fuse_pass"] == 2 and st_["fc_elementwise_layernorm_fuse_pass"] == 4
    ops_after = [o.type for o in pred.program.global_block().ops]
    assert "gelu" not in ops_after and ops_after.count("multihead_matmul") == 2
    for B in (2, 5):
        ids = torch.randint(1, 1000, (B, 16))
        seq, pooled = m(ids)
        pred.get_input_handle("input_ids").copy_from_cpu(ids.numpy())
        assert pred.run()
        names = pred.get_output_names()
        np.testing.assert_allclose(pred.get_output_handle(names[0]).copy_to_cpu(),
                                   seq.detach().numpy(), rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(pred.get_output_handle(names[1]).copy_to_cpu(),
                                   pooled.detach().numpy(), rtol=1e-5, atol=1e-5)
