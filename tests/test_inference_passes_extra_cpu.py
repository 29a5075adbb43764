"""The rest of the reference GPU IR pass list (`inference/passes_extra.py`), the reference
`ir/inference/test_*_fuse_pass.py` way: build a Paddle-wire program, run the Predictor with and
without IR optimisation, assert the pass fired (op types / pass_stats) and the outputs match."""
import numpy as np
import pytest
import torch

from paddle_infer_amd import inference as pinf
from paddle_infer_amd.static import proto

A = proto.ATTR


def _op(t, ins, outs, attrs=()):
    return {"type": t, "inputs": [{"parameter": k, "arguments": v} for k, v in ins.items()],
            "outputs": [{"parameter": k, "arguments": v} for k, v in outs.items()], "attrs": list(attrs)}


def _var(name, dims, persistable=False, dt="float32"):
    return {"name": name, "persistable": persistable,
            "type": {"type": proto.VT_LOD_TENSOR, "lod_tensor": {"tensor": {"data_type": proto.VT[dt], "dims": dims}}}}


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


CONV_ATTRS = [_ints("strides", [1, 1]), _ints("paddings", [1, 1]), _ints("dilations", [1, 1]), _i("groups", 1)]


def _save(tmp_path, name, ops, feeds, params, act_vars):
    """feeds: {name: dims}; act_vars: {name: rank} of intermediates (symbolic dims)."""
    ops = [_op("feed", {"X": ["feed"]}, {"Out": [n]}, [_i("col", i)]) for i, n in enumerate(feeds)] + ops
    vars_ = [_var(n, d) for n, d in feeds.items()] + [_var(n, list(v.shape), True) for n, v in params.items()]
    vars_ += [_var(n, [-1] * r) for n, r in act_vars.items()]
    path = str(tmp_path / name)
    open(path + ".pdmodel", "wb").write(proto.encode("ProgramDesc", {"blocks": [{"idx": 0, "parent_idx": -1, "vars": vars_, "ops": ops}]}))
    with open(path + ".pdiparams", "wb") as f:
        for n in sorted(params):
            f.write(proto.tensor_to_stream(params[n].astype("float32"), proto.VT["float32"]))
    return path


def _both(path, inputs):
    outs, preds = [], []
    for opt in (False, True):
        cfg = pinf.Config(path + ".pdmodel", path + ".pdiparams")
        cfg.switch_ir_optim(opt)
        pred = pinf.create_predictor(cfg)
        outs.append(pred.run([torch.from_numpy(x) for x in inputs])[0].numpy())
        preds.append(pred)
    np.testing.assert_allclose(outs[1], outs[0], rtol=1e-4, atol=1e-5)
    return preds[1]


def _types(pred):
    return [o.type for o in pred.program.global_block().ops]


rng = np.random.RandomState(0)


@pytest.mark.parametrize("act", ["relu", "sigmoid"])
def test_conv_elementwise_add_act_fuse(tmp_path, act):
    P = {"w": rng.randn(8, 4, 3, 3) * 0.2, "b": rng.randn(8)}
    ops = [_op("conv2d", {"Input": ["x"], "Filter": ["w"]}, {"Output": ["c"]}, CONV_ATTRS),
           _op("elementwise_add", {"X": ["c"], "Y": ["b"]}, {"Out": ["a"]}, [_i("axis", 1)]),
           _op(act, {"X": ["a"]}, {"Out": ["out"]}),
           _op("fetch", {"X": ["out"]}, {"Out": ["fetch"]}, [_i("col", 0)])]
    path = _save(tmp_path, "cea", ops, {"x": [-1, 4, 8, 8]}, P, {"c": 4, "a": 4, "out": 4})
    pred = _both(path, [rng.randn(2, 4, 8, 8).astype("float32")])
    assert pred.pass_stats["conv_elementwise_add_act_fuse_pass"] == 1
    assert _types(pred) == ["conv2d_fusion"]


def test_conv_elementwise_add2_act_fuse(tmp_path):
    P = {"w": rng.randn(4, 4, 3, 3) * 0.2, "b": rng.randn(4)}
    ops = [_op("conv2d", {"Input": ["x"], "Filter": ["w"]}, {"Output": ["c"]}, CONV_ATTRS),
           _op("elementwise_add", {"X": ["c"], "Y": ["b"]}, {"Out": ["a"]}, [_i("axis", 1)]),
           _op("elementwise_add", {"X": ["a"], "Y": ["x"]}, {"Out": ["r"]}, [_i("axis", -1)]),
           _op("relu", {"X": ["r"]}, {"Out": ["out"]}),
           _op("fetch", {"X": ["out"]}, {"Out": ["fetch"]}, [_i("col", 0)])]
    path = _save(tmp_path, "cea2", ops, {"x": [-1, 4, 8, 8]}, P, {"c": 4, "a": 4, "r": 4, "out": 4})
    pred = _both(path, [rng.randn(2, 4, 8, 8).astype("float32")])
    assert pred.pass_stats["conv_elementwise_add2_act_fuse_pass"] == 1
    assert _types(pred) == ["conv2d_fusion"]


def test_conv_eltwiseadd_bn_and_plain_bias_fuse(tmp_path):
    P = {"w": rng.randn(6, 3, 3, 3) * 0.2, "b": rng.randn(6), "g": 1 + rng.rand(6), "be": rng.randn(6),
         "m": rng.randn(6), "v": rng.rand(6) + 0.5, "w2": rng.randn(6, 6, 3, 3) * 0.2, "b2": rng.randn(6)}
    ops = [_op("conv2d", {"Input": ["x"], "Filter": ["w"]}, {"Output": ["c"]}, CONV_ATTRS),
           _op("elementwise_add", {"X": ["c"], "Y": ["b"]}, {"Out": ["a"]}, [_i("axis", 1)]),
           _op("batch_norm", {"X": ["a"], "Scale": ["g"], "Bias": ["be"], "Mean": ["m"], "Variance": ["v"]},
               {"Y": ["y"]}, [_f("epsilon", 1e-5), _b("is_test", True)]),
           _op("conv2d", {"Input": ["y"], "Filter": ["w2"]}, {"Output": ["c2"]}, CONV_ATTRS),
           _op("elementwise_add", {"X": ["c2"], "Y": ["b2"]}, {"Out": ["out"]}, [_i("axis", 1)]),
           _op("fetch", {"X": ["out"]}, {"Out": ["fetch"]}, [_i("col", 0)])]
    path = _save(tmp_path, "ceb", ops, {"x": [-1, 3, 8, 8]}, P, {"c": 4, "a": 4, "y": 4, "c2": 4, "out": 4})
    pred = _both(path, [rng.randn(2, 3, 8, 8).astype("float32")])
    st = pred.pass_stats
    assert st["conv_eltwiseadd_bn_fuse_pass"] == 1 and st["conv_elementwise_add_fuse_pass"] == 1, st
    assert _types(pred) == ["conv2d", "conv2d"]


@pytest.mark.parametrize("shape_op", ["squeeze2", "reshape2", "flatten2"])
def test_shape_op_matmul_to_fc(tmp_path, shape_op):
    P = {"w": rng.randn(16, 5) * 0.2, "b": rng.randn(5)}
    attrs = {"squeeze2": [_ints("axes", [2, 3])], "reshape2": [_ints("shape", [0, 16])],
             "flatten2": [_i("axis", 1)]}[shape_op]
    ops = [_op(shape_op, {"X": ["x"]}, {"Out": ["f"], "XShape": ["xs"]}, attrs),
           _op("matmul_v2", {"X": ["f"], "Y": ["w"]}, {"Out": ["t"]}, [_b("trans_x", False), _b("trans_y", False)]),
           _op("elementwise_add", {"X": ["t"], "Y": ["b"]}, {"Out": ["out"]}, [_i("axis", -1)]),
           _op("fetch", {"X": ["out"]}, {"Out": ["fetch"]}, [_i("col", 0)])]
    path = _save(tmp_path, "sm", ops, {"x": [-1, 16, 1, 1]}, P, {"f": 2, "t": 2, "out": 2})
    pred = _both(path, [rng.randn(3, 16, 1, 1).astype("float32")])
    assert pred.pass_stats[f"gpu_cpu_{'flatten2' if shape_op == 'flatten2' else shape_op}_matmul_fuse_pass"] == 1
    assert _types(pred) == ["fc"]


def test_matmul_maps_and_scale_fuse(tmp_path):
    P = {"w": rng.randn(8, 6) * 0.2, "w2": rng.randn(6, 4) * 0.2}
    ops = [_op("matmul_v2", {"X": ["x"], "Y": ["w"]}, {"Out": ["t"]}, [_b("trans_x", False), _b("trans_y", False)]),
           _op("scale", {"X": ["t"]}, {"Out": ["s"]}, [_f("scale", 0.5), _f("bias", 0.0), _b("bias_after_scale", True)]),
           _op("matmul_v2", {"X": ["s"], "Y": ["w2"]}, {"Out": ["u"]}, [_b("trans_x", False), _b("trans_y", False)]),
           _op("matmul_v2", {"X": ["u"], "Y": ["u"]}, {"Out": ["out"]}, [_b("trans_x", True), _b("trans_y", False)]),
           _op("fetch", {"X": ["out"]}, {"Out": ["fetch"]}, [_i("col", 0)])]
    path = _save(tmp_path, "mm", ops, {"x": [-1, 8]}, P, {"t": 2, "s": 2, "u": 2, "out": 2})
    pred = _both(path, [rng.randn(5, 8).astype("float32")])
    st = pred.pass_stats
    assert st["matmul_scale_fuse_pass"] == 1, st
    assert st["gpu_cpu_map_matmul_v2_to_mul_pass"] == 2 and st["gpu_cpu_map_matmul_v2_to_matmul_pass"] == 1, st
    assert _types(pred) == ["mul", "mul", "matmul"]


def test_transpose_flatten_concat_fuse(tmp_path):
    ops, srcs = [], []
    for i in range(3):
        ops += [_op("transpose2", {"X": [f"x{i}"]}, {"Out": [f"t{i}"], "XShape": [f"xs{i}"]}, [_ints("axis", [0, 2, 3, 1])]),
                _op("flatten2", {"X": [f"t{i}"]}, {"Out": [f"f{i}"], "XShape": [f"fs{i}"]}, [_i("axis", 1)])]
        srcs.append(f"f{i}")
    ops += [_op("concat", {"X": srcs}, {"Out": ["out"]}, [_i("axis", 1)]),
            _op("fetch", {"X": ["out"]}, {"Out": ["fetch"]}, [_i("col", 0)])]
    feeds = {f"x{i}": [-1, 4, 3, 3] for i in range(3)}
    acts = {**{f"t{i}": 4 for i in range(3)}, **{f"f{i}": 2 for i in range(3)}, "out": 2}
    path = _save(tmp_path, "tfc", ops, feeds, {}, acts)
    pred = _both(path, [rng.randn(2, 4, 3, 3).astype("float32") for _ in range(3)])
    assert pred.pass_stats["transpose_flatten_concat_fuse_pass"] == 1
    assert _types(pred) == ["fusion_transpose_flatten_concat"]


def test_constant_folding_and_is_test(tmp_path):
    P = {"w": rng.randn(6, 4) * 0.2}
    ops = [_op("scale", {"X": ["w"]}, {"Out": ["w2"]}, [_f("scale", 3.0), _f("bias", 0.5), _b("bias_after_scale", True)]),
           _op("transpose2", {"X": ["w2"]}, {"Out": ["w3"], "XShape": ["wx"]}, [_ints("axis", [1, 0])]),
           _op("matmul_v2", {"X": ["x"], "Y": ["w3"]}, {"Out": ["t"]}, [_b("trans_x", False), _b("trans_y", True)]),
           _op("dropout", {"X": ["t"]}, {"Out": ["out"], "Mask": ["mk"]},
               [_f("dropout_prob", 0.2), _b("is_test", False), _s("dropout_implementation", "upscale_in_train")]),
           _op("fetch", {"X": ["out"]}, {"Out": ["fetch"]}, [_i("col", 0)])]
    path = _save(tmp_path, "cf", ops, {"x": [-1, 6]}, P, {"w2": 2, "w3": 2, "t": 2, "out": 2})
    pred = _both(path, [rng.randn(3, 6).astype("float32")])
    st = pred.pass_stats
    assert st["is_test_pass"] == 1 and st["constant_folding_pass"] == 2, st
    assert "scale" not in _types(pred) and "transpose2" not in _types(pred) and "dropout" not in _types(pred)


def test_gpu_pass_list_covers_reference():
    """Every non-TensorRT, non-placement pass of the reference GpuPassStrategy is in the list."""
    from paddle_infer_amd.inference.passes import GPU_PASSES
    ref = {"conv_bn_fuse_pass", "conv_eltwiseadd_bn_fuse_pass", "embedding_eltwise_layernorm_fuse_pass",
           "multihead_matmul_fuse_pass", "fused_multi_transformer_encoder_pass",
           "fused_multi_transformer_decoder_pass", "fused_multi_transformer_encoder_fuse_qkv_pass",
           "fused_multi_transformer_decoder_fuse_qkv_pass",
           "multi_devices_fused_multi_transformer_encoder_fuse_qkv_pass",
           "multi_devices_fused_multi_transformer_decoder_fuse_qkv_pass", "fuse_multi_transformer_layer_pass",
           "gpu_cpu_squeeze2_matmul_fuse_pass", "gpu_cpu_reshape2_matmul_fuse_pass",
           "gpu_cpu_flatten2_matmul_fuse_pass", "gpu_cpu_map_matmul_v2_to_mul_pass",
           "gpu_cpu_map_matmul_v2_to_matmul_pass", "matmul_scale_fuse_pass", "gpu_cpu_map_matmul_to_mul_pass",
           "fc_fuse_pass", "fc_elementwise_layernorm_fuse_pass", "conv_elementwise_add_act_fuse_pass",
           "conv_elementwise_add2_act_fuse_pass", "conv_elementwise_add_fuse_pass",
           "transpose_flatten_concat_fuse_pass", "constant_folding_pass", "is_test_pass",
           "simplify_with_basic_ops_pass", "identity_scale_op_clean_pass"}
    assert ref <= set(GPU_PASSES), ref - set(GPU_PASSES)
