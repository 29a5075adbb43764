"""Build a Paddle-wire ``.pdmodel`` / ``.pdiparams`` holding ONE fused_multi_transformer op with the
reference's slot names (`fused_multi_transformer_op.cc:152-190`), from a dygraph
FusedMultiTransformer layer's weights. Shared by the CPU and GPU predictor tests."""
import numpy as np

from paddle_infer_amd.static import proto


def _op(t, ins, outs, attrs=()):
    return {"type": t, "inputs": [{"parameter": k, "arguments": v} for k, v in ins.items()],
            "outputs": [{"parameter": k, "arguments": v} for k, v in outs.items()], "attrs": list(attrs)}


def _var(n, dims, persistable=False, dt="float32"):
    return {"name": n, "type": {"type": proto.VT_LOD_TENSOR, "lod_tensor": {
        "tensor": {"data_type": proto.VT[dt], "dims": dims}, "lod_level": 0}},
        "persistable": persistable}


SLOTS = {"LnScale": "ln_scales", "LnBias": "ln_biases", "QKVW": "qkv_weights", "QKVBias": "qkv_biases",
         "OutLinearW": "linear_weights", "OutLinearBias": "linear_biases",
         "FFNLnScale": "ffn_ln_scales", "FFNLnBias": "ffn_ln_biases", "FFN1Weight": "ffn1_weights",
         "FFN1Bias": "ffn1_biases", "FFN2Weight": "ffn2_weights", "FFN2Bias": "ffn2_biases"}


def write_fmt_program(layer, prefix, decode, num_layers, E, causal=True):
    A = proto.ATTR
    params, ins = {}, {"X": ["x"]}
    vars_ = [_var("x", [-1, -1, E])]
    for slot, attr in SLOTS.items():
        names = []
        for i, p in enumerate(getattr(layer, attr)[:num_layers]):
            n = f"{attr}.{i}"
            params[n] = p.detach().float().cpu().numpy()
            vars_.append(_var(n, list(params[n].shape), True))
            names.append(n)
        ins[slot] = names
    caches = [f"cache_kv.{i}" for i in range(num_layers)]
    ins["CacheKV"] = caches
    vars_ += [_var(c, [2, -1, -1, -1, -1]) for c in caches]
    feeds = ["x"] + caches
    if decode:
        ins["TimeStep"] = ["time_step"]
        vars_.append(_var("time_step", [1], dt="int32"))
        feeds.append("time_step")
    vars_.append(_var("out", [-1, -1, E]))
    attrs = [{"name": "pre_layer_norm", "type": A["BOOLEAN"], "b": True},
             {"name": "epsilon", "type": A["FLOAT"], "f": 1e-5},
             {"name": "act_method", "type": A["STRING"], "s": "gelu"},
             {"name": "trans_qkvw", "type": A["BOOLEAN"], "b": True},
             {"name": "ring_id", "type": A["INT"], "i": -1},
             {"name": "dropout_rate", "type": A["FLOAT"], "f": 0.0},
             {"name": "is_test", "type": A["BOOLEAN"], "b": True},
             {"name": "causal", "type": A["BOOLEAN"], "b": bool(causal)}]
    ops = [_op("feed", {"X": ["feed"]}, {"Out": [n]}, [{"name": "col", "type": A["INT"], "i": i}])
           for i, n in enumerate(feeds)]
    ops.append(_op("fused_multi_transformer", ins, {"Out": ["out"], "CacheKVOut": caches}, attrs))
    ops.append(_op("fetch", {"X": ["out"]}, {"Out": ["fetch"]}, [{"name": "col", "type": A["INT"], "i": 0}]))
    desc = {"blocks": [{"idx": 0, "parent_idx": -1, "vars": vars_, "ops": ops}]}
    with open(prefix + ".pdmodel", "wb") as f:
        f.write(proto.encode("ProgramDesc", desc))
    with open(prefix + ".pdiparams", "wb") as f:
        for n in sorted(params):
            f.write(proto.tensor_to_stream(np.ascontiguousarray(params[n]), proto.VT["float32"]))
    return feeds
