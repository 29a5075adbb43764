"""fused_multi_transformer encoder / decoder (+ fuse_qkv, + multi_devices) passes over exported-LLM
op programs (reference `fused_multi_transformer_{encoder,decoder}_pass.cc`): a hand-built Paddle
program of plain ops — two pre-LN layers over a prompt whose K / V feed two decode-step layers
through concat caches — runs through the Predictor with and without IR optimisation; the fused
program holds only fused_multi_transformer ops with CacheKV / TimeStep and matches the plain one.
The multi-devices form runs on 2 gloo ranks (c_identity / c_allreduce_sum with ring 0, half the
heads and FFN columns per rank) and must match the single-rank full program."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(__file__))
from dist_utils import run_distributed  # noqa: E402
from fmt_wire import _op, _var  # noqa: E402

from paddle_infer_amd.static import proto  # noqa: E402

A = proto.ATTR


def _a(name, v):
    if isinstance(v, bool):
        return {"name": name, "type": A["BOOLEAN"], "b": v}
    if isinstance(v, int):
        return {"name": name, "type": A["INT"], "i": v}
    if isinstance(v, float):
        return {"name": name, "type": A["FLOAT"], "f": v}
    if isinstance(v, str):
        return {"name": name, "type": A["STRING"], "s": v}
    return {"name": name, "type": A["INTS"], "ints": list(v)}


class Builder:
    def __init__(self):
        self.ops, self.vars, self.params = [], {}, {}

    def var(self, n, dims=(-1,)):
        self.vars.setdefault(n, _var(n, list(dims)))
        return n

    def param(self, n, arr):
        self.params[n] = np.ascontiguousarray(arr, dtype=np.float32)
        self.vars[n] = _var(n, list(arr.shape), True)
        return n

    def op(self, t, ins, outs, **attrs):
        for v in outs.values():
            for n in v:
                self.var(n)
        self.ops.append(_op(t, ins, outs, [_a(k, v) for k, v in attrs.items()]))
        return outs[next(iter(outs))][0]


def _weights(rng, E, H, F):
    D = E // H
    return {"ln1_s": 1 + 0.1 * rng.randn(E), "ln1_b": 0.1 * rng.randn(E),
            "qkv_w": rng.randn(E, H, 3, D) / np.sqrt(E), "qkv_b": 0.1 * rng.randn(H, 3, D),
            "out_w": rng.randn(H * D, E) / np.sqrt(E), "out_b": 0.1 * rng.randn(E),
            "ln2_s": 1 + 0.1 * rng.randn(E), "ln2_b": 0.1 * rng.randn(E),
            "f1_w": rng.randn(E, F) / np.sqrt(E), "f1_b": 0.1 * rng.randn(F),
            "f2_w": rng.randn(F, E) / np.sqrt(F), "f2_b": 0.1 * rng.randn(E)}


def _shard(W, rank, mp, H, F):
    """This rank's heads (QKV columns, out-proj rows) and FFN columns / rows."""
    h = H // mp
    f = F // mp
    hs, fs = slice(rank * h, (rank + 1) * h), slice(rank * f, (rank + 1) * f)
    D = W["qkv_w"].shape[-1]
    return dict(W, qkv_w=W["qkv_w"][:, hs], qkv_b=W["qkv_b"][hs],
                out_w=W["out_w"].reshape(H, D, -1)[hs].reshape(h * D, -1), f1_w=W["f1_w"][:, fs],
                f1_b=W["f1_b"][fs], f2_w=W["f2_w"][fs])


def _layer(b, pfx, x, W, H, mask, mp, cache=None, fuse_qkv=True):
    """One pre-LN layer in exported-op form; returns (out, k, v) (k / v before any cache concat)."""
    E = W["ln1_s"].shape[0]
    D = W["qkv_w"].shape[-1]
    p = {k: b.param(f"{pfx}.{k}", v) for k, v in W.items() if k not in ("qkv_w", "qkv_b")}
    y = b.op("layer_norm", {"X": [x], "Scale": [p["ln1_s"]], "Bias": [p["ln1_b"]]},
             {"Y": [f"{pfx}.ln1"], "Mean": [f"{pfx}.m1"], "Variance": [f"{pfx}.v1"]},
             epsilon=1e-5, begin_norm_axis=2)
    if mp:
        y = b.op("c_identity", {"X": [y]}, {"Out": [f"{pfx}.ci1"]}, ring_id=0)
    if fuse_qkv:
        wq = b.param(f"{pfx}.qkv_w", W["qkv_w"].reshape(E, -1))
        bq = b.param(f"{pfx}.qkv_b", W["qkv_b"].reshape(-1))
        t = b.op("matmul_v2", {"X": [y], "Y": [wq]}, {"Out": [f"{pfx}.qkv0"]}, trans_x=False, trans_y=False)
        t = b.op("elementwise_add", {"X": [t], "Y": [bq]}, {"Out": [f"{pfx}.qkv1"]}, axis=-1)
        t = b.op("reshape2", {"X": [t]}, {"Out": [f"{pfx}.qkv2"], "XShape": [f"{pfx}.xs0"]}, shape=[0, 0, H, 3 * D])
        t = b.op("transpose2", {"X": [t]}, {"Out": [f"{pfx}.qkv3"], "XShape": [f"{pfx}.xs1"]}, axis=[0, 2, 1, 3])
        q, k, v = f"{pfx}.q", f"{pfx}.k", f"{pfx}.v"
        b.op("split", {"X": [t]}, {"Out": [q, k, v]}, axis=3, num=3, sections=[])
    else:
        outs = []
        for j, nm in enumerate("qkv"):
            w = b.param(f"{pfx}.{nm}_w", W["qkv_w"][:, :, j].reshape(E, -1))
            bb = b.param(f"{pfx}.{nm}_b", W["qkv_b"][:, j].reshape(-1))
            t = b.op("matmul_v2", {"X": [y], "Y": [w]}, {"Out": [f"{pfx}.{nm}0"]}, trans_x=False, trans_y=False)
            t = b.op("elementwise_add", {"X": [t], "Y": [bb]}, {"Out": [f"{pfx}.{nm}1"]}, axis=-1)
            t = b.op("reshape2", {"X": [t]}, {"Out": [f"{pfx}.{nm}2"], "XShape": [f"{pfx}.{nm}xs0"]}, shape=[0, 0, H, D])
            outs.append(b.op("transpose2", {"X": [t]}, {"Out": [f"{pfx}.{nm}"], "XShape": [f"{pfx}.{nm}xs1"]},
                             axis=[0, 2, 1, 3]))
        q, k, v = outs
    ka, va = k, v
    if cache is not None:
        ka = b.op("concat", {"X": [cache[0], k]}, {"Out": [f"{pfx}.kall"]}, axis=2)
        va = b.op("concat", {"X": [cache[1], v]}, {"Out": [f"{pfx}.vall"]}, axis=2)
        b.op("assign", {"X": [ka]}, {"Out": [f"{pfx}.kcache_out"]})
        b.op("assign", {"X": [va]}, {"Out": [f"{pfx}.vcache_out"]})
    s = b.op("matmul", {"X": [q], "Y": [ka]}, {"Out": [f"{pfx}.s"]}, transpose_X=False, transpose_Y=True,
             alpha=float(1.0 / np.sqrt(D)))
    s = b.op("elementwise_add", {"X": [s], "Y": [mask]}, {"Out": [f"{pfx}.sm"]}, axis=-1)
    s = b.op("softmax", {"X": [s]}, {"Out": [f"{pfx}.p"]}, axis=-1)
    o = b.op("matmul_v2", {"X": [s], "Y": [va]}, {"Out": [f"{pfx}.o"]}, trans_x=False, trans_y=False)
    o = b.op("transpose2", {"X": [o]}, {"Out": [f"{pfx}.ot"], "XShape": [f"{pfx}.xs2"]}, axis=[0, 2, 1, 3])
    o = b.op("reshape2", {"X": [o]}, {"Out": [f"{pfx}.or"], "XShape": [f"{pfx}.xs3"]}, shape=[0, 0, H * D])
    o = b.op("matmul_v2", {"X": [o], "Y": [p["out_w"]]}, {"Out": [f"{pfx}.o1"]}, trans_x=False, trans_y=False)
    if mp:
        o = b.op("c_allreduce_sum", {"X": [o]}, {"Out": [f"{pfx}.o1r"]}, ring_id=0, use_calc_stream=True)
    o = b.op("elementwise_add", {"X": [o], "Y": [p["out_b"]]}, {"Out": [f"{pfx}.o2"]}, axis=-1)
    x2 = b.op("elementwise_add", {"X": [x], "Y": [o]}, {"Out": [f"{pfx}.x2"]}, axis=-1)
    y2 = b.op("layer_norm", {"X": [x2], "Scale": [p["ln2_s"]], "Bias": [p["ln2_b"]]},
              {"Y": [f"{pfx}.ln2"], "Mean": [f"{pfx}.m2"], "Variance": [f"{pfx}.v2"]},
              epsilon=1e-5, begin_norm_axis=2)
    if mp:
        y2 = b.op("c_identity", {"X": [y2]}, {"Out": [f"{pfx}.ci2"]}, ring_id=0)
    h = b.op("matmul_v2", {"X": [y2], "Y": [p["f1_w"]]}, {"Out": [f"{pfx}.h0"]}, trans_x=False, trans_y=False)
    h = b.op("elementwise_add", {"X": [h], "Y": [p["f1_b"]]}, {"Out": [f"{pfx}.h1"]}, axis=-1)
    h = b.op("gelu", {"X": [h]}, {"Out": [f"{pfx}.h2"]}, approximate=False)
    f = b.op("matmul_v2", {"X": [h], "Y": [p["f2_w"]]}, {"Out": [f"{pfx}.f0"]}, trans_x=False, trans_y=False)
    if mp:
        f = b.op("c_allreduce_sum", {"X": [f]}, {"Out": [f"{pfx}.f0r"]}, ring_id=0, use_calc_stream=True)
    f = b.op("elementwise_add", {"X": [f], "Y": [p["f2_b"]]}, {"Out": [f"{pfx}.f1"]}, axis=-1)
    out = b.op("elementwise_add", {"X": [x2], "Y": [f]}, {"Out": [f"{pfx}.out"]}, axis=-1)
    return out, k, v


E, H, F, L = 32, 4, 64, 2


def write_program(prefix, rank=0, mp=1, fuse_qkv=True):
    rng = np.random.RandomState(0)
    Ws = [_weights(rng, E, H, F) for _ in range(2 * L)]  # encoder and decoder share nothing here
    b = Builder()
    feeds = ["x", "mask", "x1", "mask1"]
    b.var("x", [-1, -1, E]), b.var("mask", [-1, 1, -1, -1]), b.var("x1", [-1, 1, E]), b.var("mask1", [-1, 1, 1, -1])
    for i, n in enumerate(feeds):
        b.ops.append(_op("feed", {"X": ["feed"]}, {"Out": [n]}, [_a("col", i)]))
    h, caches = "x", []
    hl = H // mp
    for i in range(L):
        W = _shard(Ws[i], rank, mp, H, F) if mp > 1 else Ws[i]
        h, k, v = _layer(b, f"enc{i}", h, W, hl, "mask", mp > 1, fuse_qkv=fuse_qkv)
        caches.append((k, v))
    enc_out = h
    h = "x1"
    for i in range(L):
        # the decode step's layer i reuses the ENCODER layer i weights (same model, one more token)
        W = _shard(Ws[i], rank, mp, H, F) if mp > 1 else Ws[i]
        h, _, _ = _layer(b, f"dec{i}", h, W, hl, "mask1", mp > 1, cache=caches[i], fuse_qkv=fuse_qkv)
    for i, n in enumerate((enc_out, h)):
        b.ops.append(_op("fetch", {"X": [n]}, {"Out": ["fetch"]}, [_a("col", i)]))
    desc = {"blocks": [{"idx": 0, "parent_idx": -1, "vars": list(b.vars.values()) + [
        {"name": "feed", "type": {"type": proto.VT_FEED}, "persistable": True},
        {"name": "fetch", "type": {"type": proto.VT_FETCH}, "persistable": True}], "ops": b.ops}]}
    with open(prefix + ".pdmodel", "wb") as f:
        f.write(proto.encode("ProgramDesc", desc))
    with open(prefix + ".pdiparams", "wb") as f:
        for n in sorted(b.params):
            f.write(proto.tensor_to_stream(b.params[n], proto.VT["float32"]))


def _inputs(B=2, S=5):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, S, E, generator=g)
    causal = torch.triu(torch.full((S, S), -1e4), 1)
    mask = causal.expand(B, 1, S, S).contiguous()
    x1 = torch.randn(B, 1, E, generator=g)
    mask1 = torch.zeros(B, 1, 1, S + 1)
    return {"x": x, "mask": mask, "x1": x1, "mask1": mask1}


def _run(prefix, ir, feeds):
    from paddle_infer_amd import inference as pinf
    c = pinf.Config(prefix + ".pdmodel", prefix + ".pdiparams")
    c.switch_ir_optim(ir)
    p = pinf.create_predictor(c)
    for n, t in feeds.items():
        p.get_input_handle(n).copy_from_cpu(t.numpy())
    assert p.run()
    outs = [p.get_output_handle(n).copy_to_cpu() for n in p.get_output_names()]
    types = [op.type for b in p._program.blocks for op in b.ops] if hasattr(p, "_program") else None
    return outs, types, getattr(p, "pass_stats", {})


@pytest.mark.parametrize("fuse_qkv", [True, False])
def test_encoder_decoder_passes_match_plain_program(tmp_path, fuse_qkv):
    pre = str(tmp_path / "gen")
    write_program(pre, fuse_qkv=fuse_qkv)
    feeds = _inputs()
    ref, _, _ = _run(pre, False, feeds)
    got, types, stats = _run(pre, True, feeds)
    enc, dec = (("fused_multi_transformer_encoder_fuse_qkv_pass", "fused_multi_transformer_decoder_fuse_qkv_pass")
                if fuse_qkv else ("fused_multi_transformer_encoder_pass", "fused_multi_transformer_decoder_pass"))
    assert stats.get(enc) == 2 * L, stats  # the encoder pass also rewires the decoder layers' caches
    if types is not None:
        assert "fused_multi_transformer" in types and "softmax" not in types and "concat" not in types
    for a, b in zip(got, ref):
        np.testing.assert_allclose(a, b, rtol=2e-4, atol=2e-4)
    dec  # noqa: B018


def _mp_worker(rank, world, prefix):
    pre = f"{prefix}_r{rank}"
    write_program(pre, rank, world)
    feeds = _inputs()
    ref, _, _ = _run(pre, False, feeds)
    got, types, stats = _run(pre, True, feeds)
    return {"ref": ref, "got": got, "stats": stats, "types": types}


def test_multi_devices_fused_transformer_with_ring_id_matches_single_rank(tmp_path):
    single = str(tmp_path / "single")
    write_program(single)
    full, _, _ = _run(single, False, _inputs())
    res = run_distributed(_mp_worker, 2, str(tmp_path / "mp"))
    for r in range(2):
        assert res[r]["stats"].get("multi_devices_fused_multi_transformer_encoder_fuse_qkv_pass") == 2 * L
        for a, b, c in zip(res[r]["got"], res[r]["ref"], full):
            np.testing.assert_allclose(b, c, rtol=2e-4, atol=2e-4)  # plain TP program == single rank
            np.testing.assert_allclose(a, c, rtol=2e-4, atol=2e-4)  # fused TP program == single rank
