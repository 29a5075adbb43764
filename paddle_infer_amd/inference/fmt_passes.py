"""fused_multi_transformer passes over the op form exported LLM programs carry (reference
`paddle/fluid/framework/ir/fused_multi_transformer_{encoder,decoder}_pass.cc`, GPU pass list in
`paddle_pass_builder.cc`):

  fused_multi_transformer_encoder_pass / _fuse_qkv_pass
  fused_multi_transformer_decoder_pass / _fuse_qkv_pass
  multi_devices_fused_multi_transformer_encoder_fuse_qkv_pass
  multi_devices_fused_multi_transformer_decoder_fuse_qkv_pass

One pre-LN transformer layer written with plain Paddle ops —

    ln = layer_norm(x) [→ c_identity]
    QKV: matmul_v2 + elementwise_add + reshape2 [0,0,H,3D] + transpose2 [0,2,1,3] + split(3, axis 3)
         (fuse_qkv)  |  three matmul_v2 + elementwise_add + reshape2 [0,0,H,D] + transpose2 (Q/K/V)
    decoder only:    k = concat([cache_k, k], axis 2) (+ assign → cache_k), same for v
    attention:       matmul(q, k, transpose_Y, alpha) [| matmul_v2 + scale] + elementwise_add(mask)
                     + softmax + matmul_v2(·, v) + transpose2 [0,2,1,3] + reshape2 [0,0,E]
    out:             matmul_v2 [→ c_allreduce_sum] + elementwise_add(b) + elementwise_add(x)
    FFN:             layer_norm [→ c_identity] + matmul_v2 + elementwise_add + gelu|relu
                     + matmul_v2 [→ c_allreduce_sum] + elementwise_add(b) + elementwise_add(residual)

→ one ``fused_multi_transformer`` op (the MI355X LLM kernels: fused LN prologues, packed QKV GEMM,
flash / split-K decode attention over a KV cache, epilogue GEMMs; ``ring_id`` all-reduces after the
row-parallel projections in the multi-devices form).

KV cache plumbing (as the reference): an ENCODER layer whose K / V also leave the layer (exported as
the decode loop's initial caches) gets ``CacheKV`` = ``cache_kv<i>`` — a [2, B, H, max_len, D]
buffer created by ``fill_constant_batch_size_like`` — written by the fused op (``CacheKVOut``);
every consumer of the old K / V names (a ``while`` op's X / Out lists, a decoder layer's concat)
is rewired to that buffer. A DECODER layer's ``concat(cache, new)`` + ``assign`` pair becomes
``CacheKV`` = the buffer its cache came from and ``TimeStep`` = mask length - 1 (``shape`` +
``slice`` + ``scale`` ops, so the step count stays a device value inside the loop).
"""
from __future__ import annotations

import numpy as np
import torch

from .passes import Graph, _new, _out, _pop

DEFAULT_MAX_LEN = 1024


def _typed(ops):
    return [o for o in ops if o.func is None and o.paddle_inputs is not None]


def _only(g, name, types):
    """The single typed consumer of ``name`` with a type in ``types`` (others must not exist)."""
    cs = g.consumers(name)
    if len(cs) != 1 or cs[0].func is not None or cs[0].type not in types or name in g.keep:
        return None
    return cs[0]


def _consumer(g, name, types):
    """The unique consumer of ``name`` among ``types`` (other consumers allowed)."""
    cs = [c for c in g.consumers(name) if c.func is None and c.type in types]
    return cs[0] if len(cs) == 1 else None


def _ints(v):
    return [int(x) for x in (v or [])]


def _linear(g, x, mp):
    """x → [c_identity] → matmul_v2(x, W param) → elementwise_add(bias param):
    (ops, W, b, out) or None."""
    ops = []
    if mp:
        ci = _only(g, x, ("c_identity",))
        if ci is None:
            return None
        ops.append(ci)
        x = _out(ci)
    mm = _consumer(g, x, ("matmul_v2", "matmul"))
    if mm is None or _pop(mm, "X") != x or not g.is_param(_pop(mm, "Y")):
        return None
    if mm.attrs.get("trans_x") or mm.attrs.get("trans_y") or mm.attrs.get("transpose_X") \
            or mm.attrs.get("transpose_Y") or float(mm.attrs.get("alpha", 1.0)) != 1.0:
        return None
    add = _only(g, _out(mm), ("elementwise_add",))
    if add is None or not g.is_param(_pop(add, "Y")):
        return None
    return ops + [mm, add], _pop(mm, "Y"), _pop(add, "Y"), _out(add)


def _row_linear(g, x, mp):
    """x → matmul_v2(W) [→ c_allreduce_sum] → elementwise_add(bias): (ops, W, b, out, ring)."""
    mm = _only(g, x, ("matmul_v2", "matmul"))
    if mm is None or _pop(mm, "X") != x or not g.is_param(_pop(mm, "Y")):
        return None
    if mm.attrs.get("trans_y") or mm.attrs.get("transpose_Y"):
        return None
    ops, y, ring = [mm], _out(mm), -1
    if mp:
        ar = _only(g, y, ("c_allreduce_sum", "mp_allreduce_sum"))
        if ar is None:
            return None
        ops.append(ar)
        y, ring = _out(ar), int(ar.attrs.get("ring_id", 0))
    add = _only(g, y, ("elementwise_add",))
    if add is None or not g.is_param(_pop(add, "Y")):
        return None
    return ops + [add], _pop(mm, "Y"), _pop(add, "Y"), _out(add), ring


def _heads(g, x, last):
    """x → reshape2 [0, 0, H, last*?] → transpose2 [0, 2, 1, 3]: (ops, H, inner, out)."""
    r = _only(g, x, ("reshape2", "reshape"))
    if r is None or r.paddle_inputs.get("Shape") or r.paddle_inputs.get("ShapeTensor"):
        return None
    shp = _ints(r.attrs.get("shape"))
    if len(shp) != 4 or shp[0] != 0 or shp[1] != 0:
        return None
    t = _only(g, _out(r), ("transpose2", "transpose"))
    if t is None or _ints(t.attrs.get("axis")) != [0, 2, 1, 3]:
        return None
    return [r, t], shp[2], shp[3], _out(t)


def _residual(g, base, other):
    add = _only(g, other, ("elementwise_add",))
    if add is None or {_pop(add, "X"), _pop(add, "Y")} != {base, other}:
        return None
    return add


def _cache_concat(g, t):
    """Decoder: concat([cache, t], axis 2) → (ops [concat, assign?], cache name, out name)."""
    c = _consumer(g, t, ("concat",))
    if c is None:
        return None
    xs = c.paddle_inputs.get("X") or []
    if len(xs) != 2 or xs[1] != t or int(c.attrs.get("axis", 0)) != 2:
        return None
    ops = [c]
    for a in g.consumers(_out(c)):
        if a.func is None and a.type == "assign":
            ops.append(a)
    return ops, xs[0], _out(c)


def _match_layer(g, ln1, fuse_qkv, mp, decoder):
    """The whole layer starting at ``ln1`` → dict, or None."""
    x = _pop(ln1, "X")
    y1 = _out(ln1, "Y")
    ops = [ln1]
    if fuse_qkv:
        lin = _linear(g, y1, mp)
        if lin is None:
            return None
        lops, wqkv, bqkv, qkv = lin
        hd = _heads(g, qkv, 3)
        if hd is None:
            return None
        hops, H, D3, tq = hd
        sp = _only(g, tq, ("split",))
        if sp is None or int(sp.attrs.get("axis", -1)) not in (3, -1) or len(sp.paddle_outputs.get("Out", [])) != 3:
            return None
        if D3 % 3:
            return None
        D = D3 // 3
        q, k, v = sp.paddle_outputs["Out"]
        ops += lops + hops + [sp]
        weights = ("fused", wqkv, bqkv)
    else:
        cons = [c for c in g.consumers(y1) if c.func is None and c.type in ("matmul_v2", "matmul", "c_identity")]
        if mp:
            ci = _only(g, y1, ("c_identity",))
            if ci is None:
                return None
            ops.append(ci)
            src = _out(ci)
            cons = [c for c in g.consumers(src) if c.func is None and c.type in ("matmul_v2", "matmul")]
        else:
            src = y1
        if len(cons) != 3 or len(g.consumers(src)) != 3:
            return None
        branches = []
        for mm in cons:
            if not g.is_param(_pop(mm, "Y")) or _pop(mm, "X") != src:
                return None
            add = _only(g, _out(mm), ("elementwise_add",))
            if add is None or not g.is_param(_pop(add, "Y")):
                return None
            hd = _heads(g, _out(add), 1)
            if hd is None:
                return None
            branches.append(([mm, add] + hd[0], _pop(mm, "Y"), _pop(add, "Y"), hd[1], hd[2], hd[3]))
        # which branch is Q: the one feeding the QK matmul as X
        qi = [i for i, b in enumerate(branches)
              if any(c.func is None and c.type in ("matmul", "matmul_v2") and _pop(c, "X") == b[5]
                     for c in g.consumers(b[5]))]
        if len(qi) != 1:
            return None
        qb = branches.pop(qi[0])
        # K: the branch whose output (or its cache concat) is the QK matmul's Y
        qk_tmp = _consumer(g, qb[5], ("matmul", "matmul_v2"))
        kname = _pop(qk_tmp, "Y") if qk_tmp is not None else None

        def is_k(b):
            if b[5] == kname:
                return True
            cc = _cache_concat(g, b[5]) if decoder else None
            return cc is not None and cc[2] == kname
        ks = [b for b in branches if is_k(b)]
        if len(ks) != 1:
            return None
        kb = ks[0]
        vb = branches[0] if branches[1] is kb else branches[1]
        H, D = qb[3], qb[4]
        if (kb[3], kb[4], vb[3], vb[4]) != (H, D, H, D):
            return None
        for b in (qb, kb, vb):
            ops += b[0]
        q, k, v = qb[5], kb[5], vb[5]
        weights = ("separate", (qb[1], kb[1], vb[1]), (qb[2], kb[2], vb[2]))
    cache_k = cache_v = None
    if decoder:
        ck, cv = _cache_concat(g, k), _cache_concat(g, v)
        if ck is None or cv is None:
            return None
        ops += ck[0] + cv[0]
        cache_k, cache_v = ck[1], cv[1]
        k_all, v_all = ck[2], cv[2]
        for t in (k_all, v_all):  # the concatenated cache feeds attention and its write-back only
            if t in g.keep or any(c.type not in ("matmul", "matmul_v2", "assign") for c in g.consumers(t)):
                return None
    else:
        k_all, v_all = k, v
    qk = _consumer(g, q, ("matmul", "matmul_v2"))
    if qk is None or _pop(qk, "Y") != k_all:
        return None
    if not (qk.attrs.get("transpose_Y") or qk.attrs.get("trans_y")):
        return None
    ops.append(qk)
    s = _out(qk)
    nxt = _only(g, s, ("scale", "elementwise_add", "softmax"))
    if nxt is not None and nxt.type == "scale":
        ops.append(nxt)
        s = _out(nxt)
        nxt = _only(g, s, ("elementwise_add", "softmax"))
    mask = None
    if nxt is not None and nxt.type == "elementwise_add":
        mask = _pop(nxt, "Y") if _pop(nxt, "X") == s else _pop(nxt, "X")
        ops.append(nxt)
        s = _out(nxt)
        nxt = _only(g, s, ("softmax",))
    if nxt is None or nxt.type != "softmax":
        return None
    ops.append(nxt)
    pv = _only(g, _out(nxt), ("matmul_v2", "matmul"))
    if pv is None or _pop(pv, "Y") != v_all:
        return None
    ops.append(pv)
    t2 = _only(g, _out(pv), ("transpose2", "transpose"))
    if t2 is None or _ints(t2.attrs.get("axis")) != [0, 2, 1, 3]:
        return None
    r2 = _only(g, _out(t2), ("reshape2", "reshape"))
    if r2 is None or len(_ints(r2.attrs.get("shape"))) != 3:
        return None
    ops += [t2, r2]
    ol = _row_linear(g, _out(r2), mp)
    if ol is None:
        return None
    oops, wo, bo, o, ring = ol
    add1 = _residual(g, x, o)
    if add1 is None:
        return None
    ops += oops + [add1]
    x2 = _out(add1)
    ln2s = [c for c in g.consumers(x2) if c.func is None and c.type == "layer_norm"]
    if len(ln2s) != 1 or len(g.consumers(x2)) != 2 or x2 in g.keep:
        return None
    ln2 = ln2s[0]
    f1 = _linear(g, _out(ln2, "Y"), mp)
    if f1 is None:
        return None
    f1ops, w1, b1, h = f1
    act = _only(g, h, ("gelu", "relu"))
    if act is None:
        return None
    f2 = _row_linear(g, _out(act), mp)
    if f2 is None:
        return None
    f2ops, w2, b2, f, ring2 = f2
    add2 = _residual(g, x2, f)
    if add2 is None:
        return None
    ops += [ln2] + f1ops + [act] + f2ops + [add2]
    if len(set(map(id, ops))) != len(ops):
        return None
    eps = float(ln1.attrs.get("epsilon", 1e-5))
    if abs(eps - float(ln2.attrs.get("epsilon", 1e-5))) > 1e-12:
        return None
    # the scaling of QK must be 1/sqrt(D) (the fused kernel's)
    alpha = float(qk.attrs.get("alpha", 1.0))
    for o_ in ops:
        if o_.type == "scale" and o_ is not ln1:
            alpha *= float(o_.attrs.get("scale", 1.0))
    if abs(alpha - 1.0 / np.sqrt(D)) > 1e-4 * alpha:
        return None
    return dict(ops=ops, x=x, ln1=ln1, ln2=ln2, weights=weights, H=H, D=D, k=k, v=v, mask=mask,
                cache=(cache_k, cache_v), wo=wo, bo=bo, w1=w1, b1=b1, w2=w2, b2=b2,
                act=act.type if not (act.type == "gelu" and act.attrs.get("approximate")) else "gelu",
                out=_out(add2), eps=eps, ring=ring if mp else -1, ring_ok=(ring == ring2))


def _qkv_params(g, m, tag):
    """The fused op's QKVW [E, 3, H, D] (trans_qkvw=False) and QKVBias [3, H, D]."""
    H, D = m["H"], m["D"]
    kind, w, b = m["weights"]
    if kind == "fused":  # per-head [Q | K | V] columns: [E, H, 3, D]
        W = g.param(w)
        E = W.shape[0]
        Wn = W.reshape(E, H, 3, D).permute(0, 2, 1, 3).contiguous()
        Bn = g.param(b).reshape(H, 3, D).permute(1, 0, 2).contiguous()
    else:
        Ws = [g.param(n) for n in w]
        E = Ws[0].shape[0]
        Wn = torch.stack([x.reshape(E, H, D) for x in Ws], 1).contiguous()
        Bn = torch.stack([g.param(n).reshape(H, D) for n in b], 0).contiguous()
    names = []
    for suffix, t in (("w", Wn), ("b", Bn)):
        n = f"{tag}.qkv_{suffix}"
        g.program.params[n] = t
        g.block.create_var(n, list(t.shape), "float32", persistable=True)
        names.append(n)
    return names


def _fmt_op(g, m, idx, cache_kv, time_step, mp):
    wn, bn = _qkv_params(g, m, f"fmt{idx}")
    ins = {"X": [m["x"]], "LnScale": [_pop(m["ln1"], "Scale")], "LnBias": [_pop(m["ln1"], "Bias")],
           "QKVW": [wn], "QKVBias": [bn], "OutLinearW": [m["wo"]], "OutLinearBias": [m["bo"]],
           "FFNLnScale": [_pop(m["ln2"], "Scale")], "FFNLnBias": [_pop(m["ln2"], "Bias")],
           "FFN1Weight": [m["w1"]], "FFN1Bias": [m["b1"]], "FFN2Weight": [m["w2"]], "FFN2Bias": [m["b2"]]}
    outs = {"Out": [m["out"]]}
    if m["mask"] is not None:
        ins["SrcMask"] = [m["mask"]]
    if cache_kv is not None:
        ins["CacheKV"] = [cache_kv]
        outs["CacheKVOut"] = [cache_kv]
    if time_step is not None:
        ins["TimeStep"] = [time_step]
    attrs = {"pre_layer_norm": True, "epsilon": m["eps"], "dropout_rate": 0.0, "is_test": True,
             "dropout_implementation": "upscale_in_train", "act_method": m["act"],
             "trans_qkvw": False, "ring_id": m["ring"] if mp else -1, "causal": m["mask"] is None}
    return _new(g.block, "fused_multi_transformer", ins, outs, attrs)


def _cache_map(program):
    if not hasattr(program, "_fmt_cache_of"):
        program._fmt_cache_of = {}
    return program._fmt_cache_of


def _rename_everywhere(program, old, new):
    """Point every op of every block that reads / writes ``old`` at ``new`` (a while op's carried
    lists, a later layer's concat input)."""
    for b in program.blocks:
        for op in b.ops:
            for slots in (op.paddle_inputs, op.paddle_outputs):
                if not slots:
                    continue
                for k, v in slots.items():
                    if old in v:
                        slots[k] = list(dict.fromkeys(new if n == old else n for n in v))


def _block_graphs(g):
    out = []
    for b in g.program.blocks:
        gb = Graph(g.program, g.keep)
        gb.block = b
        out.append(gb)
    return out


def _matches(gbs, fuse_qkv, mp, decoder):
    res = []
    for gb in gbs:
        for ln1 in list(_typed(gb.ops)):
            if ln1.type != "layer_norm":
                continue
            m = _match_layer(gb, ln1, fuse_qkv, mp, decoder)
            if m is not None and m["ring_ok"] and (not decoder or m["mask"] is not None):
                res.append((gb, m))
    return res


def _splice(gb, m, new_ops):
    idx0 = min(gb.ops.index(o) for o in m["ops"])
    for o in m["ops"]:
        gb.ops.remove(o)
    for o in reversed(new_ops):
        gb.ops.insert(idx0, o)
    gb.program._version += 1


def _rewrite_decoder(gb, m, cache, n, mp):
    shp, sl, ts = (f"{cache}.shape", f"{cache}.mask_len", f"{cache}.time_step")
    for nm, dims, dt in ((shp, [4], "int32"), (sl, [1], "int32"), (ts, [1], "float32")):
        gb.block.create_var(nm, dims, dt)
    pre = [_new(gb.block, "shape", {"Input": [m["mask"]]}, {"Out": [shp]}, {}),
           _new(gb.block, "slice", {"Input": [shp]}, {"Out": [sl]},
                {"axes": [0], "starts": [3], "ends": [4], "decrease_axis": []}),
           _new(gb.block, "scale", {"X": [sl]}, {"Out": [ts]},
                {"scale": 1.0, "bias": -1.0, "bias_after_scale": True})]
    _splice(gb, m, pre + [_fmt_op(gb, m, f"dec{n}_{cache}", cache, ts, mp)])


def _fuse(g, fuse_qkv, mp, encoders=True, max_len=DEFAULT_MAX_LEN):
    """Encoder layers (with their KV-cache export) and the decoder layers that read those caches.
    An encoder layer whose K / V are read outside it by anything but a decode loop (``while``) or
    a matched decoder layer's cache concat is left alone (its K / V must stay materialised)."""
    gbs = _block_graphs(g)
    decs = _matches(gbs, fuse_qkv, mp, decoder=True)
    dec_concat = {}
    for gb, m in decs:
        for c in m["ops"]:
            if c.type == "concat":
                dec_concat[id(c)] = m
    cmap = _cache_map(g.program)
    n = 0
    fills = {}
    if encoders:
        for gb, m in _matches(gbs, fuse_qkv, mp, decoder=False):
            if any(o not in gb.ops for o in m["ops"]):
                continue
            inner = set(map(id, m["ops"]))
            readers = [op for b in gbs for op in b.ops if id(op) not in inner
                       and (m["k"] in op.input_names() or m["v"] in op.input_names())]
            if any(op.type not in ("while", "assign") and id(op) not in dec_concat for op in readers):
                continue
            cache, new_ops = None, []
            if readers or m["k"] in g.keep or m["v"] in g.keep:
                if m["k"] in g.keep or m["v"] in g.keep:
                    continue
                cache = f"cache_kv{len({c for c, _ in cmap.values()})}"
                gb.block.create_var(cache, [2, -1, m["H"], max_len, m["D"]], "float32")
                new_ops.append(_new(gb.block, "fill_constant_batch_size_like", {"Input": [m["x"]]},
                                    {"Out": [cache]},
                                    {"shape": [2, -1, m["H"], max_len, m["D"]], "input_dim_idx": 0,
                                     "output_dim_idx": 1, "value": 0.0, "dtype": 5}))
                cmap[m["k"]], cmap[m["v"]] = (cache, 0), (cache, 1)
            _splice(gb, m, new_ops + [_fmt_op(gb, m, f"enc{n}", cache, None, mp)])
            if new_ops:
                fills.setdefault(id(gb.block), (gb, m["x"], []))[2].append(new_ops[0])
            if cache is not None:
                for t in (m["k"], m["v"]):
                    _rename_everywhere(g.program, t, cache)
            n += 1
    for gb, x0, fl in fills.values():
        # every cache buffer is created up front from the FIRST fused layer's input (batch size
        # only), so consecutive fused layers stay adjacent for fuse_multi_transformer_layer_pass
        first = min(gb.ops.index(o) for o in gb.ops if o.type == "fused_multi_transformer")
        for f in fl:
            f.paddle_inputs["Input"] = [x0]
            gb.ops.remove(f)
        first = min(gb.ops.index(o) for o in gb.ops if o.type == "fused_multi_transformer")
        for f in reversed(fl):
            gb.ops.insert(first, f)
    for gb, m in decs:
        if any(o not in gb.ops for o in m["ops"]):
            continue
        ck, cv = m["cache"]
        if ck in cmap and cv in cmap and cmap[ck][0] == cmap[cv][0]:
            _rewrite_decoder(gb, m, cmap[ck][0], n, mp)
            n += 1
    return n


fused_multi_transformer_encoder_pass_ops = lambda g: _fuse(g, False, False)  # noqa: E731
fused_multi_transformer_encoder_fuse_qkv_pass = lambda g: _fuse(g, True, False)  # noqa: E731
fused_multi_transformer_decoder_pass = lambda g: _fuse(g, False, False, encoders=False)  # noqa: E731
fused_multi_transformer_decoder_fuse_qkv_pass = lambda g: _fuse(g, True, False, encoders=False)  # noqa: E731
multi_devices_fused_multi_transformer_encoder_fuse_qkv_pass = lambda g: _fuse(g, True, True)  # noqa: E731
multi_devices_fused_multi_transformer_decoder_fuse_qkv_pass = lambda g: _fuse(g, True, True, encoders=False)  # noqa: E731

# reference order (paddle_pass_builder.cc GpuPassStrategy): encoder passes, then decoder passes
PASS_ORDER = [
    "fused_multi_transformer_encoder_pass", "fused_multi_transformer_decoder_pass",
    "fused_multi_transformer_encoder_fuse_qkv_pass", "fused_multi_transformer_decoder_fuse_qkv_pass",
    "multi_devices_fused_multi_transformer_encoder_fuse_qkv_pass",
    "multi_devices_fused_multi_transformer_decoder_fuse_qkv_pass",
]
