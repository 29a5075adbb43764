"""Program op types of exported / static-training models beyond the other registries:

* QAT / PTQ quantization: ``quantize_linear`` / ``dequantize_linear`` (PaddleSlim's ONNX-style
  export, reference `paddle/fluid/operators/quantize_linear_op.cc:200,209`, kernels
  `quantize_linear_op.h`) and the older fake-quant family (`fake_quantize_op.cc`,
  `fake_dequantize_op.cc`): ``fake_quantize_dequantize_abs_max``,
  ``fake_quantize_dequantize_moving_average_abs_max``,
  ``fake_channel_wise_quantize_dequantize_abs_max``, ``fake_dequantize_max_abs``,
  ``fake_channel_wise_dequantize_max_abs``, ``moving_average_abs_max_scale``. The weight side of
  an exported QAT model (int8 weight → ``dequantize_linear`` → matmul) is folded at load time by
  ``inference/passes_quant.py`` into the int8 weight-only MFMA GEMM.
* ``fused_batch_norm_act`` (`fused/fused_bn_activation_op.cc:342`): Y = act(BN(X)), NHWC, on the
  fused BN-activation HIP kernel (`ops/batchnorm.py batch_norm_act`).
* ``c_softmax_with_cross_entropy`` (+ ``_grad``) (`collective/c_softmax_with_cross_entropy_op.cc:191`,
  `.cu`): vocab-parallel softmax cross-entropy of a static tensor-parallel program; the loss
  statistics run on ``xent.hip`` and are all-reduced over the ``ring_id`` group.
* ``fused_gate_attention`` (`fused/fused_gate_attention_op.cc:337`): AlphaFold-style gated
  attention (Q/K/V projections, mask + non-batched bias, softmax, sigmoid gate, output projection)
  on the framework's GEMMs and flash attention.
* ``beam_search`` / ``beam_search_decode`` (`beam_search_op.cc:142`, `beam_search_decode_op.cc:106`,
  algorithm `operators/math/beam_search.cc`, `beam_search_decode_op_def.h`): LoD beam search over
  packed tensors carrying ``.lod`` (the framework's LoD convention, `static/nn_extra.py`).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from .ops_registry import register
from .grad_kernels import register_grad


def _one(ins, slot, default=None):
    v = ins.get(slot)
    return v[0] if v else default


# ------------------------------------------------------------------------------ quantization
def _round(x, round_type):
    """round_type 0: nearest, ties to even (torch.round); 1: nearest, ties away from zero."""
    if int(round_type) == 0:
        return torch.round(x)
    return torch.sign(x) * torch.floor(x.abs() + 0.5)


def _inv(s):
    """Reference `fake_quantize_op.cu.h` inverse(): 1/(s+1e-6) for s ≤ 1e-30, else 1/s."""
    return torch.where(s <= 1e-30, 1.0 / (s + 1e-6), 1.0 / s)


def _chan_view(s, x, axis):
    shape = [1] * x.dim()
    shape[axis] = -1
    return s.reshape(shape)


def _quant(x, s, bin_cnt, round_type):
    """Integer grid values (as floats) of x at scale s (s broadcastable to x)."""
    xf = x.float()
    s = s.float()
    if int(round_type) == 0:
        q = _round(bin_cnt * _inv(s) * xf, 0)
        return q.clamp(-bin_cnt - 1, bin_cnt)
    v = torch.minimum(torch.maximum(xf, -s), s)
    return _round(bin_cnt * _inv(s) * v, 1)


def _abs_max_channel(x, axis):
    dims = [d for d in range(x.dim()) if d != axis]
    return x.float().abs().amax(dim=dims)


def _moving_scale(x, ins, a):
    """FindMovingAverageAbsMaxFunctor: state = r·state + 1, accum = r·accum + max|x|,
    scale = accum / state (InState / InAccum optional: a fresh start)."""
    r = float(a.get("moving_rate", 0.9))
    cur = x.float().abs().max()
    st0, ac0 = _one(ins, "InState"), _one(ins, "InAccum")
    st = r * (st0.float().reshape(()) if st0 is not None else torch.zeros((), device=x.device)) + 1.0
    ac = r * (ac0.float().reshape(()) if ac0 is not None else torch.zeros((), device=x.device)) + cur
    return (ac / st).reshape(1), st.reshape(1), ac.reshape(1)


@register("quantize_linear")
def _quantize_linear(ins, a):
    """Y = clamp(round(x·bin/scale)) with bin = 2^(bit_length−1) − 1, per tensor (quant_axis −1)
    or per channel; is_test=False computes the scale (moving-average abs-max / channel abs-max)
    and reports it in OutScale (+ OutState / OutAccum). Y keeps X's float dtype."""
    x = ins["X"][0]
    bits = int(a.get("bit_length", 8))
    bin_cnt = float(2 ** (bits - 1) - 1)
    axis = int(a.get("quant_axis", 0))
    rt = int(a.get("round_type", 0))
    test = bool(a.get("is_test", True))
    outs = {}
    if axis < 0:
        if test:
            s = ins["Scale"][0].float().reshape(())
        else:
            sc, st, ac = _moving_scale(x, ins, a)
            s = sc.reshape(())
            outs.update(OutScale=sc, OutState=st, OutAccum=ac)
        y = _quant(x, s, bin_cnt, rt)
    else:
        s = ins["Scale"][0].float().reshape(-1) if test else _abs_max_channel(x, axis)
        if not test:
            outs["OutScale"] = s
        y = _quant(x, _chan_view(s, x, axis), bin_cnt, rt)
    outs["Y"] = y.to(x.dtype) if x.is_floating_point() else y
    return outs


@register("dequantize_linear")
def _dequantize_linear(ins, a):
    """Y = X · scale / (2^(bit_length−1) − 1), per tensor or along quant_axis; X may be int8
    (exported weights) or float grid values; Y is float32 (or X's float dtype)."""
    x = ins["X"][0]
    bits = int(a.get("bit_length", 8))
    rng = float(2 ** (bits - 1) - 1)
    axis = int(a.get("quant_axis", 0))
    s = ins["Scale"][0].float()
    xf = x.float()
    if axis < 0 or s.numel() == 1:
        y = xf * s.reshape(()) / rng
    else:
        if s.numel() != x.shape[axis]:
            raise ValueError(f"dequantize_linear: {s.numel()} scales for axis {axis} of {tuple(x.shape)}")
        y = xf * _chan_view(s, x, axis) / rng
    return {"Y": y.to(x.dtype) if x.is_floating_point() else y}


@register("fake_quantize_dequantize_abs_max")
def _fqd_abs_max(ins, a):
    x = ins["X"][0]
    bin_cnt = float(2 ** (int(a.get("bit_length", 8)) - 1) - 1)
    s = x.float().abs().max()
    q = _quant(x, s, bin_cnt, a.get("round_type", 1))
    return {"Out": (q * s / bin_cnt).to(x.dtype), "OutScale": s.reshape(1)}


@register("fake_quantize_dequantize_moving_average_abs_max")
def _fqd_mavg(ins, a):
    x = ins["X"][0]
    bin_cnt = float(2 ** (int(a.get("bit_length", 8)) - 1) - 1)
    outs = {}
    if bool(a.get("is_test", False)):
        s = ins["InScale"][0].float().reshape(())
    else:
        sc, st, ac = _moving_scale(x, ins, a)
        s = sc.reshape(())
        outs.update(OutState=st, OutAccum=ac)
    outs["OutScale"] = s.reshape(1)
    q = _quant(x, s, bin_cnt, a.get("round_type", 1))
    outs["Out"] = (q * s / bin_cnt).to(x.dtype)
    return outs


@register("fake_channel_wise_quantize_dequantize_abs_max")
def _fcqd(ins, a):
    x = ins["X"][0]
    bin_cnt = float(2 ** (int(a.get("bit_length", 8)) - 1) - 1)
    axis = int(a.get("quant_axis", 0))
    s = _abs_max_channel(x, axis)
    sv = _chan_view(s, x, axis)
    q = _quant(x, sv, bin_cnt, a.get("round_type", 1))
    return {"Out": (q * sv / bin_cnt).to(x.dtype), "OutScale": s}


@register("moving_average_abs_max_scale")
def _mavg_scale(ins, a):
    x = ins["X"][0]
    outs = {"Out": x}
    if not bool(a.get("is_test", False)):
        sc, st, ac = _moving_scale(x, ins, a)
        outs.update(OutScale=sc, OutState=st, OutAccum=ac)
    return outs


@register("fake_dequantize_max_abs")
def _fdq_max_abs(ins, a):
    x = ins["X"][0]
    return {"Out": x.float() * ins["Scale"][0].float().reshape(()) / float(a.get("max_range", 127.0))}


@register("fake_channel_wise_dequantize_max_abs")
def _fcdq(ins, a):
    """Out = X · scale_0[c] (· scale_1) / (range_0 (· range_1)), range_i = 2^(bits_i − 1) − 1."""
    x = ins["X"][0].float()
    scales = ins["Scales"]
    bits = list(a.get("quant_bits", [8] * len(scales)))
    axis = int(a.get("quant_axis", 0))
    y = x * _chan_view(scales[0].float(), x, axis) / float(2 ** (bits[0] - 1) - 1)
    if len(scales) > 1:
        y = y * scales[1].float().reshape(()) / float(2 ** (bits[1] - 1) - 1)
    return {"Out": y}


# ------------------------------------------------------------------------------ fused BN + act
@register("fused_batch_norm_act")
def _fused_bn_act(ins, a):
    """Reference `fused_bn_activation_op.cc` (NHWC): Y = act(BN(X)); training statistics by
    default (the op is a training fusion), running mean / variance updated in place and returned
    as MeanOut / VarianceOut; SavedMean / SavedVariance are the batch statistics (1/σ form)."""
    from .ops_registry_more import _bn_act
    x = ins["X"][0]
    training = not bool(a.get("is_test", False))
    act = a.get("act_type", "relu") or "none"
    eps = float(a.get("epsilon", 1e-5))
    outs = {}
    if training:
        dims = tuple(range(x.dim() - 1))
        xf = x.detach().float()
        mu = xf.mean(dims)
        var = xf.var(dims, unbiased=False)
        outs["SavedMean"] = mu
        outs["SavedVariance"] = torch.rsqrt(var + eps)
    y, rm, rv = _bn_act(x, _one(ins, "Scale"), _one(ins, "Bias"), _one(ins, "Mean"), _one(ins, "Variance"),
                        float(a.get("momentum", 0.9)), eps, act, None, "NHWC", training)
    outs.update(Y=y, MeanOut=rm, VarianceOut=rv)
    return outs


# ------------------------------------------------------------------------------ vocab-parallel CE
def _group(a):
    from .ops_registry import _ring_group
    nranks = int(a.get("nranks", 1) or 1)
    if nranks <= 1:
        return None
    return _ring_group({"ring_id": a.get("ring_id", 0)})


@register("c_softmax_with_cross_entropy")
def _c_softmax_xent(ins, a):
    """Logits [N.., V/nranks] (this rank's vocab slice, rank r owning [r·V_local, (r+1)·V_local)),
    Label [N.., 1] → Softmax (globally normalised slice) and Loss [N.., 1]; ignore_index rows give 0."""
    from ..ops.loss import vocab_parallel_softmax_xent
    logits, label = ins["Logits"][0], ins["Label"][0]
    ig = int(a.get("ignore_index", -100))
    softmax, loss = vocab_parallel_softmax_xent(logits, label.reshape(logits.shape[:-1]), ig, _group(a),
                                                rank=int(a.get("rank", 0)))
    return {"Softmax": softmax, "Loss": loss.unsqueeze(-1)}


@register_grad("c_softmax_with_cross_entropy_grad")
def _c_softmax_xent_grad(ins, a):
    """Logits@GRAD = (Softmax − onehot_local(Label)) · Loss@GRAD (reference
    `c_softmax_with_cross_entropy_op.cu` CaculateSoftmaxWithCrossEntropyGrad)."""
    sm = _one(ins, "Softmax")
    lab = _one(ins, "Label")
    dl = _one(ins, "Loss@GRAD")
    V = sm.shape[-1]
    rank = int(a.get("rank", 0))
    ig = int(a.get("ignore_index", -100))
    start = rank * V
    lab2 = lab.reshape(-1).long()
    d = dl.reshape(-1).float() if dl is not None else torch.ones(lab2.shape, device=sm.device)
    d = torch.where(lab2 == ig, torch.zeros_like(d), d)
    g = sm.reshape(-1, V).float() * d[:, None]
    inr = (lab2 >= start) & (lab2 < start + V)
    rows = torch.nonzero(inr).reshape(-1)
    g[rows, lab2[rows] - start] -= d[rows]
    return {"Logits@GRAD": g.reshape(sm.shape).to(sm.dtype)}


# ------------------------------------------------------------------------------ gated attention
def _proj(x, w2d):
    """x [..., K] · w2d [K, N] on the framework's GEMM dispatcher (own kernels for 16-bit)."""
    from ..ops.gemm import matmul
    return matmul(x.reshape(-1, x.shape[-1]), w2d).reshape(*x.shape[:-1], w2d.shape[-1])


@register("fused_gate_attention")
def _fused_gate_attention(ins, a):
    """Query [B, M, R, Qd] (Key [B, M, Mk, Kd] unless merge_qkv) → Out [B, M, R, O]:
    q,k,v = projections ([3, H, D, Qd] QKVWeight or [Qd, H, D] weights), logits = q·kᵀ/√D +
    SrcMask [B, M, 1, 1, Mk] (+ NonbatchedBias [B, H, R, Mk]), softmax, ·v; gate = sigmoid(Query ·
    GateWeight + GateBias) ⊙ that; Out = gate · OutLinearWeight [H, D, O] + OutLinearBias.
    The attention runs as ONE flash-attention call over the B·M rows with the mask and bias as an
    additive mask."""
    from ..ops.attention import flash_attention
    q_in = ins["Query"][0]
    B, Mm, R, Qd = q_in.shape
    merge = bool(a.get("merge_qkv", True))
    if merge:
        w = ins["QKVWeight"][0]  # [3, H, D, Qd]
        _, H, D, _ = w.shape
        qkv = _proj(q_in, w.reshape(3 * H * D, Qd).t())
        q, k, v = qkv.reshape(B, Mm, R, 3, H, D).unbind(3)
        Mk = R
    else:
        k_in = ins["Key"][0]
        wq, wk, wv = ins["QueryWeight"][0], ins["KeyWeight"][0], ins["ValueWeight"][0]
        H, D = wq.shape[1], wq.shape[2]
        Mk = k_in.shape[2]
        q = _proj(q_in, wq.reshape(Qd, H * D)).reshape(B, Mm, R, H, D)
        k = _proj(k_in, wk.reshape(k_in.shape[-1], H * D)).reshape(B, Mm, Mk, H, D)
        v = _proj(k_in, wv.reshape(k_in.shape[-1], H * D)).reshape(B, Mm, Mk, H, D)
    mask = ins["SrcMask"][0].reshape(B, Mm, 1, 1, Mk).to(torch.float32)
    nb = _one(ins, "NonbatchedBias")
    if nb is not None:
        nb = nb.reshape(B, 1, H, R, Mk).to(torch.float32)
        mask = mask + nb  # [B, M, H, R, Mk]
    mask = mask.expand(B, Mm, H, R, Mk).reshape(B * Mm, H, R, Mk)
    o = flash_attention(q.reshape(B * Mm, R, H, D), k.reshape(B * Mm, Mk, H, D),
                        v.reshape(B * Mm, Mk, H, D), causal=False, scale=1.0 / math.sqrt(D),
                        attn_mask=mask.to(q.dtype) if q.dtype != torch.float32 else mask)
    fmha = o.reshape(B, Mm, R, H, D)
    outs = {"FMHAOut": fmha}
    gate = fmha
    if bool(a.get("has_gating", True)):
        gw, gb = ins["GateWeight"][0], ins["GateBias"][0]
        gv = _proj(q_in, gw.reshape(Qd, H * D)).reshape(B, Mm, R, H, D) + gb.reshape(H, D)
        gate = fmha * torch.sigmoid(gv)
        outs["GateOut"] = gate
    ow, ob = ins["OutLinearWeight"][0], ins["OutLinearBias"][0]
    out = _proj(gate.reshape(B, Mm, R, H * D), ow.reshape(H * D, -1)) + ob
    outs["Out"] = out
    return outs


# ------------------------------------------------------------------------------ LoD beam search
def _lod_of(t, name):
    lod = getattr(t, "lod", None)
    if not lod:
        raise ValueError(f"{name}: a LoD tensor (with .lod offsets) is required")
    return [list(map(int, lv)) for lv in lod]


def _abs_offsets(lod):
    """Reference `lod_tensor.cc` ToAbsOffset: every level's offsets in rows of the packed tensor."""
    out = [list(lv) for lv in lod]
    for i in range(len(out) - 2, -1, -1):
        out[i] = [out[i + 1][j] for j in out[i]]
    return out


def _with_lod(t, lod):
    t.lod = [list(lv) for lv in lod]
    return t


def beam_search_step(pre_ids, pre_scores, ids, scores, beam_size, end_id, level=0, is_accumulated=True):
    """One LoD beam-search step (reference `operators/math/beam_search.cc` BeamSearchFunctor):
    per source sequence (``scores.lod[level]``), keep the beam_size best (score, -offset) items
    among every prefix's candidates (a prefix already ending in end_id contributes itself
    once), prune sources whose every prefix and every selection is end_id, and return
    (selected_ids [n, 1] int64, selected_scores [n, 1] f32, parent_idx [n] int32) with the 2-level
    LoD [source offsets, per-prefix selection offsets]."""
    lod = _lod_of(scores, "beam_search scores")
    high = _abs_offsets(lod)[level]  # row offsets of each source (reference ToAbsOffset)
    n_rows = scores.shape[0]
    width = int(np.prod(scores.shape[1:])) if scores.dim() > 1 else 1
    sc = scores.detach().reshape(n_rows, width).float()
    pid = pre_ids.detach().reshape(-1).to(torch.int64)
    psc = pre_scores.detach().reshape(-1).float()
    idt = ids.detach().reshape(n_rows, width).to(torch.int64) if ids is not None else \
        torch.arange(width, device=sc.device).expand(n_rows, width)
    cand = sc if is_accumulated else psc[:, None] + torch.log(sc)
    ended = pid == end_id
    # an ended prefix offers exactly one item (end_id, its pre_score)
    col0 = torch.zeros(n_rows, width, dtype=torch.bool, device=sc.device)
    col0[:, 0] = True
    valid = torch.where(ended[:, None], col0, torch.ones_like(col0))
    cand = torch.where(ended[:, None], psc[:, None].expand(n_rows, width), cand)
    idt = torch.where(ended[:, None], torch.full_like(idt, end_id), idt)
    cand_h = cand.cpu().numpy()
    id_h = idt.cpu().numpy()
    valid_h = valid.cpu().numpy()
    pid_h = pid.cpu().numpy()
    per_row = [[] for _ in range(n_rows)]
    for s in range(len(high) - 1):
        r0, r1 = high[s], high[s + 1]
        if r1 <= r0:
            continue
        rows = np.repeat(np.arange(r0, r1), width)
        cols = np.tile(np.arange(width), r1 - r0)
        m = valid_h[r0:r1].reshape(-1)
        rows, cols = rows[m], cols[m]
        vals = cand_h[rows, cols]
        # reference Item order: score desc, then larger offset first; insertion order breaks ties
        order = np.lexsort((np.arange(len(vals)), -rows, -vals))[:beam_size]
        for i in order:
            per_row[rows[i]].append((int(id_h[rows[i], cols[i]]), float(vals[i])))
    # prune sources that finished (every prefix ended and selected end_id again)
    for s in range(len(high) - 1):
        r0, r1 = high[s], high[s + 1]
        fin = all(pid_h[r] == end_id and all(i == end_id for i, _ in per_row[r]) for r in range(r0, r1))
        if fin:
            for r in range(r0, r1):
                per_row[r] = []
    sel_ids, sel_sc, parent, low_lod = [], [], [], [0]
    for r in range(n_rows):
        for i, v in per_row[r]:
            sel_ids.append(i)
            sel_sc.append(v)
            parent.append(r)
        low_lod.append(len(sel_ids))
    dev = scores.device
    out_lod = [list(high), low_lod]
    si = _with_lod(torch.tensor(sel_ids, dtype=torch.int64, device=dev).reshape(-1, 1), out_lod)
    ss = _with_lod(torch.tensor(sel_sc, dtype=torch.float32, device=dev).reshape(-1, 1), out_lod)
    pi = torch.tensor(parent, dtype=torch.int32, device=dev)
    return si, ss, pi


@register("beam_search")
def _beam_search(ins, a):
    si, ss, pi = beam_search_step(ins["pre_ids"][0], ins["pre_scores"][0], _one(ins, "ids"), ins["scores"][0],
                                  int(a["beam_size"]), int(a["end_id"]), int(a.get("level", 0)),
                                  bool(a.get("is_accumulated", True)))
    return {"selected_ids": si, "selected_scores": ss, "parent_idx": pi}


def beam_search_backtrace(step_ids, step_scores, beam_size, end_id):
    """Reference `beam_search_decode_op_def.h` BeamSearchDecoder::Backtrace: walk the per-step
    LoD trees from the last step back, one hypothesis per surviving candidate (a source pruned at
    step t starts its hypotheses from step t's candidates), drop repeated end_ids, then emit each
    source's hypotheses sorted by their final score, word order restored. Returns the ids and the
    scores as 1-D tensors with the 2-level LoD [source → sentence, sentence → word]."""
    T = len(step_ids)
    lods = [_lod_of(t, "beam_search_decode Ids") for t in step_ids]
    ids_h = [t.detach().reshape(-1).cpu().numpy() for t in step_ids]
    sc_h = [t.detach().reshape(-1).float().cpu().numpy() for t in step_scores]
    n_src = len(lods[0][0]) - 1
    sents = [[] for _ in range(n_src)]  # per source: list of [word_ids(rev), scores(rev)]
    prefix = [[] for _ in range(n_src)]
    for t in range(T - 1, -1, -1):
        src_l, sen_l = lods[t][0], lods[t][1]
        for s in range(n_src):
            p0, p1 = src_l[s], src_l[s + 1]
            if not prefix[s]:
                for p in range(p0, p1):
                    for c in range(sen_l[p], sen_l[p + 1]):
                        prefix[s].append(p)
                        sents[s].append([[int(ids_h[t][c])], [float(sc_h[t][c])]])
                continue
            c_start = sen_l[p0]
            p = p0
            cnum = sen_l[p + 1] - sen_l[p]
            for j, cand in enumerate(prefix[s]):
                cid, csc = int(ids_h[t][cand]), float(sc_h[t][cand])
                if cid != end_id or not sents[s][j][0]:
                    sents[s][j][0].append(cid)
                    sents[s][j][1].append(csc)
                while c_start + cnum <= cand:
                    p += 1
                    cnum += sen_l[p + 1] - sen_l[p]
                prefix[s][j] = p
    src_lod, sen_lod, out_ids, out_sc = [0], [0], [], []
    for s in range(n_src):
        hyps = sorted(sents[s], key=lambda h: -h[1][0])  # stable, by the final (last-step) score
        for w, sc in hyps:
            out_ids.extend(reversed(w))
            out_sc.extend(reversed(sc))
            sen_lod.append(sen_lod[-1] + len(w))
        src_lod.append(src_lod[-1] + len(hyps))
    lod = [src_lod, sen_lod]
    dev = step_ids[0].device
    sdt = step_scores[0].dtype if step_scores[0].is_floating_point() else torch.float32
    return (_with_lod(torch.tensor(out_ids, dtype=torch.int64, device=dev), lod),
            _with_lod(torch.tensor(out_sc, dtype=torch.float32, device=dev).to(sdt), lod))


@register("beam_search_decode")
def _beam_search_decode(ins, a):
    ids, scores = ins["Ids"], ins["Scores"]
    if len(ids) == 1 and isinstance(ids[0], (list, tuple)):  # a LoDTensorArray value
        ids, scores = list(ids[0]), list(scores[0])
    si, ss = beam_search_backtrace(ids, scores, int(a["beam_size"]), int(a["end_id"]))
    return {"SentenceIds": si, "SentenceScores": ss}


np  # noqa
F  # noqa
