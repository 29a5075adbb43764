"""Program op types that exported Paddle models carry beyond ``ops_registry`` / ``_ext``: the fused
training / inference blocks (``fused_attention``, ``fused_feedforward``,
``fused_bias_dropout_residual_layer_norm``, ``fused_bn_add_activation``, ``resnet_unit``), the
cuDNN-style ``rnn`` op, 3-D conv / pooling, ``grid_sampler`` and the detection set (``yolo_box``,
``multiclass_nms3`` / ``multiclass_nms``, ``roi_align``, ``prior_box``, ``box_coder``).

Slot and attribute names follow the reference op makers (`paddle/fluid/operators/fused/
fused_attention_op.cc:718`, `fused_feedforward_op.cc:428`,
`fused_bias_dropout_residual_layer_norm_op.cc:252`, `fused_bn_add_activation_op.cc:290`,
`resnet_unit_op.cc:470`, `rnn_op.cc:196`, `grid_sampler_op.cc`, `detection/yolo_box_op.cc:257`,
`detection/multiclass_nms_op.cc:639`, `roi_align_op.cc`, `detection/prior_box_op.cc`). Every kernel
is a differentiable composition of the framework's ops, so the ``<type>_grad`` OpDescs that
``append_backward`` emits for them run as the VJP of the forward (`static/executor.py`
``_run_grad_op``): static training through these ops needs no separate grad kernel. Intermediate
outputs the reference keeps for its hand-written grad kernels (LnMean, Dropout masks, QKOut, …)
are not materialised.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .ops_registry import register


def _one(ins, slot, default=None):
    v = ins.get(slot)
    return v[0] if v else default


def _drop_mode(a, key="dropout_implementation"):
    m = a.get(key, "downgrade_in_infer") or "downgrade_in_infer"
    return "downscale_in_infer" if m == "downgrade_in_infer" else m


def _training(a):
    return not bool(a.get("is_test", False))


# ------------------------------------------------------------------------------- fused blocks
@register("fused_attention")
def _fused_attention(ins, a):
    """Reference `fused_attention_op.cc`: X [B, S, E], QKVW [3, H, D, E], pre / post LayerNorm,
    SrcMask, optional CacheKV [2, B, H, S_cache, D] (→ CacheKVOut), residual + dropouts."""
    from ..incubate.nn import functional as IF
    x, qkvw = ins["X"][0], ins["QKVW"][0]
    H = qkvw.shape[1]
    tr = _training(a)
    res = IF.fused_multi_head_attention(
        x, qkvw, ins["OutLinearW"][0], pre_layer_norm=bool(a.get("pre_layer_norm", False)),
        pre_ln_scale=_one(ins, "LnScale"), pre_ln_bias=_one(ins, "LnBias"),
        ln_scale=_one(ins, "Ln2Scale"), ln_bias=_one(ins, "Ln2Bias"),
        pre_ln_epsilon=float(a.get("epsilon", 1e-5)), qkv_bias=_one(ins, "QKVBias"),
        linear_bias=_one(ins, "OutLinearBias"), cache_kv=_one(ins, "CacheKV"),
        attn_mask=_one(ins, "SrcMask"), dropout_rate=float(a.get("dropout_rate", 0.5)),
        attn_dropout_rate=float(a.get("attn_dropout_rate", 0.5)),
        ln_epsilon=float(a.get("ln_epsilon", 1e-5)), training=tr,
        mode=_drop_mode(a, "attn_dropout_implementation"),
        add_residual=bool(a.get("add_residual", True)), num_heads=H)
    if isinstance(res, tuple):
        return {"Y": res[0], "CacheKVOut": res[1]}
    return {"Y": res}


@register("fused_feedforward")
def _fused_feedforward(ins, a):
    """Reference `fused_feedforward_op.cc`: Out = residual + dropout2(linear2(dropout1(
    act(linear1(LN1?(X)))))) with LN2 after the residual when not pre_layer_norm."""
    from ..incubate.nn import functional as IF
    out = IF.fused_feedforward(
        ins["X"][0], ins["Linear1Weight"][0], ins["Linear2Weight"][0], _one(ins, "Linear1Bias"),
        _one(ins, "Linear2Bias"), _one(ins, "Ln1Scale"), _one(ins, "Ln1Bias"), _one(ins, "Ln2Scale"),
        _one(ins, "Ln2Bias"), dropout1_rate=float(a.get("dropout1_rate", 0.5)),
        dropout2_rate=float(a.get("dropout2_rate", 0.5)), activation=a.get("act_method", "relu"),
        ln1_epsilon=float(a.get("ln1_epsilon", 1e-5)), ln2_epsilon=float(a.get("ln2_epsilon", 1e-5)),
        pre_layer_norm=bool(a.get("pre_layer_norm", False)), training=_training(a),
        mode=_drop_mode(a, "dropout1_implementation"), add_residual=bool(a.get("add_residual", True)))
    return {"Out": out}


@register("fused_bias_dropout_residual_layer_norm")
def _fused_bdrln(ins, a):
    """Reference `fused_bias_dropout_residual_layer_norm_op.cc`: Y = LN(Residual + dropout(X + Bias))."""
    from ..incubate.nn import functional as IF
    y = IF.fused_bias_dropout_residual_layer_norm(
        ins["X"][0], ins["Residual"][0], _one(ins, "Bias"), _one(ins, "LnScale"), _one(ins, "LnBias"),
        dropout_rate=float(a.get("dropout_rate", 0.5)), ln_epsilon=float(a.get("ln_epsilon", 1e-5)),
        training=_training(a), mode=_drop_mode(a))
    return {"Y": y}


def _bn_act(x, scale, bias, mean, var, momentum, eps, act, residual, data_format, training):
    from ..ops.batchnorm import batch_norm_act
    rm = mean if mean is not None else torch.zeros(x.shape[1 if data_format == "NCHW" else -1],
                                                   device=x.device, dtype=torch.float32)
    rv = var if var is not None else torch.ones_like(rm)
    return batch_norm_act(x, rm, rv, scale, bias, training=training, momentum=momentum, epsilon=eps,
                          act=act, residual=residual, data_format=data_format), rm, rv


@register("fused_bn_add_activation")
def _fused_bn_add_act(ins, a):
    """Reference `fused_bn_add_activation_op.cc` (NHWC, training BN): Y = act(BN(X) + Z), running
    statistics updated in place (MeanOut / VarianceOut alias Mean / Variance)."""
    x, z = ins["X"][0], ins["Z"][0]
    y, rm, rv = _bn_act(x, _one(ins, "Scale"), _one(ins, "Bias"), _one(ins, "Mean"),
                        _one(ins, "Variance"), float(a.get("momentum", 0.9)),
                        float(a.get("epsilon", 1e-5)), a.get("act_type", "relu") or "none", z,
                        "NHWC", True)
    return {"Y": y, "MeanOut": rm, "VarianceOut": rv}


@register("resnet_unit")
def _resnet_unit(ins, a):
    """Reference `resnet_unit_op.cc`: Y = act(BN(conv(X, FilterX)) + [BN(conv(Z, FilterZ)) |
    Z | 0]) — the conv + BN (+ shortcut conv + BN) + add + ReLU of a ResNet block, NHWC or NCHW,
    on the framework's conv kernels and the fused BN-residual-activation kernel."""
    from ..nn import functional as PF
    fmt = a.get("data_format", "NHWC") or "NHWC"
    train = _training(a) and not bool(a.get("use_global_stats", False))
    mom, eps = float(a.get("momentum", 0.9)), float(a.get("epsilon", 1e-5))
    act = a.get("act_type", "relu") or "none"
    st, pad, dil, grp = int(a.get("stride", 1)), int(a.get("padding", 0)), int(a.get("dilation", 1)), int(a.get("group", 1))

    def conv(x, w, stride):
        return PF.conv2d(x, w, None, stride, pad, dil, grp, data_format=fmt)
    x = ins["X"][0]
    cx = conv(x, ins["FilterX"][0], st)
    res = None
    outs = {"ConvX": cx}
    if a.get("has_shortcut", False):
        cz = conv(ins["Z"][0], ins["FilterZ"][0], int(a.get("stride_z", 1)))
        res, rmz, rvz = _bn_act(cz, _one(ins, "ScaleZ"), _one(ins, "BiasZ"), _one(ins, "MeanZ"),
                                _one(ins, "VarZ"), mom, eps, "none", None, fmt, train)
        outs.update(ConvZ=cz, RunningMeanZ=rmz, RunningVarZ=rvz)
    elif a.get("fuse_add", False):
        res = ins["Z"][0]
    y, rmx, rvx = _bn_act(cx, _one(ins, "ScaleX"), _one(ins, "BiasX"), _one(ins, "MeanX"),
                          _one(ins, "VarX"), mom, eps, act, res, fmt, train)
    outs.update(Y=y, RunningMeanX=rmx, RunningVarX=rvx)
    return outs


# ------------------------------------------------------------------------------- rnn
def _rnn_cell(mode, gx, h, c, w_hh, b_hh):
    """One step from the precomputed input projection gx = x_t·W_ihᵀ + b_ih."""
    from ..ops.gemm import matmul
    gh = matmul(h, w_hh, False, True)
    if b_hh is not None:
        gh = gh + b_hh
    if mode == "GRU":  # reset gate applied after the hidden projection (reference GRUCell)
        xr, xz, xc = gx.chunk(3, -1)
        hr, hz, hc = gh.chunk(3, -1)
        r, z = torch.sigmoid(xr + hr), torch.sigmoid(xz + hz)
        cc = torch.tanh(xc + r * hc)
        return (h - cc) * z + cc, None
    g = gx + gh
    if mode == "LSTM":
        i, f, gg, o = g.chunk(4, -1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        return torch.sigmoid(o) * torch.tanh(c), c
    return (torch.relu(g) if mode == "RNN_RELU" else torch.tanh(g)), None


@register("rnn")
def _rnn(ins, a):
    """Reference `rnn_op.cc` (cuDNN-layout RNN): Input [T, B, I] time-major; WeightList = all
    w_ih / w_hh of (layer, direction) pairs, then all b_ih / b_hh; PreState = [h0] or [h0, c0]
    ([L·D, B, H]); SequenceLength [B]: padded steps output 0 and leave the state unchanged (the
    reverse direction starts at each sequence's own last step). Out [T, B, D·H], State alike."""
    x = ins["Input"][0]
    mode = a.get("mode", "LSTM")
    L, Hs = int(a.get("num_layers", 1)), int(a.get("hidden_size"))
    D = 2 if a.get("is_bidirec", False) else 1
    ws = ins["WeightList"]
    nw = 2 * L * D
    has_b = len(ws) >= 2 * nw
    pre = ins.get("PreState") or []
    T, B = x.shape[0], x.shape[1]
    seq = _one(ins, "SequenceLength")
    lens = seq.to(x.device).long() if seq is not None else torch.full((B,), T, device=x.device, dtype=torch.long)
    h0 = pre[0] if pre else x.new_zeros(L * D, B, Hs)
    c0 = pre[1] if len(pre) > 1 else (x.new_zeros(L * D, B, Hs) if mode == "LSTM" else None)
    p_drop = float(a.get("dropout_prob", 0.0) or 0.0)
    train = _training(a)
    bi = torch.arange(B, device=x.device)
    from ..ops.gemm import matmul
    inp = x
    hN, cN = [], []
    for layer in range(L):
        outs = []
        for d in range(D):
            k = layer * D + d
            w_ih, w_hh = ws[2 * k], ws[2 * k + 1]
            b_ih, b_hh = (ws[nw + 2 * k], ws[nw + 2 * k + 1]) if has_b else (None, None)
            h, c = h0[k], (c0[k] if c0 is not None else None)
            # the input projection of every step as ONE GEMM ([T·B, I]·W_ihᵀ); only the hidden
            # projection stays inside the time loop
            gx_all = matmul(inp.reshape(T * B, -1), w_ih, False, True).view(T, B, -1)
            if b_ih is not None:
                gx_all = gx_all + b_ih
            y = x.new_zeros(T, B, Hs)
            for s_ in range(T):
                # forward: position s_; reverse: each sequence walked back from its own last step
                src = torch.full_like(lens, s_) if d == 0 else lens - 1 - s_
                m = (src >= 0) & (src < lens)
                srcc = src.clamp(0, T - 1)
                hn, cn = _rnn_cell(mode, gx_all[srcc, bi], h, c, w_hh, b_hh)
                mk = m[:, None]
                h = torch.where(mk, hn, h)
                if c is not None:
                    c = torch.where(mk, cn, c)
                # masked write without a host sync: inactive rows write back their current value
                # ((srcc, b) pairs are distinct within a step; a later real write overrides)
                y.index_put_((srcc, bi), torch.where(mk, hn.to(y.dtype), y[srcc, bi]))
            outs.append(y)
            hN.append(h)
            if c is not None:
                cN.append(c)
        inp = torch.cat(outs, -1) if D == 2 else outs[0]
        if train and p_drop > 0 and layer < L - 1:
            inp = F.dropout(inp, p_drop, True)
    state = [torch.stack(hN)] + ([torch.stack(cN)] if mode == "LSTM" else [])
    return {"Out": inp, "State": state}


# ------------------------------------------------------------------------------- 3-D conv / pool
def _trip(v, n=3):
    v = list(v) if isinstance(v, (list, tuple)) else [v] * n
    return v if len(v) == n else [v[0]] * n


def _pad3(a):
    p = list(a.get("paddings") or [0, 0, 0])
    if len(p) == 6:
        if p[0::2] == p[1::2]:
            return p[0::2]
        return ("explicit", p)
    return _trip(p)


@register("conv3d")
def _conv3d(ins, a):
    """Reference `conv_op.cc` conv3d (NCDHW / NDHWC)."""
    x, w = ins["Input"][0], ins["Filter"][0]
    ndhwc = a.get("data_format", "NCDHW") in ("NDHWC", "NHWC")
    if ndhwc:
        x = x.permute(0, 4, 1, 2, 3)
    pad = _pad3(a)
    if a.get("padding_algorithm", "EXPLICIT") == "SAME":
        pad = "same"
    elif a.get("padding_algorithm", "EXPLICIT") == "VALID":
        pad = 0
    if isinstance(pad, tuple):
        p = pad[1]
        x = F.pad(x, (p[4], p[5], p[2], p[3], p[0], p[1]))
        pad = 0
    y = F.conv3d(x, w, _one(ins, "Bias"), _trip(a.get("strides", 1)), pad, _trip(a.get("dilations", 1)),
                 int(a.get("groups", 1) or 1))
    return {"Output": y.permute(0, 2, 3, 4, 1) if ndhwc else y}


@register("conv3d_transpose")
def _conv3d_t(ins, a):
    x, w = ins["Input"][0], ins["Filter"][0]
    ndhwc = a.get("data_format", "NCDHW") in ("NDHWC", "NHWC")
    if ndhwc:
        x = x.permute(0, 4, 1, 2, 3)
    pad = _pad3(a)
    pad = pad[1][0::2] if isinstance(pad, tuple) else pad
    y = F.conv_transpose3d(x, w, _one(ins, "Bias"), _trip(a.get("strides", 1)), pad,
                           _trip(a.get("output_padding") or 0), int(a.get("groups", 1) or 1),
                           _trip(a.get("dilations", 1)))
    return {"Output": y.permute(0, 2, 3, 4, 1) if ndhwc else y}


@register("pool3d")
def _pool3d(ins, a):
    """Reference `pool_op.cc` pool3d: max / avg, global / adaptive, exclusive averaging."""
    x = ins["X"][0]
    ndhwc = a.get("data_format", "NCDHW") in ("NDHWC", "NHWC")
    if ndhwc:
        x = x.permute(0, 4, 1, 2, 3)
    typ = a.get("pooling_type", "max")
    ks = _trip(a.get("ksize", [1, 1, 1]))
    if a.get("global_pooling", False):
        y = F.adaptive_max_pool3d(x, 1) if typ == "max" else F.adaptive_avg_pool3d(x, 1)
    elif a.get("adaptive", False):
        y = F.adaptive_max_pool3d(x, ks) if typ == "max" else F.adaptive_avg_pool3d(x, ks)
    else:
        pad = _pad3(a)
        pad = pad[1][0::2] if isinstance(pad, tuple) else pad
        st = _trip(a.get("strides", ks))
        ceil = bool(a.get("ceil_mode", False))
        if typ == "max":
            y = F.max_pool3d(x, ks, st, pad, ceil_mode=ceil)
        else:
            y = F.avg_pool3d(x, ks, st, pad, ceil_mode=ceil,
                             count_include_pad=not bool(a.get("exclusive", True)))
    return {"Out": y.permute(0, 2, 3, 4, 1) if ndhwc else y}


@register("grid_sampler")
def _grid_sampler(ins, a):
    """Reference `grid_sampler_op.cc` / phi grid_sample: X [N, C, H, W], Grid [N, Ho, Wo, 2]."""
    x, g = ins["X"][0], ins["Grid"][0]
    y = F.grid_sample(x, g.to(x.dtype), mode=a.get("mode", "bilinear") or "bilinear",
                      padding_mode=a.get("padding_mode", "zeros") or "zeros",
                      align_corners=bool(a.get("align_corners", True)))
    return {"Output": y}


# ------------------------------------------------------------------------------- detection
@register("yolo_box")
def _yolo_box(ins, a):
    from ..vision.ops import yolo_box
    boxes, scores = yolo_box(ins["X"][0], ins["ImgSize"][0], list(a["anchors"]), int(a["class_num"]),
                             float(a.get("conf_thresh", 0.01)), int(a["downsample_ratio"]),
                             bool(a.get("clip_bbox", True)), scale_x_y=float(a.get("scale_x_y", 1.0)),
                             iou_aware=bool(a.get("iou_aware", False)),
                             iou_aware_factor=float(a.get("iou_aware_factor", 0.5)))
    return {"Boxes": boxes, "Scores": scores}


@register("multiclass_nms3", "multiclass_nms2", "multiclass_nms")
def _multiclass_nms(ins, a):
    from ..vision.ops import multiclass_nms
    out, index, num = multiclass_nms(
        ins["BBoxes"][0], ins["Scores"][0], float(a.get("score_threshold", 0.05)),
        int(a.get("nms_top_k", -1)), int(a.get("keep_top_k", -1)), float(a.get("nms_threshold", 0.3)),
        bool(a.get("normalized", True)), float(a.get("nms_eta", 1.0)),
        int(a.get("background_label", 0)), _one(ins, "RoisNum"))
    return {"Out": out, "Index": index, "NmsRoisNum": num}


@register("roi_align")
def _roi_align(ins, a):
    from ..vision.ops import roi_align
    x, rois = ins["X"][0], ins["ROIs"][0]
    num = _one(ins, "RoisNum")
    if num is None:
        num = torch.tensor([rois.shape[0]], dtype=torch.int32)
    out = roi_align(x, rois, num, (int(a.get("pooled_height", 1)), int(a.get("pooled_width", 1))),
                    float(a.get("spatial_scale", 1.0)), int(a.get("sampling_ratio", -1)),
                    bool(a.get("aligned", False)))
    return {"Out": out}


@register("prior_box")
def _prior_box(ins, a):
    from ..vision.ops import prior_box
    b, v = prior_box(ins["Input"][0], ins["Image"][0], list(a.get("min_sizes", [])),
                     list(a.get("max_sizes", []) or []), list(a.get("aspect_ratios", [1.0]) or [1.0]),
                     list(a.get("variances", [0.1, 0.1, 0.2, 0.2])), bool(a.get("flip", False)),
                     bool(a.get("clip", False)), (float(a.get("step_w", 0.0)), float(a.get("step_h", 0.0))),
                     float(a.get("offset", 0.5)), bool(a.get("min_max_aspect_ratios_order", False)))
    return {"Boxes": b, "Variances": v}


@register("box_coder")
def _box_coder(ins, a):
    from ..vision.ops import box_coder
    pv = _one(ins, "PriorBoxVar")
    if pv is None:
        pv = torch.tensor(list(a.get("variance") or [1.0, 1.0, 1.0, 1.0]))
    out = box_coder(ins["PriorBox"][0], pv, ins["TargetBox"][0], a.get("code_type", "encode_center_size"),
                    bool(a.get("box_normalized", True)), int(a.get("axis", 0)))
    return {"OutputBox": out}


math  # noqa
