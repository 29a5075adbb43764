"""Program op types added for exported models (`static/ops_registry_more.py`) against fp32
compositions / literal transcriptions of the reference kernels: fused_attention, fused_feedforward,
fused_bias_dropout_residual_layer_norm (+ gradients, which the executor takes as the op's VJP),
fused_bn_add_activation, resnet_unit, rnn (LSTM / GRU, bidirectional, sequence lengths), conv3d /
pool3d, grid_sampler, yolo_box, multiclass_nms3, roi_align, prior_box."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from paddle_infer_amd.static.ops_registry import REGISTRY

torch.manual_seed(0)


def _r(*s, sc=0.3):
    return sc * torch.randn(*s)


def _ln(x, g, b, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), g, b, eps)


# ----------------------------------------------------------------------------- fused blocks
@pytest.mark.parametrize("pre_ln", [True, False])
def test_fused_attention(pre_ln):
    B, S, E, H = 2, 6, 32, 4
    D = E // H
    x = _r(B, S, E, sc=1.0).requires_grad_()
    qkvw = _r(3, H, D, E).requires_grad_()
    qkvb, ow, ob = _r(3, H, D), _r(E, E), _r(E)
    lns, lnb, ln2s, ln2b = 1 + _r(E), _r(E), 1 + _r(E), _r(E)
    mask = torch.zeros(B, 1, S, S)
    mask[:, :, :, -1] = -1e4
    ins = {"X": [x], "QKVW": [qkvw], "QKVBias": [qkvb], "OutLinearW": [ow], "OutLinearBias": [ob],
           "LnScale": [lns], "LnBias": [lnb], "Ln2Scale": [ln2s], "Ln2Bias": [ln2b], "SrcMask": [mask]}
    y = REGISTRY["fused_attention"](ins, {"pre_layer_norm": pre_ln, "is_test": True, "epsilon": 1e-5,
                                          "ln_epsilon": 1e-5, "dropout_rate": 0.1, "attn_dropout_rate": 0.1,
                                          "attn_dropout_implementation": "upscale_in_train"})["Y"]
    h = _ln(x, lns, lnb) if pre_ln else x
    qkv = (h @ qkvw.reshape(3 * E, E).t() + qkvb.reshape(-1)).reshape(B, S, 3, H, D)
    q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))
    a = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(D) + mask, -1) @ v
    o = a.transpose(1, 2).reshape(B, S, E) @ ow + ob
    ref = x + o if pre_ln else _ln(x + o, ln2s, ln2b)
    torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(y)
    gx, gw = torch.autograd.grad(y, (x, qkvw), g)
    rx, rw = torch.autograd.grad(ref, (x, qkvw), g)
    torch.testing.assert_close(gx, rx, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(gw, rw, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("pre_ln", [True, False])
@pytest.mark.parametrize("act", ["relu", "gelu"])
def test_fused_feedforward(pre_ln, act):
    B, S, E, FF = 2, 5, 16, 48
    x = _r(B, S, E, sc=1.0).requires_grad_()
    w1, b1, w2, b2 = _r(E, FF).requires_grad_(), _r(FF), _r(FF, E), _r(E)
    g1, be1, g2, be2 = 1 + _r(E), _r(E), 1 + _r(E), _r(E)
    ins = {"X": [x], "Linear1Weight": [w1], "Linear1Bias": [b1], "Linear2Weight": [w2],
           "Linear2Bias": [b2], "Ln1Scale": [g1], "Ln1Bias": [be1], "Ln2Scale": [g2], "Ln2Bias": [be2]}
    out = REGISTRY["fused_feedforward"](ins, {"pre_layer_norm": pre_ln, "act_method": act, "is_test": True,
                                              "dropout1_rate": 0.2, "dropout2_rate": 0.2,
                                              "dropout1_implementation": "upscale_in_train",
                                              "dropout2_implementation": "upscale_in_train"})["Out"]
    h = _ln(x, g1, be1) if pre_ln else x
    fa = F.relu if act == "relu" else F.gelu
    o = fa(h @ w1 + b1) @ w2 + b2
    ref = x + o if pre_ln else _ln(x + o, g2, be2)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(out)
    torch.testing.assert_close(torch.autograd.grad(out, w1, g)[0], torch.autograd.grad(ref, w1, g)[0],
                               rtol=1e-4, atol=1e-4)


def test_fused_bias_dropout_residual_ln():
    x, r, b, g, be = _r(3, 7, 24), _r(3, 7, 24), _r(24), 1 + _r(24), _r(24)
    y = REGISTRY["fused_bias_dropout_residual_layer_norm"](
        {"X": [x], "Residual": [r], "Bias": [b], "LnScale": [g], "LnBias": [be]},
        {"is_test": True, "dropout_rate": 0.3, "dropout_implementation": "upscale_in_train",
         "ln_epsilon": 1e-5})["Y"]
    torch.testing.assert_close(y, _ln(r + x + b, g, be), rtol=1e-5, atol=1e-5)


def _bn_train_ref(x, g, b, eps, axis):
    dims = [d for d in range(x.dim()) if d != axis]
    m = x.mean(dims, keepdim=True)
    v = x.var(dims, keepdim=True, unbiased=False)
    shp = [1] * x.dim()
    shp[axis] = -1
    return (x - m) / torch.sqrt(v + eps) * g.view(shp) + b.view(shp), x.mean(dims), x.var(dims, unbiased=True)


def test_fused_bn_add_activation():
    x, z = _r(4, 5, 5, 8, sc=1.0), _r(4, 5, 5, 8)
    g, b = 1 + _r(8), _r(8)
    mean, var = torch.zeros(8), torch.ones(8)
    out = REGISTRY["fused_bn_add_activation"](
        {"X": [x], "Z": [z], "Scale": [g], "Bias": [b], "Mean": [mean], "Variance": [var]},
        {"momentum": 0.9, "epsilon": 1e-5, "act_type": "relu"})
    bn, bm, bv = _bn_train_ref(x, g, b, 1e-5, 3)
    torch.testing.assert_close(out["Y"], F.relu(bn + z), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out["MeanOut"], 0.1 * bm, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("shortcut", [True, False])
def test_resnet_unit(shortcut):
    N, H, W, C, K = 2, 6, 6, 8, 16
    x = _r(N, H, W, C, sc=1.0)
    z = _r(N, H, W, C if shortcut else K, sc=1.0)
    fx, fz = _r(K, C, 3, 3), _r(K, C, 3, 3)  # one `padding` attr serves both convs (reference)
    sx, bx, sz, bz = 1 + _r(K), _r(K), 1 + _r(K), _r(K)
    st = [torch.zeros(K), torch.ones(K), torch.zeros(K), torch.ones(K)]
    ins = {"X": [x], "FilterX": [fx], "ScaleX": [sx], "BiasX": [bx], "MeanX": [st[0]], "VarX": [st[1]],
           "Z": [z], "FilterZ": [fz], "ScaleZ": [sz], "BiasZ": [bz], "MeanZ": [st[2]], "VarZ": [st[3]]}
    out = REGISTRY["resnet_unit"](ins, {"stride": 1, "padding": 1, "stride_z": 1, "data_format": "NHWC",
                                        "has_shortcut": shortcut, "fuse_add": not shortcut,
                                        "act_type": "relu", "is_test": False})
    cx = F.conv2d(x.permute(0, 3, 1, 2), fx, padding=1).permute(0, 2, 3, 1)
    y, _, _ = _bn_train_ref(cx, sx, bx, 1e-5, 3)
    if shortcut:
        cz = F.conv2d(z.permute(0, 3, 1, 2), fz, padding=1).permute(0, 2, 3, 1)
        res, _, _ = _bn_train_ref(cz, sz, bz, 1e-5, 3)
    else:
        res = z
    torch.testing.assert_close(out["Y"], F.relu(y + res), rtol=1e-3, atol=1e-3)


# ----------------------------------------------------------------------------- rnn
@pytest.mark.parametrize("mode", ["LSTM", "GRU", "RNN_TANH"])
@pytest.mark.parametrize("bidir", [False, True])
def test_rnn_op_matches_torch(mode, bidir):
    T, B, I, Hs, L = 7, 3, 5, 6, 2
    cls = {"LSTM": torch.nn.LSTM, "GRU": torch.nn.GRU, "RNN_TANH": torch.nn.RNN}[mode]
    net = cls(I, Hs, num_layers=L, bidirectional=bidir)
    D = 2 if bidir else 1
    x = torch.randn(T, B, I)
    lens = torch.tensor([7, 4, 1])
    h0 = torch.randn(L * D, B, Hs)
    c0 = torch.randn(L * D, B, Hs)
    ws, bs = [], []
    for l in range(L):
        for d in range(D):
            sfx = f"_l{l}" + ("_reverse" if d else "")
            ws += [getattr(net, "weight_ih" + sfx), getattr(net, "weight_hh" + sfx)]
            bs += [getattr(net, "bias_ih" + sfx), getattr(net, "bias_hh" + sfx)]
    pre = [h0, c0] if mode == "LSTM" else [h0]
    out = REGISTRY["rnn"]({"Input": [x], "WeightList": ws + bs, "PreState": pre, "SequenceLength": [lens]},
                          {"mode": mode, "hidden_size": Hs, "num_layers": L, "is_bidirec": bidir,
                           "is_test": True})
    packed = torch.nn.utils.rnn.pack_padded_sequence(x, lens, enforce_sorted=False)
    with torch.no_grad():
        ro, rs = net(packed, (h0, c0) if mode == "LSTM" else h0)
    ro, _ = torch.nn.utils.rnn.pad_packed_sequence(ro, total_length=T)
    torch.testing.assert_close(out["Out"], ro, rtol=1e-5, atol=1e-5)
    rs = list(rs) if mode == "LSTM" else [rs]
    for a, b in zip(out["State"], rs):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)


# ----------------------------------------------------------------------------- 3-D / sampling
def test_conv3d_pool3d_grid_sampler():
    x = torch.randn(2, 4, 5, 6, 7)
    w, b = torch.randn(8, 4, 3, 3, 3), torch.randn(8)
    y = REGISTRY["conv3d"]({"Input": [x], "Filter": [w], "Bias": [b]},
                           {"strides": [1, 2, 1], "paddings": [1, 1, 0], "dilations": [1, 1, 1], "groups": 1})["Output"]
    torch.testing.assert_close(y, F.conv3d(x, w, b, (1, 2, 1), (1, 1, 0)))
    p = REGISTRY["pool3d"]({"X": [x]}, {"pooling_type": "avg", "ksize": [2, 2, 2], "strides": [2, 2, 2],
                                         "paddings": [0, 0, 0], "exclusive": True})["Out"]
    torch.testing.assert_close(p, F.avg_pool3d(x, 2, 2))
    p = REGISTRY["pool3d"]({"X": [x]}, {"pooling_type": "max", "ksize": [1, 1, 1], "global_pooling": True})["Out"]
    torch.testing.assert_close(p, x.amax((2, 3, 4), keepdim=True))
    img = torch.randn(2, 3, 8, 9)
    grid = torch.rand(2, 4, 5, 2) * 2 - 1
    o = REGISTRY["grid_sampler"]({"X": [img], "Grid": [grid]}, {"align_corners": False, "mode": "bilinear",
                                                                 "padding_mode": "border"})["Output"]
    torch.testing.assert_close(o, F.grid_sample(img, grid, padding_mode="border", align_corners=False))


# ----------------------------------------------------------------------------- detection
def _sig(v):
    return 1.0 / (1.0 + math.exp(-v))


def _yolo_ref(x, img, anchors, C, thr, ds, clip, scale, iou_aware, f):
    """Literal transcription of `phi/kernels/cpu/yolo_box_kernel.cc`."""
    n, _, h, w = x.shape
    an = len(anchors) // 2
    xd = x.reshape(-1).tolist()
    stride, an_stride = h * w, (C + 5) * h * w
    box_num = an * h * w
    boxes = np.zeros((n, box_num, 4))
    scores = np.zeros((n, box_num, C))
    bias = -0.5 * (scale - 1.0)

    def entry(i, j, hw, e):
        if iou_aware:
            return (i * an + j) * an_stride + (i * an + an + e) * stride + hw
        return (i * an + j) * an_stride + e * stride + hw
    for i in range(n):
        ih, iw = int(img[i, 0]), int(img[i, 1])
        for j in range(an):
            for k in range(h):
                for l in range(w):
                    conf = _sig(xd[entry(i, j, k * w + l, 4)])
                    if iou_aware:
                        iou = _sig(xd[i * an * an_stride + (i * an + j) * stride + k * w + l])
                        conf = conf ** (1 - f) * iou ** f
                    if conf < thr:
                        continue
                    bi = entry(i, j, k * w + l, 0)
                    bx = (l + _sig(xd[bi]) * scale + bias) * iw / w
                    by = (k + _sig(xd[bi + stride]) * scale + bias) * ih / h
                    bw = math.exp(xd[bi + 2 * stride]) * anchors[2 * j] * iw / (ds * w)
                    bh = math.exp(xd[bi + 3 * stride]) * anchors[2 * j + 1] * ih / (ds * h)
                    bb = [bx - bw / 2, by - bh / 2, bx + bw / 2, by + bh / 2]
                    if clip:
                        bb = [max(bb[0], 0), max(bb[1], 0), min(bb[2], iw - 1), min(bb[3], ih - 1)]
                    o = j * stride + k * w + l
                    boxes[i, o] = bb
                    li = entry(i, j, k * w + l, 5)
                    for c in range(C):
                        scores[i, o, c] = conf * _sig(xd[li + c * stride])
    return boxes, scores


@pytest.mark.parametrize("iou_aware", [False, True])
def test_yolo_box(iou_aware):
    C, anchors, H, W = 3, [10, 13, 16, 30], 4, 5
    A = len(anchors) // 2
    x = torch.randn(2, A * (5 + C) + (A if iou_aware else 0), H, W)
    img = torch.tensor([[320, 416], [200, 300]], dtype=torch.int32)
    out = REGISTRY["yolo_box"]({"X": [x], "ImgSize": [img]},
                               {"anchors": anchors, "class_num": C, "conf_thresh": 0.4, "downsample_ratio": 32,
                                "clip_bbox": True, "scale_x_y": 1.2, "iou_aware": iou_aware,
                                "iou_aware_factor": 0.4})
    rb, rs = _yolo_ref(x, img, anchors, C, 0.4, 32, True, 1.2, iou_aware, 0.4)
    np.testing.assert_allclose(out["Boxes"].numpy(), rb, rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(out["Scores"].numpy(), rs, rtol=1e-4, atol=1e-5)


def test_multiclass_nms3():
    # image 0: two overlapping boxes of class 1 (one suppressed), one box of class 2; background 0
    boxes = torch.tensor([[[0., 0., 10., 10.], [1., 1., 10., 10.], [20., 20., 30., 30.], [50, 50, 60, 60]],
                          [[0., 0., 5., 5.], [6., 6., 9., 9.], [0., 0., 5.2, 5.2], [1, 1, 2, 2]]])
    scores = torch.zeros(2, 3, 4)
    scores[0, 1] = torch.tensor([0.9, 0.8, 0.1, 0.02])
    scores[0, 2] = torch.tensor([0.0, 0.0, 0.7, 0.0])
    scores[1, 1] = torch.tensor([0.6, 0.5, 0.55, 0.3])
    scores[1, 0] = 0.99  # background: ignored
    out = REGISTRY["multiclass_nms3"]({"BBoxes": [boxes], "Scores": [scores]},
                                      {"score_threshold": 0.05, "nms_top_k": -1, "keep_top_k": -1,
                                       "nms_threshold": 0.5, "normalized": False, "background_label": 0})
    o = out["Out"].numpy()
    # image 0: class 1 → idx 0 (box 1 suppressed, IoU 0.83), idx 2 (0.1); class 2 → idx 2
    # image 1: class 1 → idx 0 (0.6), then 2 is suppressed by 0, then 1 (0.5), then 3 (0.3)
    assert out["NmsRoisNum"].tolist() == [3, 3]
    np.testing.assert_allclose(o[:, 0], [1, 1, 2, 1, 1, 1])
    np.testing.assert_allclose(o[:, 1], [0.9, 0.1, 0.7, 0.6, 0.5, 0.3], rtol=1e-6)
    assert out["Index"].reshape(-1).tolist() == [0, 2, 2, 4, 5, 7]
    # keep_top_k across classes
    out = REGISTRY["multiclass_nms3"]({"BBoxes": [boxes[:1]], "Scores": [scores[:1]]},
                                      {"score_threshold": 0.05, "nms_top_k": -1, "keep_top_k": 2,
                                       "nms_threshold": 0.5, "normalized": False})
    np.testing.assert_allclose(out["Out"][:, 1].numpy(), [0.9, 0.7], rtol=1e-6)


def _roi_align_ref(x, rois, batch, ph, pw, scale, sr, aligned):
    """Literal transcription of `phi/kernels/cpu/roi_align_kernel.cc`."""
    N, C, H, W = x.shape
    out = np.zeros((len(rois), C, ph, pw))
    xd = x.numpy()
    off = 0.5 if aligned else 0.0
    for n, (roi, b) in enumerate(zip(rois.tolist(), batch)):
        x0, y0, x1, y1 = [v * scale - off for v in roi]
        rw, rh = x1 - x0, y1 - y0
        if not aligned:
            rw, rh = max(rw, 1.0), max(rh, 1.0)
        gh = sr if sr > 0 else math.ceil(rh / ph)
        gw = sr if sr > 0 else math.ceil(rw / pw)
        bw, bh = rw / pw, rh / ph
        for py in range(ph):
            for px in range(pw):
                acc = np.zeros(C)
                for iy in range(gh):
                    y = y0 + bh * (py + (iy + .5) / gh)
                    for ix in range(gw):
                        xx = x0 + bw * (px + (ix + .5) / gw)
                        if y < -1.0 or y > H or xx < -1.0 or xx > W:
                            continue
                        y, xx = max(y, 0), max(xx, 0)
                        yl, xl = int(y), int(xx)
                        if yl >= H - 1:
                            yh = yl = H - 1
                            y = float(yl)
                        else:
                            yh = yl + 1
                        if xl >= W - 1:
                            xh = xl = W - 1
                            xx = float(xl)
                        else:
                            xh = xl + 1
                        ly, lx = yh - y, xh - xx
                        acc += (lx * ly * xd[b, :, yl, xl] + lx * (1 - ly) * xd[b, :, yh, xl]
                                + (1 - lx) * ly * xd[b, :, yl, xh] + (1 - lx) * (1 - ly) * xd[b, :, yh, xh])
                out[n, :, py, px] = acc / (gh * gw)
    return out


@pytest.mark.parametrize("aligned,sr", [(False, -1), (True, 2), (True, -1)])
def test_roi_align(aligned, sr):
    x = torch.randn(2, 3, 12, 14)
    rois = torch.tensor([[1.0, 2.0, 9.5, 7.0], [0.0, 0.0, 3.0, 3.0], [4.0, 1.0, 13.9, 11.9], [-2.0, -1.0, 4.0, 5.0]])
    num = torch.tensor([1, 3], dtype=torch.int32)
    out = REGISTRY["roi_align"]({"X": [x], "ROIs": [rois], "RoisNum": [num]},
                                {"pooled_height": 3, "pooled_width": 4, "spatial_scale": 0.8,
                                 "sampling_ratio": sr, "aligned": aligned})["Out"]
    ref = _roi_align_ref(x, rois, [0, 1, 1, 1], 3, 4, 0.8, sr, aligned)
    np.testing.assert_allclose(out.numpy(), ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("order", [False, True])
def test_prior_box(order):
    feat, img = torch.zeros(1, 8, 3, 4), torch.zeros(1, 3, 30, 40)
    attrs = {"min_sizes": [4.0, 8.0], "max_sizes": [9.0, 12.0], "aspect_ratios": [2.0, 3.0],
             "variances": [0.1, 0.1, 0.2, 0.2], "flip": True, "clip": True, "step_w": 0.0, "step_h": 0.0,
             "offset": 0.5, "min_max_aspect_ratios_order": order}
    out = REGISTRY["prior_box"]({"Input": [feat], "Image": [img]}, attrs)
    ars = [1.0, 2.0, 0.5, 3.0, 1.0 / 3]
    ref = []
    for h in range(3):
        for w in range(4):
            cx, cy = (w + 0.5) * 10.0, (h + 0.5) * 10.0
            cell = []
            for s, mn in enumerate(attrs["min_sizes"]):
                mx = math.sqrt(mn * attrs["max_sizes"][s])
                if order:
                    whs = [(mn, mn), (mx, mx)] + [(mn * math.sqrt(a), mn / math.sqrt(a)) for a in ars[1:]]
                else:
                    whs = [(mn * math.sqrt(a), mn / math.sqrt(a)) for a in ars] + [(mx, mx)]
                for bw, bh in whs:
                    cell.append([(cx - bw / 2) / 40, (cy - bh / 2) / 30, (cx + bw / 2) / 40, (cy + bh / 2) / 30])
            ref.append(cell)
    ref = np.clip(np.array(ref).reshape(3, 4, -1, 4), 0, 1)
    np.testing.assert_allclose(out["Boxes"].numpy(), ref, rtol=1e-5, atol=1e-6)
    assert out["Variances"].shape == out["Boxes"].shape
    np.testing.assert_allclose(out["Variances"][1, 2, 3].numpy(), [0.1, 0.1, 0.2, 0.2], rtol=1e-6)
