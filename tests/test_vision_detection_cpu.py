"""paddle.vision.ops detection set against literal (loop) transcriptions of the reference CPU
kernels: matrix_nms (`phi/kernels/cpu/matrix_nms_kernel.cc`), generate_proposals
(`cpu/generate_proposals_v2_kernel.cc`), distribute_fpn_proposals
(`cpu/distribute_fpn_proposals_kernel.cc`), psroi_pool (`cpu/psroi_pool_kernel.cc`), yolo_loss
(`cpu/yolov3_loss_kernel.cc`); plus the layer wrappers and read_file / decode_jpeg."""
import math

import numpy as np
import pytest
import torch

from paddle_infer_amd.vision import ops as V


def _iou(a, b, normalized):
    if b[0] > a[2] or b[2] < a[0] or b[1] > a[3] or b[3] < a[1]:
        return 0.0
    n = 0.0 if normalized else 1.0
    iw = min(a[2], b[2]) - max(a[0], b[0]) + n
    ih = min(a[3], b[3]) - max(a[1], b[1]) + n

    def area(x):
        if x[2] < x[0] or x[3] < x[1]:
            return 0.0
        return (x[2] - x[0] + n) * (x[3] - x[1] + n)
    inter = iw * ih
    return inter / (area(a) + area(b) - inter)


def _boxes(n, seed):
    r = np.random.RandomState(seed)
    xy = r.rand(n, 2) * 0.6
    wh = r.rand(n, 2) * 0.4 + 0.05
    return np.concatenate([xy, xy + wh], 1).astype("float32")


@pytest.mark.parametrize("gaussian", [False, True])
def test_matrix_nms_matches_loop_reference(gaussian):
    N, C, M = 2, 3, 12
    bb = np.stack([_boxes(M, s) for s in range(N)])
    sc = np.random.RandomState(5).rand(N, C, M).astype("float32")
    st, pt, topk, keep, sigma = 0.2, 0.1, 8, 10, 2.0
    ref_rows, ref_num = [], []
    for i in range(N):
        cand = []
        for c in range(C):
            if c == 0:
                continue
            s = sc[i, c]
            perm = [j for j in np.argsort(-s, kind="stable") if s[j] > st][:topk]
            n = len(perm)
            iou = np.zeros((n, n))
            imax = np.zeros(n)
            for a in range(1, n):
                for b in range(a):
                    iou[a, b] = _iou(bb[i, perm[a]], bb[i, perm[b]], True)
                imax[a] = iou[a, :a].max()
            if n and s[perm[0]] > pt:
                cand.append((s[perm[0]], c, perm[0]))
            for a in range(1, n):
                md = 1.0
                for b in range(a):
                    d = math.exp((imax[b] ** 2 - iou[a, b] ** 2) * sigma) if gaussian else \
                        (1 - iou[a, b]) / (1 - imax[b])
                    md = min(md, d)
                ds = md * s[perm[a]]
                if ds > pt:
                    cand.append((ds, c, perm[a]))
        cand = sorted(cand, key=lambda t: -t[0])[:keep]
        ref_num.append(len(cand))
        ref_rows += [[c, s] + list(bb[i, j]) for s, c, j in cand]
    out, num, idx = V.matrix_nms(torch.tensor(bb), torch.tensor(sc), st, pt, topk, keep,
                                 use_gaussian=gaussian, gaussian_sigma=sigma, return_index=True)
    assert num.tolist() == ref_num
    np.testing.assert_allclose(out.numpy(), np.array(ref_rows, dtype="float32"), rtol=1e-5, atol=1e-6)
    assert idx.shape == (sum(ref_num), 1)


def test_generate_proposals_matches_loop_reference():
    r = np.random.RandomState(0)
    N, A, H, W = 2, 3, 4, 5
    scores = r.rand(N, A, H, W).astype("float32")
    deltas = (r.randn(N, 4 * A, H, W) * 0.2).astype("float32")
    base = np.array([[0, 0, 15, 15], [0, 0, 31, 15], [0, 0, 15, 31]], "float32")
    anchors = np.zeros((H, W, A, 4), "float32")
    for y in range(H):
        for x in range(W):
            anchors[y, x] = base + np.array([x * 8, y * 8, x * 8, y * 8], "float32")
    var = np.full((H, W, A, 4), 1.0, "float32")
    im = np.array([[40, 50], [35, 45]], "float32")
    pre, post, thr, ms = 20, 6, 0.5, 2.0
    rois, probs, num = V.generate_proposals(torch.tensor(scores), torch.tensor(deltas), torch.tensor(im),
                                            torch.tensor(anchors), torch.tensor(var), pre, post, thr, ms,
                                            1.0, pixel_offset=True, return_rois_num=True)
    clip = math.log(1000.0 / 16.0)
    start = 0
    for i in range(N):
        s = scores[i].transpose(1, 2, 0).reshape(-1)
        d = deltas[i].transpose(1, 2, 0).reshape(-1, 4)
        a, v = anchors.reshape(-1, 4), var.reshape(-1, 4)
        order = np.argsort(-s, kind="stable")[:pre]
        props = []
        for j in order:
            aw, ah = a[j, 2] - a[j, 0] + 1, a[j, 3] - a[j, 1] + 1
            cx, cy = v[j, 0] * d[j, 0] * aw + a[j, 0] + 0.5 * aw, v[j, 1] * d[j, 1] * ah + a[j, 1] + 0.5 * ah
            w, h = math.exp(min(v[j, 2] * d[j, 2], clip)) * aw, math.exp(min(v[j, 3] * d[j, 3], clip)) * ah
            b = [cx - w / 2, cy - h / 2, cx + w / 2 - 1, cy + h / 2 - 1]
            b = [max(min(b[0], im[i, 1] - 1), 0), max(min(b[1], im[i, 0] - 1), 0),
                 max(min(b[2], im[i, 1] - 1), 0), max(min(b[3], im[i, 0] - 1), 0)]
            ws, hs = b[2] - b[0] + 1, b[3] - b[1] + 1
            if ws >= ms and hs >= ms and b[0] + ws / 2 <= im[i, 1] and b[1] + hs / 2 <= im[i, 0]:
                props.append((s[j], b))
        kept = []
        for sc_, b in sorted(props, key=lambda t: -t[0]):
            if all(_iou(b, k[1], False) <= thr for k in kept):
                kept.append((sc_, b))
        kept = kept[:post]
        assert int(num[i]) == len(kept)
        np.testing.assert_allclose(rois[start:start + len(kept)].numpy(),
                                   np.array([k[1] for k in kept], "float32"), rtol=1e-5, atol=1e-4)
        np.testing.assert_allclose(probs[start:start + len(kept), 0].numpy(),
                                   np.array([k[0] for k in kept], "float32"), rtol=1e-6)
        start += len(kept)


def test_distribute_fpn_proposals_restores_order():
    r = np.random.RandomState(1)
    xy = r.rand(10, 2) * 100
    wh = r.rand(10, 2) * 300 + 2
    rois = torch.tensor(np.concatenate([xy, xy + wh], 1), dtype=torch.float32)
    rn = torch.tensor([3, 4, 3], dtype=torch.int32)
    multi, restore, per = V.distribute_fpn_proposals(rois, 2, 5, 4, 224, pixel_offset=True, rois_num=rn)
    assert len(multi) == 4 and len(per) == 4
    for L, m in enumerate(multi, start=2):
        for b in m.numpy():
            s = math.sqrt((b[2] - b[0] + 1) * (b[3] - b[1] + 1))
            lvl = min(5, max(2, math.floor(math.log2(s / 224 + 1e-6) + 4)))
            assert lvl == L
    cat = torch.cat(multi)
    torch.testing.assert_close(cat[restore.reshape(-1).long()], rois)
    assert sum(int(p.sum()) for p in per) == 10


def test_psroi_pool_matches_loop_reference():
    torch.manual_seed(0)
    oh = ow = 2
    Co = 3
    x = torch.randn(2, Co * oh * ow, 9, 11, requires_grad=True)
    boxes = torch.tensor([[1.2, 0.7, 7.6, 6.1], [0, 0, 10, 8], [3, 2, 3.4, 2.2]])
    bn = torch.tensor([2, 1])
    out = V.psroi_pool(x, boxes, bn, 2, spatial_scale=0.9)
    ref = torch.zeros_like(out)
    bid = [0, 0, 1]
    for n in range(3):
        b = boxes[n].tolist()
        sw, sh = round(b[0]) * 0.9, round(b[1]) * 0.9
        ew, eh = (round(b[2]) + 1) * 0.9, (round(b[3]) + 1) * 0.9
        rh, rw = max(eh - sh, 0.1), max(ew - sw, 0.1)
        for c in range(Co):
            for ph in range(oh):
                for pw in range(ow):
                    hs = min(max(math.floor(ph * rh / oh + sh), 0), 9)
                    ws = min(max(math.floor(pw * rw / ow + sw), 0), 11)
                    he = min(max(math.ceil((ph + 1) * rh / oh + sh), 0), 9)
                    we = min(max(math.ceil((pw + 1) * rw / ow + sw), 0), 11)
                    ch = (c * oh + ph) * ow + pw
                    if he > hs and we > ws:
                        ref[n, c, ph, pw] = x[bid[n], ch, hs:he, ws:we].mean()
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    out.sum().backward()
    assert x.grad is not None and x.grad.abs().sum() > 0
    layer = V.PSRoIPool(2, 0.9)
    torch.testing.assert_close(layer(x, boxes, bn), out)


def _yolo_ref(x, gt_box, gt_label, anchors, mask, C, ignore, ds, smooth):
    sig = lambda v: 1 / (1 + math.exp(-v))  # noqa: E731
    sce = lambda v, t: max(v, 0) - v * t + math.log(1 + math.exp(-abs(v)))  # noqa: E731
    N, _, H, W = x.shape
    A, B = len(mask), gt_box.shape[1]
    xr = x.reshape(N, A, 5 + C, H, W)
    ins = ds * H
    pos, neg = (1 - min(1 / C, 1 / 40), min(1 / C, 1 / 40)) if smooth else (1.0, 0.0)

    def iou(a, b):
        def ov(c1, w1, c2, w2):
            return min(c1 + w1 / 2, c2 + w2 / 2) - max(c1 - w1 / 2, c2 - w2 / 2)
        w, h = ov(a[0], a[2], b[0], b[2]), ov(a[1], a[3], b[1], b[3])
        inter = 0 if (w < 0 or h < 0) else w * h
        return inter / (a[2] * a[3] + b[2] * b[3] - inter)
    loss = np.zeros(N)
    for i in range(N):
        obj = np.zeros((A, H, W))
        for j in range(A):
            for k in range(H):
                for l in range(W):
                    p = [(l + sig(xr[i, j, 0, k, l])) / H, (k + sig(xr[i, j, 1, k, l])) / H,
                         math.exp(xr[i, j, 2, k, l]) * anchors[2 * mask[j]] / ins,
                         math.exp(xr[i, j, 3, k, l]) * anchors[2 * mask[j] + 1] / ins]
                    best = 0
                    for t in range(B):
                        if gt_box[i, t, 2] <= 1e-6 or gt_box[i, t, 3] <= 1e-6:
                            continue
                        best = max(best, iou(p, gt_box[i, t]))
                    if best > ignore:
                        obj[j, k, l] = -1
        for t in range(B):
            g = gt_box[i, t]
            if g[2] <= 1e-6 or g[3] <= 1e-6:
                continue
            gi, gj = int(g[0] * W), int(g[1] * H)
            bn, bv = 0, 0.0
            for a in range(len(anchors) // 2):
                v = iou([0, 0, anchors[2 * a] / ins, anchors[2 * a + 1] / ins], [0, 0, g[2], g[3]])
                if v > bv:
                    bv, bn = v, a
            if bn not in mask:
                continue
            m = mask.index(bn)
            pr = xr[i, m, :, gj, gi]
            sc = (2 - g[2] * g[3])
            loss[i] += sce(pr[0], g[0] * W - gi) * sc + sce(pr[1], g[1] * H - gj) * sc
            loss[i] += abs(pr[2] - math.log(g[2] * ins / anchors[2 * bn])) * sc
            loss[i] += abs(pr[3] - math.log(g[3] * ins / anchors[2 * bn + 1])) * sc
            obj[m, gj, gi] = 1.0
            for c in range(C):
                loss[i] += sce(pr[5 + c], pos if c == gt_label[i, t] else neg)
        for j in range(A):
            for k in range(H):
                for l in range(W):
                    if obj[j, k, l] > 1e-5:
                        loss[i] += sce(xr[i, j, 4, k, l], 1.0) * obj[j, k, l]
                    elif obj[j, k, l] > -0.5:
                        loss[i] += sce(xr[i, j, 4, k, l], 0.0)
    return loss


def test_yolo_loss_matches_loop_reference():
    r = np.random.RandomState(3)
    C, H = 2, 6
    anchors, mask = [10, 13, 16, 30, 33, 23], [0, 1]
    x = (r.randn(2, len(mask) * (5 + C), H, H) * 0.5).astype("float32")
    gt = np.concatenate([r.rand(2, 4, 2) * 0.8 + 0.1, r.rand(2, 4, 2) * 0.3 + 0.02], -1).astype("float32")
    gt[1, 3] = 0  # an invalid (padding) box
    lab = r.randint(0, C, (2, 4)).astype("int32")
    ref = _yolo_ref(x, gt, lab, anchors, mask, C, 0.5, 8, True)
    xt = torch.tensor(x, requires_grad=True)
    out = V.yolo_loss(xt, torch.tensor(gt), torch.tensor(lab), anchors, mask, C, 0.5, 8,
                      use_label_smooth=True)
    np.testing.assert_allclose(out.detach().numpy(), ref, rtol=1e-4, atol=1e-4)
    out.sum().backward()
    assert torch.isfinite(xt.grad).all()


def test_layers_and_file_decode(tmp_path):
    from PIL import Image
    torch.manual_seed(0)
    x = torch.randn(1, 4, 10, 10)
    boxes = torch.tensor([[1.0, 1.0, 6.0, 7.0]])
    bn = torch.tensor([1])
    torch.testing.assert_close(V.RoIAlign(3, 1.0)(x, boxes, bn), V.roi_align(x, boxes, bn, 3))
    torch.testing.assert_close(V.RoIPool(3, 1.0)(x, boxes, bn), V.roi_pool(x, boxes, bn, 3))
    dc = V.DeformConv2D(4, 6, 3, padding=1)
    off = torch.zeros(1, 18, 10, 10)
    y = dc(x, off)
    ref = torch.nn.functional.conv2d(x, dc.weight, dc.bias, padding=1)
    torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-4)
    img = (np.arange(8 * 6 * 3) % 251).astype("uint8").reshape(8, 6, 3)
    p = tmp_path / "a.png"
    Image.fromarray(img).save(p)
    raw = V.read_file(str(p))
    assert raw.dtype == torch.uint8 and raw.numel() == p.stat().st_size
    dec = V.decode_jpeg(raw, mode="rgb")
    assert dec.shape == (3, 8, 6)
    np.testing.assert_array_equal(dec.numpy().transpose(1, 2, 0), img)
