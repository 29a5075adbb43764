"""``paddle.vision.ops`` (reference `python/paddle/vision/ops.py`): nms, box_coder, roi_align,
roi_pool, deform_conv2d, yolo_box, distribute_fpn_proposals (subset), as tensor compositions."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def box_area(b):
    return (b[:, 2] - b[:, 0]).clamp_min(0) * (b[:, 3] - b[:, 1]).clamp_min(0)


def box_iou(a, b):
    lt = torch.maximum(a[:, None, :2], b[None, :, :2])
    rb = torch.minimum(a[:, None, 2:], b[None, :, 2:])
    inter = (rb - lt).clamp_min(0).prod(-1)
    return inter / (box_area(a)[:, None] + box_area(b)[None, :] - inter + 1e-10)


def nms(boxes, iou_threshold=0.3, scores=None, category_idxs=None, categories=None, top_k=None):
    """Greedy NMS; returns kept indices sorted by score (reference ops.py:nms)."""
    if scores is None:
        scores = torch.arange(boxes.shape[0], 0, -1, dtype=torch.float32, device=boxes.device)
    if category_idxs is not None:  # batched: offset boxes per category
        off = category_idxs.to(boxes.dtype)[:, None] * (boxes.max() + 1)
        boxes = boxes + off
    order = scores.argsort(descending=True)
    iou = box_iou(boxes[order], boxes[order])
    keep = torch.ones(order.numel(), dtype=torch.bool, device=boxes.device)
    for i in range(order.numel()):
        if keep[i]:
            sup = iou[i] > iou_threshold
            sup[: i + 1] = False
            keep &= ~sup
    out = order[keep]
    return out[:top_k] if top_k is not None else out


def box_coder(prior_box, prior_box_var, target_box, code_type="encode_center_size",
              box_normalized=True, axis=0, name=None):
    off = 0.0 if box_normalized else 1.0
    pw = prior_box[:, 2] - prior_box[:, 0] + off
    ph = prior_box[:, 3] - prior_box[:, 1] + off
    px = prior_box[:, 0] + pw / 2
    py = prior_box[:, 1] + ph / 2
    var = prior_box_var if isinstance(prior_box_var, torch.Tensor) else torch.tensor(prior_box_var or [1., 1., 1., 1.])
    if code_type == "encode_center_size":
        tw = target_box[:, 2] - target_box[:, 0] + off
        th = target_box[:, 3] - target_box[:, 1] + off
        tx = target_box[:, 0] + tw / 2
        ty = target_box[:, 1] + th / 2
        out = torch.stack([(tx[:, None] - px) / pw / var[..., 0], (ty[:, None] - py) / ph / var[..., 1],
                           torch.log(tw[:, None] / pw) / var[..., 2], torch.log(th[:, None] / ph) / var[..., 3]], -1)
        return out
    t = target_box
    cx = var[..., 0] * t[..., 0] * pw + px
    cy = var[..., 1] * t[..., 1] * ph + py
    w = torch.exp(var[..., 2] * t[..., 2]) * pw
    h = torch.exp(var[..., 3] * t[..., 3]) * ph
    return torch.stack([cx - w / 2, cy - h / 2, cx + w / 2 - off, cy + h / 2 - off], -1)


def roi_align(x, boxes, boxes_num, output_size, spatial_scale=1.0, sampling_ratio=-1, aligned=True, name=None):
    """Reference `phi/kernels/cpu/roi_align_kernel.cc`: per ROI and output bin, the average of
    roi_bin_grid_h × roi_bin_grid_w bilinear samples (``sampling_ratio`` > 0, else
    ceil(roi_size / pooled_size) per ROI); samples outside [-1, H] × [-1, W] count as 0; ``aligned``
    shifts the ROI by half a pixel. Vectorised over ROI chunks (gathers on the feature map)."""
    oh, ow = (output_size, output_size) if isinstance(output_size, int) else tuple(output_size)
    N, C, H, W = x.shape
    R = boxes.shape[0]
    out = x.new_zeros((R, C, oh, ow))
    if R == 0:
        return out
    dev = x.device
    bidx = torch.repeat_interleave(torch.arange(N, device=dev), boxes_num.to(dev).long())
    off = 0.5 if aligned else 0.0
    b = boxes.to(dev).float() * spatial_scale - off
    rw, rh = b[:, 2] - b[:, 0], b[:, 3] - b[:, 1]
    if not aligned:
        rw, rh = rw.clamp_min(1.0), rh.clamp_min(1.0)
    if sampling_ratio > 0:
        gh = torch.full((R,), sampling_ratio, device=dev, dtype=torch.long)
        gw = gh.clone()
    else:
        gh = torch.ceil(rh / oh).long().clamp_min(1)
        gw = torch.ceil(rw / ow).long().clamp_min(1)
    xf = x.float().reshape(N, C, H * W)
    for r0 in range(0, R, 32):
        sl = slice(r0, min(R, r0 + 32))
        Gh, Gw = int(gh[sl].max()), int(gw[sl].max())
        ghs, gws = gh[sl].float(), gw[sl].float()
        iy = torch.arange(Gh, device=dev).float()
        ix = torch.arange(Gw, device=dev).float()
        py = torch.arange(oh, device=dev).float()
        px = torch.arange(ow, device=dev).float()
        # sample coordinates [r, oh, Gh] / [r, ow, Gw]
        y = b[sl, 1, None, None] + (rh[sl] / oh)[:, None, None] * (py[None, :, None] + (iy[None, None, :] + 0.5) / ghs[:, None, None])
        xx = b[sl, 0, None, None] + (rw[sl] / ow)[:, None, None] * (px[None, :, None] + (ix[None, None, :] + 0.5) / gws[:, None, None])
        vy = (iy[None, None, :] < ghs[:, None, None]) & (y >= -1.0) & (y <= H)
        vx = (ix[None, None, :] < gws[:, None, None]) & (xx >= -1.0) & (xx <= W)

        def axis(t, n):
            t = t.clamp_min(0.0)
            lo = t.floor().long()
            edge = lo >= n - 1
            lo = torch.where(edge, torch.full_like(lo, n - 1), lo)
            hi = torch.where(edge, lo, lo + 1)
            t = torch.where(edge, lo.float(), t)
            w_lo = hi.float() - t
            return lo, hi, w_lo, 1.0 - w_lo
        ylo, yhi, wyl, wyh = axis(y, H)
        xlo, xhi, wxl, wxh = axis(xx, W)
        rr = ylo.shape[0]
        # corner offsets / weights on the [r, oh, Gh, ow, Gw] sample grid
        def comb(ya, xa):
            return (ya[:, :, :, None, None] * W + xa[:, None, None, :, :]).reshape(rr, -1)
        valid = (vy[:, :, :, None, None] & vx[:, None, None, :, :]).float()
        acc = 0.0
        fb = xf[bidx[sl]]  # [r, C, H*W]
        for ya, wy in ((ylo, wyl), (yhi, wyh)):
            for xa, wx in ((xlo, wxl), (xhi, wxh)):
                idx = comb(ya, xa)
                wgt = (wy[:, :, :, None, None] * wx[:, None, None, :, :] * valid).reshape(rr, 1, -1)
                acc = acc + torch.gather(fb, 2, idx[:, None, :].expand(rr, C, idx.shape[1])) * wgt
        acc = acc.reshape(rr, C, oh, Gh, ow, Gw).sum((3, 5)) / (ghs * gws)[:, None, None, None]
        out[sl] = acc.to(x.dtype)
    return out


def roi_pool(x, boxes, boxes_num, output_size, spatial_scale=1.0, name=None):
    oh, ow = (output_size, output_size) if isinstance(output_size, int) else output_size
    bidx = torch.repeat_interleave(torch.arange(len(boxes_num), device=x.device), boxes_num.to(x.device).long())
    outs = []
    for k in range(boxes.shape[0]):
        b = int(bidx[k])
        x1, y1, x2, y2 = [int(round(v)) for v in (boxes[k] * spatial_scale).tolist()]
        reg = x[b, :, max(y1, 0):max(y2 + 1, y1 + 1), max(x1, 0):max(x2 + 1, x1 + 1)]
        outs.append(F.adaptive_max_pool2d(reg, (oh, ow)))
    return torch.stack(outs) if outs else x.new_zeros((0, x.shape[1], oh, ow))


def deform_conv2d(x, offset, weight, bias=None, stride=1, padding=0, dilation=1,
                  deformable_groups=1, groups=1, mask=None, name=None):
    """Deformable conv v1/v2 by bilinear sampling + grouped GEMM (reference deform_conv2d)."""
    N, C, H, W = x.shape
    Co, Cg, kh, kw = weight.shape
    s = (stride, stride) if isinstance(stride, int) else stride
    p = (padding, padding) if isinstance(padding, int) else padding
    d = (dilation, dilation) if isinstance(dilation, int) else dilation
    Ho = (H + 2 * p[0] - d[0] * (kh - 1) - 1) // s[0] + 1
    Wo = (W + 2 * p[1] - d[1] * (kw - 1) - 1) // s[1] + 1
    base_y = torch.arange(Ho, device=x.device) * s[0] - p[0]
    base_x = torch.arange(Wo, device=x.device) * s[1] - p[1]
    ky = torch.arange(kh, device=x.device) * d[0]
    kx = torch.arange(kw, device=x.device) * d[1]
    gy = (base_y[None, :, None] + ky.repeat_interleave(kw)[:, None, None]).float()  # [K,Ho,1]
    gx = (base_x[None, None, :] + kx.repeat(kh)[:, None, None]).float()  # [K,1,Wo]
    off = offset.view(N, deformable_groups, kh * kw, 2, Ho, Wo)
    cols = []
    cpg = C // deformable_groups
    for g in range(deformable_groups):
        yy = gy[None] + off[:, g, :, 0]
        xx = gx[None] + off[:, g, :, 1]
        grid = torch.stack([xx / max(W - 1, 1) * 2 - 1, yy / max(H - 1, 1) * 2 - 1], -1)  # [N,K,Ho,Wo,2]
        smp = F.grid_sample(x[:, g * cpg:(g + 1) * cpg].float(), grid.view(N, kh * kw * Ho, Wo, 2),
                            align_corners=True).view(N, cpg, kh * kw, Ho, Wo)
        if mask is not None:
            smp = smp * mask.view(N, deformable_groups, kh * kw, Ho, Wo)[:, g:g + 1]
        cols.append(smp)
    col = torch.cat(cols, 1).reshape(N, groups, (C // groups) * kh * kw, Ho * Wo).to(x.dtype)
    w = weight.reshape(groups, Co // groups, -1)
    out = torch.einsum("gok,ngkl->ngol", w, col).reshape(N, Co, Ho, Wo)
    return out + bias.view(1, -1, 1, 1) if bias is not None else out


def yolo_box(x, img_size, anchors, class_num, conf_thresh, downsample_ratio, clip_bbox=True,
             name=None, scale_x_y=1.0, iou_aware=False, iou_aware_factor=0.5):
    """Reference `phi/kernels/cpu/yolo_box_kernel.cc` / `funcs/yolo_box_util.h`: boxes
    [N, A·H·W, 4] in image pixels and scores [N, A·H·W, C]; predictions whose objectness (with
    ``iou_aware``: obj^(1-f)·iou^f) is below ``conf_thresh`` stay all-zero. X is
    [N, A·(5+C), H, W] (``iou_aware``: A IoU channels first, then A·(5+C))."""
    N, _, H, W = x.shape
    na = len(anchors) // 2
    xf = x.float()
    if iou_aware:
        iou = torch.sigmoid(xf[:, :na])                          # [N, A, H, W]
        p = xf[:, na:].reshape(N, na, 5 + class_num, H, W)
    else:
        p = xf.reshape(N, na, 5 + class_num, H, W)
    conf = torch.sigmoid(p[:, :, 4])
    if iou_aware:
        conf = conf.pow(1.0 - iou_aware_factor) * iou.pow(iou_aware_factor)
    gy, gx = torch.meshgrid(torch.arange(H, device=x.device, dtype=torch.float32),
                            torch.arange(W, device=x.device, dtype=torch.float32), indexing="ij")
    an = torch.tensor(anchors, dtype=torch.float32, device=x.device).view(na, 2)
    ih = img_size[:, 0].to(x.device).float().view(N, 1, 1, 1)
    iw = img_size[:, 1].to(x.device).float().view(N, 1, 1, 1)
    bias = -0.5 * (scale_x_y - 1.0)
    cx = (gx + torch.sigmoid(p[:, :, 0]) * scale_x_y + bias) * iw / W
    cy = (gy + torch.sigmoid(p[:, :, 1]) * scale_x_y + bias) * ih / H
    bw = torch.exp(p[:, :, 2]) * an[:, 0, None, None] * iw / (downsample_ratio * W)
    bh = torch.exp(p[:, :, 3]) * an[:, 1, None, None] * ih / (downsample_ratio * H)
    x1, y1, x2, y2 = cx - bw / 2, cy - bh / 2, cx + bw / 2, cy + bh / 2
    if clip_bbox:
        x1, y1 = x1.clamp_min(0.0), y1.clamp_min(0.0)
        x2, y2 = torch.minimum(x2, iw - 1), torch.minimum(y2, ih - 1)
    keep = (conf >= conf_thresh).float()
    boxes = torch.stack([x1, y1, x2, y2], -1) * keep[..., None]
    scores = torch.sigmoid(p[:, :, 5:]) * (conf * keep)[:, :, None]
    return (boxes.reshape(N, -1, 4).to(x.dtype),
            scores.permute(0, 1, 3, 4, 2).reshape(N, -1, class_num).to(x.dtype))


def _expand_ratios(aspect_ratios, flip):
    out = [1.0]
    for ar in aspect_ratios:
        if all(abs(ar - o) >= 1e-6 for o in out):
            out.append(float(ar))
            if flip:
                out.append(1.0 / float(ar))
    return out


def prior_box(input, image, min_sizes, max_sizes=None, aspect_ratios=(1.0,), variance=(0.1, 0.1, 0.2, 0.2),
              flip=False, clip=False, steps=(0.0, 0.0), offset=0.5, min_max_aspect_ratios_order=False,
              name=None):
    """Reference `phi/kernels/cpu/prior_box_kernel.cc`: SSD priors per feature-map cell →
    (boxes [H, W, P, 4] normalised to the image, variances [H, W, P, 4])."""
    H, W = input.shape[2], input.shape[3]
    IH, IW = image.shape[2], image.shape[3]
    ars = _expand_ratios(list(aspect_ratios), flip)
    max_sizes = list(max_sizes or [])
    sw, sh = (float(steps[0]), float(steps[1])) if steps else (0.0, 0.0)
    if sw == 0 or sh == 0:
        sw, sh = IW / W, IH / H
    whs = []
    for s, mn in enumerate(min_sizes):
        sq = [(mn, mn)]
        mx = [(math.sqrt(mn * max_sizes[s]),) * 2] if max_sizes else []
        rat = [(mn * math.sqrt(a), mn / math.sqrt(a)) for a in ars]
        if min_max_aspect_ratios_order:
            whs += sq + mx + [r for a, r in zip(ars, rat) if abs(a - 1.0) >= 1e-6]
        else:
            whs += rat + mx
    wh = torch.tensor(whs, dtype=torch.float32, device=input.device) / 2       # [P, 2]
    cx = (torch.arange(W, device=input.device, dtype=torch.float32) + offset) * sw
    cy = (torch.arange(H, device=input.device, dtype=torch.float32) + offset) * sh
    cx = cx[None, :, None].expand(H, W, wh.shape[0])
    cy = cy[:, None, None].expand(H, W, wh.shape[0])
    boxes = torch.stack([(cx - wh[:, 0]) / IW, (cy - wh[:, 1]) / IH, (cx + wh[:, 0]) / IW,
                         (cy + wh[:, 1]) / IH], -1)
    if clip:
        boxes = boxes.clamp(0.0, 1.0)
    var = torch.tensor(list(variance), dtype=torch.float32, device=input.device).expand_as(boxes).contiguous()
    return boxes.to(input.dtype), var.to(input.dtype)


def _jaccard(box, boxes, normalized):
    """Reference JaccardOverlap of one box against [K, 4] boxes (+1 widths when not normalized)."""
    norm = 0.0 if normalized else 1.0

    def area(b):
        w, h = b[..., 2] - b[..., 0], b[..., 3] - b[..., 1]
        bad = (w < 0) | (h < 0)
        a = (w + norm) * (h + norm)
        return torch.where(bad, torch.zeros_like(a), a)
    ix1 = torch.maximum(box[0], boxes[:, 0])
    iy1 = torch.maximum(box[1], boxes[:, 1])
    ix2 = torch.minimum(box[2], boxes[:, 2])
    iy2 = torch.minimum(box[3], boxes[:, 3])
    inter = (ix2 - ix1 + norm) * (iy2 - iy1 + norm)
    disjoint = (boxes[:, 0] > box[2]) | (boxes[:, 2] < box[0]) | (boxes[:, 1] > box[3]) | (boxes[:, 3] < box[1])
    iou = inter / (area(box[None])[0] + area(boxes) - inter)
    return torch.where(disjoint, torch.zeros_like(iou), iou)


def _nms_fast(boxes, scores, score_threshold, nms_threshold, eta, top_k, normalized):
    """Reference NMSFast: score filter, stable descending sort, top_k, greedy suppression with the
    adaptive (eta) threshold. Returns kept indices in selection order."""
    cand = torch.nonzero(scores > score_threshold).reshape(-1)
    if cand.numel() == 0:
        return []
    order = cand[torch.sort(scores[cand], descending=True, stable=True).indices]
    if top_k > -1:
        order = order[:top_k]
    kept = []
    thr = float(nms_threshold)
    bx = boxes.float()
    for idx in order.tolist():
        keep = True
        if kept:
            ov = _jaccard(bx[idx], bx[kept], normalized)
            keep = bool((ov <= thr).all())
        if keep:
            kept.append(idx)
            if eta < 1 and thr > 0.5:
                thr *= eta
    return kept


def multiclass_nms(bboxes, scores, score_threshold, nms_top_k, keep_top_k, nms_threshold=0.3,
                   normalized=True, nms_eta=1.0, background_label=0, rois_num=None):
    """Reference `phi/kernels/cpu/multiclass_nms3_kernel.cc`. bboxes [N, M, 4] with scores
    [N, C, M] (or bboxes [M, C, 4] / scores [M, C] with ``rois_num`` per image). Returns
    (out [K, 6] rows = label, score, x1, y1, x2, y2 — per image by label, then selection order;
    index [K, 1] into the flattened inputs; nms_rois_num [N])."""
    three = scores.dim() == 3
    dev = bboxes.device
    if three:
        n = scores.shape[0]
        starts = None
    else:
        cnt = rois_num.to("cpu").long().tolist()
        n = len(cnt)
        starts = [0]
        for c_ in cnt:
            starts.append(starts[-1] + c_)
    rows, idxs, nums = [], [], []
    for i in range(n):
        if three:
            sc, bb, off = scores[i], bboxes[i], i * scores.shape[2]   # sc [C, M], bb [M, 4]
            C = sc.shape[0]
        else:
            s0, s1 = starts[i], starts[i + 1]
            if s0 == s1:
                nums.append(0)
                continue
            sc, bb, off = scores[s0:s1].t(), bboxes[s0:s1], s0 * scores.shape[1]  # sc [C, m]
            C = sc.shape[0]
        sel = {}
        total = 0
        for c in range(C):
            if c == background_label:
                continue
            boxes_c = bb if three else bb[:, c]
            k = _nms_fast(boxes_c, sc[c], score_threshold, nms_threshold, nms_eta, nms_top_k, normalized)
            if not three:
                k = sorted(k)
            sel[c] = k
            total += len(k)
        if keep_top_k > -1 and total > keep_top_k:
            pairs = [(float(sc[c, j]), c, j) for c in sorted(sel) for j in sel[c]]
            order = sorted(range(len(pairs)), key=lambda t: -pairs[t][0])  # stable descending
            new = {}
            for t in order[:keep_top_k]:
                _, c, j = pairs[t]
                new.setdefault(c, []).append(j)
            if not three:
                new = {c: sorted(v) for c, v in new.items()}
            sel = new
            total = keep_top_k
        for c in sorted(sel):
            for j in sel[c]:
                box = bb[j] if three else bb[j, c]
                rows.append(torch.cat([torch.tensor([float(c), float(sc[c, j])], device=dev),
                                       box.float().to(dev)]))
                idxs.append(off + (j if three else j * scores.shape[1] + c))
        nums.append(total)
    out = torch.stack(rows).to(bboxes.dtype) if rows else bboxes.new_zeros((0, 6))
    index = torch.tensor(idxs, dtype=torch.int32, device=dev).reshape(-1, 1)
    return out, index, torch.tensor(nums, dtype=torch.int32, device=dev)


# ------------------------------------------------------------------------------ detection set
def matrix_nms(bboxes, scores, score_threshold, post_threshold, nms_top_k, keep_top_k,
               use_gaussian=False, gaussian_sigma=2.0, background_label=0, normalized=True,
               return_index=False, return_rois_num=True, name=None):
    """Matrix NMS (SOLOv2; reference `phi/kernels/cpu/matrix_nms_kernel.cc`): per class the
    score-filtered top ``nms_top_k`` boxes are decayed at once — for box i, the minimum over
    higher-scored boxes j of f(iou_ij, max_iou_j) with f = (1 − iou)/(1 − max_iou) (linear) or
    exp((max_iou² − iou²)·σ) (gaussian) — instead of greedy suppression; decayed scores ≤
    ``post_threshold`` are dropped, then the best ``keep_top_k`` over all classes are kept.
    bboxes [N, M, 4], scores [N, C, M]. Returns (out [K, 6] = label, score, box; rois_num [N];
    index [K, 1]) in the reference's order of optional outputs."""
    N, C, M = scores.shape
    dev = bboxes.device
    rows, idxs, nums = [], [], []
    for i in range(N):
        cls_l, sc_l, ix_l = [], [], []
        bb = bboxes[i].float()
        for c in range(C):
            if c == background_label:
                continue
            s = scores[i, c].float()
            cand = torch.nonzero(s > score_threshold).reshape(-1)
            if cand.numel() == 0:
                continue
            order = cand[torch.sort(s[cand], descending=True, stable=True).indices]
            if nms_top_k > -1:
                order = order[:nms_top_k]
            b = bb[order]
            n = order.numel()
            iou = torch.stack([_jaccard(b[k], b, normalized) for k in range(n)])  # [n, n]
            iou = torch.tril(iou, -1)                         # iou[i, j], j < i
            iou_max = iou.max(1).values                       # max over higher-scored boxes
            if use_gaussian:
                dec = torch.exp((iou_max[None, :] ** 2 - iou ** 2) * gaussian_sigma)
            else:
                dec = (1.0 - iou) / (1.0 - iou_max[None, :])
            lower = torch.tril(torch.ones(n, n, dtype=torch.bool, device=dev), -1)
            dec = torch.where(lower, dec, torch.ones_like(dec))
            ds = dec.min(1).values * s[order]
            keep = ds > post_threshold
            cls_l.append(torch.full((int(keep.sum()),), float(c), device=dev))
            sc_l.append(ds[keep])
            ix_l.append(order[keep])
        if not sc_l or sum(t.numel() for t in sc_l) == 0:
            nums.append(0)
            continue
        cl, sc, ix = torch.cat(cls_l), torch.cat(sc_l), torch.cat(ix_l)
        num = sc.numel() if keep_top_k <= -1 else min(sc.numel(), keep_top_k)
        top = torch.sort(sc, descending=True, stable=True).indices[:num]
        for t in top.tolist():
            rows.append(torch.cat([torch.stack([cl[t], sc[t]]), bb[ix[t]]]))
            idxs.append(i * M + int(ix[t]))
        nums.append(num)
    out = torch.stack(rows).to(bboxes.dtype) if rows else bboxes.new_zeros((0, 2 + bboxes.shape[-1]))
    index = torch.tensor(idxs, dtype=torch.int32, device=dev).reshape(-1, 1)
    rn = torch.tensor(nums, dtype=torch.int32, device=dev)
    res = [out]
    if return_rois_num:
        res.append(rn)
    if return_index:
        res.append(index)
    return tuple(res) if len(res) > 1 else out


_BBOX_CLIP = math.log(1000.0 / 16.0)


def _greedy_nms(boxes, scores, thresh, eta, pixel_offset):
    """Reference `funcs/detection/nms_util.h` NMS: highest score first, adaptive threshold."""
    order = torch.sort(scores, descending=True, stable=True).indices.tolist()
    kept, thr = [], float(thresh)
    bx = boxes.float()
    for idx in order:
        keep = True
        if kept:
            keep = bool((_jaccard(bx[idx], bx[kept], not pixel_offset) <= thr).all())
        if keep:
            kept.append(idx)
            if eta < 1 and thr > 0.5:
                thr *= eta
    return torch.tensor(kept, dtype=torch.long, device=boxes.device)


def generate_proposals(scores, bbox_deltas, img_size, anchors, variances, pre_nms_top_n=6000,
                       post_nms_top_n=1000, nms_thresh=0.5, min_size=0.1, eta=1.0,
                       pixel_offset=False, return_rois_num=False, name=None):
    """RPN proposals (reference `phi/kernels/cpu/generate_proposals_v2_kernel.cc`): per image the
    top ``pre_nms_top_n`` anchors by objectness are decoded (box deltas × variances, log-size clip
    at log(1000/16)), clipped to the image, filtered by ``min_size`` (and centre inside the image
    with pixel offset), NMS'd and cut to ``post_nms_top_n``. scores [N, A, H, W], bbox_deltas
    [N, 4A, H, W], img_size [N, 2] (h, w), anchors / variances [H, W, A, 4]."""
    N = scores.shape[0]
    dev = scores.device
    sc_all = scores.permute(0, 2, 3, 1).reshape(N, -1)
    bd_all = bbox_deltas.permute(0, 2, 3, 1).reshape(N, -1, 4)
    an = anchors.reshape(-1, 4).float()
    va = variances.reshape(-1, 4).float()
    off = 1.0 if pixel_offset else 0.0
    rois, probs, nums = [], [], []
    for i in range(N):
        s = sc_all[i].float()
        k = s.numel() if pre_nms_top_n <= 0 or pre_nms_top_n >= s.numel() else pre_nms_top_n
        idx = torch.sort(s, descending=True, stable=True).indices[:k]
        s, d, a, v = s[idx], bd_all[i][idx].float(), an[idx], va[idx]
        aw = a[:, 2] - a[:, 0] + off
        ah = a[:, 3] - a[:, 1] + off
        acx, acy = a[:, 0] + 0.5 * aw, a[:, 1] + 0.5 * ah
        cx = v[:, 0] * d[:, 0] * aw + acx
        cy = v[:, 1] * d[:, 1] * ah + acy
        w = torch.exp(torch.clamp(v[:, 2] * d[:, 2], max=_BBOX_CLIP)) * aw
        h = torch.exp(torch.clamp(v[:, 3] * d[:, 3], max=_BBOX_CLIP)) * ah
        p = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2 - off, cy + h / 2 - off], -1)
        ih, iw = float(img_size[i, 0]), float(img_size[i, 1])
        p = torch.stack([p[:, 0].clamp(0, iw - off), p[:, 1].clamp(0, ih - off),
                         p[:, 2].clamp(0, iw - off), p[:, 3].clamp(0, ih - off)], -1)
        ws, hs = p[:, 2] - p[:, 0] + off, p[:, 3] - p[:, 1] + off
        ms = max(float(min_size), 1.0)
        keep = (ws >= ms) & (hs >= ms)
        if pixel_offset:
            keep &= (p[:, 0] + ws / 2 <= iw) & (p[:, 1] + hs / 2 <= ih)
        keep = torch.nonzero(keep).reshape(-1)
        if keep.numel() == 0:
            rois.append(torch.zeros((1, 4), device=dev))
            probs.append(torch.zeros((1, 1), device=dev))
            nums.append(1)
            continue
        p, s = p[keep], s[keep]
        if nms_thresh > 0:
            kn = _greedy_nms(p, s, nms_thresh, eta, pixel_offset)
            if 0 < post_nms_top_n < kn.numel():
                kn = kn[:post_nms_top_n]
            p, s = p[kn], s[kn]
        rois.append(p)
        probs.append(s.reshape(-1, 1))
        nums.append(p.shape[0])
    rpn_rois = torch.cat(rois).to(scores.dtype)
    rpn_probs = torch.cat(probs).to(scores.dtype)
    rn = torch.tensor(nums, dtype=torch.int32, device=dev)
    return (rpn_rois, rpn_probs, rn) if return_rois_num else (rpn_rois, rpn_probs, None)


def distribute_fpn_proposals(fpn_rois, min_level, max_level, refer_level, refer_scale,
                             pixel_offset=False, rois_num=None, name=None):
    """FPN level assignment (reference `phi/kernels/cpu/distribute_fpn_proposals_kernel.cc`):
    level = clamp(floor(log2(√area / refer_scale + 1e-6) + refer_level)), rois regrouped per level
    (image-major inside each level), ``restore_ind`` [N, 1] maps the concatenation back to the input
    order. Returns (multi_rois, restore_ind, rois_num_per_level or None)."""
    dev = fpn_rois.device
    b = fpn_rois.float()
    off = 1.0 if pixel_offset else 0.0
    w, h = b[:, 2] - b[:, 0], b[:, 3] - b[:, 1]
    area = torch.where((w < 0) | (h < 0), torch.zeros_like(w), (w + off) * (h + off))
    lvl = torch.floor(torch.log2(torch.sqrt(area) / refer_scale + 1e-6) + refer_level)
    lvl = lvl.clamp(min_level, max_level).long()
    R = b.shape[0]
    if rois_num is not None:
        img = torch.repeat_interleave(torch.arange(rois_num.numel(), device=dev), rois_num.to(dev).long())
        nimg = rois_num.numel()
    else:
        img = torch.zeros(R, dtype=torch.long, device=dev)
        nimg = 1
    multi, per_level_num, order = [], [], []
    for L in range(min_level, max_level + 1):
        sel = torch.nonzero(lvl == L).reshape(-1)  # input order == image-major order
        multi.append(fpn_rois[sel])
        order.append(sel)
        per_level_num.append(torch.bincount(img[sel], minlength=nimg).to(torch.int32))
    cat = torch.cat(order)
    restore = torch.empty(R, dtype=torch.int32, device=dev)
    restore[cat] = torch.arange(R, dtype=torch.int32, device=dev)
    return multi, restore.reshape(-1, 1), (per_level_num if rois_num is not None else None)


def psroi_pool(x, boxes, boxes_num, output_size, spatial_scale=1.0, name=None):
    """Position-sensitive ROI average pooling (R-FCN; reference `phi/kernels/cpu/psroi_pool_kernel.cc`):
    output channel c, bin (ph, pw) averages input channel (c·oh + ph)·ow + pw over the bin's pixels
    (ROI corners rounded, end + 1, × spatial_scale; bins floor/ceil-clipped to the map). Computed
    with an integral image, so it is vectorised and differentiable."""
    oh, ow = (output_size, output_size) if isinstance(output_size, int) else tuple(output_size)
    N, Cin, H, W = x.shape
    Co = Cin // (oh * ow)
    assert Co * oh * ow == Cin, "input channels must equal output_channels × pooled_h × pooled_w"
    dev = x.device
    R = boxes.shape[0]
    if R == 0:
        return x.new_zeros((0, Co, oh, ow))
    bidx = torch.repeat_interleave(torch.arange(N, device=dev), boxes_num.to(dev).long())
    bx = torch.round(boxes.float())
    x0, y0 = bx[:, 0] * spatial_scale, bx[:, 1] * spatial_scale
    x1, y1 = (bx[:, 2] + 1.0) * spatial_scale, (bx[:, 3] + 1.0) * spatial_scale
    rh, rw = (y1 - y0).clamp_min(0.1), (x1 - x0).clamp_min(0.1)
    ph = torch.arange(oh, device=dev).float()
    pw = torch.arange(ow, device=dev).float()
    hs = torch.floor(ph[None] * (rh / oh)[:, None] + y0[:, None]).long().clamp(0, H)
    he = torch.ceil((ph[None] + 1) * (rh / oh)[:, None] + y0[:, None]).long().clamp(0, H)
    ws = torch.floor(pw[None] * (rw / ow)[:, None] + x0[:, None]).long().clamp(0, W)
    we = torch.ceil((pw[None] + 1) * (rw / ow)[:, None] + x0[:, None]).long().clamp(0, W)
    integ = F.pad(x.float().cumsum(2).cumsum(3), (1, 0, 1, 0))      # [N, Cin, H+1, W+1]
    xc = integ[bidx].reshape(R, Co, oh, ow, H + 1, W + 1)
    # channel (c, ph, pw) reads bin (ph, pw): gather the four corners per (r, c, ph, pw)
    def at(hi, wi):  # hi [R, oh], wi [R, ow] -> [R, Co, oh, ow]
        lin = hi[:, :, None] * (W + 1) + wi[:, None, :]                  # [R, oh, ow]
        flat = xc.reshape(R, Co, oh, ow, -1)
        return torch.gather(flat, 4, lin[:, None, :, :, None].expand(R, Co, oh, ow, 1)).squeeze(-1)
    s = at(he, we) - at(hs, we) - at(he, ws) + at(hs, ws)
    cnt = ((he - hs)[:, :, None] * (we - ws)[:, None, :]).float()        # [R, oh, ow]
    empty = cnt <= 0
    out = torch.where(empty[:, None], torch.zeros_like(s), s / cnt.clamp_min(1.0)[:, None])
    return out.to(x.dtype)


def yolo_loss(x, gt_box, gt_label, anchors, anchor_mask, class_num, ignore_thresh, downsample_ratio,
              gt_score=None, use_label_smooth=True, name=None, scale_x_y=1.0):
    """YOLOv3 loss (reference `phi/kernels/cpu/yolov3_loss_kernel.cc`), vectorised: per image the
    predictions whose best IoU with any valid gt exceeds ``ignore_thresh`` are excluded from the
    negative objectness term; each valid gt picks its best-IoU anchor (shape only) and, when that
    anchor is in ``anchor_mask``, adds sigmoid-CE x/y + L1 w/h location loss (× (2 − w·h)·score),
    per-class sigmoid-CE (label smoothing min(1/C, 1/40)) and a positive objectness target.
    x [N, mask·(5 + C), H, W], gt_box [N, B, 4] (cx, cy, w, h normalised), gt_label [N, B].
    Returns the per-image loss [N]."""
    N, _, H, W = x.shape
    A = len(anchor_mask)
    B = gt_box.shape[1]
    dev = x.device
    xr = x.reshape(N, A, 5 + class_num, H, W)
    input_size = downsample_ratio * H
    an = torch.tensor(anchors, dtype=torch.float32, device=dev).reshape(-1, 2)
    am = torch.tensor(anchor_mask, dtype=torch.long, device=dev)
    scale, bias = float(scale_x_y), -0.5 * (float(scale_x_y) - 1.0)
    gs = gt_score.float() if gt_score is not None else torch.ones(N, B, device=dev)
    gb = gt_box.float()
    valid = (gb[..., 2] > 1e-6) & (gb[..., 3] > 1e-6)
    pos_t, neg_t = 1.0, 0.0
    if use_label_smooth:
        sw = min(1.0 / class_num, 1.0 / 40)
        pos_t, neg_t = 1.0 - sw, sw

    def sce(v, t):
        return torch.clamp(v, min=0) - v * t + torch.log1p(torch.exp(-v.abs()))

    with torch.no_grad():
        xf = xr.float()
        gx = torch.arange(W, device=dev).float()[None, None, None, :]
        gy = torch.arange(H, device=dev).float()[None, None, :, None]
        aw = an[am][:, 0].reshape(1, A, 1, 1)
        ah = an[am][:, 1].reshape(1, A, 1, 1)
        px = (gx + torch.sigmoid(xf[:, :, 0]) * scale + bias) / H
        py = (gy + torch.sigmoid(xf[:, :, 1]) * scale + bias) / H
        pw = torch.exp(xf[:, :, 2]) * aw / input_size
        ph = torch.exp(xf[:, :, 3]) * ah / input_size

        def iou_c(cx1, cy1, w1, h1, cx2, cy2, w2, h2):
            iw = torch.minimum(cx1 + w1 / 2, cx2 + w2 / 2) - torch.maximum(cx1 - w1 / 2, cx2 - w2 / 2)
            ih = torch.minimum(cy1 + h1 / 2, cy2 + h2 / 2) - torch.maximum(cy1 - h1 / 2, cy2 - h2 / 2)
            inter = torch.where((iw < 0) | (ih < 0), torch.zeros_like(iw), iw * ih)
            return inter / (w1 * h1 + w2 * h2 - inter)
        e = (Ellipsis, None)
        g = [gb[..., k].reshape(N, 1, 1, 1, B) for k in range(4)]
        ious = iou_c(px[e], py[e], pw[e], ph[e], *g)                     # [N, A, H, W, B]
        ious = torch.where(valid.reshape(N, 1, 1, 1, B), ious, torch.zeros_like(ious))
        best = ious.max(-1).values if B > 0 else torch.zeros_like(px)
        obj = torch.where(best > ignore_thresh, torch.full_like(best, -1.0), torch.zeros_like(best))
        # gt -> best anchor by shape
        aw_all = an[:, 0] / input_size
        ah_all = an[:, 1] / input_size
        ia = iou_c(torch.zeros(1, device=dev), torch.zeros(1, device=dev), aw_all[None, None],
                   ah_all[None, None], torch.zeros(1, device=dev), torch.zeros(1, device=dev),
                   gb[..., 2:3], gb[..., 3:4])                             # [N, B, nA]
        best_n = torch.zeros(N, B, dtype=torch.long, device=dev)
        best_v = torch.zeros(N, B, device=dev)
        for k in range(an.shape[0]):  # strict > keeps the first maximum like the reference
            upd = ia[..., k] > best_v
            best_v = torch.where(upd, ia[..., k], best_v)
            best_n = torch.where(upd, torch.full_like(best_n, k), best_n)
        lut = torch.full((an.shape[0],), -1, dtype=torch.long, device=dev)
        lut[am] = torch.arange(A, device=dev)
        midx = lut[best_n]
        gi = (gb[..., 0] * W).long().clamp(0, W - 1)
        gj = (gb[..., 1] * H).long().clamp(0, H - 1)
        posm = valid & (midx >= 0)
        # objectness targets: later gts overwrite earlier ones on the same cell (reference loop)
        for t in range(B):
            for n in torch.nonzero(posm[:, t]).reshape(-1).tolist():
                obj[n, midx[n, t], gj[n, t], gi[n, t]] = gs[n, t]
    loss = x.new_zeros(N, dtype=torch.float32)
    if bool(posm.any()):
        n_i, t_i = torch.nonzero(posm, as_tuple=True)
        a_i, j_i, i_i = midx[n_i, t_i], gj[n_i, t_i], gi[n_i, t_i]
        pr = xr[n_i, a_i, :, j_i, i_i].float()                           # [P, 5 + C]
        gt = gb[n_i, t_i]
        sc = gs[n_i, t_i]
        tx = gt[:, 0] * W - i_i.float()
        ty = gt[:, 1] * H - j_i.float()
        bn = best_n[n_i, t_i]
        tw = torch.log(gt[:, 2] * input_size / an[bn, 0])
        th = torch.log(gt[:, 3] * input_size / an[bn, 1])
        wgt = (2.0 - gt[:, 2] * gt[:, 3]) * sc
        loc = (sce(pr[:, 0], tx) + sce(pr[:, 1], ty) + (pr[:, 2] - tw).abs() + (pr[:, 3] - th).abs()) * wgt
        lab = gt_label[n_i, t_i].long()
        tgt = torch.full((lab.numel(), class_num), neg_t, device=dev)
        tgt[torch.arange(lab.numel(), device=dev), lab] = pos_t
        cls = (sce(pr[:, 5:], tgt).sum(1)) * sc
        loss = loss.index_add(0, n_i, loc + cls)
    conf = xr[:, :, 4].float()
    pos = obj > 1e-5
    negm = (obj <= 1e-5) & (obj > -0.5)
    lo = torch.where(pos, sce(conf, torch.ones_like(conf)) * obj, torch.zeros_like(conf)) + \
        torch.where(negm, sce(conf, torch.zeros_like(conf)), torch.zeros_like(conf))
    return (loss + lo.sum((1, 2, 3))).to(x.dtype)


def read_file(filename, name=None):
    """The file's bytes as a uint8 tensor (reference `read_file_op.cc`)."""
    import numpy as np
    with open(filename, "rb") as f:
        data = f.read()
    return torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy())


def decode_jpeg(x, mode="unchanged", name=None):
    """JPEG bytes (uint8 tensor) → CHW uint8 image (reference `decode_jpeg_op.cu`, nvjpeg). Decoded
    on the host with PIL (there is no HIP JPEG decoder); ``mode`` "gray" / "rgb" converts."""
    import io
    import numpy as np
    from PIL import Image
    img = Image.open(io.BytesIO(bytes(x.detach().cpu().numpy().tobytes())))
    if mode == "gray":
        img = img.convert("L")
    elif mode == "rgb":
        img = img.convert("RGB")
    a = np.asarray(img)
    if a.ndim == 2:
        a = a[None]
    else:
        a = a.transpose(2, 0, 1)
    return torch.from_numpy(np.ascontiguousarray(a)).to(x.device)


def _layer_base():
    from ..nn.layer.base import Layer
    return Layer


class RoIAlign(_layer_base()):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self._output_size, self._spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num, aligned=True):
        return roi_align(x, boxes, boxes_num, self._output_size, self._spatial_scale, aligned=aligned)


class RoIPool(_layer_base()):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self._output_size, self._spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num):
        return roi_pool(x, boxes, boxes_num, self._output_size, self._spatial_scale)


class PSRoIPool(_layer_base()):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self.output_size, self.spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num):
        return psroi_pool(x, boxes, boxes_num, self.output_size, self.spatial_scale)


class DeformConv2D(_layer_base()):
    """Deformable conv v1 (mask None) / v2 layer (reference `vision/ops.py:1093`)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 deformable_groups=1, groups=1, weight_attr=None, bias_attr=None):
        super().__init__()
        from ..nn import initializer as I
        k = (kernel_size, kernel_size) if isinstance(kernel_size, int) else tuple(kernel_size)
        self._stride, self._padding, self._dilation = stride, padding, dilation
        self._deformable_groups, self._groups = deformable_groups, groups
        fan_in = in_channels // groups * k[0] * k[1]
        std = (2.0 / fan_in) ** 0.5
        self.weight = self.create_parameter([out_channels, in_channels // groups, k[0], k[1]],
                                            attr=weight_attr, default_initializer=I.Normal(0.0, std))
        self.bias = None if bias_attr is False else self.create_parameter([out_channels], attr=bias_attr,
                                                                           is_bias=True)

    def forward(self, x, offset, mask=None):
        return deform_conv2d(x, offset, self.weight, self.bias, self._stride, self._padding,
                             self._dilation, self._deformable_groups, self._groups, mask=mask)
