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
