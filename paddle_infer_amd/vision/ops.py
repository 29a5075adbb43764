"""``paddle.vision.ops`` (reference `python/paddle/vision/ops.py`): nms, box_coder, roi_align,
roi_pool, deform_conv2d, yolo_box, distribute_fpn_proposals (subset), as tensor compositions."""
from __future__ import annotations

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
    oh, ow = (output_size, output_size) if isinstance(output_size, int) else output_size
    bidx = torch.repeat_interleave(torch.arange(len(boxes_num), device=x.device), boxes_num.to(x.device).long())
    outs = []
    for k in range(boxes.shape[0]):
        b = int(bidx[k])
        x1, y1, x2, y2 = (boxes[k] * spatial_scale - (0.5 if aligned else 0.0)).tolist()
        H, W = x.shape[-2:]
        ys = torch.linspace(y1, y2, oh * 2 + 1, device=x.device)[1::2]
        xs = torch.linspace(x1, x2, ow * 2 + 1, device=x.device)[1::2]
        gy, gx = torch.meshgrid(ys, xs, indexing="ij")
        grid = torch.stack([gx / (W - 1) * 2 - 1, gy / (H - 1) * 2 - 1], -1)[None]
        outs.append(F.grid_sample(x[b:b + 1].float(), grid, align_corners=True)[0].to(x.dtype))
    return torch.stack(outs) if outs else x.new_zeros((0, x.shape[1], oh, ow))


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
    N, _, H, W = x.shape
    na = len(anchors) // 2
    x = x.view(N, na, 5 + class_num, H, W)
    gy, gx = torch.meshgrid(torch.arange(H, device=x.device), torch.arange(W, device=x.device), indexing="ij")
    an = torch.tensor(anchors, dtype=torch.float32, device=x.device).view(na, 2)
    bx = (torch.sigmoid(x[:, :, 0]) * scale_x_y - 0.5 * (scale_x_y - 1) + gx) / W
    by = (torch.sigmoid(x[:, :, 1]) * scale_x_y - 0.5 * (scale_x_y - 1) + gy) / H
    bw = torch.exp(x[:, :, 2]) * an[:, 0, None, None] / (W * downsample_ratio)
    bh = torch.exp(x[:, :, 3]) * an[:, 1, None, None] / (H * downsample_ratio)
    conf = torch.sigmoid(x[:, :, 4])
    probs = torch.sigmoid(x[:, :, 5:]) * conf[:, :, None]
    ih, iw = img_size[:, 0].float().view(N, 1, 1, 1), img_size[:, 1].float().view(N, 1, 1, 1)
    boxes = torch.stack([(bx - bw / 2) * iw, (by - bh / 2) * ih, (bx + bw / 2) * iw, (by + bh / 2) * ih], -1)
    if clip_bbox:
        boxes = torch.stack([boxes[..., 0].clamp(min=0), boxes[..., 1].clamp(min=0),
                             torch.minimum(boxes[..., 2], iw - 1), torch.minimum(boxes[..., 3], ih - 1)], -1)
    keep = (conf > conf_thresh).float()
    boxes = boxes * keep[..., None]
    scores = probs * keep[:, :, None]
    return boxes.reshape(N, -1, 4), scores.permute(0, 1, 3, 4, 2).reshape(N, -1, class_num)
