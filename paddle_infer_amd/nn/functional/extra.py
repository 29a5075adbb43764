"""The rest of ``paddle.nn.functional`` (reference `python/paddle/nn/functional/{activation,common,
conv,distance,extension,loss,pooling,vision}.py`): in-place activations, unpooling, folding,
channel / pixel shuffles, bilinear, the metric-learning and classification losses, margin
cross-entropy with class-center sampling, and gather_tree.

Paddle layouts and semantics (NCHW / NCDHW, ``reduction`` = mean | sum | none, Paddle's argument
names); the math is composed from PyTorch-ROCm ops — none of these is a training hot path.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as TF


def _reduce(x, reduction):
    if reduction == "mean":
        return x.mean()
    if reduction == "sum":
        return x.sum()
    if reduction == "none":
        return x
    raise ValueError(f"reduction should be 'sum', 'mean' or 'none', got {reduction}")


# ----------------------------------------------------------------------------- activations
def elu_(x, alpha=1.0, name=None):
    return TF.elu_(x, alpha)


def tanh_(x, name=None):
    return x.tanh_()


def softmax_(x, axis=-1, dtype=None, name=None):
    y = torch.softmax(x if dtype is None else x.to(dtype), axis)
    return x.copy_(y)


def rrelu(x, lower=1.0 / 8.0, upper=1.0 / 3.0, training=True, name=None):
    """Randomized leaky ReLU: negative slope ~ U(lower, upper) per element in training, the mean
    slope (lower + upper) / 2 in eval (reference `activation.py:rrelu`)."""
    if not 0 <= lower <= upper <= 1:
        raise ValueError(f"need 0 <= lower ({lower}) <= upper ({upper}) <= 1")
    if training:
        a = torch.empty_like(x).uniform_(lower, upper)
    else:
        a = (lower + upper) / 2.0
    return torch.where(x >= 0, x, x * a)


# ----------------------------------------------------------------------------- common
def zeropad2d(x, padding, data_format="NCHW", name=None):
    p = [padding] * 4 if isinstance(padding, int) else list(padding)  # left, right, top, bottom
    if data_format == "NHWC":
        return TF.pad(x.permute(0, 3, 1, 2), p).permute(0, 2, 3, 1)
    return TF.pad(x, p)


def bilinear(x1, x2, weight, bias=None, name=None):
    """out[n, o] = x1[n] W[o] x2[n]ᵀ + b[o]; weight [out, in1, in2], bias [1, out]."""
    y = torch.einsum("ni,oij,nj->no", x1, weight, x2)
    return y + bias.reshape(1, -1) if bias is not None else y


def diag_embed(input, offset=0, dim1=-2, dim2=-1):  # noqa: A002
    return torch.diag_embed(input, offset, dim1, dim2)


def pairwise_distance(x, y, p=2.0, epsilon=1e-6, keepdim=False, name=None):
    return TF.pairwise_distance(x, y, p, epsilon, keepdim)


def fold(x, output_sizes, kernel_sizes, strides=1, paddings=0, dilations=1, name=None):
    """Col2im: [N, C*kh*kw, L] → [N, C, H, W] (reference `common.py:fold`); paddings may be
    [top, left, bottom, right]-style 4-lists with equal pairs."""
    p = paddings
    if isinstance(p, (list, tuple)) and len(p) == 4:
        p = [p[0], p[1]]
    return TF.fold(x, output_sizes, kernel_sizes, dilations, p, strides)


def pixel_unshuffle(x, downscale_factor, data_format="NCHW", name=None):
    if data_format == "NHWC":
        return TF.pixel_unshuffle(x.permute(0, 3, 1, 2), downscale_factor).permute(0, 2, 3, 1)
    return TF.pixel_unshuffle(x, downscale_factor)


def channel_shuffle(x, groups, data_format="NCHW", name=None):
    if data_format == "NHWC":
        N, H, W, C = x.shape
        return x.reshape(N, H, W, groups, C // groups).transpose(3, 4).reshape(N, H, W, C)
    N, C = x.shape[:2]
    return x.reshape(N, groups, C // groups, *x.shape[2:]).transpose(1, 2).reshape(x.shape)


# ----------------------------------------------------------------------------- conv / pooling
def _unpool(fn, x, indices, kernel_size, stride, padding, output_size, nd):
    if output_size is not None:
        output_size = list(output_size)[-nd:]
    return fn(x, indices, kernel_size, stride, padding, output_size)


def max_unpool1d(x, indices, kernel_size, stride=None, padding=0, data_format="NCL",
                 output_size=None, name=None):
    return _unpool(TF.max_unpool1d, x, indices, kernel_size, stride, padding, output_size, 1)


def max_unpool2d(x, indices, kernel_size, stride=None, padding=0, data_format="NCHW",
                 output_size=None, name=None):
    return _unpool(TF.max_unpool2d, x, indices, kernel_size, stride, padding, output_size, 2)


def max_unpool3d(x, indices, kernel_size, stride=None, padding=0, data_format="NCDHW",
                 output_size=None, name=None):
    return _unpool(TF.max_unpool3d, x, indices, kernel_size, stride, padding, output_size, 3)


# ----------------------------------------------------------------------------- losses
def dice_loss(input, label, epsilon=0.00001, name=None):  # noqa: A002
    """1 - 2|X∩Y| / (|X| + |Y|) per sample, averaged (label: class ids, last dim 1)."""
    C = input.shape[-1]
    lab = TF.one_hot(label.squeeze(-1).long(), C).to(input.dtype)
    dims = tuple(range(1, input.dim()))
    inter = (input * lab).sum(dims)
    union = input.sum(dims) + lab.sum(dims)
    return (1 - (2 * inter + epsilon) / (union + epsilon)).mean()


def log_loss(input, label, epsilon=1e-4, name=None):  # noqa: A002
    return -label * torch.log(input + epsilon) - (1 - label) * torch.log(1 - input + epsilon)


def soft_margin_loss(input, label, reduction="mean", name=None):  # noqa: A002
    return _reduce(torch.log1p(torch.exp(-label.to(input.dtype) * input)), reduction)


def multi_label_soft_margin_loss(input, label, weight=None, reduction="mean", name=None):  # noqa: A002
    lab = label.to(input.dtype)
    loss = -(lab * TF.logsigmoid(input) + (1 - lab) * TF.logsigmoid(-input))
    if weight is not None:
        loss = loss * weight
    return _reduce(loss.mean(-1), reduction)


def triplet_margin_with_distance_loss(input, positive, negative, distance_function=None,  # noqa: A002
                                      margin=1.0, swap=False, reduction="mean", name=None):
    dist = distance_function or (lambda a, b: TF.pairwise_distance(a, b))
    dp, dn = dist(input, positive), dist(input, negative)
    if swap:
        dn = torch.minimum(dn, dist(positive, negative))
    return _reduce(torch.clamp(margin + dp - dn, min=0), reduction)


def npair_loss(anchor, positive, labels, l2_reg=0.002):
    """Reference `loss.py:npair_loss`: softmax cross entropy over anchor·positiveᵀ with soft
    same-label targets + L2 on the embeddings."""
    lab = labels.reshape(-1, 1)
    same = (lab == lab.t()).to(anchor.dtype)
    target = same / same.sum(1, keepdim=True)
    logits = anchor @ positive.t()
    ce = -(target * torch.log_softmax(logits, -1)).sum(1).mean()
    reg = l2_reg * ((anchor ** 2).sum(1).mean() + (positive ** 2).sum(1).mean()) * 0.25
    return ce + reg


def hsigmoid_loss(input, label, num_classes, weight, bias=None, path_table=None,  # noqa: A002
                  path_code=None, is_sparse=False, name=None):
    """Hierarchical sigmoid over the default complete binary tree of ``num_classes`` leaves
    (reference `loss.py:hsigmoid_loss`): node j of class c's path is ((c + C) >> (k+1)) - 1, its
    code bit ((c + C) >> k) & 1; loss = Σ softplus(x·w_j + b_j) - bit·(x·w_j + b_j)."""
    N = input.shape[0]
    lab = label.reshape(-1).long()
    if path_table is None:
        L = max(1, int(math.ceil(math.log2(num_classes))))
        code = lab + num_classes
        ks = torch.arange(L, device=input.device)
        nodes = (code.unsqueeze(1) >> (ks + 1)) - 1
        bits = ((code.unsqueeze(1) >> ks) & 1).to(input.dtype)
        valid = nodes >= 0
    else:
        nodes = path_table.long()
        bits = path_code.to(input.dtype)
        valid = nodes >= 0
    nodes_c = nodes.clamp(min=0)
    w = weight[nodes_c]  # [N, L, D]
    pre = (w * input.unsqueeze(1)).sum(-1)
    if bias is not None:
        pre = pre + bias.reshape(-1)[nodes_c]
    loss = (TF.softplus(pre) - bits * pre) * valid.to(input.dtype)
    return loss.sum(1, keepdim=True).reshape(N, 1)


def class_center_sample(label, num_classes, num_samples, group=None):
    """Reference `common.py:class_center_sample` (PartialFC): keep every positive class, fill up to
    ``num_samples`` with random negatives; returns (remapped_label, sampled_class_index)."""
    pos = torch.unique(label)
    if pos.numel() < num_samples:
        mask = torch.ones(num_classes, dtype=torch.bool, device=label.device)
        mask[pos] = False
        neg = torch.nonzero(mask).reshape(-1)
        neg = neg[torch.randperm(neg.numel(), device=label.device)[:num_samples - pos.numel()]]
        sampled = torch.cat([pos, neg.sort().values])
    else:
        sampled = pos
    remap = torch.full((num_classes,), -1, dtype=label.dtype, device=label.device)
    remap[sampled] = torch.arange(sampled.numel(), device=label.device, dtype=label.dtype)
    return remap[label], sampled


def margin_cross_entropy(logits, label, margin1=1.0, margin2=0.5, margin3=0.0, scale=64.0,
                         group=None, return_softmax=False, reduction="mean"):
    """ArcFace-family combined margin (reference `loss.py:margin_cross_entropy`):
    target logit cos θ → cos(m1·θ + m2) - m3, all logits × scale, then softmax CE."""
    lab = label.reshape(-1).long()
    cos = logits.clamp(-1.0, 1.0)
    tgt = cos.gather(1, lab.unsqueeze(1))
    theta = torch.acos(tgt)
    tgt_m = torch.cos(margin1 * theta + margin2) - margin3
    out = cos.scatter(1, lab.unsqueeze(1), tgt_m) * scale
    loss = TF.cross_entropy(out, lab, reduction="none").unsqueeze(1)
    loss = _reduce(loss, reduction) if reduction != "none" else loss
    if return_softmax:
        return loss, torch.softmax(out, -1)
    return loss


def sparse_attention(query, key, value, sparse_csr_offset, sparse_csr_columns, key_padding_mask=None,
                     attn_mask=None, name=None):
    """Reference `sparse_attention.py`: attention restricted to the (CSR) sparsity pattern per
    [batch, head]; q/k/v [B, H, S, D], offsets [B, H, S+1], columns [B, H, nnz]."""
    B, H, S, D = query.shape
    scores = torch.matmul(query, key.transpose(-1, -2)) / math.sqrt(D)
    allow = torch.zeros(B, H, S, S, dtype=torch.bool, device=query.device)
    for b in range(B):
        for h in range(H):
            off = sparse_csr_offset[b, h].long()
            cols = sparse_csr_columns[b, h].long()
            r = torch.repeat_interleave(torch.arange(S, device=query.device), off[1:] - off[:-1])
            allow[b, h, r, cols[:r.numel()]] = True
    if key_padding_mask is not None:
        allow &= key_padding_mask.reshape(B, 1, 1, S).bool()
    if attn_mask is not None:
        allow &= attn_mask.reshape(1, 1, S, S).bool()
    p = torch.softmax(scores.masked_fill(~allow, float("-inf")), -1).nan_to_num(0.0)
    return torch.matmul(p, value)


def gather_tree(ids, parents):
    from ..layer.rnn import gather_tree as _gt
    return _gt(ids, parents)
