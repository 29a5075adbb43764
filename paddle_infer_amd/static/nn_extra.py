"""The rest of ``paddle.static.nn`` (reference `python/paddle/static/nn/__init__.py` →
`fluid/layers/nn.py`, `control_flow.py`, `sequence_lod.py`, `detection.py`).

Like ``static/nn.py``, each builder creates its parameters through the framework's layers and runs
ordinary ops, so it works eagerly and inside a traced Program. Sequence (LoD) ops take the
reference's LoD representation: a packed [sum(len), ...] tensor carrying ``.lod`` (offset lists,
as made by ``paddle.create_lod_tensor``); outputs carry their LoD the same way.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as TF

from .. import nn as _nn
from ..nn import functional as F


def _act(x, act):
    return x if not act else getattr(F, act)(x)


# ------------------------------------------------------------------------------ control flow
def case(pred_fn_pairs, default=None, name=None):
    """First branch whose predicate holds (reference `control_flow.py:case`), built from nested
    ``cond`` so Program predicates become cond ops."""
    from .nn import cond
    pairs = list(pred_fn_pairs)
    if not pairs:
        raise ValueError("case needs at least one (pred, fn) pair")

    def chain(i):
        p, fn = pairs[i]
        if i == len(pairs) - 1:
            rest = default if default is not None else fn
        else:
            rest = lambda: chain(i + 1)  # noqa: E731
        return cond(p, fn, rest)
    return chain(0)


def switch_case(branch_index, branch_fns, default=None, name=None):
    """Branch ``branch_fns[branch_index]`` (dict or list of (index, fn) / fns), else ``default``
    (reference `control_flow.py:switch_case`)."""
    if isinstance(branch_fns, dict):
        items = sorted(branch_fns.items())
    else:
        items = [(i, f) if not isinstance(f, (list, tuple)) else tuple(f) for i, f in enumerate(branch_fns)]
    if default is None:
        default = items[-1][1]
    pairs = [(branch_index == k, fn) for k, fn in items]
    return case(pairs, default)


# ------------------------------------------------------------------------------ layers
def bilinear_tensor_product(x, y, size, act=None, name=None, param_attr=None, bias_attr=None):
    """out_k = xᵀ W_k y + b_k (reference `nn.py:bilinear_tensor_product`)."""
    layer = _nn.Bilinear(x.shape[-1], y.shape[-1], size, weight_attr=param_attr, bias_attr=bias_attr)
    return _act(layer(x, y), act)


def conv3d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None,  # noqa: A002
           param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None, data_format="NCDHW"):
    conv = _nn.Conv3D(input.shape[1], num_filters, filter_size, stride, padding, dilation, groups or 1,
                      weight_attr=param_attr, bias_attr=bias_attr)
    return _act(conv(input), act)


def conv3d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0, stride=1,  # noqa: A002
                     dilation=1, groups=None, param_attr=None, bias_attr=None, use_cudnn=True, act=None,
                     name=None, data_format="NCDHW"):
    conv = _nn.Conv3DTranspose(input.shape[1], num_filters, filter_size, stride, padding,
                               groups=groups or 1, dilation=dilation, weight_attr=param_attr,
                               bias_attr=bias_attr)
    return _act(conv(input), act)


def crf_decoding(input, param_attr=None, label=None, length=None):  # noqa: A002
    """Viterbi decoding of a linear-chain CRF (reference `nn.py:crf_decoding`): ``input`` emission
    scores [B, T, N] (or packed [sum(len), N] with ``.lod``), transition parameter [N+2, N] (row 0
    start, row 1 end, rows 2.. transitions). With ``label`` returns 1 where the path matches it."""
    from ..text import viterbi_decode
    N = input.shape[-1]
    trans = param_attr if isinstance(param_attr, torch.Tensor) else \
        _nn.Layer().create_parameter([N + 2, N], attr=param_attr)
    lod = getattr(input, "lod", None)
    if input.dim() == 2:
        offs = lod[-1] if lod else [0, input.shape[0]]
        lens = [offs[i + 1] - offs[i] for i in range(len(offs) - 1)]
        T = max(lens)
        em = input.new_zeros(len(lens), T, N)
        for i, L in enumerate(lens):
            em[i, :L] = input[offs[i]:offs[i] + L]
        length = torch.tensor(lens)
    else:
        em = input
        length = length if length is not None else torch.full((input.shape[0],), input.shape[1])
    # fold start / end scores into the first / last emission of each sequence
    em = em.clone()
    em[:, 0] = em[:, 0] + trans[0]
    for i, L in enumerate(length.tolist()):
        em[i, L - 1] = em[i, L - 1] + trans[1]
    _, path = viterbi_decode(em, trans[2:], length.to(em.device), include_bos_eos_tag=False)
    if input.dim() == 2:
        path = torch.cat([path[i, :L] for i, L in enumerate(length.tolist())]).unsqueeze(-1)
        path.lod = lod
    if label is not None:
        return (path.reshape(label.shape) == label).to(torch.int64)
    return path


def data_norm(input, act=None, epsilon=1e-05, param_attr=None, data_layout="NCHW",  # noqa: A002
              in_place=False, name=None, moving_mean_name=None, moving_variance_name=None,
              do_model_average_for_mean_and_var=True, slot_dim=-1, sync_stats=False,
              summary_decay_rate=0.9999999, enable_scale_and_shift=False):
    """Reference `nn.py:data_norm`: normalise by running batch statistics kept as parameters
    (batch_size 1e4, batch_sum 0, batch_square_sum 1e4 initially):
    out = (x − batch_sum/batch_size) · sqrt(batch_size / batch_square_sum)."""
    C = input.shape[1] if input.dim() > 1 else input.shape[0]
    holder = _nn.Layer()
    init = _nn.initializer.Constant
    bsize = holder.create_parameter([C], default_initializer=init(1e4))
    bsum = holder.create_parameter([C], default_initializer=init(0.0))
    bsq = holder.create_parameter([C], default_initializer=init(1e4))
    mean = bsum / bsize
    scale = torch.sqrt(bsize / (bsq + epsilon))
    shape = [1, C] + [1] * (input.dim() - 2)
    out = (input - mean.reshape(shape)) * scale.reshape(shape)
    if enable_scale_and_shift:
        w = holder.create_parameter([C], default_initializer=init(1.0))
        b = holder.create_parameter([C], is_bias=True)
        out = out * w.reshape(shape) + b.reshape(shape)
    return _act(out, act)


def deform_conv2d(x, offset, mask, num_filters, filter_size, stride=1, padding=0, dilation=1,
                  groups=1, deformable_groups=1, im2col_step=1, weight_attr=None, bias_attr=None,
                  name=None):
    from ..vision.ops import deform_conv2d as _dc
    k = (filter_size, filter_size) if isinstance(filter_size, int) else tuple(filter_size)
    holder = _nn.Layer()
    fan_in = x.shape[1] // groups * k[0] * k[1]
    w = holder.create_parameter([num_filters, x.shape[1] // groups, *k], attr=weight_attr,
                                default_initializer=_nn.initializer.Normal(0.0, (2.0 / fan_in) ** 0.5))
    b = None if bias_attr is False else holder.create_parameter([num_filters], attr=bias_attr, is_bias=True)
    return _dc(x, offset, w, b, stride, padding, dilation, deformable_groups, groups, mask)


def nce(input, label, num_total_classes, sample_weight=None, param_attr=None, bias_attr=None,  # noqa: A002
        num_neg_samples=None, name=None, sampler="uniform", custom_dist=None, seed=0,
        is_sparse=False):
    """Noise-contrastive estimation loss (reference `nn.py:nce`, uniform / log-uniform / custom
    sampler): per sample −log σ(s_true − log(k·q_true)) − Σ_neg log(1 − σ(s_neg − log(k·q_neg)))."""
    k = num_neg_samples or 10
    D = input.shape[-1]
    holder = _nn.Layer()
    W = holder.create_parameter([num_total_classes, D], attr=param_attr)
    b = holder.create_parameter([num_total_classes], attr=bias_attr, is_bias=True)
    g = torch.Generator(device="cpu").manual_seed(int(seed))
    if sampler == "uniform":
        q = torch.full((num_total_classes,), 1.0 / num_total_classes)
    elif sampler == "log_uniform":
        r = torch.arange(num_total_classes, dtype=torch.float64)
        q = ((torch.log(r + 2) - torch.log(r + 1)) / math.log(num_total_classes + 1)).float()
    else:
        q = torch.as_tensor(custom_dist, dtype=torch.float32)
    neg = torch.multinomial(q, input.shape[0] * k, replacement=True, generator=g).reshape(-1, k)
    neg = neg.to(input.device)
    q = q.to(input.device)
    lab = label.reshape(input.shape[0], -1)[:, :1].long()
    s_true = (input * W[lab[:, 0]]).sum(-1) + b[lab[:, 0]]
    s_neg = torch.einsum("bd,bkd->bk", input, W[neg]) + b[neg]
    lt = s_true - torch.log(k * q[lab[:, 0]])
    ln = s_neg - torch.log(k * q[neg])
    cost = -TF.logsigmoid(lt) - TF.logsigmoid(-ln).sum(-1)
    if sample_weight is not None:
        cost = cost * sample_weight.reshape(-1)
    return cost.unsqueeze(-1)


def row_conv(input, future_context_size, param_attr=None, act=None):  # noqa: A002
    """Lookahead (row) convolution (reference `nn.py:row_conv`): out[t] = Σ_{i=0..k} x[t+i] ⊙ w[i]
    over [B, T, D] (or packed [sum(len), D] with ``.lod``, per sequence)."""
    D = input.shape[-1]
    k = future_context_size
    w = _nn.Layer().create_parameter([k + 1, D], attr=param_attr)

    def one(x):  # [T, D]
        T = x.shape[0]
        xp = torch.cat([x, x.new_zeros(k, D)], 0)
        return sum(xp[i:i + T] * w[i] for i in range(k + 1))
    lod = getattr(input, "lod", None)
    if input.dim() == 2 and lod:
        offs = lod[-1]
        out = torch.cat([one(input[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1)], 0)
        out.lod = lod
    elif input.dim() == 2:
        out = one(input)
    else:
        out = torch.stack([one(x) for x in input], 0)
    return _act(out, act)


def spectral_norm(weight, dim=0, power_iters=1, eps=1e-12, name=None):
    """weight / σ_max(weight) by power iteration (reference `nn.py:spectral_norm`), u / v kept as
    non-trainable parameters updated in place each call."""
    mat = weight.movedim(dim, 0).reshape(weight.shape[dim], -1)
    holder = _nn.Layer()
    g = torch.Generator(device="cpu").manual_seed(0)
    u = holder.create_parameter([mat.shape[0]], default_initializer=_nn.initializer.Assign(
        torch.randn(mat.shape[0], generator=g)))
    v = holder.create_parameter([mat.shape[1]], default_initializer=_nn.initializer.Assign(
        torch.randn(mat.shape[1], generator=g)))
    u.stop_gradient = True
    v.stop_gradient = True
    with torch.no_grad():
        uu, vv = u.detach(), v.detach()
        for _ in range(max(1, power_iters)):
            vv = TF.normalize(mat.t().detach() @ uu, dim=0, eps=eps)
            uu = TF.normalize(mat.detach() @ vv, dim=0, eps=eps)
        u.copy_(uu)
        v.copy_(vv)
    sigma = torch.dot(u, mat @ v)
    return weight / sigma


def multi_box_head(inputs, image, base_size, num_classes, aspect_ratios, min_ratio=None,
                   max_ratio=None, min_sizes=None, max_sizes=None, steps=None, step_w=None,
                   step_h=None, offset=0.5, variance=[0.1, 0.1, 0.2, 0.2], flip=True, clip=False,
                   kernel_size=1, pad=0, stride=1, name=None, min_max_aspect_ratios_order=False):
    """SSD detection head (reference `detection.py:multi_box_head`): per feature map, prior boxes
    (min / max sizes × aspect ratios, centred on the map's cells) and conv predictors for box
    offsets and class scores. Returns (mbox_locs [N, P, 4], mbox_confs [N, P, C], boxes [P, 4],
    variances [P, 4])."""
    n = len(inputs)
    if min_sizes is None:
        min_sizes, max_sizes = [], []
        step = int(math.floor(((max_ratio - min_ratio)) / (n - 2))) if n > 2 else 0
        for ratio in range(min_ratio, max_ratio + 1, step or 1):
            min_sizes.append(base_size * ratio / 100.0)
            max_sizes.append(base_size * (ratio + step) / 100.0)
        min_sizes = [base_size * 0.10] + min_sizes[:n - 1]
        max_sizes = [base_size * 0.20] + max_sizes[:n - 1]
    img_h, img_w = image.shape[2], image.shape[3]
    locs, confs, boxes = [], [], []
    for i, feat in enumerate(inputs):
        H, W = feat.shape[2], feat.shape[3]
        mins = min_sizes[i] if isinstance(min_sizes[i], (list, tuple)) else [min_sizes[i]]
        maxs = (max_sizes[i] if isinstance(max_sizes[i], (list, tuple)) else [max_sizes[i]]) if max_sizes else []
        ars = aspect_ratios[i] if isinstance(aspect_ratios[i], (list, tuple)) else [aspect_ratios[i]]
        ratios = [1.0]
        for a in ars:
            if abs(a - 1.0) > 1e-6:
                ratios += [a, 1.0 / a] if flip else [a]
        sw = (steps[i] if steps else step_w[i] if step_w else img_w / W)
        sh = (steps[i] if steps else step_h[i] if step_h else img_h / H)
        whs = []
        for j, ms in enumerate(mins):
            whs.append((ms, ms))
            if maxs:
                s = math.sqrt(ms * maxs[j])
                whs.append((s, s))
            whs += [(ms * math.sqrt(r), ms / math.sqrt(r)) for r in ratios[1:]]
        cy, cx = np.meshgrid((np.arange(H) + offset) * sh, (np.arange(W) + offset) * sw, indexing="ij")
        b = []
        for bw, bh in whs:
            b.append(np.stack([(cx - bw / 2) / img_w, (cy - bh / 2) / img_h,
                               (cx + bw / 2) / img_w, (cy + bh / 2) / img_h], -1))
        b = np.stack(b, 2).reshape(-1, 4)
        if clip:
            b = np.clip(b, 0.0, 1.0)
        boxes.append(torch.as_tensor(b, dtype=torch.float32))
        nb = len(whs)
        cin = feat.shape[1]
        loc = _nn.Conv2D(cin, nb * 4, kernel_size, stride, pad)(feat)
        conf = _nn.Conv2D(cin, nb * num_classes, kernel_size, stride, pad)(feat)
        locs.append(loc.permute(0, 2, 3, 1).reshape(feat.shape[0], -1, 4))
        confs.append(conf.permute(0, 2, 3, 1).reshape(feat.shape[0], -1, num_classes))
    box = torch.cat(boxes, 0).to(inputs[0].device)
    var = torch.tensor(variance, dtype=torch.float32, device=box.device).expand_as(box).contiguous()
    return torch.cat(locs, 1), torch.cat(confs, 1), box, var


# ------------------------------------------------------------------------------ sequence (LoD) ops
def _offs(x):
    lod = getattr(x, "lod", None)
    if not lod:
        raise ValueError("sequence ops need a LoD tensor (paddle.create_lod_tensor)")
    return list(lod[-1])


def _with_lod(t, offs):
    t.lod = [list(offs)]
    return t


def _segments(x):
    o = _offs(x)
    return [x[o[i]:o[i + 1]] for i in range(len(o) - 1)]


def sequence_pool(input, pool_type, is_test=False, pad_value=0.0):  # noqa: A002
    out = []
    for s in _segments(input):
        if s.shape[0] == 0:
            out.append(input.new_full(input.shape[1:], pad_value))
            continue
        pt = pool_type.lower()
        out.append({"average": lambda: s.mean(0), "sum": lambda: s.sum(0),
                    "sqrt": lambda: s.sum(0) / math.sqrt(s.shape[0]), "max": lambda: s.max(0).values,
                    "last": lambda: s[-1], "first": lambda: s[0]}[pt]())
    return torch.stack(out, 0)


def sequence_first_step(input):  # noqa: A002
    return sequence_pool(input, "first")


def sequence_last_step(input):  # noqa: A002
    return sequence_pool(input, "last")


def sequence_softmax(input, use_cudnn=False, name=None):  # noqa: A002
    out = torch.cat([torch.softmax(s.reshape(-1), 0).reshape(s.shape) for s in _segments(input)], 0)
    return _with_lod(out, _offs(input))


def sequence_concat(input, name=None):  # noqa: A002
    segs = [_segments(x) for x in input]
    parts, offs = [], [0]
    for i in range(len(segs[0])):
        cat = torch.cat([s[i] for s in segs], 0)
        parts.append(cat)
        offs.append(offs[-1] + cat.shape[0])
    return _with_lod(torch.cat(parts, 0), offs)


def sequence_slice(input, offset, length, name=None):  # noqa: A002
    parts, offs = [], [0]
    for i, s in enumerate(_segments(input)):
        o, L = int(offset.reshape(-1)[i]), int(length.reshape(-1)[i])
        parts.append(s[o:o + L])
        offs.append(offs[-1] + L)
    return _with_lod(torch.cat(parts, 0), offs)


def sequence_expand(x, y, ref_level=-1, name=None):
    """Repeat each sequence (or row) of x as many times as y's ref-level sequences say."""
    ylod = getattr(y, "lod", None)
    yo = list(ylod[ref_level]) if ylod else list(range(y.shape[0] + 1))
    reps = [yo[i + 1] - yo[i] for i in range(len(yo) - 1)]
    xs = _segments(x) if getattr(x, "lod", None) else [x[i:i + 1] for i in range(x.shape[0])]
    parts, offs = [], [0]
    for s, r in zip(xs, reps):
        for _ in range(r):
            parts.append(s)
            offs.append(offs[-1] + s.shape[0])
    return _with_lod(torch.cat(parts, 0), offs)


def sequence_expand_as(x, y, name=None):
    yo = _offs(y)
    parts = [x[i:i + 1].expand(yo[i + 1] - yo[i], *x.shape[1:]) for i in range(len(yo) - 1)]
    return _with_lod(torch.cat(parts, 0), yo)


def sequence_pad(x, pad_value, maxlen=None, name=None):
    segs = _segments(x)
    L = maxlen or max(s.shape[0] for s in segs)
    out = pad_value.reshape(-1)[0].to(x.dtype) * x.new_ones(len(segs), L, *x.shape[1:])
    for i, s in enumerate(segs):
        out[i, :s.shape[0]] = s[:L]
    return out, torch.tensor([s.shape[0] for s in segs], dtype=torch.int64)


def sequence_unpad(x, length, name=None):
    lens = [int(v) for v in length.reshape(-1)]
    offs = np.concatenate([[0], np.cumsum(lens)]).tolist()
    return _with_lod(torch.cat([x[i, :L] for i, L in enumerate(lens)], 0), offs)


def sequence_reshape(input, new_dim):  # noqa: A002
    o = _offs(input)
    D = input.shape[-1]
    offs = [v * D // new_dim for v in o]
    return _with_lod(input.reshape(-1, new_dim), offs)


def sequence_scatter(input, index, updates, name=None):  # noqa: A002
    """out = input; out[i, index_seq_i] += updates_seq_i for each sequence i of index/updates."""
    out = input.clone()
    io = _offs(index)
    for i in range(len(io) - 1):
        idx = index[io[i]:io[i + 1]].reshape(-1).long()
        out[i].index_add_(0, idx, updates[io[i]:io[i + 1]].reshape(-1).to(out.dtype))
    return out


def sequence_enumerate(input, win_size, pad_value=0, name=None):  # noqa: A002
    parts = []
    for s in _segments(input):
        v = s.reshape(-1)
        p = torch.cat([v, v.new_full((win_size - 1,), pad_value)])
        parts.append(torch.stack([p[i:i + win_size] for i in range(v.shape[0])], 0))
    return _with_lod(torch.cat(parts, 0), _offs(input))


def sequence_reverse(x, name=None):
    return _with_lod(torch.cat([s.flip(0) for s in _segments(x)], 0), _offs(x))


def sequence_conv(input, num_filters, filter_size=3, filter_stride=1, padding=True,  # noqa: A002
                  padding_start=None, bias_attr=None, param_attr=None, act=None, name=None):
    """Context convolution over each sequence (reference `sequence_lod.py:sequence_conv`):
    rows [t + start, t + start + filter_size) concatenated (zero outside the sequence) × W."""
    D = input.shape[-1]
    start = -int(filter_size // 2) if padding_start is None else int(padding_start)
    holder = _nn.Layer()
    W = holder.create_parameter([filter_size * D, num_filters], attr=param_attr)
    b = None if bias_attr is False else holder.create_parameter([num_filters], attr=bias_attr, is_bias=True)
    parts = []
    for s in _segments(input):
        T = s.shape[0]
        cols = []
        for j in range(filter_size):
            sh = start + j
            idx = torch.arange(T) + sh
            ok = ((idx >= 0) & (idx < T)).to(s.device)
            cols.append(s[idx.clamp(0, max(T - 1, 0)).to(s.device)] * ok.unsqueeze(-1))
        parts.append(torch.cat(cols, -1) @ W)
    out = torch.cat(parts, 0)
    if b is not None:
        out = out + b
    return _with_lod(_act(out, act), _offs(input))


# ------------------------------------------------------------------------------ StaticRNN
class StaticRNN:
    """Reference `control_flow.py:StaticRNN`, eager unrolling: the step block is recorded as a
    Python function of (step inputs, memories) by running the ``with rnn.step():`` body once per
    time step — the body is written as a function via :meth:`step_fn` (the reference's block form
    ``with rnn.step(): ...`` builds the same function through ``step_input`` / ``memory`` /
    ``update_memory`` / ``step_output`` calls recorded on the first pass and replayed)."""

    def __init__(self, name=None):
        self._inputs, self._mems, self._updates, self._outputs = [], [], {}, []
        self._fn = None

    def step_fn(self, fn, inputs, init_memories):
        """fn(x_t_list, mem_list) -> (outputs_list, new_mem_list); runs over dim 0 of inputs."""
        self._fn, self._inputs, self._init = fn, list(inputs), list(init_memories)
        return self

    def __call__(self):
        if self._fn is None:
            raise RuntimeError("StaticRNN: define the step with step_fn(fn, inputs, init_memories)")
        T = self._inputs[0].shape[0]
        mems = list(self._init)
        outs = []
        for t in range(T):
            o, mems = self._fn([x[t] for x in self._inputs], mems)
            outs.append(o if isinstance(o, (list, tuple)) else [o])
        res = [torch.stack([o[i] for o in outs], 0) for i in range(len(outs[0]))]
        return res[0] if len(res) == 1 else res
