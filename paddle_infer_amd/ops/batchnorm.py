"""Fused BatchNorm (+ residual add) (+ ReLU / ReLU6) — ``csrc/kernels/batchnorm.hip``.

Parity: reference `phi/kernels/gpu/batch_norm_kernel.cu`, `fused_bn_activation_op.cu`,
`fused_bn_add_activation_op.cu`. ``batch_norm_act(x, …, act, residual)`` computes
``act(BN(x) + residual)`` in one normalise pass after one statistics pass (training) or in a single
pass from the running statistics (eval); the backward reads the saved output for act' (the
residual itself is not kept) and returns the residual's gradient from the same pass.
NCHW and NHWC (``data_format`` "NHWC"/"NLC" or a channels_last tensor) layouts, f32 / bf16.
Running statistics are updated in place on the device with Paddle's momentum convention
(running = momentum·running + (1 − momentum)·batch). CPU tensors run the PyTorch reference.
"""
from __future__ import annotations

import threading

import torch
import torch.nn.functional as TF

from . import _lib

_ACT = {"none": 0, None: 0, "identity": 0, "relu": 1, "relu6": 2}
_MAX_PARTS = 2048  # statistics partial blocks (batchnorm.hip MAX_PARTS)
_GRID_SET = [False]


def _grid_once():
    """PIAMD_BN_GRID="elems_per_block,max_blocks" retunes the NHWC statistics / reduction grid
    (batchnorm.hip piamd_bn_set_parts); read once."""
    if _GRID_SET[0]:
        return
    _GRID_SET[0] = True
    import os
    v = os.environ.get("PIAMD_BN_GRID")
    if v:
        e, p = (int(t) for t in v.split(","))
        _lib.call("piamd_bn_set_parts", e, p)


def _layout(x, data_format):
    """(nhwc, N, C, S) for a [N, C, *spatial] (NCHW) or channels-last / NHWC tensor."""
    if data_format in ("NHWC", "NLC", "NDHWC"):
        N, C = x.shape[0], x.shape[-1]
        return True, N, C, x.numel() // (N * C)
    N, C = x.shape[0], x.shape[1]
    S = x.numel() // (N * C)
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous():
        return True, N, C, S
    return False, N, C, S


def _supported(x, nhwc, C):
    if not (x.is_cuda and x.dtype in (torch.float32, torch.bfloat16)):
        return False
    return not nhwc or C % 8 == 0 or C >= 256 or 256 % C == 0


def _reference(x, running_mean, running_var, weight, bias, training, momentum, eps, act,
               residual, data_format):
    nhwc = data_format in ("NHWC", "NLC", "NDHWC")
    dt = x.dtype
    xin = x.movedim(-1, 1) if nhwc else x
    if dt in (torch.bfloat16, torch.float16):  # f32 statistics, like the kernels
        xin = xin.float()
    y = TF.batch_norm(xin, running_mean, running_var, weight, bias, training, 1.0 - momentum, eps)
    y = y.movedim(1, -1) if nhwc else y
    if residual is not None:
        y = y + residual.to(y.dtype)
    y = y.to(dt)
    if act == 1:
        y = torch.relu(y)
    elif act == 2:
        y = torch.clamp(y, 0.0, 6.0)
    return y


def _conv_stats(x, training, nhwc, C):
    """(partials [3, C, P], P) a conv forward attached to ``x`` (unmodified since), else (None, 0)."""
    t = getattr(x, "_piamd_bn_part", None)
    if t is None or not training or not nhwc:
        return None, 0
    part, P, ver = t
    if ver != x._version or part.shape != (3, C, P) or part.device != x.device:
        return None, 0
    return part, P


_JOIN = threading.local()


class join_sink:
    """``with join_sink(j):`` the next BatchNorm with a residual hands the residual's gradient to
    the :class:`ops.conv.ResidualGradJoin` ``j`` (when its conv armed it) instead of returning it."""

    def __init__(self, j):
        self.j = j

    def __enter__(self):
        _JOIN.sink = self.j
        return self.j

    def __exit__(self, *exc):
        _JOIN.sink = None
        return False


def _take_sink():
    j = getattr(_JOIN, "sink", None)
    _JOIN.sink = None
    return j


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, training, momentum,
                eps, act, nhwc, dims, join=None):
        N, C, S = dims
        xc = x if (nhwc and not x.is_contiguous() and x.dim() == 4) else x.contiguous()
        if nhwc and x.dim() == 4 and not x.is_contiguous():  # channels_last NCHW view → [N,H,W,C]
            xc = x.permute(0, 2, 3, 1).contiguous()
        res = None
        if residual is not None:
            res = residual.permute(0, 2, 3, 1).contiguous() if (nhwc and residual.dim() == 4 and
                                                                 residual.shape[1] == C and
                                                                 not residual.is_contiguous()) \
                else residual.contiguous()
        dev = x.device
        g = weight.float().contiguous() if weight is not None else None
        b = bias.float().contiguous() if bias is not None else None
        mean = torch.empty(C, device=dev, dtype=torch.float32)
        rstd = torch.empty(C, device=dev, dtype=torch.float32)
        ws = torch.empty(2 * C + 3 * _MAX_PARTS * C, device=dev, dtype=torch.float32)
        y = torch.empty_like(xc)
        rm = running_mean if running_mean is not None and running_mean.dtype == torch.float32 else None
        rv = running_var if running_var is not None and running_var.dtype == torch.float32 else None
        if not training and (rm is None or rv is None):
            raise ValueError("eval-mode batch_norm needs f32 running statistics")
        _grid_once()
        # ReLU without a residual: keep the affine fold so the backward derives the mask from x
        # (x·scale + shift > 0, the forward's own test) instead of reading y
        ss = (torch.empty(2 * C, device=dev, dtype=torch.float32)
              if act == 1 and res is None and nhwc and C % 8 == 0 else None)
        # statistics the conv forward left on its output (ops/conv.py BN_STATS): finalize those
        # instead of a statistics pass over x
        part, P = _conv_stats(x, training, nhwc, C)
        _lib.call("piamd_bn_fwd3", int(x.dtype == torch.bfloat16), int(nhwc), xc.data_ptr(),
                  _lib.ptr(res), y.data_ptr(), N, C, S, _lib.ptr(g), _lib.ptr(b), _lib.ptr(rm),
                  _lib.ptr(rv), mean.data_ptr(), rstd.data_ptr(), float(momentum), float(eps),
                  int(training), int(act), ws.data_ptr(), _lib.ptr(ss), _lib.ptr(part), P,
                  _lib.stream())
        ctx.save_for_backward(xc, y, g, mean, rstd, ss)
        ctx.join = join if residual is not None else None
        ctx.meta = (training, act, nhwc, dims, residual is not None, weight, bias,
                    x.dim() == 4 and nhwc and not x.is_contiguous())
        if ctx.meta[-1]:
            return y.permute(0, 3, 1, 2)  # back to the caller's NCHW (channels_last) view
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, y, g, mean, rstd, ss = ctx.saved_tensors
        training, act, nhwc, (N, C, S), has_res, weight, bias, cl_view = ctx.meta
        dyc = dy.permute(0, 2, 3, 1).contiguous() if cl_view else dy.contiguous()
        dx = torch.empty_like(xc)
        dres = torch.empty_like(xc) if has_res else None
        dg = torch.empty(C, device=xc.device, dtype=torch.float32)
        db = torch.empty(C, device=xc.device, dtype=torch.float32)
        ws = torch.empty(3 * C + 2 * _MAX_PARTS * C, device=xc.device, dtype=torch.float32)
        _lib.call("piamd_bn_bwd2", int(xc.dtype == torch.bfloat16), int(nhwc), dyc.data_ptr(),
                  y.data_ptr(), xc.data_ptr(), dx.data_ptr(), _lib.ptr(dres), N, C, S, _lib.ptr(g),
                  mean.data_ptr(), rstd.data_ptr(), dg.data_ptr(), db.data_ptr(), int(training),
                  int(act), ws.data_ptr(), _lib.ptr(ss), _lib.stream())
        j = ctx.join
        if j is not None and j.armed and dres is not None:  # the joined conv adds it (ops/conv.py)
            j.dres = dres
            dres = None
        if cl_view:
            dx = dx.permute(0, 3, 1, 2)
            dres = dres.permute(0, 3, 1, 2) if dres is not None else None
        gw = dg.to(weight.dtype) if weight is not None and ctx.needs_input_grad[1] else None
        gb = db.to(bias.dtype) if bias is not None and ctx.needs_input_grad[2] else None
        return dx, gw, gb, dres, None, None, None, None, None, None, None, None, None


def batch_norm_act(x, running_mean, running_var, weight=None, bias=None, training=False,
                   momentum=0.9, epsilon=1e-5, act="none", residual=None, data_format="NCHW"):
    """``act(batch_norm(x) + residual)`` (Paddle momentum convention)."""
    a = _ACT[act]
    nhwc, N, C, S = _layout(x, data_format)
    if (nhwc and x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and x.dim() >= 3
            and not _supported(x, nhwc, C)
            and (residual is None or residual.shape == x.shape)):
        # channel counts the NHWC kernels do not tile (C ∤ 256, C % 8, C < 256): the NCHW kernels
        # take any C — run them on channel-major copies (own kernels, autograd through the moves)
        cl = x.dim() == 4 and not x.is_contiguous() and data_format not in ("NHWC", "NLC", "NDHWC")
        to_cm = (lambda t: t.contiguous()) if cl else (lambda t: t.movedim(-1, 1).contiguous())
        y = batch_norm_act(to_cm(x), running_mean, running_var, weight, bias, training, momentum,
                           epsilon, act, to_cm(residual) if residual is not None else None, "NCHW")
        return y.contiguous(memory_format=torch.channels_last) if cl else y.movedim(1, -1).contiguous()
    if not _supported(x, nhwc, C) or (residual is not None and residual.shape != x.shape):
        return _reference(x, running_mean, running_var, weight, bias, training, momentum, epsilon,
                          a, residual, data_format)
    join = _take_sink() if residual is not None else None
    return _BNAct.apply(x, weight, bias, residual, running_mean, running_var, bool(training),
                        momentum, epsilon, a, nhwc, (N, C, S), join)


# ------------------------------------------------------------------------------ SyncBatchNorm
def _all_gather_stats(local, group):
    import torch.distributed as dist
    W = dist.get_world_size(group)
    out = torch.empty(W * local.numel(), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous().reshape(-1), group=group)
    return out.view((W,) + tuple(local.shape))


def _welford_merge(g):
    """g [W, 3, C] (count, mean, M2) → (n [C], mean [C], M2 [C]) — parallel Welford merge."""
    n = g[:, 0].sum(0)
    mean = (g[:, 0] * g[:, 1]).sum(0) / n.clamp_min(1)
    m2 = g[:, 2].sum(0) + (g[:, 0] * (g[:, 1] - mean) ** 2).sum(0)
    return n, mean, m2


class _SyncBN(torch.autograd.Function):
    """Cross-rank batch norm: Welford (count, mean, M2) triples all-gathered over ``group`` and
    merged (GPU: inside ``piamd_bn_fwd3`` as channel-major partials), backward sums all-reduced.
    Reference `phi/kernels/gpu/sync_batch_norm_kernel.cu:192` (dγ / dβ are the local sums, like
    the reference's KeBNBackwardScaleBias; the data-parallel gradient reduction sums them)."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, group, nhwc):
        import torch.distributed as dist
        if nhwc:
            N, C = x.shape[0], x.shape[-1]
        else:
            N, C = x.shape[0], x.shape[1]
        S = x.numel() // (N * C)
        xc = x.contiguous()
        dev = x.device
        gpu = x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and _supported(x, nhwc, C)
        if gpu:
            local = torch.empty((3, C), device=dev, dtype=torch.float32)
            ws = torch.empty(3 * _MAX_PARTS * C + 3 * C, device=dev, dtype=torch.float32)
            _lib.call("piamd_bn_local_stats", int(x.dtype == torch.bfloat16), int(nhwc), xc.data_ptr(),
                      N, C, S, ws.data_ptr(), local.data_ptr(), _lib.stream())
        else:
            xf = xc.float().movedim(-1, 1) if nhwc else xc.float()
            dims = [0] + list(range(2, xf.dim()))
            m = xf.mean(dims)
            shp = [1, C] + [1] * (xf.dim() - 2)
            local = torch.stack([torch.full_like(m, float(N * S)), m, ((xf - m.view(shp)) ** 2).sum(dims)])
        multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        g = _all_gather_stats(local, group) if multi else local[None]
        n_tot = float(g[:, 0, 0].sum())
        if gpu:
            part_t = g.permute(1, 2, 0).contiguous()  # [3][C][W] channel-major partials
            mean = torch.empty(C, device=dev, dtype=torch.float32)
            rstd = torch.empty(C, device=dev, dtype=torch.float32)
            y = torch.empty_like(xc)
            gw = weight.float().contiguous() if weight is not None else None
            gb = bias.float().contiguous() if bias is not None else None
            rm = running_mean if running_mean is not None and running_mean.dtype == torch.float32 else None
            rv = running_var if running_var is not None and running_var.dtype == torch.float32 else None
            _lib.call("piamd_bn_fwd3", int(x.dtype == torch.bfloat16), int(nhwc), xc.data_ptr(), None,
                      y.data_ptr(), N, C, S, _lib.ptr(gw), _lib.ptr(gb), _lib.ptr(rm), _lib.ptr(rv),
                      mean.data_ptr(), rstd.data_ptr(), float(momentum), float(eps), 1, 0,
                      ws.data_ptr(), None, part_t.data_ptr(), part_t.shape[-1], _lib.stream())
            if running_mean is not None and rm is None:  # non-f32 running statistics
                with torch.no_grad():
                    var_u = (g[:, 2].sum(0) + (g[:, 0] * (g[:, 1] - mean) ** 2).sum(0)) / max(n_tot - 1, 1)
                    running_mean.mul_(momentum).add_((1 - momentum) * mean.to(running_mean.dtype))
                    running_var.mul_(momentum).add_((1 - momentum) * var_u.to(running_var.dtype))
            ctx.save_for_backward(xc, y, gw, mean, rstd)
        else:
            n, mean, m2 = _welford_merge(g)
            var = m2 / n.clamp_min(1)
            rstd = torch.rsqrt(var + eps)
            if running_mean is not None:
                with torch.no_grad():
                    running_mean.mul_(momentum).add_((1 - momentum) * mean.to(running_mean.dtype))
                    running_var.mul_(momentum).add_((1 - momentum) * (m2 / (n - 1).clamp_min(1)).to(running_var.dtype))
            xf = xc.float().movedim(-1, 1) if nhwc else xc.float()
            shp = [1, C] + [1] * (xf.dim() - 2)
            xh = (xf - mean.view(shp)) * rstd.view(shp)
            yf = xh * (weight.float().view(shp) if weight is not None else 1.0) + \
                (bias.float().view(shp) if bias is not None else 0.0)
            y = (yf.movedim(1, -1) if nhwc else yf).to(x.dtype).contiguous()
            ctx.save_for_backward(xc, y, weight, mean, rstd)
        ctx.meta = (gpu, nhwc, N, C, S, n_tot, group, weight is not None, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        import torch.distributed as dist
        xc, y, gw, mean, rstd = ctx.saved_tensors
        gpu, nhwc, N, C, S, n_tot, group, has_w, has_b = ctx.meta
        dyc = dy.contiguous()
        multi = dist.is_initialized() and dist.get_world_size(group) > 1
        if gpu:
            sums = torch.empty((2, C), device=xc.device, dtype=torch.float32)
            ws = torch.empty(2 * _MAX_PARTS * C + 3 * C, device=xc.device, dtype=torch.float32)
            _lib.call("piamd_bn_bwd_local_sums", int(xc.dtype == torch.bfloat16), int(nhwc), dyc.data_ptr(),
                      y.data_ptr(), xc.data_ptr(), N, C, S, mean.data_ptr(), rstd.data_ptr(), 0,
                      ws.data_ptr(), None, sums.data_ptr(), _lib.stream())
            gs = sums.clone()
            if multi:
                dist.all_reduce(gs, group=group)
            dx = torch.empty_like(xc)
            _lib.call("piamd_bn_bwd_apply_sums", int(xc.dtype == torch.bfloat16), int(nhwc), dyc.data_ptr(),
                      y.data_ptr(), xc.data_ptr(), dx.data_ptr(), None, N, C, S, _lib.ptr(gw),
                      mean.data_ptr(), rstd.data_ptr(), 0, gs.data_ptr(), float(n_tot), ws.data_ptr(),
                      None, _lib.stream())
        else:
            xf = xc.float().movedim(-1, 1) if nhwc else xc.float()
            df = dyc.float().movedim(-1, 1) if nhwc else dyc.float()
            dims = [0] + list(range(2, xf.dim()))
            shp = [1, C] + [1] * (xf.dim() - 2)
            xh = (xf - mean.view(shp)) * rstd.view(shp)
            sums = torch.stack([df.sum(dims), (df * xh).sum(dims)])
            gs = sums.clone()
            if multi:
                dist.all_reduce(gs, group=group)
            gam = gw.float().view(shp) if gw is not None else 1.0
            dxf = gam * rstd.view(shp) * (df - gs[0].view(shp) / n_tot - xh * gs[1].view(shp) / n_tot)
            dx = (dxf.movedim(1, -1) if nhwc else dxf).to(xc.dtype)
        dwt = sums[1].to(gw.dtype) if has_w and ctx.needs_input_grad[1] else None
        dbs = sums[0].to(gw.dtype if gw is not None else torch.float32) if has_b and ctx.needs_input_grad[2] else None
        return dx, dwt, dbs, None, None, None, None, None, None


def sync_batch_norm(x, running_mean, running_var, weight=None, bias=None, training=True, momentum=0.9,
                    epsilon=1e-5, group=None, data_format="NCHW"):
    """Batch norm with statistics over every rank of ``group`` (training); eval = plain BN."""
    import torch.distributed as dist
    nhwc = data_format in ("NHWC", "NLC", "NDHWC")
    if not training or not (dist.is_available() and dist.is_initialized()):
        return batch_norm_act(x, running_mean, running_var, weight, bias, training, momentum, epsilon,
                              data_format=data_format)
    return _SyncBN.apply(x, weight, bias, running_mean, running_var, momentum, epsilon, group, nhwc)
