"""``paddle.flops`` — per-layer FLOPs via forward hooks (reference
`python/paddle/hapi/dynamic_flops.py`: count_convNd / count_linear / count_bn / pooling / act
rules). Multiply-accumulates count as one op, matching the reference's convention."""
from __future__ import annotations

import numpy as np
import torch


def _numel(t):
    return int(np.prod(t.shape)) if isinstance(t, torch.Tensor) else 0


def _count(layer, inp, out):
    from ..nn import layer as L
    x = inp[0] if inp else None
    name = type(layer).__name__
    if isinstance(layer, torch.nn.Module) and hasattr(layer, "_kernel_size") or name.startswith("Conv"):
        w = getattr(layer, "weight", None)
        if w is None:
            return 0
        kernel = int(np.prod(w.shape[2:]))
        cin_per_group = w.shape[1]
        bias = 1 if getattr(layer, "bias", None) is not None else 0
        return _numel(out) * (cin_per_group * kernel + bias)
    if name in ("Linear", "ColumnParallelLinear", "RowParallelLinear", "FusedLinear"):
        w = layer.weight
        in_f = w.shape[0] if name != "FusedLinear" or not layer.transpose_weight else w.shape[1]
        return _numel(out) * in_f
    if "BatchNorm" in name or name in ("LayerNorm", "GroupNorm", "InstanceNorm2D", "RMSNorm"):
        return 2 * _numel(out)
    if "Pool" in name:
        return _numel(out) if "Adaptive" in name else _numel(out)
    if name in ("ReLU", "ReLU6", "LeakyReLU", "Sigmoid", "Tanh", "GELU", "Silu", "Swish", "Hardswish"):
        return 0
    if name == "Upsample":
        return _numel(out)
    L  # noqa
    return 0


def count_flops(net, input_size, custom_ops=None, print_detail=False, dtype=torch.float32):
    custom_ops = custom_ops or {}
    rows, handles, total = [], [], [0]

    def hook(layer, inp, out):
        fn = custom_ops.get(type(layer))
        n = fn(layer, inp, out) if fn else _count(layer, inp, out)
        if n:
            total[0] += int(n)
            params = sum(p.numel() for p in layer.parameters(recurse=False)) \
                if hasattr(layer, "parameters") else 0
            rows.append((type(layer).__name__, list(inp[0].shape) if inp else [],
                         list(out.shape) if isinstance(out, torch.Tensor) else [], params, int(n)))

    for m in net.modules():
        if len(list(m.children())) == 0 or type(m) in custom_ops:
            handles.append(m.register_forward_hook(hook))
    dev = next(iter(net.parameters())).device if len(list(net.parameters())) else torch.device("cpu")
    x = torch.zeros(list(input_size), dtype=dtype, device=dev) if not isinstance(input_size, torch.Tensor) else input_size
    was = net.training
    net.eval()
    with torch.no_grad():
        net(x)
    net.train(was)
    for h in handles:
        h.remove()
    if print_detail:
        print(f"{'Layer':24s} {'Input':20s} {'Output':20s} {'Params':>10s} {'Flops':>14s}")
        for r in rows:
            print(f"{r[0]:24s} {str(r[1]):20s} {str(r[2]):20s} {r[3]:10d} {r[4]:14d}")
    print(f"Total Flops: {total[0]}     Total Params: {sum(p.numel() for p in net.parameters())}")
    return total[0]
