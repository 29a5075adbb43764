"""Tensor-parallel ColumnParallelLinear with a FROZEN weight (LoRA / BitFit style): the input
gradient must still be all-reduced over the model-parallel group (reference
`fleet/layers/mpu/mp_layers.py:155`, c_identity in ColumnParallelLinear.forward)."""
import torch

from dist_utils import run_distributed


def _worker(rank, world, full_w, x0):
    import torch.distributed as dist
    from paddle_infer_amd.distributed.fleet.mp_layers import ColumnParallelLinear
    g = dist.new_group(list(range(world)))
    layer = ColumnParallelLinear(full_w.shape[0], full_w.shape[1], gather_output=False,
                                 mp_group=g, has_bias=True)
    with torch.no_grad():
        layer.weight.copy_(full_w.chunk(world, dim=1)[rank])
        layer.bias.zero_()
    layer.weight.requires_grad_(False)  # frozen: the plain-linear branch
    x = x0.clone().requires_grad_(True)
    y = layer(x)
    (y * (rank + 1.0)).sum().backward()  # rank-dependent upstream gradient
    return x.grad, layer.bias.grad


def test_column_parallel_frozen_weight_input_grad_allreduced():
    torch.manual_seed(0)
    w = torch.randn(8, 6)
    x = torch.randn(3, 8)
    res = run_distributed(_worker, 2, w, x)
    # single-process reference: dX = Σ_r (r+1)·1·W_rᵀ
    ref = torch.zeros_like(x)
    for r, wr in enumerate(w.chunk(2, dim=1)):
        ref += (r + 1.0) * torch.ones(3, wr.shape[1]) @ wr.t()
    for r in range(2):
        dx, db = res[r]
        assert torch.allclose(dx, ref, atol=1e-5), (r, dx, ref)
        assert torch.allclose(db, torch.full((3,), 3.0 * (r + 1)), atol=1e-5)
