"""Merged (multi-tensor) optimizer update (``optim.hip`` multi_tensor_kernel, reference
merged_momentum / merged_adam) against the per-parameter PyTorch update of the same optimizer:
SGD / Momentum (nesterov, L2 decay, per-parameter lr multiplier) through paddle.optimizer, and the
raw Adam / AdamW ops, over mixed shapes incl. channels_last 4-D weights and bf16 gradients."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(64, 3, 7, 7), (10,), (4099,), (256, 128, 3, 3), (1000, 2048), (1,)]
    ps = []
    for s in shapes:
        p = torch.randn(*s, generator=g).cuda()
        if len(s) == 4:
            p = p.contiguous(memory_format=torch.channels_last)
        ps.append(p.requires_grad_(True))
    return ps


@pytest.mark.parametrize("kind", ["sgd", "momentum", "nesterov"])
def test_paddle_optimizer_merged_matches_per_param(kind):
    import paddle_infer_amd as paddle
    res = {}
    for merged in (True, False):
        ps = _params(0)
        ps[1].optimize_attr = {"learning_rate": 0.5}
        if kind == "sgd":
            opt = paddle.optimizer.SGD(learning_rate=0.1, parameters=ps, weight_decay=1e-3)
        else:
            opt = paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9, parameters=ps,
                                            use_nesterov=kind == "nesterov", weight_decay=1e-3)
        if not merged:
            opt._merged_op = None
        g = torch.Generator().manual_seed(7)
        for _ in range(3):
            for p in ps:
                p.grad = torch.randn(p.shape, generator=g).cuda().to(memory_format=torch.preserve_format)
                if p.dim() == 4:
                    p.grad = p.grad.contiguous(memory_format=torch.channels_last)
            assert opt._merged_ok([(p, p.grad) for p in ps]) == merged
            opt.step()
        torch.cuda.synchronize()
        res[merged] = [p.detach().clone() for p in ps]
    for a, b in zip(res[True], res[False]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("op", [2, 3])
@pytest.mark.parametrize("gbf16", [False, True])
def test_multi_tensor_adam_ops_match_reference(op, gbf16):
    from paddle_infer_amd.ops.optim import multi_tensor_update
    ps = [p.detach() for p in _params(1)]
    ref = [p.cpu().clone() for p in ps]
    s1 = [torch.zeros_like(p) for p in ps]
    s2 = [torch.zeros_like(p) for p in ps]
    r1 = [torch.zeros_like(p) for p in ref]
    r2 = [torch.zeros_like(p) for p in ref]
    g = torch.Generator().manual_seed(3)
    cache = {}
    for step in (1, 2, 3):
        grads = [torch.randn(p.shape, generator=g) for p in ref]
        gg = [x.cuda().to(torch.bfloat16 if gbf16 else torch.float32) for x in grads]
        gg = [x.contiguous(memory_format=torch.channels_last) if x.dim() == 4 else x for x in gg]
        multi_tensor_update(op, [(p, x, a, b, 0.01, 1.0) for p, x, a, b in zip(ps, gg, s1, s2)],
                            1e-2, cache, beta1=0.9, beta2=0.99, eps=1e-8, step=step)
        multi_tensor_update(op, [(p, x.float().cpu(), a, b, 0.01, 1.0)
                                 for p, x, a, b in zip(ref, gg, r1, r2)],
                            1e-2, None, beta1=0.9, beta2=0.99, eps=1e-8, step=step)
    for a, b in zip(ps, ref):
        torch.testing.assert_close(a.cpu(), b, rtol=1e-4, atol=1e-5)
