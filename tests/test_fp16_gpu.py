"""fp16 instantiations of the elementwise / softmax / dropout / cross-entropy HIP kernels vs a
plain PyTorch fp32 reference (the BERT-Large fp16 inference config runs on these)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
H = torch.float16


@pytest.fixture(autouse=True)
def _hip_only():
    import paddle_infer_amd  # noqa: F401
    from paddle_infer_amd.ops import _lib
    _lib.lib()
    _lib.FALLBACKS.clear()
    yield
    assert not _lib.FALLBACKS, f"ops left the HIP path: {_lib.FALLBACKS}"


def _close(a, b, atol, rtol=1e-2):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    assert err <= atol + rtol * b.abs().max().item(), err


@pytest.mark.parametrize("act", ["gelu", "gelu_tanh", "relu", "silu"])
def test_bias_act_fp16(act):
    from paddle_infer_amd.ops import bias_act
    from paddle_infer_amd.ops.activation import _ref_act, ACTS
    x = torch.randn(300, 1024, device=DEV, dtype=H, requires_grad=True)
    b = (0.1 * torch.randn(1024, device=DEV)).to(H).requires_grad_()
    y = bias_act(x, b, act)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, br = x.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    yr = _ref_act(xr + br, ACTS[act])
    yr.backward(dy.float())
    _close(y, yr, 4e-3)
    _close(x.grad, xr.grad, 4e-3)
    _close(b.grad, br.grad, 0.1, 2e-2)


def test_softmax_mask_fp16():
    from paddle_infer_amd.ops import fused_softmax_mask
    x = torch.randn(4, 8, 128, 128, device=DEV, dtype=H, requires_grad=True)
    m = torch.randn(4, 1, 128, 128, device=DEV, dtype=H).expand(4, 8, 128, 128).contiguous()
    y = fused_softmax_mask(x, m, 0.5)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    yr = torch.softmax(xr * 0.5 + m.float(), -1)
    yr.backward(dy.float())
    _close(y, yr, 2e-3)
    _close(x.grad, xr.grad, 2e-3)


def test_dropout_fp16_mask_consistent():
    from paddle_infer_amd.ops import dropout
    x = torch.randn(1000, 512, device=DEV, dtype=H, requires_grad=True)
    y = dropout(x, 0.4)
    kept = y != 0
    assert abs(kept.float().mean().item() - 0.6) < 0.01
    _close(y[kept], (x.detach() / 0.6)[kept], 2e-3)
    y.backward(torch.ones_like(y))
    assert torch.equal(x.grad != 0, kept)


def test_cross_entropy_fp16():
    from paddle_infer_amd.ops import softmax_cross_entropy
    logits = (3 * torch.randn(256, 4000, device=DEV)).to(H).requires_grad_()
    lab = torch.randint(0, 4000, (256,), device=DEV)
    lab[::7] = -100
    loss = softmax_cross_entropy(logits, lab)
    loss.sum().backward()
    lr = logits.detach().float().requires_grad_()
    ref = F.cross_entropy(lr, lab, ignore_index=-100, reduction="none")
    ref.sum().backward()
    _close(loss, ref, 2e-3)
    _close(logits.grad, lr.grad, 2e-3)
