"""Own MFMA convolution backward kernels against the plain PyTorch fp32 convolution gradients:

* ``conv2d_wgrad`` — the implicit-GEMM weight gradient (``gemm.hip`` conv_wgrad_kernel: reduction
  over N·OH·OW pixels, taps × channels packed into the 256-row tile, split-K partial planes);
* ``conv2d_dgrad_strided`` — strided data gradient as one stride-1 HIP convolution per output phase.

Shapes: every distinct ResNet-50 convolution geometry (batch 2) plus odd sizes, dilation and
strides 2/3; the autograd path must not record a library fallback for them."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, tol):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    assert err <= tol * max(1.0, b.abs().max().item()), err


# N, H, W, C, K, R, stride, pad, dil   (ResNet-50 bottleneck geometries at reduced spatial size)
RESNET = [
    (2, 16, 16, 64, 64, 1, 1, 0, 1),
    (2, 16, 16, 64, 64, 3, 1, 1, 1),
    (2, 16, 16, 64, 256, 1, 1, 0, 1),
    (2, 16, 16, 256, 64, 1, 1, 0, 1),
    (2, 16, 16, 256, 128, 1, 1, 0, 1),
    (2, 16, 16, 128, 128, 3, 2, 1, 1),
    (2, 16, 16, 256, 512, 1, 2, 0, 1),
    (2, 8, 8, 512, 256, 1, 1, 0, 1),
    (2, 8, 8, 256, 256, 3, 2, 1, 1),
    (2, 4, 4, 1024, 2048, 1, 2, 0, 1),
    (1, 4, 4, 512, 512, 3, 1, 1, 1),
]
ODD = [
    (1, 13, 11, 64, 128, 3, 1, 2, 2),
    (2, 15, 13, 128, 192, 3, 2, 1, 1),
    (1, 17, 19, 64, 64, 5, 3, 2, 1),
    (1, 9, 9, 72, 64, 3, 1, 1, 1),
]


def _ref(x, w, st, pad, dil, g):
    xr, wr = x.float().clone().requires_grad_(True), w.float().clone().requires_grad_(True)
    yr = F.conv2d(xr.permute(0, 3, 1, 2), wr, None, st, pad, dil)
    yr.backward(g.float().permute(0, 3, 1, 2))
    return xr.grad, wr.grad


@pytest.mark.parametrize("N,H,W,C,K,R,st,pad,dil", RESNET + ODD)
def test_wgrad_matches_fp32(N, H, W, C, K, R, st, pad, dil):
    from paddle_infer_amd.ops import conv as CV
    torch.manual_seed(C + K + R)
    x = torch.randn(N, H, W, C, device=DEV).bfloat16()
    w = (torch.randn(K, C, R, R, device=DEV) / (C * R * R) ** 0.5).bfloat16()
    OH, OW = CV._out_hw(H, W, R, R, (st, st), (pad, pad), (dil, dil))
    g = torch.randn(N, OH, OW, K, device=DEV).bfloat16()
    _, dw_ref = _ref(x, w, st, pad, dil, g)
    dw = CV.conv2d_wgrad(x, g, R, R, (st, st), (pad, pad), (dil, dil))
    assert dw.shape == dw_ref.shape
    _close(dw, dw_ref, 1e-2)


@pytest.mark.parametrize("plan", [(64, 1), (64, 5), (128, 2), (256, 3)])
def test_wgrad_tile_and_splitk_variants(plan):
    from paddle_infer_amd.ops import conv as CV
    torch.manual_seed(3)
    x = torch.randn(3, 12, 10, 64, device=DEV).bfloat16()
    w = (torch.randn(256, 64, 3, 3, device=DEV) / 24).bfloat16()
    g = torch.randn(3, 12, 10, 256, device=DEV).bfloat16()
    _, dw_ref = _ref(x, w, 1, 1, 1, g)
    CV.WGRAD_PLAN_OVERRIDE = plan
    try:
        dw = CV.conv2d_wgrad(x, g, 3, 3, (1, 1), (1, 1), (1, 1))
    finally:
        CV.WGRAD_PLAN_OVERRIDE = None
    _close(dw, dw_ref, 1e-2)


@pytest.mark.parametrize("N,H,W,C,K,R,st,pad,dil", [c for c in RESNET + ODD if c[6] > 1])
def test_strided_dgrad_matches_fp32(N, H, W, C, K, R, st, pad, dil):
    from paddle_infer_amd.ops import conv as CV
    torch.manual_seed(C * 3 + K)
    x = torch.randn(N, H, W, C, device=DEV).bfloat16()
    w = (torch.randn(K, C, R, R, device=DEV) / (C * R * R) ** 0.5).bfloat16()
    OH, OW = CV._out_hw(H, W, R, R, (st, st), (pad, pad), (dil, dil))
    g = torch.randn(N, OH, OW, K, device=DEV).bfloat16()
    dx_ref, _ = _ref(x, w, st, pad, dil, g)
    dx = CV.conv2d_dgrad_strided(g, w, H, W, (st, st), (pad, pad), (dil, dil))
    _close(dx, dx_ref, 2e-2)


@pytest.mark.parametrize("N,H,W,C,K,R,st,pad,dil", RESNET)
def test_autograd_conv_backward_stays_on_hip(N, H, W, C, K, R, st, pad, dil):
    from paddle_infer_amd.ops import _lib
    from paddle_infer_amd.ops.conv import conv2d_nhwc
    torch.manual_seed(K)
    x = torch.randn(N, H, W, C, device=DEV).bfloat16().requires_grad_(True)
    w = (torch.randn(K, C, R, R, device=DEV) / (C * R * R) ** 0.5).requires_grad_(True)
    before = dict(_lib.FALLBACKS)
    y = conv2d_nhwc(x, w, None, st, pad, dil, "relu")
    y.backward(torch.randn_like(y))
    torch.cuda.synchronize()
    new = {k: v for k, v in _lib.FALLBACKS.items() if before.get(k) != v}
    assert not [k for k in new if k[0].startswith("conv2d")], new
    assert w.grad.dtype == torch.float32 and torch.isfinite(w.grad).all()
    assert torch.isfinite(x.grad.float()).all()


def test_resnet50_loss_curve_parity_hip_vs_library():
    """20 same-seed ResNet-50 steps on a fixed batch through paddle.DataParallel +
    paddle.optimizer.Momentum: the HIP-conv loss curve tracks the library-conv curve (both fit the
    batch; per-step gap within bf16 run-to-run noise) — the round-1 8.55-vs-5.96 gap came from
    lr 0.1 chaos on a random-init ResNet-50, not from the kernels."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "bench_resnet", os.path.join(os.path.dirname(__file__), "..", "tools", "bench_resnet.py"))
    br = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(br)
    r = br.parity(20, batch=32, res=112, lr=0.02)
    lib, hip = r["library_conv"], r["hip_conv"]
    assert abs(lib[0] - hip[0]) < 0.02 * lib[0], r
    assert lib[-1] < 0.25 * lib[0] and hip[-1] < 0.25 * hip[0], r
    # later steps: both trajectories descend together (mean gap well inside the descent)
    gap = sum(abs(a - b) for a, b in zip(lib, hip)) / len(lib)
    assert gap < 0.1 * (lib[0] - lib[-1]), r


@pytest.mark.parametrize("C,st", [(3, 2), (8, 1), (5, 1)])
def test_stem_mode_small_channel_conv(C, st):
    """C ≤ 8 (ResNet stem, 7×7 stride 2 over 3 channels): channels zero-padded to 8, eight taps per
    k-step — forward, weight and data gradients against fp32 with no library fallback."""
    from paddle_infer_amd.ops import _lib
    from paddle_infer_amd.ops.conv import conv2d_nhwc
    torch.manual_seed(C)
    x = torch.randn(2, 30, 26, C, device=DEV).bfloat16()
    w = (torch.randn(64, C, 7, 7, device=DEV) / (C * 49) ** 0.5).bfloat16()
    xh, wh = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    before = dict(_lib.FALLBACKS)
    y = conv2d_nhwc(xh, wh, None, st, 3, 1, "relu")
    xr, wr = x.float().clone().requires_grad_(True), w.float().clone().requires_grad_(True)
    yr = torch.relu(F.conv2d(xr.permute(0, 3, 1, 2), wr, None, st, 3)).permute(0, 2, 3, 1)
    _close(y, yr, 2e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    _close(wh.grad, wr.grad, 2e-2)
    _close(xh.grad, xr.grad, 3e-2)
    new = {k: v for k, v in _lib.FALLBACKS.items() if before.get(k) != v}
    assert not [k for k in new if k[0].startswith("conv2d")], new


def test_runtime_autotune_conv_plans(tmp_path):
    """With own-kernel autotuning on, conv forward / dgrad / wgrad plans are measured on the live
    operands, cached per shape, and the tuned launches stay numerically exact."""
    from paddle_infer_amd.ops import autotune as AT
    from paddle_infer_amd.ops.conv import conv2d_nhwc
    AT.CACHE.clear()
    AT.configure(enable=True, tuning_range=[0, 1 << 30], cache_file=str(tmp_path / "t.json"))
    try:
        torch.manual_seed(5)
        x = torch.randn(4, 14, 14, 128, device=DEV).bfloat16().requires_grad_(True)
        w = (torch.randn(256, 128, 3, 3, device=DEV) / 34).requires_grad_(True)
        y = conv2d_nhwc(x, w, None, 2, 1, 1, None)
        g = torch.randn_like(y)
        y.backward(g)
        xr, wr = x.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
        yr = F.conv2d(xr.permute(0, 3, 1, 2), wr, None, 2, 1).permute(0, 2, 3, 1)
        yr.backward(g.float())
        _close(y, yr, 2e-2)
        _close(x.grad, xr.grad, 3e-2)
        _close(w.grad, wr.grad, 1e-2)
        kinds = {k.split(":")[0] for k in AT.CACHE}
        assert {"conv2d_fwd", "conv2d_wgrad", "conv2d_dgrad"} <= kinds, AT.CACHE
    finally:
        AT.configure(enable=False)
        AT.CACHE.clear()
        AT._STATE["cache_file"] = None
