"""The framework's own GEMMs beyond the bf16 training linears, against fp32 PyTorch references:
fp16 assembly-GEMM variants (every layout, accumulate, fused epilogues), the batched assembly GEMM
(broadcast and layouts), the skinny MFMA kernel (`csrc/kernels/gemm_small.hip`: every tile shape,
split-K, bias / activation / alpha / residual epilogues), the ``gemm_nt`` padding paths, and the
``matmul`` dispatcher with its autograd (paddle.matmul, bmm, static matmul_v2, linear inference,
linear_bias_act, fused_matmul_bias). An autouse fixture asserts no op left the HIP path."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _no_fallback():
    from paddle_infer_amd.ops import _lib
    _lib.FALLBACKS.clear()
    yield
    assert not _lib.FALLBACKS, f"ops left the HIP path: {_lib.FALLBACKS}"


def _close(got, ref, rel=0.02, atol=0.0):
    got, ref = got.float(), ref.float()
    err = (got - ref).abs().max().item()
    tol = atol + rel * max(ref.abs().max().item(), 1e-3)
    assert err <= tol, (err, tol)


def _rand(*shape, dtype=torch.bfloat16, scale=1.0, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed + sum(shape))
    return (scale * torch.randn(*shape, device=DEV, generator=g)).to(dtype)


# ---------------------------------------------------------------------------- asm fp16 variants
@pytest.mark.parametrize("ta,tb", [(False, True), (True, False), (False, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (1000, 1008, 448), (4352, 520, 256)])
@pytest.mark.parametrize("kind", ["h16", "h16acc", "f32", "f32acc"])
def test_asm_fp16_layouts(M, N, K, ta, tb, kind):
    from paddle_infer_amd.ops.gemm import asm_gemm
    a = _rand(*((K, M) if ta else (M, K)), dtype=torch.float16)
    b = _rand(*((N, K) if tb else (K, N)), dtype=torch.float16, seed=1)
    r = (a.t() if ta else a).float() @ (b.t() if tb else b).float()
    if kind.endswith("acc"):
        c = _rand(M, N, dtype=torch.float16 if kind == "h16acc" else torch.float32, seed=2)
        r = r + c.float()
        asm_gemm(a, b, ta, tb, out=c, accumulate=True)
    else:
        c = asm_gemm(a, b, ta, tb, out_f32=kind == "f32")
        assert c.dtype == (torch.float32 if kind == "f32" else torch.float16)
    _close(c, r, 0.01)


@pytest.mark.parametrize("act", ["none", "gelu_tanh", "relu"])
def test_asm_fp16_fused_epilogues(act):
    from paddle_infer_amd.ops.gemm import asm_gemm
    M, N, K = 520, 768, 256
    x = _rand(M, K, dtype=torch.float16)
    w = _rand(N, K, dtype=torch.float16, scale=0.1, seed=1)
    bias = _rand(N, dtype=torch.float16, seed=2)
    aux = torch.empty(M, N, device=DEV, dtype=torch.float16)
    y = asm_gemm(x, w, trans_b=True, epi="bias_act", act=act, bias=bias, aux=aux)
    pre = x.float() @ w.float().t() + bias.float()
    _close(aux, pre, 0.01)
    ref = {"none": pre, "relu": torch.relu(pre),
           "gelu_tanh": torch.nn.functional.gelu(pre, approximate="tanh")}[act]
    _close(y, ref, 0.01)
    if act != "none":
        dy = _rand(M, K, dtype=torch.float16, seed=3)
        w2 = _rand(N, K, dtype=torch.float16, scale=0.1, seed=4)
        d = asm_gemm(dy, w2, trans_b=True, epi="dact", act=act, aux=aux)
        h = aux.float().requires_grad_(True)
        fn = torch.relu if act == "relu" else (lambda t: torch.nn.functional.gelu(t, approximate="tanh"))
        gd = torch.autograd.grad(fn(h).sum(), h)[0]
        _close(d, (dy.float() @ w2.float().t()) * gd, 0.01)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("with_aux", [False, True])
def test_asm_exact_gelu_epilogue(dtype, with_aux):
    """bias + exact (erf) GELU fused into the asm epilogue: within the output dtype's rounding of
    the erf reference, including the negative tail where the tanh form drifts."""
    from paddle_infer_amd.ops.gemm import asm_gemm
    M, N, K = 1030, 1024, 512
    x = _rand(M, K, dtype=dtype)
    w = _rand(N, K, dtype=dtype, scale=0.12, seed=1)
    bias = _rand(N, dtype=dtype, seed=2)
    aux = torch.empty(M, N, device=DEV, dtype=dtype) if with_aux else None
    y = asm_gemm(x, w, trans_b=True, epi="bias_act", act="gelu", bias=bias, aux=aux)
    pre = (x.float() @ w.float().t() + bias.float()).requires_grad_(True)
    ref = torch.nn.functional.gelu(pre)
    dg, = torch.autograd.grad(ref.sum(), pre)
    pre, ref = pre.detach(), ref.detach()
    ulp = 2.0 ** (-8 if dtype == torch.bfloat16 else -11)
    # the 16-bit rounding of pre (one ulp either way vs the fp32 reference) plus the output's
    tol = 1.5 * ulp * (ref.abs() + (pre * dg).abs()) + 1e-5
    err = (y.float() - ref).abs()
    bad = err > tol
    assert not bad.any(), (pre[bad][:8], ref[bad][:8], y.float()[bad][:8])
    if with_aux:  # exactly the GELU of the stored pre-activation, up to the output rounding
        r2 = torch.nn.functional.gelu(aux.float())
        assert ((y.float() - r2).abs() <= ulp * r2.abs() + 1e-6).all()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("ks", [2, 4])
def test_asm_splitk_16bit_output(dtype, ks):
    """Split-K into 16-bit C: the deterministic reduce writes the operands' dtype (fp16 too)."""
    from paddle_infer_amd.ops.gemm import asm_gemm
    M, N, K = 520, 768, 1024
    a = _rand(M, K, dtype=dtype, scale=0.5)
    b = _rand(N, K, dtype=dtype, scale=0.05, seed=1)
    c = asm_gemm(a, b, trans_b=True, ksplit=ks)
    assert c.dtype == dtype
    _close(c, a.float() @ b.float().t(), 0.01)


# ---------------------------------------------------------------------------- batched asm
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("bcast", ["none", "a", "b"])
def test_asm_batched(dtype, ta, tb, bcast):
    from paddle_infer_amd.ops.gemm import asm_gemm
    nb, M, N, K = 5, 264, 320, 192
    a = _rand(*(() if bcast == "a" else (nb,)), *((K, M) if ta else (M, K)), dtype=dtype)
    b = _rand(*(() if bcast == "b" else (nb,)), *((N, K) if tb else (K, N)), dtype=dtype, seed=1)
    c = asm_gemm(a, b, ta, tb)
    assert c.shape == (nb, M, N)
    A = a.transpose(-1, -2) if ta else a
    B = b.transpose(-1, -2) if tb else b
    _close(c, A.float() @ B.float(), 0.01)


# ---------------------------------------------------------------------------- skinny kernel
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(1, 1024, 1024), (7, 4100, 320), (33, 3072, 1024), (128, 1024, 4096),
                                   (200, 516, 256)])
def test_small_gemm_configs(dtype, M, N, K):
    from paddle_infer_amd.ops.gemm import small_gemm, small_cfg, _SG_SHAPES
    a = _rand(M, K, dtype=dtype)
    b = _rand(N, K, dtype=dtype, scale=0.1, seed=1)
    ref = a.float() @ b.float().t()
    cfgs = {small_cfg(M, N, K)}
    for mb, nb in sorted(_SG_SHAPES):
        for wn in (1, 2, 4):
            for ks in (1, 2, 4):
                if ks <= K // 64:
                    cfgs.add((mb, nb, wn, 1 + (ks + wn) % 2, ks))
                    if wn == 1:  # B-deep rings: the weight stream DB k64 steps ahead of A
                        cfgs.add((mb, nb, 1, 1 | ({1: 2, 2: 4, 4: 8}[ks] << 4), ks))
    for cfg in sorted(cfgs):
        _close(small_gemm(a, b, cfg=cfg), ref, 0.01)
        if cfg[4] > 1:
            _close(small_gemm(a, b, cfg=cfg, slices=True), ref, 0.01)
    # the fixup workspace is left zeroed: a second call gives the same result
    _close(small_gemm(a, b), ref, 0.01)


@pytest.mark.parametrize("act", ["none", "gelu_tanh", "gelu", "relu", "silu"])
def test_small_gemm_epilogue(act):
    from paddle_infer_amd.ops.gemm import small_gemm
    M, N, K = 96, 1028, 512
    a = _rand(M, K)
    b = _rand(N, K, scale=0.1, seed=1)
    bias = _rand(N, seed=2)
    resid = _rand(M, N, seed=3)
    pre = 0.5 * (a.float() @ b.float().t()) + bias.float()
    ref = {"none": pre, "relu": torch.relu(pre), "silu": torch.nn.functional.silu(pre),
           "gelu": torch.nn.functional.gelu(pre),
           "gelu_tanh": torch.nn.functional.gelu(pre, approximate="tanh")}[act] + resid.float()
    for ks in (1, 4):
        got = small_gemm(a, b, alpha=0.5, bias=bias, act=act, resid=resid, cfg=(4, 2, 2, 2, ks))
        _close(got, ref, 0.01)
    got = small_gemm(a, b, out_f32=True, alpha=0.5, bias=bias, act=act, resid=resid)
    assert got.dtype == torch.float32
    _close(got, ref, 0.01)


# ---------------------------------------------------------------------------- gemm_nt + dispatcher
@pytest.mark.parametrize("M,N,K", [(3, 1000, 100), (130, 1002, 1000), (700, 3000, 520), (4096, 1024, 96)])
@pytest.mark.parametrize("act", ["none", "gelu_tanh", "gelu", "relu", "silu"])
def test_gemm_nt_padding(M, N, K, act):
    from paddle_infer_amd.ops.gemm import gemm_nt
    a = _rand(M, K, dtype=torch.float16)
    b = _rand(N, K, dtype=torch.float16, scale=0.1, seed=1)
    bias = _rand(N, dtype=torch.float16, seed=2)
    got = gemm_nt(a, b, bias=bias, act=act)
    pre = a.float() @ b.float().t() + bias.float()
    ref = {"none": pre, "relu": torch.relu(pre), "silu": torch.nn.functional.silu(pre),
           "gelu": torch.nn.functional.gelu(pre),
           "gelu_tanh": torch.nn.functional.gelu(pre, approximate="tanh")}[act]
    assert got.shape == (M, N)
    _close(got, ref, 0.01)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("xs,ys,tx,ty", [
    ((64, 256), (256, 512), False, False),
    ((2, 130, 96), (96, 200), False, False),        # N-D x, 2-D weight, K off the 64-grid
    ((4, 3, 128, 64), (4, 3, 64, 128), False, False),  # batched attention-like (K = 64)
    ((4, 3, 128, 64), (4, 3, 128, 64), False, True),   # q·kᵀ
    ((8, 256, 128), (8, 256, 384), True, False),       # transposed x
    ((2, 1, 300, 256), (5, 256, 260), False, False),   # broadcast batch dims
    ((256,), (256, 512), False, False),                # vector · matrix
    ((3, 40, 256), (256,), False, False),              # matrix · vector
])
def test_matmul_dispatch_fwd_bwd(dtype, xs, ys, tx, ty):
    import paddle_infer_amd as paddle
    x = _rand(*xs, dtype=dtype, scale=0.5).requires_grad_()
    y = _rand(*ys, dtype=dtype, scale=0.5, seed=1).requires_grad_()
    out = paddle.matmul(x, y, transpose_x=tx, transpose_y=ty)
    xf = x.detach().float().requires_grad_()
    yf = y.detach().float().requires_grad_()
    ref = torch.matmul(xf.transpose(-1, -2) if tx else xf, yf.transpose(-1, -2) if ty else yf)
    assert out.shape == ref.shape and out.dtype == dtype
    _close(out, ref, 0.02)
    g = _rand(*ref.shape, dtype=dtype, seed=3)
    out.backward(g)
    ref.backward(g.float())
    _close(x.grad, xf.grad, 0.03)
    _close(y.grad, yf.grad, 0.03)


def test_bmm_mm_addmm_and_method():
    import paddle_infer_amd as paddle
    a = _rand(6, 200, 128)
    b = _rand(6, 128, 264, seed=1)
    _close(paddle.bmm(a, b), a.float() @ b.float(), 0.02)
    _close(paddle.mm(a[0], b[0]), a[0].float() @ b[0].float(), 0.02)
    c = _rand(200, 264, seed=2)
    _close(paddle.addmm(c, a[0], b[0], beta=0.5, alpha=2.0),
           0.5 * c.float() + 2.0 * (a[0].float() @ b[0].float()), 0.02)
    _close(a.matmul(b[0, :, :200].transpose(0, 1), transpose_y=True),
           a.float() @ b[0, :, :200].float(), 0.02)


@pytest.mark.parametrize("M", [1, 16, 128, 2048])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_linear_inference_and_bias_act(M, dtype):
    from paddle_infer_amd.ops.linear import linear, linear_bias_act
    x = _rand(M, 1024, dtype=dtype, scale=0.5)
    w = _rand(1024, 3072, dtype=dtype, scale=0.05, seed=1)
    b = _rand(3072, dtype=dtype, seed=2)
    with torch.no_grad():
        _close(linear(x, w, b), x.float() @ w.float() + b.float(), 0.02)
        pre = x.float() @ w.float() + b.float()
        _close(linear_bias_act(x, w, b, "gelu"), torch.nn.functional.gelu(pre), 0.02)
        _close(linear_bias_act(x, w.t().contiguous(), b, "relu", weight_out_in=True), torch.relu(pre), 0.02)


def test_fused_matmul_bias_and_static_ops():
    from paddle_infer_amd.incubate.nn import functional as IF
    from paddle_infer_amd.static.ops_registry import REGISTRY as OPS
    x = _rand(3, 50, 256, dtype=torch.float16)
    w = _rand(256, 384, dtype=torch.float16, scale=0.1, seed=1)
    b = _rand(384, dtype=torch.float16, seed=2)
    ref = x.float() @ w.float() + b.float()
    with torch.no_grad():
        _close(IF.fused_matmul_bias(x, w, b), ref, 0.02)
        _close(IF.fused_linear(x, w.t().contiguous(), b, transpose_weight=True), ref, 0.02)
        _close(IF.fused_linear_activation(x, w, b, activation="relu"), torch.relu(ref), 0.02)
        out = OPS["matmul_v2"]({"X": [x], "Y": [w]}, {"trans_x": False, "trans_y": False})["Out"]
        _close(out, x.float() @ w.float(), 0.02)
        out = OPS["matmul"]({"X": [x], "Y": [x]}, {"transpose_Y": True, "alpha": 0.25})["Out"]
        _close(out, 0.25 * (x.float() @ x.float().transpose(-1, -2)), 0.02)
        out = OPS["mul"]({"X": [x], "Y": [w]}, {"x_num_col_dims": 2})["Out"]
        _close(out, x.float() @ w.float(), 0.02)


def test_no_library_gemm_kernels_in_fp16_bert_layer():
    """A BERT-Large-shaped fp16 encoder layer (inference, batch 1 and 32) launches no hipBLASLt /
    rocBLAS kernel: every product is the assembly GEMM or the skinny kernel."""
    from torch.profiler import ProfilerActivity, profile
    from paddle_infer_amd.ops.linear import linear, linear_bias_act
    from paddle_infer_amd import ops
    E, F_, S = 1024, 4096, 128
    ws = [_rand(E, 3 * E, dtype=torch.float16, scale=0.03, seed=1), _rand(E, E, dtype=torch.float16, scale=0.03, seed=2),
          _rand(E, F_, dtype=torch.float16, scale=0.03, seed=3), _rand(F_, E, dtype=torch.float16, scale=0.03, seed=4)]
    bs = [_rand(w.shape[1], dtype=torch.float16, seed=5) for w in ws]

    def layer(x):
        B = x.shape[0]
        qkv = linear(x, ws[0], bs[0]).reshape(B, S, 48, 64)
        a = ops.flash_attention_packed(qkv, 16, 16, causal=False).reshape(B, S, E)
        h = linear(a, ws[1], bs[1]) + x
        f = linear_bias_act(h, ws[2], bs[2], "gelu")
        return linear(f, ws[3], bs[3]) + h
    with torch.no_grad():
        for B in (1, 32):
            x = _rand(B, S, E, dtype=torch.float16, scale=0.5)
            layer(x)
            torch.cuda.synchronize()
            with profile(activities=[ProfilerActivity.CUDA]) as prof:
                layer(x)
                torch.cuda.synchronize()
            names = [e.key for e in prof.key_averages()]
            lib = [n for n in names if n.startswith("Cijk") or "rocblas" in n.lower() or "gemm" in n.lower()
                   and "piamd" not in n and "small_gemm" not in n and "agemm" not in n]
            assert not lib, lib
