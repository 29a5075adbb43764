"""The OpTest cases of ``test_op_cases_cpu.py`` on the MI355X: forward of the HIP kernels (fp32 and
bf16) against the numpy references, and their gradients against the float64 CPU autograd gradients
(which the CPU tier checks by finite differences). No case may take a recorded fallback."""
import numpy as np
import pytest
import torch

from paddle_infer_amd.ops import _lib
import test_op_cases_cpu as C

pytestmark = pytest.mark.gpu

F32, BF16, F16 = (torch.float32, 1e-5), (torch.bfloat16, 3e-2), (torch.float16, 4e-3)
# (case, dtype) pairs that have a HIP kernel: LN / RMSNorm / cross-entropy / softmax / GeLU in all
# three dtypes (elementwise.hip takes f32 rows as well as 16-bit ones)
KERNEL_CASES = [(c, d) for c in (C.LayerNormCase, C.RMSNormCase, C.CrossEntropyCase, C.SoftmaxCase, C.GeluCase)
                for d in (F32, BF16, F16)]


def _grads(case, device, dtype):
    case.device = device
    names = C.GRADS[type(case)]
    t = case._tensors(requires_grad=set(names), dtype=dtype)
    out = case._run(t)[0]
    w = torch.from_numpy(np.random.default_rng(7).standard_normal(tuple(out.shape))).to(out)
    (out * w).sum().backward()
    return [t[n].grad.double().cpu() for n in names]


@pytest.mark.parametrize("case,dt", KERNEL_CASES, ids=[f"{c.__name__}-{str(d[0])[6:]}" for c, d in KERNEL_CASES])
def test_kernel_output_and_grad(case, dt):
    dtype, tol = dt
    _lib.FALLBACKS.clear()
    c = case()
    c.device = "cuda"
    if case is C.CrossEntropyCase:
        c.setup()
        got = c._run(c._tensors(dtype=dtype))[0].detach().float().reshape(-1).cpu().numpy()
        np.testing.assert_allclose(got, c.outputs["loss"], atol=tol * 4, rtol=tol)
    else:
        c.check_output(atol=tol * 4, rtol=tol, dtype=dtype)
    c = case()
    c.setup()  # one draw of the inputs, run on both devices
    ref = _grads(c, "cpu", torch.float64)
    got = _grads(c, "cuda", dtype)
    for g, r in zip(got, ref):
        torch.testing.assert_close(g, r, atol=tol * 8, rtol=tol * 4)
    assert not _lib.FALLBACKS, f"fallbacks taken: {_lib.FALLBACKS}"
