"""Hand-written MFMA GEMM with fused epilogues (``csrc/kernels/gemm.hip``).

``gemm(a, b)`` computes ``A·B`` for 2-D operands where ``trans_a`` means ``a`` is stored
[K, M] and ``trans_b`` means ``b`` is stored [N, K] (so weights kept [in, out] serve forward,
data-gradient and weight-gradient products without copies). Epilogues:

* ``epi="bias_act"``: ``pre = A·B + bias`` is written to ``aux`` and ``act(pre)`` to C (FFN1);
* ``epi="dact"``: ``C = (A·B) ⊙ act'(aux)`` (the FFN1 activation backward fused into the FFN2
  data-gradient GEMM);
* ``out`` f32 with ``accumulate=True``: C += A·B (weight gradient straight into main_grad).

CPU tensors run the PyTorch reference of the same contract (tests' numerics reference).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib
from .activation import ACTS, _ref_act

_EPI = {"none": 0, "bias_act": 1, "dact": 2}


def _act_grad_ref(h, act):
    h = h.float().detach().requires_grad_(True)
    with torch.enable_grad():
        y = _ref_act(h, act)
        (g,) = torch.autograd.grad(y.sum(), h)
    return g


def supported(a, b, trans_a=False, trans_b=False):
    """Shapes/layouts the hand-written GEMM (either kernel) accepts."""
    if not (a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16):
        return False
    return pipe_supported(a, b, trans_a, trans_b) or _v1_supported(a, b, trans_a, trans_b)


def _v1_supported(a, b, trans_a, trans_b):
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    N = b.shape[0] if trans_b else b.shape[1]
    return (K % 64 == 0 and N % 4 == 0 and (not trans_a or M % 256 == 0)
            and (trans_b or N % 256 == 0) and a.stride(-1) == 1 and b.stride(-1) == 1)


def pipe_supported(a, b, trans_a=False, trans_b=False):
    """Contract of the pipelined kernel (`gemm_pipe.hip`): K % 64, N % 4, 8-element aligned
    leading dims, M % 8 when A is stored [K, M], N % 8 when B is stored [K, N]; fused epilogues
    need A stored [M, K]."""
    if not (a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16):
        return False
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    N = b.shape[0] if trans_b else b.shape[1]
    return (K % 64 == 0 and N % 4 == 0 and M > 0 and (not trans_a or M % 8 == 0)
            and (trans_b or N % 8 == 0) and a.stride(-1) == 1 and b.stride(-1) == 1
            and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0
            and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0
            and a.stride(0) < (1 << 22) and b.stride(0) < (1 << 22))


NUM_CUS = 256

_AGEMM_READY = [False]


def _agemm_load():
    """Load the assembled code object (`_lib/piamd_agemm.hsaco`) into the HIP runtime once."""
    if _AGEMM_READY[0]:
        return
    import os
    from .. import _build
    path = os.environ.get("PIAMD_AGEMM_HSACO") or _build.AGEMM_HSACO  # ablation builds (tools/)
    if not os.path.exists(path):
        raise RuntimeError(f"assembly GEMM code object missing ({path}); run "
                           "`python -m paddle_infer_amd._build`")
    _lib.call("piamd_agemm_load", path.encode())
    _AGEMM_READY[0] = True


def asm_supported(a, b, trans_a=False, trans_b=False, ksplit=1):
    """Contract of the assembly GEMM (`csrc/asm/gemm_gen.py`): K % (64·ksplit) with ≥ 2 K-blocks
    per split, N % 4, 8-element aligned leading dims < 2^22, M % 8 when A is stored [K, M],
    N % 8 when B is stored [K, N], 16-byte aligned operands."""
    if not (a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16):
        return False
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    N = b.shape[0] if trans_b else b.shape[1]
    return (K % (64 * ksplit) == 0 and K // ksplit >= 128 and N % 4 == 0 and M > 0
            and (not trans_a or M % 8 == 0) and (trans_b or N % 8 == 0)
            and a.stride(-1) == 1 and b.stride(-1) == 1
            and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0
            and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0
            and a.stride(0) < (1 << 22) and b.stride(0) < (1 << 22))


def asm_gemm(a, b, trans_a=False, trans_b=False, out=None, out_f32=False, accumulate=False,
             ksplit=1, epi="none", act="none", bias=None, aux=None):
    """C (+)= op(A)·op(B) on the hand-scheduled assembly kernels. Fused epilogues (A stored
    [M, K], B stored [N, K], bf16 C): ``epi="bias_act"`` — pre = bf16(A·B + bias) written to
    ``aux`` (optional), C = act(pre); ``epi="dact"`` — C = (A·B) ⊙ act'(aux). act ∈ none / gelu_tanh
    / relu."""
    _agemm_load()
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    N = b.shape[0] if trans_b else b.shape[1]
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32 if out_f32 else torch.bfloat16, device=a.device)
    assert out.shape == (M, N) and out.stride(-1) == 1 and out.data_ptr() % 16 == 0
    ws = None
    if ksplit > 1:
        ws = torch.empty((ksplit, M, N), dtype=torch.float32, device=a.device)
    if aux is not None:
        assert aux.shape == (M, N) and aux.dtype == torch.bfloat16 and aux.stride(-1) == 1
    _lib.call("piamd_agemm", a.data_ptr(), a.stride(0), int(trans_a), b.data_ptr(), b.stride(0),
              int(trans_b), out.data_ptr(), out.stride(0), int(out.dtype == torch.float32),
              int(accumulate), M, N, K, _EPI[epi], ACTS[act], _lib.ptr(bias), _lib.ptr(aux),
              aux.stride(0) if aux is not None else 0, ksplit, _lib.ptr(ws), _lib.stream())
    return out


def pick_ksplit(M, N, K):
    """Split-K degree for the pipelined kernel: fill the 256 CUs (one 256x256 tile per CU) when
    the tile grid is small and K is long (weight gradients: 2048 x 2048 tiles over 65k tokens)."""
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    nk = K // 64
    if tiles >= 2 * NUM_CUS or nk < 32:
        return 1
    best, best_t = 1, None
    for ks in (1, 2, 4, 8):
        if nk // ks < 16 or nk % ks:
            break
        waves = -(-tiles * ks // NUM_CUS)
        t = waves / ks
        if best_t is None or t < best_t - 1e-9:
            best, best_t = ks, t
    return best


def gemm(a, b, trans_a=False, trans_b=False, out=None, out_f32=False, accumulate=False,
         epi="none", act="none", bias=None, aux=None, ksplit=None, impl="auto"):
    """C = op(A)·op(B) on the hand-written MFMA kernels (CPU: fp32 PyTorch reference).
    ``impl``: "auto" (pipelined kernel when its contract holds), "pipe", or "v1" (the 2-stage
    kernel of gemm.hip). ``ksplit``: split-K degree (pipe, epi "none" only; None = heuristic)."""
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    N = b.shape[0] if trans_b else b.shape[1]
    e, ac = _EPI[epi], ACTS[act]
    if epi == "bias_act" and aux is None and a.is_cuda:
        pass  # aux optional (inference)
    if not a.is_cuda:
        A = a.t() if trans_a else a
        B = b.t() if trans_b else b
        y = A.float() @ B.float()
        if e == 1:
            y = y + (bias.float() if bias is not None else 0.0)
            pre = y.to(torch.bfloat16)
            if aux is not None:
                aux.copy_(pre)
            y = _ref_act(pre.float(), ac)
        elif e == 2:
            y = y * _act_grad_ref(aux, ac)
        if out is None:
            return y.to(torch.float32 if out_f32 else a.dtype)
        if accumulate:
            out.add_(y.to(out.dtype))
        else:
            out.copy_(y)
        return out
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32 if out_f32 else torch.bfloat16, device=a.device)
    assert out.stride(-1) == 1 and out.shape == (M, N)
    if aux is not None:
        assert aux.shape == (M, N) and aux.dtype == torch.bfloat16 and aux.stride(-1) == 1
    fused_ok = e == 0 or (not trans_a and out.dtype == torch.bfloat16 and not accumulate)
    use_pipe = impl == "pipe" or (impl == "auto" and fused_ok and pipe_supported(a, b, trans_a, trans_b))
    if use_pipe:
        assert out.stride(0) % 4 == 0 and out.data_ptr() % 16 == 0
        ks = ksplit if ksplit is not None else (pick_ksplit(M, N, K) if e == 0 else 1)
        ws = None
        if ks > 1:
            ws = torch.empty((ks, M, N), dtype=torch.float32, device=a.device)
        _lib.call("piamd_gemm_pipe", a.data_ptr(), a.stride(0), int(trans_a), b.data_ptr(),
                  b.stride(0), int(trans_b), out.data_ptr(), out.stride(0),
                  int(out.dtype == torch.float32), int(accumulate), M, N, K, e, ac, _lib.ptr(bias),
                  _lib.ptr(aux), aux.stride(0) if aux is not None else 0, ks, _lib.ptr(ws),
                  _lib.stream())
        return out
    _lib.call("piamd_gemm", a.data_ptr(), a.stride(0), int(trans_a), b.data_ptr(), b.stride(0),
              int(trans_b), out.data_ptr(), out.stride(0), int(out.dtype == torch.float32),
              int(accumulate), M, N, K, e, ac, _lib.ptr(bias), _lib.ptr(aux),
              aux.stride(0) if aux is not None else 0, _lib.stream())
    return out


F  # noqa
