"""MoE expert routing + grouped expert GEMMs (``csrc/kernels/gemm.hip`` moe_gemm / moe_wgrad,
``infer.hip`` wo_moe_gemm).

Parity: reference `fluid/operators/fused/fused_moe_op.cu` + `moe_expert_gemm.h` (CUTLASS grouped
GEMM over expert row ranges) and the expert FFN of `fused_multi_transformer_moe{,_weight_only}_op.cu`.

MI355X design — everything after the gate stays on the device, no host synchronisation:

* :func:`permute` sorts the (token, choice) assignments by expert with one stable argsort and
  lays every expert's rows out as a segment padded to ``align`` rows (64: the MFMA K-step, so the
  weight-gradient GEMM can reduce over whole segments). Segment offsets are a device int32 tensor;
  the worst-case row count ``T·k + E·(align-1)`` sizes the buffers, so routing never reads a
  count back and the whole MoE FFN is hipGraph-capturable (decode).
* one grouped launch per GEMM: the kernel's workgroups resolve their expert from the device
  offsets and surplus workgroups of the worst-case grid exit at once (256×256 MFMA tiles for
  prefill / training; 32-row weight-only tiles — int8 / int4 / packed bf16 — for decode).
* training: forward stores the FFN1 pre-activation from the GEMM epilogue; backward fuses the
  activation gradient into the FFN2 data-gradient GEMM (epilogue ``dact``) and reduces the weight
  gradients per expert segment in one launch each.

CPU tensors run a per-expert PyTorch reference of the same contract.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _lib
from .activation import ACTS, _ref_act

ALIGN = 64


@dataclass
class Routing:
    """Expert-sorted layout of the (token, choice) assignments."""
    slot: torch.Tensor      # [T, k] int64: row of each assignment in the sorted buffer (-1 dropped)
    src: torch.Tensor       # [rows_cap] int64: source token of each sorted row (-1 = padding)
    offs: torch.Tensor      # [E+1] int32: padded expert segment offsets (device)
    counts: torch.Tensor    # [E] int64: assignments per expert
    rows_cap: int           # static worst-case number of sorted rows
    num_tokens: int
    align: int


def permute(expert_idx: torch.Tensor, num_experts: int, align: int = ALIGN) -> Routing:
    """expert_idx [T, k] (ids in [0, E), -1 = dropped) → :class:`Routing`."""
    T, k = expert_idx.shape
    n = T * k
    E = num_experts
    dev = expert_idx.device
    flat = expert_idx.reshape(-1).long()
    valid = flat >= 0
    key = torch.where(valid, flat, torch.full_like(flat, E))
    order = torch.argsort(key, stable=True)
    counts_all = torch.bincount(key, minlength=E + 1)
    counts = counts_all[:E]
    padded = (counts + (align - 1)) // align * align
    offs = torch.zeros(E + 1, dtype=torch.long, device=dev)
    offs[1:] = torch.cumsum(padded, 0)
    uoffs = torch.zeros(E + 1, dtype=torch.long, device=dev)
    uoffs[1:] = torch.cumsum(counts, 0)
    skey = key[order]
    ke = skey.clamp(max=E - 1)
    rank = torch.arange(n, device=dev) - uoffs[ke]
    rows_cap = n + E * (align - 1)
    svalid = skey < E
    slot_sorted = torch.where(svalid, offs[ke] + rank, torch.full_like(rank, rows_cap))
    slot = torch.empty(n, dtype=torch.long, device=dev)
    slot[order] = torch.where(svalid, slot_sorted, torch.full_like(slot_sorted, -1))
    src = torch.full((rows_cap + 1,), -1, dtype=torch.long, device=dev)
    src[slot_sorted] = order // k  # invalid assignments land on the discarded extra row
    return Routing(slot.view(T, k), src[:rows_cap], offs.to(torch.int32), counts, rows_cap, T,
                   align)


def gather(x: torch.Tensor, r: Routing) -> torch.Tensor:
    """x [T, H] → sorted rows [rows_cap, H] (padding rows are zero). Differentiable."""
    xp = torch.cat([x, x.new_zeros(1, x.shape[-1])], 0)
    idx = torch.where(r.src >= 0, r.src, torch.full_like(r.src, r.num_tokens))
    return xp.index_select(0, idx)


def combine(y: torch.Tensor, weights: torch.Tensor, r: Routing) -> torch.Tensor:
    """Sorted expert outputs [rows_cap, H] + gate weights [T, k] → [T, H]. Differentiable."""
    yp = torch.cat([y, y.new_zeros(1, y.shape[-1])], 0)
    idx = torch.where(r.slot >= 0, r.slot, torch.full_like(r.slot, r.rows_cap))
    g = yp.index_select(0, idx.reshape(-1)).view(*idx.shape, y.shape[-1])
    w = torch.where(r.slot >= 0, weights, torch.zeros_like(weights)).to(torch.float32)
    return (g.float() * w[..., None]).sum(1).to(y.dtype)


def _segments(offs):
    o = offs.tolist()
    return [(o[e], o[e + 1]) for e in range(len(o) - 1)]


def _row_expert(offs, rows):
    return torch.searchsorted(offs[1:].long(), torch.arange(rows, device=offs.device), right=True) \
        .clamp_(max=offs.numel() - 2)


# ------------------------------------------------------------------------- grouped bf16 GEMM
def grouped_gemm(x, w, offs, rows_cap=None, bias=None, act="none", trans_w=False, aux=None,
                 epi=None, out=None):
    """y[rows of e] = act(x[rows of e] · W_e + b_e). x [R, K]; w [E, K, N] (or [E, N, K] with
    ``trans_w``); bias [E, N]; ``aux`` [R, N] receives the pre-activation (bias_act epilogue) or
    supplies it (``epi="dact"``: y = (x·W_e) ⊙ act'(aux)). Rows outside every segment are left
    untouched."""
    R, K = x.shape
    E = w.shape[0]
    N = w.shape[1] if trans_w else w.shape[2]
    rows_cap = R if rows_cap is None else rows_cap
    epi = epi or ("bias_act" if (bias is not None or act != "none" or aux is not None) else "none")
    if not x.is_cuda:
        y = out if out is not None else torch.zeros((R, N), dtype=x.dtype)
        for e, (a, b) in enumerate(_segments(offs)):
            if b <= a:
                continue
            we = w[e].float().t() if trans_w else w[e].float()
            v = x[a:b].float() @ we
            if epi == "bias_act":
                if bias is not None:
                    v = v + bias[e].float()
                pre = v.to(x.dtype)
                if aux is not None:
                    aux[a:b] = pre
                v = _ref_act(pre.float(), ACTS[act])
            elif epi == "dact":
                from .gemm import _act_grad_ref
                v = v * _act_grad_ref(aux[a:b], ACTS[act])
            y[a:b] = v.to(y.dtype)
        return y
    assert x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.stride(-1) == 1
    assert K % 64 == 0 and (trans_w or N % 256 == 0) and N % 4 == 0, (K, N)
    w = w.contiguous()
    y = out if out is not None else torch.empty((R, N), dtype=torch.bfloat16, device=x.device)
    e_code = {"none": 0, "bias_act": 1, "dact": 2}[epi]
    _lib.call("piamd_moe_gemm", x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(1), w.stride(0),
              int(trans_w), offs.data_ptr(), E, rows_cap, y.data_ptr(), y.stride(0),
              int(y.dtype == torch.float32), N, K, e_code, ACTS[act], _lib.ptr(bias),
              _lib.ptr(aux), aux.stride(0) if aux is not None else 0, _lib.stream())
    return y


def grouped_wgrad(x, dy, offs, out=None, accumulate=False):
    """dW_e = x_eᵀ · dy_e per expert segment (segments 64-aligned, zero padded) → [E, K, N]."""
    R, K = x.shape
    N = dy.shape[1]
    E = offs.numel() - 1
    if out is None:
        out = torch.empty((E, K, N), dtype=torch.float32 if not x.is_cuda else torch.bfloat16,
                          device=x.device)
        accumulate = False
    if not x.is_cuda or K % 256 or N % 256:
        for e, (a, b) in enumerate(_segments(offs)):
            v = x[a:b].float().t() @ dy[a:b].float()
            if accumulate:
                out[e] += v.to(out.dtype)
            else:
                out[e] = v.to(out.dtype)
        return out
    _lib.call("piamd_moe_wgrad", x.data_ptr(), x.stride(0), dy.data_ptr(), dy.stride(0),
              offs.data_ptr(), E, out.data_ptr(), out.stride(0), int(out.dtype == torch.float32),
              int(accumulate), K, N, _lib.stream())
    return out


def segment_sum(dy, offs, E):
    """Per-expert column sums of sorted rows → [E, N] f32 (bias gradients)."""
    R = dy.shape[0]
    re = _row_expert(offs, R)
    inside = torch.arange(R, device=dy.device) < offs[-1].long()
    d = torch.where(inside[:, None], dy.float(), torch.zeros((), device=dy.device))
    return torch.zeros((E, dy.shape[1]), dtype=torch.float32, device=dy.device).index_add_(0, re, d)


class _GroupedFFN(torch.autograd.Function):
    """y = act(x·W1_e + b1_e)·W2_e + b2_e over expert-sorted rows (training-capable)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, offs, rows_cap, act):
        R = x.shape[0]
        Fd = w1.shape[2]
        pre = torch.empty((R, Fd), dtype=x.dtype, device=x.device) if x.is_cuda else \
            torch.zeros((R, Fd), dtype=x.dtype)
        h = grouped_gemm(x, w1, offs, rows_cap, b1, act, aux=pre)
        y = grouped_gemm(h, w2, offs, rows_cap, b2, "none")
        ctx.save_for_backward(x, w1, w2, pre, h, offs)
        ctx.act, ctx.rows_cap = act, rows_cap
        ctx.has_b = (b1 is not None, b2 is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w1, w2, pre, h, offs = ctx.saved_tensors
        E = w1.shape[0]
        dy = dy.contiguous()
        # activation gradient fused into the FFN2 data-gradient epilogue: dpre = (dy·W2ᵀ) ⊙ act'(pre)
        dpre = grouped_gemm(dy, w2, offs, ctx.rows_cap, act=ctx.act, trans_w=True, aux=pre,
                            epi="dact")
        dx = grouped_gemm(dpre, w1, offs, ctx.rows_cap, trans_w=True, epi="none")
        dw2 = grouped_wgrad(h, dy, offs).to(w2.dtype)
        dw1 = grouped_wgrad(x, dpre, offs).to(w1.dtype)
        db1 = segment_sum(dpre, offs, E).to(w1.dtype) if ctx.has_b[0] else None
        db2 = segment_sum(dy, offs, E).to(w2.dtype) if ctx.has_b[1] else None
        return dx, dw1, db1, dw2, db2, None, None, None


def grouped_ffn(x, w1, b1, w2, b2, r: Routing, act="gelu"):
    """Expert FFN over rows laid out by :func:`permute` (align must be 64 for training)."""
    return _GroupedFFN.apply(x, w1, b1, w2, b2, r.offs, r.rows_cap, act)


# ------------------------------------------------------------------ grouped weight-only GEMM
def grouped_weight_only_linear(x, wq, scale, offs, rows_cap, bias=None, bits=8, act="none",
                               out=None):
    """Expert GEMM on weight-only packed weights (decode / small batch). x [R, K] sorted rows;
    wq [E, N_packed, K] packed per expert (``weight_quantize`` of each expert's [K, N], or
    ``pack_bf16`` with bits=16); scale [E, N] f32 (None for bits 16); bias [E, N]."""
    R, K = x.shape
    E = wq.shape[0]
    N = scale.shape[1] if scale is not None else wq.shape[1]
    if not x.is_cuda:
        from .inference import _unpack
        y = out if out is not None else torch.zeros((R, N), dtype=x.dtype)
        for e, (a, b) in enumerate(_segments(offs)):
            if b <= a:
                continue
            if bits == 16:
                we = wq[e].view(N // 32, K // 16, 2, 32, 8).permute(0, 3, 1, 2, 4).reshape(N, K).float()
            else:
                we = _unpack(wq[e], bits, N, K).float() * scale[e].float()[:, None]
            v = x[a:b].float() @ we.t()
            if bias is not None:
                v = v + bias[e].float()
            y[a:b] = _ref_act(v, ACTS[act]).to(y.dtype)
        return y
    assert x.dtype == torch.bfloat16 and x.stride(-1) == 1
    y = out if out is not None else torch.empty((R, N), dtype=torch.bfloat16, device=x.device)
    wq = wq.contiguous()
    sc = None if scale is None else scale.float().contiguous()
    _lib.call("piamd_wo_moe_gemm", bits, x.data_ptr(), x.stride(0), wq.data_ptr(),
              wq[0].numel() * wq.element_size(), _lib.ptr(sc), _lib.ptr(bias), offs.data_ptr(), E,
              rows_cap, y.data_ptr(), y.stride(0), N, K, ACTS[act], _lib.stream())
    return y
