"""Fused token (+ position) embedding with a deterministic sort-based backward
(``csrc/kernels/embedding.hip``).

Parity: reference `phi/kernels/gpu/embedding_kernel.cu` + `embedding_grad_kernel.cu`,
`c_embedding_op.cu` (vocab-parallel shard lookup) and GPT's word + learned-position embedding.

The weight gradients go straight into ``main_grad`` when the training engine installed one (the
flat gradient buffer; the tied LM head adds its part there too) and the engine's ready hook is
fired — otherwise they are returned to autograd. CPU tensors run the PyTorch reference.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib


def _ref(ids, w, start, pos_table, pos_ids):
    V = w.shape[0]
    local = ids - start
    ok = (local >= 0) & (local < V)
    out = F.embedding(torch.where(ok, local, torch.zeros_like(local)), w)
    out = out * ok.unsqueeze(-1).to(out.dtype)
    if pos_table is not None:
        if pos_ids is None:
            S = ids.shape[-1]
            out = out + pos_table[:S]
        else:
            out = out + F.embedding(pos_ids, pos_table)
    return out


def _grad_target(p, dtype):
    mg = _lib.main_grad(p)
    if mg is not None:
        return mg, True
    return torch.zeros(p.shape, dtype=torch.float32, device=p.device), False


class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, w, pos_table, pos_ids, start):
        shp = ids.shape
        H = w.shape[1]
        idf = ids.reshape(-1).contiguous().long()
        T = idf.numel()
        S = shp[-1] if len(shp) > 1 else T
        out = torch.empty((T, H), dtype=w.dtype, device=w.device)
        pf = None if pos_ids is None else pos_ids.reshape(-1).contiguous().long()
        _lib.call("piamd_embedding_fwd", idf.data_ptr(), w.data_ptr(), start, w.shape[0],
                  _lib.ptr(pos_table), _lib.ptr(pf), S, out.data_ptr(), T, H, _lib.stream())
        ctx.save_for_backward(idf, pf)
        ctx.w, ctx.pt = w, pos_table
        ctx.start, ctx.shape, ctx.S = start, shp, S
        return out.view(*shp, H)

    @staticmethod
    def backward(ctx, dy):
        idf, pf = ctx.saved_tensors
        w, pt = ctx.w, ctx.pt
        H = w.shape[1]
        dy = dy.reshape(-1, H).contiguous()
        T = dy.shape[0]
        dw = dpt = None
        if ctx.needs_input_grad[1]:
            sorted_ids, order = torch.sort(idf)
            tgt, engine = _grad_target(w, w.dtype)
            _lib.call("piamd_embedding_bwd", sorted_ids.data_ptr(), order.data_ptr(), dy.data_ptr(),
                      tgt.data_ptr(), int(tgt.dtype == torch.float32), ctx.start, w.shape[0], T, H,
                      1, _lib.stream())
            if engine:
                _lib.fire(w)
            else:
                dw = tgt.to(w.dtype)
        if pt is not None and ctx.needs_input_grad[2]:
            tgt, engine = _grad_target(pt, pt.dtype)
            if pf is None:
                S = ctx.S
                _lib.call("piamd_pos_embedding_bwd", dy.data_ptr(), tgt.data_ptr(),
                          int(tgt.dtype == torch.float32), T // S, S, H, 1, _lib.stream())
            else:
                sp, order = torch.sort(pf)
                _lib.call("piamd_embedding_bwd", sp.data_ptr(), order.data_ptr(), dy.data_ptr(),
                          tgt.data_ptr(), int(tgt.dtype == torch.float32), 0, pt.shape[0], T, H,
                          1, _lib.stream())
            if engine:
                _lib.fire(pt)
            else:
                dpt = tgt.to(pt.dtype)
        return None, dw, dpt, None, None


def embedding(ids, weight, vocab_start=0, pos_table=None, pos_ids=None):
    """out = weight[ids - vocab_start] (zero rows for ids outside this shard) + pos_table[pos].
    ``pos_ids=None`` means positions 0..S-1 along the last id dimension."""
    if not weight.is_cuda or weight.dtype != torch.bfloat16 or weight.shape[1] % 8 or \
            (pos_table is not None and pos_table.dtype != weight.dtype):
        return _ref(ids, weight, vocab_start, pos_table, pos_ids)
    return _Embedding.apply(ids, weight, pos_table, pos_ids, int(vocab_start))


_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


class _Lookup(torch.autograd.Function):
    """Plain table lookup of any float dtype (``paddle.nn.functional.embedding``); padding ids
    arrive remapped to −1, which the kernels treat as out of range: a zero output row and no
    gradient (reference `embedding_kernel.cu` PaddingFlag / `embedding_grad_kernel.cu`)."""

    @staticmethod
    def forward(ctx, ids, w):
        shp = ids.shape
        H = w.shape[1]
        idf = ids.reshape(-1).contiguous()
        T = idf.numel()
        out = torch.empty((T, H), dtype=w.dtype, device=w.device)
        _lib.call("piamd_embedding_fwd_dt", _DT[w.dtype], idf.data_ptr(), w.data_ptr(), 0, w.shape[0],
                  None, None, 1, out.data_ptr(), T, H, _lib.stream())
        ctx.save_for_backward(idf)
        ctx.w = w
        return out.view(*shp, H)

    @staticmethod
    def backward(ctx, dy):
        (idf,) = ctx.saved_tensors
        w = ctx.w
        if not ctx.needs_input_grad[1]:
            return None, None
        H = w.shape[1]
        dy = dy.reshape(-1, H).contiguous().to(w.dtype)
        sorted_ids, order = torch.sort(idf)
        tgt, engine = _grad_target(w, w.dtype)
        _lib.call("piamd_embedding_bwd_dt", _DT[w.dtype], sorted_ids.data_ptr(), order.data_ptr(), dy.data_ptr(),
                  tgt.data_ptr(), 0, w.shape[0], idf.numel(), H, 1, _lib.stream())
        if engine:
            _lib.fire(w)
            return None, None
        return None, tgt.to(w.dtype)


def lookup(ids, weight, padding_idx=None):
    """out[..., :] = weight[ids] with Paddle's padding semantics (rows of ``padding_idx`` are zero
    and get no gradient); the own kernels for CUDA f32 / bf16 / fp16 tables with H % 8 == 0."""
    V = weight.shape[0]
    pad = padding_idx  # Paddle: negative = counted from the end of the table
    if pad is not None and pad < 0:
        pad = pad + V
    ids = ids.long()
    if weight.is_cuda and ids.device != weight.device:  # the kernels read the ids on the device
        ids = ids.to(weight.device)
    if weight.is_cuda and weight.dtype in _DT and weight.dim() == 2 and weight.shape[1] % 8 == 0 \
            and weight.is_contiguous() and _lib.available():
        if pad is not None:
            ids = ids.masked_fill(ids == pad, -1)
        return _Lookup.apply(ids, weight)
    if weight.is_cuda:
        _lib.fallback("embedding", "table width % 8 != 0 / non-contiguous / non-float table (ATen)")
    out = F.embedding(ids, weight, pad)
    if pad is not None:
        out = out * (ids != pad).unsqueeze(-1).to(out.dtype)
    return out
