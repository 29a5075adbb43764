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
