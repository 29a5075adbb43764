"""``beam_search_softmax`` — one beam-search decode step (``csrc/kernels/search.hip``).

Parity: reference `python/paddle/tensor/search.py:1111` / `phi/kernels/fusion/gpu/beam_search_softmax.cu`.
Inputs (``R = batch * beam``): logits [R, V] (f32 / bf16), cum_scores [R] f32, sequence_lengths
[R] int32, stop_flags [R] bool, end_ids [1] int32, step_ids [R] int32, last_cache_ids
[R, max_dec_len] int32, last_beam_offsets [batch, beam, max_seq_len + max_dec_len] int32.
Returns (ids_this_time, out_cum_scores, cache_ids, beam_offsets, parent_idx, stop_flags_out,
seq_lens_out, step_ids_out). GPU tensors run the two HIP launches (beam ≤ 16); CPU tensors run the
PyTorch reference below, which spells out the exact semantics.
"""
from __future__ import annotations

import math

import torch

from . import _lib

_KEY_BIG = 2 ** 31 - 1


def _topk_sorted(vals, ids, k):
    """Sort by (value desc, id asc) — the reference TopK insertion order — and keep k."""
    order = sorted(range(len(vals)), key=lambda i: (-vals[i], ids[i] if ids[i] >= 0 else _KEY_BIG, i))
    return [(vals[i], ids[i], i) for i in order[:k]]


def _reference(logits, cum_scores, seq_lens, stop_flags, end_ids, step_ids, last_cache_ids,
               last_beam_offsets, beam, max_seq_len, max_dec_len, fuse_softmax, early_stop,
               length_penalty):
    R, V = logits.shape
    bs = R // beam
    lg = logits.float()
    eid = int(end_ids.reshape(-1)[0])
    stop = stop_flags.reshape(-1).bool().tolist()
    step = step_ids.reshape(-1).tolist()
    sl = seq_lens.reshape(-1).tolist()
    cum = cum_scores.reshape(-1).float().tolist()
    max_len = max_seq_len + max_dec_len
    ids_out = torch.zeros(R, dtype=torch.int32)
    cum_out = torch.zeros(R, dtype=torch.float32)
    parent = torch.zeros(R, dtype=torch.int32)
    stop_out = stop_flags.reshape(-1).clone().bool()
    sl_out = seq_lens.reshape(-1).clone().int()
    st_out = step_ids.reshape(-1).clone().int()
    cache = last_cache_ids.reshape(R, max_dec_len).clone().int()
    offs = last_beam_offsets.reshape(R, max_len).clone().int()
    lco = last_cache_ids.reshape(R, max_dec_len)
    lbo = last_beam_offsets.reshape(R, max_len)
    for b in range(bs):
        cands_v, cands_i = [], []
        for j in range(beam):
            r = b * beam + j
            if stop[r]:
                x = torch.full((V,), -torch.finfo(torch.float32).max)
                x[eid] = torch.finfo(torch.float32).max if fuse_softmax else 0.0
            else:
                x = lg[r]
            if fuse_softmax:
                m = x.max()
                lse = (m + torch.log(torch.exp((x - m).double()).sum()).float()).item()
            else:
                lse = 0.0
            cl, pen = cum[r], 1.0
            if length_penalty != 0.0 and not stop[r]:
                prev = math.pow(step[r], length_penalty)
                pen = math.pow(step[r] + 1, length_penalty)
                cl = cl * prev / pen
            # (value desc, id asc): a stable sort of -x keeps ascending ids among ties
            order = torch.sort(-x, stable=True).indices[:beam].tolist()
            for i in order:
                v = float(x[i])
                cands_v.append((v - lse) / pen + cl)
                cands_i.append(i)
        first = step[0] == 0
        nc = beam if first else beam * beam
        live = [c for c in range(nc) if not (early_stop and not first and stop[b * beam + c // beam])]
        best = _topk_sorted([cands_v[c] for c in live], [cands_i[c] for c in live], beam)
        best = [(v, i, live[k]) for v, i, k in best]
        slots = [j for j in range(beam) if not (early_stop and stop[b * beam + j])]
        sel = {}
        for (v, i, c), slot in zip(best, slots):
            o = b * beam + slot
            par = c // beam
            ids_out[o], cum_out[o], parent[o] = i, v, par
            sel[slot] = par
            src = b * beam + par
            stop_out[o], sl_out[o], st_out[o] = stop[src], sl[src], step[src]
        if early_stop:
            for j in range(beam):
                o = b * beam + j
                if stop[o]:
                    ids_out[o], cum_out[o], parent[o] = eid, cum[o], j
                    sel[j] = j
        for j in range(beam):
            o = b * beam + j
            src = b * beam + sel.get(j, 0)
            if sl[src] != 0:
                for t in range(min(sl[src] + 1, max_len)):
                    offs[o, t] = sel.get(j, 0) if t == sl[src] else lbo[src, t]
                for t in range(min(step[src] + 1, max_dec_len)):
                    cache[o, t] = ids_out[o] if t == step[src] else lco[src, t]
    return (ids_out, cum_out, cache.reshape(last_cache_ids.shape),
            offs.reshape(last_beam_offsets.shape), parent, stop_out, sl_out, st_out)


def argmax_rows(logits, out=None):
    """Greedy token choice: int64 argmax over the last dim of [R, V] logits (ties → smaller id) in
    one HIP launch (`search.hip` piamd_argmax_rows; hipGraph-capturable). CPU: torch.argmax."""
    if not logits.is_cuda:
        return logits.argmax(-1)
    lg = logits if logits.stride(-1) == 1 else logits.contiguous()
    lg2 = lg.reshape(-1, lg.shape[-1]) if lg.dim() != 2 else lg
    code = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}.get(lg2.dtype)
    if code is None:
        return logits.argmax(-1)
    R, V = lg2.shape
    if out is None:
        out = torch.empty(R, dtype=torch.int64, device=lg2.device)
    _lib.call("piamd_argmax_rows", lg2.data_ptr(), lg2.stride(0), R, V, code, out.data_ptr(), _lib.stream())
    return out.view(logits.shape[:-1])


def beam_search_softmax(logits, cum_scores, sequence_lengths, stop_flags, end_ids, step_ids,
                        last_cache_ids, last_beam_offsets, beam_size, max_seq_len, max_dec_len,
                        fuse_softmax=True, early_stop=False, length_penalty=0.0,
                        one_stage_topk=False):
    assert not (one_stage_topk and fuse_softmax), "one stage topk not support fuse softmax now."
    R, V = logits.shape
    bs = R // beam_size
    if max_seq_len == 0:  # dynamic: from the beam-offset history width
        max_seq_len = last_beam_offsets.shape[-1] - max_dec_len
    if not logits.is_cuda or beam_size > 16:
        outs = _reference(logits.cpu(), cum_scores.cpu(), sequence_lengths.cpu(), stop_flags.cpu(),
                          end_ids.cpu(), step_ids.cpu(), last_cache_ids.cpu(),
                          last_beam_offsets.cpu(), beam_size, max_seq_len, max_dec_len,
                          fuse_softmax, early_stop, length_penalty)
        return tuple(o.to(logits.device) for o in outs)
    dev = logits.device
    lg = logits.contiguous()
    P = max(1, min(64, -(-1024 // R), -(-V // 1024)))
    part = torch.empty(R * P * (2 * beam_size + 2), dtype=torch.float32, device=dev)
    i32 = lambda t: t.reshape(-1).to(device=dev, dtype=torch.int32).contiguous()  # noqa: E731
    cum = cum_scores.reshape(-1).float().contiguous()
    sl, st, eid = i32(sequence_lengths), i32(step_ids), i32(end_ids)
    stop = stop_flags.reshape(-1).to(device=dev, dtype=torch.bool).contiguous()
    lco = last_cache_ids.to(torch.int32).contiguous()
    lbo = last_beam_offsets.to(torch.int32).contiguous()
    ids = torch.empty(R, dtype=torch.int32, device=dev)
    cum_out = torch.empty(R, dtype=torch.float32, device=dev)
    parent = torch.empty(R, dtype=torch.int32, device=dev)
    cache, offs = lco.clone(), lbo.clone()
    stop_out, sl_out, st_out = stop.clone(), sl.clone(), st.clone()
    _lib.call("piamd_beam_search_softmax", lg.data_ptr(), int(lg.dtype == torch.bfloat16),
              cum.data_ptr(), sl.data_ptr(), stop.data_ptr(), eid.data_ptr(), st.data_ptr(),
              lco.data_ptr(), lbo.data_ptr(), bs, beam_size, V, int(max_seq_len), int(max_dec_len),
              int(fuse_softmax), int(early_stop), float(length_penalty), P, part.data_ptr(),
              ids.data_ptr(), cum_out.data_ptr(), cache.data_ptr(), offs.data_ptr(),
              parent.data_ptr(), stop_out.data_ptr(), sl_out.data_ptr(), st_out.data_ptr(),
              _lib.stream())
    return ids, cum_out, cache, offs, parent, stop_out, sl_out, st_out
