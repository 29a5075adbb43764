"""Sparse 3-D convolution / submanifold convolution / max pooling / mask attention on the active
sites only — no dense grid is ever allocated.

Parity: reference `paddle/phi/kernels/sparse/gpu/conv_kernel.cu:290` (rulebook + gather → GEMM →
scatter), `gather_gemm_scatter.h`, `sparse/gpu/pool_kernel.cu`, `sparse/gpu/fused_attention_kernel.cu`.

MI355X design:

* **Rulebook** (all device tensor ops, no per-site host loop): active sites are keyed
  ((b·D + z)·H + y)·W + x in int64. For every kernel offset k and input site the candidate output
  site is computed arithmetically; a regular conv's output set is the sorted unique candidates,
  a submanifold conv's is the input set itself. Candidate → output row is one ``searchsorted`` on
  the sorted keys (match = equal key), so the rulebook is (in row, out row, offset k) triples.
* **Gather → grouped MFMA GEMM → scatter-add**: the triples are routed by offset exactly like MoE
  tokens to experts (`ops/moe.py permute`: one stable argsort, 64-aligned segments, worst-case
  sizing — no count read back), the input rows gathered once, and ONE grouped GEMM launch
  (`gemm.hip` moe_gemm, per-offset weight W[k] = [Cin, Cout]) computes every offset's products;
  the outputs scatter-add (``index_add_``) into the active output rows. The backward runs the same
  rulebook: dX = grouped GEMM with W[k]ᵀ then scatter into the input rows, dW[k] = per-segment
  Xᵀ·dY (`moe_wgrad`). bf16 on the GPU kernels (channels padded to the kernel's 64-multiple);
  other dtypes / CPU take the per-offset reference of the same contract.
* Max pooling reduces the gathered rows per output with ``scatter_reduce(amax)``; mask attention
  evaluates scores only at the CSR mask's entries (SDDMM), a per-row segment softmax, then the
  sparse × dense product (SpMM).
"""
from __future__ import annotations

import torch

from ...ops import moe as _moe


def _triple(v):
    return (v,) * 3 if isinstance(v, int) else tuple(int(x) for x in v)


def _keys(idx, shape):
    """Site coordinates [4, n] (b, z, y, x) → int64 keys (batch-major)."""
    B, D, H, W = shape
    return ((idx[0] * D + idx[1]) * H + idx[2]) * W + idx[3]


def _unkey(key, shape):
    B, D, H, W = shape
    x = key % W
    r = key // W
    y = r % H
    r = r // H
    z = r % D
    return torch.stack([r // D, z, y, x])


class Rulebook:
    """(in row, out row, kernel offset) triples of a sparse conv / pool, routed by offset."""

    def __init__(self, idx, in_shape, ksize, stride, padding, dilation, subm):
        B, D, H, W = in_shape
        kd, kh, kw = ksize
        sd, sh, sw = stride
        pd, ph, pw = padding
        dd, dh, dw = dilation
        dev = idx.device
        if subm:
            assert stride == (1, 1, 1), "submanifold convolution needs stride 1"
            out_shape = (B, D, H, W)
        else:
            out_shape = (B, (D + 2 * pd - dd * (kd - 1) - 1) // sd + 1,
                         (H + 2 * ph - dh * (kh - 1) - 1) // sh + 1, (W + 2 * pw - dw * (kw - 1) - 1) // sw + 1)
        K = kd * kh * kw
        n = idx.shape[1]
        ko = torch.arange(K, device=dev)
        offs = torch.stack([ko // (kh * kw), (ko // kw) % kh, ko % kw])          # [3, K]
        if subm:  # centred kernel: out site o receives input o + (k − c)·dil
            cen = torch.tensor([(kd - 1) // 2, (kh - 1) // 2, (kw - 1) // 2], device=dev)
            delta = (offs - cen[:, None]) * torch.tensor([dd, dh, dw], device=dev)[:, None]
            oc = idx[1:, :, None] - delta[:, None, :]                              # [3, n, K]
            ok = ((oc >= 0) & (oc < torch.tensor([D, H, W], device=dev)[:, None, None])).all(0)
        else:  # input p = o·stride − pad + k·dil  →  o = (p + pad − k·dil) / stride
            num = (idx[1:, :, None] + torch.tensor([pd, ph, pw], device=dev)[:, None, None]
                   - offs[:, None, :] * torch.tensor([dd, dh, dw], device=dev)[:, None, None])
            st = torch.tensor([sd, sh, sw], device=dev)[:, None, None]
            oc = torch.div(num, st, rounding_mode="floor")
            ok = ((num % st) == 0).all(0) & (oc >= 0).all(0) & \
                (oc < torch.tensor(out_shape[1:], device=dev)[:, None, None]).all(0)
        b = idx[0][:, None].expand(n, K)
        cand = ((b * out_shape[1] + oc[0]) * out_shape[2] + oc[1]) * out_shape[3] + oc[2]  # [n, K]
        cand = torch.where(ok, cand, torch.full_like(cand, -1))
        if subm:
            keys = _keys(idx, in_shape)
            skeys, order = torch.sort(keys)
            out_keys = keys
            pos = torch.searchsorted(skeys, cand.clamp_min(0)).clamp_(max=max(n - 1, 0))
            hit = ok & (skeys[pos] == cand) if n else ok
            out_row = order[pos]
            n_out = n
            out_idx = idx
        else:
            valid = cand[ok]
            out_keys = torch.unique(valid)                                          # sorted
            n_out = int(out_keys.numel())
            pos = torch.searchsorted(out_keys, cand.clamp_min(0)).clamp_(max=max(n_out - 1, 0))
            hit = ok
            out_row = pos
            out_idx = _unkey(out_keys, out_shape)
        kk = torch.where(hit, ko[None, :].expand(n, K), torch.full_like(cand, -1))
        # pairs (in row i, offset k) → output row; routed by offset (MoE-style 64-row segments)
        self.route = _moe.permute(kk, K)
        self.in_row = self.route.src                                 # [rows_cap] (-1 = padding)
        dst = torch.full((self.route.rows_cap + 1,), -1, dtype=torch.long, device=dev)
        slot = self.route.slot.reshape(-1)
        sel = slot >= 0
        dst[slot[sel]] = out_row.reshape(-1)[sel]
        self.out_row = dst[:self.route.rows_cap]                     # [rows_cap] (-1 = padding)
        self.K, self.n_in, self.n_out = K, n, n_out
        self.out_idx, self.out_shape = out_idx, out_shape


def _pad_to(t, n, dim):
    if t.shape[dim] == n:
        return t
    pad = [0, 0] * (t.dim() - 1 - dim % t.dim()) + [0, n - t.shape[dim]]
    return torch.nn.functional.pad(t, pad)


def _gpu_ok(x, w):
    return x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16


def _gpu_f32(x, w):
    return x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32


def _ceil(n, m):
    return -(-n // m) * m


def _w_hhl(w, Kp, Np):
    """f32 [E, K, N] → bf16 [E, 3·Kp, Np] = [w_hi; w_hi; w_lo] along K (the right operand of the
    split-bf16 product, `ops/gemm.py` split3 convention)."""
    hi = w.to(torch.bfloat16)
    lo = (w - hi.float()).to(torch.bfloat16)
    parts = [_pad_to(_pad_to(t, Kp, 1), Np, 2) for t in (hi, hi, lo)]
    return torch.cat(parts, 1).contiguous()


def _split_rows(x, Cp):
    """f32 [R, C] → (hi, lo) bf16 [R, Cp] (zero-padded columns)."""
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    return _pad_to(hi, Cp, 1).contiguous(), _pad_to(lo, Cp, 1).contiguous()


def _wgrad(xs, gs, route, w):
    """dW[k] = Σ_pairs x[in]ᵀ · dY[out] on the grouped MFMA wgrad kernel (channels zero-padded
    to its 256 tiles; fp32 operands as split-bf16 hi·hi + hi·lo + lo·hi into an f32 result)."""
    E, Cin, Cout = w.shape
    Kp, Np = _ceil(Cin, 256), _ceil(Cout, 256)
    out = torch.zeros((E, Kp, Np), dtype=torch.float32, device=xs.device)
    if xs.dtype == torch.bfloat16:
        _moe.grouped_wgrad(_pad_to(xs, Kp, 1).contiguous(), _pad_to(gs, Np, 1).contiguous(), route.offs,
                           out=out, accumulate=True)
    else:
        xh, xl = _split_rows(xs.float(), Kp)
        gh, gl = _split_rows(gs.float(), Np)
        for a, b in ((xh, gh), (xh, gl), (xl, gh)):
            _moe.grouped_wgrad(a, b, route.offs, out=out, accumulate=True)
    return out[:, :Cin, :Cout].to(w.dtype)


class _GatherGemmScatter(torch.autograd.Function):
    """out[out_row] += x[in_row] · W[k] for every rulebook pair (see module docstring)."""

    @staticmethod
    def forward(ctx, x, w, rb):
        ctx.rb = rb
        ctx.save_for_backward(x, w)
        return _ggs(x, w, rb.in_row, rb.out_row, rb.route, rb.n_out)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        rb = ctx.rb
        g = g.contiguous()
        dx = dw = None
        if ctx.needs_input_grad[0]:  # dX[in_row] += dY[out_row] · W[k]ᵀ
            dx = _ggs(g, w.transpose(1, 2), rb.out_row, rb.in_row, rb.route, rb.n_in)
        if ctx.needs_input_grad[1]:  # dW[k] = Σ_pairs x[in_row]ᵀ · dY[out_row]
            xs = _gather_rows(x, rb.in_row)
            gs = _gather_rows(g, rb.out_row)
            if _gpu_ok(xs, w) or _gpu_f32(xs, w):
                dw = _wgrad(xs, gs, rb.route, w)
            else:
                dw = torch.zeros_like(w, dtype=torch.float32)
                for e, (a, b) in enumerate(_moe._segments(rb.route.offs)):
                    if b > a:
                        dw[e] = xs[a:b].float().t() @ gs[a:b].float()
                dw = dw.to(w.dtype)
        return dx, dw, None


def _gather_rows(x, rows):
    xp = torch.cat([x, x.new_zeros(1, x.shape[-1])], 0)
    return xp.index_select(0, torch.where(rows >= 0, rows, torch.full_like(rows, x.shape[0])))


def _ggs(x, w, src_row, dst_row, route, n_dst):
    """Σ over pairs: out[dst_row] += x[src_row] · w[k] with the pairs in offset segments."""
    Cin, Cout = w.shape[1], w.shape[2]
    xs = _gather_rows(x, src_row)                                           # [rows_cap, Cin]
    if _gpu_ok(xs, w):
        Kp = max(64, -(-Cin // 64) * 64)
        Np = max(256, -(-Cout // 256) * 256)
        wp = _pad_to(_pad_to(w, Kp, 1), Np, 2).contiguous()
        ys = _moe.grouped_gemm(_pad_to(xs, Kp, 1).contiguous(), wp, route.offs, route.rows_cap)[:, :Cout]
    elif _gpu_f32(xs, w):
        # fp32: ONE grouped bf16 MFMA GEMM over the 3×-long reduction [x_hi | x_lo | x_hi] ·
        # [w_hi; w_hi; w_lo] with an f32 result (≈2^-16 relative per product, `ops/gemm.py`)
        from ...ops.gemm import split3
        Kp = max(64, _ceil(Cin, 64))
        Np = max(256, _ceil(Cout, 256))
        x3 = split3(xs.contiguous(), "hlh", 0, Cp=Kp)
        ys = torch.zeros((xs.shape[0], Np), dtype=torch.float32, device=x.device)
        _moe.grouped_gemm(x3, _w_hhl(w, Kp, Np), route.offs, route.rows_cap, out=ys)
        ys = ys[:, :Cout]
    else:
        ys = torch.zeros((xs.shape[0], Cout), dtype=torch.float32, device=x.device)
        for e, (a, b) in enumerate(_moe._segments(route.offs)):
            if b > a:
                ys[a:b] = xs[a:b].float() @ w[e].float()
    keep = dst_row >= 0
    out = torch.zeros((n_dst, Cout), dtype=torch.float32, device=x.device)
    out.index_add_(0, dst_row[keep], ys[keep].float())
    return out.to(x.dtype)


def _coo_parts(x):
    x = x.coalesce()
    idx, val = x.indices(), x.values()
    assert x.sparse_dim() == 4 and val.dim() == 2, "sparse conv takes [N, D, H, W, C] COO (4 sparse dims)"
    return idx, val, tuple(x.shape[:4]), x.shape[4]


def conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NDHWC", subm=False,
           rulebook=None):
    """x: sparse COO [N, D, H, W, C]; weight [kd, kh, kw, Cin, Cout] → sparse COO output."""
    assert groups == 1, "grouped sparse convolution is not supported"
    assert data_format == "NDHWC"
    idx, val, shape, C = _coo_parts(x)
    kd, kh, kw, Cin, Cout = weight.shape
    assert Cin == C
    rb = rulebook or Rulebook(idx, shape, (kd, kh, kw), _triple(stride), _triple(padding), _triple(dilation), subm)
    w = weight.reshape(kd * kh * kw, Cin, Cout)
    out = _GatherGemmScatter.apply(val, w.to(val.dtype), rb)
    if bias is not None:
        out = out + bias.to(out.dtype)
    return torch.sparse_coo_tensor(rb.out_idx, out, (*rb.out_shape, Cout)).coalesce()


def max_pool3d(x, kernel_size, stride=None, padding=0, ceil_mode=False, data_format="NDHWC"):
    """Per output site the max over its active input neighbours (reference sparse pool: inactive
    sites do not take part)."""
    assert not ceil_mode, "ceil_mode is not supported for sparse max pooling"
    idx, val, shape, C = _coo_parts(x)
    k = _triple(kernel_size)
    rb = Rulebook(idx, shape, k, _triple(stride if stride is not None else kernel_size), _triple(padding),
                  (1, 1, 1), False)
    keep = rb.out_row >= 0
    src = _gather_rows(val, rb.in_row)[keep]
    dst = rb.out_row[keep]
    out = torch.full((rb.n_out, C), float("-inf"), dtype=val.dtype, device=val.device)
    out = out.scatter_reduce(0, dst[:, None].expand(-1, C), src, "amax", include_self=False)
    return torch.sparse_coo_tensor(rb.out_idx, out, (*rb.out_shape, C)).coalesce()


def mask_attention(query, key, value, sparse_mask, key_padding_mask=None, attn_mask=None):
    """softmax(QKᵀ/√d + masks) V evaluated only at the CSR mask's entries: SDDMM → per-row segment
    softmax → SpMM. query/key/value [B, H, S, d]; sparse_mask CSR [B·H, S, S]."""
    B, Hh, S, d = query.shape
    m = sparse_mask if sparse_mask.layout == torch.sparse_coo else sparse_mask.to_sparse_coo()
    m = m.coalesce()
    bi, ri, ci = m.indices()
    q = query.reshape(B * Hh, S, d)
    k = key.reshape(B * Hh, S, d)
    v = value.reshape(B * Hh, S, d)
    s = (q[bi, ri].float() * k[bi, ci].float()).sum(-1) * d ** -0.5          # SDDMM
    if attn_mask is not None:
        s = s + attn_mask.float()[ri, ci]
    if key_padding_mask is not None:
        s = s + key_padding_mask.float()[bi // Hh, ci]
    row = bi * S + ri
    mx = torch.full((B * Hh * S,), float("-inf"), device=s.device).scatter_reduce(0, row, s, "amax")
    e = torch.exp(s - mx[row])
    den = torch.zeros(B * Hh * S, device=s.device).index_add_(0, row, e)
    p = e / den[row]
    out = torch.zeros((B * Hh * S, d), dtype=torch.float32, device=s.device)
    out.index_add_(0, row, p[:, None] * v[bi, ci].float())                  # SpMM
    return out.reshape(B, Hh, S, d).to(query.dtype)
