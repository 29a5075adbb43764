"""Single-launch batch-1 decode step: the whole layer stack in one persistent HIP kernel.

``csrc/kernels/decode_mega.hip`` runs LN → QKV GEMV → cache write + attention → out GEMV +
residual → LN → FFN1 + GELU → FFN2 + residual for every layer in ONE launch: 256 workgroups (one
per CU) hand activations to each other through a grid barrier, and each workgroup streams its
slice of the next projection's weights into LDS while the barrier settles, so the weight stream
no longer pays a launch ramp per GEMV (5 per layer on the per-op path).

Parity: one ``FusedMultiTransformer`` decode step with ``time_step``
(`paddle/fluid/operators/fused/fused_multi_transformer_op.cu`); the per-op path
(``incubate.nn.functional.multi_transformer_forward(decode=True)``) stays the reference and the
fallback for shapes the kernel does not take (widths / batch sizes not instantiated in
``decode_mega.hip`` — GPT-3 1.3B / 350M and a GQA 4:1 variant, each with or without whole-head
rotary, at 1 row; 2 and 4 rows for 1.3B, 350M and GQA 4:1 + rotary — other weight-only
layouts, TP).

Batched steps (2 / 4 rows: small serving batches, beams) apply every workgroup's LDS weight
slice to all rows, so the weight stream — the whole cost at these sizes — is paid once per step
instead of once per row; attention runs one workgroup per (row, head, split) at each row's own
cache position.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch

from ..ops import _lib

# the shape the greedy tail
# (decode_head_kernel) are built for; every shape of the plain kernel is listed at ``mega_fn`` in
# decode_mega.hip and queried through piamd_decode_mega_shape_supported
E, D, HQ, HK, F = 2048, 128, 16, 16, 8192
# default for PIAMD_DECODE_MEGA (1 = batch-1 decode steps run the single-launch kernel, launched
# cooperatively; 0 = the per-op path)
DEFAULT = "1"


def enabled() -> bool:
    return os.environ.get("PIAMD_DECODE_MEGA", DEFAULT) != "0"


def shape_of(gen):
    """(E, D, Hq, Hk, F, rot) of generator ``gen``'s decoder stack."""
    ffn = gen.layers[0]["ffn1"]
    if ffn.bits:  # packed weight-only codes: the output width is the per-channel scale count
        F_ = ffn.scale.numel()
    else:
        F_ = ffn.w.shape[0] if ffn.trans else ffn.w.shape[-1]
    return gen.cfg.hidden_size, gen.D, gen.H, gen.Hk, int(F_), int(getattr(gen, "rotary_dim", 0))


def _w8(gen):
    """Weight format code of the stack: 1 when every projection is int8 weight-only, 2 when every
    one is int4, 0 when every one is bf16, None otherwise."""
    bits = {spec[k].bits for spec in gen.layers for k in ("qkv", "out", "ffn1", "ffn2")}
    if bits == {8}:
        return 1
    if bits == {4}:
        return 2
    if bits == {0} and all(spec[k].w.dtype == torch.bfloat16 for spec in gen.layers
                           for k in ("qkv", "out", "ffn1", "ffn2")):
        return 0
    return None


BATCHES = (1, 2, 4)  # rows per step with an instantiated kernel (MegaCfg::NB)


def max_splits(B: int, hq: int) -> int:
    """Attention splits available at ``B`` rows: one workgroup per (row, head, split) ≤ 256."""
    return 256 // (B * hq)


def eligible(gen, B: int) -> bool:
    """True when generator ``gen``'s decode step at batch ``B`` can run as one launch."""
    if not enabled():
        return False
    if (B not in BATCHES or B > gen.max_batch or gen.device.type != "cuda" or gen.dtype != torch.bfloat16
            or gen.group is not None):
        return False
    E_, D_, hq, hk, F_, rot = shape_of(gen)
    # each split holds ≤ 256 keys (one score per thread)
    if (rot not in (0, D_) or math.ceil(gen.max_seq_len / 256) > max_splits(B, hq)
            or gen.act not in ("gelu", "gelu_tanh")):
        return False
    w8 = _w8(gen)
    if w8 is None:
        return False
    for spec in gen.layers:
        for key in ("ln_scale", "ln_bias", "ffn_ln_scale", "ffn_ln_bias", "qkv_bias", "out_bias",
                    "ffn1_bias", "ffn2_bias"):
            t = spec.get(key)
            if t is None or t.dtype != torch.bfloat16:
                return False
    return (_lib.available() and _lib.has("piamd_decode_mega_batch_supported")
            and _lib.lib().piamd_decode_mega_batch_supported(E_, D_, hq, hk, F_, rot, w8, B) == 1)


def _out_in(lin):
    """[out, in] contiguous copy of a projection (each workgroup's slice is then one contiguous
    run of rows): bf16, or (weight-only) the int8 codes / int4 codes packed two per byte (k
    ascending from the low nibble) with their f32 per-output scales, recovered from the packed
    GEMV layout (exact: dequantised value / scale is the code)."""
    if lin.bits in (4, 8):
        from ..ops.inference import weight_dequantize
        s = lin.scale.float().contiguous()
        algo = "weight_only_int8" if lin.bits == 8 else "weight_only_int4"
        deq = weight_dequantize(lin.w, s, algo, "float32").t()  # [K, N] → [out, in]
        lo, hi = (-127, 127) if lin.bits == 8 else (-8, 7)
        q = torch.round(deq.float() / s[:, None]).clamp(lo, hi).to(torch.int8)
        if lin.bits == 4:
            u = (q.to(torch.int16) & 0xF).to(torch.uint8)
            q = u[:, 0::2] | (u[:, 1::2] << 4)
        return q.contiguous(), s
    w = lin.w.detach()
    return (w if lin.trans else w.t()).contiguous(), None


class MegaDecoder:
    """Owns the [out, in] weight copies, the per-layer pointer table and the scratch buffers of
    the ``nb``-row step."""

    def __init__(self, gen, nb: int = 1, shared: "MegaDecoder | None" = None):
        """``shared``: a decoder of the same generator at another row count — its [out, in] weight
        copies and pointer table are reused (they do not depend on the rows; one copy per model)."""
        dev = gen.device
        self.gen = gen
        self.w8 = _w8(gen) or 0
        if shared is not None and shared.gen is gen:
            self._keep, self.table, self.nl = shared._keep, shared.table, shared.nl
        else:
            self._keep = []
            rows = []
            for spec, (kc, vc) in zip(gen.layers, gen.caches):
                ws = [_out_in(spec[k]) for k in ("qkv", "out", "ffn1", "ffn2")]
                ts = [spec["ln_scale"], spec["ln_bias"], ws[0][0], spec["qkv_bias"], ws[1][0], spec["out_bias"],
                      spec["ffn_ln_scale"], spec["ffn_ln_bias"], ws[2][0], spec["ffn1_bias"], ws[3][0],
                      spec["ffn2_bias"], kc, vc] + [w[1] for w in ws]
                ts = [t.contiguous() if t is not None else None for t in ts]
                self._keep += [t for t in ts if t is not None]
                rows.append([t.data_ptr() if t is not None else 0 for t in ts])
            self.table = torch.tensor(rows, dtype=torch.int64, device=dev)
            self.nl = len(rows)
        self.maxS = gen.max_seq_len
        self.E, self.D, self.HQ, self.HK, self.F, self.rot = shape_of(gen)
        E_, D_, HQ_, HK_, F_ = self.E, self.D, self.HQ, self.HK, self.F
        # attention splits (≤ 256 keys each, Hq·nsplit ≤ 256). More splits shorten the attention
        # phase; the out-projection prologue requests 8 splits' partials at once, so up to 8 the
        # combine stays one load round (round 4, 24 layers: 8 splits 989 µs kernel vs 1 split
        # 1066, 4 splits 1019, 16 splits 1044; profiles/decode_mega_r4.txt)
        self.nb = nb
        # batched steps keep ~128 attention workgroups (8 // nb splits): the others then stream
        # their FFN1 slice during the attention phase instead of in the out-projection prologue
        want = max(1, int(os.environ.get("PIAMD_MEGA_NSPLIT", "8")) // nb)
        self.nsplit = min(16, max_splits(nb, HQ_), max(want, math.ceil(self.maxS / 256)))
        assert math.ceil(self.maxS / 256) <= self.nsplit, "max_seq_len too long for the split count"
        # long contexts (batch 1): every workgroup attends — at prompt 1024 16 splits beat 8
        # (greedy generate 1.169 -> 1.096 ms/token), at prompt 128 they lose (0.894 -> 0.978: the
        # FFN1 stream no longer overlaps the attention phase); profiles/decode_r6.txt
        self.nsplit_long = min(16, max_splits(nb, HQ_)) if nb == 1 else self.nsplit
        self.long_ctx = int(os.environ.get("PIAMD_MEGA_LONG_CTX", "512"))
        # one slot per layer (and per residual update) for every vector handed between
        # workgroups: each address is written once per launch, so readers may use cached loads
        nl, f32, bf = self.nl, dict(dtype=torch.float32, device=dev), dict(dtype=torch.bfloat16, device=dev)
        pstride = (HQ_ * max(self.nsplit, self.nsplit_long) * (D_ + 2) + 63) // 64 * 64
        self.rbuf = torch.zeros(2 * nl * nb, E_, **bf)
        self.qn = torch.zeros(nl * nb, HQ_ * D_, **f32)
        self.kvn = torch.zeros(nl * nb, 2 * HK_ * D_, **f32)
        self.part = torch.zeros(nl * nb * pstride, **f32)
        self.h = torch.zeros(nl * nb, F_, **bf)
        self.neox = 1 if getattr(gen, "neox_rotary", True) else 0
        self.log2_base = math.log2(float(getattr(gen, "rope_base", 10000.0)))
        self.bar = torch.zeros(19 * 64, dtype=torch.int32, device=dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self.act = 1 if gen.act == "gelu_tanh" else 0
        self.eps = float(gen.cfg.layer_norm_eps)
        self.trace = None  # set to a zeroed int64 [256, 5·nl, 4] tensor to record phase times
        # FFN phases issue the next weight slice only after their GEMV (1, default) or half of it
        # at the GEMV midpoint (0): the loader waves are compute waves too, and a 64 KiB DMA burst
        # stalls their issue for ~2 us (FFN1 / FFN2 GEMV 5.1 / 4.5 us -> 2.7 / 1.8 us late; kernel
        # 985 -> 956 us, profiles/decode_mega_r4.txt)
        # bit 2 (batch 1 default): the FFN2 slice head is read through the memory-side cache right
        # behind the FFN1 head, so the FFN1 → FFN2 hand-over DMA is served from it (kernel
        # 832 → 816 µs; at 4 rows every workgroup attends and the touch only moves the wait)
        self.late_dma = int(os.environ.get("PIAMD_MEGA_LATE_DMA", "5" if nb == 1 else "1"))
        # the round-4 dedicated-loader-wave variant is retired (the MFMA 4-wave kernel beat it:
        # 834 vs 908 µs); the field stays 0
        self.loader = 0
        # GEMV phases on MFMA (1, default: 16 weight columns × 32 k per instruction, no per-column
        # butterfly; kernel 869 vs 976 µs on the VALU, profiles/decode_mega_r5.txt) or the VALU
        # (0; A/B instantiations for GPT-1.3B bf16 and int8)
        self.mm = int(os.environ.get("PIAMD_MEGA_MFMA", "1"))
        if not self._variant_ok(self.mm):
            self.mm = 1 - self.mm
        # greedy tail (decode_head_kernel): LM head + argmax + bookkeeping + next embedding
        self.head_ok = nb == 1 and _lib.has("piamd_decode_head_greedy") and self._head_tables(gen)
        self.best = torch.zeros(8 * 32, dtype=torch.int64, device=dev)
        self.cnt = torch.zeros(9 * 64, dtype=torch.int32, device=dev)

    def _variant_ok(self, mm: int) -> bool:
        return _lib.lib().piamd_decode_mega_variant_supported(
            self.E, self.D, self.HQ, self.HK, self.F, self.rot, self.w8, self.nb, mm) == 1

    def _head_tables(self, gen) -> bool:
        m = gen.model
        emb = getattr(getattr(m, "gpt", None), "embeddings", None)
        if emb is None or not hasattr(m, "head_weight"):
            return False
        self.head_w = m.head_weight().detach()
        self.wemb = emb.word_embeddings.weight.detach()
        self.pemb = getattr(emb, "position_embeddings", None)
        ts = [self.head_w, self.wemb, self.pemb, *gen.final_ln[:2]]
        if any(t is None or t.dtype != torch.bfloat16 or not t.is_contiguous() or not t.is_cuda for t in ts):
            return False
        self.pemb = self.pemb.detach()
        return (self.E == E and self.head_w.dim() == 2 and self.head_w.shape[1] == E
                and self.wemb.shape[1] == E and self.pemb.shape[1] == E
                and self.head_w.shape[0] == self.wemb.shape[0])

    def greedy_tail(self, y, out, t, done, eos, pad, pos, tok, resid) -> None:
        """After a step: final LN + LM head + argmax on ``y`` [E] → token (``pad`` once ``done``)
        into ``out[0, t]`` and ``tok``; ``done`` |= token == ``eos``; ``pos`` += 1; ``resid`` =
        the next step's embedding (word_emb[token] + pos_emb[pos]). One launch."""
        assert out.dtype == torch.int64 and out.is_contiguous() and 0 <= t < out.shape[-1]
        assert done.dtype == torch.bool and tok.dtype == torch.int64 and resid.numel() == E
        g, b, eps = self.gen.final_ln
        a = _lib.HeadArgs(y.data_ptr(), g.data_ptr(), b.data_ptr(), float(eps), self.head_w.shape[0],
                          self.head_w.data_ptr(), self.best.data_ptr(), self.cnt.data_ptr(),
                          out.data_ptr() + 8 * t, done.data_ptr(), -1 if eos is None else int(eos),
                          int(pad), pos.data_ptr(), tok.data_ptr(), self.wemb.data_ptr(),
                          self.pemb.data_ptr(), self.pemb.shape[0], resid.data_ptr())
        _lib.call("piamd_decode_head_greedy", ctypes.byref(a), E, _lib.stream())

    def splits_for(self, ctx) -> int:
        """Attention splits of a step whose longest row holds ``ctx`` keys (None: unknown)."""
        return self.nsplit_long if ctx is not None and ctx > self.long_ctx else self.nsplit

    def __call__(self, resid: torch.Tensor, pos: torch.Tensor, ctx=None) -> torch.Tensor:
        """resid: bf16 [nb, E] (or [E] at nb = 1) embedding output; pos: device int32 [nb] = each
        row's cache slot for this token; ``ctx`` (host int, optional): the longest row's key count,
        which picks the attention split count. Returns the last layer's residual stream [nb, E]
        ([E] at nb = 1; a view of an internal buffer)."""
        nb = self.nb
        assert resid.is_contiguous() and resid.numel() == nb * self.E and resid.dtype == torch.bfloat16
        assert pos.dtype == torch.int32 and pos.is_cuda and pos.is_contiguous() and pos.numel() == nb
        if self.trace is not None:  # the kernel writes 4 int64 slots per (workgroup, phase)
            assert (self.trace.dtype == torch.int64 and self.trace.is_cuda
                    and self.trace.numel() >= 256 * 5 * self.nl * 4), "trace must be int64 [256, 5*nl, 4]"
        a = _lib.MegaArgs(self.table.data_ptr(), self.nl, self.maxS, self.splits_for(ctx), self.act,
                          self.eps, (1.0 / math.sqrt(self.D)) * 1.4426950408889634, resid.data_ptr(),
                          self.rbuf.data_ptr(), self.qn.data_ptr(), self.kvn.data_ptr(), self.part.data_ptr(),
                          self.h.data_ptr(), self.bar.data_ptr(), self.err.data_ptr(),
                          pos.data_ptr(), _lib.ptr(self.trace), self.late_dma, self.loader,
                          self.rot, self.neox, self.log2_base, self.w8, nb, self.mm)
        _lib.call("piamd_decode_mega", ctypes.byref(a), self.E, self.D, self.HQ, self.HK, self.F,
                  _lib.stream())
        return self.rbuf[-1] if nb == 1 else self.rbuf[-nb:]

    def check(self) -> None:
        """Raise if a grid barrier of an earlier launch timed out (synchronises)."""
        n = int(self.err.item())
        if n:
            raise RuntimeError(f"decode_mega: a grid barrier timed out in {n} launch(es) "
                               "(workgroups not co-resident?)")
