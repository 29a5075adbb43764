"""LLM serving: KV-cached generation for the GPT family on the fused multi-transformer path.

Parity: the reference serves GPT-style models through ``FusedMultiTransformer`` (context pass
writes the KV cache, then one decode step per token with ``time_step``) plus the sampling /
beam-search helpers (`phi/kernels/fusion/gpu/beam_search_softmax.cu`, top-k / top-p sampling).

MI355X design:
* the trained ``GPTForPretraining`` weights are used in place (no conversion copies);
* context pass: hipBLASLt GEMMs + flash attention + fused QKV-prep writing the cache;
* decode step: embedding → L × (LN → QKV GEMM → bias/RoPE/cache-write → split-K decode attention
  → out GEMM → add+LN → FFN) → add+LN → LM head, captured ONCE per batch size into a hipGraph
  (``torch.cuda.CUDAGraph``) over static token / position buffers; positions and lengths are
  device-resident so a replay is one host call per generated token;
* KV caches are one HBM allocation per layer sized for ``max_batch × max_seq_len`` (288 GB HBM3E
  fits hundreds of thousands of cached tokens for a 1.3B model).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..ops.search import beam_search_softmax

from ..incubate.nn import functional as IF
from ..incubate.nn.functional import _lin


class GPTGenerator:
    def __init__(self, model, max_batch: int = 8, max_seq_len: int | None = None,
                 use_hip_graph: bool = True, cache_dtype=None, weight_only: str | None = None,
                 prepack: bool = True, rotary_dim: int = 0, neox_rotary: bool = True,
                 rope_base: float = 10000.0):
        """``rotary_dim`` / ``neox_rotary`` / ``rope_base``: rotary position embedding applied to q
        and k in every layer (reference ``fused_multi_transformer`` ``rotary_emb_dims``), on top of
        whatever the model's embedding layer adds."""
        self.model = model.eval()
        self.rotary_dim, self.neox_rotary, self.rope_base = int(rotary_dim), bool(neox_rotary), float(rope_base)
        cfg = model.cfg
        self.cfg = cfg
        p0 = next(iter(model.parameters()))
        self.device, self.dtype = p0.device, (cache_dtype or p0.dtype)
        self.H = model.gpt.layers[0].attn.heads
        self.Hk = model.gpt.layers[0].attn.kv_heads
        self.D = cfg.head_dim
        self.max_batch = max_batch
        self.max_seq_len = max_seq_len or cfg.max_position_embeddings
        self.group = model.mp_group if getattr(model, "mp_group", None) is not None else None
        self.layers = []
        for L in model.gpt.layers:
            self.layers.append(dict(
                head_dim=self.D, ln_scale=L.ln1.weight, ln_bias=L.ln1.bias,
                qkv=_lin(L.attn.qkv_proj.weight), qkv_bias=L.attn.qkv_proj.bias,
                out=_lin(L.attn.out_proj.weight), out_bias=L.attn.out_proj.bias,
                ffn_ln_scale=L.ln2.weight, ffn_ln_bias=L.ln2.bias,
                ffn1=_lin(L.mlp.fc1.weight), ffn1_bias=L.mlp.fc1.bias,
                ffn2=_lin(L.mlp.fc2.weight), ffn2_bias=L.mlp.fc2.bias))
        if weight_only in ("int8", "int4"):  # FusedMultiTransformerWeightOnly path
            from ..ops.inference import weight_quantize
            algo, bits = f"weight_only_{weight_only}", 4 if weight_only == "int4" else 8
            for spec in self.layers:
                for key in ("qkv", "out", "ffn1", "ffn2"):
                    q, s = weight_quantize(spec[key].w.detach(), algo)
                    spec[key] = _lin(q, s, bits)
        elif self.device.type == "cuda" and prepack:  # MFMA-tile copies for decode GEMVs
            for spec in self.layers:
                for key in ("qkv", "out", "ffn1", "ffn2"):
                    spec[key].prepack()
        self.act = "gelu_tanh" if cfg.activation in ("gelu_tanh", "gelu_new") else "gelu"
        self.final_ln = (model.gpt.final_ln.weight, model.gpt.final_ln.bias, cfg.layer_norm_eps)
        shape = (max_batch, self.Hk, self.max_seq_len, self.D)
        self.caches = [(torch.zeros(shape, dtype=self.dtype, device=self.device),
                        torch.zeros(shape, dtype=self.dtype, device=self.device))
                       for _ in self.layers]
        self.use_graph = use_hip_graph and self.device.type == "cuda"
        self._graphs = {}
        self._mega = {}  # batch rows → MegaDecoder (False: not eligible), built on first use
        self.use_mega = True  # False: every decode step takes the per-op path

    # ------------------------------------------------------------------------------ model
    def _mp_gather(self, logits):
        if self.group is None or torch.distributed.get_world_size(self.group) == 1:
            return logits
        ws = torch.distributed.get_world_size(self.group)
        parts = [torch.empty_like(logits) for _ in range(ws)]
        torch.distributed.all_gather(parts, logits.contiguous(), group=self.group)
        return torch.cat(parts, -1)

    def _forward(self, ids, pos, lens, B, decode):
        S = ids.shape[1]
        caches = [(k[:B], v[:B]) for k, v in self.caches]
        if decode:
            position_ids = pos.long().view(B, 1)
        else:
            position_ids = torch.arange(S, device=ids.device).unsqueeze(0).expand(B, S)
        emb = self.model.gpt.embeddings(ids, position_ids)
        y = IF.multi_transformer_forward(
            emb, self.layers, self.H, self.Hk, True, self.cfg.layer_norm_eps, caches, pos, lens,
            None, decode, self.act, rotary_dim=self.rotary_dim, neox_rotary=self.neox_rotary,
            rope_base=self.rope_base, causal=True, group=self.group, max_len=self.max_seq_len,
            final_ln=self.final_ln)
        return y

    def _logits(self, y):
        from ..ops.linear import mm_nt  # own GEMM: the [V, h] table is already K-contiguous
        w = self.model.head_weight()
        y2 = y.reshape(-1, y.shape[-1])
        return self._mp_gather(mm_nt(y2.contiguous(), w).reshape(*y.shape[:-1], w.shape[0]))

    @torch.no_grad()
    def prefill(self, input_ids, lengths):
        """input_ids [B, S] right-padded; lengths [B]. Writes cache [0, S); returns last-token
        logits [B, V]."""
        B, S = input_ids.shape
        pos0 = torch.zeros(B, dtype=torch.int32, device=self.device)
        y = self._forward(input_ids, pos0, None, B, decode=False)
        last = y[torch.arange(B, device=y.device), lengths.long() - 1]
        return self._logits(last)

    def _mega_decoder(self, B):
        """The single-launch decode step (inference/mega_decode.py) when this model / batch fits
        it, else None (per-op path)."""
        from . import mega_decode
        if not self.use_mega or B not in mega_decode.BATCHES or not mega_decode.enabled():
            return None
        if B not in self._mega:  # the shape / dtype gate is static: evaluated once per batch size
            other = next((m for m in self._mega.values() if m), None)  # shares its weight copies
            self._mega[B] = mega_decode.MegaDecoder(self, B, other) if mega_decode.eligible(self, B) else False
        return self._mega[B] or None

    def _decode_eager(self, tok, pos, B):
        mega = self._mega_decoder(B)
        if mega is not None:
            from ..ops.norm import layer_norm
            resid = self.model.gpt.embeddings(tok.view(B, 1), pos.long().view(B, 1))
            resid = resid.reshape(B, -1).contiguous()
            y = layer_norm(mega(resid, pos.contiguous()).view(B, -1), *self.final_ln)
            return self._logits(y)
        lens = pos + 1
        y = self._forward(tok.view(B, 1), pos, lens, B, decode=True)
        return self._logits(y.view(B, -1))

    @torch.no_grad()
    def decode(self, tok, pos):
        """One step: tok [B] int64, pos [B] int32 (cache slot to write). Returns logits [B, V]."""
        B = tok.shape[0]
        # the single-launch step runs without a graph: it is ~6 launches, and a hipGraph replay
        # of it measured slower than direct launches (tools/mega_graph_probe.py)
        if not self.use_graph or self._mega_decoder(B) is not None:
            return self._decode_eager(tok, pos, B)
        ent = self._graphs.get(B)
        if ent is None:
            st_tok = tok.clone()
            st_pos = pos.clone()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    self._decode_eager(st_tok, st_pos, B)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                st_out = self._decode_eager(st_tok, st_pos, B)
            ent = self._graphs[B] = (g, st_tok, st_pos, st_out)
        g, st_tok, st_pos, st_out = ent
        st_tok.copy_(tok, non_blocking=True)
        st_pos.copy_(pos, non_blocking=True)
        g.replay()
        return st_out

    # ------------------------------------------------------------------------------ sampling
    @staticmethod
    def sample(logits, strategy="greedy_search", top_k=0, top_p=1.0, temperature=1.0,
               generator=None):
        if strategy == "greedy_search":
            from ..ops.search import argmax_rows
            return argmax_rows(logits)
        lg = logits.float() / max(temperature, 1e-6)
        if top_k and top_k > 0:
            kth = torch.topk(lg, top_k, -1).values[:, -1:]
            lg = lg.masked_fill(lg < kth, float("-inf"))
        if top_p < 1.0:
            sp, si = torch.sort(lg, -1, descending=True)
            cp = torch.softmax(sp, -1).cumsum(-1)
            drop = cp - torch.softmax(sp, -1) > top_p
            sp = sp.masked_fill(drop, float("-inf"))
            lg = torch.full_like(lg, float("-inf")).scatter(-1, si, sp)
        probs = torch.softmax(lg, -1)
        return torch.multinomial(probs, 1, generator=generator).squeeze(-1)

    @torch.no_grad()
    def generate(self, input_ids, lengths=None, max_new_tokens=32, decode_strategy="greedy_search",
                 top_k=0, top_p=1.0, temperature=1.0, eos_token_id=None, pad_token_id=0,
                 num_beams=1, length_penalty=1.0, seed=None):
        """Returns generated ids [B, max_new_tokens] (pad after EOS)."""
        B, S = input_ids.shape
        if num_beams > 1 or decode_strategy == "beam_search":
            return self._beam_search(input_ids, lengths, max_new_tokens, max(num_beams, 2),
                                     eos_token_id, pad_token_id, length_penalty)
        assert B <= self.max_batch and S + max_new_tokens <= self.max_seq_len
        ids = input_ids.to(self.device)
        lens = (lengths if lengths is not None else torch.full((B,), S)).to(self.device)
        gen = torch.Generator(device=self.device).manual_seed(seed) if seed is not None else None
        logits = self.prefill(ids, lens)
        out = torch.full((B, max_new_tokens), pad_token_id, dtype=torch.long, device=self.device)
        done = torch.zeros(B, dtype=torch.bool, device=self.device)
        pos = lens.to(torch.int32)
        mega = self._mega_decoder(B)
        if decode_strategy == "greedy_search" and mega is not None and mega.head_ok:
            return self._greedy_mega_loop(mega, logits, pos, out, done, max_new_tokens, eos_token_id,
                                          pad_token_id, ctx0=S)
        if decode_strategy == "greedy_search" and self.use_graph and mega is None:
            return self._greedy_graph_loop(logits, pos, out, done, max_new_tokens, eos_token_id,
                                           pad_token_id)
        for t in range(max_new_tokens):
            tok = self.sample(logits, decode_strategy, top_k, top_p, temperature, gen)
            tok = torch.where(done, torch.full_like(tok, pad_token_id), tok)
            out[:, t] = tok
            if eos_token_id is not None:
                done = done | (tok == eos_token_id)
                if (t & 7) == 7 and bool(done.all()):
                    break
            if t + 1 < max_new_tokens:
                logits = self.decode(tok, pos)
                pos = pos + 1
        for m in self._mega.values():  # one sync per generate(): a timed-out step fails loudly
            if m:
                m.check()
        return out

    def _greedy_mega_loop(self, mega, logits, pos, out, done, max_new_tokens, eos, pad, ctx0=None):
        """Batch-1 greedy decoding on the single-launch step: two launches per token, the layer
        stack (decode_mega_kernel) and the greedy tail (decode_head_kernel: final LN, LM head,
        argmax, pad / EOS bookkeeping, token store, position advance, next embedding). Same
        tokens as the eager loop up to logit ties within bf16 rounding."""
        from ..ops.search import argmax_rows
        tok = torch.where(done, torch.full_like(pos, pad, dtype=torch.long), argmax_rows(logits))
        out[:, 0] = tok
        if eos is not None:
            done = done | (tok == eos)
        pos = pos.clone()  # advanced in place by the tail kernel
        resid = self.model.gpt.embeddings(tok.view(1, 1), pos.long().view(1, 1)).reshape(-1).contiguous()
        tok = tok.clone()
        for t in range(1, max_new_tokens):
            ctx = None if ctx0 is None else ctx0 + t  # host-side key count: picks the split count
            mega.greedy_tail(mega(resid, pos, ctx), out, t, done, eos, pad, pos, tok, resid)
            if eos is not None and (t & 7) == 7 and bool(done.all()):
                break
        mega.check()
        return out

    def _greedy_graph_loop(self, logits, pos, out, done, max_new_tokens, eos, pad):
        """Greedy decoding with the token choice INSIDE the captured step: one graph replay per
        token runs the decoder, the argmax (own kernel), the EOS / pad bookkeeping and feeds the
        chosen token and position back into its own static inputs — the host only copies the token
        column out (same tokens as the eager loop)."""
        from ..ops.search import argmax_rows
        B = pos.shape[0]
        tok = torch.where(done, torch.full_like(pos, pad, dtype=torch.long), argmax_rows(logits))
        if eos is not None:
            done = done | (tok == eos)

        def load(st):
            st["tok"].copy_(tok)
            st["pos"].copy_(pos)
            st["done"].copy_(done)
            st["pad"].fill_(pad)
            if eos is not None:  # the graph reads the EOS id from st["eos"]: refresh per call
                st["eos"].fill_(eos)
        key = ("greedy", B, eos is not None)
        ent = self._graphs.get(key)
        if ent is None:
            st = dict(tok=torch.zeros(B, dtype=torch.long, device=self.device),
                      pos=torch.zeros(B, dtype=torch.int32, device=self.device),
                      done=torch.zeros(B, dtype=torch.bool, device=self.device),
                      eos=torch.tensor(eos if eos is not None else -1, device=self.device),
                      pad=torch.tensor(pad, device=self.device))

            def step():
                lg = self._decode_eager(st["tok"], st["pos"], B)
                nxt = torch.where(st["done"], st["pad"], argmax_rows(lg))
                if eos is not None:
                    st["done"].logical_or_(nxt == st["eos"])
                st["tok"].copy_(nxt)
                st["pos"].add_(1)
            # warm-up from the real state: it writes the KV slots pos and pos + 1, which the real
            # steps rewrite before anything reads them
            load(st)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    step()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
            ent = self._graphs[key] = (g, st)
        g, st = ent
        load(st)
        for t in range(max_new_tokens):
            out[:, t].copy_(st["tok"])
            if eos is not None and (t & 7) == 7 and bool(st["done"].all()):
                break
            if t + 1 < max_new_tokens:
                g.replay()
        return out

    def _reorder(self, src, B, L=None):
        """Caches of rows [0, B) gathered by source beam ``src``; only the first ``L`` positions
        (the ones written so far) move."""
        L = self.max_seq_len if L is None else min(int(L), self.max_seq_len)
        for k, v in self.caches:
            k[:B, :, :L].copy_(k[:B, :, :L].index_select(0, src))
            v[:B, :, :L].copy_(v[:B, :, :L].index_select(0, src))

    def _beam_search(self, input_ids, lengths, max_new_tokens, nb, eos, pad, length_penalty):
        """Beam search (reference `beam_search_softmax`): beams live as batch rows; each step the
        caches are gathered by source beam."""
        B0, S = input_ids.shape
        B = B0 * nb
        assert B <= self.max_batch
        ids = input_ids.to(self.device).repeat_interleave(nb, 0)
        lens = (lengths if lengths is not None else torch.full((B0,), S)).to(self.device).repeat_interleave(nb)
        logits = self.prefill(ids, lens)
        dev = self.device
        # one fused beam_search_softmax launch pair per step (ops/search.py): log-softmax, per-beam
        # top-k, per-batch top-beam, token-history (cache_ids) rewrite by parent beam
        end = torch.tensor([eos if eos is not None else -1], dtype=torch.int32, device=dev)
        cum = torch.zeros(B, dtype=torch.float32, device=dev)
        stop = torch.zeros(B, dtype=torch.bool, device=dev)
        seq_lens = lens.to(torch.int32).clamp_min(1)
        hist = torch.full((B, max_new_tokens), pad, dtype=torch.int32, device=dev)
        offs = torch.zeros((B0, nb, S + max_new_tokens), dtype=torch.int32, device=dev)
        pos = lens.to(torch.int32)
        ar = torch.arange(B0, device=dev).repeat_interleave(nb) * nb
        for t in range(max_new_tokens):
            step = torch.full((B,), t, dtype=torch.int32, device=dev)
            tok, cum, hist, offs, parent, stop, seq_lens, _ = beam_search_softmax(
                logits, cum, seq_lens, stop, end, step, hist, offs, nb, S, max_new_tokens,
                fuse_softmax=True, early_stop=False, length_penalty=0.0)
            src = ar + parent.long()
            if eos is not None:
                stop = stop | (tok == eos)
            self._reorder(src, B, S + t)  # positions [0, S + t) are written (prompt + t steps)
            if t + 1 < max_new_tokens:
                logits = self.decode(tok.long(), pos)
                pos = pos + 1
        seqs = hist.long()
        L = (seqs != pad).sum(-1).clamp_min(1).float().view(B0, nb)
        best = (cum.view(B0, nb) / L ** length_penalty).argmax(-1)
        return seqs.view(B0, nb, -1)[torch.arange(B0, device=dev), best]


def generate(model, input_ids, **kw):
    """Functional helper: build (and cache on the model) a :class:`GPTGenerator`."""
    gen_kw = {k: kw.pop(k) for k in ("max_batch", "max_seq_len", "use_hip_graph") if k in kw}
    g = getattr(model, "_piamd_generator", None)
    if g is None:
        g = GPTGenerator(model, max_batch=gen_kw.get("max_batch", max(8, input_ids.shape[0] * kw.get("num_beams", 1))),
                         max_seq_len=gen_kw.get("max_seq_len"), use_hip_graph=gen_kw.get("use_hip_graph", True))
        model._piamd_generator = g
    return g.generate(input_ids, **kw)
