"""Single-launch decode step (csrc/kernels/decode_mega.hip) against the per-op decode path
(LN-fused GEMVs + split-K decode attention, itself checked against fp32 in
test_infer_kernels_gpu.py) on a GPT-1.3B-width model (E 2048, 16 heads, FFN 8192), the GPT-3
350M width (E 1024, D 64, FFN 4096) and a GQA 4:1 stack with rotary embedding (NeoX and GPT-J
styles)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(autouse=True)
def _mega_on(monkeypatch):
    monkeypatch.setenv("PIAMD_DECODE_MEGA", "1")


def _gpt13b_width(layers, max_pos, preset="gpt3-1.3b", **over):
    import paddle_infer_amd as paddle
    from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config
    paddle.seed(11)
    cfg = gpt_config(preset, dtype="float32", num_layers=layers, vocab_size=2048,
                     hidden_dropout_prob=0.0, max_position_embeddings=max_pos, **over)
    m = GPTForPretraining(cfg).eval()
    with torch.no_grad():  # non-trivial LN / bias values so every epilogue term is exercised
        for L in m.gpt.layers:
            for t in (L.ln1.weight, L.ln2.weight):
                t.add_(torch.randn_like(t) * 0.1)
            for t in (L.ln1.bias, L.ln2.bias, L.attn.qkv_proj.bias, L.attn.out_proj.bias,
                      L.mlp.fc1.bias, L.mlp.fc2.bias):
                t.copy_(torch.randn_like(t) * 0.05)
    return m.to(DEV).to(torch.bfloat16)


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm()).item()


# GEMV phases on MFMA (default) / on the VALU (A/B instantiation)
@pytest.mark.parametrize("loader", ["mfma", "valu"])
@pytest.mark.parametrize("max_seq,prompt", [(256, 37), (1024, 300)])
def test_mega_decode_matches_per_op_path(max_seq, prompt, loader, monkeypatch):
    monkeypatch.setenv("PIAMD_MEGA_MFMA", "1" if loader == "mfma" else "0")
    from paddle_infer_amd.inference import mega_decode
    from paddle_infer_amd.inference.generation import GPTGenerator
    m = _gpt13b_width(2, max_seq)
    g_mega = GPTGenerator(m, max_batch=1, max_seq_len=max_seq, use_hip_graph=False)
    g_ref = GPTGenerator(m, max_batch=1, max_seq_len=max_seq, use_hip_graph=False)
    g_ref.use_mega = False  # force the per-op path
    assert mega_decode.eligible(g_mega, 1) and not mega_decode.eligible(g_mega, 2)
    ids = torch.randint(0, 2048, (1, prompt), device=DEV)
    lens = torch.full((1,), prompt, device=DEV)
    la, lb = g_mega.prefill(ids, lens), g_ref.prefill(ids, lens)
    pos = torch.full((1,), prompt, dtype=torch.int32, device=DEV)
    for step in range(6):
        tok = lb.argmax(-1)
        la, lb = g_mega.decode(tok, pos), g_ref.decode(tok, pos)
        assert isinstance(g_mega._mega[1], mega_decode.MegaDecoder)
        assert g_mega._mega[1].loader == 0 and g_mega._mega[1].mm == (loader == "mfma")
        assert _rel(la, lb) < 2e-2, (step, _rel(la, lb))
        for (ka, va), (kb, vb) in zip(g_mega.caches, g_ref.caches):
            p = int(pos[0])
            assert _rel(ka[0, :, p], kb[0, :, p]) < 1e-2 and _rel(va[0, :, p], vb[0, :, p]) < 1e-2
        pos += 1
    g_mega._mega[1].check()


def test_mega_decode_graph_generate_matches_eager():
    from paddle_infer_amd.inference.generation import GPTGenerator
    m = _gpt13b_width(2, 256)
    ids = torch.randint(0, 2048, (1, 9))
    eager = GPTGenerator(m, max_batch=1, max_seq_len=256, use_hip_graph=False)
    graph = GPTGenerator(m, max_batch=1, max_seq_len=256, use_hip_graph=True)
    a = eager.generate(ids, max_new_tokens=12)
    for _ in range(2):  # second call replays the cached graph
        b = graph.generate(ids, max_new_tokens=12)
        assert torch.equal(a.cpu(), b.cpu()), (a, b)
    graph._mega[1].check()


def test_mega_greedy_tail_matches_logits_path():
    """Fused greedy tail (decode_head_kernel) against the launch-per-op tail: every chosen token
    is a maximiser of the per-op path's logits (teacher-forced on the chosen tokens, so a wrong
    position, embedding or cache slot shows up as a logit mismatch), and EOS masks to pad."""
    from paddle_infer_amd.inference.generation import GPTGenerator
    m = _gpt13b_width(2, 256)
    torch.manual_seed(3)
    ids = torch.randint(0, 2048, (1, 9), device=DEV)
    n = 12
    g = GPTGenerator(m, max_batch=1, max_seq_len=256, use_hip_graph=False)
    out = g.generate(ids, max_new_tokens=n)
    assert g._mega[1].head_ok
    ref = GPTGenerator(m, max_batch=1, max_seq_len=256, use_hip_graph=False)
    logits = ref.prefill(ids, torch.full((1,), 9, device=DEV))
    pos = torch.full((1,), 9, dtype=torch.int32, device=DEV)
    for t in range(n):
        lg = logits[0].float()
        tok = int(out[0, t])
        assert lg[tok] >= lg.max() - 0.02 * lg.abs().max(), (t, tok, lg.argmax().item())
        if t + 1 < n:
            logits = ref.decode(out[:, t].contiguous(), pos)
            pos += 1
    # EOS: the first occurrence of the token at step 3 ends the sequence, pad after it
    eos = int(out[0, 3])
    k = int((out[0] == eos).nonzero()[0])
    out2 = g.generate(ids, max_new_tokens=n, eos_token_id=eos, pad_token_id=7)
    assert torch.equal(out2[0, :k + 1].cpu(), out[0, :k + 1].cpu()), (out, out2)
    assert (out2[0, k + 1:] == 7).all(), out2
    g._mega[1].check()


@pytest.mark.parametrize("shape", ["gpt3-350m", "gqa4_rope_neox", "gqa4_rope_gptj", "gpt13_rope"])
def test_mega_decode_other_shapes_match_per_op_path(shape):
    """The templated kernel at the other instantiated shapes: a second width (E 1024, D 64 —
    waves 2-3 idle in the dot products, 8 lanes per head row), GQA 4:1 (4 KV heads shared by 16
    query heads) and whole-head rotary embedding in both pairing styles (q and the new k rotated in
    the attention phase, k cached after rotation), each against the per-op decode path."""
    from paddle_infer_amd.inference import mega_decode
    from paddle_infer_amd.inference.generation import GPTGenerator
    preset, over, rope = {"gpt3-350m": ("gpt3-350m", {}, None),
                          "gqa4_rope_neox": ("gpt3-1.3b", {"num_kv_heads": 4}, True),
                          "gqa4_rope_gptj": ("gpt3-1.3b", {"num_kv_heads": 4}, False),
                          "gpt13_rope": ("gpt3-1.3b", {}, True)}[shape]
    m = _gpt13b_width(2, 512, preset, **over)
    kw = dict(rotary_dim=m.cfg.head_dim, neox_rotary=rope) if rope is not None else {}
    g_mega = GPTGenerator(m, max_batch=1, max_seq_len=512, use_hip_graph=False, **kw)
    g_ref = GPTGenerator(m, max_batch=1, max_seq_len=512, use_hip_graph=False, **kw)
    g_ref.use_mega = False
    assert mega_decode.eligible(g_mega, 1), mega_decode.shape_of(g_mega)
    prompt = 77
    ids = torch.randint(0, 2048, (1, prompt), device=DEV)
    lens = torch.full((1,), prompt, device=DEV)
    la, lb = g_mega.prefill(ids, lens), g_ref.prefill(ids, lens)
    pos = torch.full((1,), prompt, dtype=torch.int32, device=DEV)
    for step in range(5):
        tok = lb.argmax(-1)
        la, lb = g_mega.decode(tok, pos), g_ref.decode(tok, pos)
        assert isinstance(g_mega._mega[1], mega_decode.MegaDecoder) and g_mega._mega[1].loader == 0
        assert _rel(la, lb) < 2e-2, (step, _rel(la, lb))
        for (ka, va), (kb, vb) in zip(g_mega.caches, g_ref.caches):
            p = int(pos[0])
            assert _rel(ka[0, :, p], kb[0, :, p]) < 1e-2 and _rel(va[0, :, p], vb[0, :, p]) < 1e-2
        pos += 1
    g_mega._mega[1].check()


def test_mega_decode_shape_gate():
    """Shapes without an instantiation are refused (per-op path), never launched."""
    from paddle_infer_amd.ops import _lib
    f = _lib.lib().piamd_decode_mega_shape_supported
    assert f(2048, 128, 16, 16, 8192, 0, 0) == 1 and f(1024, 64, 16, 16, 4096, 64, 0) == 1
    assert f(2048, 128, 16, 16, 8192, 0, 1) == 1 and f(2048, 128, 16, 4, 8192, 128, 1) == 1
    assert f(2560, 80, 32, 32, 10240, 0, 0) == 0 and f(2048, 128, 16, 8, 8192, 0, 0) == 0
    assert f(1024, 64, 16, 16, 4096, 0, 1) == 0
    fb = _lib.lib().piamd_decode_mega_batch_supported
    assert fb(2048, 128, 16, 16, 8192, 0, 0, 2) == 1 and fb(2048, 128, 16, 4, 8192, 128, 0, 4) == 1
    assert fb(2048, 128, 16, 16, 8192, 0, 0, 3) == 0 and fb(2048, 128, 16, 16, 8192, 0, 1, 2) == 1
    assert fb(1024, 64, 16, 16, 4096, 0, 1, 2) == 0
    assert f(2048, 128, 16, 16, 8192, 0, 2) == 1 and f(1024, 64, 16, 16, 4096, 0, 2) == 0  # int4
    fv = _lib.lib().piamd_decode_mega_variant_supported  # GEMV kind: 1 MFMA, 0 VALU
    assert fv(2048, 128, 16, 16, 8192, 0, 0, 1, 1) == 1 and fv(2048, 128, 16, 16, 8192, 0, 0, 1, 0) == 1
    assert fv(1024, 64, 16, 16, 4096, 0, 0, 1, 0) == 0 and fv(2048, 128, 16, 16, 8192, 0, 1, 1, 1) == 1
    assert fv(2048, 128, 16, 16, 8192, 0, 1, 1, 0) == 1 and fv(2048, 128, 16, 4, 8192, 128, 1, 1, 0) == 0
    assert fv(2048, 128, 16, 16, 8192, 0, 0, 4, 0) == 0 and fv(1024, 64, 16, 16, 4096, 64, 0, 4, 1) == 1


@pytest.mark.parametrize("shape", ["gpt13_int8", "gqa4_rope_int8", "gpt13_int8_valu", "gpt13_int4",
                                   "gqa4_rope_int4"])
def test_mega_decode_int8_weight_only_matches_per_op_path(shape, monkeypatch):
    """int8 weight-only projections (FusedMultiTransformerWeightOnly decode): the kernel streams
    the int8 codes (half the bytes) and applies the per-output-channel scales after each column
    sum; against the per-op weight-only GEMV path of the same generator settings."""
    from paddle_infer_amd.inference import mega_decode
    from paddle_infer_amd.inference.generation import GPTGenerator
    monkeypatch.setenv("PIAMD_MEGA_MFMA", "0" if shape.endswith("valu") else "1")
    over, kw = ({}, {}) if shape.startswith("gpt13") else \
        ({"num_kv_heads": 4}, dict(rotary_dim=128, neox_rotary=True))
    m = _gpt13b_width(2, 512, "gpt3-1.3b", **over)
    wo = "int4" if "int4" in shape else "int8"
    g_mega = GPTGenerator(m, max_batch=1, max_seq_len=512, use_hip_graph=False, weight_only=wo, **kw)
    g_ref = GPTGenerator(m, max_batch=1, max_seq_len=512, use_hip_graph=False, weight_only=wo, **kw)
    g_ref.use_mega = False
    assert mega_decode.eligible(g_mega, 1)
    prompt = 50
    ids = torch.randint(0, 2048, (1, prompt), device=DEV)
    lens = torch.full((1,), prompt, device=DEV)
    la, lb = g_mega.prefill(ids, lens), g_ref.prefill(ids, lens)
    pos = torch.full((1,), prompt, dtype=torch.int32, device=DEV)
    for step in range(4):
        tok = lb.argmax(-1)
        la, lb = g_mega.decode(tok, pos), g_ref.decode(tok, pos)
        assert g_mega._mega[1].w8 == (2 if wo == "int4" else 1) and g_mega._mega[1].loader == 0
        assert g_mega._mega[1].mm == (0 if shape.endswith("valu") else 1)
        assert _rel(la, lb) < 2e-2, (step, _rel(la, lb))
        pos += 1
    g_mega._mega[1].check()


@pytest.mark.parametrize("B", [2, 4])
@pytest.mark.parametrize("shape", ["gpt13", "gpt3-350m", "gqa4_rope_neox", "gpt13_int8", "gpt13_int4"])
def test_mega_decode_batched_rows_match_per_op_path(shape, B):
    """Batched single-launch steps (MegaCfg NB = 2 / 4: one LDS weight slice applied to every row,
    one attention workgroup per (row, head, split)) with a different prompt length per row — each
    row attends over its own cache length and writes its own slot — against the per-op path."""
    from paddle_infer_amd.inference import mega_decode
    from paddle_infer_amd.inference.generation import GPTGenerator
    preset, over, rope = {"gpt13": ("gpt3-1.3b", {}, None), "gpt13_int8": ("gpt3-1.3b", {}, None),
                          "gpt13_int4": ("gpt3-1.3b", {}, None),
                          "gpt3-350m": ("gpt3-350m", {}, None),
                          "gqa4_rope_neox": ("gpt3-1.3b", {"num_kv_heads": 4}, True)}[shape]
    m = _gpt13b_width(2, 512, preset, **over)
    kw = dict(rotary_dim=m.cfg.head_dim, neox_rotary=rope) if rope is not None else {}
    if shape.endswith(("int8", "int4")):
        kw["weight_only"] = shape[-4:]
    g_mega = GPTGenerator(m, max_batch=B, max_seq_len=512, use_hip_graph=False, **kw)
    g_ref = GPTGenerator(m, max_batch=B, max_seq_len=512, use_hip_graph=False, **kw)
    g_ref.use_mega = False
    assert mega_decode.eligible(g_mega, B) and not mega_decode.eligible(g_mega, 3)
    torch.manual_seed(5)
    lens = torch.tensor([61, 200, 3, 130][:B], device=DEV)
    ids = torch.randint(0, 2048, (B, int(lens.max())), device=DEV)
    la, lb = g_mega.prefill(ids, lens), g_ref.prefill(ids, lens)
    pos = lens.to(torch.int32)
    for step in range(4):
        tok = lb.argmax(-1)
        la, lb = g_mega.decode(tok, pos), g_ref.decode(tok, pos)
        mg = g_mega._mega[B]
        assert isinstance(mg, mega_decode.MegaDecoder) and mg.nb == B and mg.loader == 0
        for b in range(B):
            assert _rel(la[b], lb[b]) < 2e-2, (step, b, _rel(la[b], lb[b]))
        for (ka, va), (kb, vb) in zip(g_mega.caches, g_ref.caches):
            for b in range(B):
                p = int(pos[b])
                assert _rel(ka[b, :, p], kb[b, :, p]) < 1e-2 and _rel(va[b, :, p], vb[b, :, p]) < 1e-2
        pos = pos + 1
    g_mega._mega[B].check()


def test_mega_decode_batched_generate_and_beams():
    """generate() at batch 2 (greedy, eager loop over the batched step) matches the per-op
    generator token for token, and beam search with 4 beams (beams are batch rows) runs on the
    4-row step."""
    from paddle_infer_amd.inference.generation import GPTGenerator
    m = _gpt13b_width(2, 256)
    torch.manual_seed(9)
    ids = torch.randint(0, 2048, (2, 11), device=DEV)
    a = GPTGenerator(m, max_batch=4, max_seq_len=256, use_hip_graph=False)
    ref = GPTGenerator(m, max_batch=4, max_seq_len=256, use_hip_graph=False)
    ref.use_mega = False
    out_a, out_r = a.generate(ids, max_new_tokens=8), ref.generate(ids, max_new_tokens=8)
    assert a._mega.get(2), a._mega
    # bf16 near-ties may flip a late token; the first steps must agree
    assert torch.equal(out_a[:, :4].cpu(), out_r[:, :4].cpu()), (out_a, out_r)
    b = a.generate(ids[:1], max_new_tokens=6, num_beams=4)
    assert a._mega.get(4) and b.shape == (1, 6)
    assert a._mega[4].table is a._mega[2].table  # one set of weight copies per model
    a._mega[4].check()


def test_mega_decode_long_context_split_count():
    """Long contexts run the attention phase on 16 splits (every workgroup) instead of 8: the
    same layer-stack output either way, and the greedy loop picks 16 past ``long_ctx`` keys."""
    from paddle_infer_amd.inference.generation import GPTGenerator
    m = _gpt13b_width(2, 1024)
    g = GPTGenerator(m, max_batch=1, max_seq_len=1024, use_hip_graph=False)
    prompt = 700
    ids = torch.randint(0, 2048, (1, prompt), device=DEV)
    lens = torch.full((1,), prompt, device=DEV)
    g.prefill(ids, lens)
    mega = g._mega_decoder(1)
    assert mega.nsplit == 8 and mega.nsplit_long == 16
    assert mega.splits_for(prompt + 1) == 16 and mega.splits_for(100) == 8 and mega.splits_for(None) == 8
    tok = torch.tensor([5], device=DEV)
    pos = torch.full((1,), prompt, dtype=torch.int32, device=DEV)
    resid = m.gpt.embeddings(tok.view(1, 1), pos.long().view(1, 1)).reshape(-1).contiguous()
    a = mega(resid, pos, None).clone()   # 8 splits (rewrites the same cache slot both times)
    b = mega(resid, pos, prompt + 1).clone()  # 16 splits
    assert _rel(a, b) < 1e-2, _rel(a, b)
    out = g.generate(ids, lens, max_new_tokens=4)
    assert out.shape == (1, 4)
    mega.check()
