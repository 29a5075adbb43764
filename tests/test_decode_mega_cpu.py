"""Single-launch decode step: the eligibility gate and the ctypes mirror of MegaArgs (the kernel
itself is covered by tests/test_decode_mega_gpu.py)."""
import re
import os

import torch


def test_not_eligible_off_gpu_or_off_shape(monkeypatch):
    import paddle_infer_amd as paddle
    from paddle_infer_amd.inference import mega_decode
    from paddle_infer_amd.inference.generation import GPTGenerator
    from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config
    monkeypatch.setenv("PIAMD_DECODE_MEGA", "1")
    paddle.seed(0)
    m = GPTForPretraining(gpt_config("gpt3-tiny", dtype="float32", hidden_dropout_prob=0.0)).eval()
    gen = GPTGenerator(m, max_batch=2, max_seq_len=64)
    assert not mega_decode.eligible(gen, 1)          # CPU, fp32, E 256
    assert gen._mega_decoder(1) is None
    ids = torch.randint(0, 1024, (1, 5))
    assert gen.generate(ids, max_new_tokens=3).shape == (1, 3)  # per-op path still serves


def test_megaargs_mirror_matches_kernel_struct():
    from paddle_infer_amd.ops import _lib
    src = open(os.path.join(os.path.dirname(_lib.__file__), "..", "csrc", "kernels",
                            "decode_mega.hip")).read()
    body = src[src.index("struct MegaArgs {"):]
    body = body[:body.index("};")]
    body = re.sub(r"//[^\n]*", "", body)
    names = re.findall(r"\b(\w+);", body)
    assert names == [f[0] for f in _lib.MegaArgs._fields_], names


def test_headargs_mirror_matches_kernel_struct():
    import ctypes
    from paddle_infer_amd.ops import _lib
    src = open(os.path.join(os.path.dirname(_lib.__file__), "..", "csrc", "kernels",
                            "decode_mega.hip")).read()
    body = src[src.index("struct HeadArgs {") + len("struct HeadArgs {"):]
    body = re.sub(r"//[^\n]*", "", body[:body.index("};")])
    names = [re.findall(r"\w+", part)[-1] for stmt in body.split(";") if stmt.strip()
             for part in stmt.split(",")]
    assert names == [f[0] for f in _lib.HeadArgs._fields_], names
    assert ctypes.sizeof(_lib.HeadArgs) == 136


def test_out_in_weight_codes_roundtrip():
    """The decode kernel's [out, in] weight images: int8 codes and int4 codes packed two per byte
    (k ascending from the low nibble) times the per-channel scales reproduce the weight-only
    dequantisation exactly; bf16 weights come out transposed to [out, in]."""
    from paddle_infer_amd.incubate.nn.functional import _lin
    from paddle_infer_amd.inference.mega_decode import _out_in
    from paddle_infer_amd.ops.inference import weight_dequantize, weight_quantize
    torch.manual_seed(0)
    w = torch.randn(64, 96)  # [K (in), N (out)] as the generator stores it
    for algo, bits in (("weight_only_int8", 8), ("weight_only_int4", 4)):
        q, s = weight_quantize(w, algo)
        codes, scale = _out_in(_lin(q, s, bits))
        if bits == 4:
            u = codes.to(torch.int16)
            lo, hi = u & 0xF, (u >> 4) & 0xF
            codes = torch.stack([lo, hi], -1).reshape(codes.shape[0], -1)
            codes = torch.where(codes >= 8, codes - 16, codes)
        deq = weight_dequantize(q, s, algo, "float32").t()  # [out, in]
        assert codes.shape == deq.shape
        assert torch.equal(codes.float() * scale[:, None], deq.float()), algo
    wb = w.to(torch.bfloat16)
    t, none = _out_in(_lin(wb))
    assert none is None and torch.equal(t, wb.t().contiguous())


def test_batched_split_budget():
    """One attention workgroup per (row, head, split) ≤ 256: the split budget per row count."""
    from paddle_infer_amd.inference import mega_decode
    assert mega_decode.BATCHES == (1, 2, 4)
    assert [mega_decode.max_splits(b, 16) for b in (1, 2, 4)] == [16, 8, 4]
