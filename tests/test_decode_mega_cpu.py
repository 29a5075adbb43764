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
