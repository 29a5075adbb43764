"""Paddle-wire fused_multi_transformer program on the GPU (bf16 Predictor): context + decode
through create_predictor match the dygraph FusedMultiTransformer; a jit-saved GPT is rewritten
into one fused_multi_transformer op and matches dygraph logits."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.dirname(__file__))


@pytest.fixture(autouse=True)
def _lib():
    import paddle_infer_amd  # noqa: F401
    from paddle_infer_amd.ops import _lib
    _lib.lib()


def test_fused_multi_transformer_wire_program_gpu(tmp_path):
    from test_program_ops_cpu import run_fmt_wire
    run_fmt_wire(tmp_path, "cuda")


def test_gpt_export_fused_multi_transformer_gpu(tmp_path):
    from paddle_infer_amd import inference as pinf, jit
    from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config
    from paddle_infer_amd.static import InputSpec
    torch.manual_seed(0)
    m = GPTForPretraining(gpt_config("gpt3-tiny", hidden_size=256, num_heads=2, num_layers=2,
                                     vocab_size=512))
    m.eval()
    path = str(tmp_path / "gpt")
    jit.save(jit.to_static(m, input_spec=[InputSpec([None, 64], "int64", "ids")]), path)
    c = pinf.Config(path + ".pdmodel", path + ".pdiparams")
    c.enable_use_gpu(256, 0)
    c.exp_enable_mixed_precision(pinf.PrecisionType.Bfloat16)
    pred = pinf.create_predictor(c)
    assert pred.pass_stats["fused_multi_transformer_encoder_traced_pass"] == 2
    ids = torch.randint(0, 512, (2, 64), device="cuda")
    mg = m.to("cuda")
    with torch.no_grad():
        ref = mg(ids)
    ref = ref[0] if isinstance(ref, (tuple, list)) else ref
    pred.get_input_handle("ids").share_external_data(ids)
    assert pred.run()
    got = pred.get_output_handle(pred.get_output_names()[0]).to_torch().float()
    torch.testing.assert_close(got, ref.float(), rtol=6e-2, atol=6e-2)
