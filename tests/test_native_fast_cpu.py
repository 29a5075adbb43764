"""The IR-optimised model the native C++ predictor's GPU path consumes
(`Predictor.save_optimized_model`, `Config.enable_save_optim_model`): the fused program
(multihead_matmul, fc, fused_fc_elementwise_layernorm, skip_layernorm, ...) round-trips through
the Paddle wire format and reproduces the unoptimised model's outputs."""
import os

import numpy as np
import torch

from paddle_infer_amd import inference as pinf
from paddle_infer_amd import jit
from paddle_infer_amd.models.bert import BertModel, bert_config
from paddle_infer_amd.static import InputSpec


def _export(tmp_path):
    torch.manual_seed(0)
    m = BertModel(bert_config("bert-tiny"))
    m.eval()
    d = str(tmp_path / "bert")
    os.makedirs(d, exist_ok=True)
    jit.save(jit.to_static(m, input_spec=[InputSpec([None, 64], "int64", "input_ids")]), os.path.join(d, "model"))
    return d


def _run(prog, params, ids, ir):
    c = pinf.Config(prog, params)
    c.switch_ir_optim(ir)
    p = pinf.create_predictor(c)
    p.get_input_handle(p.get_input_names()[0]).copy_from_cpu(ids)
    p.run()
    return p, [p.get_output_handle(n).copy_to_cpu() for n in p.get_output_names()]


def test_optimized_model_round_trip(tmp_path):
    d = _export(tmp_path)
    ids = np.random.RandomState(0).randint(1, 1000, size=(2, 64)).astype("int64")
    _, ref = _run(os.path.join(d, "model.pdmodel"), os.path.join(d, "model.pdiparams"), ids, False)
    c = pinf.Config(os.path.join(d, "model.pdmodel"), os.path.join(d, "model.pdiparams"))
    c.enable_save_optim_model(True)
    c.set_optim_cache_dir(str(tmp_path))
    pinf.create_predictor(c)
    pre = str(tmp_path / "_optimized")
    assert os.path.exists(pre + ".pdmodel") and os.path.exists(pre + ".pdiparams")
    p, got = _run(pre + ".pdmodel", pre + ".pdiparams", ids, False)
    types = {op.type for op in p.program.global_block().ops}
    assert {"multihead_matmul", "fc", "skip_layernorm"} <= types, types
    for a, b in zip(got, ref):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)
