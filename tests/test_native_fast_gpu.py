"""Native C++ predictor on the framework's GPU kernels (`csrc/native/fast_ops.hip`: skinny / assembly
GEMMs with fused epilogues, flash attention, LayerNorm, embedding — no Python in the process) for
an IR-optimised fp16 / bf16 BERT saved by the Python Predictor, eager and hipGraph, against the
Python Predictor running the same optimised program."""
import os

import numpy as np
import pytest
import torch

from native_infer_util import RUN, native_outputs

from paddle_infer_amd import inference as pinf
from paddle_infer_amd import jit
from paddle_infer_amd.models.bert import BertModel, bert_config
from paddle_infer_amd.static import InputSpec

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not os.path.exists(RUN), reason="native engine not built")]


def _optimized(tmp_path, dtype, ids, name="bert-tiny", **over):
    torch.manual_seed(0)
    m = BertModel(bert_config(name, **over))
    m.eval()
    d = str(tmp_path / "bert")
    os.makedirs(d, exist_ok=True)
    jit.save(jit.to_static(m, input_spec=[InputSpec([None, ids.shape[1]], "int64", "input_ids")]),
             os.path.join(d, "model"))
    c = pinf.Config(os.path.join(d, "model.pdmodel"), os.path.join(d, "model.pdiparams"))
    c.enable_use_gpu(256, 0)
    c.exp_enable_mixed_precision(pinf.PrecisionType.Half if dtype == "fp16" else pinf.PrecisionType.Bfloat16)
    c.enable_save_optim_model(True)
    c.set_optim_cache_dir(str(tmp_path))
    p = pinf.create_predictor(c)
    p.get_input_handle(p.get_input_names()[0]).copy_from_cpu(ids)
    p.run()
    outs = [p.get_output_handle(n).copy_to_cpu() for n in p.get_output_names()]
    return str(tmp_path / "_optimized"), [np.asarray(o, dtype=np.float32) for o in outs]


@pytest.mark.parametrize("dtype", ["fp16", "bf16"])
@pytest.mark.parametrize("B", [2, 16])
@pytest.mark.parametrize("graph", [False, True])
def test_native_bert_matches_python_predictor(tmp_path, dtype, B, graph):
    ids = np.random.RandomState(B).randint(1, 1000, size=(B, 64)).astype("int64")
    pre, ref = _optimized(tmp_path, dtype, ids)
    got, ms, _ = native_outputs(pre, {"input_ids": ids}, tmp_path, gpu=0, graph=graph,
                                warmup=1 if graph else 0, repeat=3)
    tol = 2e-2 if dtype == "fp16" else 6e-2
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        assert a.shape == b.shape
        np.testing.assert_allclose(a, b, rtol=tol, atol=tol)
    assert ms is not None and ms > 0


def test_native_bert_large_layer_shapes(tmp_path):
    """BERT-Large widths (E 1024, 16 heads, FFN 4096) with 2 layers: the assembly-GEMM epilogues
    (bias, exact GELU) and the 128-row skinny GEMMs of the real model."""
    ids = np.random.RandomState(7).randint(1, 1000, size=(4, 128)).astype("int64")
    pre, ref = _optimized(tmp_path, "fp16", ids, name="bert-large", num_hidden_layers=2, vocab_size=1024,
                          max_position_embeddings=128)
    got, _, _ = native_outputs(pre, {"input_ids": ids}, tmp_path, gpu=0, graph=True, warmup=1, repeat=2)
    for a, b in zip(got, ref):
        np.testing.assert_allclose(a, b, rtol=2e-2, atol=2e-2)
