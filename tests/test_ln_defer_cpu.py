"""ln_defer_pass (inference/passes.py): marks exactly the post-LN fc+LN producers whose outputs feed
only fold-aware consumers; on the CPU (no deferral at run time) the Predictor output is unchanged
and a deferred tensor materialises to the LayerNorm it owes."""
import os
import tempfile

import numpy as np
import torch
import torch.nn.functional as F


def test_ln_defer_pass_marks_bert_producers():
    from paddle_infer_amd import inference as pinf, jit
    from paddle_infer_amd.models.bert import BertModel, bert_config
    from paddle_infer_amd.static import InputSpec
    torch.manual_seed(0)
    cfg = bert_config("bert-large", num_hidden_layers=2, hidden_size=128, num_attention_heads=2,
                      intermediate_size=512, vocab_size=1000)
    m = BertModel(cfg)
    m.eval()
    d = tempfile.mkdtemp()
    st = jit.to_static(m, input_spec=[InputSpec([None, 16], "int64", "input_ids")])
    jit.save(st, os.path.join(d, "model"))
    c = pinf.Config(os.path.join(d, "model.pdmodel"), os.path.join(d, "model.pdiparams"))
    pred = pinf.create_predictor(c)
    assert pred.pass_stats.get("ln_defer_pass") == 3
    ops = [o for o in pred.program.global_block().ops if o.type == "fused_fc_elementwise_layernorm"]
    assert [bool(o.attrs.get("defer_ln")) for o in ops] == [True, True, True, False]
    ids = torch.randint(0, 1000, (2, 16))
    pred.get_input_handle(pred.get_input_names()[0]).copy_from_cpu(ids.numpy())
    pred.run()
    out = pred.get_output_handle(pred.get_output_names()[0]).copy_to_cpu()
    ref = m(ids)
    ref = ref[0] if isinstance(ref, (tuple, list)) else ref
    np.testing.assert_allclose(out, ref.detach().numpy(), atol=1e-4, rtol=1e-4)


def test_deferred_materialize_and_resid_args():
    from paddle_infer_amd.inference import ln_defer
    torch.manual_seed(1)
    h = torch.randn(4, 64)
    g, b = torch.rand(64) + 0.5, torch.randn(64)
    ln_defer.defer(h, g, b, 1e-5)
    assert ln_defer.of(h) is not None
    y = ln_defer.materialize(h)
    torch.testing.assert_close(y, F.layer_norm(h, (64,), g, b, 1e-5), atol=1e-5, rtol=1e-5)
    assert ln_defer.materialize(h) is y  # computed once
    r, rln = ln_defer.resid_args(h, 4)  # no folding GEMM filled the statistics: materialised
    assert rln is None and r is y
    assert not ln_defer.can_defer(h, 4, 64)  # CPU rows never stay raw


def _ref_small_gemm(a, b, out=None, out_f32=False, alpha=1.0, bias=None, act="none", resid=None, cfg=None,
                    slices=False, ln=None, ln_stats=None, resid_ln=None):
    """fp32 reference of ops.gemm.small_gemm's contract (LN fold, statistics out, LN'd residual)."""
    a, b = a.float(), b.float()
    if ln is not None:
        c1, b2, eps = ln
        mean = a.mean(1)
        rstd = torch.rsqrt((a * a).mean(1) - mean * mean + eps)
        y = rstd[:, None] * (a @ b.t() - mean[:, None] * c1[None]) + b2[None]
        if ln_stats is not None:
            ln_stats[:, 0], ln_stats[:, 1] = mean, rstd
    else:
        y = alpha * (a @ b.t()) + (bias.float() if bias is not None else 0)
    y = {"none": y, "gelu": F.gelu(y), "relu": torch.relu(y)}[act]
    if resid is not None:
        r = resid.float()
        if resid_ln is not None:
            st, g, be = resid_ln
            r = (r - st[:, :1]) * st[:, 1:] * g.float() + be.float()
        y = y + r
    return y


def test_ln_defer_dataflow_simulated(monkeypatch):
    """The deferral's data flow on the CPU: producers stay raw, the QKV / FFN1 GEMMs fold the owed
    LayerNorm and publish statistics, the residual epilogues apply it — with an fp32 reference
    standing in for the skinny kernel the Predictor output matches the plain path."""
    from paddle_infer_amd import inference as pinf, jit
    from paddle_infer_amd.inference import ln_defer
    from paddle_infer_amd.models.bert import BertModel, bert_config
    from paddle_infer_amd.ops import gemm as G, linear as L
    from paddle_infer_amd.static import InputSpec
    torch.manual_seed(0)
    cfg = bert_config("bert-large", num_hidden_layers=2, hidden_size=128, num_attention_heads=2,
                      intermediate_size=512, vocab_size=1000)
    m = BertModel(cfg)
    m.eval()
    d = tempfile.mkdtemp()
    st = jit.to_static(m, input_spec=[InputSpec([None, 16], "int64", "input_ids")])
    jit.save(st, os.path.join(d, "model"))
    ids = torch.randint(0, 1000, (2, 16))

    def run():
        c = pinf.Config(os.path.join(d, "model.pdmodel"), os.path.join(d, "model.pdiparams"))
        pred = pinf.create_predictor(c)
        pred.get_input_handle(pred.get_input_names()[0]).copy_from_cpu(ids.numpy())
        pred.run()
        return pred.get_output_handle(pred.get_output_names()[0]).copy_to_cpu()

    plain = run()
    folds = []
    orig_linear = ln_defer.linear

    def spy(*a, **k):
        y = orig_linear(*a, **k)
        folds.append(y is not None)
        return y
    monkeypatch.setattr(ln_defer, "can_defer", lambda x2, M, N: True)
    monkeypatch.setattr(ln_defer, "linear", spy)
    monkeypatch.setattr(G, "small_gemm", _ref_small_gemm)
    monkeypatch.setattr(L, "transposed", lambda w: w.t().contiguous())
    deferred = run()
    assert folds == [True] * 3  # FFN1 of layer 0, QKV + FFN1 of layer 1
    np.testing.assert_allclose(deferred, plain, atol=2e-4, rtol=2e-4)
