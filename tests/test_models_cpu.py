"""Model-family tests (CPU): BERT padding-mask invariance + trains; GPT tiny trains.
Parity model: reference `unittests/test_imperative_bert*.py` / bert_dygraph_model tests."""
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd.models import BertForPretraining, BertModel, bert_config


def test_bert_padding_invariance():
    paddle.seed(0)
    cfg = bert_config("bert-tiny", hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    m = BertModel(cfg).eval()
    ids = torch.randint(1, 1024, (1, 10))
    padded = torch.cat([ids, torch.zeros(1, 6, dtype=torch.long)], 1)
    a, _ = m(ids)
    b, _ = m(padded)
    torch.testing.assert_close(b[:, :10], a, rtol=1e-4, atol=1e-4)


def test_bert_pretraining_loss_decreases():
    paddle.seed(1)
    cfg = bert_config("bert-tiny", hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    m = BertForPretraining(cfg)
    opt = paddle.optimizer.AdamW(learning_rate=1e-3, parameters=m.parameters())
    ids = torch.randint(1, 1024, (4, 16))
    lab = torch.full((4, 16), -1)
    lab[:, 2], lab[:, 7] = ids[:, 2], ids[:, 7]
    nsp = torch.tensor([0, 1, 0, 1])
    losses = []
    for _ in range(20):
        loss = m(ids, masked_lm_labels=lab, next_sentence_labels=nsp)
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    assert losses[-1] < 0.5 * losses[0]


def test_gpt_recompute_with_dropout_matches_plain():
    """Layer recompute re-runs each decoder layer in backward; with hidden dropout > 0 the re-run
    must draw the forward's masks (fleet recompute restores the torch AND kernel-dropout RNG), so
    gradients equal the non-recomputed model's for a fixed seed."""
    import torch
    from paddle_infer_amd.framework import random as prand
    from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config

    def grads(recompute):
        prand.seed(7)
        cfg = gpt_config("gpt3-tiny", hidden_dropout_prob=0.1, recompute=recompute, dtype="float32")
        torch.manual_seed(0)
        m = GPTForPretraining(cfg)
        m.train()
        ids = torch.randint(0, cfg.vocab_size, (2, 17), generator=torch.Generator().manual_seed(1))
        prand.seed(11)
        loss = m(ids[:, :-1], labels=ids[:, 1:])
        loss.backward()
        return loss.detach(), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}

    l0, g0 = grads(False)
    l1, g1 = grads(True)
    assert torch.allclose(l0, l1)
    assert g0.keys() == g1.keys() and len(g0) > 10
    for n in g0:
        assert torch.allclose(g0[n], g1[n], atol=1e-6, rtol=1e-5), n
