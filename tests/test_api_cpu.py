"""Paddle-API parity on CPU: tensor semantics, layers, optimizers, schedulers, io, autograd."""
import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
import paddle_infer_amd.nn.functional as F


def test_tensor_semantics():
    x = paddle.to_tensor(np.arange(24, dtype=np.float32).reshape(2, 3, 4))
    assert paddle.reshape(x, [0, -1]).shape == (2, 12)
    assert paddle.transpose(x, [2, 0, 1]).shape == (4, 2, 3)
    assert [t.shape[1] for t in paddle.split(x, [1, -1], axis=1)] == [1, 2]
    v, i = paddle.topk(paddle.to_tensor([3.0, 1.0, 2.0]), 2)
    assert v.tolist() == [3.0, 2.0] and i.tolist() == [0, 2]
    assert paddle.sum(x, axis=[0, 2]).tolist() == x.numpy().sum((0, 2)).tolist()
    assert paddle.max(x, axis=1).shape == (2, 4)
    assert paddle.arange(5).dtype == torch.int64
    assert paddle.ones([2, 3]).dtype == torch.float32
    g = paddle.gather(x, paddle.to_tensor([1, 0]), axis=0)
    assert torch.equal(g[0], x[1])
    nd = paddle.gather_nd(x, paddle.to_tensor([[0, 1], [1, 2]]))
    assert torch.equal(nd[1], x[1, 2])
    s = paddle.scatter(paddle.zeros([3, 2]), paddle.to_tensor([2, 0]), paddle.ones([2, 2]))
    assert s[2].tolist() == [1.0, 1.0] and s[1].tolist() == [0.0, 0.0]
    assert paddle.slice(x, [1, 2], [0, 1], [2, 3]).shape == (2, 2, 2)
    assert paddle.unsqueeze(paddle.ones([3]), [0, 2]).shape == (1, 3, 1)
    assert paddle.matmul(paddle.ones([2, 3]), paddle.ones([2, 3]), transpose_y=True).shape == (2, 2)
    assert paddle.expand(paddle.ones([1, 3]), [4, -1]).shape == (4, 3)
    assert paddle.cast(x, "int32").dtype == torch.int32
    assert paddle.linalg.norm(paddle.ones([3, 4])).item() == pytest.approx(np.sqrt(12))


def test_layers_and_state_dict():
    m = paddle.nn.Sequential(paddle.nn.Conv2D(3, 4, 3, padding=1), paddle.nn.BatchNorm2D(4),
                             paddle.nn.ReLU(), paddle.nn.AdaptiveAvgPool2D(1), paddle.nn.Flatten(),
                             paddle.nn.Linear(4, 2))
    sd = m.state_dict()
    assert "1._mean" in sd and "1._variance" in sd and sd["5.weight"].shape == (4, 2)
    y = m(paddle.randn([2, 3, 8, 8]))
    assert y.shape == (2, 2)
    m2 = paddle.nn.Sequential(paddle.nn.Conv2D(3, 4, 3, padding=1), paddle.nn.BatchNorm2D(4),
                              paddle.nn.ReLU(), paddle.nn.AdaptiveAvgPool2D(1), paddle.nn.Flatten(),
                              paddle.nn.Linear(4, 2))
    m2.set_state_dict(sd)
    m.eval(), m2.eval()
    x = paddle.randn([2, 3, 8, 8])
    assert torch.allclose(m(x), m2(x))


def test_batchnorm_momentum_semantics():
    bn = paddle.nn.BatchNorm1D(3, momentum=0.9)
    x = paddle.randn([16, 3]) + 5
    bn(x)
    expect = 0.9 * 0 + 0.1 * x.mean(0)
    assert torch.allclose(bn._mean, expect, atol=1e-5)


def test_cross_entropy_and_losses():
    logits = paddle.randn([6, 5])
    lab = paddle.to_tensor([0, 1, 2, 3, 4, -100])
    a = F.cross_entropy(logits, lab, ignore_index=-100)
    b = torch.nn.functional.cross_entropy(logits, lab, ignore_index=-100)
    assert a.item() == pytest.approx(b.item(), rel=1e-5)
    soft = torch.softmax(paddle.randn([6, 5]), -1)
    c = F.cross_entropy(logits, soft, soft_label=True)
    d = -(soft * torch.log_softmax(logits, -1)).sum(-1).mean()
    assert c.item() == pytest.approx(d.item(), rel=1e-5)


@pytest.mark.parametrize("name", ["SGD", "Momentum", "Adam", "AdamW", "Adagrad", "RMSProp", "Lamb", "Adamax", "Adadelta"])
def test_optimizers_decrease_loss(name):
    torch.manual_seed(0)
    m = paddle.nn.Linear(8, 1)
    cls = getattr(paddle.optimizer, name)
    kw = {"learning_rate": 0.05, "parameters": m.parameters()}
    o = cls(**kw)
    x = paddle.randn([64, 8])
    y = x @ torch.randn(8, 1)
    l0 = None
    for _ in range(30):
        loss = ((m(x) - y) ** 2).mean()
        l0 = l0 if l0 is not None else loss.item()
        loss.backward()
        o.step()
        o.clear_grad()
    assert loss.item() < l0


def test_adamw_matches_reference_math():
    p0 = torch.randn(10)
    g = torch.randn(10)
    p = torch.nn.Parameter(p0.clone())
    o = paddle.optimizer.AdamW(learning_rate=0.01, parameters=[p], weight_decay=0.1, beta1=0.9, beta2=0.99)
    p.grad = g.clone()
    o.step()
    ref = p0 * (1 - 0.01 * 0.1)
    m = 0.1 * g
    v = 0.01 * g * g
    lr_t = 0.01 * np.sqrt(1 - 0.99) / (1 - 0.9)
    ref = ref - lr_t * m / (v.sqrt() + 1e-8 * np.sqrt(1 - 0.99))
    assert torch.allclose(p.detach(), ref, atol=1e-6)


def test_lr_schedulers():
    s = paddle.optimizer.lr.LinearWarmup(0.1, 5, 0.0, 0.1)
    vals = []
    for _ in range(7):
        vals.append(s())
        s.step()
    assert vals[0] == 0.0 and vals[5] == pytest.approx(0.1)
    c = paddle.optimizer.lr.CosineAnnealingDecay(1.0, 10)
    for _ in range(10):
        c.step()
    assert c() == pytest.approx(0.0, abs=1e-9)
    p = paddle.optimizer.lr.PiecewiseDecay([2, 4], [1.0, 0.5, 0.1])
    out = []
    for _ in range(5):
        out.append(p())
        p.step()
    assert out == [1.0, 1.0, 0.5, 0.5, 0.1]


def test_save_load_roundtrip(tmp_path):
    sd = {"a": torch.randn(3, 4), "b": torch.randn(5).bfloat16(), "n": {"c": torch.arange(3)}, "s": 7}
    paddle.save(sd, str(tmp_path / "x.pdparams"))
    back = paddle.load(str(tmp_path / "x.pdparams"))
    assert torch.equal(back["a"], sd["a"]) and back["b"].dtype == torch.bfloat16
    assert torch.equal(back["b"], sd["b"]) and back["s"] == 7 and torch.equal(back["n"]["c"], sd["n"]["c"])


def test_restricted_loader_refuses_code(tmp_path):
    import pickle
    import os

    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))
    with open(tmp_path / "evil.pdparams", "wb") as f:
        pickle.dump({"x": Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        paddle.load(str(tmp_path / "evil.pdparams"))


def test_pylayer_and_grad():
    class Cube(paddle.autograd.PyLayer):
        @staticmethod
        def forward(ctx, x):
            ctx.save_for_backward(x)
            return x ** 3

        @staticmethod
        def backward(ctx, dy):
            (x,) = ctx.saved_tensor()
            return 3 * x ** 2 * dy
    x = paddle.to_tensor([2.0], stop_gradient=False)
    y = Cube.apply(x)
    (g,) = paddle.grad(y, x)
    assert g.item() == pytest.approx(12.0)


def test_dataloader_and_distributed_sampler():
    ds = paddle.io.TensorDataset([torch.arange(10).float(), torch.arange(10)])
    dl = paddle.io.DataLoader(ds, batch_size=4, shuffle=False, drop_last=False)
    batches = list(dl)
    assert len(batches) == 3 and batches[0][1].tolist() == [0, 1, 2, 3]
    s0 = list(paddle.io.DistributedBatchSampler(ds, 2, num_replicas=2, rank=0))
    s1 = list(paddle.io.DistributedBatchSampler(ds, 2, num_replicas=2, rank=1))
    flat = sorted(i for b in s0 + s1 for i in b)
    assert flat == list(range(10))


def test_grad_scaler():
    m = paddle.nn.Linear(2, 1)
    o = paddle.optimizer.SGD(learning_rate=0.1, parameters=m.parameters())
    sc = paddle.amp.GradScaler(init_loss_scaling=1024.0)
    loss = m(paddle.ones([1, 2])).sum()
    sc.scale(loss).backward()
    w0 = m.weight.detach().clone()
    sc.minimize(o, loss)
    assert torch.allclose(m.weight, w0 - 0.1 * torch.ones_like(w0), atol=1e-6)
