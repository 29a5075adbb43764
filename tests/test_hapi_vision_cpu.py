"""hapi Model / metrics / callbacks / vision models + transforms (CPU).
Parity model: reference `unittests/test_model.py` (fit/evaluate/predict/save/load on LeNet),
`test_metrics.py`, `test_callbacks.py`, `test_vision_models.py`, `test_transforms.py`."""
import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import metric, nn, vision
from paddle_infer_amd.vision import transforms as T


class _Blobs(paddle.io.Dataset):
    """Linearly separable 2-class images."""

    def __init__(self, n=64):
        rng = np.random.RandomState(0)
        self.y = rng.randint(0, 2, n).astype(np.int64)
        self.x = (rng.randn(n, 1, 28, 28) * 0.1 + self.y[:, None, None, None]).astype(np.float32)

    def __getitem__(self, i):
        return self.x[i], self.y[i:i + 1]

    def __len__(self):
        return len(self.y)


def test_model_fit_evaluate_predict_save_load(tmp_path):
    paddle.seed(0)
    net = vision.LeNet(num_classes=2)
    model = paddle.Model(net)
    opt = paddle.optimizer.Adam(learning_rate=1e-3, parameters=net.parameters())
    model.prepare(opt, nn.CrossEntropyLoss(), metric.Accuracy())
    ds = _Blobs()
    model.fit(ds, ds, batch_size=16, epochs=3, verbose=0, save_dir=str(tmp_path / "ckpt"))
    res = model.evaluate(ds, batch_size=16, verbose=0)
    assert res["acc"] > 0.9
    preds = model.predict(ds, batch_size=16, stack_outputs=True)
    assert preds[0].shape == (64, 2)
    model.save(str(tmp_path / "m"))
    net2 = vision.LeNet(num_classes=2)
    m2 = paddle.Model(net2)
    m2.prepare(paddle.optimizer.Adam(parameters=net2.parameters()), nn.CrossEntropyLoss(), metric.Accuracy())
    m2.load(str(tmp_path / "m"))
    np.testing.assert_allclose(m2.predict(ds, batch_size=64, stack_outputs=True)[0], preds[0], rtol=1e-5, atol=1e-5)


def test_early_stopping_stops():
    net = vision.LeNet(num_classes=2)
    model = paddle.Model(net)
    model.prepare(paddle.optimizer.SGD(learning_rate=0.0, parameters=net.parameters()), nn.CrossEntropyLoss())
    es = paddle.callbacks.EarlyStopping(monitor="loss", patience=0, save_best_model=False)
    ds = _Blobs(16)
    model.fit(ds, ds, batch_size=8, epochs=10, verbose=0, callbacks=[es])
    assert model.stop_training


def test_metrics():
    acc = metric.Accuracy(topk=(1, 2))
    pred = torch.tensor([[0.1, 0.7, 0.2], [0.5, 0.3, 0.2]])
    lab = torch.tensor([[2], [0]])
    acc.update(acc.compute(pred, lab))
    top1, top2 = acc.accumulate()
    assert top1 == 0.5 and top2 == 1.0
    p, r, auc = metric.Precision(), metric.Recall(), metric.Auc()
    preds = np.array([0.9, 0.8, 0.3, 0.1])
    labels = np.array([1, 0, 1, 0])
    p.update(preds, labels)
    r.update(preds, labels)
    auc.update(np.stack([1 - preds, preds], 1), labels)
    assert p.accumulate() == 0.5 and r.accumulate() == 0.5
    assert auc.accumulate() == pytest.approx(0.75, abs=1e-3)
    assert float(metric.accuracy(pred, lab.reshape(-1), k=2)) == 1.0


@pytest.mark.parametrize("ctor,shape", [
    (vision.resnet18, (1, 3, 64, 64)), (vision.resnet50, (1, 3, 64, 64)),
    (vision.mobilenet_v2, (1, 3, 64, 64)), (vision.mobilenet_v3_small, (1, 3, 64, 64)),
    (vision.vgg11, (1, 3, 32, 32)), (vision.squeezenet1_1, (1, 3, 64, 64)),
    (vision.shufflenet_v2_x1_0, (1, 3, 64, 64)), (vision.densenet121, (1, 3, 64, 64)),
    (vision.mobilenet_v1, (1, 3, 64, 64)), (vision.alexnet, (1, 3, 96, 96))])
def test_vision_models_forward(ctor, shape):
    net = ctor(num_classes=7)
    net.eval()
    with torch.no_grad():
        y = net(torch.randn(*shape))
    assert y.shape == (1, 7)


def test_transforms_pipeline():
    img = (np.random.RandomState(0).rand(40, 50, 3) * 255).astype(np.uint8)
    tf = T.Compose([T.Resize(32), T.CenterCrop(28), T.RandomHorizontalFlip(0.5),
                    T.ColorJitter(0.2, 0.2, 0.2, 0.05), T.ToTensor(),
                    T.Normalize([0.5] * 3, [0.5] * 3)])
    out = tf(img)
    assert out.shape == (3, 28, 28) and out.dtype == torch.float32
    rc = T.RandomResizedCrop(16)(img)
    assert rc.shape[:2] == (16, 16)
    pad = T.Pad(2)(img)
    assert pad.shape == (44, 54, 3)
    fake = vision.datasets.FakeData(4, (3, 8, 8), 3)
    x, y = fake[1]
    assert x.shape == (3, 8, 8) and 0 <= y < 3


def test_vision_ops_nms():
    boxes = torch.tensor([[0, 0, 10, 10], [1, 1, 10, 10], [20, 20, 30, 30]], dtype=torch.float32)
    scores = torch.tensor([0.9, 0.8, 0.7])
    keep = vision.ops.nms(boxes, 0.5, scores)
    assert keep.tolist() == [0, 2]
