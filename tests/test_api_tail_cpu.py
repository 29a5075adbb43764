"""The long tail closing the reference ``__all__`` diff (tools/api_diff.py → 0 missing):
static.nn control-flow / layer / LoD-sequence builders, static EMA / auc / exponential_decay,
distributed InMemoryDataset + MultiSlot data generator, fleet Fleet / UtilBase / Role, vision
affine / perspective transforms and GoogLeNet / InceptionV3."""
import math
import os

import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import static
from paddle_infer_amd.static import nn as snn


def test_case_and_switch_case_eager():
    x = torch.tensor(3.0)
    assert snn.case([(x > 5, lambda: 1), (x > 2, lambda: 2)], lambda: 3) == 2
    assert snn.case([(x > 5, lambda: 1)], lambda: 3) == 3
    assert snn.switch_case(torch.tensor(1), {0: lambda: "a", 1: lambda: "b"}, lambda: "z") == "b"
    assert snn.switch_case(torch.tensor(7), [lambda: "a", lambda: "b"], lambda: "z") == "z"


def _lod(data, lens):
    return static.create_lod_tensor(torch.as_tensor(data, dtype=torch.float32), [lens])


def test_sequence_ops():
    x = _lod(np.arange(12, dtype=np.float32).reshape(6, 2), [2, 3, 1])
    assert torch.equal(snn.sequence_pool(x, "sum"), torch.tensor([[2., 4.], [18., 21.], [10., 11.]]))
    assert torch.equal(snn.sequence_last_step(x), torch.tensor([[2., 3.], [8., 9.], [10., 11.]]))
    assert torch.equal(snn.sequence_first_step(x)[1], torch.tensor([4., 5.]))
    r = snn.sequence_reverse(x)
    assert torch.equal(r[:2], x[:2].flip(0)) and r.lod == x.lod
    p, lens = snn.sequence_pad(x, torch.tensor([0.0]))
    assert p.shape == (3, 3, 2) and lens.tolist() == [2, 3, 1]
    u = snn.sequence_unpad(p, lens)
    assert torch.equal(u, x) and u.lod == x.lod
    s = snn.sequence_softmax(_lod([[1.], [2.], [3.]], [1, 2]))
    assert torch.allclose(s.reshape(-1)[1:].sum(), torch.tensor(1.0))
    c = snn.sequence_concat([x, x])
    assert c.lod == [[0, 4, 10, 12]]
    sl = snn.sequence_slice(x, torch.tensor([0, 1, 0]), torch.tensor([1, 2, 1]))
    assert sl.lod == [[0, 1, 3, 4]] and torch.equal(sl[1], x[3])
    e = snn.sequence_enumerate(_lod([[1.], [2.], [3.]], [3]), 2)
    assert e.tolist() == [[1., 2.], [2., 3.], [3., 0.]]
    ex = snn.sequence_expand_as(torch.tensor([[1.], [2.]]), _lod(np.zeros((3, 1)), [1, 2]))
    assert ex.reshape(-1).tolist() == [1., 2., 2.]
    torch.manual_seed(0)
    conv = snn.sequence_conv(x, 4, 3)
    assert conv.shape == (6, 4) and conv.lod == x.lod


def test_row_conv_nce_spectral_crf_data_norm():
    torch.manual_seed(0)
    x = torch.randn(2, 5, 3)
    assert snn.row_conv(x, 2).shape == (2, 5, 3)
    cost = snn.nce(torch.randn(4, 8), torch.tensor([[1], [2], [3], [0]]), 10, num_neg_samples=5)
    assert cost.shape == (4, 1) and torch.isfinite(cost).all() and (cost > 0).all()
    w = torch.randn(6, 4)
    wn = snn.spectral_norm(w, power_iters=30)
    assert abs(torch.linalg.matrix_norm(wn, 2).item() - 1.0) < 1e-3
    em = torch.randn(2, 4, 3)
    trans = torch.randn(5, 3)
    path = snn.crf_decoding(em, trans, length=torch.tensor([4, 2]))
    assert path.shape[0] == 2
    y = snn.data_norm(torch.randn(8, 3))
    assert y.shape == (8, 3)
    out = snn.bilinear_tensor_product(torch.randn(2, 3), torch.randn(2, 4), 5)
    assert out.shape == (2, 5)
    locs, confs, boxes, var = snn.multi_box_head(
        [torch.randn(1, 8, 4, 4), torch.randn(1, 8, 2, 2)], torch.randn(1, 3, 32, 32), 32, 3,
        [[2.0], [2.0]], min_sizes=[8.0, 16.0], max_sizes=[16.0, 24.0])
    assert locs.shape[1] == boxes.shape[0] == confs.shape[1] and var.shape == boxes.shape


def test_static_ema_auc_exponential_decay():
    from sklearn.metrics import roc_auc_score
    rs = np.random.RandomState(0)
    p = rs.rand(200)
    y = (rs.rand(200) < p).astype(np.int64)
    g, b, stats = static.auc(torch.tensor(np.stack([1 - p, p], 1)), torch.tensor(y).reshape(-1, 1))
    assert abs(float(b) - roc_auc_score(y, p)) < 2e-3
    sched = static.exponential_decay(0.1, 10, 0.5, staircase=True)
    for _ in range(10):
        sched.step()
    assert math.isclose(sched(), 0.05)
    paddle.enable_static()
    try:
        torch.manual_seed(0)
        main, startup = static.Program(), static.Program()
        with static.program_guard(main, startup):
            x = static.data("x", [None, 4], "float32")
            loss = paddle.mean(static.nn.fc(x, 1) ** 2)
            paddle.optimizer.SGD(learning_rate=0.1).minimize(loss)
            ema = static.ExponentialMovingAverage(0.9)
            ema.update()
        exe = static.Executor("cpu")
        scope = static.Scope()
        with static.scope_guard(scope):
            rs = np.random.RandomState(0)
            for _ in range(5):
                exe.run(main, feed={"x": rs.randn(2, 4).astype("float32")}, fetch_list=[loss])
            assert ema._step == 5 and ema._ema
            changed = 0
            for name in ema._ema:
                cur = scope.get(name).detach().clone()
                with ema.apply(exe):
                    avg = scope.get(name).detach().clone()
                assert torch.equal(scope.get(name).detach(), cur)  # restored
                changed += int(not torch.equal(avg, cur))
            assert changed > 0
    finally:
        paddle.disable_static()


def test_inmemory_dataset_and_data_generator(tmp_path):
    from paddle_infer_amd.distributed import fleet

    class Gen(fleet.MultiSlotDataGenerator):
        def generate_sample(self, line):
            def it():
                vals = [int(v) for v in line.split()]
                yield [("ids", vals), ("label", [vals[0] % 2])]
            return it

    text = Gen().run_from_memory(["1 2 3", "4 5", "6"])
    assert text.splitlines()[0] == "3 1 2 3 1 1"
    f = tmp_path / "part-0"
    f.write_text(text)
    ds = paddle.distributed.InMemoryDataset()
    ds.init(batch_size=2, thread_num=2, use_var=["ids", "label"], pipe_command="cat")
    ds.set_filelist([str(f)])
    ds.load_into_memory()
    assert ds.get_memory_data_size() == 3
    batches = list(ds)
    assert batches[0]["ids"].lod == [[0, 3, 5]] and batches[0]["label"].shape == (2, 1)
    qd = paddle.distributed.QueueDataset()
    qd.init(batch_size=3, use_var=["ids", "label"])
    qd.set_filelist([str(f)])
    assert sum(b["label"].shape[0] for b in qd) == 3
    assert paddle.distributed.CountFilterEntry(5)._to_attr() == "count_filter_entry:5"
    assert fleet.Role.SERVER == 2 and fleet.util.get_file_shard(["a", "b", "c"]) == ["a", "b", "c"]
    assert fleet.Fleet().worker_num() == 1


def test_vision_affine_perspective_and_models():
    from paddle_infer_amd.vision import models as M, transforms as T
    img = (np.random.RandomState(0).rand(20, 24, 3) * 255).astype(np.uint8)
    assert (T.affine(img, 0, (0, 0), 1.0, 0) == img).all()
    assert (T.affine(img, 0, (2, 0), 1.0, 0)[:, 2:] == img[:, :-2]).all()
    rot = T.affine(img, 90, (0, 0), 1.0, 0)
    assert rot.shape == img.shape
    pts = [(0, 0), (23, 0), (23, 19), (0, 19)]
    assert (T.perspective(img, pts, pts) == img).all()
    assert T.RandomPerspective(1.0)(img).shape == img.shape
    with torch.no_grad():
        out, a1, a2 = M.googlenet(num_classes=7).eval()(torch.randn(1, 3, 224, 224))
        assert out.shape == a1.shape == a2.shape == (1, 7)
        assert M.inception_v3(num_classes=5).eval()(torch.randn(1, 3, 299, 299)).shape == (1, 5)
        assert M.shufflenet_v2_swish(num_classes=3).eval()(torch.randn(1, 3, 64, 64)).shape == (1, 3)


def test_api_diff_is_empty():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "api_diff.py")], cwd=root,
                       capture_output=True, text=True, env={**os.environ, "PYTHONPATH": root},
                       timeout=300)
    assert r.stdout.strip().endswith("total missing: 0"), r.stdout[-2000:]
