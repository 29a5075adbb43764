"""Op cases on the OpTest harness (`tests/op_test.py`, modelled on the reference's
`unittests/test_*_op.py` pattern): numpy forward references + float64 finite-difference gradient
checks, for the normalisation / activation / loss ops and the long-tail API that has no HIP kernel.
The GPU variants (same cases, ``device="cuda"``, fp32/bf16 kernels vs these numpy references) are
in ``test_op_cases_gpu.py``."""
import math

import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
import paddle_infer_amd.nn.functional as F
from paddle_infer_amd import nn
from op_test import OpTest

rng = np.random.default_rng(0)


def _np_layer_norm(x, w, b, eps):
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    return (x - mu) / np.sqrt(var + eps) * w + b


class LayerNormCase(OpTest):
    op = staticmethod(lambda x, w, b, eps: F.layer_norm(x, x.shape[-1:], w, b, eps))

    def setup(self):
        x = rng.standard_normal((3, 8))
        w, b = rng.standard_normal(8), rng.standard_normal(8)
        self.inputs = {"x": x, "w": w, "b": b}
        self.attrs = {"eps": 1e-5}
        self.outputs = {"y": _np_layer_norm(x, w, b, 1e-5)}


class RMSNormCase(OpTest):
    op = staticmethod(lambda x, w, eps: F.rms_norm(x, w, eps))

    def setup(self):
        x, w = rng.standard_normal((4, 8)), rng.standard_normal(8)
        self.inputs = {"x": x, "w": w}
        self.attrs = {"eps": 1e-6}
        self.outputs = {"y": x / np.sqrt((x ** 2).mean(-1, keepdims=True) + 1e-6) * w}


class SoftmaxCase(OpTest):
    op = staticmethod(lambda x, axis: F.softmax(x, axis))

    def setup(self):
        x = rng.standard_normal((3, 8))
        e = np.exp(x - x.max(1, keepdims=True))
        self.inputs, self.attrs = {"x": x}, {"axis": 1}
        self.outputs = {"y": e / e.sum(1, keepdims=True)}


class GeluCase(OpTest):
    op = staticmethod(lambda x, approximate: F.gelu(x, approximate))

    def setup(self):
        from scipy.special import erf
        x = rng.standard_normal((4, 8))
        self.inputs, self.attrs = {"x": x}, {"approximate": False}
        self.outputs = {"y": 0.5 * x * (1 + erf(x / math.sqrt(2)))}


class CrossEntropyCase(OpTest):
    op = staticmethod(lambda logits, label: F.cross_entropy(logits, label, reduction="none"))

    def setup(self):
        logits = rng.standard_normal((5, 8))
        label = rng.integers(0, 8, (5,))
        lse = np.log(np.exp(logits).sum(1))
        self.inputs = {"logits": logits, "label": label}
        self.attrs = {}
        self.outputs = {"loss": (lse - logits[np.arange(5), label]).reshape(-1)}

    def check_output(self, **kw):  # loss may come back [N] or [N, 1]
        self.setup()
        got = self._run(self._tensors())[0].detach().reshape(-1).numpy()
        np.testing.assert_allclose(got, self.outputs["loss"], atol=1e-6, rtol=1e-6)


class HSigmoidCase(OpTest):
    op = staticmethod(lambda x, w, b, label, C: F.hsigmoid_loss(x, label, C, w, b))

    def setup(self):
        N, D, C = 4, 3, 6
        x, w, b = rng.standard_normal((N, D)), rng.standard_normal((C - 1, D)), rng.standard_normal((C - 1, 1))
        label = rng.integers(0, C, (N,))
        out = np.zeros((N, 1))
        L = int(math.ceil(math.log2(C)))
        for n in range(N):
            code = label[n] + C
            for k in range(L):
                node = (code >> (k + 1)) - 1
                if node < 0:
                    continue
                bit = (code >> k) & 1
                pre = x[n] @ w[node] + b[node, 0]
                out[n, 0] += np.log1p(np.exp(pre)) - bit * pre
        self.inputs = {"x": x, "w": w, "b": b, "label": label}
        self.attrs = {"C": C}
        self.outputs = {"loss": out}


class MarginCECase(OpTest):
    op = staticmethod(lambda logits, label: F.margin_cross_entropy(
        logits, label, 1.0, 0.5, 0.0, 64.0, reduction="none"))

    def setup(self):
        N, C = 4, 6
        logits = rng.uniform(-0.9, 0.9, (N, C))
        label = rng.integers(0, C, (N,))
        z = logits.copy()
        z[np.arange(N), label] = np.cos(np.arccos(logits[np.arange(N), label]) + 0.5)
        z *= 64.0
        lse = np.log(np.exp(z - z.max(1, keepdims=True)).sum(1)) + z.max(1)
        self.inputs = {"logits": logits, "label": label}
        self.outputs = {"loss": (lse - z[np.arange(N), label]).reshape(N, 1)}


class SoftMarginCase(OpTest):
    op = staticmethod(lambda x, y: F.soft_margin_loss(x, y, reduction="none"))

    def setup(self):
        x, y = rng.standard_normal((3, 4)), rng.choice([-1.0, 1.0], (3, 4))
        self.inputs = {"x": x, "y": y}
        self.outputs = {"l": np.log1p(np.exp(-y * x))}


class BilinearCase(OpTest):
    op = staticmethod(lambda a, b, w, bias: F.bilinear(a, b, w, bias))

    def setup(self):
        a, b = rng.standard_normal((3, 4)), rng.standard_normal((3, 5))
        w, bias = rng.standard_normal((2, 4, 5)), rng.standard_normal((1, 2))
        self.inputs = {"a": a, "b": b, "w": w, "bias": bias}
        self.outputs = {"y": np.einsum("ni,oij,nj->no", a, w, b) + bias}


class ChannelShuffleCase(OpTest):
    op = staticmethod(lambda x, groups: F.channel_shuffle(x, groups))

    def setup(self):
        x = rng.standard_normal((2, 6, 2, 2))
        self.inputs, self.attrs = {"x": x}, {"groups": 3}
        self.outputs = {"y": x.reshape(2, 3, 2, 2, 2).transpose(0, 2, 1, 3, 4).reshape(2, 6, 2, 2)}


class MultiplexCase(OpTest):
    op = staticmethod(lambda a, b, index: paddle.multiplex([a, b], index))

    def setup(self):
        a, b = rng.standard_normal((4, 3)), rng.standard_normal((4, 3))
        idx = np.array([[1], [0], [1], [0]], dtype=np.int32)
        self.inputs = {"a": a, "b": b, "index": idx}
        self.outputs = {"y": np.where(idx == 1, b, a)}


CASES = [LayerNormCase, RMSNormCase, SoftmaxCase, GeluCase, CrossEntropyCase, HSigmoidCase,
         MarginCECase, SoftMarginCase, BilinearCase, ChannelShuffleCase, MultiplexCase]
GRADS = {LayerNormCase: ["x", "w", "b"], RMSNormCase: ["x", "w"], SoftmaxCase: ["x"], GeluCase: ["x"],
         CrossEntropyCase: ["logits"], HSigmoidCase: ["x", "w", "b"], MarginCECase: ["logits"],
         SoftMarginCase: ["x"], BilinearCase: ["a", "b", "w"], MultiplexCase: ["a", "b"]}


@pytest.mark.parametrize("case", CASES, ids=lambda c: c.__name__)
def test_op_output(case):
    case().check_output(atol=1e-6, rtol=1e-6)


@pytest.mark.parametrize("case", list(GRADS), ids=lambda c: c.__name__)
def test_op_grad(case):
    case().check_grad(GRADS[case], max_relative_error=1e-4)


# ----------------------------------------------------------------------------- long-tail API
def test_fold_inverts_unfold_counts():
    x = torch.randn(1, 2, 4, 4, dtype=torch.float64)
    cols = F.unfold(x, [2, 2], 1, 0, 1)
    back = F.fold(cols, [4, 4], [2, 2])
    ones = F.fold(F.unfold(torch.ones_like(x), [2, 2], 1, 0, 1), [4, 4], [2, 2])
    torch.testing.assert_close(back / ones, x)
    assert nn.Fold([4, 4], [2, 2])(cols).shape == x.shape


def test_pixel_unshuffle_and_layers():
    x = torch.randn(1, 2, 4, 4)
    y = nn.PixelUnshuffle(2)(x)
    assert y.shape == (1, 8, 2, 2)
    torch.testing.assert_close(nn.PixelShuffle(2)(y), x)
    assert nn.ZeroPad2D([1, 2, 0, 1])(x).shape == (1, 2, 5, 7)
    sm = nn.Softmax2D()(x)
    torch.testing.assert_close(sm.sum(1), torch.ones(1, 4, 4))
    r = nn.RReLU(0.1, 0.3)
    r.eval()
    torch.testing.assert_close(r(torch.tensor([-1.0, 2.0])), torch.tensor([-0.2, 2.0]))


def test_max_unpool_roundtrip():
    x = torch.randn(1, 1, 4, 4)
    y, idx = torch.nn.functional.max_pool2d(x, 2, 2, return_indices=True)
    up = nn.MaxUnPool2D(2, 2)(y, idx)
    assert up.shape == x.shape and torch.equal(up.flatten()[idx.flatten()], y.flatten())


def test_conv3d_transpose_and_adaptive_max3d():
    m = nn.Conv3DTranspose(2, 3, 3, stride=2, padding=1)
    assert m(torch.randn(1, 2, 3, 3, 3)).shape == (1, 3, 5, 5, 5)
    assert nn.AdaptiveMaxPool3D(2)(torch.randn(1, 2, 4, 4, 4)).shape == (1, 2, 2, 2, 2)


def test_spectral_norm_unit_sigma():
    w = torch.randn(6, 4, dtype=torch.float32)
    sn = nn.SpectralNorm(list(w.shape), dim=0, power_iters=50)
    out = sn(w)
    assert abs(torch.linalg.matrix_norm(out, 2).item() - 1.0) < 1e-3


def test_initializers_dirac_gain():
    w = torch.empty(4, 2, 3, 3)
    nn.initializer.Dirac(groups=2)(w)
    x = torch.randn(1, 2, 5, 5)
    y = torch.nn.functional.conv2d(x, w, padding=1)
    torch.testing.assert_close(y[:, :2], x)
    torch.testing.assert_close(y[:, 2:], x)
    assert nn.initializer.calculate_gain("relu") == math.sqrt(2)
    assert math.isclose(nn.initializer.calculate_gain("leaky_relu", 0.2), math.sqrt(2 / 1.04))


def test_losses_layers():
    x, y = torch.randn(3, 4), (torch.rand(3, 4) > 0.5).float()
    l = nn.MultiLabelSoftMarginLoss()(x, y)
    ref = torch.nn.functional.multilabel_soft_margin_loss(x, y)
    torch.testing.assert_close(l, ref)
    a, p, n = torch.randn(3, 5), torch.randn(3, 5), torch.randn(3, 5)
    torch.testing.assert_close(nn.TripletMarginWithDistanceLoss(margin=0.5)(a, p, n),
                               torch.nn.functional.triplet_margin_with_distance_loss(a, p, n, margin=0.5))
    hs = nn.HSigmoidLoss(5, 6)
    assert hs(torch.randn(4, 5), torch.tensor([0, 1, 4, 5])).shape == (4, 1)


def test_class_center_sample():
    label = torch.tensor([3, 7, 3, 1])
    remapped, sampled = F.class_center_sample(label, 10, 6)
    assert sampled.numel() == 6 and set([1, 3, 7]) <= set(sampled.tolist())
    assert torch.equal(sampled[remapped], label)


def test_sparse_attention_full_pattern_equals_dense():
    B, H, S, D = 1, 2, 4, 8
    q, k, v = (torch.randn(B, H, S, D) for _ in range(3))
    off = torch.arange(0, S * S + 1, S).repeat(B, H, 1)
    cols = torch.arange(S).repeat(S).repeat(B, H, 1)
    out = F.sparse_attention(q, k, v, off, cols)
    ref = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(D), -1) @ v
    torch.testing.assert_close(out, ref)


def test_top_level_misc():
    assert paddle.iinfo(paddle.int32).max == 2 ** 31 - 1
    assert paddle.finfo("float16").eps > 0
    assert isinstance(paddle.float32, paddle.dtype)
    x = torch.tensor([1.0, float("nan"), 3.0, 2.0])
    assert paddle.nanmedian(x).item() == 2.0
    assert paddle.tril_indices(3, 3).shape == (2, 6)
    assert paddle.triu_indices(3).shape == (2, 6)
    assert paddle.reverse(torch.arange(3), 0).tolist() == [2, 1, 0]
    t = torch.zeros(3)
    paddle.index_add_(t, torch.tensor([0, 2]), 0, torch.tensor([1.0, 2.0]))
    assert t.tolist() == [1.0, 0.0, 2.0]
    assert paddle.tolist(torch.tensor([1, 2])) == [1, 2]
    torch.testing.assert_close(paddle.renorm(torch.ones(2, 4), 2, 0, 1.0).norm(dim=1), torch.ones(2))
    paddle.check_shape([2, -1, 3])
    with pytest.raises(ValueError):
        paddle.check_shape([2, -3])
    with paddle.LazyGuard():
        lin = torch.nn.Linear(4, 4)
    assert lin.weight.is_meta
    st = paddle.get_cuda_rng_state()
    paddle.set_cuda_rng_state(st)
    import paddle_infer_amd.linalg as LA
    a = torch.randn(3, 3, dtype=torch.float64)
    torch.testing.assert_close(LA.inv(a) @ a, torch.eye(3, dtype=torch.float64))
    P, L, U = LA.lu_unpack(*LA.lu(a))
    torch.testing.assert_close(P @ L @ U, a)
