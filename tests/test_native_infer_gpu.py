"""Native C++ predictor on the MI355X (`pd_infer_run --gpu 0`: HIP kernels + rocBLAS, no Python
in the process) against the Python Predictor on the CPU."""
import os

import numpy as np
import pytest

from native_infer_util import MLP, RUN, Encoder, export, native_outputs, python_outputs

from paddle_infer_amd.static import InputSpec

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not os.path.exists(RUN), reason="native engine not built")]


@pytest.mark.parametrize("E,B", [(32, 2), (256, 8)])
def test_native_gpu_encoder(tmp_path, E, B):
    path = str(tmp_path / "enc")
    export(Encoder(V=1000, E=E), path, [InputSpec([None, 64], "int64", "ids")])
    ids = np.random.RandomState(E).randint(0, 1000, size=(B, 64)).astype("int64")
    ref = python_outputs(path, {"ids": ids})
    got, ms, _ = native_outputs(path, {"ids": ids}, tmp_path, gpu=0, repeat=5)
    np.testing.assert_allclose(got[0], ref[0], rtol=2e-3, atol=2e-4)
    assert ms is not None and ms > 0


def test_native_gpu_mlp(tmp_path):
    path = str(tmp_path / "mlp")
    export(MLP(), path, [InputSpec([None, 16], "float32", "x")])
    x = np.random.RandomState(1).randn(33, 16).astype("float32")
    ref = python_outputs(path, {"x": x})
    got, _, _ = native_outputs(path, {"x": x}, tmp_path, gpu=0)
    for a, b in zip(got, ref):
        np.testing.assert_allclose(a, b, rtol=2e-3, atol=2e-4)


@pytest.mark.parametrize("arch", ["small_cnn", "mobilenet_v2", "resnet18"])
def test_native_gpu_cnn(tmp_path, arch):
    """conv2d (im2col + rocBLAS, depthwise HIP kernel), batch_norm, pool2d, relu6 / hard_swish on
    the GPU engine vs the Python predictor."""
    import torch
    from native_infer_util import SmallCNN
    from paddle_infer_amd.vision import models as VM
    torch.manual_seed(0)
    m = SmallCNN() if arch == "small_cnn" else getattr(VM, arch)(num_classes=10)
    path = str(tmp_path / arch)
    export(m, path, [InputSpec([None, 3, 64, 64], "float32", "x")])
    x = np.random.RandomState(3).randn(2, 3, 64, 64).astype("float32")
    ref = python_outputs(path, {"x": x})
    got, ms, _ = native_outputs(path, {"x": x}, tmp_path, gpu=0, repeat=3)
    np.testing.assert_allclose(got[0], ref[0], rtol=2e-3, atol=2e-3)
    assert ms is not None and ms > 0
