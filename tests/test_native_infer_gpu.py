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


def test_native_gpu_cnn_hip_graph(tmp_path):
    """conv + batch_norm under hipGraph capture: the BN fold is computed once on the eager warm-up
    and kept on the device, so the captured Runs match the eager ones (a capture that cannot
    proceed would fall back to eager for that feed signature instead of failing every Run)."""
    import torch
    from native_infer_util import SmallCNN
    torch.manual_seed(0)
    path = str(tmp_path / "cnn")
    export(SmallCNN(), path, [InputSpec([None, 3, 64, 64], "float32", "x")])
    x = np.random.RandomState(3).randn(2, 3, 64, 64).astype("float32")
    ref = python_outputs(path, {"x": x})
    got, ms, _ = native_outputs(path, {"x": x}, tmp_path, gpu=0, repeat=4, graph=True)
    np.testing.assert_allclose(got[0], ref[0], rtol=2e-3, atol=2e-3)


def test_native_graph_share_external_data_new_pointer(tmp_path):
    """ShareExternalData + hipGraph: a feed shared from a NEW device pointer (the old buffer freed)
    re-captures instead of copying into the old address; results follow the current buffer."""
    import torch
    import native_capi as nc
    path = str(tmp_path / "mlp")
    export(MLP(), path, [InputSpec([None, 16], "float32", "x")])
    xs = [np.random.RandomState(i).randn(8, 16).astype("float32") for i in range(3)]
    refs = [python_outputs(path, {"x": x}) for x in xs]
    p = nc.Predictor(path, gpu=0, hip_graph=True)
    try:
        for i, x in enumerate(xs):
            t = torch.from_numpy(x).cuda()
            torch.cuda.synchronize()
            p.share("x", t)
            p.run()
            p.run()  # second Run: graph replay on the same pointer
            got = p.fetch_float(p_out_name(path, 0), refs[i][0].shape)
            np.testing.assert_allclose(got, refs[i][0], rtol=2e-3, atol=2e-4)
            del t
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
    finally:
        p.close()


def p_out_name(path, i):
    from paddle_infer_amd import inference as pinf
    c = pinf.Config(path + ".pdmodel", path + ".pdiparams")
    return pinf.create_predictor(c).get_output_names()[i]


def test_native_graph_lru_alternating_pointers(tmp_path):
    """Two KV-cache-style feed buffers used alternately: the predictor keeps one captured graph
    per signature (LRU) and replays it — 2 captures for 6 Runs, each Run's output follows the
    buffer it was given."""
    import ctypes
    import torch
    import native_capi as nc
    path = str(tmp_path / "mlp")
    export(MLP(), path, [InputSpec([None, 16], "float32", "x")])
    xs = [np.random.RandomState(10 + i).randn(8, 16).astype("float32") for i in range(2)]
    refs = [python_outputs(path, {"x": x}) for x in xs]
    ts = [torch.from_numpy(x).cuda() for x in xs]
    torch.cuda.synchronize()
    p = nc.Predictor(path, gpu=0, hip_graph=True)
    cap = nc.lib().piamd_native_graph_captures
    cap.restype = ctypes.c_long
    try:
        before = cap()
        for r in range(6):
            i = r % 2
            p.share("x", ts[i])
            p.run()
            got = p.fetch_float(p_out_name(path, 0), refs[i][0].shape)
            np.testing.assert_allclose(got, refs[i][0], rtol=2e-3, atol=2e-4)
        assert cap() - before == 2, f"captures: {cap() - before}"
    finally:
        p.close()
