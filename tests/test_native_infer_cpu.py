"""Native C++ inference API (`csrc/native`, reference `paddle_inference_api.h:80`): the
`pd_infer_run` driver (a C++ paddle_infer::Predictor — no Python interpreter, no torch) loads
exported programs and matches the Python Predictor; unknown op types are refused at load."""
import os
import subprocess

import numpy as np
import torch
import pytest

from native_infer_util import MLP, RUN, Encoder, export, native_outputs, python_outputs

import paddle_infer_amd as paddle
from paddle_infer_amd import static
from paddle_infer_amd.static import InputSpec

pytestmark = pytest.mark.skipif(not os.path.exists(RUN), reason="native engine not built")


def test_native_runner_links_no_python():
    r = subprocess.run(["ldd", RUN], capture_output=True, text=True)
    assert "libpython" not in r.stdout and "libtorch" not in r.stdout and "libpiamd_infer" in r.stdout


@pytest.mark.parametrize("B", [1, 3])
def test_encoder_matches_python_predictor(tmp_path, B):
    path = str(tmp_path / "enc")
    export(Encoder(), path, [InputSpec([None, 8], "int64", "ids")])
    ids = np.random.RandomState(B).randint(0, 100, size=(B, 8)).astype("int64")
    ref = python_outputs(path, {"ids": ids})
    got, _, _ = native_outputs(path, {"ids": ids}, tmp_path)
    assert len(got) == len(ref) == 1
    np.testing.assert_allclose(got[0], ref[0], rtol=1e-4, atol=1e-5)


def test_mlp_two_outputs_concat_softmax(tmp_path):
    path = str(tmp_path / "mlp")
    export(MLP(), path, [InputSpec([None, 16], "float32", "x")])
    x = np.random.RandomState(0).randn(5, 16).astype("float32")
    ref = python_outputs(path, {"x": x})
    got, _, out = native_outputs(path, {"x": x}, tmp_path)
    assert len(got) == 2
    for a, b in zip(got, ref):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)
    assert "gfx950" in out


def test_unknown_op_refused_at_load(tmp_path):
    import torch

    from paddle_infer_amd import jit

    class Odd(torch.nn.Module):
        def forward(self, x):
            return torch.special.erfcx(x)
    path = str(tmp_path / "odd")
    jit.save(Odd(), path, input_spec=[InputSpec([None, 4], "float32", "x")], allow_custom_ops=True)
    x = np.ones((2, 4), "float32")
    r = subprocess.run([RUN, path + ".pdmodel", path + ".pdiparams", "--input", "x", "float32", "2,4",
                        str(tmp_path / "x.bin")], capture_output=True, text=True)
    x.tofile(str(tmp_path / "x.bin"))
    assert r.returncode != 0 and "no kernel for op type" in r.stderr


@pytest.mark.skipif(__import__("shutil").which("gcc") is None, reason="needs a C compiler")
def test_reference_c_api_on_native_engine(tmp_path):
    """The capi_exp C client (tests/capi/capi_demo.c) linked against libpiamd_infer.so: the PD_*
    entry points run on the native engine (copy path, MutableData path, cloned predictor)."""
    from paddle_infer_amd import _build
    from paddle_infer_amd.inference import Config, create_predictor
    prefix = str(tmp_path / "mlp")
    _save_model(prefix)
    exe = tmp_path / "capi_native"
    here = os.path.dirname(os.path.abspath(__file__))
    subprocess.run(["gcc", "-O1", os.path.join(here, "capi", "capi_demo.c"), f"-I{_build.CDIR}",
                    f"-L{_build.LIBDIR}", "-lpiamd_infer", f"-Wl,-rpath,{_build.LIBDIR}", "-o", str(exe)],
                   check=True)
    assert "libpython" not in subprocess.run(["ldd", str(exe)], capture_output=True, text=True).stdout
    r = subprocess.run([str(exe), prefix + ".pdmodel", prefix + ".pdiparams", "3"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "native" in r.stdout.splitlines()[0]
    pred = create_predictor(Config(prefix + ".pdmodel", prefix + ".pdiparams"))
    x = (np.arange(3 * 8) * 7 % 13).astype("float32").reshape(3, 8) / 13.0 - 0.5
    h = pred.get_input_handle(pred.get_input_names()[0])
    h.reshape([3, 8])
    h.copy_from_cpu(x)
    pred.run()
    ref = pred.get_output_handle(pred.get_output_names()[0]).copy_to_cpu()
    outs = [ln for ln in r.stdout.splitlines() if ln.startswith(("copy", "mutable"))]
    assert len(outs) == 3
    for ln in outs:
        parts = ln.split()
        vals = np.array([float(v) for v in parts[7:]], dtype=np.float32).reshape(3, 3)
        np.testing.assert_allclose(vals, ref, rtol=1e-5, atol=1e-6)


def test_cnn_ops_match_python_predictor(tmp_path):
    """conv2d (grouped / depthwise / 1×1 / strided / dilated), batch_norm, pool2d (max ceil-mode,
    avg, adaptive), relu6 and hard_swish on the native engine."""
    from native_infer_util import SmallCNN
    path = str(tmp_path / "cnn")
    export(SmallCNN(), path, [InputSpec([None, 3, 33, 30], "float32", "x")])
    x = np.random.RandomState(1).randn(2, 3, 33, 30).astype("float32")
    ref = python_outputs(path, {"x": x})
    got, _, _ = native_outputs(path, {"x": x}, tmp_path)
    np.testing.assert_allclose(got[0], ref[0], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("arch", ["mobilenet_v2", "resnet18"])
def test_vision_models_match_python_predictor(tmp_path, arch):
    """Whole paddle.vision models exported with jit.save run on the native engine."""
    from paddle_infer_amd.vision import models as VM
    torch.manual_seed(0)
    m = getattr(VM, arch)(num_classes=10)
    path = str(tmp_path / arch)
    export(m, path, [InputSpec([None, 3, 64, 64], "float32", "x")])
    x = np.random.RandomState(2).randn(1, 3, 64, 64).astype("float32")
    ref = python_outputs(path, {"x": x})
    got, _, _ = native_outputs(path, {"x": x}, tmp_path)
    np.testing.assert_allclose(got[0], ref[0], rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("damage", ["truncate_mid", "extra_bytes", "missing_tensor", "neg_desc"])
def test_corrupt_params_file_refused(tmp_path, damage):
    """The .pdiparams reader bounds-checks every read: truncated, padded or corrupted files are
    refused with an error, never read out of range (reference LoadCombine errors likewise)."""
    import struct
    path = str(tmp_path / "mlp")
    export(MLP(), path, [InputSpec([None, 16], "float32", "x")])
    data = open(path + ".pdiparams", "rb").read()
    if damage == "truncate_mid":
        data = data[: len(data) // 2]
    elif damage == "extra_bytes":
        data = data + b"\0" * 16
    elif damage == "missing_tensor":
        # keep only the first tensor record: version(4) lod(8) ver(4) dsz(4) desc data
        dsz = struct.unpack_from("<i", data, 16)[0]
        pos = 20 + dsz
        desc = data[20:pos]
        # numel from the desc is not needed: cut right after the first record's header + desc
        data = data[:pos]
    elif damage == "neg_desc":
        data = data[:16] + struct.pack("<i", -5) + data[20:]
    bad = str(tmp_path / "bad.pdiparams")
    open(bad, "wb").write(data)
    x = np.ones((2, 16), "float32")
    x.tofile(str(tmp_path / "x.bin"))
    r = subprocess.run([RUN, path + ".pdmodel", bad, "--input", "x", "float32", "2,16",
                        str(tmp_path / "x.bin")], capture_output=True, text=True)
    assert r.returncode != 0, r.stdout
    assert "params file" in r.stderr or "truncated" in r.stderr, r.stderr


def _save_model(prefix):
    torch.manual_seed(0)
    paddle.enable_static()
    try:
        main = static.Program()
        with static.program_guard(main):
            x = static.data("x", [None, 8], "float32")
            h = static.nn.fc(x, 16, activation="relu")
            y = static.nn.fc(h, 3)
        exe = static.Executor(paddle.CPUPlace())
        static.save_inference_model(prefix, [x], [y], exe, program=main)
    finally:
        paddle.disable_static()


def test_native_c_api_ctypes_in_process(tmp_path):
    from paddle_infer_amd import _build
    """The native C API library (no Python inside) loaded into a Python process with ctypes."""
    import ctypes
    prefix = str(tmp_path / "mlp")
    _save_model(prefix)
    lib = ctypes.CDLL(_build.NATIVE_LIB)
    lib.PD_ConfigCreate.restype = ctypes.c_void_p
    lib.PD_PredictorCreate.restype = ctypes.c_void_p
    lib.PD_PredictorCreate.argtypes = [ctypes.c_void_p]
    lib.PD_ConfigSetModel.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p]
    lib.PD_PredictorGetInputNum.restype = ctypes.c_size_t
    lib.PD_PredictorGetInputNum.argtypes = [ctypes.c_void_p]
    lib.PD_PredictorDestroy.argtypes = [ctypes.c_void_p]
    cfg = lib.PD_ConfigCreate()
    lib.PD_ConfigSetModel(cfg, (prefix + ".pdmodel").encode(), (prefix + ".pdiparams").encode())
    pred = lib.PD_PredictorCreate(cfg)
    assert pred
    assert lib.PD_PredictorGetInputNum(pred) == 1
    lib.PD_PredictorDestroy(pred)
