"""C inference API (libpiamd_capi.so, reference `paddle/fluid/inference/capi_exp`): a plain C
program built against `csrc/capi/pd_inference_api.h` loads a saved inference model, runs it through
the copy and the MutableData paths and a cloned predictor, and matches the Python Predictor."""
import os
import shutil
import subprocess

import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import _build, static
from paddle_infer_amd.inference import Config, create_predictor

HERE = os.path.dirname(os.path.abspath(__file__))


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


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs a C compiler")
def test_c_program_matches_python_predictor(tmp_path):
    _build.build(verbose=False)
    prefix = str(tmp_path / "mlp")
    _save_model(prefix)
    exe = tmp_path / "capi_demo"
    subprocess.run(["gcc", "-O1", os.path.join(HERE, "capi", "capi_demo.c"),
                    f"-I{_build.CDIR}", f"-L{_build.LIBDIR}", "-lpiamd_capi",
                    f"-Wl,-rpath,{_build.LIBDIR}", "-o", str(exe)], check=True)
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([str(exe), prefix + ".pdmodel", prefix + ".pdiparams", "3"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = {ln.split()[0]: ln for ln in r.stdout.splitlines() if ln.strip()}
    assert "paddle_infer_amd" in lines["version"]
    assert lines["inputs"].split()[1:] == ["1", "outputs", "1"]
    assert "use_gpu 0 ir_optim 1 trt 0" in lines["use_gpu"]
    # Python reference on the same input
    cfg = Config(prefix + ".pdmodel", prefix + ".pdiparams")
    pred = create_predictor(cfg)
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
        assert parts[1:5] == ["shape", "3", "3", "dtype"] and parts[5] == "0", ln
        vals = np.array([float(v) for v in parts[7:]], dtype=np.float32).reshape(3, 3)
        np.testing.assert_allclose(vals, ref, rtol=1e-5, atol=1e-6)


def test_ctypes_in_process(tmp_path):
    """The same library loaded into a Python process (GIL taken per call)."""
    import ctypes
    _build.build(verbose=False)
    prefix = str(tmp_path / "mlp")
    _save_model(prefix)
    lib = ctypes.CDLL(_build.CAPI_LIB)
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
