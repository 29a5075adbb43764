"""Native C++ inference API (`csrc/native`, reference `paddle_inference_api.h:80`): the
`pd_infer_run` driver (a C++ paddle_infer::Predictor — no Python interpreter, no torch) loads
exported programs and matches the Python Predictor; unknown op types are refused at load."""
import os
import subprocess

import numpy as np
import pytest

from native_infer_util import MLP, RUN, Encoder, export, native_outputs, python_outputs

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
