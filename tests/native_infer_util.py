"""Shared by the native C++ predictor tests: export models, run `_lib/pd_infer_run` (the C++
paddle_infer::Predictor, no Python inside) and the Python Predictor on the same inputs."""
import os
import subprocess

import numpy as np
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import inference as pinf
from paddle_infer_amd import jit
from paddle_infer_amd.static import InputSpec

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUN = os.path.join(ROOT, "paddle_infer_amd", "_lib", "pd_infer_run")


class Encoder(paddle.nn.Layer):
    """Embedding → single-head self-attention (matmul / scale / softmax) → residual LayerNorm →
    GELU MLP → tanh: the exported-inference op core (lookup_table_v2, matmul_v2, transpose2,
    elementwise_add, scale, softmax, layer_norm, gelu, tanh)."""

    def __init__(self, V=100, E=32):
        super().__init__()
        self.emb = paddle.nn.Embedding(V, E)
        self.q = paddle.nn.Linear(E, E)
        self.l1 = paddle.nn.Linear(E, 2 * E)
        self.l2 = paddle.nn.Linear(2 * E, E)
        self.ln = paddle.nn.LayerNorm(E)

    def forward(self, ids):
        h = self.emb(ids)
        a = self.q(h)
        att = paddle.nn.functional.softmax(paddle.matmul(a, h, transpose_y=True) * 0.125, -1)
        h = self.ln(h + paddle.matmul(att, h))
        return self.l2(paddle.nn.functional.gelu(self.l1(h))).tanh()


class MLP(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.a = paddle.nn.Linear(16, 64)
        self.b = paddle.nn.Linear(64, 8)

    def forward(self, x):
        h = paddle.nn.functional.relu(self.a(x))
        y = self.b(h)
        return paddle.nn.functional.softmax(y, -1), paddle.concat([y, y * 2.0], axis=-1)


def export(model, path, spec):
    torch.manual_seed(0)
    model.eval()
    jit.save(model, path, input_spec=spec)


def python_outputs(path, feeds):
    c = pinf.Config(path + ".pdmodel", path + ".pdiparams")
    c.switch_ir_optim(False)
    p = pinf.create_predictor(c)
    for n, a in feeds.items():
        p.get_input_handle(n).copy_from_cpu(a)
    p.run()
    return [p.get_output_handle(n).copy_to_cpu() for n in p.get_output_names()]


def native_outputs(path, feeds, tmp, gpu=None, repeat=1):
    cmd = [RUN, path + ".pdmodel", path + ".pdiparams", "--output-dir", str(tmp), "--repeat", str(repeat)]
    if gpu is not None:
        cmd += ["--gpu", str(gpu)]
    for n, a in feeds.items():
        f = os.path.join(str(tmp), f"in_{n}.bin")
        np.ascontiguousarray(a).tofile(f)
        cmd += ["--input", n, str(a.dtype), ",".join(map(str, a.shape)), f]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    outs, ms = [], None
    for line in r.stdout.splitlines():
        parts = line.split()
        if parts and parts[0] == "output":
            i, dt, dims = int(parts[1]), parts[3], [int(d) for d in parts[4].split(",") if d]
            outs.append(np.fromfile(os.path.join(str(tmp), f"{i}.bin"), dtype=dt).reshape(dims))
        elif parts and parts[0] == "run_ms":
            ms = float(parts[1])
    return outs, ms, r.stdout
