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


def native_outputs(path, feeds, tmp, gpu=None, repeat=1, graph=False, warmup=0):
    cmd = [RUN, path + ".pdmodel", path + ".pdiparams", "--output-dir", str(tmp), "--repeat", str(repeat),
           "--warmup", str(warmup)]
    if gpu is not None:
        cmd += ["--gpu", str(gpu)]
    if graph:
        cmd += ["--graph"]
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


class SmallCNN(paddle.nn.Layer):
    """conv (strided, padded, bias) → BN → ReLU6 → max-pool (ceil) → grouped conv → BN → hardswish
    → depthwise 3×3 (dilation 2) → avg-pool → 1×1 conv → adaptive avg-pool → flatten → linear:
    conv2d (im2col + GEMM, 1×1 direct, depthwise kernel), batch_norm, pool2d, relu6, hard_swish."""

    def __init__(self):
        super().__init__()
        nn = paddle.nn
        self.c1 = nn.Conv2D(3, 16, 3, stride=2, padding=1)
        self.b1 = nn.BatchNorm2D(16)
        self.c2 = nn.Conv2D(16, 32, 3, padding=1, groups=4, bias_attr=False)
        self.b2 = nn.BatchNorm2D(32)
        self.dw = nn.Conv2D(32, 32, 3, padding=2, dilation=2, groups=32)
        self.pw = nn.Conv2D(32, 24, 1)
        self.fc = nn.Linear(24, 10)
        for b in (self.b1, self.b2):  # non-trivial running statistics
            b._mean.data.uniform_(-0.5, 0.5)
            b._variance.data.uniform_(0.5, 2.0)

    def forward(self, x):
        F = paddle.nn.functional
        h = F.relu6(self.b1(self.c1(x)))
        h = F.max_pool2d(h, 3, 2, 1, ceil_mode=True)
        h = F.hardswish(self.b2(self.c2(h)))
        h = F.avg_pool2d(self.dw(h), 2, 2)
        h = F.adaptive_avg_pool2d(self.pw(h), 1)
        return self.fc(paddle.flatten(h, 1))
