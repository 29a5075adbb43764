"""Reference (numpy) interpreter of the ONNX operator subset ``converter.py`` emits — the
numerical check of an exported graph without onnxruntime (not installed here): nodes run in
file order (ONNX graphs are topologically sorted) with the opset-13 semantics of each operator.
Convolution / pooling use torch CPU functional ops as the numeric kernels."""
from __future__ import annotations



import numpy as np

from . import proto as P


def _erf(x):
    import torch
    return torch.erf(torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64))).numpy().astype(x.dtype)


def _t(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x))


def _conv(ins, a):
    import torch.nn.functional as F
    x, w = ins[0], ins[1]
    b = ins[2] if len(ins) > 2 else None
    pads = a.get("pads", [0, 0, 0, 0])
    if a.get("auto_pad", "NOTSET") in ("SAME_UPPER", "SAME_LOWER"):
        raise NotImplementedError("reference Conv auto_pad SAME")
    xt = _t(x)
    if pads[0] != pads[2] or pads[1] != pads[3]:
        xt = F.pad(xt, (pads[1], pads[3], pads[0], pads[2]))
        pad = 0
    else:
        pad = (pads[0], pads[1])
    y = F.conv2d(xt, _t(w), None if b is None else _t(b), a.get("strides", [1, 1]), pad,
                 a.get("dilations", [1, 1]), a.get("group", 1))
    return y.numpy()


def _pool(ins, a, mx):
    import torch.nn.functional as F
    x = _t(ins[0])
    k, st, pads = a["kernel_shape"], a.get("strides", a["kernel_shape"]), a.get("pads", [0, 0, 0, 0])
    ceil = bool(a.get("ceil_mode", 0))
    if pads[0] != pads[2] or pads[1] != pads[3]:
        raise NotImplementedError("asymmetric pool pads")
    if mx:
        return F.max_pool2d(x, k, st, (pads[0], pads[1]), ceil_mode=ceil).numpy()
    return F.avg_pool2d(x, k, st, (pads[0], pads[1]), ceil_mode=ceil,
                        count_include_pad=bool(a.get("count_include_pad", 0))).numpy()


def _softmax(x, axis):
    m = np.max(x, axis=axis, keepdims=True)
    e = np.exp(x - m)
    return e / np.sum(e, axis=axis, keepdims=True)


def _slice(ins):
    x, starts, ends = ins[0], ins[1], ins[2]
    axes = ins[3] if len(ins) > 3 else np.arange(len(starts))
    steps = ins[4] if len(ins) > 4 else np.ones(len(starts), dtype=np.int64)
    sl = [slice(None)] * x.ndim
    for s, e, ax, st in zip(starts, ends, axes, steps):
        ax = int(ax) % x.ndim
        n = x.shape[ax]
        s, e = int(s), int(e)
        sl[ax] = slice(max(-n - 1, min(s, n)), max(-n - 1, min(e, n)), int(st))
    return x[tuple(sl)]


def _reshape(x, shape):
    shape = [int(s) for s in shape]
    shape = [x.shape[i] if s == 0 else s for i, s in enumerate(shape)]
    return x.reshape(shape)


OPS = {
    "Add": lambda i, a: i[0] + i[1], "Sub": lambda i, a: i[0] - i[1], "Mul": lambda i, a: i[0] * i[1],
    "Div": lambda i, a: (i[0] // i[1]) if np.issubdtype(i[0].dtype, np.integer) else i[0] / i[1],
    "Pow": lambda i, a: np.power(i[0], i[1]).astype(i[0].dtype),
    "Max": lambda i, a: np.maximum(i[0], i[1]), "Min": lambda i, a: np.minimum(i[0], i[1]),
    "MatMul": lambda i, a: np.matmul(i[0], i[1]),
    "Relu": lambda i, a: np.maximum(i[0], 0).astype(i[0].dtype), "Tanh": lambda i, a: np.tanh(i[0]),
    "Sigmoid": lambda i, a: 1.0 / (1.0 + np.exp(-i[0])), "Exp": lambda i, a: np.exp(i[0]),
    "Log": lambda i, a: np.log(i[0]), "Sqrt": lambda i, a: np.sqrt(i[0]), "Abs": lambda i, a: np.abs(i[0]),
    "Floor": lambda i, a: np.floor(i[0]), "Sin": lambda i, a: np.sin(i[0]), "Cos": lambda i, a: np.cos(i[0]),
    "Erf": lambda i, a: _erf(i[0]), "Reciprocal": lambda i, a: 1.0 / i[0],
    "Identity": lambda i, a: i[0], "Not": lambda i, a: np.logical_not(i[0]),
    "LeakyRelu": lambda i, a: np.where(i[0] >= 0, i[0], i[0] * a.get("alpha", 0.01)).astype(i[0].dtype),
    "Clip": lambda i, a: np.clip(i[0], i[1], i[2]).astype(i[0].dtype),
    "GreaterOrEqual": lambda i, a: i[0] >= i[1], "Greater": lambda i, a: i[0] > i[1],
    "LessOrEqual": lambda i, a: i[0] <= i[1], "Less": lambda i, a: i[0] < i[1],
    "Equal": lambda i, a: i[0] == i[1], "And": lambda i, a: np.logical_and(i[0], i[1]),
    "Or": lambda i, a: np.logical_or(i[0], i[1]), "Where": lambda i, a: np.where(i[0], i[1], i[2]),
    "ConstantOfShape": lambda i, a: np.full([int(s) for s in i[0]], a["value"].reshape(-1)[0],
                                            dtype=a["value"].dtype),
    "Shape": lambda i, a: np.asarray(i[0].shape, dtype=np.int64),
    "Cast": lambda i, a: i[0].astype(P.ONNX2NP[a["to"]]),
    "Reshape": lambda i, a: _reshape(i[0], i[1]),
    "Transpose": lambda i, a: np.transpose(i[0], a.get("perm")),
    "Unsqueeze": lambda i, a: np.expand_dims(i[0], tuple(int(x) % (i[0].ndim + len(i[1])) for x in i[1])),
    "Squeeze": lambda i, a: np.squeeze(i[0], tuple(int(x) for x in i[1]) if len(i) > 1 else None),
    "Concat": lambda i, a: np.concatenate(i, axis=a["axis"]),
    "Split": lambda i, a: np.split(i[0], np.cumsum(i[1])[:-1].tolist(), axis=a.get("axis", 0)),
    "Slice": lambda i, a: _slice(i),
    "Expand": lambda i, a: i[0] * np.ones([int(s) for s in i[1]], dtype=i[0].dtype),
    "ReduceMean": lambda i, a: np.mean(i[0], axis=tuple(a["axes"]), keepdims=bool(a.get("keepdims", 1))),
    "ReduceSum": lambda i, a: np.sum(i[0], axis=tuple(int(x) for x in i[1]), keepdims=bool(a.get("keepdims", 1))),
    "ReduceMax": lambda i, a: np.max(i[0], axis=tuple(a["axes"]), keepdims=bool(a.get("keepdims", 1))),
    "ReduceMin": lambda i, a: np.min(i[0], axis=tuple(a["axes"]), keepdims=bool(a.get("keepdims", 1))),
    "ReduceProd": lambda i, a: np.prod(i[0], axis=tuple(a["axes"]), keepdims=bool(a.get("keepdims", 1))),
    "Softmax": lambda i, a: _softmax(i[0], a.get("axis", -1)),
    "Gather": lambda i, a: np.take(i[0], i[1].astype(np.int64), axis=a.get("axis", 0)),
    "Range": lambda i, a: np.arange(int(i[0]), int(i[1]), int(i[2]), dtype=np.int64),
    "Conv": lambda i, a: _conv(i, a),
    "BatchNormalization": lambda i, a: ((i[0] - i[3].reshape(1, -1, *([1] * (i[0].ndim - 2)))) /
                                        np.sqrt(i[4].reshape(1, -1, *([1] * (i[0].ndim - 2))) + a.get("epsilon", 1e-5)) *
                                        i[1].reshape(1, -1, *([1] * (i[0].ndim - 2))) +
                                        i[2].reshape(1, -1, *([1] * (i[0].ndim - 2)))).astype(i[0].dtype),
    "MaxPool": lambda i, a: _pool(i, a, True), "AveragePool": lambda i, a: _pool(i, a, False),
    "GlobalAveragePool": lambda i, a: np.mean(i[0], axis=tuple(range(2, i[0].ndim)), keepdims=True),
    "GlobalMaxPool": lambda i, a: np.max(i[0], axis=tuple(range(2, i[0].ndim)), keepdims=True),
}


def run(model, feeds: dict):
    """Execute an ONNX model (path, bytes or decoded dict) on numpy ``feeds``; returns the graph
    outputs in order."""
    if isinstance(model, str):
        with open(model, "rb") as f:
            model = P.decode_model(f.read())
    elif isinstance(model, (bytes, bytearray)):
        model = P.decode_model(bytes(model))
    g = model["graph"]
    env = {t["name"]: P.tensor_to_numpy(t) for t in g.get("initializer", [])}
    for vi, (k, v) in zip(g.get("input", []), feeds.items()):
        env[vi["name"]] = np.asarray(v)
    for k, v in feeds.items():
        env.setdefault(k, np.asarray(v))
    for n in g.get("node", []):
        a = {x["name"]: P.attr_value(x) for x in n.get("attribute", [])}
        fn = OPS.get(n["op_type"])
        if fn is None:
            raise NotImplementedError(f"reference ONNX op {n['op_type']}")
        ins = [env[x] for x in n.get("input", []) if x != ""]
        out = fn(ins, a)
        outs = n.get("output", [])
        if isinstance(out, list):
            for name, val in zip(outs, out):
                env[name] = val
        else:
            env[outs[0]] = out if isinstance(out, np.ndarray) else np.asarray(out)
    return [env[o["name"]] for o in g.get("output", [])]



