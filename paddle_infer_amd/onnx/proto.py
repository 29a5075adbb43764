"""ONNX ``onnx.proto3`` wire schema for the generic codec of ``static/proto.py`` (no ``onnx`` /
``protobuf`` generated code needed: field numbers below follow the public ONNX IR spec).

Kinds: v = varint, f = float32, d = float64, s = string, y = bytes, m = message."""
from __future__ import annotations

import numpy as np

from ..static import proto as _p

SCHEMA = {
    "ModelProto": {1: ("ir_version", "v", False, None), 8: ("opset_import", "m", True, "OperatorSetIdProto"),
                   2: ("producer_name", "s", False, None), 3: ("producer_version", "s", False, None),
                   4: ("domain", "s", False, None), 5: ("model_version", "v", False, None),
                   6: ("doc_string", "s", False, None), 7: ("graph", "m", False, "GraphProto")},
    "OperatorSetIdProto": {1: ("domain", "s", False, None), 2: ("version", "v", False, None)},
    "GraphProto": {1: ("node", "m", True, "NodeProto"), 2: ("name", "s", False, None),
                   5: ("initializer", "m", True, "TensorProto"), 10: ("doc_string", "s", False, None),
                   11: ("input", "m", True, "ValueInfoProto"), 12: ("output", "m", True, "ValueInfoProto"),
                   13: ("value_info", "m", True, "ValueInfoProto")},
    "NodeProto": {1: ("input", "s", True, None), 2: ("output", "s", True, None), 3: ("name", "s", False, None),
                  4: ("op_type", "s", False, None), 7: ("domain", "s", False, None),
                  5: ("attribute", "m", True, "AttributeProto"), 6: ("doc_string", "s", False, None)},
    "AttributeProto": {1: ("name", "s", False, None), 20: ("type", "v", False, None),
                       2: ("f", "f", False, None), 3: ("i", "v", False, None), 4: ("s", "y", False, None),
                       5: ("t", "m", False, "TensorProto"), 7: ("floats", "f", True, None),
                       8: ("ints", "v", True, None), 9: ("strings", "y", True, None)},
    "TensorProto": {1: ("dims", "v", True, None), 2: ("data_type", "v", False, None),
                    8: ("name", "s", False, None), 9: ("raw_data", "y", False, None),
                    4: ("float_data", "f", True, None), 7: ("int64_data", "v", True, None)},
    "ValueInfoProto": {1: ("name", "s", False, None), 2: ("type", "m", False, "TypeProto")},
    "TypeProto": {1: ("tensor_type", "m", False, "TypeProtoTensor")},
    "TypeProtoTensor": {1: ("elem_type", "v", False, None), 2: ("shape", "m", False, "TensorShapeProto")},
    "TensorShapeProto": {1: ("dim", "m", True, "Dimension")},
    "Dimension": {1: ("dim_value", "v", False, None), 2: ("dim_param", "s", False, None)},
}

# AttributeProto.AttributeType
A_FLOAT, A_INT, A_STRING, A_TENSOR, A_FLOATS, A_INTS, A_STRINGS = 1, 2, 3, 4, 6, 7, 8
# TensorProto.DataType <-> numpy
NP2ONNX = {np.dtype(np.float32): 1, np.dtype(np.uint8): 2, np.dtype(np.int8): 3, np.dtype(np.uint16): 4,
           np.dtype(np.int16): 5, np.dtype(np.int32): 6, np.dtype(np.int64): 7, np.dtype(np.bool_): 9,
           np.dtype(np.float16): 10, np.dtype(np.float64): 11}
ONNX2NP = {v: k for k, v in NP2ONNX.items()}
# Paddle VarType code (static/proto.VT) -> ONNX data type
PADDLE2ONNX = {0: 9, 1: 5, 2: 6, 3: 7, 4: 10, 5: 1, 6: 11, 20: 2, 21: 3, 22: 16}


def encode_model(model: dict) -> bytes:
    return _p.encode("ModelProto", model, SCHEMA)


def decode_model(buf: bytes) -> dict:
    return _p.decode("ModelProto", buf, SCHEMA)


def tensor(name: str, arr: np.ndarray) -> dict:
    arr = np.ascontiguousarray(arr)
    if arr.dtype not in NP2ONNX:
        raise TypeError(f"ONNX export: unsupported tensor dtype {arr.dtype}")
    return {"name": name, "dims": list(arr.shape), "data_type": NP2ONNX[arr.dtype],
            "raw_data": arr.tobytes()}


def tensor_to_numpy(t: dict) -> np.ndarray:
    dt = ONNX2NP[t.get("data_type", 1)]
    dims = t.get("dims", [])
    if "raw_data" in t:
        a = np.frombuffer(t["raw_data"], dtype=dt).copy()
    elif t.get("float_data"):
        a = np.asarray(t["float_data"], dtype=dt)
    elif t.get("int64_data"):
        a = np.asarray(t["int64_data"], dtype=dt)
    else:
        a = np.zeros(0, dtype=dt)
    return a.reshape(dims)


def attr(name: str, v) -> dict:
    if isinstance(v, dict):  # a TensorProto
        return {"name": name, "type": A_TENSOR, "t": v}
    if isinstance(v, bool) or isinstance(v, (int, np.integer)):
        return {"name": name, "type": A_INT, "i": int(v)}
    if isinstance(v, (float, np.floating)):
        return {"name": name, "type": A_FLOAT, "f": float(v)}
    if isinstance(v, (str, bytes)):
        return {"name": name, "type": A_STRING, "s": v.encode() if isinstance(v, str) else v}
    v = list(v)
    if all(isinstance(x, (int, np.integer, bool)) for x in v):
        return {"name": name, "type": A_INTS, "ints": [int(x) for x in v]}
    if all(isinstance(x, (int, float, np.number)) for x in v):
        return {"name": name, "type": A_FLOATS, "floats": [float(x) for x in v]}
    return {"name": name, "type": A_STRINGS, "strings": [x.encode() if isinstance(x, str) else x for x in v]}


def attr_value(a: dict):
    t = a.get("type")
    if t == A_FLOAT:
        return a.get("f", 0.0)
    if t == A_INT:
        return a.get("i", 0)
    if t == A_STRING:
        s = a.get("s", b"")
        return s.decode() if isinstance(s, bytes) else s
    if t == A_TENSOR:
        return tensor_to_numpy(a["t"])
    if t == A_FLOATS:
        return list(a.get("floats", []))
    if t == A_INTS:
        return list(a.get("ints", []))
    if t == A_STRINGS:
        return [x.decode() if isinstance(x, bytes) else x for x in a.get("strings", [])]
    raise ValueError(f"unsupported ONNX attribute type {t}")


def value_info(name: str, elem_type: int, dims) -> dict:
    ds = []
    for i, d in enumerate(dims):
        ds.append({"dim_value": int(d)} if d is not None and int(d) >= 0 else {"dim_param": f"{name}_d{i}"})
    return {"name": name, "type": {"tensor_type": {"elem_type": elem_type, "shape": {"dim": ds}}}}
