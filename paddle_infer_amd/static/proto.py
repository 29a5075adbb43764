"""Wire-format codec for Paddle's ``framework.proto`` (ProgramDesc) and the combined-params
(``.pdiparams``) tensor stream — no protoc, no generated code.

Parity: reference `paddle/fluid/framework/framework.proto` (field numbers below match it
exactly) and `paddle/fluid/framework/lod_tensor.cc:SerializeToStream` / `tensor_util.cc:
TensorToStream` (uint32 version, uint64 lod levels, uint32 version, int32 desc size, TensorDesc
bytes, raw data), used by `save_combine` for ``.pdiparams``.
"""
from __future__ import annotations

import struct

import numpy as np

# kind: v=varint(int), b=bool, s=string, f=float32, d=float64, m=message, e=enum
SCHEMA = {
    "ProgramDesc": {1: ("blocks", "m", True, "BlockDesc"), 4: ("version", "m", False, "Version"),
                    5: ("op_version_map", "m", False, "OpVersionMap")},
    "Version": {1: ("version", "v", False, None)},
    "OpVersionMap": {1: ("pair", "m", True, "OpVersionPair")},
    "OpVersionPair": {1: ("op_name", "s", False, None), 2: ("op_version", "m", False, "OpVersion")},
    "OpVersion": {1: ("version", "v", False, None)},
    "BlockDesc": {1: ("idx", "v", False, None), 2: ("parent_idx", "v", False, None),
                  3: ("vars", "m", True, "VarDesc"), 4: ("ops", "m", True, "OpDesc"),
                  5: ("forward_block_idx", "v", False, None)},
    "VarDesc": {1: ("name", "s", False, None), 2: ("type", "m", False, "VarType"),
                3: ("persistable", "b", False, None), 4: ("need_check_feed", "b", False, None),
                5: ("is_parameter", "b", False, None), 6: ("stop_gradient", "b", False, None),
                7: ("attrs", "m", True, "VarAttr")},
    "VarAttr": {1: ("name", "s", False, None), 2: ("type", "v", False, None), 3: ("i", "v", False, None),
                4: ("s", "s", False, None), 5: ("ints", "v", True, None)},
    "VarType": {1: ("type", "v", False, None), 2: ("selected_rows", "m", False, "TensorDesc"),
                3: ("lod_tensor", "m", False, "LoDTensorDesc"),
                4: ("tensor_array", "m", False, "LoDTensorDesc")},
    "TensorDesc": {1: ("data_type", "v", False, None), 2: ("dims", "v", True, None)},
    "LoDTensorDesc": {1: ("tensor", "m", False, "TensorDesc"), 2: ("lod_level", "v", False, None)},
    "OpDesc": {3: ("type", "s", False, None), 1: ("inputs", "m", True, "OpVar"),
               2: ("outputs", "m", True, "OpVar"), 4: ("attrs", "m", True, "OpAttr"),
               5: ("is_target", "b", False, None)},
    "OpVar": {1: ("parameter", "s", False, None), 2: ("arguments", "s", True, None)},
    "OpAttr": {1: ("name", "s", False, None), 2: ("type", "v", False, None), 3: ("i", "v", False, None),
               4: ("f", "f", False, None), 5: ("s", "s", False, None), 6: ("ints", "v", True, None),
               7: ("floats", "f", True, None), 8: ("strings", "s", True, None), 10: ("b", "b", False, None),
               11: ("bools", "b", True, None), 12: ("block_idx", "v", False, None),
               13: ("l", "v", False, None), 14: ("blocks_idx", "v", True, None),
               15: ("longs", "v", True, None), 16: ("float64s", "d", True, None),
               17: ("var_name", "s", False, None), 18: ("vars_name", "s", True, None),
               19: ("float64", "d", False, None)},
}

ATTR = {"INT": 0, "FLOAT": 1, "STRING": 2, "INTS": 3, "FLOATS": 4, "STRINGS": 5, "BOOLEAN": 6,
        "BOOLEANS": 7, "BLOCK": 8, "LONG": 9, "BLOCKS": 10, "LONGS": 11, "FLOAT64S": 12, "VAR": 13,
        "VARS": 14, "FLOAT64": 15}
VT = {"bool": 0, "int16": 1, "int32": 2, "int64": 3, "float16": 4, "float32": 5, "float64": 6,
      "uint8": 20, "int8": 21, "bfloat16": 22, "complex64": 23, "complex128": 24}
VT_LOD_TENSOR, VT_FEED, VT_FETCH = 7, 9, 10
NP = {0: np.bool_, 1: np.int16, 2: np.int32, 3: np.int64, 4: np.float16, 5: np.float32,
      6: np.float64, 20: np.uint8, 21: np.int8, 22: np.uint16, 23: np.complex64, 24: np.complex128}


def _varint(n: int) -> bytes:
    if n < 0:
        n += 1 << 64
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, pos):
    n = shift = 0
    while True:
        b = buf[pos]
        pos += 1
        n |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            return n, pos


def _signed(n, bits=64):
    return n - (1 << 64) if n >= 1 << 63 else n


def encode(msg_name: str, obj: dict, schemas=None) -> bytes:
    """Encode ``obj`` as message ``msg_name`` of ``schemas`` (default: framework.proto)."""
    schemas = SCHEMA if schemas is None else schemas
    schema = schemas[msg_name]
    out = bytearray()
    for fno in sorted(schema, key=lambda f: f if msg_name != "OpDesc" else {3: 0, 1: 1, 2: 2, 4: 3, 5: 4}[f]):
        name, kind, rep, sub = schema[fno]
        if name not in obj or obj[name] is None:
            continue
        vals = obj[name] if rep else [obj[name]]
        for v in vals:
            if kind in ("v", "b", "e"):
                out += _varint((fno << 3) | 0) + _varint(int(v))
            elif kind == "f":
                out += _varint((fno << 3) | 5) + struct.pack("<f", float(v))
            elif kind == "d":
                out += _varint((fno << 3) | 1) + struct.pack("<d", float(v))
            elif kind in ("s", "y"):
                b = v.encode() if isinstance(v, str) else bytes(v)
                out += _varint((fno << 3) | 2) + _varint(len(b)) + b
            elif kind == "m":
                b = encode(sub, v, schemas)
                out += _varint((fno << 3) | 2) + _varint(len(b)) + b
    return bytes(out)


def decode(msg_name: str, buf: bytes, schemas=None) -> dict:
    schemas = SCHEMA if schemas is None else schemas
    schema = schemas[msg_name]
    obj = {}
    pos, end = 0, len(buf)
    while pos < end:
        key, pos = _read_varint(buf, pos)
        fno, wt = key >> 3, key & 7
        spec = schema.get(fno)
        if wt == 0:
            v, pos = _read_varint(buf, pos)
            val = [_signed(v)]
        elif wt == 1:
            val = [struct.unpack_from("<d", buf, pos)[0]]
            pos += 8
        elif wt == 5:
            val = [struct.unpack_from("<f", buf, pos)[0]]
            pos += 4
        elif wt == 2:
            ln, pos = _read_varint(buf, pos)
            raw = bytes(buf[pos:pos + ln])
            pos += ln
            if spec is None:
                continue
            kind = spec[1]
            if kind == "m":
                val = [decode(spec[3], raw, schemas)]
            elif kind == "s":
                val = [raw.decode("utf-8", errors="replace")]
            elif kind == "y":  # bytes field (kept raw)
                val = [raw]
            else:  # packed repeated scalars
                val, p2 = [], 0
                while p2 < len(raw):
                    if kind in ("v", "b", "e"):
                        v, p2 = _read_varint(raw, p2)
                        val.append(_signed(v))
                    elif kind == "f":
                        val.append(struct.unpack_from("<f", raw, p2)[0])
                        p2 += 4
                    else:
                        val.append(struct.unpack_from("<d", raw, p2)[0])
                        p2 += 8
        else:
            raise ValueError(f"unsupported wire type {wt}")
        if spec is None:
            continue
        name, kind, rep, _ = spec
        if kind == "b":
            val = [bool(x) for x in val]
        if rep:
            obj.setdefault(name, []).extend(val)
        else:
            obj[name] = val[-1]
    return obj


# ---------------------------------------------------------------------------- tensors
def tensor_to_stream(arr: np.ndarray, vt: int) -> bytes:
    desc = encode("TensorDesc", {"data_type": vt, "dims": list(arr.shape)})
    return (struct.pack("<I", 0) + struct.pack("<Q", 0) + struct.pack("<I", 0) +
            struct.pack("<i", len(desc)) + desc + np.ascontiguousarray(arr).tobytes())


def tensor_from_stream(buf: bytes, pos: int):
    (_ver,) = struct.unpack_from("<I", buf, pos)
    pos += 4
    (lod_levels,) = struct.unpack_from("<Q", buf, pos)
    pos += 8
    for _ in range(lod_levels):
        (sz,) = struct.unpack_from("<Q", buf, pos)
        pos += 8 + sz
    (_tver,) = struct.unpack_from("<I", buf, pos)
    pos += 4
    (dsz,) = struct.unpack_from("<i", buf, pos)
    pos += 4
    desc = decode("TensorDesc", buf[pos:pos + dsz])
    pos += dsz
    dt = NP[desc.get("data_type", 5)]
    dims = desc.get("dims", [])
    n = int(np.prod(dims)) if dims else 1
    nbytes = n * np.dtype(dt).itemsize
    arr = np.frombuffer(buf, dtype=dt, count=n, offset=pos).reshape(dims).copy()
    pos += nbytes
    return arr, desc.get("data_type", 5), pos
