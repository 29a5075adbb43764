"""Native token-window loader for LLM pre-training (``csrc/runtime/dataloader.cc``).

Parity: reference native data feed (`paddle/fluid/framework/data_feed.cc` reader threads →
channel → trainer) and the GPT pre-training dataset used by its GPT-3 benchmarks (fixed-length
windows over a flat token file, per-epoch shuffle, data-parallel sharding).

The C++ side mmaps the token file and keeps a ring of ready batches filled by worker threads; this
wrapper copies each batch into a pinned host buffer and issues the H2D on a side HIP stream, so the
consumer's stream only waits on an event (the copy overlaps the previous step's compute).
Batches are int64 [batch, seq_len + 1]: ``x = b[:, :-1]``, ``labels = b[:, 1:]``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        from ..static.executor import runtime_lib
        lib = runtime_lib()
        lib.piamd_tokloader_create.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_ulonglong, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int, ctypes.c_int]
        lib.piamd_tokloader_create.restype = ctypes.c_void_p
        lib.piamd_tokloader_next.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        lib.piamd_tokloader_next.restype = ctypes.c_longlong
        lib.piamd_tokloader_seek.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
        lib.piamd_tokloader_seek.restype = None
        lib.piamd_tokloader_batches_per_epoch.argtypes = [ctypes.c_void_p]
        lib.piamd_tokloader_batches_per_epoch.restype = ctypes.c_longlong
        lib.piamd_tokloader_destroy.argtypes = [ctypes.c_void_p]
        lib.piamd_tokloader_destroy.restype = None
        _LIB = lib
    return _LIB


def write_token_file(path, tokens, dtype=np.uint16):
    """Write a flat token-id file (uint16 for vocab < 65536, else int32)."""
    np.ascontiguousarray(np.asarray(tokens), dtype=dtype).tofile(path)


class TokenDataLoader:
    """Infinite iterator of [batch, seq_len+1] int64 token windows.

    Args:
        path: flat binary token file.  dtype: np.uint16 or np.int32.
        rank / world_size: data-parallel coordinates (default: torch.distributed's).
        device: target device ('cuda:N' → async H2D via pinned buffers, 'cpu' → host tensors).
        prefetch: ring depth (batches prepared ahead by the native workers).
        start_batch: resume position (the loader is deterministic given seed, rank and world).
    """

    def __init__(self, path, seq_len, batch_size, dtype=np.uint16, seed=1234, rank=None,
                 world_size=None, device=None, prefetch=4, num_threads=2, start_batch=0):
        import torch.distributed as dist
        if rank is None:
            rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        if world_size is None:
            world_size = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        tb = np.dtype(dtype).itemsize
        if tb not in (2, 4):
            raise ValueError("token dtype must be 2 or 4 bytes")
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.seq_len, self.batch_size = int(seq_len), int(batch_size)
        self._h = _lib().piamd_tokloader_create(os.fsencode(path), tb, self.seq_len, self.batch_size,
                                                int(seed), int(rank), int(world_size),
                                                int(prefetch), int(num_threads))
        if not self._h:
            raise ValueError(f"cannot open token file {path} for seq_len={seq_len}, "
                             f"batch={batch_size}, world={world_size} (file too small?)")
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.batch_idx = int(start_batch)
        if start_batch:
            _lib().piamd_tokloader_seek(self._h, int(start_batch))
        self._cuda = self.device.type == "cuda"
        shape = (self.batch_size, self.seq_len + 1)
        if self._cuda:
            from ..device import side_stream
            self._stream = side_stream(self.device, key="token_loader")
            # two pinned staging buffers: one may still be in flight while the other is filled
            self._pinned = [torch.empty(shape, dtype=torch.int64).pin_memory() for _ in range(2)]
            self._events = [None, None]
            self._slot = 0

    @property
    def batches_per_epoch(self):
        return int(_lib().piamd_tokloader_batches_per_epoch(self._h))

    def state_dict(self):
        return {"batch_idx": self.batch_idx}

    def set_state_dict(self, sd):
        self.batch_idx = int(sd["batch_idx"])
        _lib().piamd_tokloader_seek(self._h, self.batch_idx)

    def __iter__(self):
        return self

    def __next__(self):
        shape = (self.batch_size, self.seq_len + 1)
        if not self._cuda:
            out = torch.empty(shape, dtype=torch.int64)
            self.batch_idx = _lib().piamd_tokloader_next(self._h, out.data_ptr()) + 1
            return out
        s = self._slot
        self._slot ^= 1
        if self._events[s] is not None:
            self._events[s].synchronize()  # previous H2D out of this staging buffer has finished
        buf = self._pinned[s]
        self.batch_idx = _lib().piamd_tokloader_next(self._h, buf.data_ptr()) + 1
        with torch.cuda.stream(self._stream):
            dev = buf.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._stream)
        self._events[s] = ev
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(ev)
        dev.record_stream(cur)
        return dev

    def close(self):
        if getattr(self, "_h", None):
            _lib().piamd_tokloader_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
