"""``paddle.device.cuda.graphs`` — user-facing HIP graph capture (reference
`python/paddle/device/cuda/graphs.py:38`: ``CUDAGraph`` with capture_begin / capture_end / replay /
reset / print_to_dot_files, ``wrap_cuda_graph``, ``is_cuda_graph_supported``).

On ROCm ``torch.cuda.CUDAGraph`` is a hipGraph: the capture runs on a dedicated side stream (graph
capture is illegal on the legacy default stream), every framework HIP kernel, hipBLASLt call and
RCCL collective issued between ``capture_begin`` and ``capture_end`` is recorded into one graph,
and ``replay`` launches it with one ``hipGraphLaunch``. Capture modes map one-to-one onto HIP's
stream-capture modes ("global", "thread_local", "relaxed"). Memory allocated inside the capture
comes from a graph-private pool (``pool_id`` shares one between graphs, as the reference's
memory_pool argument does).
"""
from __future__ import annotations

import os

import torch

ALL_MODES = ["global", "thread_local", "relaxed"]


def is_cuda_graph_supported() -> bool:
    return torch.cuda.is_available()


_POOLS: dict = {}


def _pool(pool_id):
    if pool_id is None:
        return None
    if pool_id not in _POOLS:
        _POOLS[pool_id] = torch.cuda.graph_pool_handle()
    return _POOLS[pool_id]


class CUDAGraph:
    def __init__(self, place=None, mode="thread_local", pool_id=None):
        assert is_cuda_graph_supported(), "HIP graphs need a GPU"
        assert mode in ALL_MODES, mode
        self._mode = mode
        idx = getattr(place, "index", None) if place is not None else None
        self._device = torch.device("cuda", idx if idx is not None else torch.cuda.current_device())
        self._pool_id = pool_id
        self._graph = None
        self._stream = None
        self._ctx = None
        self._debug = True

    def capture_begin(self):
        self._graph = torch.cuda.CUDAGraph()
        if self._debug:
            self._graph.enable_debug_mode()
        cur = torch.cuda.current_stream(self._device)
        self._stream = torch.cuda.Stream(device=self._device)
        self._stream.wait_stream(cur)
        self._ctx = torch.cuda.stream(self._stream)
        self._ctx.__enter__()
        self._graph.capture_begin(pool=_pool(self._pool_id), capture_error_mode=self._mode)

    def capture_end(self):
        try:
            self._graph.capture_end()
        finally:
            self._ctx.__exit__(None, None, None)
            torch.cuda.current_stream(self._device).wait_stream(self._stream)
            self._ctx = None

    def replay(self):
        self._graph.replay()

    def reset(self):
        if self._graph is not None:
            self._graph.reset()
        self._graph = None

    def print_to_dot_files(self, dirname, flags=None):
        if not isinstance(dirname, (str, bytes)):
            dirname = dirname.name
        os.makedirs(dirname, exist_ok=True)
        path = os.path.join(dirname, "hip_graph.dot")
        self._graph.debug_dump(path)
        return path


class _GraphedFn:
    """Dygraph ``wrap_cuda_graph``: the first call runs eagerly (warm-up: allocator, autotune and
    lazily built weight caches), the second captures into a graph on static copies of the inputs,
    every later call copies the new inputs into those buffers and replays."""

    def __init__(self, fn, mode, pool_id):
        self.fn, self.mode, self.pool_id = fn, mode, pool_id
        self.calls = 0
        self.graph = None
        self.static_in = None
        self.static_out = None

    def __call__(self, *args):
        tens = [a for a in args if isinstance(a, torch.Tensor)]
        if self.calls == 0 or not tens or not tens[0].is_cuda:
            self.calls += 1
            return self.fn(*args)
        if self.graph is None:
            self.static_in = [a.clone() if isinstance(a, torch.Tensor) else a for a in args]
            torch.cuda.synchronize()
            self.graph = CUDAGraph(mode=self.mode, pool_id=self.pool_id)
            self.graph._debug = False
            self.graph.capture_begin()
            try:
                self.static_out = self.fn(*self.static_in)
            finally:
                self.graph.capture_end()
        else:
            for s, a in zip(self.static_in, args):
                if isinstance(s, torch.Tensor):
                    assert s.shape == a.shape and s.dtype == a.dtype, "graphed call: input signature changed"
                    s.copy_(a)
        self.graph.replay()
        self.calls += 1
        return self.static_out


_NEXT_POOL = [1]


def wrap_cuda_graph(function, mode="thread_local", memory_pool="default"):
    """Graph-capture ``function`` (or a Layer's forward) — reference `graphs.py` wrap_cuda_graph.
    ``memory_pool``: "default" (shared pool 0), "new" (a private pool) or another wrapped function /
    Layer whose pool is shared."""
    assert mode in ALL_MODES
    if memory_pool == "default":
        pid = 0
    elif memory_pool == "new":
        pid = _NEXT_POOL[0]
        _NEXT_POOL[0] += 1
    else:
        src = memory_pool.forward if hasattr(memory_pool, "forward") and not isinstance(memory_pool, _GraphedFn) \
            else memory_pool
        pid = getattr(src, "pool_id", 0)
    if hasattr(function, "forward") and callable(function.forward) and not isinstance(function, _GraphedFn):
        g = _GraphedFn(function.forward, mode, pid)
        function.forward = g
        return function
    return _GraphedFn(function, mode, pid)
