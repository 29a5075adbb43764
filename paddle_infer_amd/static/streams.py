"""Multi-stream execution of static Programs: communication ops on their own stream.

Parity: reference `paddle/fluid/framework/new_executor/interpreter/stream_analyzer.cc` (each
instruction gets a device context / stream — collective ops `c_allreduce_*`, `c_reducescatter`,
`c_allgather`, `c_broadcast`, `send_v2` / `recv_v2`, … run on the communication stream — and
cross-stream dependencies become event waits) and `interpretercore.cc:907` (asynchronous
instruction scheduling with those events), plus the data-parallel gradient all-reduce of
`ParallelExecutor` (`fuse_all_reduce_op_pass`: bucketed, overlapped with the rest of backward).

* The plan (`csrc/runtime/scheduler.cc` ``piamd_stream_plan``) assigns stream 0 (compute) / 1
  (communication) and, per op, the minimal set of cross-stream events to wait on: the latest
  predecessor of the other stream, skipped when that stream already waited on it or a later one.
* On a GPU the communication ops run under a dedicated high-priority HIP stream (native, from
  ``csrc/device`` via ``device.side_stream``): RCCL
  is enqueued behind the events of the compute work that produced its inputs, the compute stream
  only waits where a consumer needs the result, and the allocator is told about cross-stream use
  (``record_stream``) so the executor's early frees stay safe.
* Without a GPU (gloo) the all-reduce family runs as asynchronous collectives
  (``async_op=True``) completed at the first op that waits on them per the same plan.
* ``GradBuckets``: the data-parallel gradient all-reduce of ``CompiledProgram.with_data_parallel``
  is issued per bucket as soon as the backward op producing the bucket's last gradient has run
  (buckets filled in production order, ``BUCKET_MB`` each), asynchronously, and waited for before
  the first optimizer op — instead of one blocking all-reduce after the whole backward.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

ALLREDUCE_OPS = {"c_allreduce_sum": "SUM", "mp_allreduce_sum": "SUM", "c_allreduce_max": "MAX",
                 "c_allreduce_min": "MIN", "c_allreduce_prod": "PRODUCT"}
COMM_OPS = set(ALLREDUCE_OPS) | {"c_reducescatter", "c_allgather", "c_broadcast", "send_v2", "recv_v2",
                                 "c_concat", "alltoall", "c_reduce_sum", "c_reduce_max", "partial_send",
                                 "partial_recv", "partial_allgather", "global_scatter", "global_gather"}
# xGMI ring all-reduce is per-link bound: large buckets amortise the per-collective latency; a
# bucket is still closed early enough to overlap the remaining backward
BUCKET_MB = float(os.environ.get("PIAMD_STATIC_DP_BUCKET_MB", "128"))


def stream_plan(ops, order):
    """(stream_of[op index], waits[position] → op indices, record[op index]) for ``ops`` issued
    in ``order`` (`piamd_stream_plan`)."""
    from .executor import runtime_lib, _arr
    names = {}
    for op in ops:
        for n in op.input_names() + op.output_names():
            names.setdefault(n, len(names))
    in_ptr, in_idx, out_ptr, out_idx = [0], [], [0], []
    for op in ops:
        in_idx += [names[n] for n in op.input_names()]
        in_ptr.append(len(in_idx))
        out_idx += [names[n] for n in op.output_names()]
        out_ptr.append(len(out_idx))
    nops = len(ops)
    lib = runtime_lib()
    if not getattr(lib, "_stream_sig", False):
        P = ctypes.POINTER
        i32p, u8p = P(ctypes.c_int), P(ctypes.c_ubyte)
        lib.piamd_stream_plan.argtypes = [ctypes.c_int, ctypes.c_int, i32p, i32p, i32p, i32p, i32p, u8p,
                                          i32p, i32p, i32p, u8p]
        lib.piamd_stream_plan.restype = ctypes.c_int
        lib._stream_sig = True
    a_ip, p_ip = _arr(in_ptr, ctypes.c_int)
    a_ii, p_ii = _arr(in_idx or [0], ctypes.c_int)
    a_op, p_op = _arr(out_ptr, ctypes.c_int)
    a_oi, p_oi = _arr(out_idx or [0], ctypes.c_int)
    a_or, p_or = _arr(list(order) or [0], ctypes.c_int)
    a_c, p_c = _arr([1 if op.type in COMM_OPS else 0 for op in ops] or [0], ctypes.c_ubyte)
    stream_of = np.zeros(max(nops, 1), np.int32)
    wait_ptr = np.zeros(nops + 1, np.int32)
    wait_idx = np.zeros(max(nops * 2, 1), np.int32)
    record = np.zeros(max(nops, 1), np.uint8)
    P = ctypes.POINTER(ctypes.c_int)
    rc = lib.piamd_stream_plan(nops, len(names), p_ip, p_ii, p_op, p_oi, p_or, p_c,
                               stream_of.ctypes.data_as(P), wait_ptr.ctypes.data_as(P),
                               wait_idx.ctypes.data_as(P), record.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)))
    if rc != 0:
        raise RuntimeError(f"piamd_stream_plan failed ({rc})")
    waits = [[int(v) for v in wait_idx[wait_ptr[i]:wait_ptr[i + 1]]] for i in range(nops)]
    return [int(s) for s in stream_of[:nops]], waits, [bool(r) for r in record[:nops]]


def _tensors(vals):
    for v in vals:
        if isinstance(v, torch.Tensor):
            yield v
        elif isinstance(v, (list, tuple)):
            yield from _tensors(v)


class StreamRunner:
    """Issues one Program run's ops on the compute / communication streams of the plan."""

    def __init__(self, device, stream_of, waits, record):
        self.stream_of, self.waits, self.record = stream_of, waits, record
        self.cuda = device.type == "cuda"
        self.events = {}
        self.pending = {}  # op index → async Work (CPU / gloo path)
        self.pending_out = {}  # op index → output names of that pending collective
        self.issued_on = {}  # op index → stream id, for tests / introspection
        if self.cuda:
            from ..device import side_stream
            self.compute = torch.cuda.current_stream(device)
            # native high-priority HIP stream: collectives are scheduled ahead of queued compute
            self.comm = side_stream(device, priority=1, key="static_comm")

    def run(self, pos, oi, op, run_fn, env):
        s = self.stream_of[oi]
        self.issued_on[oi] = s
        for a in self.waits[pos]:
            if self.cuda:
                ev = self.events.get(a)
                if ev is not None:
                    (self.comm if s else self.compute).wait_event(ev)
            else:
                w = self.pending.pop(a, None)
                if w is not None:
                    w.wait()
                    self.pending_out.pop(a, None)
        if not self.cuda and self.pending:
            # async collectives are not stream-ordered: an op reading the output of an earlier
            # pending collective (same "stream" or not) waits for that Work first
            ins = set(op.input_names())
            for a in [a for a, outs in self.pending_out.items() if outs & ins]:
                w = self.pending.pop(a, None)
                if w is not None:
                    w.wait()
                self.pending_out.pop(a, None)
        if not self.cuda:
            # forward-role collectives of a training program keep the executor's autograd leaves
            from .backward import op_role, FORWARD
            if (s == 1 and op.type in ALLREDUCE_OPS and op.func is None and op.paddle_inputs is not None
                    and (not torch.is_grad_enabled() or op_role(op) != FORWARD)
                    and self._async_allreduce(oi, op, env)):
                return
            run_fn()
            return
        if s == 0:
            run_fn()
            if self.record[oi]:
                ev = torch.cuda.Event()
                ev.record(self.compute)
                self.events[oi] = ev
            return
        ins = [env.get(n) for n in op.input_names()]
        for t in _tensors(ins):
            if t.is_cuda:
                t.record_stream(self.comm)
        with torch.cuda.stream(self.comm):
            run_fn()
        for t in _tensors([env.get(n) for n in op.output_names()]):
            if t.is_cuda:
                t.record_stream(self.compute)
        if self.record[oi]:
            ev = torch.cuda.Event()
            ev.record(self.comm)
            self.events[oi] = ev

    def _async_allreduce(self, oi, op, env):
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return False
        from .ops_registry_ext import _group
        x = env.get(op.input_names()[0]) if op.input_names() else None
        if not isinstance(x, torch.Tensor):
            return False
        g = _group(op.attrs)
        out = x.detach().clone()
        if dist.get_world_size(g) > 1:
            self.pending[oi] = dist.all_reduce(out, op=getattr(dist.ReduceOp, ALLREDUCE_OPS[op.type]),
                                               group=g, async_op=True)
            self.pending_out[oi] = set(op.output_names())
        for n in op.output_names():
            env[n] = out
        return True

    def finish(self):
        """Every outstanding collective complete (end of the run), compute stream behind comm."""
        for w in self.pending.values():
            w.wait()
        self.pending.clear()
        self.pending_out.clear()
        if self.cuda:
            self.compute.wait_stream(self.comm)


class GradBuckets:
    """Data-parallel gradient all-reduce in buckets launched during backward (see module doc)."""

    def __init__(self, ops, order, grad_names, size_of=None, bucket_mb=None, world=1):
        self.world = world
        size_of = size_of or (lambda n: 0)
        import sys
        limit = (bucket_mb if bucket_mb is not None else sys.modules[__name__].BUCKET_MB) * (1 << 20)
        produced = {}
        for pos, oi in enumerate(order):
            for n in ops[oi].output_names():
                if n in grad_names:
                    produced[n] = pos  # the last write of the gradient
        names = sorted(produced, key=lambda n: produced[n])
        self.buckets, self.launch_at = [], {}
        cur, cur_bytes = [], 0.0
        for n in names:
            cur.append(n)
            cur_bytes += size_of(n)
            if cur_bytes >= limit:
                self.buckets.append(cur)
                cur, cur_bytes = [], 0.0
        if cur:
            self.buckets.append(cur)
        for bi, b in enumerate(self.buckets):
            self.launch_at.setdefault(max(produced[n] for n in b), []).append(bi)
        self.works = []
        self.flat = {}        # (bucket, dtype, device) → (layout, persistent flat buffer)
        self.flat_allocs = 0  # flat buffers allocated so far (tests: none after the first run)

    def after(self, pos, env):
        """Launch every bucket completed at position ``pos``: its gradients are packed into the
        bucket's PERSISTENT flat buffer (allocated on the first run, reused every step) and
        all-reduced asynchronously."""
        import torch.distributed as dist
        for bi in self.launch_at.get(pos, ()):
            ts = [(n, env[n]) for n in self.buckets[bi] if isinstance(env.get(n), torch.Tensor)]
            if not ts:
                continue
            by_dtype = {}
            for n, t in ts:
                by_dtype.setdefault((t.dtype, t.device), []).append((n, t))
            for (dt, dev), group in by_dtype.items():
                layout = tuple((n, tuple(t.shape)) for n, t in group)
                key = (bi, dt, dev)
                ent = self.flat.get(key)
                if ent is None or ent[0] != layout:
                    total = sum(t.numel() for _, t in group)
                    ent = self.flat[key] = (layout, torch.empty(total, dtype=dt, device=dev))
                    self.flat_allocs += 1
                flat = ent[1]
                off = 0
                views = []
                for n, t in group:
                    k = t.numel()
                    v = flat[off:off + k]
                    if t.data_ptr() != v.data_ptr():
                        v.copy_(t.detach().reshape(-1))
                    views.append((n, v.view(t.shape), t))
                    off += k
                self.works.append((dist.all_reduce(flat, async_op=True), flat, views))

    def wait(self, env=None):
        """All buckets reduced and averaged (before the optimizer ops). With ``env`` the gradient
        names are re-bound to views of the flat buffers — no copy back."""
        for work, flat, views in self.works:
            work.wait()
            flat.div_(self.world)
            for n, v, t in views:
                if env is not None and env.get(n) is t:
                    env[n] = v
                else:
                    with torch.no_grad():
                        t.copy_(v)
        self.works = []
