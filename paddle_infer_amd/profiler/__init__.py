"""``paddle.profiler`` — Profiler / RecordEvent / schedulers / benchmark timer.

Parity: reference `python/paddle/profiler/profiler.py` (Profiler:340, make_scheduler:113,
export_chrome_tracing:211, step_info:684, summary:830), `utils.py` (RecordEvent) and `timer.py`
(the ips / reader_cost / batch_cost benchmark timer).

MI355X design: the framework's own tracer (``csrc/device/device.cc``, reference
`fluid/platform/profiler/host_tracer.cc` + `chrometracing_logger.cc`) records every RecordEvent
range natively — a per-thread append-only log, plus a HIP event pair per range on the current
stream when the GPU target is on, resolved only at export — and writes them into the exported
chrome trace (pid "host ranges" / "device ranges") and the summary's UDF view. Per-kernel device
activity comes from roctracer through torch.profiler's kineto (the ROCm analogue of the
reference's CUPTI tracer; ``tracer="native"`` skips it for a low-overhead ranges-only profile).
RecordEvent ranges are also roctx ranges (``rocprofv3 --marker-trace``). Chrome traces open in
Perfetto / chrome://tracing like the reference's.
"""
from __future__ import annotations

import enum
import json
import os
import time

import torch


class ProfilerState(enum.Enum):
    CLOSED = 0
    READY = 1
    RECORD = 2
    RECORD_AND_RETURN = 3


class ProfilerTarget(enum.Enum):
    CPU = 0
    GPU = 1
    MLU = 2
    CUSTOM_DEVICE = 3


class SortedKeys(enum.Enum):
    CPUTotal = 0
    CPUAvg = 1
    CPUMax = 2
    CPUMin = 3
    GPUTotal = 4
    GPUAvg = 5
    GPUMax = 6
    GPUMin = 7


class SummaryView(enum.Enum):
    DeviceView = 0
    OverView = 1
    ModelView = 2
    DistributedView = 3
    KernelView = 4
    OperatorView = 5
    MemoryView = 6
    MemoryManipulationView = 7
    UDFView = 8


class TracerEventType(enum.Enum):
    Operator = 0
    Dataloader = 1
    ProfileStep = 2
    CudaRuntime = 3
    Kernel = 4
    Memcpy = 5
    Memset = 6
    UserDefined = 7
    OperatorInner = 8
    Forward = 9
    Backward = 10
    Optimization = 11
    Communication = 12
    PythonOp = 13
    PythonUserDefined = 14


def make_scheduler(*, closed: int, ready: int, record: int, repeat: int = 0, skip_first: int = 0):
    period = closed + ready + record

    def fn(step):
        s = step - skip_first
        if s < 0:
            return ProfilerState.CLOSED
        if repeat > 0 and s // period >= repeat:
            return ProfilerState.CLOSED
        m = s % period
        if m < closed:
            return ProfilerState.CLOSED
        if m < closed + ready:
            return ProfilerState.READY
        return ProfilerState.RECORD_AND_RETURN if m == period - 1 else ProfilerState.RECORD
    fn._args = (closed, ready, record, repeat, skip_first)
    return fn


def _default_state_scheduler(step):
    return ProfilerState.RECORD


def export_chrome_tracing(dir_name: str, worker_name: str | None = None):
    os.makedirs(dir_name, exist_ok=True)

    def handle_fn(prof):
        name = worker_name or f"host_{os.uname().nodename}pid_{os.getpid()}"
        path = os.path.join(dir_name, f"{name}_time_{time.strftime('%Y_%m_%d_%H_%M_%S')}.paddle_trace.json")
        prof.export(path, "json")
    return handle_fn


def export_protobuf(dir_name: str, worker_name: str | None = None):
    return export_chrome_tracing(dir_name, worker_name)


def _roctx_push(name):
    try:
        torch.cuda.nvtx.range_push(name)  # roctx on ROCm builds
        return True
    except Exception:  # noqa: BLE001
        return False


def _roctx_pop():
    try:
        torch.cuda.nvtx.range_pop()
    except Exception:  # noqa: BLE001
        pass


_NATIVE = {"on": False}


def _native():
    """The device-runtime library when the native tracer is recording, else None."""
    if not _NATIVE["on"]:
        return None
    from ..framework import device_rt
    return device_rt.lib()


def _cur_stream():
    return torch.cuda.current_stream().cuda_stream if torch.cuda.is_available() else None


class RecordEvent:
    """User range: ``with RecordEvent("name"):`` or ``e.begin() ... e.end()``."""

    def __init__(self, name: str, event_type=TracerEventType.PythonUserDefined):
        self.name, self.event_type = name, event_type
        self._rf = None
        self._pushed = False
        self._nat = False

    def begin(self):
        L = _native()
        if L is not None:
            L.piamd_trace_push(self.name.encode(), _cur_stream())
            self._nat = True
        self._rf = torch.profiler.record_function(self.name)
        self._rf.__enter__()
        self._pushed = torch.cuda.is_available() and _roctx_push(self.name)

    def end(self):
        if self._rf is not None:
            self._rf.__exit__(None, None, None)
            self._rf = None
        if self._pushed:
            _roctx_pop()
            self._pushed = False
        if self._nat:
            L = _native()
            if L is not None:
                L.piamd_trace_pop(_cur_stream())
            self._nat = False

    def __enter__(self):
        self.begin()
        return self

    def __exit__(self, *a):
        self.end()


class _Timer:
    """Benchmark timer (reference profiler/timer.py): reader_cost, batch_cost, ips."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.steps, self.samples = 0, 0
        self.batch_cost = self.reader_cost = 0.0
        self._t_step = time.perf_counter()
        self._t_reader = None

    def before_reader(self):
        self._t_reader = time.perf_counter()

    def after_reader(self):
        if self._t_reader is not None:
            self.reader_cost += time.perf_counter() - self._t_reader
            self._t_reader = None

    def step(self, num_samples=None):
        now = time.perf_counter()
        self.batch_cost += now - self._t_step
        self._t_step = now
        self.steps += 1
        if num_samples:
            self.samples += num_samples

    def info(self, unit="samples"):
        n = max(self.steps, 1)
        bc, rc = self.batch_cost / n, self.reader_cost / n
        s = f"reader_cost: {rc:.5f} s batch_cost: {bc:.5f} s"
        if self.samples:
            s += f" ips: {self.samples / max(self.batch_cost, 1e-12):.3f} {unit}/s"
        return s


benchmark = _Timer


class Profiler:
    def __init__(self, *, targets=None, scheduler=None, on_trace_ready=None, record_shapes=False,
                 profile_memory=False, timer_only=False, emit_nvtx=False, custom_device_types=None,
                 with_flops=False, tracer="both"):
        targets = list(targets or [ProfilerTarget.CPU] + ([ProfilerTarget.GPU] if torch.cuda.is_available() else []))
        self.targets = targets
        if scheduler is None:
            self.scheduler = _default_state_scheduler
        elif isinstance(scheduler, (tuple, list)):
            start, end = scheduler
            self.scheduler = make_scheduler(closed=max(start - 1, 0), ready=1 if start > 0 else 0,
                                            record=end - start, repeat=1)
        else:
            self.scheduler = scheduler
        self.on_trace_ready = on_trace_ready
        self.record_shapes, self.profile_memory, self.with_flops = record_shapes, profile_memory, with_flops
        self.timer_only = timer_only
        self.timer = _Timer()
        self.step_num = 0
        self._prof = None
        self._state = ProfilerState.CLOSED
        self._last_events = None
        # "both": native ranges + kineto kernel activity; "native": ranges only (no kineto)
        self.tracer = tracer
        self._native_trace = None  # path of the last native dump
        self._native_open = False

    # -- torch profiler lifecycle ------------------------------------------------------------
    def _activities(self):
        acts = [torch.profiler.ProfilerActivity.CPU]
        if ProfilerTarget.GPU in self.targets and torch.cuda.is_available():
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        return acts

    def _open(self):
        if self.timer_only:
            return
        if not self._native_open:
            from ..framework import device_rt
            if device_rt.available():
                dev = ProfilerTarget.GPU in self.targets and torch.cuda.is_available()
                device_rt.lib().piamd_trace_enable(1, int(dev), _cur_stream() if dev else None)
                _NATIVE["on"] = self._native_open = True
        if self._prof is None and self.tracer != "native":
            self._prof = torch.profiler.profile(activities=self._activities(),
                                                record_shapes=self.record_shapes,
                                                profile_memory=self.profile_memory,
                                                with_flops=self.with_flops)
            self._prof.__enter__()

    def _close_native(self):
        if not self._native_open:
            return
        import tempfile
        from ..framework import device_rt
        L = device_rt.lib()
        L.piamd_trace_enable(0, 0, None)
        _NATIVE["on"] = self._native_open = False
        fd, path = tempfile.mkstemp(suffix=".native_trace.json")
        os.close(fd)
        L.piamd_trace_dump(path.encode(), 0)
        self._native_trace = path

    def _close(self, deliver=True):
        opened = self._prof is not None or self._native_open
        self._close_native()
        if self._prof is not None:
            self._prof.__exit__(None, None, None)
            self._last_events = self._prof
            self._prof = None
        if opened and deliver and self.on_trace_ready is not None:
            self.on_trace_ready(self)

    def _apply(self, state):
        if state in (ProfilerState.RECORD, ProfilerState.RECORD_AND_RETURN, ProfilerState.READY):
            self._open()
        elif self._prof is not None or self._native_open:
            self._close()
        self._state = state

    def start(self):
        self.timer.reset()
        self._apply(self.scheduler(self.step_num))

    def stop(self):
        if self._prof is not None or self._native_open:
            self._close()
        self._state = ProfilerState.CLOSED

    def step(self, num_samples=None):
        self.timer.step(num_samples)
        prev = self._state
        self.step_num += 1
        if prev == ProfilerState.RECORD_AND_RETURN and (self._prof is not None or self._native_open):
            self._close()
        new = self.scheduler(self.step_num)
        if new != prev or (self._prof is None and not self._native_open):
            self._apply(new)

    def step_info(self, unit=None):
        return self.timer.info(unit or "samples")

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, *a):
        self.stop()

    # -- results --------------------------------------------------------------------------
    def native_events(self):
        """The native tracer's events of the last recording (chrome-trace dicts: cat "host" /
        "device")."""
        if self._native_trace is None or not os.path.exists(self._native_trace):
            return []
        with open(self._native_trace) as f:
            return json.load(f).get("traceEvents", [])

    def export(self, path="", format="json"):
        src = self._prof or self._last_events
        nat = self.native_events()
        if src is None and not nat:
            raise RuntimeError("no profiling data (record at least one step)")
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        if src is not None:
            src.export_chrome_trace(path)
            with open(path) as f:
                doc = json.load(f)
        else:
            doc = {"traceEvents": [], "displayTimeUnit": "ms"}
        # the native ranges on their own processes (names shown by the metadata events)
        base = 1 << 20
        for e in nat:
            e = dict(e)
            e["pid"] = base + (1 if e.get("cat") == "device" else 0)
            doc.setdefault("traceEvents", []).append(e)
        for off, label in ((0, "paddle host ranges"), (1, "paddle device ranges (HIP events)")):
            doc["traceEvents"].append({"ph": "M", "name": "process_name", "pid": base + off,
                                       "args": {"name": label}})
        with open(path, "w") as f:
            json.dump(doc, f)

    def summary(self, sorted_by=SortedKeys.CPUTotal, op_detail=True, thread_sep=False,
                time_unit="ms", views=None, row_limit=40):
        src = self._prof or self._last_events
        if src is None and not self.native_events():
            print(self.step_info())
            return ""
        key = {SortedKeys.CPUTotal: "cpu_time_total", SortedKeys.CPUAvg: "cpu_time",
               SortedKeys.CPUMax: "cpu_time_total", SortedKeys.CPUMin: "cpu_time",
               SortedKeys.GPUTotal: "device_time_total", SortedKeys.GPUAvg: "device_time",
               SortedKeys.GPUMax: "device_time_total", SortedKeys.GPUMin: "device_time"}[sorted_by]
        table = ""
        if src is not None:
            try:
                table = src.key_averages().table(sort_by=key, row_limit=row_limit)
            except (KeyError, RuntimeError, AttributeError):
                table = src.key_averages().table(row_limit=row_limit)
        udf = self._udf_table(time_unit)
        table = table + ("\n" if table and udf else "") + udf
        print(table)
        return table

    def _udf_table(self, time_unit="ms"):
        """UDF view (reference summary ``SummaryView.UDFView``): per RecordEvent name, calls and
        host / device time from the native tracer."""
        nat = self.native_events()
        if not nat:
            return ""
        scale = {"s": 1e-6, "ms": 1e-3, "us": 1.0, "ns": 1e3}.get(time_unit, 1e-3)
        agg = {}
        for e in nat:
            a = agg.setdefault(e["name"], {"calls": 0, "host": 0.0, "dev": 0.0, "ndev": 0})
            if e.get("cat") == "device":
                a["dev"] += e["dur"]
                a["ndev"] += 1
            else:
                a["calls"] += 1
                a["host"] += e["dur"]
        rows = [f"{'UDF range':40s} {'calls':>7s} {'host total':>12s} {'host avg':>10s} "
                f"{'device total':>13s} {'device avg':>11s}   ({time_unit})"]
        for name, a in sorted(agg.items(), key=lambda kv: -kv[1]["host"]):
            n, nd = max(a["calls"], 1), max(a["ndev"], 1)
            rows.append(f"{name[:40]:40s} {a['calls']:7d} {a['host'] * scale:12.4f} {a['host'] * scale / n:10.4f} "
                        f"{a['dev'] * scale:13.4f} {a['dev'] * scale / nd:11.4f}")
        return "\n".join(rows)


def load_profiler_result(filename: str):
    with open(filename) as f:
        return json.load(f)


def get_profiler(config_path):
    with open(config_path) as f:
        cfg = json.load(f)
    return Profiler(timer_only=cfg.get("timer_only", False))


__all__ = ["Profiler", "ProfilerState", "ProfilerTarget", "RecordEvent", "make_scheduler",
           "export_chrome_tracing", "export_protobuf", "load_profiler_result", "SortedKeys",
           "SummaryView", "TracerEventType"]
