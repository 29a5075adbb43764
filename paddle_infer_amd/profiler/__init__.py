"""``paddle.profiler`` — Profiler / RecordEvent / schedulers / benchmark timer.

Parity: reference `python/paddle/profiler/profiler.py` (Profiler:340, make_scheduler:113,
export_chrome_tracing:211, step_info:684, summary:830), `utils.py` (RecordEvent) and `timer.py`
(the ips / reader_cost / batch_cost benchmark timer).

MI355X design: host + device activity come from torch.profiler (kineto over roctracer on ROCm,
i.e. the same HIP kernel records rocprofv3 sees); RecordEvent ranges are emitted both as profiler
record_function scopes and as roctx ranges (visible to ``rocprofv3 --marker-trace``). Chrome
traces open in Perfetto / chrome://tracing like the reference's.
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


class RecordEvent:
    """User range: ``with RecordEvent("name"):`` or ``e.begin() ... e.end()``."""

    def __init__(self, name: str, event_type=TracerEventType.PythonUserDefined):
        self.name, self.event_type = name, event_type
        self._rf = None
        self._pushed = False

    def begin(self):
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
                 with_flops=False):
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

    # -- torch profiler lifecycle ------------------------------------------------------------
    def _activities(self):
        acts = [torch.profiler.ProfilerActivity.CPU]
        if ProfilerTarget.GPU in self.targets and torch.cuda.is_available():
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        return acts

    def _open(self):
        if self._prof is None and not self.timer_only:
            self._prof = torch.profiler.profile(activities=self._activities(),
                                                record_shapes=self.record_shapes,
                                                profile_memory=self.profile_memory,
                                                with_flops=self.with_flops)
            self._prof.__enter__()

    def _close(self, deliver=True):
        if self._prof is not None:
            self._prof.__exit__(None, None, None)
            self._last_events = self._prof
            self._prof = None
            if deliver and self.on_trace_ready is not None:
                self.on_trace_ready(self)

    def _apply(self, state):
        if state in (ProfilerState.RECORD, ProfilerState.RECORD_AND_RETURN, ProfilerState.READY):
            self._open()
        elif self._prof is not None:
            self._close()
        self._state = state

    def start(self):
        self.timer.reset()
        self._apply(self.scheduler(self.step_num))

    def stop(self):
        if self._prof is not None:
            self._close()
        self._state = ProfilerState.CLOSED

    def step(self, num_samples=None):
        self.timer.step(num_samples)
        prev = self._state
        self.step_num += 1
        if prev == ProfilerState.RECORD_AND_RETURN and self._prof is not None:
            self._close()
        new = self.scheduler(self.step_num)
        if new != prev or self._prof is None:
            self._apply(new)

    def step_info(self, unit=None):
        return self.timer.info(unit or "samples")

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, *a):
        self.stop()

    # -- results --------------------------------------------------------------------------
    def export(self, path="", format="json"):
        src = self._prof or self._last_events
        if src is None:
            raise RuntimeError("no profiling data (record at least one step)")
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        src.export_chrome_trace(path)

    def summary(self, sorted_by=SortedKeys.CPUTotal, op_detail=True, thread_sep=False,
                time_unit="ms", views=None, row_limit=40):
        src = self._prof or self._last_events
        if src is None:
            print(self.step_info())
            return ""
        key = {SortedKeys.CPUTotal: "cpu_time_total", SortedKeys.CPUAvg: "cpu_time",
               SortedKeys.CPUMax: "cpu_time_total", SortedKeys.CPUMin: "cpu_time",
               SortedKeys.GPUTotal: "device_time_total", SortedKeys.GPUAvg: "device_time",
               SortedKeys.GPUMax: "device_time_total", SortedKeys.GPUMin: "device_time"}[sorted_by]
        try:
            table = src.key_averages().table(sort_by=key, row_limit=row_limit)
        except (KeyError, RuntimeError, AttributeError):
            table = src.key_averages().table(row_limit=row_limit)
        print(table)
        return table


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
