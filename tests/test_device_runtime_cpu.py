"""Native device runtime (csrc/device) on the CPU tier: the host range tracer behind
paddle.profiler (nested RecordEvent ranges, chrome-trace export, UDF summary) — no GPU needed."""
import json
import threading

import paddle_infer_amd as paddle
from paddle_infer_amd import profiler as P
from paddle_infer_amd.framework import device_rt


def test_native_tracer_ranges_export_and_summary(tmp_path):
    assert device_rt.available()
    prof = P.Profiler(targets=[P.ProfilerTarget.CPU], tracer="native")
    prof.start()
    with P.RecordEvent("outer"):
        for _ in range(3):
            with P.RecordEvent("inner"):
                sum(range(1000))

    def worker():
        with P.RecordEvent("thread_range"):
            pass
    t = threading.Thread(target=worker)
    t.start()
    t.join()
    prof.stop()
    ev = prof.native_events()
    names = [e["name"] for e in ev if e["cat"] == "host"]
    assert names.count("inner") == 3 and names.count("outer") == 1 and "thread_range" in names
    outer = next(e for e in ev if e["name"] == "outer")
    inner = [e for e in ev if e["name"] == "inner"]
    assert all(e["args"]["depth"] == 1 for e in inner) and outer["args"]["depth"] == 0
    assert all(outer["ts"] <= e["ts"] and e["ts"] + e["dur"] <= outer["ts"] + outer["dur"] + 1e-3 for e in inner)
    assert len({e["tid"] for e in ev}) == 2  # the worker thread has its own track
    path = tmp_path / "trace.json"
    prof.export(str(path))
    doc = json.loads(path.read_text())
    assert sum(e.get("name") == "inner" for e in doc["traceEvents"]) == 3
    table = prof.summary()
    assert "UDF range" in table and "inner" in table


def test_ranges_outside_a_recording_are_not_kept():
    prof = P.Profiler(targets=[P.ProfilerTarget.CPU], tracer="native")
    with P.RecordEvent("before"):
        pass
    prof.start()
    with P.RecordEvent("during"):
        pass
    prof.stop()
    with P.RecordEvent("after"):
        pass
    assert [e["name"] for e in prof.native_events()] == ["during"]
    assert paddle.device.cuda.Stream is not None
