"""Native device runtime on the GPU: streams with priorities adopted by torch (ops and framework
kernels in a stream_guard run on the native stream), events (ordering, timing), device properties,
and the profiler's device-timed ranges; the static executor's comm stream is a native one."""
import json

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_native_stream_event_roundtrip():
    import paddle_infer_amd as paddle
    cuda = paddle.device.cuda
    hi, lo = cuda.Stream(priority=1), cuda.Stream(priority=2)
    assert hi.cuda_stream != lo.cuda_stream
    from paddle_infer_amd.framework import device_rt
    import ctypes
    p = ctypes.c_int()
    device_rt.lib().piamd_stream_get_priority(hi.cuda_stream, ctypes.byref(p))
    least, greatest = device_rt.priority_range()
    assert p.value == greatest
    x = torch.randn(4096, 4096, device="cuda")
    start, end = cuda.Event(enable_timing=True), cuda.Event(enable_timing=True)
    with cuda.stream_guard(hi):
        assert torch.cuda.current_stream().cuda_stream == hi.cuda_stream
        start.record()
        y = x @ x  # torch op on the native stream
        from paddle_infer_amd.ops.norm import layer_norm
        z = layer_norm(y, torch.ones(4096, device="cuda"), torch.zeros(4096, device="cuda"), 1e-5)
        end.record()
    lo.wait_event(end)  # cross-stream order through a native event
    with cuda.stream_guard(lo):
        w = z * 2
    lo.synchronize()
    assert end.query() and hi.query()
    assert start.elapsed_time(end) > 0
    ref = torch.nn.functional.layer_norm(x @ x, (4096,)) * 2
    torch.testing.assert_close(w, ref, rtol=1e-3, atol=1e-3)


def test_native_device_properties():
    import paddle_infer_amd as paddle
    p = paddle.device.cuda.get_device_properties(0)
    assert p.gcnArchName.startswith("gfx950") and p.multi_processor_count == 256
    assert p.warp_size == 64 and p.total_memory > 200 * (1 << 30)
    free, total = paddle.device.cuda.mem_get_info()
    assert 0 < free <= total


def test_profiler_device_ranges(tmp_path):
    from paddle_infer_amd import profiler as P
    x = torch.randn(2048, 2048, device="cuda")
    prof = P.Profiler(tracer="native")
    prof.start()
    with P.RecordEvent("matmul_block"):
        for _ in range(5):
            x = (x @ x).clamp(-1, 1)
    prof.stop()
    ev = prof.native_events()
    dev = [e for e in ev if e["cat"] == "device" and e["name"] == "matmul_block"]
    assert len(dev) == 1 and dev[0]["dur"] > 0
    prof.export(str(tmp_path / "t.json"))
    assert any(e.get("cat") == "device" for e in json.loads((tmp_path / "t.json").read_text())["traceEvents"])


def test_static_comm_stream_is_native():
    from paddle_infer_amd.device import side_stream, _SIDE
    s = side_stream(torch.device("cuda", 0), priority=1, key="static_comm")
    assert any(v.torch_stream is s and v.priority == 1 for v in _SIDE.values())


def test_device_level_stream_api():
    import paddle_infer_amd as paddle
    s = paddle.device.Stream(priority=1)
    prev = paddle.device.set_stream(s)
    try:
        assert paddle.device.current_stream().cuda_stream == s.cuda_stream
        y = torch.ones(8, device="cuda") * 3
    finally:
        paddle.device.set_stream(prev)
    s.synchronize()
    assert float(y.sum()) == 24.0 and paddle.device.current_stream().cuda_stream == prev.cuda_stream
