"""Own auto-growth best-fit HIP allocator (csrc/alloc/allocator.cc) installed through
FLAGS_allocator_strategy=auto_growth in a fresh process: a GPT train step and inference run on
it with the same loss as PyTorch's caching allocator, blocks are reused (few chunk hipMallocs for
many allocations), the paddle memory-stat APIs report its counters, and empty_cache returns
wholly free chunks."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import json, sys, torch
sys.path.insert(0, sys.argv[1])
import paddle_infer_amd as paddle
from paddle_infer_amd.framework import allocator
from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config
torch.manual_seed(0)
dev = torch.device("cuda", 0)
cfg = gpt_config("gpt3-tiny", hidden_size=256, num_heads=2, num_layers=2, vocab_size=1024)
with torch.device(dev):
    m = GPTForPretraining(cfg)
opt = paddle.optimizer.AdamW(learning_rate=1e-3, parameters=m.parameters())
g = torch.Generator(device=dev).manual_seed(1)
ids = torch.randint(0, 1024, (2, 129), device=dev, generator=g)
losses = []
for _ in range(3):
    loss = m(ids[:, :-1], labels=ids[:, 1:])
    loss.backward()
    opt.step()
    opt.clear_grad()
    losses.append(loss.item())
torch.cuda.synchronize()
big = torch.empty(300 << 20, dtype=torch.uint8, device=dev)
del big
torch.cuda.synchronize()
out = {"active": allocator.active(), "losses": losses}
if allocator.active():
    s = allocator.stats(0)
    out["stats"] = s
    out["api_alloc"] = paddle.device.cuda.memory_allocated(0)
    out["api_peak"] = paddle.device.cuda.max_memory_allocated()
    paddle.device.cuda.empty_cache()
    out["after_release"] = allocator.stats(0)
print("RESULT " + json.dumps(out))
"""


def _run(env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", SCRIPT, ROOT], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")][-1]
    return json.loads(line[7:])


def test_auto_growth_allocator_end_to_end():
    ref = _run({"FLAGS_allocator_strategy": "naive_best_fit"})
    own = _run({"FLAGS_allocator_strategy": "auto_growth", "PIAMD_ALLOC_CHUNK_MB": "64"})
    assert not ref["active"] and own["active"]
    for a, b in zip(own["losses"], ref["losses"]):
        assert abs(a - b) < 1e-3 * max(1.0, abs(b)), (own["losses"], ref["losses"])
    s = own["stats"]
    assert s["num_alloc"] > 20 * s["num_chunk_alloc"]  # blocks are reused, chunks are few
    assert s["peak_allocated"] >= (300 << 20)
    assert s["reserved"] >= s["allocated"] > 0
    assert own["api_alloc"] == s["allocated"] and own["api_peak"] == s["peak_allocated"]
    # the 300 MiB chunk (wholly free after `del big`) is returned to the device
    assert own["after_release"]["reserved"] <= s["reserved"] - (300 << 20)


STREAM_GRAPH = r"""
import json, sys, torch
sys.path.insert(0, sys.argv[1])
import paddle_infer_amd as paddle
from paddle_infer_amd.framework import allocator
assert allocator.active()
dev = torch.device("cuda", 0)
out = {}
# 1) record_stream: a block used on a side stream is not handed out before that stream's work ends
side = torch.cuda.Stream()
x = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
xp = x.data_ptr()
torch.cuda.synchronize()
with torch.cuda.stream(side):
    torch.cuda._sleep(200_000_000)  # keep the side stream busy
    x.fill_(7)
x.record_stream(side)
del x
y = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
out["reused_while_busy"] = y.data_ptr() == xp
side.synchronize()
del y
z1 = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
z2 = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
out["reused_after"] = xp in (z1.data_ptr(), z2.data_ptr())  # the deferred block is back in use
del z1, z2
# 2) hipGraph capture into a private pool, replayed; outside allocations never alias it
a = torch.randn(1 << 20, device=dev)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        b = a * 2.0 + 1.0
    torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(g):
    tmp = a * 3.0
    b = tmp + 1.0
gp = {b.data_ptr(), tmp.data_ptr()}
del tmp
outside = [torch.empty(4 << 20, dtype=torch.uint8, device=dev) for _ in range(8)]
out["alias"] = any(o.data_ptr() in gp for o in outside)
a.copy_(torch.ones_like(a))
g.replay()
torch.cuda.synchronize()
out["graph_ok"] = bool(torch.all(b == 4.0).item())
out["api_peak"] = torch.cuda.max_memory_allocated() == allocator.stats(0)["peak_allocated"]
print("RESULT " + json.dumps(out))
"""


def test_record_stream_and_graph_pools():
    env = dict(os.environ, FLAGS_allocator_strategy="auto_growth", PIAMD_ALLOC_CHUNK_MB="64")
    r = subprocess.run([sys.executable, "-c", STREAM_GRAPH, ROOT], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("RESULT ")][-1][7:])
    assert not out["reused_while_busy"] and out["reused_after"], out
    assert not out["alias"] and out["graph_ok"] and out["api_peak"], out
