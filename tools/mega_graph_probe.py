"""Bench-order probe of the single-launch decode step: generate(4) → prefill ×3 → decode graph
loop with argmax feedback (tools/bench_generate.py's sequence), with the phase trace of the
last launch. Usage: PIAMD_DECODE_MEGA=1 python tools/mega_graph_probe.py"""
import os, sys, time, json
os.environ.setdefault("PIAMD_DECODE_MEGA", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import paddle_infer_amd as paddle
from paddle_infer_amd.inference.generation import GPTGenerator
from paddle_infer_amd.inference.mega_decode import MegaDecoder
from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config
paddle.seed(0)
cfg = gpt_config("gpt3-1.3b", hidden_dropout_prob=0.0, max_position_embeddings=2048)
with torch.device("cuda"):
    model = GPTForPretraining(cfg)
model = model.cuda().to(torch.bfloat16).eval()
gen = GPTGenerator(model, max_batch=1, max_seq_len=264, use_hip_graph=True)
LAZY, TRACE = "--lazy" in sys.argv, "--notrace" not in sys.argv
if not LAZY:
    gen._mega[1] = MegaDecoder(gen)
    if TRACE:
        gen._mega[1].trace = torch.zeros(256, 5 * gen._mega[1].nl, 4, dtype=torch.int64, device="cuda")
ids = torch.randint(0, cfg.vocab_size, (1, 128), device="cuda")
lens = torch.full((1,), 128, device="cuda")
gen.generate(ids, lens, max_new_tokens=4)
for _ in range(3):
    gen.prefill(ids, lens)
tok = torch.zeros(1, dtype=torch.long, device="cuda")
pos = torch.full((1,), 128, dtype=torch.int32, device="cuda")
gen.decode(tok, pos)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(16):
    logits = gen.decode(tok, pos + i)
    tok = logits.argmax(-1)
torch.cuda.synchronize()
print("lazy", LAZY, "trace", TRACE, "ms/step", (time.perf_counter() - t0) / 16 * 1e3,
      "timeouts", int(gen._mega[1].err.item()))
if "--eager-after" in sys.argv:  # same process, same generator, no graph
    gen.use_graph = False
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for i in range(16):
        logits = gen.decode(tok, pos + i)
        tok = logits.argmax(-1)
    torch.cuda.synchronize()
    print("eager-after ms/step", (time.perf_counter() - t0) / 16 * 1e3)
if LAZY or not TRACE:
    sys.exit(0)
nl = gen._mega[1].nl
tr = gen._mega[1].trace.cpu().double() * 0.01  # µs
st, pro, gem, arr = tr[..., 0], tr[..., 1], tr[..., 2], tr[..., 3]
t0 = st[:, 0].min()
for p in list(range(0, 10)) + [5 * nl - 2]:
    print(p, "start med %.1f max %.1f | pro %.1f gemv %.1f epi %.1f | arrive max %.1f" % (
        (st[:, p] - t0).median(), (st[:, p] - t0).max(), (pro[:, p] - st[:, p]).median(),
        (gem[:, p] - pro[:, p]).median(), (arr[:, p] - gem[:, p]).median(), (arr[:, p] - t0).max()))
# slowest workgroups in phase 0
w = (arr[:, 0] - st[:, 0]).argsort(descending=True)[:4]
print("slow wgs phase0", w.tolist(), (arr[w, 0] - st[w, 0]).tolist())
