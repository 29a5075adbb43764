"""Find host synchronisations in the eager single-launch decode step (torch sync-debug mode) and
time the step's host-side cost. Usage: python tools/mega_sync_probe.py"""
import os, sys, time
os.environ.setdefault("PIAMD_DECODE_MEGA", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import paddle_infer_amd as paddle
from paddle_infer_amd.inference.generation import GPTGenerator
from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config
paddle.seed(0)
cfg = gpt_config("gpt3-1.3b", num_layers=4, hidden_dropout_prob=0.0)
m = GPTForPretraining(cfg).cuda().to(torch.bfloat16).eval()
gen = GPTGenerator(m, max_batch=1, max_seq_len=264, use_hip_graph=True)
ids = torch.randint(0, cfg.vocab_size, (1, 128), device="cuda")
lg = gen.prefill(ids, torch.full((1,), 128, device="cuda"))
tok = lg.argmax(-1)
pos = torch.full((1,), 128, dtype=torch.int32, device="cuda")
gen.decode(tok, pos)
torch.cuda.synchronize()
torch.cuda.set_sync_debug_mode("warn")
import warnings
with warnings.catch_warnings(record=True) as ws:
    warnings.simplefilter("always")
    lg = gen.decode(tok, pos + 1)
torch.cuda.set_sync_debug_mode(0)
for w in ws:
    print("SYNC:", str(w.message)[:200])
import traceback
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(50):
    lg = gen.decode(tok, pos + i)
t_host = (time.perf_counter() - t0) / 50
torch.cuda.synchronize()
t_all = (time.perf_counter() - t0) / 50
print("host ms/step %.3f  total ms/step %.3f" % (t_host * 1e3, t_all * 1e3))
