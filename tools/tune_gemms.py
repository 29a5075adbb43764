"""Tune every GEMM of the GPT-3 1.3B training step with PyTorch TunableOp (hipBLASLt + rocBLAS
solution spaces) and write the in-tree table ``paddle_infer_amd/tuning/tunableop_gfx950.csv``.
Run on the GPU: ``python tools/tune_gemms.py [--micro-batch 32]``."""
import argparse
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--micro-batch", type=int, default=32)
    ap.add_argument("--max-ms", type=int, default=300)
    a = ap.parse_args()
    table = os.path.join(ROOT, "paddle_infer_amd", "tuning", "tunableop_gfx950.csv")
    if os.path.exists(table):
        os.remove(table)
    env = dict(os.environ, PYTORCH_TUNABLEOP_ENABLED="1", PYTORCH_TUNABLEOP_TUNING="1",
               PYTORCH_TUNABLEOP_FILENAME=table, PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=str(a.max_ms),
               PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE="0")
    p = subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--steps", "1",
                          "--warmup", "1", "--micro-batch", str(a.micro_batch)], env=env)
    t0 = time.time()
    while p.poll() is None:  # heartbeat: tuning prints nothing for minutes
        time.sleep(20)
        n = sum(1 for _ in open(table)) if os.path.exists(table) else 0
        print(f"[tune] {time.time() - t0:.0f}s, table lines so far: {n}", flush=True)
    import glob
    for f in glob.glob(table[:-4] + "*.csv"):  # TunableOp inserts the device ordinal
        if f != table:
            os.replace(f, table)
    print(f"[tune] table: {table} exists={os.path.exists(table)}", flush=True)
    sys.exit(p.returncode)
