"""``python -m paddle_infer_amd.distributed.launch`` — multi-process launcher with a watchdog.

Parity: reference `python/paddle/distributed/launch/` (collective controller, `--nproc_per_node`,
`--devices`, `--log_dir`, `--max_restart` elastic restarts) and the failure detection of
`fleet/elastic`: one process per GPU gets RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT (and
Paddle's PADDLE_TRAINER_ID/PADDLE_TRAINERS_NUM/FLAGS_selected_gpus); the watchdog polls the
children, and when one exits non-zero (crash, OOM, hang killed by --timeout) it terminates the
whole job and, if restarts remain, relaunches every rank (all-or-nothing, like the reference's
elastic collective mode). Per-rank logs go to ``--log_dir/workerlog.<rank>``.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _start(args, rank_base, world, port, restart):
    procs = []
    os.makedirs(args.log_dir, exist_ok=True)
    devices = args.devices.split(",") if args.devices else [str(i) for i in range(args.nproc_per_node)]
    for lr in range(args.nproc_per_node):
        rank = rank_base + lr
        env = dict(os.environ)
        env.update({"RANK": str(rank), "LOCAL_RANK": str(lr), "WORLD_SIZE": str(world),
                    "MASTER_ADDR": args.master_addr, "MASTER_PORT": str(port),
                    "PADDLE_TRAINER_ID": str(rank), "PADDLE_TRAINERS_NUM": str(world),
                    "FLAGS_selected_gpus": devices[lr % len(devices)],
                    "PADDLE_RESTART_COUNT": str(restart),
                    "HSA_ENABLE_IPC_MODE_LEGACY": env.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")})
        log = open(os.path.join(args.log_dir, f"workerlog.{rank}"), "a")
        cmd = [sys.executable, "-u", args.training_script, *args.training_script_args]
        procs.append((subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT,
                                       start_new_session=True), log))
    return procs


def _kill(procs):
    for p, _ in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.time() + 10
    for p, log in procs:
        try:
            p.wait(max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
        log.close()


def run(args) -> int:
    world = args.nnodes * args.nproc_per_node
    rank_base = args.node_rank * args.nproc_per_node
    for restart in range(args.max_restart + 1):
        port = args.master_port or _free_port()
        procs = _start(args, rank_base, world, port, restart)
        t0 = time.time()
        failed = None
        while True:
            codes = [p.poll() for p, _ in procs]
            if any(c not in (None, 0) for c in codes):
                failed = next(c for c in codes if c not in (None, 0))
                break
            if all(c == 0 for c in codes):
                break
            if args.timeout and time.time() - t0 > args.timeout:
                failed = 124
                break
            time.sleep(0.2)
        _kill(procs)
        if failed is None:
            return 0
        print(f"[launch] a worker failed (exit {failed}); restart {restart + 1}/{args.max_restart}",
              file=sys.stderr)
    return failed or 1


def main(argv=None):
    ap = argparse.ArgumentParser("paddle_infer_amd.distributed.launch")
    ap.add_argument("--nproc_per_node", "--nproc-per-node", type=int, default=1)
    ap.add_argument("--nnodes", type=int, default=1)
    ap.add_argument("--node_rank", type=int, default=0)
    ap.add_argument("--master_addr", "--master", default="127.0.0.1")
    ap.add_argument("--master_port", type=int, default=0)
    ap.add_argument("--devices", "--gpus", default="")
    ap.add_argument("--log_dir", default="log")
    ap.add_argument("--max_restart", type=int, default=0)
    ap.add_argument("--timeout", type=float, default=0.0)
    ap.add_argument("training_script")
    ap.add_argument("training_script_args", nargs=argparse.REMAINDER)
    args = ap.parse_args(argv)
    sys.exit(run(args))


if __name__ == "__main__":
    main()
