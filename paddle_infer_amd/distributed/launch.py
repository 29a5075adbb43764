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


def _wait_any(procs, args, t0, watch=None):
    """Poll workers; returns (failed_code | None, membership_changed)."""
    while True:
        codes = [p.poll() for p, _ in procs]
        if any(c not in (None, 0) for c in codes):
            return next(c for c in codes if c not in (None, 0)), False
        if all(c == 0 for c in codes):
            return None, False
        if args.timeout and time.time() - t0 > args.timeout:
            return 124, False
        if watch is not None and watch():
            return None, True
        time.sleep(0.2)


def run_elastic(args) -> int:
    """Elastic mode (``--elastic_server host:port --np min:max``): membership in a TCPStore,
    relaunch on every change of the live node set (see distributed/elastic.py)."""
    from .elastic import ElasticManager, parse_np
    lo, hi = parse_np(args.np)
    node_id = args.node_id or f"{socket.gethostname()}-{os.getpid()}"
    em = ElasticManager(args.elastic_server, args.job_id, node_id, lo, hi,
                        is_master=args.elastic_master, heartbeat=args.elastic_heartbeat,
                        ttl=args.elastic_ttl)
    base_port = int(args.elastic_server.rsplit(":", 1)[1])
    restarts = 0
    try:
        while True:
            nodes = em.wait_for_quorum(args.elastic_wait)
            if nodes is None:
                print("[launch] elastic: not enough nodes before the wait timeout", file=sys.stderr)
                return 1
            time.sleep(args.elastic_settle)  # let simultaneous joins land in one epoch
            nodes = em.live_nodes()
            asg = em.assignment(nodes)
            if asg is None:  # beyond np_max: stand by
                time.sleep(em.heartbeat)
                continue
            n_nodes, node_rank = asg
            members = nodes[:hi]
            world = n_nodes * args.nproc_per_node
            port = em.master_port(members, base_port)
            os.environ["PADDLE_ELASTIC_NP"] = str(n_nodes)
            procs = _start(args, node_rank * args.nproc_per_node, world, port, restarts)
            print(f"[launch] elastic epoch: nodes={members} world={world} node_rank={node_rank}",
                  file=sys.stderr)

            def changed(members=members):
                cur = em.live_nodes()[:hi]
                return cur != members and len(cur) >= lo or len(cur) < lo
            try:
                failed, memb = _wait_any(procs, args, time.time(), changed)
            finally:
                _kill(procs)
            if memb:
                restarts += 1
                print(f"[launch] elastic: membership changed -> relaunch ({restarts})", file=sys.stderr)
                continue
            if failed is None:
                return 0
            restarts += 1
            if restarts > args.max_restart:
                return failed
    finally:
        em.exit()


def run(args) -> int:
    if getattr(args, "elastic_server", None):
        return run_elastic(args)
    world = args.nnodes * args.nproc_per_node
    rank_base = args.node_rank * args.nproc_per_node
    for restart in range(args.max_restart + 1):
        port = args.master_port or _free_port()
        procs = _start(args, rank_base, world, port, restart)
        try:
            failed, _ = _wait_any(procs, args, time.time())
        finally:
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
    # elastic (reference fleet/elastic): membership in a TCPStore at --elastic_server
    ap.add_argument("--elastic_server", default="")
    ap.add_argument("--elastic_master", action="store_true",
                    help="host the membership TCPStore in this launcher")
    ap.add_argument("--np", default="", help="elastic node range 'min:max'")
    ap.add_argument("--job_id", default="default")
    ap.add_argument("--node_id", default="")
    ap.add_argument("--elastic_heartbeat", type=float, default=1.0)
    ap.add_argument("--elastic_ttl", type=float, default=4.0)
    ap.add_argument("--elastic_wait", type=float, default=120.0)
    ap.add_argument("--elastic_settle", type=float, default=1.0)
    ap.add_argument("training_script")
    ap.add_argument("training_script_args", nargs=argparse.REMAINDER)
    args = ap.parse_args(argv)

    def _term(signum, frame):  # run the finally blocks: stop workers, leave the elastic job
        raise SystemExit(128 + signum)
    signal.signal(signal.SIGTERM, _term)
    sys.exit(run(args))


if __name__ == "__main__":
    main()
