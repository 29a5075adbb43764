"""Elastic training membership (reference `python/paddle/distributed/fleet/elastic/manager.py`,
`elastic.py`, launch `--np min:max` / `--elastic_server`).

The reference keeps node membership in etcd; here it lives in a ``torch.distributed.TCPStore``
(the rendezvous store the collectives already use), so no extra service is needed:

* every node's launcher takes a slot (``store.add`` on a counter) and refreshes a heartbeat key
  ``hb/<slot> = "<node_id>|<unix time>"`` every ``heartbeat`` seconds;
* the live set = slots whose heartbeat is younger than ``ttl``; node ranks follow the sorted node
  ids, so every launcher derives the same (world size, node rank) without a coordinator;
* a change of the live set inside ``[np_min, np_max]`` makes every launcher stop its workers and
  relaunch them with the new world size (scale-in after a node loss, scale-out when a node joins);
  below ``np_min`` the launchers hold until enough nodes are back (or ``wait_timeout`` expires).

Workers see the usual RANK / WORLD_SIZE / MASTER_* plus ``PADDLE_ELASTIC_NP`` and
``PADDLE_RESTART_COUNT`` and resume from their last checkpoint (``distributed.checkpoint`` reshards
across data-parallel degrees).
"""
from __future__ import annotations

import threading
import time

import torch.distributed as dist


class ElasticStatus:
    COMPLETED = "completed"
    ERROR = "error"
    HOLD = "hold"
    RESTART = "restart"
    EXIT = "exit"


class ElasticManager:
    def __init__(self, server: str, job_id: str, node_id: str, np_min: int, np_max: int,
                 is_master: bool = False, heartbeat: float = 1.0, ttl: float = 4.0,
                 timeout: float = 60.0):
        host, port = server.rsplit(":", 1)
        self.store = dist.TCPStore(host, int(port), is_master=is_master, wait_for_workers=False,
                                   timeout=__import__("datetime").timedelta(seconds=timeout))
        self.prefix = f"/elastic/{job_id}/"
        self.node_id = node_id
        self.np_min, self.np_max = np_min, np_max
        self.heartbeat, self.ttl = heartbeat, ttl
        self.slot = self.store.add(self.prefix + "count", 1) - 1
        self._stop = threading.Event()
        self._beat()
        self._thread = threading.Thread(target=self._loop, daemon=True)
        self._thread.start()

    # ----------------------------------------------------------------- heartbeat
    def _beat(self):
        self.store.set(f"{self.prefix}hb/{self.slot}", f"{self.node_id}|{time.time():.3f}")

    def _loop(self):
        while not self._stop.wait(self.heartbeat):
            try:
                self._beat()
            except Exception:  # store gone: the job is over
                return

    def exit(self):
        """Leave the job: stop beating and tombstone the slot (immediate scale-in for the rest)."""
        self._stop.set()
        try:
            self.store.set(f"{self.prefix}hb/{self.slot}", f"{self.node_id}|0")
        except Exception:
            pass

    # ----------------------------------------------------------------- membership
    def live_nodes(self):
        n = int(self.store.add(self.prefix + "count", 0))
        now = time.time()
        live = set()
        for s in range(n):
            key = f"{self.prefix}hb/{s}"
            try:
                if not self.store.check([key]):
                    continue
                nid, ts = self.store.get(key).decode().rsplit("|", 1)
            except Exception:
                continue
            if now - float(ts) <= self.ttl:
                live.add(nid)
        return sorted(live)

    def assignment(self, nodes=None):
        """(world_nodes, node_rank) for this node, or None when it is not in the live set."""
        nodes = self.live_nodes() if nodes is None else nodes
        nodes = nodes[: self.np_max]
        if self.node_id not in nodes:
            return None
        return len(nodes), nodes.index(self.node_id)

    def wait_for_quorum(self, wait_timeout: float):
        """Block until at least ``np_min`` nodes are live (returns the live list) or time out."""
        t0 = time.time()
        while True:
            nodes = self.live_nodes()
            if len(nodes) >= self.np_min:
                return nodes
            if time.time() - t0 > wait_timeout:
                return None
            time.sleep(self.heartbeat / 2)

    def master_port(self, nodes, base_port: int):
        """Rendezvous port of a membership epoch, identical on every node (CRC of the member
        list), so each relaunch after a membership change meets on a fresh port."""
        import zlib
        return base_port + 1 + zlib.crc32(",".join(nodes).encode()) % 2000


def parse_np(np_arg):
    """``"2"`` → (2, 2); ``"2:4"`` → (2, 4) (reference `--np` elastic range)."""
    if np_arg is None or np_arg == "":
        return None
    if ":" in str(np_arg):
        a, b = str(np_arg).split(":")
        return int(a), int(b)
    return int(np_arg), int(np_arg)


def serve(endpoint: str):
    """Run a standalone membership store (the etcd role of the reference) until killed:
    ``python -m paddle_infer_amd.distributed.elastic host:port``."""
    host, port = endpoint.rsplit(":", 1)
    store = dist.TCPStore(host, int(port), is_master=True, wait_for_workers=False)  # noqa: F841
    while True:
        time.sleep(3600)


if __name__ == "__main__":
    import sys
    serve(sys.argv[1])
