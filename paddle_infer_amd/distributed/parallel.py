"""``init_parallel_env`` / ``ParallelEnv`` / ``DataParallel`` / ``spawn``
(reference `python/paddle/distributed/parallel.py`, `spawn.py`, `fluid/dygraph/parallel.py`,
`paddle/fluid/imperative/reducer.cc`).

``DataParallel`` is the generic-model data-parallel wrapper: gradients are re-bound as views into
per-bucket flat buffers (large buckets sized for xGMI rings), each bucket's all-reduce is launched
asynchronously on RCCL from the post-accumulate hook of its last gradient (overlapping the rest of
backward), and a callback queued on the autograd engine waits for all buckets and averages at the
end of ``backward()`` — the reference reducer's behaviour, on torch's autograd engine. (The
flagship GPT path uses ``parallel.flat_engine`` which also flattens parameters and optimizer
states.)
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .collective import get_rank, get_world_size, is_initialized, Group


class ParallelEnv:
    @property
    def rank(self):
        return int(os.environ.get("PADDLE_TRAINER_ID", os.environ.get("RANK", get_rank())))

    local_rank = rank

    @property
    def world_size(self):
        return int(os.environ.get("PADDLE_TRAINERS_NUM", os.environ.get("WORLD_SIZE", get_world_size())))

    nranks = world_size

    @property
    def device_id(self):
        return int(os.environ.get("LOCAL_RANK", os.environ.get("FLAGS_selected_gpus", 0)))

    dev_id = device_id

    @property
    def current_endpoint(self):
        return os.environ.get("PADDLE_CURRENT_ENDPOINT", "127.0.0.1:0")

    @property
    def trainer_endpoints(self):
        return os.environ.get("PADDLE_TRAINER_ENDPOINTS", "").split(",")


def init_parallel_env(backend=None):
    """Initialise the default process group from the launcher's env (RANK/WORLD_SIZE/MASTER_*),
    one process per GPU; RCCL when GPUs are visible, gloo otherwise."""
    if is_initialized():
        return Group(None, list(range(dist.get_world_size())), 0)
    world = int(os.environ.get("WORLD_SIZE", os.environ.get("PADDLE_TRAINERS_NUM", "1")))
    rank = int(os.environ.get("RANK", os.environ.get("PADDLE_TRAINER_ID", "0")))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    if use_gpu:
        local = int(os.environ.get("LOCAL_RANK", rank % max(1, torch.cuda.device_count())))
        torch.cuda.set_device(local)
        from .. import device as _d
        _d.set_device(f"gpu:{local}")
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return Group(None, list(range(world)), 0)


class DataParallel(torch.nn.Module):
    def __init__(self, layers, strategy=None, comm_buffer_size=256, last_comm_buffer_size=1,
                 find_unused_parameters=False, group=None):
        super().__init__()
        self._layers = layers
        self.group = group
        self.pg = group.pg if isinstance(group, Group) else group
        self.world = get_world_size(group)
        self.find_unused = find_unused_parameters
        self._buckets = []
        self._pending = {}
        self._handles = []
        self._queued = False
        # fp16_allreduce (fleet strategy): f32 gradient buckets travel as fp16, cast back after
        self.comm_fp16 = False
        params = [p for p in layers.parameters() if p.requires_grad]
        from .collective import collectives_forced
        self.multi = self.world > 1 or (collectives_forced() and self.pg is not None)
        if self.multi:
            for p in params:  # identical initial weights on every rank
                dist.broadcast(p.data, src=0, group=self.pg)
            self._build_buckets(params, int(comm_buffer_size * 2 ** 20))

    def _build_buckets(self, params, cap_bytes):
        cur, size = [], 0
        for p in reversed(params):
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= cap_bytes:
                self._buckets.append(cur)
                cur, size = [], 0
        if cur:
            self._buckets.append(cur)
        self._flat = []
        for bi, ps in enumerate(self._buckets):
            by_dtype = {}
            for p in ps:
                by_dtype.setdefault((p.dtype, p.device), []).append(p)
            for (dt, dev), group_ps in by_dtype.items():
                n = sum(p.numel() for p in group_ps)
                flat = torch.zeros(n, dtype=dt, device=dev)
                off = 0
                views = []
                for p in group_ps:
                    v = flat[off:off + p.numel()].view(p.shape)
                    views.append((p, v))
                    off += p.numel()
                self._flat.append((flat, views))
        self._hook_handles = []
        for fi, (flat, views) in enumerate(self._flat):
            for p, v in views:
                p.grad = v
                p._dp_bucket = fi
                self._hook_handles.append(p.register_post_accumulate_grad_hook(self._hook))
        self._reset()

    def _detach_reducer(self):
        """Hand gradient reduction to another engine (the flat-buffer optimizer of
        fleet.distributed_optimizer): remove the hooks and buckets of this reducer."""
        for h in getattr(self, "_hook_handles", []):
            h.remove()
        self._hook_handles = []
        for flat, views in getattr(self, "_flat", []):
            for p, _ in views:
                if hasattr(p, "_dp_bucket"):
                    del p._dp_bucket
        self._flat, self._buckets = [], []
        self._pending, self._launched, self._handles = {}, set(), []

    def _reset(self):
        self._pending = {fi: len(views) for fi, (_, views) in enumerate(self._flat)}
        self._launched = set()
        self._handles = []
        self._queued = False
        for flat, views in self._flat:
            for p, v in views:
                if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                    p.grad = v

    def _hook(self, p):
        if not self._queued:
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
            self._queued = True
        fi = p._dp_bucket
        self._pending[fi] -= 1
        if self._pending[fi] == 0:
            self._launch(fi)

    def _launch(self, fi):
        if fi in self._launched:
            return
        self._launched.add(fi)
        flat = self._flat[fi][0]
        if self.comm_fp16 and flat.dtype == torch.float32:
            tmp = flat.to(torch.float16)
            self._handles.append((flat, tmp, dist.all_reduce(tmp, group=self.pg, async_op=True)))
        else:
            self._handles.append((flat, flat, dist.all_reduce(flat, group=self.pg, async_op=True)))

    def _finalize(self):
        for fi in range(len(self._flat)):  # unused params: their buckets still reduce, in order
            self._launch(fi)
        for flat, comm, h in self._handles:
            h.wait()
            if comm is not flat:
                flat.copy_(comm)
            flat.div_(self.world)
        self._pending = {fi: len(views) for fi, (_, views) in enumerate(self._flat)}
        self._launched = set()
        self._handles = []
        self._queued = False

    def forward(self, *inputs, **kwargs):
        if self.multi:
            for flat, views in self._flat:
                for p, v in views:
                    if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                        if p.grad is not None:
                            v.copy_(p.grad)
                        p.grad = v
        return self._layers(*inputs, **kwargs)

    # Layer API passthroughs
    def parameters(self, include_sublayers=True, recurse=True):
        return list(self._layers.parameters())

    def state_dict(self, *a, **k):
        return self._layers.state_dict(*a, **k)

    def set_state_dict(self, sd, *a, **k):
        return self._layers.set_state_dict(sd)

    def scale_loss(self, loss):
        return loss

    def apply_collective_grads(self):
        pass

    @property
    def _sub_layers(self):
        return dict(self._layers.named_children())


def _spawn_entry(rank, func, args, nprocs, port, backend):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(nprocs),
                       "PADDLE_TRAINER_ID": str(rank), "PADDLE_TRAINERS_NUM": str(nprocs),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    if backend:
        os.environ["PIAMD_BACKEND"] = backend
    func(*args)


def spawn(func, args=(), nprocs=-1, join=True, daemon=False, **options):
    """Start ``nprocs`` processes (default: one per visible GPU) running ``func(*args)``."""
    import socket
    import torch.multiprocessing as mp
    if nprocs == -1:
        nprocs = max(1, torch.cuda.device_count())
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return mp.start_processes(_spawn_entry, args=(func, args, nprocs, port, options.get("backend")),
                              nprocs=nprocs, join=join, daemon=daemon, start_method="spawn")
