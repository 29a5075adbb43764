"""``paddle.distributed.auto_parallel`` (reference `distributed/auto_parallel/`): semi-automatic
parallelism — ProcessMesh, ``shard_tensor`` / ``shard_op`` annotations, Strategy, Engine.

Static programs: ``complete`` / ``partition`` (`partitioner.py`) propagate the annotations through a
static Program and build each rank's program (local parameter shards, RCCL all-gather / all-reduce
/ slice inserted where layouts change) — the reference's Completer / Partitioner / Resharder.

MI355X design (dynamic mode): annotations become ``torch.distributed.tensor`` DTensors on a DeviceMesh (RCCL
collectives over xGMI inserted by the DTensor propagation rules), instead of the reference's
static-graph completion / partition / reshard passes. ``shard_spec`` follows Paddle: one entry per
tensor dim naming the mesh dim it is split over (or None = replicated). Engine drives training /
evaluation / prediction of a (possibly DTensor-sharded) model with the hapi loop.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist

__all__ = ["ProcessMesh", "shard_tensor", "shard_op", "recompute", "fetch", "Strategy", "Engine",
           "get_current_process_mesh", "reshard", "complete", "partition", "Completer", "Partitioner"]

_CUR = {"mesh": None}


def complete(program, process_mesh, annotations=None):
    from .partitioner import complete as _c
    return _c(program, process_mesh, annotations)


def partition(program, process_mesh, rank=None, annotations=None, fetch_list=()):
    from .partitioner import partition as _p
    return _p(program, process_mesh, rank, annotations, fetch_list)


def __getattr__(name):
    if name in ("Completer", "Partitioner", "DistAttr"):
        from . import partitioner
        return getattr(partitioner, name)
    raise AttributeError(name)


class ProcessMesh:
    """An N-d arrangement of ranks with named dims (``ProcessMesh([[0, 1], [2, 3]], ["dp", "mp"])``).
    Usable as a context manager that sets the current mesh."""

    def __init__(self, mesh=None, dim_names=None, shape=None, process_ids=None):
        if mesh is None:
            mesh = torch.tensor(process_ids).reshape(shape).tolist()
        self._mesh = torch.as_tensor(mesh, dtype=torch.long)
        self._dim_names = list(dim_names) if dim_names else [f"d{i}" for i in range(self._mesh.dim())]
        self._device_mesh = None

    @property
    def shape(self):
        return list(self._mesh.shape)

    @property
    def ndim(self):
        return self._mesh.dim()

    @property
    def dim_names(self):
        return self._dim_names

    @property
    def process_ids(self):
        return self._mesh.reshape(-1).tolist()

    @property
    def mesh(self):
        return self._mesh

    def get_dim_size(self, dim):
        return self.shape[self._dim_names.index(dim) if isinstance(dim, str) else dim]

    def __eq__(self, other):
        return isinstance(other, ProcessMesh) and torch.equal(self._mesh, other._mesh) and \
            self._dim_names == other._dim_names

    def __hash__(self):
        return hash((tuple(self.process_ids), tuple(self.shape), tuple(self._dim_names)))

    def __enter__(self):
        self._prev = _CUR["mesh"]
        _CUR["mesh"] = self
        return self

    def __exit__(self, *exc):
        _CUR["mesh"] = self._prev

    def device_mesh(self):
        """The torch DeviceMesh of this ProcessMesh (needs an initialised process group)."""
        if self._device_mesh is None:
            from torch.distributed.device_mesh import DeviceMesh
            dev = "cuda" if torch.cuda.is_available() and dist.get_backend() == "nccl" else "cpu"
            self._device_mesh = DeviceMesh(dev, self._mesh, mesh_dim_names=tuple(self._dim_names))
        return self._device_mesh

    def __repr__(self):
        return f"ProcessMesh(shape={self.shape}, process_ids={self.process_ids}, dim_names={self._dim_names})"


def get_current_process_mesh():
    return _CUR["mesh"]


def _placements(mesh, shard_spec, ndim):
    from torch.distributed.tensor import Replicate, Shard
    pl = [Replicate() for _ in range(mesh.ndim)]
    for tdim, name in enumerate(shard_spec or [None] * ndim):
        if name is None:
            continue
        md = mesh.dim_names.index(name) if isinstance(name, str) else int(name)
        pl[md] = Shard(tdim)
    return pl


def _distributed():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def shard_tensor(x, process_mesh=None, shard_spec=None):
    """Shard ``x`` over ``process_mesh`` per ``shard_spec``. Multi-rank: returns a DTensor (each
    rank holds its shard); single process: records the annotation on the tensor and returns it."""
    mesh = process_mesh or get_current_process_mesh()
    assert mesh is not None, "shard_tensor needs a process_mesh (argument or `with ProcessMesh`)"
    if shard_spec is not None:
        assert len(shard_spec) == x.dim(), "shard_spec needs one entry per tensor dim"
    from ...static.framework import Variable
    from ... import in_dynamic_mode
    if not _distributed() or isinstance(x, Variable) or not in_dynamic_mode():
        # single process, or a static program: an annotation for the static completion /
        # partition passes (partitioner.py)
        x.process_mesh, x.shard_spec = mesh, shard_spec
        return x
    from torch.distributed.tensor import distribute_tensor
    dt = distribute_tensor(x.detach() if not x.requires_grad else x, mesh.device_mesh(),
                           _placements(mesh, shard_spec, x.dim()))
    if isinstance(x, torch.nn.Parameter):
        return torch.nn.Parameter(dt, requires_grad=x.requires_grad)
    return dt


def reshard(x, process_mesh, shard_spec):
    """Move a DTensor to another layout (RCCL all-gather / all-to-all as needed)."""
    if not hasattr(x, "redistribute"):
        return shard_tensor(x, process_mesh, shard_spec)
    return x.redistribute(process_mesh.device_mesh(), _placements(process_mesh, shard_spec, x.dim()))


def shard_op(op, process_mesh=None, in_shard_specs=None, out_shard_specs=None):
    """Wrap ``op`` so its inputs / outputs carry the given shardings."""
    def wrapped(*args, **kwargs):
        mesh = process_mesh or get_current_process_mesh()
        if in_shard_specs is not None:
            args = tuple(shard_tensor(a, mesh, s) if isinstance(a, torch.Tensor) and s is not None else a
                         for a, s in zip(args, list(in_shard_specs) + [None] * len(args)))
        out = op(*args, **kwargs)
        if out_shard_specs is not None:
            outs = out if isinstance(out, (list, tuple)) else [out]
            outs = [reshard(o, mesh, s) if s is not None and _distributed() else o
                    for o, s in zip(outs, out_shard_specs)]
            out = type(out)(outs) if isinstance(out, (list, tuple)) else outs[0]
        return out
    return wrapped


def recompute(op):
    """Activation-checkpoint ``op`` (a Layer or callable)."""
    def wrapped(*args, **kwargs):
        return torch.utils.checkpoint.checkpoint(op, *args, use_reentrant=False, **kwargs)
    return wrapped


_COLLECTION = {}


def fetch(tensor, name=None, logging=False):
    _COLLECTION.setdefault("fetches", []).append((name, tensor))
    return tensor


class _Cfg(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


class Strategy:
    """Reference `auto_parallel/strategy.py`: nested config groups (sharding, amp, recompute,
    gradient_merge, pipeline, ...), each with ``enable`` plus options."""

    def __init__(self, config=None):
        self.auto_mode = "semi"
        self.seed = None
        self.split_data = True
        self.sharding = _Cfg(enable=False, stage=1, degree=8)
        self.amp = _Cfg(enable=False, dtype="bfloat16", level="o1", init_loss_scaling=32768.0)
        self.recompute = _Cfg(enable=False, checkpoints=None)
        self.gradient_merge = _Cfg(enable=False, k_steps=1, avg=True)
        self.pipeline = _Cfg(enable=False, schedule_mode="1F1B", micro_batch_size=1,
                             accumulate_steps=1)
        self.fused_passes = _Cfg(enable=False, fused_passes_list=[])
        self.dataset = _Cfg(enable=False, num_shards=1)
        for k, v in (config or {}).items():
            cur = getattr(self, k, None)
            if isinstance(cur, _Cfg) and isinstance(v, dict):
                cur.update(v)
            else:
                setattr(self, k, v)


class Engine:
    """High-level train / eval / predict driver (reference `auto_parallel/engine.py`): the model's
    sharding comes from its ``shard_tensor`` annotations; Strategy.amp enables bf16 autocast,
    gradient_merge accumulates ``k_steps`` micro-steps per optimizer step."""

    def __init__(self, model=None, loss=None, optimizer=None, metrics=None, cluster=None,
                 strategy=None):
        self.model, self.loss, self.optimizer = model, loss, optimizer
        self.metrics = list(metrics or []) if not isinstance(metrics, (list, tuple)) else list(metrics)
        self.strategy = strategy or Strategy()
        self.history = {"loss": []}

    def plan(self, global_batch, n_gpus=None, seq_len=None, cluster=None):
        """``Strategy.auto_mode = "full"``: search the parallel layout (dp / tp / pp, sharding
        stage, micro-batch, recompute) for this model with the MI355X cost model
        (``planner.py``), write it into ``self.strategy`` and return the Plan."""
        from . import planner as _pl
        cfg = getattr(self.model, "config", None) or getattr(self.model, "cfg", None)
        if cfg is None and hasattr(self.model, "gpt"):
            cfg = getattr(self.model.gpt, "config", None)
        if cfg is None:
            raise ValueError("auto planning needs a transformer model with a .config")
        spec = _pl.ModelSpec.from_gpt_config(cfg)
        if seq_len:
            spec.seq_len = int(seq_len)
        if n_gpus is None:
            import torch.distributed as dist
            n_gpus = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        c = cluster or _pl.ClusterSpec(n_gpus=int(n_gpus))
        best = _pl.plan(spec, c, int(global_batch))[0]
        self.hybrid_configs = _pl.apply_to_strategy(best, self.strategy, int(global_batch))
        return best

    # ---- static auto-parallel path (reference Engine.prepare -> completion / partition) ----------
    def prepare(self, inputs_spec=None, labels_spec=None, inputs=None, labels=None,
                main_program=None, startup_program=None, mode="train", process_mesh=None):
        """Trace the model (and loss) into a static Program from ``inputs_spec`` / ``labels_spec``
        (InputSpec lists), complete the ``shard_tensor`` annotations made while tracing, partition
        the program for this rank and — for ``mode="train"`` — append backward + optimizer ops to
        the partitioned program. ``fit`` / ``evaluate`` / ``predict`` then run the per-rank
        program in a private Scope (feeds are global batches; split feeds are sliced locally)."""
        import torch.distributed as dist
        from ... import static, enable_static, disable_static, in_dynamic_mode
        from .partitioner import complete, Partitioner
        was_dyn = in_dynamic_mode()
        enable_static()
        try:
            main, startup = static.Program(), static.Program()
            with static.program_guard(main, startup):
                xs = [static.data(s.name or f"input_{i}", list(s.shape), s.dtype)
                      for i, s in enumerate(inputs_spec or [])]
                ys = [static.data(s.name or f"label_{i}", list(s.shape), s.dtype)
                      for i, s in enumerate(labels_spec or [])]
                out = self.model(*xs)
                loss = self.loss(out, *ys) if (self.loss is not None and ys) else None
            mesh = process_mesh or get_current_process_mesh() or self._annotation_mesh(main)
            rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
            if mesh is None:
                mesh = ProcessMesh([rank])
            c = complete(main, mesh)
            fetch = [out] + ([loss] if loss is not None else [])
            local = Partitioner(c).partition(rank, fetch_list=fetch)
            lvars = local.global_block().vars
            lloss = lvars[loss.var_name] if loss is not None else None
            if mode == "train" and lloss is not None and self.optimizer is not None:
                with static.program_guard(local, static.Program()):
                    self._static_opt().minimize(lloss)
            self._static = {"program": local, "inputs": [x.var_name for x in xs],
                            "labels": [y.var_name for y in ys], "out": out.var_name,
                            "loss": loss.var_name if loss is not None else None,
                            "exe": static.Executor("cuda" if torch.cuda.is_available() else "cpu"),
                            "scope": static.Scope(), "mode": mode}
            return local
        finally:
            if was_dyn:
                disable_static()

    @staticmethod
    def _annotation_mesh(program):
        for t in list(program.params.values()) + list(program.global_block().vars.values()):
            pm = getattr(t, "process_mesh", None)
            if pm is not None:
                return pm
        return None

    def _static_opt(self):
        """A static-mode optimizer of the same kind / learning rate as ``self.optimizer``."""
        from ... import optimizer as O
        opt = self.optimizer
        lr = opt.get_lr() if hasattr(opt, "get_lr") else getattr(opt, "_learning_rate", 0.001)
        cls = getattr(O, type(opt).__name__, O.SGD)
        try:
            return cls(learning_rate=lr)
        except TypeError:
            return O.SGD(learning_rate=lr)

    def _run_static(self, batch, fetch_loss=True):
        from ... import static
        st = self._static
        ins, lab = self._split(batch) if st["labels"] else (tuple(batch) if isinstance(batch, (list, tuple)) else (batch,), None)
        feed = dict(zip(st["inputs"], [i.detach().cpu().numpy() if isinstance(i, torch.Tensor) else i for i in ins]))
        if st["labels"] and lab is not None:
            feed[st["labels"][0]] = lab.detach().cpu().numpy() if isinstance(lab, torch.Tensor) else lab
        fetch = [st["loss"]] if fetch_loss and st["loss"] else [st["out"]]
        with static.scope_guard(st["scope"]):
            return st["exe"].run(st["program"], feed=feed, fetch_list=fetch)[0]

    def _ctx(self):
        if self.strategy.amp.enable:
            dev = "cuda" if torch.cuda.is_available() else "cpu"
            return torch.autocast(dev, dtype=torch.bfloat16)
        return contextlib.nullcontext()

    def _batches(self, data, batch_size):
        from ...io import DataLoader
        return data if not hasattr(data, "__getitem__") or isinstance(data, DataLoader) else \
            DataLoader(data, batch_size=batch_size, shuffle=False)

    @staticmethod
    def _split(batch):
        if isinstance(batch, (list, tuple)) and len(batch) >= 2:
            return batch[:-1], batch[-1]
        return (batch,), None

    def fit(self, train_data, valid_data=None, train_sample_split=None, batch_size=1, epochs=1,
            steps_per_epoch=None, log_freq=10, save_dir=None, save_freq=1, valid_sample_split=None,
            valid_freq=1, valid_steps=None, collate_fn=None, callbacks=None, verbose=2,
            nvprof_range=[-1, -1]):
        if getattr(self, "_static", None) is not None:  # prepared: per-rank static program
            for _ in range(epochs):
                for i, batch in enumerate(self._batches(train_data, batch_size)):
                    if steps_per_epoch is not None and i >= steps_per_epoch:
                        break
                    self.history["loss"].append(float(self._run_static(batch)))
            return self.history
        self.model.train()
        k = max(1, int(self.strategy.gradient_merge.k_steps)) if self.strategy.gradient_merge.enable else 1
        step = 0
        for _ in range(epochs):
            for i, batch in enumerate(self._batches(train_data, batch_size)):
                if steps_per_epoch is not None and i >= steps_per_epoch:
                    break
                ins, lab = self._split(batch)
                with self._ctx():
                    out = self.model(*ins)
                    l = self.loss(out, lab) if self.loss is not None else out
                (l / k).backward()
                step += 1
                if step % k == 0:
                    self.optimizer.step()
                    self.optimizer.clear_grad()
                self.history["loss"].append(float(l.detach().float().mean()))
        return self.history

    @torch.no_grad()
    def evaluate(self, valid_data, valid_sample_split=None, batch_size=1, steps=None, log_freq=10,
                 collate_fn=None, callbacks=None, verbose=2):
        self.model.eval()
        losses = []
        for m in self.metrics:
            m.reset()
        for i, batch in enumerate(self._batches(valid_data, batch_size)):
            if steps is not None and i >= steps:
                break
            ins, lab = self._split(batch)
            with self._ctx():
                out = self.model(*ins)
            if self.loss is not None and lab is not None:
                losses.append(float(self.loss(out, lab).float().mean()))
            for m in self.metrics:
                m.update(*m.compute(out, lab)) if hasattr(m, "compute") else m.update(out, lab)
        res = {"loss": sum(losses) / max(1, len(losses))} if losses else {}
        for m in self.metrics:
            res[m.name() if callable(getattr(m, "name", None)) else str(m)] = m.accumulate()
        return res

    @torch.no_grad()
    def predict(self, test_data, test_sample_split=None, batch_size=1, steps=None, collate_fn=None,
                callbacks=None, verbose=2):
        self.model.eval()
        outs = []
        for i, batch in enumerate(self._batches(test_data, batch_size)):
            if steps is not None and i >= steps:
                break
            ins, _ = self._split(batch) if isinstance(batch, (list, tuple)) and len(batch) > 1 else ((batch,) if not isinstance(batch, (list, tuple)) else tuple(batch), None)
            with self._ctx():
                outs.append(self.model(*ins))
        return outs

    def save(self, path, training=True):
        from ...framework.io import save
        save(self.model.state_dict(), path + ".pdparams")
        if training and self.optimizer is not None:
            save(self.optimizer.state_dict(), path + ".pdopt")

    def load(self, path, strict=True, load_optimizer=True):
        import os
        from ...framework.io import load
        self.model.set_state_dict(load(path + ".pdparams"))
        if load_optimizer and self.optimizer is not None and os.path.exists(path + ".pdopt"):
            self.optimizer.set_state_dict(load(path + ".pdopt"))
