"""Auto checkpoint: an epoch loop that survives a job restart.

Parity: reference `python/paddle/fluid/incubate/checkpoint/auto_checkpoint.py:597`
(``train_epoch_range``; ``_auto_checkpoint`` registering every (executor, program) pair that runs
inside the range; ``TrainEpochRange._save_checkpoint`` / ``_get_last_valid_checkpoint``;
environment ``PADDLE_RUNNING_ENV=PADDLE_EDL_AUTO_CHECKPOINT``, ``PADDLE_JOB_ID``,
``PADDLE_EDL_HDFS_CHECKPOINT_PATH``, ``PADDLE_TRAINER_ID``, ``PADDLE_EDL_SAVE_CHECKPOINT_INTER``).

MI355X-native differences: the checkpoint root is a (shared) filesystem path instead of an HDFS
client, checkpoints are written as a temp directory renamed into place (a crash mid-save never
leaves a half checkpoint that a restart would pick), the last ``keep`` checkpoints are kept, and
besides static programs (registered automatically by ``Executor.run`` inside the range, as in the
reference) dygraph objects with ``state_dict`` / ``set_state_dict`` (Layers, optimizers, the
flat-buffer engines, LR schedulers) can be registered with :func:`register`.

Layout: ``<root>/<job_id>/range/<range_name>/checkpoint.<n>/{status.json, <key>.pdstate}``.
"""
from __future__ import annotations

import json
import logging
import os
import shutil
import time

logger = logging.getLogger("auto_checkpoint")

ENV_ON = "PADDLE_EDL_AUTO_CHECKPOINT"
_RANGE = None  # the active TrainEpochRange


class AutoCheckpointChecker:
    """Reads the job environment (reference ``AutoCheckpointChecker``)."""

    def __init__(self):
        self.run_env = os.getenv("PADDLE_RUNNING_ENV")
        self.job_id = os.getenv("PADDLE_JOB_ID", "")
        self.root = os.getenv("PADDLE_EDL_HDFS_CHECKPOINT_PATH", "")
        self.trainer_id = int(os.getenv("PADDLE_TRAINER_ID", os.getenv("RANK", "0")))
        self.save_checkpoint_inter = int(os.getenv("PADDLE_EDL_SAVE_CHECKPOINT_INTER", "900"))
        self.keep = int(os.getenv("PADDLE_EDL_KEEP_CHECKPOINTS", "2"))

    def valid(self):
        return self.run_env == ENV_ON and bool(self.job_id) and bool(self.root)

    def range_path(self, name):
        return os.path.join(self.root, self.job_id, "range", name)

    def __str__(self):
        return (f"AutoCheckpointChecker(run_env={self.run_env}, job_id={self.job_id}, "
                f"root={self.root}, trainer_id={self.trainer_id}, inter={self.save_checkpoint_inter})")


class _Entry:
    """One registered object: a static (executor, program) pair or a dygraph state holder."""

    def __init__(self, key, program=None, obj=None):
        self.key, self.program, self.obj = key, program, obj

    def state(self):
        if self.obj is not None:
            return self.obj.state_dict()
        from ...static.framework import global_scope
        scope = global_scope()
        return {n: (scope.get(n) if scope.get(n) is not None else t) for n, t in self.program.params.items()}

    def restore(self, state):
        if self.obj is not None:
            self.obj.set_state_dict(state)
            return
        from ...static.io import set_program_state
        names = list(self.program.params)
        if set(state) != set(names) and len(state) == len(names):
            # same program rebuilt under other generated names (e.g. in one process): the
            # persistables are created in the same order, so restore by position (shapes checked)
            vals = list(state.values())
            if all(tuple(v.shape) == tuple(self.program.params[n].shape) for n, v in zip(names, vals)):
                state = dict(zip(names, vals))
        set_program_state(self.program, state)


class TrainEpochRange:
    def __init__(self, max_epoch_num, name, checkpoint_inter=None, checker=None):
        self.checker = checker or AutoCheckpointChecker()
        self.max_epoch_num = max_epoch_num if max_epoch_num >= 0 else 2 ** 62
        self.name = name
        self.inter = self.checker.save_checkpoint_inter if checkpoint_inter is None else checkpoint_inter
        assert self.inter >= 0, f"checkpoint interval {self.inter} must be >= 0"
        self.epoch_no = -1
        self.entries = {}
        self.restored = {}  # key -> path of the saved state, from the checkpoint we resumed
        self.restored_from = None
        self.path = self.checker.range_path(name)
        self._last_save = time.time()
        self._load_last()

    # ---- restore ----------------------------------------------------------------------------
    def _checkpoints(self):
        if not os.path.isdir(self.path):
            return []
        nos = []
        for d in os.listdir(self.path):
            if d.startswith("checkpoint.") and d[len("checkpoint."):].isdigit():
                if os.path.exists(os.path.join(self.path, d, "status.json")):
                    nos.append(int(d[len("checkpoint."):]))
        return sorted(nos)

    def _load_last(self):
        nos = self._checkpoints()
        if not nos:
            logger.info("auto checkpoint: no checkpoint under %s, training from epoch 0", self.path)
            return
        d = os.path.join(self.path, f"checkpoint.{nos[-1]}")
        with open(os.path.join(d, "status.json")) as f:
            st = json.load(f)
        self.epoch_no = int(st["epoch_no"])
        self.restored = {k: os.path.join(d, v) for k, v in st["states"].items()}
        self.restored_from = d
        logger.info("auto checkpoint: resuming after epoch %d from %s", self.epoch_no, d)

    def register(self, key, program=None, obj=None):
        if key in self.entries:
            return self.entries[key]
        e = self.entries[key] = _Entry(key, program, obj)
        src = self.restored.get(key)
        if src is not None:
            from ...framework.io import load
            e.restore(load(src))
            logger.info("auto checkpoint: restored %s", key)
        return e

    # ---- epochs -----------------------------------------------------------------------------
    def next(self):
        for i in range(self.epoch_no + 1, self.max_epoch_num):
            self.epoch_no = i
            yield i
            self.save_checkpoint()

    def get(self):
        return self.epoch_no

    def save_checkpoint(self, force=False):
        if self.checker.trainer_id != 0 or not self.entries:
            return
        if not force and time.time() - self._last_save < self.inter:
            return
        if not force and self.epoch_no == self.max_epoch_num - 1:
            return  # the reference does not checkpoint the finished range
        self._save()
        self._last_save = time.time()

    def _save(self):
        from ...framework.io import save
        nos = self._checkpoints()
        no = (nos[-1] + 1) if nos else 0
        os.makedirs(self.path, exist_ok=True)
        tmp = os.path.join(self.path, f".tmp.checkpoint.{no}.{os.getpid()}")
        os.makedirs(tmp, exist_ok=True)
        states = {}
        for key, e in self.entries.items():
            fn = f"{len(states)}.pdstate"
            save(e.state(), os.path.join(tmp, fn))
            states[key] = fn
        with open(os.path.join(tmp, "status.json"), "w") as f:
            json.dump({"epoch_no": self.epoch_no, "states": states, "name": self.name,
                       "time": time.time()}, f)
        os.replace(tmp, os.path.join(self.path, f"checkpoint.{no}"))  # atomic publish
        for old in nos[:max(0, len(nos) + 1 - self.checker.keep)]:
            shutil.rmtree(os.path.join(self.path, f"checkpoint.{old}"), ignore_errors=True)
        logger.info("auto checkpoint: saved epoch %d as checkpoint.%d", self.epoch_no, no)


def _normal_yield(max_epoch_num):
    n = max_epoch_num if max_epoch_num >= 0 else 2 ** 62
    yield from range(n)


def train_epoch_range(max_epoch_num, save_checkpoint_inter=None, name="range_0"):
    """Epoch generator; under ``PADDLE_RUNNING_ENV=PADDLE_EDL_AUTO_CHECKPOINT`` it resumes after
    the last checkpointed epoch of this job and checkpoints every registered program / object
    after an epoch when ``save_checkpoint_inter`` seconds have passed (trainer 0 only)."""
    global _RANGE
    checker = AutoCheckpointChecker()
    if not checker.valid():
        logger.warning("auto checkpoint is off (PADDLE_RUNNING_ENV != %s or no job id / path)", ENV_ON)
        yield from _normal_yield(max_epoch_num)
        return
    _RANGE = TrainEpochRange(max_epoch_num, name, save_checkpoint_inter, checker)
    try:
        yield from _RANGE.next()
    finally:
        _RANGE = None


def current_range():
    return _RANGE


def register(*objs, keys=None):
    """Register dygraph state holders (``state_dict`` / ``set_state_dict``) with the active range;
    restores them at once when the job resumed from a checkpoint. No-op outside a range."""
    if _RANGE is None:
        return
    for i, o in enumerate(objs):
        key = keys[i] if keys else f"obj_{len(_RANGE.entries)}_{type(o).__name__}"
        _RANGE.register(key, obj=o)


def _auto_checkpoint(exe, program):
    """Called by ``static.Executor.run``: inside an active range, registers the (executor,
    program) pair under a stable key (and restores it on a resumed job)."""
    if _RANGE is None or program is None:
        return
    from ...static.backward import op_role, FORWARD
    if not any(op_role(op) != FORWARD for op in program.global_block().ops):
        return  # inference programs hold no training state (reference _can_auto_checkpoint)
    name = getattr(program, "_auto_checkpoint_name", None)
    if name is None:
        name = program._auto_checkpoint_name = f"program_{len(_RANGE.entries)}"
    exe_name = getattr(exe, "_auto_checkpoint_name", None)
    if exe_name is None:
        exe_name = exe._auto_checkpoint_name = "executor_0"
    _RANGE.register(f"{exe_name}_{name}", program=program)
