"""``paddle.distributed.InMemoryDataset`` / ``QueueDataset`` and the sparse-table entry configs
(reference `python/paddle/distributed/fleet/dataset/dataset.py`, `distributed/entry_attr.py`).

Files in the MultiSlot text format (per line and per ``use_var``: a value count followed by that
many values — what ``fleet.MultiSlotDataGenerator`` writes) are read through an optional
``pipe_command`` (run as a child process per file, like the reference's data feed), parsed in a
thread pool of ``thread_num`` workers, and batched: a dense slot (every instance one value / a
fixed count) becomes a [batch, count] tensor, a variable-length slot a packed tensor with ``.lod``.
``InMemoryDataset`` loads everything (``load_into_memory``) and supports local / global shuffle
(global = every rank shuffles with the same seed and keeps its stripe); ``QueueDataset`` streams.
"""
from __future__ import annotations

import random
import subprocess
from concurrent.futures import ThreadPoolExecutor

import torch


class _EntryAttr:
    def _to_attr(self):
        raise NotImplementedError


class ProbabilityEntry(_EntryAttr):
    def __init__(self, probability):
        if not 0 < float(probability) <= 1:
            raise ValueError("probability must be in (0, 1]")
        self._probability = float(probability)

    def _to_attr(self):
        return f"probability_entry:{self._probability}"


class CountFilterEntry(_EntryAttr):
    def __init__(self, count_filter):
        if int(count_filter) < 0:
            raise ValueError("count_filter must be >= 0")
        self._count_filter = int(count_filter)

    def _to_attr(self):
        return f"count_filter_entry:{self._count_filter}"


class ShowClickEntry(_EntryAttr):
    def __init__(self, show_name, click_name):
        self._show, self._click = str(show_name), str(click_name)

    def _to_attr(self):
        return f"show_click_entry:{self._show}:{self._click}"


class _DatasetBase:
    def __init__(self):
        self._batch_size, self._thread_num = 1, 1
        self._use_var, self._pipe = [], "cat"
        self._files = []

    def init(self, batch_size=1, thread_num=1, use_var=None, pipe_command="cat", input_type=0,
             fs_name="", fs_ugi="", download_cmd="cat", **kw):
        self._batch_size, self._thread_num = int(batch_size), max(1, int(thread_num))
        self._use_var = list(use_var or [])
        self._pipe = pipe_command or "cat"
        return self

    _init_distributed_settings = init

    def set_filelist(self, filelist):
        self._files = list(filelist)

    def _var_names(self):
        return [getattr(v, "var_name", getattr(v, "name", str(v))) for v in self._use_var]

    def _read_file(self, path):
        if self._pipe.strip() == "cat":
            with open(path) as f:
                text = f.read()
        else:
            with open(path, "rb") as f:
                text = subprocess.run(self._pipe, shell=True, stdin=f, capture_output=True,
                                      check=True).stdout.decode()
        recs = []
        n = len(self._use_var)
        for line in text.splitlines():
            tok = line.split()
            if not tok:
                continue
            pos, rec = 0, []
            for _ in range(n):
                c = int(tok[pos])
                rec.append([float(t) for t in tok[pos + 1:pos + 1 + c]])
                pos += 1 + c
            recs.append(rec)
        return recs

    def _load(self):
        with ThreadPoolExecutor(self._thread_num) as ex:
            out = []
            for recs in ex.map(self._read_file, self._files):
                out.extend(recs)
        return out

    def _batches(self, recs):
        names = self._var_names()
        dtypes = [getattr(v, "dtype", torch.float32) for v in self._use_var]
        for i in range(0, len(recs), self._batch_size):
            chunk = recs[i:i + self._batch_size]
            batch = {}
            for s, name in enumerate(names):
                vals = [r[s] for r in chunk]
                dt = dtypes[s] if isinstance(dtypes[s], torch.dtype) else torch.float32
                if len({len(v) for v in vals}) == 1:
                    batch[name] = torch.tensor(vals, dtype=dt)
                else:
                    flat = torch.tensor([x for v in vals for x in v], dtype=dt).reshape(-1, 1)
                    offs = [0]
                    for v in vals:
                        offs.append(offs[-1] + len(v))
                    flat.lod = [offs]
                    batch[name] = flat
            yield batch


class InMemoryDataset(_DatasetBase):
    def __init__(self):
        super().__init__()
        self._data = None

    def load_into_memory(self, is_shuffle=False):
        self._data = self._load()
        if is_shuffle:
            self.local_shuffle()

    def preload_into_memory(self, thread_num=None):
        self.load_into_memory()

    def wait_preload_done(self):
        return None

    def local_shuffle(self):
        random.shuffle(self._data)

    def global_shuffle(self, fleet=None, thread_num=12):
        """Same-seed shuffle of the concatenated data on every rank, each keeping its stripe."""
        import torch.distributed as dist
        rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        rng = random.Random(2024)
        rng.shuffle(self._data)
        self._data = self._data[rank::world]

    def release_memory(self):
        self._data = None

    def get_memory_data_size(self, fleet=None):
        return len(self._data or [])

    def get_shuffle_data_size(self, fleet=None):
        return len(self._data or [])

    def __iter__(self):
        if self._data is None:
            raise RuntimeError("call load_into_memory() first")
        return self._batches(self._data)


class QueueDataset(_DatasetBase):
    def __iter__(self):
        for path in self._files:
            yield from self._batches(self._read_file(path))
