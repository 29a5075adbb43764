"""``paddle.io`` — datasets, samplers, DataLoader (reference `python/paddle/io/`,
`python/paddle/fluid/dataloader/`, `paddle/fluid/operators/reader/buffered_reader.cc`).

Workers are processes with shared-memory batch transfer (torch's worker machinery); on GPU the
loader adds the reference's *buffered reader*: the next ``prefetch`` batches are copied host→device
from pinned memory on a dedicated HIP stream while the current step computes, and the consumer
stream waits on a per-batch event (no host sync).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.utils.data as tud

Dataset = tud.Dataset
IterableDataset = tud.IterableDataset
Subset = tud.Subset
ChainDataset = tud.ChainDataset
get_worker_info = tud.get_worker_info
random_split = tud.random_split


class TensorDataset(Dataset):
    def __init__(self, tensors):
        self.tensors = list(tensors)
        n = len(self.tensors[0])
        assert all(len(t) == n for t in self.tensors)

    def __getitem__(self, i):
        return tuple(t[i] for t in self.tensors)

    def __len__(self):
        return len(self.tensors[0])


class ComposeDataset(Dataset):
    def __init__(self, datasets):
        self.datasets = list(datasets)

    def __len__(self):
        return len(self.datasets[0])

    def __getitem__(self, i):
        out = []
        for d in self.datasets:
            s = d[i]
            out.extend(s if isinstance(s, (list, tuple)) else [s])
        return tuple(out)


class Sampler:
    def __init__(self, data_source=None):
        self.data_source = data_source

    def __iter__(self):  # pragma: no cover
        raise NotImplementedError

    def __len__(self):
        return len(self.data_source)


class SequenceSampler(Sampler):
    def __iter__(self):
        return iter(range(len(self.data_source)))


class RandomSampler(Sampler):
    def __init__(self, data_source, replacement=False, num_samples=None, generator=None):
        super().__init__(data_source)
        self.replacement, self._n, self.generator = replacement, num_samples, generator

    def __len__(self):
        return self._n or len(self.data_source)

    def __iter__(self):
        n = len(self.data_source)
        if self.replacement:
            return iter(np.random.randint(0, n, len(self)).tolist())
        return iter(np.random.permutation(n)[:len(self)].tolist())


class WeightedRandomSampler(Sampler):
    def __init__(self, weights, num_samples, replacement=True):
        self.weights = np.asarray(weights, dtype=np.float64)
        self.num_samples, self.replacement = num_samples, replacement

    def __len__(self):
        return self.num_samples

    def __iter__(self):
        p = self.weights / self.weights.sum()
        return iter(np.random.choice(len(p), self.num_samples, self.replacement, p).tolist())


class SubsetRandomSampler(Sampler):
    def __init__(self, indices):
        self.indices = list(indices)

    def __len__(self):
        return len(self.indices)

    def __iter__(self):
        return iter([self.indices[i] for i in np.random.permutation(len(self.indices))])


class BatchSampler(Sampler):
    def __init__(self, dataset=None, sampler=None, shuffle=False, batch_size=1, drop_last=False):
        if sampler is None:
            sampler = RandomSampler(dataset) if shuffle else SequenceSampler(dataset)
        self.sampler, self.batch_size, self.drop_last = sampler, batch_size, drop_last

    def __iter__(self):
        b = []
        for i in self.sampler:
            b.append(i)
            if len(b) == self.batch_size:
                yield b
                b = []
        if b and not self.drop_last:
            yield b

    def __len__(self):
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)


class DistributedBatchSampler(BatchSampler):
    """Shards the (optionally shuffled, epoch-seeded) index list over data-parallel ranks."""

    def __init__(self, dataset, batch_size, num_replicas=None, rank=None, shuffle=False,
                 drop_last=False):
        import torch.distributed as dist
        self.dataset, self.batch_size, self.shuffle, self.drop_last = dataset, batch_size, shuffle, drop_last
        init = dist.is_available() and dist.is_initialized()
        self.nranks = num_replicas if num_replicas is not None else (dist.get_world_size() if init else 1)
        self.local_rank = rank if rank is not None else (dist.get_rank() if init else 0)
        self.epoch = 0
        self.num_samples = int(math.ceil(len(dataset) / self.nranks))
        self.total_size = self.num_samples * self.nranks

    def set_epoch(self, epoch):
        self.epoch = epoch

    def __iter__(self):
        idx = np.arange(len(self.dataset)).tolist()
        if self.shuffle:
            rng = np.random.RandomState(self.epoch)
            rng.shuffle(idx)
            self.epoch += 1
        idx += idx[: self.total_size - len(idx)]
        local = idx[self.local_rank:self.total_size:self.nranks]
        b = []
        for i in local:
            b.append(i)
            if len(b) == self.batch_size:
                yield b
                b = []
        if b and not self.drop_last:
            yield b

    def __len__(self):
        n = self.num_samples
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)


def default_collate_fn(batch):
    s = batch[0]
    if isinstance(s, torch.Tensor):
        return torch.stack(batch)
    if isinstance(s, np.ndarray):
        return torch.from_numpy(np.stack(batch))
    if isinstance(s, (int, np.integer)):
        return torch.tensor(batch, dtype=torch.int64)
    if isinstance(s, (float, np.floating)):
        return torch.tensor(batch, dtype=torch.float32)
    if isinstance(s, dict):
        return {k: default_collate_fn([b[k] for b in batch]) for k in s}
    if isinstance(s, (list, tuple)):
        return [default_collate_fn(list(x)) for x in zip(*batch)]
    return batch


default_convert_fn = tud.default_convert


class _DevicePrefetcher:
    """Buffered reader: async H2D of upcoming batches on a side HIP stream."""

    def __init__(self, it, device, depth=2):
        self.it, self.device, self.depth = it, device, depth
        from ..device import side_stream
        self.stream = side_stream(device, key="h2d_prefetch")
        self.q = []

    def _to(self, b):
        if isinstance(b, torch.Tensor):
            return b.pin_memory().to(self.device, non_blocking=True) if b.device.type == "cpu" else b
        if isinstance(b, dict):
            return {k: self._to(v) for k, v in b.items()}
        if isinstance(b, (list, tuple)):
            return type(b)(self._to(v) for v in b)
        return b

    def _fill(self):
        while len(self.q) < self.depth:
            try:
                b = next(self.it)
            except StopIteration:
                return
            with torch.cuda.stream(self.stream):
                d = self._to(b)
                ev = torch.cuda.Event()
                ev.record(self.stream)
            self.q.append((d, ev))

    def __iter__(self):
        return self

    def __next__(self):
        self._fill()
        if not self.q:
            raise StopIteration
        d, ev = self.q.pop(0)
        torch.cuda.current_stream(self.device).wait_event(ev)
        self._fill()
        return d


class DataLoader:
    def __init__(self, dataset, feed_list=None, places=None, return_list=True, batch_sampler=None,
                 batch_size=1, shuffle=False, drop_last=False, collate_fn=None, num_workers=0,
                 use_buffer_reader=True, prefetch_factor=2, use_shared_memory=True, timeout=0,
                 worker_init_fn=None, persistent_workers=False):
        self.dataset = dataset
        self.return_list = return_list
        self.places = places
        self.use_buffer_reader = use_buffer_reader
        self.prefetch = max(1, prefetch_factor)
        collate = collate_fn or default_collate_fn
        if isinstance(dataset, IterableDataset):
            self._loader = tud.DataLoader(dataset, batch_size=batch_size, drop_last=drop_last,
                                          collate_fn=collate, num_workers=num_workers,
                                          worker_init_fn=worker_init_fn, timeout=timeout)
            self.batch_sampler = None
        else:
            if batch_sampler is None:
                batch_sampler = BatchSampler(dataset, shuffle=shuffle, batch_size=batch_size,
                                             drop_last=drop_last)
            self.batch_sampler = batch_sampler
            kw = {}
            if num_workers > 0:
                kw = dict(prefetch_factor=prefetch_factor, persistent_workers=persistent_workers)
            self._loader = tud.DataLoader(dataset, batch_sampler=batch_sampler, collate_fn=collate,
                                          num_workers=num_workers, worker_init_fn=worker_init_fn,
                                          timeout=timeout, **kw)

    def _device(self):
        from .. import device as _d
        p = self.places[0] if isinstance(self.places, (list, tuple)) and self.places else self.places
        return _d._resolve(p)

    def __iter__(self):
        it = iter(self._loader)
        dev = self._device()
        if self.use_buffer_reader and dev.type == "cuda":
            return _DevicePrefetcher(it, dev, self.prefetch)
        return it

    def __len__(self):
        return len(self._loader)

    @staticmethod
    def from_generator(feed_list=None, capacity=None, use_double_buffer=True, iterable=True,
                       return_list=False, use_multiprocess=False, drop_last=True):
        return _GeneratorLoader(return_list)


class _GeneratorLoader:
    def __init__(self, return_list):
        self._gen = None
        self.return_list = return_list

    def set_batch_generator(self, reader, places=None):
        self._gen = reader
        return self

    def set_sample_list_generator(self, reader, places=None):
        def gen():
            for samples in reader():
                yield default_collate_fn(samples)
        self._gen = gen
        return self

    def set_sample_generator(self, reader, batch_size, drop_last=True, places=None):
        def gen():
            buf = []
            for s in reader():
                buf.append(s)
                if len(buf) == batch_size:
                    yield default_collate_fn(buf)
                    buf = []
            if buf and not drop_last:
                yield default_collate_fn(buf)
        self._gen = gen
        return self

    def __iter__(self):
        for b in self._gen():
            yield [torch.as_tensor(np.asarray(x)) if not isinstance(x, torch.Tensor) else x for x in b] \
                if isinstance(b, (list, tuple)) else b


from .token_loader import TokenDataLoader, write_token_file  # noqa: E402,F401
