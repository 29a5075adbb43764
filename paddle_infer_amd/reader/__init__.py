"""``paddle.reader`` / ``paddle.batch`` — legacy reader decorators (reference
`python/paddle/reader/decorator.py`, `python/paddle/batch.py`). A reader is a zero-argument
callable returning an iterator of samples."""
from __future__ import annotations

import itertools
import queue
import random
import threading

__all__ = ["batch", "cache", "map_readers", "buffered", "compose", "chain", "shuffle", "firstn",
           "xmap_readers", "multiprocess_reader", "ComposeNotAligned"]


class ComposeNotAligned(ValueError):
    pass


def batch(reader, batch_size, drop_last=False):
    if batch_size <= 0:
        raise ValueError(f"batch_size should be a positive integer value, but got {batch_size}")

    def r():
        b = []
        for s in reader():
            b.append(s)
            if len(b) == batch_size:
                yield b
                b = []
        if b and not drop_last:
            yield b
    return r


def cache(reader):
    data = list(reader())
    return lambda: iter(data)


def map_readers(func, *readers):
    def r():
        for items in zip(*[rd() for rd in readers]):
            yield func(*items)
    return r


def shuffle(reader, buf_size):
    def r():
        buf = []
        for s in reader():
            buf.append(s)
            if len(buf) >= buf_size:
                random.shuffle(buf)
                yield from buf
                buf = []
        random.shuffle(buf)
        yield from buf
    return r


def chain(*readers):
    return lambda: itertools.chain(*[r() for r in readers])


def compose(*readers, check_alignment=True):
    def flat(x):
        return x if isinstance(x, tuple) else (x,)

    def r():
        its = [rd() for rd in readers]
        for outs in itertools.zip_longest(*its):
            if any(o is None for o in outs):
                if check_alignment:
                    raise ComposeNotAligned("outputs of readers are not aligned.")
                return
            yield sum((flat(o) for o in outs), ())
    return r


def buffered(reader, size):
    end = object()

    def r():
        q = queue.Queue(maxsize=size)

        def fill():
            for s in reader():
                q.put(s)
            q.put(end)
        threading.Thread(target=fill, daemon=True).start()
        while True:
            s = q.get()
            if s is end:
                return
            yield s
    return r


def firstn(reader, n):
    return lambda: itertools.islice(reader(), n)


def xmap_readers(mapper, reader, process_num, buffer_size, order=False):
    """Map with a thread pool (``process_num`` workers), optionally keeping the input order."""
    from concurrent.futures import ThreadPoolExecutor

    def r():
        with ThreadPoolExecutor(process_num) as ex:
            if order:
                yield from ex.map(mapper, reader())
            else:
                futs = [ex.submit(mapper, s) for s in reader()]
                for f in futs:
                    yield f.result()
    return r


def multiprocess_reader(readers, use_pipe=True, queue_size=1000):
    return chain(*readers)
