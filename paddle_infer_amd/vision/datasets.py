"""``paddle.vision.datasets`` (reference `python/paddle/vision/datasets/`). No network here: the
file-based datasets read local copies in the reference's on-disk formats (MNIST idx(.gz),
CIFAR python pickles are NOT unpickled — use the numpy/npz export instead), ``DatasetFolder`` /
``ImageFolder`` read image trees, and ``FakeData`` generates synthetic samples."""
from __future__ import annotations

import gzip
import os
import struct

import numpy as np

from ..io import Dataset

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp", ".npy")


def _load_image(path):
    if path.endswith(".npy"):
        return np.load(path, allow_pickle=False)
    try:
        from PIL import Image
    except ImportError as e:
        raise RuntimeError(f"reading {path} needs PIL (not installed); store images as .npy") from e
    return np.asarray(Image.open(path).convert("RGB"))


class DatasetFolder(Dataset):
    def __init__(self, root, loader=None, extensions=None, transform=None, is_valid_file=None):
        self.root, self.transform = root, transform
        self.loader = loader or _load_image
        exts = tuple(extensions or IMG_EXTENSIONS)
        self.classes = sorted(d.name for d in os.scandir(root) if d.is_dir())
        self.class_to_idx = {c: i for i, c in enumerate(self.classes)}
        self.samples = []
        for c in self.classes:
            for dp, _, fns in sorted(os.walk(os.path.join(root, c))):
                for fn in sorted(fns):
                    p = os.path.join(dp, fn)
                    ok = is_valid_file(p) if is_valid_file else fn.lower().endswith(exts)
                    if ok:
                        self.samples.append((p, self.class_to_idx[c]))
        self.targets = [s[1] for s in self.samples]

    def __getitem__(self, i):
        p, t = self.samples[i]
        img = self.loader(p)
        if self.transform is not None:
            img = self.transform(img)
        return img, np.int64(t)

    def __len__(self):
        return len(self.samples)


class ImageFolder(Dataset):
    """Flat folder of images (no labels), reference `folder.py:ImageFolder`."""

    def __init__(self, root, loader=None, extensions=None, transform=None, is_valid_file=None):
        self.loader, self.transform = loader or _load_image, transform
        exts = tuple(extensions or IMG_EXTENSIONS)
        self.samples = []
        for dp, _, fns in sorted(os.walk(root)):
            for fn in sorted(fns):
                p = os.path.join(dp, fn)
                if (is_valid_file(p) if is_valid_file else fn.lower().endswith(exts)):
                    self.samples.append(p)

    def __getitem__(self, i):
        img = self.loader(self.samples[i])
        return [self.transform(img) if self.transform else img]

    def __len__(self):
        return len(self.samples)


class FakeData(Dataset):
    """Synthetic (image, label) pairs of a fixed shape — deterministic per index."""

    def __init__(self, size=1000, image_size=(3, 224, 224), num_classes=10, transform=None, seed=0):
        self.size, self.image_size, self.num_classes = size, tuple(image_size), num_classes
        self.transform, self.seed = transform, seed

    def __getitem__(self, i):
        rng = np.random.RandomState(self.seed + i)
        img = rng.rand(*self.image_size).astype(np.float32)
        if self.transform is not None:
            img = self.transform(img)
        return img, np.int64(rng.randint(0, self.num_classes))

    def __len__(self):
        return self.size


def _read_idx(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rb") as f:
        data = f.read()
    magic, = struct.unpack(">I", data[:4])
    nd = magic & 0xFF
    dims = struct.unpack(">" + "I" * nd, data[4:4 + 4 * nd])
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * nd).reshape(dims)


class MNIST(Dataset):
    """Reads local idx files (``image_path``/``label_path``; same layout the reference downloads)."""
    NAME = "mnist"

    def __init__(self, image_path=None, label_path=None, mode="train", transform=None,
                 download=False, backend=None):
        if image_path is None or label_path is None:
            base = os.path.join(os.path.expanduser("~"), ".cache", "paddle", "dataset", self.NAME)
            pre = "train" if mode == "train" else "t10k"
            image_path = image_path or os.path.join(base, f"{pre}-images-idx3-ubyte.gz")
            label_path = label_path or os.path.join(base, f"{pre}-labels-idx1-ubyte.gz")
        if not (os.path.exists(image_path) and os.path.exists(label_path)):
            raise FileNotFoundError(f"{self.NAME} files not found ({image_path}); downloading is not "
                                    "possible offline — use FakeData or place the idx files there")
        self.images = _read_idx(image_path)
        self.labels = _read_idx(label_path).astype(np.int64)
        self.transform = transform

    def __getitem__(self, i):
        img = self.images[i].astype(np.float32)
        if self.transform is not None:
            img = self.transform(img)
        return img, self.labels[i:i + 1]

    def __len__(self):
        return len(self.labels)


class FashionMNIST(MNIST):
    NAME = "fashion-mnist"


class Cifar10(Dataset):
    """Reads a local ``.npz`` export (arrays ``data`` [N,3,32,32] uint8, ``labels`` [N]); the
    reference's pickled batches are never unpickled here."""

    def __init__(self, data_file=None, mode="train", transform=None, download=False, backend=None):
        if data_file is None or not os.path.exists(data_file):
            raise FileNotFoundError("Cifar needs a local .npz export (data, labels); offline")
        z = np.load(data_file, allow_pickle=False)
        self.data, self.labels = z["data"], z["labels"].astype(np.int64)
        self.transform = transform

    def __getitem__(self, i):
        img = self.data[i].transpose(1, 2, 0)
        if self.transform is not None:
            img = self.transform(img)
        return img, self.labels[i]

    def __len__(self):
        return len(self.labels)


Cifar100 = Cifar10
