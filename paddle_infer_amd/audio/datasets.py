"""Audio datasets (reference `audio/datasets/`: ESC50, TESS). They download archives; without
network access they read an already-extracted local ``data_dir`` of WAV files + labels."""
from __future__ import annotations

import os

from .backends import load

__all__ = ["ESC50", "TESS"]


class _AudioFolder:
    def __init__(self, mode="train", data_dir=None, feat_type="raw", **kw):
        if data_dir is None:
            raise RuntimeError(f"{type(self).__name__}: no network access; pass data_dir=")
        self.files = sorted(os.path.join(r, f) for r, _, fs in os.walk(data_dir) for f in fs
                            if f.endswith(".wav"))
        labels = sorted({os.path.basename(os.path.dirname(p)) for p in self.files})
        self.label_ids = {l: i for i, l in enumerate(labels)}

    def __getitem__(self, i):
        wav, _ = load(self.files[i])
        return wav[0], self.label_ids[os.path.basename(os.path.dirname(self.files[i]))]

    def __len__(self):
        return len(self.files)


class ESC50(_AudioFolder):
    pass


class TESS(_AudioFolder):
    pass
