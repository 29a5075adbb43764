"""``paddle.utils.cpp_extension`` — build user C++/HIP extensions for gfx950.

Parity: reference `python/paddle/utils/cpp_extension/` (load / setup / CppExtension /
CUDAExtension for custom operators). The reference binds custom ops through its PD_BUILD_OP C++
API; here an extension is either
* a plain shared library of ``extern "C"`` HIP launchers (``load`` → ``ctypes.CDLL``), the same
  convention as this framework's own kernel library, or
* a PyTorch C++/HIP extension (``CppExtension`` / ``CUDAExtension`` → torch's builder with
  ``PYTORCH_ROCM_ARCH=gfx950``), whose ops are then wrapped with ``autograd.PyLayer``.
Builds are in-tree (``build_directory``) so the artefacts travel with the repository.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _default_build_dir(name):
    d = os.path.join(os.getcwd(), "build_ext", name)
    os.makedirs(d, exist_ok=True)
    return d


def load(name, sources, extra_cflags=None, extra_cuda_cflags=None, extra_ldflags=None,
         extra_include_paths=None, build_directory=None, verbose=False, arch="gfx950"):
    """Compile ``sources`` (.hip / .cu-as-HIP / .cc / .cpp) into ``lib<name>.so`` and load it."""
    bdir = build_directory or _default_build_dir(name)
    os.makedirs(bdir, exist_ok=True)
    out = os.path.join(bdir, f"lib{name}.so")
    h = hashlib.sha1()
    for s in sources:
        with open(s, "rb") as f:
            h.update(f.read())
    flags = list(extra_cflags or []) + list(extra_cuda_cflags or [])
    h.update(" ".join(flags).encode())
    stamp = out + ".sha1"
    if not (os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == h.hexdigest()):
        inc = sum((["-I", p] for p in (extra_include_paths or [])), [])
        cmd = [HIPCC, "-O3", "-fPIC", "-shared", f"--offload-arch={arch}", "-std=c++17",
               *inc, *flags, *sources, "-o", out, *(extra_ldflags or [])]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True, capture_output=not verbose)
        with open(stamp, "w") as f:
            f.write(h.hexdigest())
    return ctypes.CDLL(out, mode=ctypes.RTLD_GLOBAL)


def CppExtension(sources, *args, **kwargs):  # noqa: N802
    from torch.utils.cpp_extension import CppExtension as _C
    return _C(kwargs.pop("name", "paddle_ext"), sources, *args, **kwargs)


def CUDAExtension(sources, *args, **kwargs):  # noqa: N802
    """HIP extension (torch's CUDAExtension is the HIP builder on ROCm)."""
    os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
    from torch.utils.cpp_extension import CUDAExtension as _C
    return _C(kwargs.pop("name", "paddle_ext"), sources, *args, **kwargs)


def setup(**attr):
    os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
    from setuptools import setup as _setup
    from torch.utils.cpp_extension import BuildExtension
    attr.setdefault("cmdclass", {"build_ext": BuildExtension})
    return _setup(**attr)


def get_build_directory(verbose=False):
    return _default_build_dir("")
