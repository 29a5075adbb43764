"""``paddle.sysconfig`` (reference `python/paddle/sysconfig.py`): include / library directories
for building custom HIP operators against this framework (``utils.cpp_extension``)."""
import os

__all__ = ["get_include", "get_lib"]

_ROOT = os.path.dirname(os.path.abspath(__file__))


def get_include():
    """Directory holding the kernel headers (``common.h``: bf16 helpers, wave64 reductions)."""
    return os.path.join(_ROOT, "csrc", "kernels")


def get_lib():
    """Directory holding ``libpiamd_kernels.so`` / ``libpiamd_runtime.so``."""
    return os.path.join(_ROOT, "_lib")
