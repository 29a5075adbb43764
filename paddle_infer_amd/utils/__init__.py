"""``paddle.utils``: NaN/Inf checker, FLOPs counter, deprecation helper, run_check,
cpp_extension (in-tree HIP extension builder)."""
from . import nan_inf  # noqa: F401
from . import flops  # noqa: F401
from . import cpp_extension  # noqa: F401


def deprecated(update_to="", since="", reason="", level=0):
    def deco(fn):
        return fn
    return deco


def run_check():
    """Reference `paddle.utils.run_check`: build the kernels, run one kernel on every GPU."""
    import torch
    from .. import _build
    from ..ops import _lib
    _build.build(verbose=False)
    n = torch.cuda.device_count() if torch.cuda.is_available() else 0
    if n == 0:
        print("paddle_infer_amd is installed (CPU only: no MI355X visible).")
        return
    from ..ops import layer_norm
    for i in range(n):
        x = torch.randn(4, 256, device=f"cuda:{i}", dtype=torch.bfloat16)
        layer_norm(x, None, None)
    torch.cuda.synchronize()
    _lib.lib()
    print(f"paddle_infer_amd works well on {n} GPU(s) (HIP kernel library {_lib.lib_path()}).")


def unique_name(prefix="tmp"):
    from ..static.framework import unique_name as _u
    return _u(prefix)


def try_import(module_name):
    import importlib
    return importlib.import_module(module_name)


def require_version(min_version, max_version=None):
    """Reference `utils/install_check.py`-style version gate: raise unless this framework's version
    lies in [min_version, max_version]."""
    from .. import __version__

    def parse(v):
        return tuple(int(p) for p in str(v).split(".")[:3] if p.isdigit())
    cur = parse(__version__)
    if parse(min_version) > cur or (max_version is not None and cur > parse(max_version)):
        raise Exception(f"paddle_infer_amd version {__version__} is not in "
                        f"[{min_version}, {max_version or 'any'}]")
    return True
