"""``paddle.linalg`` (reference `python/paddle/linalg.py`): the linear-algebra namespace, backed by
the functions in ``paddle_infer_amd.tensor`` (torch.linalg / rocSOLVER on the GPU)."""
from .tensor import linalg as _ns, matmul, multi_dot  # noqa: F401

for _k, _v in vars(_ns).items():
    if not _k.startswith("_"):
        globals()[_k] = _v.__func__ if isinstance(_v, staticmethod) else _v
del _k, _v

__all__ = ["cholesky", "norm", "cond", "cov", "corrcoef", "inv", "eig", "eigvals", "multi_dot",
           "matrix_rank", "svd", "qr", "lu", "lu_unpack", "matrix_power", "det", "slogdet", "eigh",
           "eigvalsh", "pinv", "solve", "cholesky_solve", "triangular_solve", "lstsq"]
