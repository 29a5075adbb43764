"""``paddle.jit.dy2static`` namespace (reference `python/paddle/jit/dy2static/`). The
AST-conversion machinery has no counterpart here (see jit/__init__.py); the public helpers that
user code touches are provided."""
from . import ProgramTranslator, not_to_static  # noqa: F401


def convert_call(func):
    return func


def convert_ifelse(pred, true_fn, false_fn, *args, **kwargs):
    return true_fn() if bool(pred) else false_fn()
