"""List reference ``__all__`` names missing from paddle_infer_amd, module by module.

Parses the reference's ``__init__.py`` files with ``ast`` (nothing in them is imported or run)."""
import ast
import importlib
import os
import sys

REF = "/root/reference/python/paddle"
MODS = ["", "nn", "nn.functional", "nn.initializer", "static", "static.nn", "distributed", "distributed.fleet",
        "optimizer", "optimizer.lr", "io", "jit", "inference", "amp", "device", "linalg", "fft", "signal",
        "metric", "vision", "vision.transforms", "vision.models", "text", "utils", "autograd", "incubate",
        "incubate.nn", "incubate.nn.functional", "sparse", "distribution", "profiler", "regularizer",
        "callbacks", "hub", "onnx", "quantization", "geometric", "audio"]


def ref_all(mod):
    base = os.path.join(REF, *mod.split(".")) if mod else REF
    path = os.path.join(base, "__init__.py") if os.path.isdir(base) else base + ".py"
    if not os.path.exists(path):
        return None
    tree = ast.parse(open(path).read())
    names = []
    for node in ast.walk(tree):
        if isinstance(node, ast.Assign) and any(getattr(t, "id", None) == "__all__" for t in node.targets):
            try:
                names += list(ast.literal_eval(node.value))
            except ValueError:
                pass
        if isinstance(node, ast.AugAssign) and getattr(node.target, "id", None) == "__all__":
            try:
                names += list(ast.literal_eval(node.value))
            except ValueError:
                pass
    return names


def main():
    total = 0
    for mod in MODS:
        names = ref_all(mod)
        if not names:
            continue
        try:
            m = importlib.import_module("paddle_infer_amd" + ("." + mod if mod else ""))
        except Exception as e:  # noqa: BLE001
            print(f"[{mod}] MODULE MISSING ({e.__class__.__name__}: {e})")
            total += len(names)
            continue
        miss = [n for n in names if not hasattr(m, n)]
        total += len(miss)
        if miss:
            print(f"[{mod or 'paddle'}] {len(miss)}/{len(names)} missing: {' '.join(miss)}")
    print("total missing:", total)


if __name__ == "__main__":
    sys.exit(main())
