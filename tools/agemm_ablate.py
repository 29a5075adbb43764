"""Build ablated variants of the assembly GEMM (measurement only; results are garbage):

  python tools/agemm_ablate.py nodma noreads nomfma nobar   # -> _lib/piamd_agemm_abl_<tag>.hsaco

then time with PIAMD_AGEMM_HSACO=<file> python tools/agemm_check.py --stage probe (one process per
variant: the code object is loaded once per process)."""
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def main():
    from paddle_infer_amd import _build
    for tag in sys.argv[1:] or ["nodma", "noreads", "nomfma"]:
        env = dict(os.environ, PIAMD_AGEMM_ABL=tag.replace("+", ","))
        src = os.path.join(_build.OBJDIR, f"agemm_abl_{tag}.s")
        obj = src[:-2] + ".o"
        out = os.path.join(_build.LIBDIR, f"piamd_agemm_abl_{tag}.hsaco")
        os.makedirs(_build.OBJDIR, exist_ok=True)
        subprocess.check_call([sys.executable, os.path.join(_build.ASMDIR, "gemm_gen.py"), src], env=env)
        subprocess.check_call([os.path.join(_build.LLVM_BIN, "clang"), "-x", "assembler", "-target",
                               "amdgcn-amd-amdhsa", f"-mcpu={_build.ARCH}", "-c", src, "-o", obj])
        subprocess.check_call([os.path.join(_build.LLVM_BIN, "ld.lld"), "-shared", obj, "-o", out])
        print(out)


if __name__ == "__main__":
    main()
