"""Build assembly-GEMM code objects with alternative main-loop slot schedules (measurement):

  python tools/agemm_sched_sweep.py NAME=Y_END,BAR1,DMA0,DMA_GAP,BAR2,X0,X_END ...
  -> _lib/piamd_agemm_s_<NAME>.hsaco (time with PIAMD_AGEMM_HSACO=<file>)"""
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def main():
    from paddle_infer_amd import _build
    for spec in sys.argv[1:]:
        name, sched = spec.split("=")
        env = dict(os.environ, PIAMD_AGEMM_SCHED=sched)
        src = os.path.join(_build.OBJDIR, f"agemm_s_{name}.s")
        obj = src[:-2] + ".o"
        out = os.path.join(_build.LIBDIR, f"piamd_agemm_s_{name}.hsaco")
        os.makedirs(_build.OBJDIR, exist_ok=True)
        subprocess.check_call([sys.executable, os.path.join(_build.ASMDIR, "gemm_gen.py"), src], env=env)
        subprocess.check_call([os.path.join(_build.LLVM_BIN, "clang"), "-x", "assembler", "-target",
                               "amdgcn-amd-amdhsa", f"-mcpu={_build.ARCH}", "-c", src, "-o", obj])
        subprocess.check_call([os.path.join(_build.LLVM_BIN, "ld.lld"), "-shared", obj, "-o", out])
        print(out)


if __name__ == "__main__":
    main()
