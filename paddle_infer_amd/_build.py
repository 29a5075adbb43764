"""In-tree build of the native libraries.

* ``_lib/libpiamd_kernels.so`` — every ``csrc/kernels/*.hip`` compiled for gfx950 with hipcc
  (C ABI, loaded with ctypes AFTER torch so it binds to the HIP runtime torch already loaded).
* ``_lib/libpiamd_runtime.so`` — the C++ host runtime (``csrc/runtime/*.cc``: static-graph
  executor scheduler, data-loader ring) built with g++.
* ``_lib/libpiamd_alloc.so`` — the auto-growth best-fit device allocator (``csrc/alloc``,
  host-only HIP runtime code, g++ against the HIP headers; plugged into PyTorch's HIP allocator).
* ``_lib/libpiamd_device.so`` — the device runtime (``csrc/device``: properties, stream pool with
  priorities, events, the host/device range tracer behind ``paddle.profiler``), host-only HIP.
* ``_lib/piamd_agemm.hsaco`` — the hand-scheduled assembly GEMM kernels: ``csrc/asm/gemm_gen.py``
  emits the gfx950 assembly, clang assembles it and ld.lld links the code object (loaded at run
  time by ``csrc/kernels/agemm_host.hip`` through ``hipModuleLoad``).
* ``_lib/piamd_fa.hsaco`` — the hand-scheduled assembly flash-attention dK/dV kernels
  (``csrc/asm/fa_gen.py``; loaded by ``csrc/kernels/fa_asm_host.hip``).
* ``_lib/libpiamd_infer.so`` + ``_lib/pd_infer_run`` — the native C++ inference engine and its
  command-line driver (``csrc/native``: reference ``paddle_inference_api.h`` Config / Predictor /
  Tensor with no Python at run time; CPU loops and gfx950 HIP kernels + rocBLAS).
* the C inference API (reference ``capi_exp`` ``pd_inference_api.h``, header in ``csrc/capi``) is
  part of ``libpiamd_infer.so`` (``csrc/native/pd_capi_native.cc``), no Python.

Incremental: an object is rebuilt only when its source (or a header in the same dir) is newer.
Run ``python -m paddle_infer_amd._build`` or ``__graft_entry__.build()``.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
KDIR = os.path.join(ROOT, "csrc", "kernels")
RDIR = os.path.join(ROOT, "csrc", "runtime")
LIBDIR = os.path.join(ROOT, "_lib")
OBJDIR = os.path.join(ROOT, "_lib", "obj")
KERNEL_LIB = os.path.join(LIBDIR, "libpiamd_kernels.so")
RUNTIME_LIB = os.path.join(LIBDIR, "libpiamd_runtime.so")
CDIR = os.path.join(ROOT, "csrc", "capi")
NDIR = os.path.join(ROOT, "csrc", "native")
NATIVE_LIB = os.path.join(LIBDIR, "libpiamd_infer.so")
NATIVE_RUN = os.path.join(LIBDIR, "pd_infer_run")
ADIR = os.path.join(ROOT, "csrc", "alloc")
ALLOC_LIB = os.path.join(LIBDIR, "libpiamd_alloc.so")
DDIR = os.path.join(ROOT, "csrc", "device")
DEVICE_LIB = os.path.join(LIBDIR, "libpiamd_device.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PIAMD_ARCH", "gfx950")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
ASMDIR = os.path.join(ROOT, "csrc", "asm")
AGEMM_HSACO = os.path.join(LIBDIR, "piamd_agemm.hsaco")
FA_HSACO = os.path.join(LIBDIR, "piamd_fa.hsaco")
LLVM_BIN = os.path.join(ROCM, "lib", "llvm", "bin")

HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-ffp-contract=fast", "-Wno-unused-result"]
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-pthread"]


def _newest_header(d: str) -> float:
    hs = glob.glob(os.path.join(d, "*.h"))
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _file_flags(src: str) -> list:
    """Per-source extra compiler flags from a `// piamd-hipcc-flags: ...` line in the first 40
    lines (e.g. gemm_pipe.hip keeps its MFMA accumulators in VGPRs and operands in AGPRs)."""
    with open(src, encoding="utf-8") as f:
        for _, line in zip(range(40), f):
            if line.startswith("// piamd-hipcc-flags:"):
                return line.split(":", 1)[1].split()
    return []


def _compile(cmd: list, src: str) -> str:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return src


def _build_lib(srcs, out, compiler, flags, link_flags, hdr_time, verbose, jobs) -> bool:
    os.makedirs(OBJDIR, exist_ok=True)
    todo = []
    objs = []
    for s in srcs:
        o = os.path.join(OBJDIR, os.path.basename(s) + ".o")
        objs.append(o)
        if not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), hdr_time):
            todo.append((s, o))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(_compile, [compiler, *flags, *_file_flags(s), "-c", s, "-o", o], s)
                    for s, o in todo]
            for f in cf.as_completed(futs):
                if verbose:
                    print(f"[piamd build] compiled {os.path.basename(f.result())}", flush=True)
    # the object list is recorded next to the library: a removed or added source relinks too
    manifest = out + ".objs"
    listing = "\n".join(sorted(os.path.basename(o) for o in objs))
    same_set = os.path.exists(manifest) and open(manifest).read() == listing
    need_link = todo or not same_set or not os.path.exists(out) or any(
        os.path.getmtime(o) > os.path.getmtime(out) for o in objs)
    if need_link:
        tmp = out + ".tmp"
        _compile([compiler, "-shared", *objs, "-o", tmp, *link_flags], out)
        os.replace(tmp, out)
        with open(manifest, "w") as f:
            f.write(listing)
        if verbose:
            print(f"[piamd build] linked {out}", flush=True)
    return bool(need_link)


def _build_hsaco(gen_name: str, stem: str, out: str, verbose: bool) -> bool:
    gen = os.path.join(ASMDIR, gen_name)
    if os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(gen):
        return False
    os.makedirs(OBJDIR, exist_ok=True)
    src = os.path.join(OBJDIR, stem + ".s")
    obj = os.path.join(OBJDIR, stem + ".o")
    _compile([sys.executable, gen, src], gen)
    _compile([os.path.join(LLVM_BIN, "clang"), "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
              f"-mcpu={ARCH}", "-c", src, "-o", obj], src)
    tmp = out + ".tmp"
    _compile([os.path.join(LLVM_BIN, "ld.lld"), "-shared", obj, "-o", tmp], obj)
    os.replace(tmp, out)
    if verbose:
        print(f"[piamd build] assembled {out}", flush=True)
    return True


def build_asm(verbose: bool = True) -> bool:
    """Generate, assemble and link the assembly code objects (GEMM: gemm_gen.py; flash-attention
    backward: fa_gen.py), each rebuilt when its generator is newer than the code object."""
    a = _build_hsaco("gemm_gen.py", "agemm", AGEMM_HSACO, verbose)
    b = _build_hsaco("fa_gen.py", "fa", FA_HSACO, verbose)
    return a or b


def build_native(verbose: bool = True, jobs: int = 4) -> None:
    """csrc/native → libpiamd_infer.so (hipcc: gfx950 kernels + host C++, rocBLAS) and the
    pd_infer_run driver linked against it (rpath $ORIGIN)."""
    srcs = sorted(glob.glob(os.path.join(NDIR, "*.cc")) + glob.glob(os.path.join(NDIR, "*.hip")))
    lib_srcs = [x for x in srcs if not x.endswith("pd_infer_run.cc")]
    objdir = os.path.join(OBJDIR, "native")
    os.makedirs(objdir, exist_ok=True)
    hdr = _newest_header(NDIR)
    todo, objs = [], []
    for src in lib_srcs:
        o = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(o)
        if not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(src), hdr):
            flags = ["-O3", "-std=c++17", "-fPIC"]
            if src.endswith(".hip"):
                cmd = [HIPCC, *flags, f"--offload-arch={ARCH}", "-c", src, "-o", o]
            else:
                cmd = ["g++", *flags, "-Wall", "-pthread", "-c", src, "-o", o]
            todo.append((cmd, src))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for f in cf.as_completed([ex.submit(_compile, c, src) for c, src in todo]):
                if verbose:
                    print(f"[piamd build] compiled native/{os.path.basename(f.result())}", flush=True)
    if todo or not os.path.exists(NATIVE_LIB) or os.path.getmtime(NATIVE_LIB) < os.path.getmtime(KERNEL_LIB):
        # the 16-bit GPU path (fast_ops.hip) calls the framework's kernels: link libpiamd_kernels.so
        # from the same directory (rpath $ORIGIN), no Python
        _compile([HIPCC, "-shared", *objs, "-o", NATIVE_LIB + ".tmp", f"--offload-arch={ARCH}",
                  f"-L{LIBDIR}", "-lpiamd_kernels", "-Wl,-rpath,$ORIGIN", "-ldl",
                  f"-L{ROCM}/lib", "-lrocblas", "-pthread", f"-Wl,-rpath,{ROCM}/lib"], NATIVE_LIB)
        os.replace(NATIVE_LIB + ".tmp", NATIVE_LIB)
        if verbose:
            print(f"[piamd build] linked {NATIVE_LIB}", flush=True)
    run_src = os.path.join(NDIR, "pd_infer_run.cc")
    if not os.path.exists(NATIVE_RUN) or os.path.getmtime(NATIVE_RUN) < max(
            os.path.getmtime(run_src), os.path.getmtime(NATIVE_LIB), hdr):
        _compile(["g++", "-O2", "-std=c++17", run_src, "-o", NATIVE_RUN + ".tmp", f"-L{LIBDIR}",
                  "-lpiamd_infer", "-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{ROCM}/lib"], run_src)
        os.replace(NATIVE_RUN + ".tmp", NATIVE_RUN)
        if verbose:
            print(f"[piamd build] linked {NATIVE_RUN}", flush=True)


def build(verbose: bool = True, jobs: int | None = None) -> None:
    jobs = jobs or min(8, os.cpu_count() or 4)
    os.makedirs(LIBDIR, exist_ok=True)
    build_asm(verbose)
    ksrcs = sorted(glob.glob(os.path.join(KDIR, "*.hip")))
    if ksrcs:
        _build_lib(ksrcs, KERNEL_LIB, HIPCC, HIP_FLAGS, [f"--offload-arch={ARCH}"],
                   _newest_header(KDIR), verbose, jobs)
    rsrcs = sorted(glob.glob(os.path.join(RDIR, "*.cc")))
    if rsrcs:
        _build_lib(rsrcs, RUNTIME_LIB, "g++", CXX_FLAGS, ["-pthread"], _newest_header(RDIR),
                   verbose, jobs)
    asrcs = sorted(glob.glob(os.path.join(ADIR, "*.cc")))
    if asrcs:  # host-only HIP runtime code (no kernels): g++ against the HIP headers
        _build_lib(asrcs, ALLOC_LIB, "g++", CXX_FLAGS + ["-D__HIP_PLATFORM_AMD__", f"-I{ROCM}/include"],
                   ["-pthread", f"-L{ROCM}/lib", "-lamdhip64", f"-Wl,-rpath,{ROCM}/lib"],
                   _newest_header(ADIR), verbose, jobs)
    dsrcs = sorted(glob.glob(os.path.join(DDIR, "*.cc")))
    if dsrcs:  # device runtime (streams / events / properties / tracer): host HIP runtime code
        _build_lib(dsrcs, DEVICE_LIB, "g++", CXX_FLAGS + ["-D__HIP_PLATFORM_AMD__", f"-I{ROCM}/include"],
                   ["-pthread", f"-L{ROCM}/lib", "-lamdhip64", f"-Wl,-rpath,{ROCM}/lib"],
                   _newest_header(DDIR), verbose, jobs)
    build_native(verbose, jobs)


if __name__ == "__main__":
    build(verbose=True, jobs=int(sys.argv[1]) if len(sys.argv) > 1 else None)
