"""Bring-up check + timing of the assembly GEMM against an fp32 reference and hipBLASLt.

  python tools/agemm_check.py --stage small     # tiny shapes, every layout / epilogue
  python tools/agemm_check.py --stage bench     # GPT-3 1.3B training shapes vs hipBLASLt
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def ref(a, b, ta, tb):
    A = a.t() if ta else a
    B = b.t() if tb else b
    return A.float() @ B.float()


def check(M, N, K, ta, tb, kind, ksplit=1, gen=None):
    from paddle_infer_amd.ops.gemm import asm_gemm
    a = torch.randn((K, M) if ta else (M, K), device="cuda", generator=gen).bfloat16()
    b = torch.randn((N, K) if tb else (K, N), device="cuda", generator=gen).bfloat16()
    r = ref(a, b, ta, tb)
    if kind == "bf16":
        c = asm_gemm(a, b, ta, tb, ksplit=ksplit).float()
    elif kind == "f32":
        c = asm_gemm(a, b, ta, tb, out_f32=True, ksplit=ksplit)
    else:
        c0 = torch.randn(M, N, device="cuda", generator=gen)
        c = c0.clone()
        asm_gemm(a, b, ta, tb, out=c, accumulate=True, ksplit=ksplit)
        r = r + c0
    torch.cuda.synchronize()
    err = (c - r).abs().max().item()
    tol = 0.02 * r.abs().max().item() + 1e-3 if kind == "bf16" else 1e-3 * (K ** 0.5)
    return err, tol


def small():
    gen = torch.Generator(device="cuda").manual_seed(0)
    fails = 0
    cases = [(256, 256, 128), (256, 256, 192), (512, 256, 256), (256, 512, 320), (304, 264, 128),
             (1000, 1008, 448), (2048, 768, 512), (136, 2056, 256)]
    for (M, N, K) in cases:
        for ta, tb in ((False, True), (True, False), (False, False), (True, True)):
            for kind in ("bf16", "f32", "f32acc"):
                err, tol = check(M, N, K, ta, tb, kind, gen=gen)
                ok = err <= tol
                fails += not ok
                print(json.dumps({"M": M, "N": N, "K": K, "ta": ta, "tb": tb, "kind": kind,
                                  "err": round(err, 5), "tol": round(tol, 5), "ok": ok}), flush=True)
    for (M, N, K, ks) in [(512, 512, 1024, 4), (256, 768, 512, 2)]:
        err, tol = check(M, N, K, True, False, "f32acc", ksplit=ks, gen=gen)
        fails += err > tol
        print(json.dumps({"M": M, "N": N, "K": K, "ksplit": ks, "err": err, "ok": err <= tol}), flush=True)
    print("FAILS", fails)
    return fails


def timeit(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def bench(T, rounds, shapes):
    from paddle_infer_amd.ops.gemm import asm_gemm, pick_ksplit
    allshapes = {"qkv": (2048, 6144), "out": (2048, 2048), "ffn1": (2048, 8192), "ffn2": (8192, 2048),
                 "head": (2048, 50304)}
    gen = torch.Generator(device="cuda").manual_seed(0)
    for name in shapes:
        K, N = allshapes[name]
        x = torch.randn(T, K, device="cuda", generator=gen).bfloat16()
        dy = (0.1 * torch.randn(T, N, device="cuda", generator=gen)).bfloat16()
        w = (0.02 * torch.randn(K, N, device="cuda", generator=gen)).bfloat16()
        wt = w.t().contiguous()
        mg = torch.zeros(K, N, device="cuda", dtype=torch.float32)
        fl = 2.0 * T * K * N
        ks = pick_ksplit(K, N, T)
        cases = [
            ("fwd", "hipblaslt", lambda: torch.mm(x, wt.t())),
            ("fwd", "asm", lambda: asm_gemm(x, wt, trans_b=True)),
            ("dgrad", "hipblaslt", lambda: torch.mm(dy, w.t())),
            ("dgrad", "asm", lambda: asm_gemm(dy, w, trans_b=True)),
            ("wgrad", "hipblaslt", lambda: mg.addmm_(x.t().float(), dy.float()) if False else mg.add_(torch.mm(x.t(), dy))),
            ("wgrad", f"asm_ks{ks}", lambda: asm_gemm(x, dy, trans_a=True, out=mg, accumulate=True, ksplit=ks)),
        ]
        outs = {}
        for pas, impl, fn in cases:
            if pas == "wgrad":
                mg.zero_()
                fn()
                outs[(pas, impl)] = mg.clone()
            else:
                outs[(pas, impl)] = fn().float()
        torch.cuda.synchronize()
        times = {(p, i): [] for p, i, _ in cases}
        for _ in range(rounds):
            for pas, impl, fn in cases:
                times[(pas, impl)].append(timeit(fn, 5))
        base = {}
        for (pas, impl), ts in times.items():
            ms = statistics.median(ts)
            if impl == "hipblaslt":
                base[pas] = ms
            ref_o = outs[(pas, "hipblaslt")]
            err = (outs[(pas, impl)] - ref_o).abs().max().item()
            print(json.dumps({"shape": name, "T": T, "pass": pas, "impl": impl, "ms": round(ms, 4),
                              "tflops": round(fl / ms / 1e9, 1),
                              "vs_blaslt": round(base[pas] / ms, 3),
                              "max_diff_vs_blaslt": round(err, 4)}), flush=True)
        del x, dy, w, wt, mg, outs
        torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stage", default="small")
    ap.add_argument("--T", type=int, default=98304)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--shapes", default="qkv,out,ffn1,ffn2,head")
    args = ap.parse_args()
    import paddle_infer_amd  # noqa: F401
    if args.stage == "small":
        sys.exit(1 if small() else 0)
    bench(args.T, args.rounds, args.shapes.split(","))


if __name__ == "__main__":
    main()
