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
    elif kind == "bf16acc":
        c0 = torch.randn(M, N, device="cuda", generator=gen).bfloat16()
        c = c0.clone()
        asm_gemm(a, b, ta, tb, out=c, accumulate=True, ksplit=ksplit)
        c = c.float()
        r = r + c0.float()
    else:
        c0 = torch.randn(M, N, device="cuda", generator=gen)
        c = c0.clone()
        asm_gemm(a, b, ta, tb, out=c, accumulate=True, ksplit=ksplit)
        r = r + c0
    torch.cuda.synchronize()
    err = (c - r).abs().max().item()
    tol = 0.02 * r.abs().max().item() + 1e-3 if kind.startswith("bf16") else 1e-3 * (K ** 0.5)
    return err, tol


def small():
    gen = torch.Generator(device="cuda").manual_seed(0)
    fails = 0
    cases = [(256, 256, 128), (256, 256, 192), (512, 256, 256), (256, 512, 320), (304, 264, 128),
             (1000, 1008, 448), (2048, 768, 512), (136, 2056, 256), (4352, 4104, 256),
             (8192, 2048, 384)]
    for (M, N, K) in cases:
        for ta, tb in ((False, True), (True, False), (False, False), (True, True)):
            for kind in ("bf16", "bf16acc", "f32", "f32acc"):
                err, tol = check(M, N, K, ta, tb, kind, gen=gen)
                ok = err <= tol
                fails += not ok
                print(json.dumps({"M": M, "N": N, "K": K, "ta": ta, "tb": tb, "kind": kind,
                                  "err": round(err, 5), "tol": round(tol, 5), "ok": ok}), flush=True)
    for (M, N, K, ks, kind) in [(512, 512, 1024, 4, "f32acc"), (256, 768, 512, 2, "f32acc"),
                                (512, 256, 1024, 4, "bf16acc")]:
        err, tol = check(M, N, K, True, False, kind, ksplit=ks, gen=gen)
        fails += err > tol
        print(json.dumps({"M": M, "N": N, "K": K, "ksplit": ks, "err": err, "ok": err <= tol}), flush=True)
    fails += fused(gen)
    print("FAILS", fails)
    return fails


def fused(gen):
    from paddle_infer_amd.ops.gemm import asm_gemm, _act_grad_ref
    from paddle_infer_amd.ops.activation import _ref_act, ACTS
    fails = 0
    for (M, N, K) in [(256, 256, 128), (512, 1024, 256), (304, 520, 192)]:
        a = torch.randn(M, K, device="cuda", generator=gen).bfloat16()
        b = (0.1 * torch.randn(N, K, device="cuda", generator=gen)).bfloat16()
        bias = torch.randn(N, device="cuda", generator=gen).bfloat16()
        r = a.float() @ b.float().t()
        for act in ("none", "gelu_tanh", "relu"):
            aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            c = asm_gemm(a, b, trans_b=True, epi="bias_act", act=act, bias=bias, aux=aux)
            pre = (r + bias.float()).bfloat16()
            ref_c = _ref_act(pre.float(), ACTS[act])
            e1 = (aux.float() - pre.float()).abs().max().item()
            e2 = (c.float() - ref_c).abs().max().item()
            ok = e1 <= 0.02 * pre.float().abs().max().item() and e2 <= 0.02 * ref_c.abs().max().item() + 1e-2
            fails += not ok
            print(json.dumps({"fused": "bias_act", "act": act, "M": M, "N": N, "K": K,
                              "aux_err": round(e1, 4), "c_err": round(e2, 4), "ok": ok}), flush=True)
            if act == "none":
                continue
            h = torch.randn(M, N, device="cuda", generator=gen).bfloat16()
            d = asm_gemm(a, b, trans_b=True, epi="dact", act=act, aux=h)
            ref_d = r * _act_grad_ref(h, ACTS[act])
            e3 = (d.float() - ref_d).abs().max().item()
            ok = e3 <= 0.02 * ref_d.abs().max().item() + 1e-2
            fails += not ok
            print(json.dumps({"fused": "dact", "act": act, "M": M, "N": N, "K": K,
                              "err": round(e3, 4), "ok": ok}), flush=True)
    # bias without aux
    a = torch.randn(256, 128, device="cuda", generator=gen).bfloat16()
    b = torch.randn(256, 128, device="cuda", generator=gen).bfloat16()
    c = asm_gemm(a, b, trans_b=True, epi="bias_act", act="gelu_tanh", bias=None, aux=None)
    ref_c = _ref_act((a.float() @ b.float().t()).bfloat16().float(), 1)
    e = (c.float() - ref_c).abs().max().item()
    fails += e > 0.02 * ref_c.abs().max().item() + 1e-2
    print(json.dumps({"fused": "act_noaux_nobias", "err": e}), flush=True)
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
                 "head": (2048, 50304),
                 # BERT-Large (T = batch 128 × seq 128 = 16384)
                 "bqkv": (1024, 3072), "bout": (1024, 1024), "bffn1": (1024, 4096), "bffn2": (4096, 1024)}
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


def probe(rounds):
    """Loop efficiency vs per-tile overhead: long-K (few tiles, many K-blocks) and short-K
    (many tiles) products in both layouts, one line per case (asm only; hipBLASLt alongside)."""
    from paddle_infer_amd.ops.gemm import asm_gemm
    gen = torch.Generator(device="cuda").manual_seed(0)
    cases = [("nt_longK", 4096, 4096, 32768, False, True), ("tn_longK", 4096, 4096, 32768, True, False),
             ("nt_ffn1", 98304, 8192, 2048, False, True), ("nt_ffn2", 98304, 2048, 8192, False, True)]
    for name, M, N, K, ta, tb in cases:
        a = torch.randn((K, M) if ta else (M, K), device="cuda", generator=gen).bfloat16()
        b = torch.randn((N, K) if tb else (K, N), device="cuda", generator=gen).bfloat16()
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        A = a.t() if ta else a
        B = b.t() if tb else b
        fns = {"asm": lambda: asm_gemm(a, b, ta, tb, out=c), "hipblaslt": lambda: torch.mm(A, B)}
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        ts = {k: [] for k in fns}
        for _ in range(rounds):
            for k, f in fns.items():
                ts[k].append(timeit(f, 3))
        fl = 2.0 * M * N * K
        print(json.dumps({"case": name, **{k: round(fl / statistics.median(v) / 1e9, 1) for k, v in ts.items()},
                          "hsaco": os.path.basename(os.environ.get("PIAMD_AGEMM_HSACO", "default"))}), flush=True)


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
    if args.stage == "probe":
        probe(args.rounds)
        return
    bench(args.T, args.rounds, args.shapes.split(","))


if __name__ == "__main__":
    main()
