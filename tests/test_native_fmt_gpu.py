"""GPT fused_multi_transformer on the native C++ engine (no Python inside it, driven through its C
API): a hand-built context program and a decode program (reference slot names, fp32 weights run in
bf16) against the Python Predictor over the same shared KV caches — the context output, the cache
contents and every decode step match; decode latency is reported next to the Python Predictor's.
Also the C++ driver `pd_infer_run` over the decode program (caches resident across Run calls,
TimeStep advanced per call), eager vs hipGraph replay."""
import os
import subprocess
import time

import numpy as np
import pytest
import torch

from fmt_wire import write_fmt_program
from native_capi import PD_PRECISION_BFLOAT16, Predictor

pytestmark = pytest.mark.gpu
RUN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "paddle_infer_amd", "_lib",
                   "pd_infer_run")


def _python_predictor(prefix):
    from paddle_infer_amd import inference as pinf
    c = pinf.Config(prefix + ".pdmodel", prefix + ".pdiparams")
    c.enable_use_gpu(256, 0)
    c.exp_enable_mixed_precision(pinf.PrecisionType.Bfloat16)
    return pinf.create_predictor(c)


@pytest.mark.parametrize("E,H,L,B", [(256, 4, 2, 2), (512, 4, 2, 1)])
def test_native_fmt_context_and_decode_match_python_predictor(tmp_path, E, H, L, B):
    from paddle_infer_amd.incubate.nn import FusedMultiTransformer
    torch.manual_seed(0)
    S, MAXS, STEPS = 8, 32, 6
    layer = FusedMultiTransformer(E, H, 2 * E, num_layers=L)
    layer.eval()
    ctx_p, dec_p = str(tmp_path / "ctx"), str(tmp_path / "dec")
    write_fmt_program(layer, ctx_p, False, L, E)
    write_fmt_program(layer, dec_p, True, L, E)
    D = E // H
    dev = torch.device("cuda")
    x = torch.randn(B, S, E).to(torch.bfloat16).to(dev)
    xs = [torch.randn(B, 1, E).to(torch.bfloat16).to(dev) for _ in range(STEPS)]
    caches_py = [torch.zeros(2, B, H, MAXS, D, dtype=torch.bfloat16, device=dev) for _ in range(L)]
    caches_nat = [torch.zeros_like(c) for c in caches_py]

    # Python Predictor
    pc, pd = _python_predictor(ctx_p), _python_predictor(dec_p)
    pc.get_input_handle("x").share_external_data(x)
    for i, c in enumerate(caches_py):
        pc.get_input_handle(f"cache_kv.{i}").share_external_data(c)
    assert pc.run()
    ref_ctx = pc.get_output_handle("out").to_torch().float().cpu()
    ref_steps, py_ms = [], []
    for t, xt in enumerate(xs):
        pd.get_input_handle("x").share_external_data(xt)
        for i, c in enumerate(caches_py):
            pd.get_input_handle(f"cache_kv.{i}").share_external_data(c)
        pd.get_input_handle("time_step").copy_from_cpu(np.array([S + t], dtype=np.int32))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        assert pd.run()
        ref_steps.append(pd.get_output_handle("out").to_torch().float().cpu())
        py_ms.append((time.perf_counter() - t0) * 1e3)

    # native engine through its C API, caches shared zero-copy
    nc = Predictor(ctx_p, 0, PD_PRECISION_BFLOAT16)
    nd = Predictor(dec_p, 0, PD_PRECISION_BFLOAT16)
    torch.cuda.synchronize()
    nc.share("x", x)
    for i, c in enumerate(caches_nat):
        nc.share(f"cache_kv.{i}", c)
    nc.run()
    got_ctx = torch.from_numpy(nc.fetch_float("out", (B, S, E)))
    torch.testing.assert_close(got_ctx, ref_ctx, rtol=2e-2, atol=2e-2)
    for cn, cp in zip(caches_nat, caches_py):
        torch.testing.assert_close(cn[:, :, :, :S].float(), cp[:, :, :, :S].float(), rtol=2e-2, atol=2e-2)
    for i, c in enumerate(caches_nat):
        nd.share(f"cache_kv.{i}", c)
    nat_ms = []
    for t, xt in enumerate(xs):
        nd.share("x", xt)
        nd.feed("time_step", np.array([S + t], dtype=np.int32))
        t0 = time.perf_counter()
        nd.run()
        got = torch.from_numpy(nd.fetch_float("out", (B, 1, E)))
        nat_ms.append((time.perf_counter() - t0) * 1e3)
        torch.testing.assert_close(got, ref_steps[t], rtol=3e-2, atol=3e-2)
    for cn, cp in zip(caches_nat, caches_py):
        torch.testing.assert_close(cn.float(), cp.float(), rtol=3e-2, atol=3e-2)
    nc.close()
    nd.close()
    print(f"\nFMT E{E} L{L} B{B} decode step: native {np.median(nat_ms[1:]):.3f} ms, "
          f"python predictor {np.median(py_ms[1:]):.3f} ms")


def test_pd_infer_run_decode_loop_graph_matches_eager(tmp_path):
    """pd_infer_run over the decode program: caches fed once (fp32 zeros, converted to bf16 and kept
    resident), TimeStep advanced per Run; the hipGraph replay gives the eager outputs."""
    from paddle_infer_amd.incubate.nn import FusedMultiTransformer
    torch.manual_seed(1)
    E, H, L, B, MAXS = 256, 4, 2, 1, 64
    layer = FusedMultiTransformer(E, H, 2 * E, num_layers=L)
    layer.eval()
    dec_p = str(tmp_path / "dec")
    write_fmt_program(layer, dec_p, True, L, E)
    D = E // H
    files = {"x": (np.random.RandomState(0).randn(B, 1, E).astype(np.float32), "float32"),
             "time_step": (np.array([3], dtype=np.int32), "int32")}
    for i in range(L):
        files[f"cache_kv.{i}"] = (np.random.RandomState(i + 1).randn(2, B, H, MAXS, D).astype(np.float32) * 0.5,
                                  "float32")
    args = []
    for n, (a, dt) in files.items():
        f = str(tmp_path / f"in_{n}.bin")
        a.tofile(f)
        args += ["--input", n, dt, ",".join(map(str, a.shape)), f]
    outs = {}
    for mode in ("eager", "graph"):
        od = tmp_path / mode
        od.mkdir()
        cmd = [RUN, dec_p + ".pdmodel", dec_p + ".pdiparams", "--gpu", "0", "--precision", "bf16",
               "--step-input", "time_step", "--repeat", "5", "--output-dir", str(od)] + args
        if mode == "graph":
            cmd.append("--graph")
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr + r.stdout
        assert "released" in r.stdout
        outs[mode] = np.fromfile(str(od / "0.bin"), dtype=np.float32)
        print(mode, [ln for ln in r.stdout.splitlines() if ln.startswith("run_ms")])
    assert np.isfinite(outs["eager"]).all()
    np.testing.assert_allclose(outs["graph"], outs["eager"], rtol=1e-2, atol=1e-2)
