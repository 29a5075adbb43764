"""Import of weight-only weights quantized by the reference (CUTLASS sm80 byte order,
`inference/ref_layout.py`). The reference layouts are re-derived here by LITERAL byte-level
transcriptions of the reference routines (`impl/weight_quantize_kernel_gpu_impl.h:25`
weight_permute_kernel_wint8; `cutlass_preprocessors.cu` permute_B_rows_for_mixed_gemm,
subbyte_transpose_impl, interleave_column_major_tensor, add_bias_and_interleave_int4s_inplace) and
compared with the element-level index maps; then reference bytes must give the same
weight_only_linear / static op / fused_multi_transformer_weight_only output as the framework's
own packing of the same quantized values."""
import numpy as np
import pytest
import torch

from paddle_infer_amd.inference import ref_layout as R
from paddle_infer_amd.ops import inference as I


def _lit_int8(q_kn):
    """weight_permute_kernel_wint8, one thread per source element."""
    K, N = q_kn.shape
    src = q_kn.reshape(-1)
    out = np.zeros(K * N, np.uint8)
    for lin in range(K * N):
        k, n = lin // N, lin % N
        km = k % 16
        t1 = km - km // 8 * 8
        t2 = km // 8
        pk = t1 + t2 + (t2 + 1) % 2 * km * 2 // 2 + t1 * t2 + k // 16 * 16
        pidx = pk % 64 + pk // 64 * 128 + 64 * (n % 2) + K * 2 * (n // 2)
        out[pidx] = (int(src[lin]) + 128) & 255
    return out


def _lit_int4(q_kn):
    """symmetric_quantize(PACKED_INT4) → preprocess_weights_for_mixed_gemm on sm80 (uint4 B:
    imma ldsm row permutation, column-major, 64-row tiles × 4 interleaved columns)."""
    K, N = q_kn.shape
    # row-major packing: byte jj of a row = elements 2jj (low nibble), 2jj+1
    rowmaj = np.zeros((K, N // 2), np.uint8)
    for i in range(K):
        for jj in range(N // 2):
            rowmaj[i, jj] = (int(q_kn[i, 2 * jj]) & 0xF) | ((int(q_kn[i, 2 * jj + 1]) & 0xF) << 4)
    # permute_B_rows_for_mixed_gemm (uint32 words: 8 elements = 4 bytes)
    words = rowmaj.view(np.uint32).reshape(K, -1)
    perm = np.empty_like(words)
    for base in range(0, K, 32):
        for tr in range(32):
            read = 8 * ((tr % 8) // 2) + tr % 2 + 2 * (tr // 8)
            perm[base + tr] = words[base + read]
    b = perm.view(np.uint8).reshape(K, N // 2)
    # subbyte_transpose_impl<PACKED_INT4>: 64 x 64-element tiles, nibble swap
    colb, colb_t = N // 2, K // 2
    tr = np.zeros((N, colb_t), np.uint8)
    for r0 in range(0, K, 64):
        for c0 in range(0, colb, 32):
            cache = b[r0:r0 + 64, c0:c0 + 32].copy()
            for ii in range(64):
                for jj in range(ii + 1, 64):
                    ib, io, jb, jo = ii // 2, ii % 2, jj // 2, jj % 2
                    s_e = 0xF & (int(cache[ii, jb]) >> (4 * jo))
                    t_e = 0xF & (int(cache[jj, ib]) >> (4 * io))
                    cache[ii, jb] = (int(cache[ii, jb]) & (0xF0 >> (4 * jo))) | (t_e << (4 * jo))
                    cache[jj, ib] = (int(cache[jj, ib]) & (0xF0 >> (4 * io))) | (s_e << (4 * io))
            tr[c0 * 2:c0 * 2 + 64, r0 // 2:r0 // 2 + 32] = cache
    # interleave_column_major_tensor (uint32 vec rows of the column-major [N][K])
    inw = tr.view(np.uint32).reshape(-1)
    nvr, vpt, il = K // 8, 64 // 8, 4
    outw = np.zeros_like(inw)
    for rc in range(N):
        wc = rc // il
        for bvr in range(0, nvr, vpt):
            for vr in range(bvr, min(nvr, bvr + vpt)):
                wr = il * bvr + vpt * (rc % il) + vr % vpt
                outw[wc * nvr * il + wr] = inw[rc * nvr + vr]
    by = outw.view(np.uint8).copy()
    # add_bias_and_interleave_int4s_inplace
    for i in range(by.size):
        v = np.int8(by[i])
        lo = (np.int8(v << 4) >> 4) + 8
        hi = (v >> 4) + 8
        by[i] = (int(lo) & 0xF) | ((int(hi) & 0xF) << 4)
    regs = by.view(np.uint32)
    res = np.zeros_like(regs)
    for i in range(regs.size):
        cur, t = int(regs[i]), 0
        for d in range(8):
            s = 2 * d if d < 4 else 2 * (d - 4) + 1
            t |= ((cur >> (4 * s)) & 0xF) << (4 * d)
        res[i] = t
    return res.view(np.uint8)


def test_int8_index_map_matches_reference_kernel():
    torch.manual_seed(0)
    w = torch.randn(64, 32)
    wb, sc = R.ref_weight_quantize(w, "weight_only_int8")
    q = R.ref_to_rowmajor(wb, 64, 32, 8).numpy()
    np.testing.assert_array_equal(_lit_int8(q), wb.view(torch.uint8).reshape(-1).numpy())
    torch.testing.assert_close(torch.from_numpy(q).float() * sc, w, atol=float(sc.max()) * 0.51, rtol=0)


def test_int4_index_map_matches_reference_preprocessing():
    torch.manual_seed(1)
    w = torch.randn(128, 64)  # the reference needs K, N multiples of 64 for int4
    wb, sc = R.ref_weight_quantize(w, "weight_only_int4")
    q = R.ref_to_rowmajor(wb, 128, 64, 4).numpy()
    np.testing.assert_array_equal(_lit_int4(q), wb.view(torch.uint8).reshape(-1).numpy())
    assert q.min() >= -8 and q.max() <= 7


@pytest.mark.parametrize("algo,wd", [("weight_only_int8", "int8"), ("weight_only_int4", "int4")])
def test_reference_bytes_give_same_linear_output(algo, wd):
    torch.manual_seed(2)
    K, N = 128, 64
    w = torch.randn(K, N)
    ref_b, sc = R.ref_weight_quantize(w, algo)
    q = R.ref_to_rowmajor(ref_b, K, N, 4 if wd == "int4" else 8)
    ours = I._pack(q.t().contiguous(), 4 if wd == "int4" else 8)  # the same values, MI355X order
    assert R.is_ref_layout(ref_b, 4 if wd == "int4" else 8) and not R.is_ref_layout(ours, 4 if wd == "int4" else 8)
    x = torch.randn(3, K)
    y_ours = I.weight_only_linear(x, ours, None, sc, wd)
    y_imp = I.weight_only_linear(x, R.import_ref_weight(ref_b, sc, algo), None, sc, wd)
    torch.testing.assert_close(y_imp, y_ours)
    torch.testing.assert_close(y_ours, x @ (q.float() * sc), rtol=1e-4, atol=1e-4)
    from paddle_infer_amd.static.ops_registry import REGISTRY
    a = {"weight_dtype": wd, "act_method": "none"}
    o1 = REGISTRY["weight_only_linear"]({"x": [x], "weight": [ref_b], "weight_scale": [sc]}, a)["out"]
    o2 = REGISTRY["weight_only_linear"]({"x": [x], "weight": [ours], "weight_scale": [sc]}, a)["out"]
    torch.testing.assert_close(o1, o2)


def test_fmt_weight_only_reference_bytes():
    from paddle_infer_amd.static.ops_registry import REGISTRY
    torch.manual_seed(3)
    E, H, F_ = 64, 4, 128
    x = torch.randn(2, 5, E)

    def qz(k, n):
        w = torch.randn(k, n) * 0.05
        rb, s = R.ref_weight_quantize(w, "weight_only_int8")
        q = R.ref_to_rowmajor(rb, k, n, 8)
        return rb, I._pack(q.t().contiguous(), 8), s
    qkv, out, f1, f2 = qz(E, 3 * E), qz(E, E), qz(E, F_), qz(F_, E)
    base = {"X": [x], "LnScale": [torch.ones(E)], "LnBias": [torch.zeros(E)], "QKVBias": [torch.zeros(3 * E)],
            "OutLinearBias": [torch.zeros(E)], "FFNLnScale": [torch.ones(E)], "FFNLnBias": [torch.zeros(E)],
            "FFN1Bias": [torch.zeros(F_)], "FFN2Bias": [torch.zeros(E)],
            "QKVWScale": [qkv[2]], "OutLinearWScale": [out[2]], "FFN1WeightScale": [f1[2]],
            "FFN2WeightScale": [f2[2]]}
    a = {"weight_dtype": "int8", "num_heads": H, "pre_layer_norm": True, "epsilon": 1e-5,
         "act_method": "gelu"}
    outs = []
    for i in (0, 1):
        ins = dict(base, QKVW=[qkv[i]], OutLinearW=[out[i]], FFN1Weight=[f1[i]], FFN2Weight=[f2[i]])
        outs.append(REGISTRY["fused_multi_transformer_weight_only"](ins, a)["Out"])
    torch.testing.assert_close(outs[0], outs[1])
