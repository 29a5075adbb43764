"""CPU model of the assembly GEMM's LDS images (`csrc/asm/gemm_gen.py`): the lane-linear LDS-DMA
fill plus the swizzled fragment reads must deliver exactly the MFMA operand fragments, and the
reads must be bank-conflict-free under the gfx950 lane-group rules (MI355X_MICROARCH.md §LDS)."""
import importlib.util
import os

import numpy as np

_P = os.path.join(os.path.dirname(__file__), "..", "paddle_infer_amd", "csrc", "asm", "gemm_gen.py")
_spec = importlib.util.spec_from_file_location("gemm_gen", _P)
gg = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(gg)

B128_GROUPS = [
    list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
    list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
    list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
    list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64)),
]


def _conflicts(addrs, nbytes, groups):
    """Extra LDS cycles: per group, max over banks of distinct addresses touching the bank - 1."""
    worst = 0
    for g in groups:
        banks = {}
        for lane in g:
            a = addrs[lane]
            for d in range(nbytes // 4):
                banks.setdefault(((a + 4 * d) // 4) % 64, set()).add(a)
        worst = max(worst, max(len(s) for s in banks.values()) - 1)
    return worst


def test_kc_image_fragments_and_banks():
    rng = np.random.default_rng(0)
    glob = rng.integers(0, 60000, size=(256, 64), dtype=np.int64)  # [rows][k] of one K-block
    lds = np.full(32768 // 2, -1, dtype=np.int64)
    for i in range(8):
        for w in range(4):
            for L in range(64):
                row, g, off = gg.kc_dma(i, w, L)
                lds[off // 2: off // 2 + 8] = glob[row, 8 * g: 8 * g + 8]
    assert (lds >= 0).all()
    for WO in (0, 128):
        for h in (0, 1):
            for blk in range(8):
                addrs = [gg.kc_read(WO, h, blk, l) for l in range(64)]
                for l in range(64):
                    got = lds[addrs[l] // 2: addrs[l] // 2 + 8]
                    r = WO + 16 * blk + (l & 15)
                    k0 = 32 * h + 8 * (l >> 4)
                    assert (got == glob[r, k0:k0 + 8]).all()
                assert _conflicts(addrs, 16, B128_GROUPS) == 0


def test_mc_image_fragments_and_banks():
    rng = np.random.default_rng(1)
    glob = rng.integers(0, 60000, size=(64, 256), dtype=np.int64)  # [k][cols] of one K-block
    lds = np.full(32768 // 2, -1, dtype=np.int64)
    for i in range(8):
        for w in range(4):
            for L in range(64):
                k, col, off = gg.mc_dma(i, w, L)
                lds[off // 2: off // 2 + 8] = glob[k, col: col + 8]
    assert (lds >= 0).all()
    halves = [list(range(0, 32)), list(range(32, 64))]
    for WO in (0, 128):
        for h in (0, 1):
            for blk in range(8):
                for j in (0, 1):
                    addrs = [gg.mc_read(WO, h, blk, j, l) for l in range(64)]
                    for l in range(64):
                        grp, i = l >> 4, l & 15
                        for q in range(4):
                            src = addrs[16 * grp + 4 * q + (i >> 2)] // 2 + (i & 3)
                            k = 32 * h + 8 * grp + 4 * j + q
                            assert lds[src] == glob[k, WO + 16 * blk + i]
                    assert _conflicts(addrs, 8, halves) == 0


def test_generator_emits_every_variant():
    text = gg.generate()
    for name, *_ in gg.variants():
        assert f"{name}:" in text and f".amdhsa_kernel {name}" in text
    # every store is a vector buffer store
    mnems = {ln.split()[0] for ln in text.splitlines() if ln.strip()}
    stores = {m for m in mnems if "store" in m}
    assert stores <= {"buffer_store_dwordx2", "buffer_store_dwordx4"}, stores


# ---------------------------------------------------------------------------- ping-pong kernel
