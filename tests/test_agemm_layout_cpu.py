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
pp = gg.pp_module()


def test_pp_image_fragments_and_banks():
    """8-wave kernel: 16-row × 64-B LDS-DMA pieces (8 waves × 2 pieces per operand) and the
    swizzled fragment reads of every wave origin deliver the MFMA fragments, conflict-free."""
    rng = np.random.default_rng(2)
    glob = rng.integers(0, 60000, size=(256, 32), dtype=np.int64)  # [rows][k] of one 32-block
    lds = np.full(16384 // 2, -1, dtype=np.int64)
    for w in range(8):
        for j in range(2):
            for L in range(64):
                row, g, off = pp.q_dma(j, w, L)
                lds[off // 2: off // 2 + 8] = glob[row, 8 * g: 8 * g + 8]
    assert (lds >= 0).all()
    for R0 in (0, 64, 128, 192):
        for blk in range(8 if R0 in (0, 128) else 4):
            addrs = [pp.q_read(R0, blk, l) for l in range(64)]
            for l in range(64):
                got = lds[addrs[l] // 2: addrs[l] // 2 + 8]
                r = R0 + 16 * blk + (l & 15)
                assert (got == glob[r, 8 * (l >> 4): 8 * (l >> 4) + 8]).all()
            assert _conflicts(addrs, 16, B128_GROUPS) == 0


def _check_schedule(streams, nk32, ntiles):
    """Simulate the two wave groups barrier interval by barrier interval: every fragment read sees
    a stage whose DMAs (both groups') were retired by a counted vmcnt before an earlier barrier and
    that nobody re-fills during the read's interval; a stage is re-filled only after both groups'
    reads of its block retired; each group computes blocks 0..nk32-1 of every tile in order (zero-
    initialised at a tile's first block) with its epilogue between tiles."""
    ivs = []
    for ev in streams:
        cur, out = [], []
        for e in ev:
            cur.append(e)
            if e[0] == "bar":
                out.append(cur)
                cur = []
        out.append(cur)
        ivs.append(out)
    assert len(ivs[0]) == len(ivs[1]), "barrier counts differ"
    base = [0, 0]
    nsw = [0, 0]
    queue = [[], []]                 # outstanding VMEM ops: [kind, block, retired_interval]
    content = {}                     # stage -> block (latest DMA issue, any group)
    dma_ops = {}                     # block -> list of op records
    write_iv = {}                    # stage -> list of (interval, block)
    reads = {}                       # block -> list of (group, interval)
    frag = [None, None]
    computed = [[], []]
    since_epi = [0, 0]
    for k in range(len(ivs[0])):
        for g in (0, 1):
            for e in ivs[g][k]:
                kind = e[0]
                if kind == "adv":
                    base[g] += 4
                elif kind == "switch":
                    nsw[g] += 1
                    base[g] = nsw[g] * nk32
                elif kind == "dma":
                    stage, kk = e[1], e[2]
                    b = base[g] + kk
                    assert b % 4 == stage, (g, k, b, stage)
                    old = content.get(stage)
                    if old is not None and old != b:
                        rd = reads.get(old, [])
                        assert len({gg_ for gg_, _ in rd}) == 2 or old >= ntiles * nk32, \
                            f"stage {stage} refilled with {b} before both groups read {old}"
                        assert all(iv < k for _, iv in rd), f"WAR on stage {stage} (block {old})"
                    content[stage] = b
                    rec = ["D", b, None]
                    queue[g].append(rec)
                    dma_ops.setdefault(b, []).append(rec)
                    write_iv.setdefault(stage, []).append((k, b))
                elif kind == "epi":
                    assert since_epi[g] == nk32, (g, since_epi[g])
                    since_epi[g] = 0
                    queue[g] += [["S", None, None] for _ in range(e[1])]
                elif kind == "vmcnt":
                    n = e[1]
                    for rec in queue[g][:max(0, len(queue[g]) - n)]:
                        if rec[2] is None:
                            rec[2] = k
                    queue[g] = queue[g][max(0, len(queue[g]) - n):]
                elif kind == "read":
                    stage = e[1]
                    b = content[stage]
                    ops = dma_ops[b]
                    assert len(ops) == 8, f"block {b}: {len(ops)} DMA ops issued (want 4 per group)"
                    assert all(r[2] is not None and r[2] < k for r in ops), \
                        f"group {g} reads block {b} (stage {stage}) in interval {k} before its DMAs retired"
                    assert not any(iv == k and bb != b for iv, bb in write_iv.get(stage, [])), \
                        f"stage {stage} re-filled during the read interval {k}"
                    reads.setdefault(b, []).append((g, k))
                    frag[g] = b
                elif kind == "compute":
                    b = frag[g]
                    assert b == len(computed[g]), (g, b, len(computed[g]))
                    assert e[1] == (b % nk32 == 0), (g, b, e[1])
                    computed[g].append(b)
                    since_epi[g] += 1
            # the stage a group reads must stay untouched until its lgkmcnt(0) (same interval)
    for g in (0, 1):
        assert computed[g] == list(range(ntiles * nk32)), g
        assert since_epi[g] == 0


def test_pp_schedule_races():
    K = pp.make_kernel_pp(gg.this_module())
    for ek, kw in (("bf16", {}), ("biasgelu", {}), ("f32acc", {}), ("bf16", {"prio": True, "dma_first": True})):
        k = K("x", ek, **kw)
        for nk64, ntiles in ((4, 1), (4, 3), (6, 2), (16, 2)):
            _check_schedule(k.schedule_trace(nk64, ntiles), 2 * nk64, ntiles)


def test_pp_kernels_emitted():
    text = gg.generate()
    for name, ek, f16, _ in pp.variants_pp(gg.this_module()):
        assert f"{name}:" in text and f".amdhsa_kernel {name}" in text
    assert ".amdhsa_accum_offset 128" in text and ".max_flat_workgroup_size: 512" in text
