"""Structural checks of the assembly flash-attention dK/dV generator (csrc/asm/fa_gen.py) on the
CPU: the softmax list-scheduler places every op inside its dependency window, ring slots are
not overwritten while an MFMA may still read them, every LDS address stays inside the 3-buffer
image, the per-lane offset formulas match the HIP kernel's (flash_attn.h `lane_offs`, the
hardware-verified layout) and the text assembles for gfx950."""
import importlib.util
import os
import re
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GEN = os.path.join(HERE, "..", "paddle_infer_amd", "csrc", "asm", "fa_gen.py")


def _gen():
    spec = importlib.util.spec_from_file_location("fa_gen_t", GEN)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_softmax_schedule_windows():
    F = _gen()
    k = F.FaDkdv("t", True)
    ops = k.body_ops(0)
    gap_of = {}
    m = -1
    for e in ops:
        if e[0] == "mfma":
            m = e[1]
        elif e[0] == "txt" and e[1].startswith(("v_mul_f32", "v_exp_f32", "v_cvt_pk_bf16_f32")):
            gap_of[e[1]] = m
    # S' reads after S final (+2 MFMAs), bf16 fragments ≥ 1 MFMA before their first consumer
    for t, g in gap_of.items():
        regs = [int(x) for x in re.findall(r"v(\d+)", t)]
        if any(F.V_SACC <= r < F.V_SACC + 16 for r in regs[1:]) and t.startswith("v_exp"):
            assert g >= 9
        if any(F.V_SACC + 16 <= r < F.V_SACC + 32 for r in regs[1:]) and t.startswith("v_exp"):
            assert g >= 25
        if t.startswith("v_cvt_pk_bf16_f32"):
            d = regs[0]
            ks = ((d - F.V_PB) % 16) // 4
            assert g <= (30 if ks < 2 else 46), (t, g)
    assert sum(1 for t in gap_of if t.startswith("v_exp")) == 32


def test_ring_slots_not_reused_early():
    F = _gen()
    # the read for MFMA m (issued LA MFMAs ahead) lands in the slot of MFMA m - RING
    assert F.RING - F.LA >= 4
    for b in range(3):
        for m in range(64):
            assert F.FaDkdv.slot(b, m) == F.FaDkdv.slot((b + 1) % 3, m - 64) if m >= 64 else True
    # continuity across the 3-tile cycle: 3 tiles = a whole number of ring turns
    assert (3 * 64) % F.RING == 0


def test_lds_offsets_in_range_and_match_hip_layout():
    F = _gen()
    ROWB = 256

    def x(r):
        return ((r & 3) << 2) | ((r >> 2) & 3)

    for lane in range(64):
        l32, hh, gi, g = lane & 31, lane >> 5, lane & 15, lane >> 4
        # row reads (flash_attn.h lane_offs: row[kk] = l32*ROWB + ((2kk + hh) ^ x(l32)) << 4)
        for kk in range(8):
            row = l32 * ROWB + (((2 * kk + hh) ^ x(l32)) << 4)
            for b in range(3):
                s, imm = F.buf_set(b)
                base = row + (2 * F.BUF_B if s else 0)
                for off in (imm, imm + F.OFF_DO + 8192):
                    assert 0 <= base + off and base + off + 16 <= F.LDS_BYTES
                    assert (base + off) // F.BUF_B == b or b == 2
        # transposed reads: tr[jj][dt] = tr[jj][0] ^ (dt << 6)
        for jj in (0, 1):
            rl = 4 * hh + 8 * jj + (gi >> 2)
            for dt in range(4):
                col = 32 * dt + 16 * (g & 1) + 4 * (gi & 3)
                tr = rl * ROWB + (((col >> 3) ^ x(rl)) << 4) + ((col & 7) << 1)
                col0 = 16 * (g & 1) + 4 * (gi & 3)
                tr0 = rl * ROWB + (((col0 >> 3) ^ x(rl)) << 4) + ((col0 & 7) << 1)
                assert tr == tr0 ^ (dt << 6)
                assert tr + 2 * F.BUF_B + F.OFF_DO + 3 * 16 * ROWB + 8 <= F.LDS_BYTES
    # DMA pieces: every (row, logical chunk) of a 64 × 256-B tile written exactly once
    seen = set()
    for w in range(4):
        for i in range(4):
            for lane in range(64):
                r = 16 * w + 4 * i + (lane >> 4)
                lc = (lane & 15) ^ ((((lane >> 4)) << 2) | i)
                assert lc == (lane & 15) ^ x(r)
                phys = (4 * w + i) * 1024 + 16 * lane
                assert phys == r * ROWB + 16 * (lane & 15)
                seen.add((r, lc))
    assert len(seen) == 64 * 16


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/clang"), reason="no ROCm LLVM")
def test_assembles(tmp_path):
    F = _gen()
    src = tmp_path / "fa.s"
    src.write_text(F.generate())
    txt = src.read_text()
    assert txt.count("v_mfma_f32_32x32x16_bf16") == 2 * 3 * 64 + 2 * 3 * 48 + 2 * 2 * 2 * 32  # dK/dV, dQ, fwd (4- and 8-wave)
    r = subprocess.run(["/opt/rocm/lib/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                        "-mcpu=gfx950", "-c", str(src), "-o", str(tmp_path / "fa.o")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
