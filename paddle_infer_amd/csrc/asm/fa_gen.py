"""Generator of the hand-scheduled gfx950 flash-attention backward dK/dV kernel (``fa_dkdv``).

Why assembly: the HIP `bwd_dkdv_kernel` (csrc/kernels/flash_attn.h) runs ONE wave per SIMD and
spends ≈7.5k cycles per 64-query tile for 64 MFMAs (2,048 cycles of matrix work): the softmax
VALU work, LDS waits and barriers sit BETWEEN the MFMA phases instead of under them, and hipcc
does not keep a requested interleave (profiles/fa_bwd_experiments_r3.txt). At one wave per SIMD
an MFMA gap (32 cycles for v_mfma_f32_32x32x16_bf16) hides ≈24 cycles of other issue
(MI355X_MICROARCH.md constants table), so every LDS read, every softmax op, every LDS-DMA and
the barrier is placed here by hand into the MFMA stream.

Math (same as the HIP kernel, reference `paddle/phi/kernels/gpu/flash_attn_grad_kernel.cu`):
workgroup = 128 keys of one (batch, kv-head), 4 waves × 32 keys (key on the MFMA lane). For
every 64-query tile of every q-head of the GQA group (causal: tiles from the diagonal on):
  Sᵀ' = K·Qᵀ − lse/scale,  dPᵀ' = V·dOᵀ − δ          (accumulators start at the row constants)
  P = exp2(c·S'),  dS = P ∘ dP'                        (c = scale·log2 e)
  dVᵀ += dOᵀ·P,   dKᵀ += Qᵀ·dS                         (dK scaled by `scale` at the end)
K and V fragments of the wave's keys live in AGPRs for the whole sweep (MFMA B operands may be
AGPRs), dKᵀ/dVᵀ in AGPRs; S/dP accumulators in VGPRs for the softmax.

Schedule of one tile (64 MFMAs: A0 = S,dP of queries 0-31, A1 = queries 32-63, C0 = dV/dK with
keys' query-k 0-31, C1 = 32-63):
* every MFMA operand read from LDS is issued LA MFMAs ahead into a 12-slot register ring
  (ds_read_b128 row fragments for A, ds_read_b64_tr_b16 transposed pairs for C); the last LA
  reads of a tile fetch the NEXT tile's first fragments;
* the softmax (16 exp + 48 other VALU per 32 queries) is list-scheduled into the A1 / C0 MFMA
  gaps within its dependency window (S final → P → dS → bf16 fragments before their C MFMA);
* Q/dO tiles + the (−lse/scale, −δ) rows arrive by LDS-DMA in a 3-buffer ring; ONE barrier per
  tile (after C0) publishes tile t+1 and frees the buffer of tile t−1, whose DMA for tile t+2
  is then issued half in C1, half in the next tile's A0;
* diagonal (causal) tiles initialise the masked S' entries to −inf (one branch per tile).

Restrictions of this kernel (the launcher falls back to the HIP kernel otherwise): bf16, D = 128,
no dropout / additive mask / varlen, Sq == Sk, Sq % 256 == 0 (key blocks pair up), tensors < 2 GiB.

``python fa_gen.py OUT.s`` writes the kernels; `_build.py` assembles them into
``_lib/piamd_fa.hsaco`` (loaded by ``csrc/kernels/fa_asm_host.hip``).
"""
from __future__ import annotations

import os
import sys

# ---- kernel arguments (byte offsets; mirrored by struct FaDkdvArgs in fa_asm_host.hip) ----------
ARGS = [
    ("q", 0, 8), ("k", 8, 8), ("v", 16, 8), ("dout", 24, 8), ("dk", 32, 8), ("dv", 40, 8),
    ("nl", 48, 8), ("nd", 56, 8),
    ("q_bytes", 64, 4), ("k_bytes", 68, 4), ("v_bytes", 72, 4), ("o_bytes", 76, 4), ("st_bytes", 80, 4),
    ("sqs", 84, 4), ("sqh", 88, 4), ("sqb", 92, 4),
    ("sks", 96, 4), ("skh", 100, 4), ("skb", 104, 4),
    ("svs", 108, 4), ("svh", 112, 4), ("svb", 116, 4),
    ("sos", 120, 4), ("soh", 124, 4), ("sob", 128, 4),
    ("Hq", 132, 4), ("Hk", 136, 4), ("group", 140, 4), ("Sq", 144, 4), ("coff", 148, 4),
    ("nqt", 152, 4), ("npair", 156, 4), ("nkb1", 160, 4), ("c", 164, 4), ("scale", 168, 4),
    ("rcp_npair", 172, 4), ("rcp_Hk", 176, 4), ("nitems", 180, 4), ("G", 184, 4), ("G2m1", 188, 4),
]
ARGS_SIZE = 192


def sarg(name):
    """SGPR holding argument `name` (the 192 argument bytes are loaded to s[4:51])."""
    for n, off, _ in ARGS:
        if n == name:
            return 4 + off // 4
    raise KeyError(name)


# ---- SGPR map ----------------------------------------------------------------------------------
S_WG = 2
# s4..s19 hold the 8 argument pointers until the descriptors are built, then:
S_QB, S_OB, S_STB, S_W, S_LDSW, S_LDSST = 4, 5, 6, 7, 8, 9
S_T = 10                                                  # temps s10..s17
SRD_Q, SRD_O, SRD_K, SRD_V, SRD_ST, SRD_DK, SRD_DV = 52, 56, 60, 64, 68, 72, 76   # descriptors
# compute side: the work item whose tiles the MFMAs run
S_U, S_B, S_HK, S_N0, S_QF, S_TOT, S_IT, S_CQ0, S_KW31, S_SOFFK, S_SOFFV = range(80, 91)
# DMA side: the item / tile the LDS-DMA stream is fetching (runs 1.5 tiles ahead, across items)
S_DU, S_DQF, S_DTOT, S_DIT, S_DQ0, S_DHQ, S_SQ, S_SO, S_SST = range(91, 100)
NSGPR = 101

# ---- VGPR / AGPR map -----------------------------------------------------------------------------
V_TID, V_LANE = 0, 1
V_DQ, V_DO, V_DST = 2, 6, 10       # LDS-DMA lane offsets: Q pieces 0-3, dO pieces 0-3, stats
V_ROW = 11                         # [set 2][kk 8] row-fragment read offsets
V_TR = 27                          # [set 2][jj 2][dt 4] transposed-read offsets
V_STB = 43                         # [set 2] stats read offsets
V_KT, V_THR, V_NINF = 45, 46, 47   # key − coff − 4hh, per-tile threshold, −inf
V_RING = 48                        # 12 slots × 4
RING = 12
V_SACC, V_PACC = 96, 128           # S' / dP' accumulators: [qt 2][16]
V_PB, V_DB = 160, 176              # bf16 fragments of P / dS: [ks 4][4]
V_TMP = 192                        # temps v192..v199
V_KT0, V_KVK, V_KVV = 200, 201, 202  # 32w + l32 − coff − 4hh; K / V fragment-load lane offsets
V_STK, V_STV = 203, 204            # dK / dV store lane offsets
NV = 208                           # accum_offset
# AGPRs: dVᵀ [dt][16], dKᵀ, K / V fragments [kk][4] of the current item, and of the next item
# (prefetched during the current one)
A_DV, A_DK, A_KF, A_VF, A_KN, A_VN = 0, 64, 128, 160, 192, 224
NA = 256

LA = 6                             # ring-read lookahead (MFMAs)
BUF_B = 33280                      # per buffer: Q 16 KiB, dO 16 KiB, (−lse/scale, −δ) 2 × 256 B
OFF_DO, OFF_ST = 16384, 32768
LDS_BYTES = 3 * BUF_B
MFMA = "v_mfma_f32_32x32x16_bf16"
# ablation builds for measurement only (numerically wrong): nodma / nobar / novmwait / novalu /
# noreads / nomfma drop that part of the tile loop
ABL = set(filter(None, os.environ.get("PIAMD_FA_ABL", "").split(",")))
# timestamp build (measurement only): s_memtime at 6 points of every tile, written over dV
# ([wg][wave][tile < 256][8] u64; the dV output itself is not written) — tools/fa_stamps.py
STAMP = os.environ.get("PIAMD_FA_STAMP", "0") == "1"


def fhex(x):
    import struct
    return "0x%08x" % struct.unpack("<I", struct.pack("<f", x))[0]


def buf_set(b):
    """(offset-register set, immediate base) of LDS buffer b: buffers 0/1 share set 0 (the 16-bit
    ds offset reaches buffer 1), buffer 2 has its own set based at 2·BUF_B."""
    return (0, 0) if b == 0 else (0, BUF_B) if b == 1 else (1, 0)


class FaDkdv:
    VTMP_UDIV = V_TMP

    def __init__(self, name, causal):
        self.name, self.causal = name, causal
        self.lines = []
        self.nlab = 0

    def e(self, s):
        if ABL and getattr(self, "in_loop", False):
            m = s.split(" ", 1)[0]
            if (("nodma" in ABL and m.startswith("buffer_load") and s.endswith(" lds"))
                    or ("nobar" in ABL and m == "s_barrier")
                    or ("novmwait" in ABL and (m == "s_barrier" or s.startswith("s_waitcnt vmcnt")))
                    or ("noreads" in ABL and (m.startswith("ds_read") or s.startswith("s_waitcnt lgkmcnt")))):
                return
            if "nomfma" in ABL and m.startswith("v_mfma"):
                s = "s_nop 0"
        self.lines.append("\t" + s)

    def lab(self, s):
        self.lines.append(s + ":")

    def newlab(self, tag):
        self.nlab += 1
        return f".L{self.name}_{tag}_{self.nlab}"

    # -- helpers --------------------------------------------------------------------------------
    def udiv(self, q, r, n, d, rcp):
        """q = n / d, r = n % d (SGPRs, n < 2^24) from the f32 reciprocal in SGPR rcp, ±1 fixed."""
        v = self.VTMP_UDIV
        self.e(f"v_cvt_f32_u32 v{v}, s{n}")
        self.e(f"v_mul_f32 v{v}, s{rcp}, v{v}")
        self.e(f"v_cvt_u32_f32 v{v}, v{v}")
        self.e("s_nop 1")
        self.e(f"v_readfirstlane_b32 s{q}, v{v}")
        self.e("s_nop 1")
        t = S_T + 5
        self.e(f"s_mul_i32 s{t}, s{q}, s{d}")
        self.e(f"s_sub_i32 s{r}, s{n}, s{t}")
        l1, l2 = self.newlab("dv"), self.newlab("dv")
        self.e(f"s_cmp_lt_i32 s{r}, 0")
        self.e(f"s_cbranch_scc0 {l1}")
        self.e(f"s_sub_u32 s{q}, s{q}, 1")
        self.e(f"s_add_u32 s{r}, s{r}, s{d}")
        self.lab(l1)
        self.e(f"s_cmp_ge_u32 s{r}, s{d}")
        self.e(f"s_cbranch_scc0 {l2}")
        self.e(f"s_add_u32 s{q}, s{q}, 1")
        self.e(f"s_sub_u32 s{r}, s{r}, s{d}")
        self.lab(l2)

    def srd(self, srd, ptr, nbytes):
        self.e(f"s_mov_b32 s{srd}, s{ptr}")
        self.e(f"s_and_b32 s{srd + 1}, s{ptr + 1}, 0xffff")
        self.e(f"s_mov_b32 s{srd + 2}, s{nbytes}")
        self.e(f"s_mov_b32 s{srd + 3}, 0x20000")

    def pending_soffs(self):
        """Q / dO / stats soffsets of the pending DMA tile (S_DHQ, S_DQ0); past the last tile the
        soffsets point past the descriptor ranges (the DMA then moves nothing from memory)."""
        T = S_T
        self.e(f"s_mul_i32 s{T}, s{S_DHQ}, s{sarg('sqh')}")
        self.e(f"s_mul_i32 s{T + 1}, s{S_DQ0}, s{sarg('sqs')}")
        self.e(f"s_add_u32 s{T}, s{T}, s{T + 1}")
        self.e(f"s_add_u32 s{S_SQ}, s{T}, s{S_QB}")
        self.e(f"s_mul_i32 s{T}, s{S_DHQ}, s{sarg('soh')}")
        self.e(f"s_mul_i32 s{T + 1}, s{S_DQ0}, s{sarg('sos')}")
        self.e(f"s_add_u32 s{T}, s{T}, s{T + 1}")
        self.e(f"s_add_u32 s{S_SO}, s{T}, s{S_OB}")
        self.e(f"s_mul_i32 s{T}, s{S_DHQ}, s{sarg('Sq')}")
        self.e(f"s_add_u32 s{T}, s{T}, s{S_DQ0}")
        self.e(f"s_lshl_b32 s{T}, s{T}, 2")
        self.e(f"s_add_u32 s{S_SST}, s{T}, s{S_STB}")
        self.e(f"s_cmp_ge_u32 s{S_DU}, s{sarg('nitems')}")
        self.e(f"s_cselect_b32 s{S_SQ}, s{sarg('q_bytes')}, s{S_SQ}")
        self.e(f"s_cselect_b32 s{S_SO}, s{sarg('o_bytes')}, s{S_SO}")
        self.e(f"s_cselect_b32 s{S_SST}, s{sarg('st_bytes')}, s{S_SST}")

    def advance_pending(self):
        """Next tile of the DMA stream: next query tile, next q-head of the group, or the first
        tile of the workgroup's next work item."""
        self.e(f"s_add_u32 s{S_DIT}, s{S_DIT}, 1")
        self.e(f"s_add_u32 s{S_DQ0}, s{S_DQ0}, 64")
        self.e(f"s_cmp_ge_u32 s{S_DQ0}, s{sarg('Sq')}")
        self.e(f"s_cselect_b32 s{S_DQ0}, s{S_DQF}, s{S_DQ0}")
        self.e(f"s_addc_u32 s{S_DHQ}, s{S_DHQ}, 0")       # SCC still holds the wrap
        same = self.newlab("sameitem")
        self.e(f"s_cmp_lt_u32 s{S_DIT}, s{S_DTOT}")
        self.e(f"s_cbranch_scc1 {same}")
        self.next_item(S_DU)
        self.e(f"s_cmp_ge_u32 s{S_DU}, s{sarg('nitems')}")
        self.e(f"s_cbranch_scc1 {same}")
        self.pending_item_setup()
        self.lab(same)
        self.pending_soffs()

    # -- work items -------------------------------------------------------------------------------
    def decode(self, u, kb, b, hk):
        """Work item u → key block kb, batch b, kv-head hk (SGPRs; kb may be a temp).
        u = 2·m + s: member m = group·npair + j of a (batch, kv-head) group takes key blocks j
        (s = 0) and nkb−1−j (s = 1) — equal causal work per member (16 + 2 = 14 + 4 = … tiles) —
        and the npair members of a group sit on one XCD at once (see next_item), so the group's
        Q / dO tiles come from that XCD's L2 after the first member fetched them."""
        T = S_T
        self.e(f"s_lshr_b32 s{T + 7}, s{u}, 1")
        self.udiv(T + 6, kb, T + 7, sarg("npair"), sarg("rcp_npair"))     # group, j
        self.e(f"s_sub_u32 s{T + 7}, s{sarg('nkb1')}, s{kb}")
        self.e(f"s_bitcmp1_b32 s{u}, 0")
        self.e(f"s_cselect_b32 s{kb}, s{T + 7}, s{kb}")
        self.udiv(b, hk, T + 6, sarg("Hk"), sarg("rcp_Hk"))

    def next_item(self, u):
        """The workgroup's next item: the second key block of its pair, or its pair in the next
        round (u += 2G − 1)."""
        T = S_T
        self.e(f"s_bitcmp1_b32 s{u}, 0")
        self.e(f"s_cselect_b32 s{T + 7}, s{sarg('G2m1')}, 1")
        self.e(f"s_add_u32 s{u}, s{u}, s{T + 7}")

    def q_first(self, dst, n0):
        self.e(f"s_mov_b32 s{dst}, 0")
        if self.causal:
            self.e(f"s_sub_i32 s{dst}, s{n0}, s{sarg('coff')}")
            self.e(f"s_max_i32 s{dst}, s{dst}, 0")
            self.e(f"s_and_b32 s{dst}, s{dst}, 0xffffffc0")

    def tiles_of(self, dst, qf):
        self.e(f"s_lshr_b32 s{dst}, s{qf}, 6")
        self.e(f"s_sub_u32 s{dst}, s{sarg('nqt')}, s{dst}")
        self.e(f"s_mul_i32 s{dst}, s{dst}, s{sarg('group')}")

    def kv_soffs(self, b, hk, n0, dk, dv):
        T = S_T
        for soff, sb, sh, ss in ((dk, "skb", "skh", "sks"), (dv, "svb", "svh", "svs")):
            self.e(f"s_mul_i32 s{soff}, s{b}, s{sarg(sb)}")
            self.e(f"s_mul_i32 s{T + 7}, s{hk}, s{sarg(sh)}")
            self.e(f"s_add_u32 s{soff}, s{soff}, s{T + 7}")
            self.e(f"s_mul_i32 s{T + 7}, s{n0}, s{sarg(ss)}")
            self.e(f"s_add_u32 s{soff}, s{soff}, s{T + 7}")

    def compute_item_setup(self):
        """Compute-side state of item S_U: batch / head / key block, tile count, K/V/dK/dV
        soffsets, causal thresholds."""
        T = S_T
        self.decode(S_U, T, S_B, S_HK)
        self.e(f"s_lshl_b32 s{S_N0}, s{T}, 7")
        self.q_first(S_QF, S_N0)
        self.tiles_of(S_TOT, S_QF)
        self.e(f"s_mov_b32 s{S_IT}, 0")
        self.e(f"s_mov_b32 s{S_CQ0}, s{S_QF}")
        self.kv_soffs(S_B, S_HK, S_N0, S_SOFFK, S_SOFFV)
        self.e(f"s_lshl_b32 s{S_KW31}, s{S_W}, 5")
        self.e(f"s_add_u32 s{S_KW31}, s{S_KW31}, s{S_N0}")
        self.e(f"s_add_u32 s{S_KW31}, s{S_KW31}, 31")
        self.e(f"v_add_u32 v{V_KT}, s{S_N0}, v{V_KT0}")

    def pending_item_setup(self):
        """DMA-side state of item S_DU (its first tile)."""
        T = S_T
        self.decode(S_DU, T, T + 1, T + 2)
        self.e(f"s_lshl_b32 s{T}, s{T}, 7")
        self.q_first(S_DQF, T)
        self.tiles_of(S_DTOT, S_DQF)
        self.e(f"s_mov_b32 s{S_DIT}, 0")
        self.e(f"s_mov_b32 s{S_DQ0}, s{S_DQF}")
        self.e(f"s_mul_i32 s{S_DHQ}, s{T + 2}, s{sarg('group')}")
        self.e(f"s_mul_i32 s{S_QB}, s{T + 1}, s{sarg('sqb')}")
        self.e(f"s_mul_i32 s{S_OB}, s{T + 1}, s{sarg('sob')}")
        self.e(f"s_mul_i32 s{S_STB}, s{T + 1}, s{sarg('Hq')}")
        self.e(f"s_mul_i32 s{S_STB}, s{S_STB}, s{sarg('Sq')}")
        self.e(f"s_lshl_b32 s{S_STB}, s{S_STB}, 2")

    def kv_load(self, ak, av, soffk, soffv):
        """The lane's K / V fragments (8 × 16 B each at dims 16kk + 8hh of its key row) straight
        into AGPRs."""
        for kk in range(8):
            self.e(f"buffer_load_dwordx4 a[{ak + 4 * kk}:{ak + 4 * kk + 3}], v{V_KVK}, s[{SRD_K}:{SRD_K + 3}], s{soffk} offen offset:{32 * kk}")
        for kk in range(8):
            self.e(f"buffer_load_dwordx4 a[{av + 4 * kk}:{av + 4 * kk + 3}], v{V_KVV}, s[{SRD_V}:{SRD_V + 3}], s{soffv} offen offset:{32 * kk}")

    def prefetch_next_kv(self):
        """After the first tile of an item: the next item's K / V into the spare AGPR set (the
        next tile barrier's vmcnt(0) lands them long before the item switch)."""
        T = S_T
        skip = self.newlab("nopf")
        self.e(f"s_mov_b32 s{T + 3}, s{S_U}")
        self.next_item(T + 3)
        self.e(f"s_cmp_ge_u32 s{T + 3}, s{sarg('nitems')}")
        self.e(f"s_cbranch_scc1 {skip}")
        self.decode(T + 3, T, T + 1, T + 2)
        self.e(f"s_lshl_b32 s{T}, s{T}, 7")
        self.kv_soffs(T + 1, T + 2, T, T + 3, T + 4)
        self.kv_load(A_KN, A_VN, T + 3, T + 4)
        self.lab(skip)

    def item_end(self, lab_next, lab_exit):
        """After an item's last tile: dK / dV out, accumulators zeroed, the prefetched K / V become
        current, next item's compute state (its first tile is already in LDS / in flight)."""
        self.e("s_nop 15")
        self.e("s_nop 15")
        self.store_dkdv()
        for i in range(128):
            self.e(f"v_accvgpr_write_b32 a{i}, 0")
        for i in range(64):
            self.e(f"v_accvgpr_mov_b32 a{A_KF + i}, a{A_KN + i}")
        self.next_item(S_U)
        self.e(f"s_cmp_ge_u32 s{S_U}, s{sarg('nitems')}")
        self.e(f"s_cbranch_scc1 {lab_exit}")
        self.compute_item_setup()
        self.e("s_nop 4")
        self.e(f"s_branch {lab_next}")

    def store_dkdv(self):
        """dK = scale · dKᵀ, dV = dVᵀ in bf16; lane = key, 4 consecutive dims d0 = 32dt + 8g4 +
        4hh per 8-byte store (fire and forget: nothing waits for them)."""
        t = V_TMP
        for dt in range(4):
            for g4 in range(4):
                for which in ((0,) if STAMP else (0, 1)):
                    a0 = (A_DK if which == 0 else A_DV) + 16 * dt + 4 * g4
                    for j in range(4):
                        self.e(f"v_accvgpr_read_b32 v{t + 4 + j}, a{a0 + j}")
                    if which == 0:
                        for j in range(4):
                            self.e(f"v_mul_f32 v{t + 4 + j}, s{sarg('scale')}, v{t + 4 + j}")
                    self.e(f"v_cvt_pk_bf16_f32 v{t + 4}, v{t + 4}, v{t + 5}")
                    self.e(f"v_cvt_pk_bf16_f32 v{t + 5}, v{t + 6}, v{t + 7}")
                    srd, vo, so = (SRD_DK, V_STK, S_SOFFK) if which == 0 else (SRD_DV, V_STV, S_SOFFV)
                    self.e(f"buffer_store_dwordx2 v[{t + 4}:{t + 5}], v{vo}, s[{srd}:{srd + 3}], s{so} offen offset:{64 * dt + 16 * g4}")

    def dma_first(self, buf):
        """Q pieces + the stats row of the pending tile → LDS buffer `buf` (list of line pairs)."""
        base = buf * BUF_B
        ops = []
        for i in range(4):
            ops.append([f"s_add_u32 m0, s{S_LDSW}, {base + i * 1024}\n\ts_nop 0",
                        f"buffer_load_dwordx4 v{V_DQ + i}, s[{SRD_Q}:{SRD_Q + 3}], s{S_SQ} offen lds"])
        ops.append([f"s_add_u32 m0, s{S_LDSST}, {base + OFF_ST}\n\ts_nop 0",
                    f"buffer_load_dword v{V_DST}, s[{SRD_ST}:{SRD_ST + 3}], s{S_SST} offen lds"])
        return ops

    def dma_second(self, buf):
        base = buf * BUF_B + OFF_DO
        return [[f"s_add_u32 m0, s{S_LDSW}, {base + i * 1024}\n\ts_nop 0",
                 f"buffer_load_dwordx4 v{V_DO + i}, s[{SRD_O}:{SRD_O + 3}], s{S_SO} offen lds"]
                for i in range(4)]

    # -- MFMA stream ------------------------------------------------------------------------------
    @staticmethod
    def mfma_kind(m):
        """MFMA m of a tile → ('S'|'P', qt, kk) or ('V'|'K', dt, ks)."""
        if m < 32:
            qt, r = m // 16, m % 16
            return ("S" if r < 8 else "P", qt, r % 8)
        c = m - 32
        half, cc = c // 16, c % 16
        dt, ks = cc // 4, 2 * half + (cc % 4) // 2
        return ("K" if cc % 2 else "V", dt, ks)

    @staticmethod
    def slot(b, m):
        return V_RING + 4 * ((64 * b + m) % RING)

    def ring_reads(self, b, m):
        """LDS reads of MFMA m's ring operand (tile in buffer b) → list of texts."""
        kind, x, y = self.mfma_kind(m)
        s, imm = buf_set(b)
        d = self.slot(b, m)
        if kind in ("S", "P"):
            qt, kk = x, y
            off = imm + (OFF_DO if kind == "P" else 0) + qt * 8192
            return [f"ds_read_b128 v[{d}:{d + 3}], v{V_ROW + 8 * s + kk} offset:{off}"]
        dt, ks = x, y
        off = imm + (0 if kind == "K" else OFF_DO) + ks * 16 * 256
        return [f"ds_read_b64_tr_b16 v[{d + 2 * jj}:{d + 2 * jj + 1}], v{V_TR + 8 * s + 4 * jj + dt} offset:{off}"
                for jj in (0, 1)]

    def stats_reads(self, b):
        """(−lse/scale → S', −δ → dP') row constants of the tile in buffer b: 16 ds_read_b128,
        ordered qt 0 first (the first MFMAs need them)."""
        s, imm = buf_set(b)
        out = []
        for qt in (0, 1):
            for g4 in range(4):
                for which, dst in ((0, V_SACC), (1, V_PACC)):
                    d = dst + 16 * qt + 4 * g4
                    off = imm + which * 256 + 128 * qt + 32 * g4
                    out.append(((qt, which), f"ds_read_b128 v[{d}:{d + 3}], v{V_STB + s} offset:{off}"))
        return out

    def mfma_text(self, b, m):
        kind, x, y = self.mfma_kind(m)
        a = self.slot(b, m)
        if kind in ("S", "P"):
            qt, kk = x, y
            acc = (V_SACC if kind == "S" else V_PACC) + 16 * qt
            bop = (A_KF if kind == "S" else A_VF) + 4 * kk
            return f"{MFMA} v[{acc}:{acc + 15}], v[{a}:{a + 3}], a[{bop}:{bop + 3}], v[{acc}:{acc + 15}]"
        dt, ks = x, y
        acc = (A_DK if kind == "K" else A_DV) + 16 * dt
        bop = (V_DB if kind == "K" else V_PB) + 4 * ks
        return f"{MFMA} a[{acc}:{acc + 15}], v[{a}:{a + 3}], v[{bop}:{bop + 3}], a[{acc}:{acc + 15}]"

    # -- softmax work queues ------------------------------------------------------------------------
    def finish_queues(self):
        """Four FIFO queues of (text, cost, pair) — S-part (scale, exp2) and D-part (dS, bf16
        packs) per 32-query half — with their [earliest, deadline] gap windows."""
        qs = []
        for qt in (0, 1):
            sq, dq = [], []
            for j in range(8):
                s0, s1 = V_SACC + 16 * qt + 2 * j, V_SACC + 16 * qt + 2 * j + 1
                d0, d1 = V_PACC + 16 * qt + 2 * j, V_PACC + 16 * qt + 2 * j + 1
                sq += [(f"v_mul_f32 v{s0}, s{sarg('c')}, v{s0}", 4, j),
                       (f"v_mul_f32 v{s1}, s{sarg('c')}, v{s1}", 4, j),
                       (f"v_exp_f32 v{s0}, v{s0}", 8, j),
                       (f"v_exp_f32 v{s1}, v{s1}", 8, j)]
                fr = 4 * (2 * qt + j // 4) + j % 4
                dq += [(f"v_mul_f32 v{d0}, v{s0}, v{d0}", 4, j),
                       (f"v_mul_f32 v{d1}, v{s1}, v{d1}", 4, j),
                       (f"v_cvt_pk_bf16_f32 v{V_PB + fr}, v{s0}, v{s1}", 4, j),
                       (f"v_cvt_pk_bf16_f32 v{V_DB + fr}, v{d0}, v{d1}", 4, j)]
            # windows: S' final after MFMA 16qt+7, dP' after 16qt+15 (+2 MFMAs before a VALU read);
            # bf16 fragments ≥ 1 MFMA before their first consumer (m = 32 / 48)
            s_lo, d_lo, dl = 16 * qt + 9, 16 * qt + 17, 30 + 16 * qt
            qs.append(dict(name=f"S{qt}", ops=sq, lo=s_lo, hi=dl - 2, placed=set()))
            qs.append(dict(name=f"D{qt}", ops=dq, lo=d_lo, hi=dl, placed=set(), dep=len(qs) - 1))
        return qs

    def schedule_valu(self, fixed_cost):
        """List-schedule the four softmax queues into gaps 0..63 under a per-gap issue budget of
        24 cycles (minus the gap's fixed LDS/DMA cost); a queue that would miss its deadline is
        forced. D-part pair j goes only after its S-part pair j (exp) sits in an earlier gap."""
        qs = self.finish_queues()
        gaps = [[] for _ in range(len(fixed_cost))]
        heads = [0] * len(qs)
        s_done_gap = [dict() for _ in qs]       # queue → pair → gap of its last op
        for g in range(len(fixed_cost)):
            budget = 24 - fixed_cost[g]
            while True:
                cand = []
                for qi, q in enumerate(qs):
                    if heads[qi] >= len(q["ops"]) or g < q["lo"]:
                        continue
                    text, cost, pair = q["ops"][heads[qi]]
                    if "dep" in q:
                        sg = s_done_gap[q["dep"]]
                        if pair not in sg or sg[pair] >= g or self._pair_incomplete(qs[q["dep"]], heads[q["dep"]], pair):
                            continue
                    left = len(q["ops"]) - heads[qi]
                    slack = (q["hi"] - g + 1) * 5 - left   # ≈5 single-issue fillers per gap
                    cand.append((slack, qi, cost))
                if not cand:
                    break
                cand.sort()
                slack, qi, cost = cand[0]
                if cost > budget and slack > 0:
                    break
                text, cost, pair = qs[qi]["ops"][heads[qi]]
                gaps[g].append(text)
                heads[qi] += 1
                s_done_gap[qi][pair] = g
                budget -= cost
        for qi, q in enumerate(qs):
            assert heads[qi] == len(q["ops"]), f"softmax queue {q['name']} not placed"
        return gaps

    @staticmethod
    def _pair_incomplete(q, head, pair):
        return any(p == pair for _, _, p in q["ops"][head:])

    # -- one tile body ------------------------------------------------------------------------------
    def body_ops(self, b):
        """The instruction stream of a tile in buffer b as a list of entries:
        ('lds', key, text) / ('mfma', m, deps) / ('txt', text). LDS keys: ('ring', tile, m) and
        ('stat', tile, (qt, which)) with tile 0 = this tile, 1 = the next one."""
        nb = (b + 1) % 3
        gaps = [[] for _ in range(64)]
        fixed = [0] * 64
        # ring reads, LA ahead; the last LA gaps fetch the next tile's first operands
        for m in range(64):
            g = m - LA
            if g >= 0:
                for t in self.ring_reads(b, m):
                    gaps[g].append(("lds", ("ring", 0, m), t))
                    fixed[g] += 2
        for m in range(LA):
            g = 64 - LA + m
            for t in self.ring_reads(nb, m):
                gaps[g].append(("lds", ("ring", 1, m), t))
                fixed[g] += 2
        # second half of the pending tile's DMA (→ buffer b+1) in A0, then advance the cursor
        for i, (m0, ld) in enumerate(self.dma_second(nb)):
            g = 1 + 3 * i
            gaps[g] += [("txt", m0), ("txt", ld)]
            fixed[g] += 12
        gaps[13].append(("adv",))
        fixed[13] += 8
        # barrier after C0: tile t+1 landed (its DMA was issued one tile ago), buffer t−1 free
        if STAMP:
            gaps[15].append(("stamp", 1))
            gaps[31].append(("stamp", 2))
            gaps[47].append(("stamp", 3))
        gaps[47].append(("txt", "s_waitcnt vmcnt(0)"))
        gaps[47].append(("txt", "s_barrier"))
        if STAMP:
            gaps[47].append(("stamp", 4))
        fixed[47] += 8
        # next tile's row constants (after the softmax of this tile consumed S'/dP')
        for i, (key, t) in enumerate(self.stats_reads(nb)):
            g = 47 + i // 2
            gaps[g].append(("lds", ("stat", 1, key), t))
            fixed[g] += 2
        # first half of the DMA of tile t+2 (→ buffer b+2)
        for i, (m0, ld) in enumerate(self.dma_first((b + 2) % 3)):
            g = 49 + 3 * i
            gaps[g] += [("txt", m0), ("txt", ld)]
            fixed[g] += 12
        valu = self.schedule_valu(fixed)
        if "novalu" in ABL:  # measurement only: no softmax work (control flow untouched)
            valu = [[] for _ in range(64)]
        ops = []
        for m in range(64):
            kind, x, y = self.mfma_kind(m)
            deps = [("ring", 0, m)]
            if kind in ("S", "P") and y == 0:
                deps.append(("stat", 0, (x, 0 if kind == "S" else 1)))
            ops.append(("mfma", m, deps, self.mfma_text(b, m)))
            ops += gaps[m]
            ops += [("txt", t) for t in valu[m]]
        return ops

    def stamp(self, k):
        """s_memtime → dV[(wg·4 + wave)·256 + tile][k] (STAMP builds; drains lgkmcnt)."""
        self.e("s_memtime s[18:19]")
        self.e("s_waitcnt lgkmcnt(0)")
        self.e("v_mov_b32 v206, s18")
        self.e("v_mov_b32 v207, s19")
        self.e(f"buffer_store_dwordx2 v[206:207], v205, s[{SRD_DV}:{SRD_DV + 3}], s100 offen offset:{8 * k}")

    def emit_body(self, b, lab_next, lab_epi):
        prev = self.body_ops((b + 2) % 3)
        cur = self.body_ops(b)
        # LDS issue order over (previous tile, this tile): keys of the previous body are shifted
        # one tile back so its 'next tile' reads are this body's tile-0 reads
        order = []
        for ent in prev:
            if ent[0] == "lds":
                kind, t, idx = ent[1]
                order.append((kind, t - 1, idx))
        pos = {k: i for i, k in enumerate(order)}
        done = 0                      # LDS ops [0, done) are known complete
        issued = len(order)
        if STAMP:
            self.stamp(0)
        # masked diagonal tiles: S' entries of (query < key) rows start at −inf
        if self.causal:
            skip = self.newlab("nomask")
            T = S_T
            self.e(f"s_add_u32 s{T}, s{S_CQ0}, s{sarg('coff')}")
            self.e(f"s_cmp_gt_i32 s{S_KW31}, s{T}")
            self.e(f"s_cbranch_scc0 {skip}")
            self.e("s_waitcnt lgkmcnt(0)")
            self.e(f"v_sub_u32 v{V_THR}, v{V_KT}, s{S_CQ0}")
            for qt in (0, 1):
                for g4 in range(4):
                    for e in range(4):
                        ci = 32 * qt + 8 * g4 + e
                        r = V_SACC + 16 * qt + 4 * g4 + e
                        self.e(f"v_cmp_lt_i32 vcc, {ci}, v{V_THR}")
                        self.e(f"v_cndmask_b32 v{r}, v{r}, v{V_NINF}, vcc")
            self.e("s_nop 4")
            self.lab(skip)
        for ent in cur:
            if ent[0] == "lds":
                pos[ent[1]] = issued
                issued += 1
                self.e(ent[2])
            elif ent[0] == "mfma":
                need = max(pos[d] for d in ent[2])
                if need >= done:
                    w = min(15, issued - 1 - need)
                    self.e(f"s_waitcnt lgkmcnt({w})")
                    done = issued - w
                self.e(ent[3])
            elif ent[0] == "adv":
                self.advance_pending()
            elif ent[0] == "stamp":
                self.stamp(ent[1])
                done = issued
            else:
                self.e(ent[1])
        if STAMP:
            self.stamp(5)
            self.e("s_add_u32 s3, s3, 1")
            self.e("s_min_u32 s3, s3, 255")
            self.e(f"s_lshl_b32 s100, s{S_WG}, 2")
            self.e(f"s_add_u32 s100, s100, s{S_W}")
            self.e("s_lshl_b32 s100, s100, 8")
            self.e("s_add_u32 s100, s100, s3")
            self.e("s_lshl_b32 s100, s100, 6")
        # tile bookkeeping: next tile of this item, K/V prefetch after the item's first tile,
        # item switch after its last
        self.e(f"s_add_u32 s{S_IT}, s{S_IT}, 1")
        self.e(f"s_add_u32 s{S_CQ0}, s{S_CQ0}, 64")
        self.e(f"s_cmp_ge_u32 s{S_CQ0}, s{sarg('Sq')}")
        self.e(f"s_cselect_b32 s{S_CQ0}, s{S_QF}, s{S_CQ0}")
        nopf = self.newlab("nopf")
        self.e(f"s_cmp_eq_u32 s{S_IT}, 1")
        self.e(f"s_cbranch_scc0 {nopf}")
        self.prefetch_next_kv()
        self.lab(nopf)
        self.e(f"s_cmp_lt_u32 s{S_IT}, s{S_TOT}")
        self.e(f"s_cbranch_scc1 {lab_next}")
        self.item_end(lab_next, lab_epi)

    # -- prologue / exit ------------------------------------------------------------------------------
    def prologue(self, lab_exit):
        T = S_T
        self.e("s_load_dwordx16 s[4:19], s[0:1], 0x0")
        self.e("s_load_dwordx16 s[20:35], s[0:1], 0x40")
        self.e("s_load_dwordx16 s[36:51], s[0:1], 0x80")
        self.e(f"v_and_b32 v{V_LANE}, 63, v{V_TID}")
        self.e(f"v_lshrrev_b32 v{V_TMP}, 6, v{V_TID}")
        self.e("s_waitcnt lgkmcnt(0)")
        # descriptors first (they consume the pointer arguments in s4..s19); stats row: even
        # waves −lse/scale, odd waves −δ (waves 2/3 repeat 0/1)
        self.srd(SRD_Q, sarg("q"), sarg("q_bytes"))
        self.srd(SRD_O, sarg("dout"), sarg("o_bytes"))
        self.srd(SRD_K, sarg("k"), sarg("k_bytes"))
        self.srd(SRD_V, sarg("v"), sarg("v_bytes"))
        self.srd(SRD_DK, sarg("dk"), sarg("k_bytes"))
        self.srd(SRD_DV, sarg("dv"), sarg("v_bytes"))
        self.e(f"v_readfirstlane_b32 s{SRD_ST + 2}, v{V_TMP}")      # wave id (temporarily)
        self.e(f"s_and_b32 s{SRD_ST + 3}, s{SRD_ST + 2}, 1")
        self.e(f"s_cmp_eq_u32 s{SRD_ST + 3}, 0")
        self.e(f"s_cselect_b64 s[{SRD_ST}:{SRD_ST + 1}], s[{sarg('nl')}:{sarg('nl') + 1}], s[{sarg('nd')}:{sarg('nd') + 1}]")
        self.e(f"s_mov_b32 s{S_W}, s{SRD_ST + 2}")
        self.e(f"s_lshl_b32 s{S_LDSST}, s{SRD_ST + 3}, 8")
        self.e(f"s_and_b32 s{SRD_ST + 1}, s{SRD_ST + 1}, 0xffff")
        self.e(f"s_mov_b32 s{SRD_ST + 2}, s{sarg('st_bytes')}")
        self.e(f"s_mov_b32 s{SRD_ST + 3}, 0x20000")
        self.e(f"s_lshl_b32 s{S_LDSW}, s{S_W}, 12")
        # virtual id v = (wg % 8)·(G / 8) + wg / 8: consecutive v share an XCD (dispatch deals
        # workgroups round-robin to the 8 XCDs; the host makes G a multiple of 8); u = 2v
        self.e(f"s_and_b32 s{S_U}, s{S_WG}, 7")
        self.e(f"s_lshr_b32 s{S_T}, s{sarg('G')}, 3")
        self.e(f"s_mul_i32 s{S_U}, s{S_U}, s{S_T}")
        self.e(f"s_lshr_b32 s{S_T}, s{S_WG}, 3")
        self.e(f"s_add_u32 s{S_U}, s{S_U}, s{S_T}")
        self.e(f"s_lshl_b32 s{S_U}, s{S_U}, 1")
        self.e(f"s_cmp_ge_u32 s{S_U}, s{sarg('nitems')}")
        self.e(f"s_cbranch_scc1 {lab_exit}")
        # lane decomposition: l32, hh, g = lane >> 4, gi = lane & 15
        L = V_LANE
        t = V_TMP
        self.e(f"v_and_b32 v{t}, 31, v{L}")                        # l32
        self.e(f"v_lshrrev_b32 v{t + 1}, 5, v{L}")                 # hh
        self.e(f"s_lshl_b32 s{T}, s{S_W}, 5")
        self.e(f"v_add_u32 v{t + 2}, s{T}, v{t}")                  # key - n0 = 32w + l32
        # K / V fragment loads: key row, dims 16kk + 8hh; dK / dV stores: dims +4hh
        self.e(f"v_lshlrev_b32 v{t + 3}, 4, v{t + 1}")             # 16hh
        self.e(f"v_mad_u32_u24 v{V_KVK}, v{t + 2}, s{sarg('sks')}, v{t + 3}")
        self.e(f"v_mad_u32_u24 v{V_KVV}, v{t + 2}, s{sarg('svs')}, v{t + 3}")
        self.e(f"v_lshlrev_b32 v{t + 3}, 3, v{t + 1}")             # 8hh
        self.e(f"v_mad_u32_u24 v{V_STK}, v{t + 2}, s{sarg('sks')}, v{t + 3}")
        self.e(f"v_mad_u32_u24 v{V_STV}, v{t + 2}, s{sarg('svs')}, v{t + 3}")
        # causal threshold base: 32w + l32 − coff − 4hh (+ n0 per item)
        self.e(f"v_subrev_u32 v{V_KT0}, s{sarg('coff')}, v{t + 2}")
        self.e(f"v_lshlrev_b32 v{t + 6}, 2, v{t + 1}")
        self.e(f"v_sub_u32 v{V_KT0}, v{V_KT0}, v{t + 6}")
        self.e(f"v_mov_b32 v{V_NINF}, 0xff800000")
        # LDS-DMA lane offsets: piece i of wave w = tile rows 16w + 4i + g, physical chunk pc = lane
        # & 15 holds logical chunk pc ^ x(row), x(r) = ((r & 3) << 2) | ((r >> 2) & 3) = (g << 2) | i
        self.e(f"v_lshrrev_b32 v{t + 3}, 4, v{L}")                 # g
        self.e(f"v_and_b32 v{t + 4}, 15, v{L}")                    # pc
        self.e(f"s_lshl_b32 s{T}, s{S_W}, 4")
        self.e(f"v_add_u32 v{t + 5}, s{T}, v{t + 3}")              # 16w + g
        for i in range(4):
            self.e(f"v_lshl_or_b32 v{t + 6}, v{t + 3}, 2, {i}")
            self.e(f"v_xor_b32 v{t + 6}, v{t + 6}, v{t + 4}")
            self.e(f"v_lshlrev_b32 v{t + 6}, 4, v{t + 6}")          # lc * 16
            self.e(f"v_add_u32 v{t + 7}, {4 * i}, v{t + 5}")        # row
            self.e(f"v_mad_u32_u24 v{V_DQ + i}, v{t + 7}, s{sarg('sqs')}, v{t + 6}")
            self.e(f"v_mad_u32_u24 v{V_DO + i}, v{t + 7}, s{sarg('sos')}, v{t + 6}")
        self.e(f"v_lshlrev_b32 v{V_DST}, 2, v{L}")
        # row-fragment read offsets: image row l32 (+32 qt by immediate), chunk (2kk + hh) ^ x(l32)
        self.e(f"v_and_b32 v{t + 3}, 3, v{t}")
        self.e(f"v_lshlrev_b32 v{t + 3}, 2, v{t + 3}")
        self.e(f"v_bfe_u32 v{t + 4}, v{t}, 2, 2")
        self.e(f"v_or_b32 v{t + 3}, v{t + 3}, v{t + 4}")           # xl
        self.e(f"v_lshlrev_b32 v{t + 4}, 8, v{t}")                  # l32 * 256
        for kk in range(8):
            self.e(f"v_add_u32 v{t + 5}, {2 * kk}, v{t + 1}")
            self.e(f"v_xor_b32 v{t + 5}, v{t + 5}, v{t + 3}")
            self.e(f"v_lshl_add_u32 v{V_ROW + kk}, v{t + 5}, 4, v{t + 4}")
            self.e(f"v_add_u32 v{V_ROW + 8 + kk}, {2 * BUF_B}, v{V_ROW + kk}")
        # transposed-read offsets: rows rl = 4hh + 8jj + (gi >> 2), cols 32dt + 16(g&1) + 4(gi&3)
        self.e(f"v_and_b32 v{t + 3}, 15, v{L}")                    # gi
        self.e(f"v_lshrrev_b32 v{t + 4}, 2, v{t + 3}")             # gi >> 2
        self.e(f"v_lshl_add_u32 v{t + 4}, v{t + 1}, 2, v{t + 4}")  # 4hh + (gi >> 2)
        self.e(f"v_and_b32 v{t + 5}, 3, v{t + 3}")
        self.e(f"v_lshlrev_b32 v{t + 5}, 2, v{t + 5}")             # 4(gi & 3)
        self.e(f"v_bfe_u32 v{t + 6}, v{L}, 4, 1")
        self.e(f"v_lshl_add_u32 v{t + 5}, v{t + 6}, 4, v{t + 5}")  # col (dt = 0)
        for jj in (0, 1):
            self.e(f"v_add_u32 v{t + 6}, {8 * jj}, v{t + 4}")       # rl
            self.e(f"v_and_b32 v{t + 7}, 3, v{t + 6}")
            self.e(f"v_lshlrev_b32 v{t + 7}, 2, v{t + 7}")
            self.e(f"v_bfe_u32 v{t + 2}, v{t + 6}, 2, 2")
            self.e(f"v_or_b32 v{t + 7}, v{t + 7}, v{t + 2}")        # xr
            self.e(f"v_lshrrev_b32 v{t + 2}, 3, v{t + 5}")          # col >> 3
            self.e(f"v_xor_b32 v{t + 7}, v{t + 7}, v{t + 2}")
            self.e(f"v_lshlrev_b32 v{t + 7}, 4, v{t + 7}")
            self.e(f"v_lshl_add_u32 v{t + 7}, v{t + 6}, 8, v{t + 7}")
            self.e(f"v_and_b32 v{t + 2}, 7, v{t + 5}")
            self.e(f"v_lshl_add_u32 v{t + 7}, v{t + 2}, 1, v{t + 7}")   # dt = 0 offset
            for dt in range(4):
                r = V_TR + 4 * jj + dt
                self.e(f"v_xor_b32 v{r}, {dt << 6}, v{t + 7}")
                self.e(f"v_add_u32 v{r + 8}, {2 * BUF_B}, v{r}")
        self.e(f"v_lshlrev_b32 v{t + 2}, 4, v{t + 1}")
        self.e(f"v_add_u32 v{V_STB}, {OFF_ST}, v{t + 2}")
        self.e(f"v_add_u32 v{V_STB + 1}, {2 * BUF_B + OFF_ST}, v{t + 2}")
        if STAMP:
            self.e("s_mov_b32 s3, 0")
            self.e(f"s_lshl_b32 s100, s{S_WG}, 2")
            self.e(f"s_add_u32 s100, s100, s{S_W}")
            self.e("s_lshl_b32 s100, s100, 14")
            self.e("v_mov_b32 v205, 0")
        # first item: compute state, its K / V, and the DMA stream primed with its first tiles
        self.compute_item_setup()
        self.kv_load(A_KF, A_VF, S_SOFFK, S_SOFFV)
        self.e(f"s_mov_b32 s{S_DU}, s{S_U}")
        self.pending_item_setup()
        self.pending_soffs()
        for m0, ld in self.dma_first(0) + self.dma_second(0):
            self.e(m0)
            self.e(ld)
        self.advance_pending()
        for m0, ld in self.dma_first(1):
            self.e(m0)
            self.e(ld)
        for i in range(128):
            self.e(f"v_accvgpr_write_b32 a{i}, 0")
        self.e("s_waitcnt vmcnt(5)")
        self.e("s_barrier")
        for _, txt in self.stats_reads(0):
            self.e(txt)
        for m in range(LA):
            for txt in self.ring_reads(0, m):
                self.e(txt)
        self.e("s_waitcnt lgkmcnt(0)")
        self.e("s_nop 4")

    def exit(self):
        # the LDS-DMA stream may still be landing (past-the-end tiles): LDS must stay ours until
        # it has; the dK / dV stores need no wait
        self.e("s_waitcnt vmcnt(0)")
        self.e("s_endpgm")

    def text(self):
        self.lines = []
        labs = [self.newlab(f"tile{b}") for b in range(3)]
        lexit = self.newlab("exit")
        self.prologue(lexit)
        self.in_loop = True
        for b in range(3):
            self.lab(labs[b])
            self.emit_body(b, labs[(b + 1) % 3], lexit)
        self.in_loop = False
        self.lab(lexit)
        self.exit()
        n = self.name
        head = ["\t.text", f"\t.globl {n}", "\t.p2align 8", f"\t.type {n},@function", f"{n}:"]
        tail = [
            f".L{n}_end:",
            f"\t.size {n}, .L{n}_end-{n}",
            "\t.rodata",
            "\t.p2align 6",
            f"\t.amdhsa_kernel {n}",
            f"\t\t.amdhsa_group_segment_fixed_size {LDS_BYTES}",
            "\t\t.amdhsa_private_segment_fixed_size 0",
            f"\t\t.amdhsa_kernarg_size {ARGS_SIZE}",
            "\t\t.amdhsa_user_sgpr_count 2",
            "\t\t.amdhsa_user_sgpr_kernarg_segment_ptr 1",
            "\t\t.amdhsa_system_sgpr_workgroup_id_x 1",
            "\t\t.amdhsa_system_vgpr_workitem_id 0",
            f"\t\t.amdhsa_next_free_vgpr {NV + NA}",
            f"\t\t.amdhsa_next_free_sgpr {NSGPR}",
            f"\t\t.amdhsa_accum_offset {NV}",
            "\t\t.amdhsa_reserve_vcc 1",
            "\t\t.amdhsa_float_denorm_mode_32 3",
            "\t\t.amdhsa_float_denorm_mode_16_64 3",
            "\t\t.amdhsa_ieee_mode 0",
            "\t\t.amdhsa_dx10_clamp 1",
            "\t.end_amdhsa_kernel",
            "\t.text",
        ]
        return "\n".join(head + self.lines + tail) + "\n"

    def metadata(self):
        return f"""  - .args:
      - .offset:         0
        .size:           {ARGS_SIZE}
        .value_kind:     by_value
    .group_segment_fixed_size: {LDS_BYTES}
    .kernarg_segment_align: 8
    .kernarg_segment_size: {ARGS_SIZE}
    .max_flat_workgroup_size: 256
    .name:           {self.name}
    .private_segment_fixed_size: 0
    .sgpr_count:     {NSGPR + 6}
    .sgpr_spill_count: 0
    .symbol:         {self.name}.kd
    .vgpr_count:     {NV + NA}
    .agpr_count:     {NA}
    .vgpr_spill_count: 0
    .wavefront_size: 64
"""



# =================================================================================================
# dQ kernel (`fa_dq`): the same machine with the roles of (Q, dO) and (K, V) swapped
# =================================================================================================
# workgroup = 128 queries of one (batch, q-head), 4 waves × 32 queries (query on the MFMA lane);
# for every 64-key tile (causal: up to the diagonal) of the head's kv-head:
#   Sᵀ = K·Qᵀ,  dPᵀ = V·dOᵀ        (A = K / V rows from LDS, B = Q / dO fragments in AGPRs)
#   P = exp2(c·Sᵀ + c·(−lse/scale)_q),  dS = P ∘ (dPᵀ − δ_q)   (row constants are PER LANE here)
#   dQᵀ += Kᵀ·dS                    (A = transposed K reads, B = dS fragments; dQ · scale at the end)
# Causal masking costs nothing per element: the first S MFMA of a diagonal tile starts from a
# 0 / −inf pattern register set instead of 0 (set between tiles, only for the last two tiles of an
# item). 48 MFMAs per tile: S(kb 0) P(kb 0) S(kb 1) P(kb 1) [8 each], C(ks 0,1) C(ks 2,3) [8 each].
DQ_ARGS = [
    ("q", 0, 8), ("k", 8, 8), ("v", 16, 8), ("dout", 24, 8), ("dq", 32, 8), ("pad0", 40, 8),
    ("nl", 48, 8), ("nd", 56, 8),
    ("q_bytes", 64, 4), ("k_bytes", 68, 4), ("v_bytes", 72, 4), ("o_bytes", 76, 4), ("st_bytes", 80, 4),
    ("sqs", 84, 4), ("sqh", 88, 4), ("sqb", 92, 4),
    ("sks", 96, 4), ("skh", 100, 4), ("skb", 104, 4),
    ("svs", 108, 4), ("svh", 112, 4), ("svb", 116, 4),
    ("sos", 120, 4), ("soh", 124, 4), ("sob", 128, 4),
    ("Hq", 132, 4), ("group", 136, 4), ("rcp_group", 140, 4), ("Sq", 144, 4), ("nkt", 148, 4),
    ("npair", 152, 4), ("nqb1", 156, 4), ("rcp_npair", 160, 4), ("c", 164, 4), ("scale", 168, 4),
    ("rcp_Hq", 172, 4), ("pad1", 176, 4), ("nitems", 180, 4), ("G", 184, 4), ("G2m1", 188, 4),
]


def qarg(name):
    for n, off, _ in DQ_ARGS:
        if n == name:
            return 4 + off // 4
    raise KeyError(name)


# SGPRs (s4..s19: pointer arguments until the descriptors exist)
Q_SOB, Q_SKB, Q_SVB, Q_W, Q_LDSW = 4, 5, 6, 7, 8          # DMA-side batch/head bases, wave, LDS
Q_T = 10                                                  # temps s10..s17
QSRD_K, QSRD_V, QSRD_Q, QSRD_O, QSRD_DQ, QSRD_NL, QSRD_ND = 52, 56, 60, 64, 68, 72, 76
# compute side: item, batch, q-head, query-block start, tiles, tile index, Q/dO/dQ soffset, stats soffset
Q_U, Q_B, Q_HQ, Q_Q0, Q_TOT, Q_IT, Q_SOFFQ, Q_SOFFO, Q_SOFFS = range(80, 89)
# DMA side: item, its tile count, tile index, key start, K / V soffsets
Q_DU, Q_DTOT, Q_DIT, Q_DK0, Q_SK, Q_SV = range(89, 95)
Q_NSGPR = 101

QV_DK, QV_DV = 2, 6                # LDS-DMA lane offsets: K pieces 0-3, V pieces 0-3
QV_ROW, QV_TR = 11, 27             # [set 2][kk 8] / [set 2][jj 2][dt 4] read offsets
QV_QL, QV_THR, QV_NINF = 45, 46, 47
QV_RING = 48                       # 12 slots × 4
QV_SACC, QV_PACC = 96, 128         # Sᵀ / dPᵀ accumulators [kb 2][16]
QV_DS = 160                        # dS bf16 fragments [ks 4][4]
QV_MASK = 176                      # first-S-MFMA accumulator inputs [kb 2][16] (0 / −inf)
QV_TMP = 208                       # temps v208..v215
QV_NLC, QV_ND, QV_NLCN, QV_NDN = 216, 217, 218, 219   # c·(−lse/scale), −δ (current / next item)
QV_QV, QV_OV, QV_STQ, QV_STV4 = 220, 221, 222, 223    # Q / dO fragment, dQ store, stats lane offsets
QV_NDSET = 224                     # −δ of the lane's query × 16: accumulator start of the first dP MFMA
QNV = 240
QA_DQ, QA_QF, QA_OF, QA_QN, QA_ON = 0, 64, 96, 128, 160
QNA = 192
QBUF_B = 32768                     # per buffer: K 16 KiB, V 16 KiB
Q_OFF_V = 16384
QLDS_BYTES = 3 * QBUF_B
QLA = int(os.environ.get("PIAMD_FA_QLA", "6"))  # dQ ring lookahead (≤ 8: reads stay behind the barrier at gap 39)


def qbuf_set(b):
    return (0, 0) if b == 0 else (0, QBUF_B) if b == 1 else (1, 0)


class FaDq(FaDkdv):
    NM = 48
    VTMP_UDIV = QV_TMP + 4
    QSH = 7          # log2 of the queries per work item (4 waves × 32)

    # -- DMA stream (K / V tiles of 64 keys) --------------------------------------------------------
    def pending_soffs(self):
        T = Q_T
        self.e(f"s_mul_i32 s{T}, s{Q_DK0}, s{qarg('sks')}")
        self.e(f"s_add_u32 s{Q_SK}, s{T}, s{Q_SKB}")
        self.e(f"s_mul_i32 s{T}, s{Q_DK0}, s{qarg('svs')}")
        self.e(f"s_add_u32 s{Q_SV}, s{T}, s{Q_SVB}")
        self.e(f"s_cmp_ge_u32 s{Q_DU}, s{qarg('nitems')}")
        self.e(f"s_cselect_b32 s{Q_SK}, s{qarg('k_bytes')}, s{Q_SK}")
        self.e(f"s_cselect_b32 s{Q_SV}, s{qarg('v_bytes')}, s{Q_SV}")

    def advance_pending(self):
        self.e(f"s_add_u32 s{Q_DIT}, s{Q_DIT}, 1")
        self.e(f"s_add_u32 s{Q_DK0}, s{Q_DK0}, 64")
        same = self.newlab("sameitem")
        self.e(f"s_cmp_lt_u32 s{Q_DIT}, s{Q_DTOT}")
        self.e(f"s_cbranch_scc1 {same}")
        self.next_item(Q_DU)
        self.e(f"s_cmp_ge_u32 s{Q_DU}, s{qarg('nitems')}")
        self.e(f"s_cbranch_scc1 {same}")
        self.pending_item_setup()
        self.lab(same)
        self.pending_soffs()

    def next_item(self, u):
        T = Q_T
        self.e(f"s_bitcmp1_b32 s{u}, 0")
        self.e(f"s_cselect_b32 s{T + 7}, s{qarg('G2m1')}, 1")
        self.e(f"s_add_u32 s{u}, s{u}, s{T + 7}")

    def decode(self, u, qb, b, hq):
        """Item u = 2·member + s → query block qb (pairs (j, nqb−1−j): equal causal work), batch
        b, q-head hq; a pair group = one (batch, q-head), its members on one XCD."""
        T = Q_T
        self.e(f"s_lshr_b32 s{T + 7}, s{u}, 1")
        self.udiv(T + 6, qb, T + 7, qarg("npair"), qarg("rcp_npair"))      # group, j
        self.e(f"s_sub_u32 s{T + 7}, s{qarg('nqb1')}, s{qb}")
        self.e(f"s_bitcmp1_b32 s{u}, 0")
        self.e(f"s_cselect_b32 s{qb}, s{T + 7}, s{qb}")
        self.udiv(b, hq, T + 6, qarg("Hq"), qarg("rcp_Hq"))

    def tiles_of(self, dst, qb):
        if self.causal:   # key tiles of 64 up to the item's last query
            self.e(f"s_lshl_b32 s{dst}, s{qb}, {self.QSH - 6}")
            self.e(f"s_add_u32 s{dst}, s{dst}, {1 << (self.QSH - 6)}")
        else:
            self.e(f"s_mov_b32 s{dst}, s{qarg('nkt')}")

    def kv_bases(self, b, hq, kb, vb):
        """K / V soffset bases of (batch b, kv-head hq / group)."""
        T = Q_T
        self.udiv(T + 3, T + 4, hq, qarg("group"), qarg("rcp_group"))   # hk → s{T+3}
        for dst, sb, sh in ((kb, "skb", "skh"), (vb, "svb", "svh")):
            self.e(f"s_mul_i32 s{dst}, s{b}, s{qarg(sb)}")
            self.e(f"s_mul_i32 s{T + 4}, s{T + 3}, s{qarg(sh)}")
            self.e(f"s_add_u32 s{dst}, s{dst}, s{T + 4}")

    def pending_item_setup(self):
        T = Q_T
        self.decode(Q_DU, T, T + 1, T + 2)
        self.tiles_of(Q_DTOT, T)
        self.e(f"s_mov_b32 s{Q_DIT}, 0")
        self.e(f"s_mov_b32 s{Q_DK0}, 0")
        self.kv_bases(T + 1, T + 2, Q_SKB, Q_SVB)

    def dma_first(self, buf):
        base = buf * QBUF_B
        return [[f"s_add_u32 m0, s{Q_LDSW}, {base + i * 1024}\n\ts_nop 0",
                 f"buffer_load_dwordx4 v{QV_DK + i}, s[{QSRD_K}:{QSRD_K + 3}], s{Q_SK} offen lds"]
                for i in range(4)]

    def dma_second(self, buf):
        base = buf * QBUF_B + Q_OFF_V
        return [[f"s_add_u32 m0, s{Q_LDSW}, {base + i * 1024}\n\ts_nop 0",
                 f"buffer_load_dwordx4 v{QV_DV + i}, s[{QSRD_V}:{QSRD_V + 3}], s{Q_SV} offen lds"]
                for i in range(4)]

    # -- items: Q / dO fragments + per-lane row constants -------------------------------------------
    def q_soffs(self, qb, b, hq, sq, so, ss):
        """Q/dQ, dO and stats soffsets of the wave's 32 queries of item (qb, b, hq)."""
        T = Q_T
        self.e(f"s_lshl_b32 s{T + 7}, s{qb}, {self.QSH}")               # q0
        for dst, sb, sh, st in ((sq, "sqb", "sqh", "sqs"), (so, "sob", "soh", "sos")):
            self.e(f"s_mul_i32 s{dst}, s{b}, s{qarg(sb)}")
            self.e(f"s_mul_i32 s{T + 5}, s{hq}, s{qarg(sh)}")
            self.e(f"s_add_u32 s{dst}, s{dst}, s{T + 5}")
            self.e(f"s_mul_i32 s{T + 5}, s{T + 7}, s{qarg(st)}")
            self.e(f"s_add_u32 s{dst}, s{dst}, s{T + 5}")
        self.e(f"s_mul_i32 s{ss}, s{b}, s{qarg('Hq')}")
        self.e(f"s_add_u32 s{ss}, s{ss}, s{hq}")
        self.e(f"s_mul_i32 s{ss}, s{ss}, s{qarg('Sq')}")
        self.e(f"s_add_u32 s{ss}, s{ss}, s{T + 7}")
        self.e(f"s_lshl_b32 s{ss}, s{ss}, 2")

    def q_load(self, aq, ao, nl, nd, sq, so, ss):
        for kk in range(8):
            self.e(f"buffer_load_dwordx4 a[{aq + 4 * kk}:{aq + 4 * kk + 3}], v{QV_QV}, s[{QSRD_Q}:{QSRD_Q + 3}], s{sq} offen offset:{32 * kk}")
        for kk in range(8):
            self.e(f"buffer_load_dwordx4 a[{ao + 4 * kk}:{ao + 4 * kk + 3}], v{QV_OV}, s[{QSRD_O}:{QSRD_O + 3}], s{so} offen offset:{32 * kk}")
        self.e(f"buffer_load_dword v{nl}, v{QV_STV4}, s[{QSRD_NL}:{QSRD_NL + 3}], s{ss} offen")
        self.e(f"buffer_load_dword v{nd}, v{QV_STV4}, s[{QSRD_ND}:{QSRD_ND + 3}], s{ss} offen")

    def compute_item_setup(self):
        T = Q_T
        self.decode(Q_U, T, Q_B, Q_HQ)
        self.e(f"s_lshl_b32 s{Q_Q0}, s{T}, 7")
        self.tiles_of(Q_TOT, T)
        self.e(f"s_mov_b32 s{Q_IT}, 0")
        self.q_soffs(T, Q_B, Q_HQ, Q_SOFFQ, Q_SOFFO, Q_SOFFS)
        # causal threshold base: query − 4hh (lane), per item
        self.e(f"s_lshl_b32 s{T}, s{Q_W}, 5")
        self.e(f"s_add_u32 s{T}, s{T}, s{Q_Q0}")
        self.e(f"v_add_u32 v{QV_QL}, s{T}, v{QV_TMP + 7}")              # v{TMP+7} = l32 − 4hh

    def mask_setup(self):
        """Accumulator-start pattern of the next tile's S MFMAs: 0, or −inf where key > query (the
        last two tiles of a causal item)."""
        if not self.causal:
            return
        T = Q_T
        skip, done = self.newlab("nomask"), self.newlab("maskdone")
        self.e(f"s_sub_u32 s{T}, s{Q_TOT}, 2")
        self.e(f"s_cmp_lt_i32 s{Q_IT}, s{T}")
        self.e(f"s_cbranch_scc1 {skip}")
        self.e(f"s_lshl_b32 s{T}, s{Q_IT}, 6")
        self.e(f"v_subrev_u32 v{QV_THR}, s{T}, v{QV_QL}")               # q − 4hh − 64 kt
        for kb in (0, 1):
            for g4 in range(4):
                for e in range(4):
                    ci = 32 * kb + 8 * g4 + e
                    r = QV_MASK + 16 * kb + 4 * g4 + e
                    self.e(f"v_cmp_gt_i32 vcc, {ci}, v{QV_THR}")
                    self.e(f"v_cndmask_b32 v{r}, 0, v{QV_NINF}, vcc")
        self.e(f"s_branch {done}")
        self.lab(skip)
        self.e(f"s_cmp_eq_u32 s{Q_IT}, 0")                              # item start: clear
        self.e(f"s_cbranch_scc0 {done}")
        for i in range(32):
            self.e(f"v_mov_b32 v{QV_MASK + i}, 0")
        self.lab(done)
        self.e("s_nop 4")

    def prefetch_next(self):
        T = Q_T
        skip = self.newlab("nopf")
        self.e(f"s_mov_b32 s{T + 3}, s{Q_U}")
        self.next_item(T + 3)
        self.e(f"s_cmp_ge_u32 s{T + 3}, s{qarg('nitems')}")
        self.e(f"s_cbranch_scc1 {skip}")
        self.decode(T + 3, T, T + 1, T + 2)
        self.q_soffs(T, T + 1, T + 2, T + 3, T + 4, T + 6)
        self.q_load(QA_QN, QA_ON, QV_NLCN, QV_NDN, T + 3, T + 4, T + 6)
        self.lab(skip)

    def store_dq(self):
        t = QV_TMP
        for dt in range(4):
            for g4 in range(4):
                a0 = QA_DQ + 16 * dt + 4 * g4
                for j in range(4):
                    self.e(f"v_accvgpr_read_b32 v{t + j}, a{a0 + j}")
                for j in range(4):
                    self.e(f"v_mul_f32 v{t + j}, s{qarg('scale')}, v{t + j}")
                self.e(f"v_cvt_pk_bf16_f32 v{t}, v{t}, v{t + 1}")
                self.e(f"v_cvt_pk_bf16_f32 v{t + 1}, v{t + 2}, v{t + 3}")
                self.e(f"buffer_store_dwordx2 v[{t}:{t + 1}], v{QV_STQ}, s[{QSRD_DQ}:{QSRD_DQ + 3}], s{Q_SOFFQ} offen offset:{64 * dt + 16 * g4}")

    def item_end(self, lab_next, lab_exit):
        self.e("s_nop 15")
        self.e("s_nop 15")
        self.store_dq()
        for i in range(64):
            self.e(f"v_accvgpr_write_b32 a{QA_DQ + i}, 0")
        for i in range(64):
            self.e(f"v_accvgpr_mov_b32 a{QA_QF + i}, a{QA_QN + i}")
        self.e(f"v_mul_f32 v{QV_NLC}, s{qarg('c')}, v{QV_NLCN}")
        for i in range(16):
            self.e(f"v_mov_b32 v{QV_NDSET + i}, v{QV_NDN}")
        self.next_item(Q_U)
        self.e(f"s_cmp_ge_u32 s{Q_U}, s{qarg('nitems')}")
        self.e(f"s_cbranch_scc1 {lab_exit}")
        self.compute_item_setup()
        self.mask_setup()
        self.e("s_nop 4")
        self.e(f"s_branch {lab_next}")

    # -- MFMA stream --------------------------------------------------------------------------------
    @staticmethod
    def mfma_kind(m):
        """MFMA m of a tile → ('S'|'P', kb, kk) or ('C', dt, ks)."""
        if m < 32:
            kb, r = m // 16, m % 16
            return ("S" if r < 8 else "P", kb, r % 8)
        c = m - 32
        half, cc = c // 8, c % 8
        return ("C", cc % 4, 2 * half + cc // 4)

    @staticmethod
    def slot(b, m):
        return QV_RING + 4 * ((48 * b + m) % RING)

    def ring_reads(self, b, m):
        kind, x, y = self.mfma_kind(m)
        s, imm = qbuf_set(b)
        d = self.slot(b, m)
        if kind in ("S", "P"):
            kb, kk = x, y
            off = imm + (Q_OFF_V if kind == "P" else 0) + kb * 8192
            return [f"ds_read_b128 v[{d}:{d + 3}], v{QV_ROW + 8 * s + kk} offset:{off}"]
        dt, ks = x, y
        off = imm + ks * 16 * 256
        return [f"ds_read_b64_tr_b16 v[{d + 2 * jj}:{d + 2 * jj + 1}], v{QV_TR + 8 * s + 4 * jj + dt} offset:{off}"
                for jj in (0, 1)]

    def mfma_text(self, b, m):
        kind, x, y = self.mfma_kind(m)
        a = self.slot(b, m)
        if kind in ("S", "P"):
            kb, kk = x, y
            acc = (QV_SACC if kind == "S" else QV_PACC) + 16 * kb
            bop = (QA_QF if kind == "S" else QA_OF) + 4 * kk
            if kk == 0:
                if kind == "P":   # dPᵀ − δ from the start
                    src = f"v[{QV_NDSET}:{QV_NDSET + 15}]"
                else:
                    src = f"v[{QV_MASK + 16 * kb}:{QV_MASK + 16 * kb + 15}]" if self.causal else "0"
            else:
                src = f"v[{acc}:{acc + 15}]"
            return f"{MFMA} v[{acc}:{acc + 15}], v[{a}:{a + 3}], a[{bop}:{bop + 3}], {src}"
        dt, ks = x, y
        acc = QA_DQ + 16 * dt
        bop = QV_DS + 4 * ks
        return f"{MFMA} a[{acc}:{acc + 15}], v[{a}:{a + 3}], v[{bop}:{bop + 3}], a[{acc}:{acc + 15}]"

    def finish_queues(self):
        qs = []
        for kb in (0, 1):
            sq, dq = [], []
            for j in range(8):
                s0, s1 = QV_SACC + 16 * kb + 2 * j, QV_SACC + 16 * kb + 2 * j + 1
                d0, d1 = QV_PACC + 16 * kb + 2 * j, QV_PACC + 16 * kb + 2 * j + 1
                sq += [(f"v_fma_f32 v{s0}, v{s0}, s{qarg('c')}, v{QV_NLC}", 4, j),
                       (f"v_fma_f32 v{s1}, v{s1}, s{qarg('c')}, v{QV_NLC}", 4, j),
                       (f"v_exp_f32 v{s0}, v{s0}", 8, j),
                       (f"v_exp_f32 v{s1}, v{s1}", 8, j)]
                fr = 4 * (2 * kb + j // 4) + j % 4
                dq += [(f"v_mul_f32 v{d0}, v{s0}, v{d0}", 4, j),
                       (f"v_mul_f32 v{d1}, v{s1}, v{d1}", 4, j),
                       (f"v_cvt_pk_bf16_f32 v{QV_DS + fr}, v{d0}, v{d1}", 4, j)]
            dl = 30 + 8 * kb
            qs.append(dict(name=f"S{kb}", ops=sq, lo=16 * kb + 9, hi=dl - 2))
            qs.append(dict(name=f"D{kb}", ops=dq, lo=16 * kb + 17, hi=dl, dep=len(qs) - 1))
        return qs

    def body_ops(self, b):
        nb = (b + 1) % 3
        NM = self.NM
        gaps = [[] for _ in range(NM)]
        fixed = [0] * NM
        for m in range(NM):
            g = m - QLA
            if g >= 0:
                for t in self.ring_reads(b, m):
                    gaps[g].append(("lds", ("ring", 0, m), t))
                    fixed[g] += 2
        for m in range(QLA):
            g = NM - QLA + m
            for t in self.ring_reads(nb, m):
                gaps[g].append(("lds", ("ring", 1, m), t))
                fixed[g] += 2
        # one barrier per tile: tile t+1 landed (its DMA went out one tile ago), buffer t−1 free;
        # then the whole DMA of tile t+2 and the cursor advance
        gaps[39].append(("txt", "s_waitcnt vmcnt(0)"))
        gaps[39].append(("txt", "s_barrier"))
        fixed[39] += 8
        ops2 = self.dma_first((b + 2) % 3) + self.dma_second((b + 2) % 3)
        for i, (m0, ld) in enumerate(ops2):
            g = 40 + i
            gaps[g] += [("txt", m0), ("txt", ld)]
            fixed[g] += 12
        gaps[47].append(("adv",))
        fixed[47] += 8
        valu = self.schedule_valu(fixed)
        if "novalu" in ABL:
            valu = [[] for _ in range(NM)]
        ops = []
        for m in range(NM):
            ops.append(("mfma", m, [("ring", 0, m)], self.mfma_text(b, m)))
            ops += gaps[m]
            ops += [("txt", t) for t in valu[m]]
        return ops

    def emit_body(self, b, lab_next, lab_epi):
        prev = self.body_ops((b + 2) % 3)
        cur = self.body_ops(b)
        order = []
        for ent in prev:
            if ent[0] == "lds":
                kind, t, idx = ent[1]
                order.append((kind, t - 1, idx))
        pos = {k: i for i, k in enumerate(order)}
        done = 0
        issued = len(order)
        for ent in cur:
            if ent[0] == "lds":
                pos[ent[1]] = issued
                issued += 1
                self.e(ent[2])
            elif ent[0] == "mfma":
                need = max(pos[d] for d in ent[2])
                if need >= done:
                    w = min(15, issued - 1 - need)
                    self.e(f"s_waitcnt lgkmcnt({w})")
                    done = issued - w
                self.e(ent[3])
            elif ent[0] == "adv":
                self.advance_pending()
            else:
                self.e(ent[1])
        self.e(f"s_add_u32 s{Q_IT}, s{Q_IT}, 1")
        nopf = self.newlab("nopf")
        self.e(f"s_cmp_eq_u32 s{Q_IT}, 1")
        self.e(f"s_cbranch_scc0 {nopf}")
        self.prefetch_next()
        self.lab(nopf)
        nxt = self.newlab("same")
        self.e(f"s_cmp_lt_u32 s{Q_IT}, s{Q_TOT}")
        self.e(f"s_cbranch_scc1 {nxt}")
        self.item_end(lab_next, lab_epi)
        self.lab(nxt)
        self.mask_setup()
        self.e(f"s_branch {lab_next}")

    # -- prologue ---------------------------------------------------------------------------------------
    def prologue(self, lab_exit):
        T = Q_T
        self.e("s_load_dwordx16 s[4:19], s[0:1], 0x0")
        self.e("s_load_dwordx16 s[20:35], s[0:1], 0x40")
        self.e("s_load_dwordx16 s[36:51], s[0:1], 0x80")
        self.e(f"v_and_b32 v{V_LANE}, 63, v{V_TID}")
        self.e(f"v_lshrrev_b32 v{QV_TMP}, 6, v{V_TID}")
        self.e("s_waitcnt lgkmcnt(0)")
        self.srd(QSRD_K, qarg("k"), qarg("k_bytes"))
        self.srd(QSRD_V, qarg("v"), qarg("v_bytes"))
        self.srd(QSRD_Q, qarg("q"), qarg("q_bytes"))
        self.srd(QSRD_O, qarg("dout"), qarg("o_bytes"))
        self.srd(QSRD_DQ, qarg("dq"), qarg("q_bytes"))
        self.srd(QSRD_NL, qarg("nl"), qarg("st_bytes"))
        self.srd(QSRD_ND, qarg("nd"), qarg("st_bytes"))
        self.e(f"v_readfirstlane_b32 s{Q_W}, v{QV_TMP}")
        self.e(f"s_lshl_b32 s{Q_LDSW}, s{Q_W}, 12")
        self.e(f"s_and_b32 s{Q_U}, s{S_WG}, 7")
        self.e(f"s_lshr_b32 s{T}, s{qarg('G')}, 3")
        self.e(f"s_mul_i32 s{Q_U}, s{Q_U}, s{T}")
        self.e(f"s_lshr_b32 s{T}, s{S_WG}, 3")
        self.e(f"s_add_u32 s{Q_U}, s{Q_U}, s{T}")
        self.e(f"s_lshl_b32 s{Q_U}, s{Q_U}, 1")
        self.e(f"s_cmp_ge_u32 s{Q_U}, s{qarg('nitems')}")
        self.e(f"s_cbranch_scc1 {lab_exit}")
        L = V_LANE
        t = QV_TMP
        self.e(f"v_and_b32 v{t}, 31, v{L}")                        # l32
        self.e(f"v_lshrrev_b32 v{t + 1}, 5, v{L}")                 # hh
        self.e(f"s_lshl_b32 s{T}, s{Q_W}, 5")
        self.e(f"v_add_u32 v{t + 2}, s{T}, v{t}")                  # 32w + l32 (query − q0)
        self.e(f"v_lshlrev_b32 v{t + 3}, 4, v{t + 1}")             # 16hh
        self.e(f"v_mad_u32_u24 v{QV_QV}, v{t + 2}, s{qarg('sqs')}, v{t + 3}")
        self.e(f"v_mad_u32_u24 v{QV_OV}, v{t + 2}, s{qarg('sos')}, v{t + 3}")
        self.e(f"v_lshlrev_b32 v{t + 3}, 3, v{t + 1}")             # 8hh
        self.e(f"v_mad_u32_u24 v{QV_STQ}, v{t + 2}, s{qarg('sqs')}, v{t + 3}")
        self.e(f"v_lshlrev_b32 v{QV_STV4}, 2, v{t + 2}")           # stats: 4·(32w + l32)
        self.e(f"v_lshlrev_b32 v{t + 6}, 2, v{t + 1}")
        self.e(f"v_sub_u32 v{t + 7}, v{t}, v{t + 6}")              # l32 − 4hh (kept for the items)
        self.e(f"v_mov_b32 v{QV_NINF}, 0xff800000")
        # LDS-DMA lane offsets (K / V image rows = keys; same piece mapping as the dK/dV kernel)
        self.e(f"v_lshrrev_b32 v{t + 3}, 4, v{L}")
        self.e(f"v_and_b32 v{t + 4}, 15, v{L}")
        self.e(f"s_lshl_b32 s{T}, s{Q_W}, 4")
        self.e(f"v_add_u32 v{t + 5}, s{T}, v{t + 3}")
        for i in range(4):
            self.e(f"v_lshl_or_b32 v{t + 6}, v{t + 3}, 2, {i}")
            self.e(f"v_xor_b32 v{t + 6}, v{t + 6}, v{t + 4}")
            self.e(f"v_lshlrev_b32 v{t + 6}, 4, v{t + 6}")
            self.e(f"v_add_u32 v{t + 2}, {4 * i}, v{t + 5}")
            self.e(f"v_mad_u32_u24 v{QV_DK + i}, v{t + 2}, s{qarg('sks')}, v{t + 6}")
            self.e(f"v_mad_u32_u24 v{QV_DV + i}, v{t + 2}, s{qarg('svs')}, v{t + 6}")
        # row-fragment / transposed read offsets (identical image layout to the dK/dV kernel)
        self.e(f"v_and_b32 v{t + 3}, 3, v{t}")
        self.e(f"v_lshlrev_b32 v{t + 3}, 2, v{t + 3}")
        self.e(f"v_bfe_u32 v{t + 4}, v{t}, 2, 2")
        self.e(f"v_or_b32 v{t + 3}, v{t + 3}, v{t + 4}")
        self.e(f"v_lshlrev_b32 v{t + 4}, 8, v{t}")
        for kk in range(8):
            self.e(f"v_add_u32 v{t + 5}, {2 * kk}, v{t + 1}")
            self.e(f"v_xor_b32 v{t + 5}, v{t + 5}, v{t + 3}")
            self.e(f"v_lshl_add_u32 v{QV_ROW + kk}, v{t + 5}, 4, v{t + 4}")
            self.e(f"v_add_u32 v{QV_ROW + 8 + kk}, {2 * QBUF_B}, v{QV_ROW + kk}")
        self.e(f"v_and_b32 v{t + 3}, 15, v{L}")
        self.e(f"v_lshrrev_b32 v{t + 4}, 2, v{t + 3}")
        self.e(f"v_lshl_add_u32 v{t + 4}, v{t + 1}, 2, v{t + 4}")
        self.e(f"v_and_b32 v{t + 5}, 3, v{t + 3}")
        self.e(f"v_lshlrev_b32 v{t + 5}, 2, v{t + 5}")
        self.e(f"v_bfe_u32 v{t + 6}, v{L}, 4, 1")
        self.e(f"v_lshl_add_u32 v{t + 5}, v{t + 6}, 4, v{t + 5}")
        for jj in (0, 1):
            self.e(f"v_add_u32 v{t + 6}, {8 * jj}, v{t + 4}")
            self.e(f"v_and_b32 v{QV_THR}, 3, v{t + 6}")
            self.e(f"v_lshlrev_b32 v{QV_THR}, 2, v{QV_THR}")
            self.e(f"v_bfe_u32 v{t + 2}, v{t + 6}, 2, 2")
            self.e(f"v_or_b32 v{QV_THR}, v{QV_THR}, v{t + 2}")
            self.e(f"v_lshrrev_b32 v{t + 2}, 3, v{t + 5}")
            self.e(f"v_xor_b32 v{QV_THR}, v{QV_THR}, v{t + 2}")
            self.e(f"v_lshlrev_b32 v{QV_THR}, 4, v{QV_THR}")
            self.e(f"v_lshl_add_u32 v{QV_THR}, v{t + 6}, 8, v{QV_THR}")
            self.e(f"v_and_b32 v{t + 2}, 7, v{t + 5}")
            self.e(f"v_lshl_add_u32 v{QV_THR}, v{t + 2}, 1, v{QV_THR}")
            for dt in range(4):
                r = QV_TR + 4 * jj + dt
                self.e(f"v_xor_b32 v{r}, {dt << 6}, v{QV_THR}")
                self.e(f"v_add_u32 v{r + 8}, {2 * QBUF_B}, v{r}")
        # first item: its Q / dO / row constants, the DMA stream primed with its first K/V tiles
        self.compute_item_setup()
        self.q_load(QA_QF, QA_OF, QV_NLC, QV_ND, Q_SOFFQ, Q_SOFFO, Q_SOFFS)
        self.e(f"s_mov_b32 s{Q_DU}, s{Q_U}")
        self.pending_item_setup()
        self.pending_soffs()
        for m0, ld in self.dma_first(0) + self.dma_second(0):
            self.e(m0)
            self.e(ld)
        self.advance_pending()
        for m0, ld in self.dma_first(1) + self.dma_second(1):
            self.e(m0)
            self.e(ld)
        self.advance_pending()
        for i in range(64):
            self.e(f"v_accvgpr_write_b32 a{QA_DQ + i}, 0")
        self.mask_setup()
        self.e("s_waitcnt vmcnt(8)")
        self.e(f"v_mul_f32 v{QV_NLC}, s{qarg('c')}, v{QV_NLC}")
        for i in range(16):
            self.e(f"v_mov_b32 v{QV_NDSET + i}, v{QV_ND}")
        self.e("s_barrier")
        for m in range(QLA):
            for txt in self.ring_reads(0, m):
                self.e(txt)
        self.e("s_waitcnt lgkmcnt(0)")
        self.e("s_nop 4")

    def text(self):
        self.lines = []
        labs = [self.newlab(f"tile{b}") for b in range(3)]
        lexit = self.newlab("exit")
        self.prologue(lexit)
        self.in_loop = True
        for b in range(3):
            self.lab(labs[b])
            self.emit_body(b, labs[(b + 1) % 3], lexit)
        self.in_loop = False
        self.lab(lexit)
        self.exit()
        n = self.name
        head = ["\t.text", f"\t.globl {n}", "\t.p2align 8", f"\t.type {n},@function", f"{n}:"]
        tail = [
            f".L{n}_end:", f"\t.size {n}, .L{n}_end-{n}", "\t.rodata", "\t.p2align 6",
            f"\t.amdhsa_kernel {n}",
            f"\t\t.amdhsa_group_segment_fixed_size {QLDS_BYTES}",
            "\t\t.amdhsa_private_segment_fixed_size 0",
            f"\t\t.amdhsa_kernarg_size {ARGS_SIZE}",
            "\t\t.amdhsa_user_sgpr_count 2",
            "\t\t.amdhsa_user_sgpr_kernarg_segment_ptr 1",
            "\t\t.amdhsa_system_sgpr_workgroup_id_x 1",
            "\t\t.amdhsa_system_vgpr_workitem_id 0",
            f"\t\t.amdhsa_next_free_vgpr {QNV + QNA}",
            f"\t\t.amdhsa_next_free_sgpr {Q_NSGPR}",
            f"\t\t.amdhsa_accum_offset {QNV}",
            "\t\t.amdhsa_reserve_vcc 1",
            "\t\t.amdhsa_float_denorm_mode_32 3",
            "\t\t.amdhsa_float_denorm_mode_16_64 3",
            "\t\t.amdhsa_ieee_mode 0",
            "\t\t.amdhsa_dx10_clamp 1",
            "\t.end_amdhsa_kernel",
            "\t.text",
        ]
        return "\n".join(head + self.lines + tail) + "\n"

    def metadata(self):
        return super().metadata().replace(f"group_segment_fixed_size: {LDS_BYTES}",
                                          f"group_segment_fixed_size: {QLDS_BYTES}") \
            .replace(f".vgpr_count:     {NV + NA}", f".vgpr_count:     {QNV + QNA}") \
            .replace(f".agpr_count:     {NA}", f".agpr_count:     {QNA}")



# =================================================================================================
# Forward kernel (`fa_fwd`): O = softmax(Q·Kᵀ·scale)·V with the row log-sum-exp
# =================================================================================================
# Two workgroups per CU (≤ 256 registers per lane, 64 KiB LDS each): the co-resident wave issues
# its MFMAs while this wave runs the softmax block, so no cross-tile software pipeline is needed.
# workgroup = 128 queries of one (batch, q-head), 4 waves × 32 queries on the MFMA lanes; per
# 64-key tile: Sᵀ = K·Qᵀ (16 MFMAs, B = Q fragments in AGPRs), row max over the lane's 32 keys +
# the partner half-wave's (v_permlane32_swap), lazy rescale (the running max moves only when a
# tile max exceeds it by more than 8 in log2 units — an out-of-line block that rescales O and l),
# P = exp2(c·s − m), Oᵀ += Vᵀ·P (16 MFMAs, A = transposed V reads). Causal diagonal tiles (the
# last two of an item) mask s > query to −inf before the max. Item end: l summed over the two
# half-waves, O·(1/l) stored bf16, lse = (m + log2 l)·ln 2.
# Arguments: DQ_ARGS with dq → o (output), nl → lse (output, f32 [B, Hq, Sq]), dout / nd unused.
F_V_DK, F_V_DV = 2, 6
F_V_ROW, F_V_TR = 10, 18
F_V_QL, F_V_THR, F_V_NINF, F_V_M, F_V_L, F_V_NM = 26, 27, 28, 29, 30, 31
F_V_T = 32                           # temps v32..v35
F_V_RING = 36                        # 8 slots × 4
F_RING = 8
F_V_SACC = 68                        # Sᵀ accumulators [kb 2][16] (epilogue temps at item end)
F_V_PF = 100                         # P bf16 fragments [ks 4][4]
F_V_QV, F_V_STO, F_V_LSEV, F_V_L4H = 116, 117, 118, 119    # … and l32 − 4hh
F_NV = 120
F_A_O, F_A_QF, F_A_QN = 0, 64, 96
F_NA = 128
F_BUF_B = 32768
F_LDS_BYTES = 2 * F_BUF_B
F_LA = int(os.environ.get("PIAMD_FA_FLA", "4"))  # forward ring lookahead
LN2 = 0.6931471805599453


class FaFwd(FaDq):
    NM = 32
    VTMP_UDIV = F_V_T + 3
    NWV = 4          # waves per workgroup (8: 256 queries share every K/V tile, one WG per CU)
    PPW = 4          # LDS-DMA pieces (1 KiB) per wave per 16 KiB image

    # -- work items ----------------------------------------------------------------------------------
    def q_load_f(self, aq, sq):
        for kk in range(8):
            self.e(f"buffer_load_dwordx4 a[{aq + 4 * kk}:{aq + 4 * kk + 3}], v{F_V_QV}, s[{QSRD_Q}:{QSRD_Q + 3}], s{sq} offen offset:{32 * kk}")

    def compute_item_setup(self):
        T = Q_T
        self.decode(Q_U, T, Q_B, Q_HQ)
        self.e(f"s_lshl_b32 s{Q_Q0}, s{T}, {self.QSH}")
        self.tiles_of(Q_TOT, T)
        self.e(f"s_mov_b32 s{Q_IT}, 0")
        self.q_soffs(T, Q_B, Q_HQ, Q_SOFFQ, Q_SOFFO, Q_SOFFS)
        self.e(f"s_lshl_b32 s{T}, s{Q_W}, 5")
        self.e(f"s_add_u32 s{T}, s{T}, s{Q_Q0}")
        self.e(f"v_add_u32 v{F_V_QL}, s{T}, v{F_V_L4H}")

    def prefetch_next(self):
        T = Q_T
        skip = self.newlab("nopf")
        self.e(f"s_mov_b32 s{T + 3}, s{Q_U}")
        self.next_item(T + 3)
        self.e(f"s_cmp_ge_u32 s{T + 3}, s{qarg('nitems')}")
        self.e(f"s_cbranch_scc1 {skip}")
        self.decode(T + 3, T, T + 1, T + 2)
        self.q_soffs(T, T + 1, T + 2, T + 3, T + 4, T + 6)
        self.q_load_f(F_A_QN, T + 3)
        self.lab(skip)

    def dma_first(self, buf):
        base = buf * F_BUF_B
        return [[f"s_add_u32 m0, s{Q_LDSW}, {base + i * 1024}\n\ts_nop 0",
                 f"buffer_load_dwordx4 v{F_V_DK + i}, s[{QSRD_K}:{QSRD_K + 3}], s{Q_SK} offen lds"]
                for i in range(self.PPW)]

    def dma_second(self, buf):
        base = buf * F_BUF_B + Q_OFF_V
        return [[f"s_add_u32 m0, s{Q_LDSW}, {base + i * 1024}\n\ts_nop 0",
                 f"buffer_load_dwordx4 v{F_V_DV + i}, s[{QSRD_V}:{QSRD_V + 3}], s{Q_SV} offen lds"]
                for i in range(self.PPW)]

    # -- MFMA stream ------------------------------------------------------------------------------------
    @staticmethod
    def mfma_kind(m):
        if m < 16:
            return ("S", m // 8, m % 8)
        c = m - 16
        return ("O", c % 4, c // 4)                                  # (dt, ks)

    @staticmethod
    def slot(b, m):
        return F_V_RING + 4 * ((32 * b + m) % F_RING)

    def ring_reads(self, b, m):
        kind, x, y = self.mfma_kind(m)
        d = self.slot(b, m)
        base = b * F_BUF_B
        if kind == "S":
            kb, kk = x, y
            return [f"ds_read_b128 v[{d}:{d + 3}], v{F_V_ROW + kk} offset:{base + kb * 8192}"]
        dt, ks = x, y
        off = base + Q_OFF_V + ks * 16 * 256
        return [f"ds_read_b64_tr_b16 v[{d + 2 * jj}:{d + 2 * jj + 1}], v{F_V_TR + 4 * jj + dt} offset:{off}"
                for jj in (0, 1)]

    def mfma_text(self, b, m):
        kind, x, y = self.mfma_kind(m)
        a = self.slot(b, m)
        if kind == "S":
            kb, kk = x, y
            acc = F_V_SACC + 16 * kb
            src = "0" if kk == 0 else f"v[{acc}:{acc + 15}]"
            return f"{MFMA} v[{acc}:{acc + 15}], v[{a}:{a + 3}], a[{F_A_QF + 4 * kk}:{F_A_QF + 4 * kk + 3}], {src}"
        dt, ks = x, y
        acc = F_A_O + 16 * dt
        return f"{MFMA} a[{acc}:{acc + 15}], v[{a}:{a + 3}], v[{F_V_PF + 4 * ks}:{F_V_PF + 4 * ks + 3}], a[{acc}:{acc + 15}]"

    def softmax_block(self, lab_resc, lab_back):
        """After the 16 S MFMAs: mask (diagonal tiles), row max, lazy rescale test, P = exp2(c·s −
        m) and the bf16 P fragments. The l partial sum is left for the O-phase gaps."""
        T = Q_T
        S = F_V_SACC
        t = F_V_T
        self.e("s_nop 15")                                             # MFMA result → VALU
        self.e("s_nop 15")
        if self.causal:   # the item's last key tiles cross the diagonal
            skip = self.newlab("nomask")
            self.e(f"s_sub_u32 s{T}, s{Q_TOT}, {1 << (self.QSH - 6)}")
            self.e(f"s_cmp_lt_i32 s{Q_IT}, s{T}")
            self.e(f"s_cbranch_scc1 {skip}")
            self.e(f"s_lshl_b32 s{T}, s{Q_IT}, 6")
            self.e(f"v_subrev_u32 v{F_V_THR}, s{T}, v{F_V_QL}")         # q − 4hh − 64 kt
            for kb in (0, 1):
                for g4 in range(4):
                    for e in range(4):
                        ci = 32 * kb + 8 * g4 + e
                        r = S + 16 * kb + 4 * g4 + e
                        self.e(f"v_cmp_gt_i32 vcc, {ci}, v{F_V_THR}")
                        self.e(f"v_cndmask_b32 v{r}, v{r}, v{F_V_NINF}, vcc")
            self.lab(skip)
        # row max over the lane's 32 keys (max3 tree), then the partner half-wave's
        regs = list(range(S, S + 32))
        self.e(f"v_max3_f32 v{t}, v{regs[0]}, v{regs[1]}, v{regs[2]}")
        self.e(f"v_max3_f32 v{t + 1}, v{regs[3]}, v{regs[4]}, v{regs[5]}")
        k = 6
        while k + 1 < 32:
            acc = t + (k // 2) % 2
            self.e(f"v_max3_f32 v{acc}, v{acc}, v{regs[k]}, v{regs[k + 1]}")
            k += 2
        self.e(f"v_max_f32 v{t}, v{t}, v{t + 1}")
        self.e(f"v_mov_b32 v{t + 1}, v{t}")
        self.e("s_nop 1")
        self.e(f"v_permlane32_swap_b32 v{t}, v{t + 1}")
        self.e("s_nop 1")
        self.e(f"v_max_f32 v{t}, v{t}, v{t + 1}")
        self.e(f"v_mul_f32 v{t}, s{qarg('c')}, v{t}")                   # tile row max (log2 units)
        self.e(f"v_add_f32 v{t + 1}, 0x41000000, v{F_V_M}")              # m + 8
        self.e(f"v_cmp_gt_f32 vcc, v{t}, v{t + 1}")
        self.e(f"s_cbranch_vccnz {lab_resc}")
        self.lab(lab_back)
        # −m (0 while the row has seen only masked keys)
        self.e(f"v_cmp_eq_f32 vcc, v{F_V_NINF}, v{F_V_M}")
        self.e(f"v_cndmask_b32_e64 v{F_V_NM}, -v{F_V_M}, 0, vcc")
        for r in regs:
            self.e(f"v_fma_f32 v{r}, v{r}, s{qarg('c')}, v{F_V_NM}")
        for r in regs:
            self.e(f"v_exp_f32 v{r}, v{r}")
        self.e("s_nop 0")
        for kb in (0, 1):
            for j in range(8):
                fr = 4 * (2 * kb + j // 4) + j % 4
                a = S + 16 * kb + 2 * j
                self.e(f"v_cvt_pk_bf16_f32 v{F_V_PF + fr}, v{a}, v{a + 1}")

    def rescale_block(self, lab_resc, lab_back):
        """Out of line: m ← tile max where it grew by > 8; O, l ← O·α, l·α with α = exp2(m_old −
        m_new) (α = 1 on the other lanes)."""
        t = F_V_T
        self.lab(lab_resc)
        self.e(f"v_cndmask_b32 v{t + 1}, v{F_V_M}, v{t}, vcc")         # m_new
        self.e(f"v_cmp_eq_f32 vcc, v{F_V_NINF}, v{F_V_M}")
        self.e(f"v_sub_f32 v{t + 2}, v{F_V_M}, v{t + 1}")
        self.e(f"v_exp_f32 v{t + 2}, v{t + 2}")
        self.e("s_nop 0")
        self.e(f"v_cndmask_b32 v{t + 2}, v{t + 2}, 0, vcc")           # first tile: α = 0 (O = 0)
        self.e(f"v_mul_f32 v{F_V_L}, v{F_V_L}, v{t + 2}")
        self.e(f"v_mov_b32 v{F_V_M}, v{t + 1}")
        self.e("s_nop 7")
        tmp = [t + 3, F_V_NM, F_V_PF, F_V_PF + 1]     # free here; rotated so no read follows its write
        for i0 in range(0, 64, 4):
            for j in range(4):
                self.e(f"v_accvgpr_read_b32 v{tmp[j]}, a{F_A_O + i0 + j}")
            for j in range(4):
                self.e(f"v_mul_f32 v{tmp[j]}, v{tmp[j]}, v{t + 2}")
            self.e("s_nop 1")
            for j in range(4):
                self.e(f"v_accvgpr_write_b32 a{F_A_O + i0 + j}, v{tmp[j]}")
        self.e("s_nop 4")
        self.e(f"s_branch {lab_back}")

    def lsum_ops(self):
        S = F_V_SACC
        ops = []
        # pairwise tree of the 32 P values into v{S}, then l += it
        n = 32
        step = 1
        while step < n:
            for i in range(0, n, 2 * step):
                ops.append(f"v_add_f32 v{S + i}, v{S + i}, v{S + i + step}")
            step *= 2
        ops.append(f"v_add_f32 v{F_V_L}, v{F_V_L}, v{S}")
        return ops

    def body_ops(self, b):
        nb = (b + 1) % 2
        NM = self.NM
        gaps = [[] for _ in range(NM)]
        for m in range(NM):
            g = m - F_LA
            if g >= 0:
                for t in self.ring_reads(b, m):
                    gaps[g].append(("lds", ("ring", 0, m), t))
        for m in range(F_LA):
            g = NM - F_LA + m
            for t in self.ring_reads(nb, m):
                gaps[g].append(("lds", ("ring", 1, m), t))
        # the DMA of tile t+1 into the other buffer (free: every wave passed this body's start
        # barrier, so the previous tile is consumed), cursor advance
        dgap = int(os.environ.get("PIAMD_FA_FWD_DMA_GAP", "1"))   # schedule sweeps (measurement)
        for i, (m0, ld) in enumerate(self.dma_first(nb) + self.dma_second(nb)):
            gaps[i * dgap] += [("txt", m0), ("txt", ld)]
        gaps[8 * dgap].append(("adv",))
        # tile t+1 landed before its K rows are read (the lookahead reads start at gap NM−LA)
        gaps[NM - F_LA - 1].append(("txt", "s_waitcnt vmcnt(0)"))
        gaps[NM - F_LA - 1].append(("txt", "s_barrier"))
        gaps[15].append(("softmax",))
        ls = [] if "novalu" in ABL else self.lsum_ops()
        for i, op in enumerate(ls):
            gaps[16 + (i * 14) // len(ls)].append(("txt", op))
        ops = [("txt", "s_barrier")]
        for m in range(NM):
            ops.append(("mfma", m, [("ring", 0, m)], self.mfma_text(b, m)))
            ops += gaps[m]
        return ops

    def emit_body(self, b, lab_next, lab_epi):
        prev = self.body_ops((b + 1) % 2)
        cur = self.body_ops(b)
        order = []
        for ent in prev:
            if ent[0] == "lds":
                kind, t, idx = ent[1]
                order.append((kind, t - 1, idx))
        pos = {k: i for i, k in enumerate(order)}
        done = 0
        issued = len(order)
        resc, back = self.newlab("resc"), self.newlab("back")
        for ent in cur:
            if ent[0] == "lds":
                pos[ent[1]] = issued
                issued += 1
                self.e(ent[2])
            elif ent[0] == "mfma":
                need = max(pos[d] for d in ent[2])
                if need >= done:
                    w = min(15, issued - 1 - need)
                    self.e(f"s_waitcnt lgkmcnt({w})")
                    done = issued - w
                self.e(ent[3])
            elif ent[0] == "adv":
                self.advance_pending()
            elif ent[0] == "softmax":
                if "novalu" not in ABL:   # measurement only
                    self.softmax_block(resc, back)
                else:
                    self.lab(back)
            else:
                self.e(ent[1])
        self.e(f"s_add_u32 s{Q_IT}, s{Q_IT}, 1")
        nopf = self.newlab("nopf")
        self.e(f"s_cmp_eq_u32 s{Q_IT}, 1")
        self.e(f"s_cbranch_scc0 {nopf}")
        self.prefetch_next()
        self.lab(nopf)
        self.e(f"s_cmp_lt_u32 s{Q_IT}, s{Q_TOT}")
        self.e(f"s_cbranch_scc1 {lab_next}")
        self.item_end(lab_next, lab_epi)
        self.rescale_block(resc, back)

    def store_o(self):
        """l over both half-waves, O·(1/l) → bf16 o[q][d], lse = (m + log2 l)·ln 2."""
        t = F_V_T
        S = F_V_SACC
        self.e(f"v_mov_b32 v{t}, v{F_V_L}")
        self.e(f"v_mov_b32 v{t + 1}, v{F_V_L}")
        self.e("s_nop 1")
        self.e(f"v_permlane32_swap_b32 v{t}, v{t + 1}")
        self.e("s_nop 1")
        self.e(f"v_add_f32 v{t}, v{t}, v{t + 1}")                      # l
        self.e(f"v_rcp_f32 v{t + 1}, v{t}")
        self.e(f"v_log_f32 v{t + 2}, v{t}")
        self.e("s_nop 0")
        self.e(f"v_cmp_lt_f32 vcc, 0, v{t}")
        self.e(f"v_cndmask_b32 v{t + 1}, 0, v{t + 1}, vcc")            # 1/l (0 for an empty row)
        self.e(f"v_add_f32 v{t + 2}, v{F_V_M}, v{t + 2}")
        self.e(f"v_mul_f32 v{t + 2}, {fhex(LN2)}, v{t + 2}")
        self.e(f"v_mov_b32 v{t + 3}, 0x7f800000")
        self.e(f"v_cndmask_b32 v{t + 2}, v{t + 3}, v{t + 2}, vcc")     # +inf for an empty row
        self.e(f"buffer_store_dword v{t + 2}, v{F_V_LSEV}, s[{QSRD_NL}:{QSRD_NL + 3}], s{Q_SOFFS} offen")
        for dt in range(4):
            for g4 in range(4):
                a0 = F_A_O + 16 * dt + 4 * g4
                for j in range(4):
                    self.e(f"v_accvgpr_read_b32 v{S + j}, a{a0 + j}")
                for j in range(4):
                    self.e(f"v_mul_f32 v{S + j}, v{S + j}, v{t + 1}")
                self.e(f"v_cvt_pk_bf16_f32 v{S}, v{S}, v{S + 1}")
                self.e(f"v_cvt_pk_bf16_f32 v{S + 1}, v{S + 2}, v{S + 3}")
                self.e(f"buffer_store_dwordx2 v[{S}:{S + 1}], v{F_V_STO}, s[{QSRD_DQ}:{QSRD_DQ + 3}], s{Q_SOFFO} offen offset:{64 * dt + 16 * g4}")

    def item_end(self, lab_next, lab_exit):
        self.e("s_nop 15")
        self.e("s_nop 15")
        self.store_o()
        for i in range(64):
            self.e(f"v_accvgpr_write_b32 a{F_A_O + i}, 0")
        for i in range(32):
            self.e(f"v_accvgpr_mov_b32 a{F_A_QF + i}, a{F_A_QN + i}")
        self.e(f"v_mov_b32 v{F_V_M}, v{F_V_NINF}")
        self.e(f"v_mov_b32 v{F_V_L}, 0")
        self.next_item(Q_U)
        self.e(f"s_cmp_ge_u32 s{Q_U}, s{qarg('nitems')}")
        self.e(f"s_cbranch_scc1 {lab_exit}")
        self.compute_item_setup()
        self.e("s_nop 4")
        self.e(f"s_branch {lab_next}")

    def prologue(self, lab_exit):
        T = Q_T
        self.e("s_load_dwordx16 s[4:19], s[0:1], 0x0")
        self.e("s_load_dwordx16 s[20:35], s[0:1], 0x40")
        self.e("s_load_dwordx16 s[36:51], s[0:1], 0x80")
        self.e(f"v_and_b32 v{V_LANE}, 63, v{V_TID}")
        self.e(f"v_lshrrev_b32 v{F_V_T}, 6, v{V_TID}")
        self.e("s_waitcnt lgkmcnt(0)")
        self.srd(QSRD_K, qarg("k"), qarg("k_bytes"))
        self.srd(QSRD_V, qarg("v"), qarg("v_bytes"))
        self.srd(QSRD_Q, qarg("q"), qarg("q_bytes"))
        self.srd(QSRD_DQ, qarg("dq"), qarg("o_bytes"))             # O (output)
        self.srd(QSRD_NL, qarg("nl"), qarg("st_bytes"))            # lse (output)
        self.e(f"v_readfirstlane_b32 s{Q_W}, v{F_V_T}")
        self.e(f"s_lshl_b32 s{Q_LDSW}, s{Q_W}, {10 + self.PPW.bit_length() - 1}")
        self.e(f"s_and_b32 s{Q_U}, s{S_WG}, 7")
        self.e(f"s_lshr_b32 s{T}, s{qarg('G')}, 3")
        self.e(f"s_mul_i32 s{Q_U}, s{Q_U}, s{T}")
        self.e(f"s_lshr_b32 s{T}, s{S_WG}, 3")
        self.e(f"s_add_u32 s{Q_U}, s{Q_U}, s{T}")
        self.e(f"s_lshl_b32 s{Q_U}, s{Q_U}, 1")
        self.e(f"s_cmp_ge_u32 s{Q_U}, s{qarg('nitems')}")
        self.e(f"s_cbranch_scc1 {lab_exit}")
        L = V_LANE
        t = F_V_T
        # t: l32, t+1: hh, t+2: l32 − 4hh (kept for the items), t+3: scratch
        self.e(f"v_and_b32 v{t}, 31, v{L}")
        self.e(f"v_lshrrev_b32 v{t + 1}, 5, v{L}")
        self.e(f"s_lshl_b32 s{T}, s{Q_W}, 5")
        self.e(f"v_add_u32 v{t + 3}, s{T}, v{t}")                  # 32w + l32
        self.e(f"v_lshlrev_b32 v{F_V_THR}, 4, v{t + 1}")            # 16hh
        self.e(f"v_mad_u32_u24 v{F_V_QV}, v{t + 3}, s{qarg('sqs')}, v{F_V_THR}")
        self.e(f"v_lshlrev_b32 v{F_V_THR}, 3, v{t + 1}")            # 8hh
        self.e(f"v_mad_u32_u24 v{F_V_STO}, v{t + 3}, s{qarg('sos')}, v{F_V_THR}")
        self.e(f"v_lshlrev_b32 v{F_V_LSEV}, 2, v{t + 3}")           # 4·(32w + l32)
        self.e(f"v_lshlrev_b32 v{F_V_THR}, 2, v{t + 1}")
        self.e(f"v_sub_u32 v{F_V_L4H}, v{t}, v{F_V_THR}")           # l32 − 4hh
        self.e(f"v_mov_b32 v{F_V_NINF}, 0xff800000")
        self.e(f"v_mov_b32 v{F_V_M}, v{F_V_NINF}")
        self.e(f"v_mov_b32 v{F_V_L}, 0")
        # scratch for the offset set-up: S accumulator registers (free until the first tile)
        # LDS-DMA: piece P = PPW·w + i holds image rows 4P + g (g = lane >> 4), physical chunk
        # lane & 15 = logical chunk ^ x(row), x = (g << 2) | (P & 3)
        x = F_V_SACC
        self.e(f"v_lshrrev_b32 v{x + 3}, 4, v{L}")
        self.e(f"v_and_b32 v{x + 4}, 15, v{L}")
        self.e(f"s_mul_i32 s{T}, s{Q_W}, {4 * self.PPW}")
        self.e(f"v_add_u32 v{x + 5}, s{T}, v{x + 3}")
        self.e(f"s_mul_i32 s{T + 1}, s{Q_W}, {self.PPW}")
        for i in range(self.PPW):
            self.e(f"s_add_u32 s{T + 2}, s{T + 1}, {i}")
            self.e(f"s_and_b32 s{T + 2}, s{T + 2}, 3")
            self.e(f"v_lshl_or_b32 v{x + 6}, v{x + 3}, 2, s{T + 2}")
            self.e(f"v_xor_b32 v{x + 6}, v{x + 6}, v{x + 4}")
            self.e(f"v_lshlrev_b32 v{x + 6}, 4, v{x + 6}")
            self.e(f"v_add_u32 v{x + 2}, {4 * i}, v{x + 5}")
            self.e(f"v_mad_u32_u24 v{F_V_DK + i}, v{x + 2}, s{qarg('sks')}, v{x + 6}")
            self.e(f"v_mad_u32_u24 v{F_V_DV + i}, v{x + 2}, s{qarg('svs')}, v{x + 6}")
        self.e(f"v_and_b32 v{x + 3}, 3, v{t}")
        self.e(f"v_lshlrev_b32 v{x + 3}, 2, v{x + 3}")
        self.e(f"v_bfe_u32 v{x + 4}, v{t}, 2, 2")
        self.e(f"v_or_b32 v{x + 3}, v{x + 3}, v{x + 4}")
        self.e(f"v_lshlrev_b32 v{x + 4}, 8, v{t}")
        for kk in range(8):
            self.e(f"v_add_u32 v{x + 5}, {2 * kk}, v{t + 1}")
            self.e(f"v_xor_b32 v{x + 5}, v{x + 5}, v{x + 3}")
            self.e(f"v_lshl_add_u32 v{F_V_ROW + kk}, v{x + 5}, 4, v{x + 4}")
        self.e(f"v_and_b32 v{x + 3}, 15, v{L}")
        self.e(f"v_lshrrev_b32 v{x + 4}, 2, v{x + 3}")
        self.e(f"v_lshl_add_u32 v{x + 4}, v{t + 1}, 2, v{x + 4}")
        self.e(f"v_and_b32 v{x + 5}, 3, v{x + 3}")
        self.e(f"v_lshlrev_b32 v{x + 5}, 2, v{x + 5}")
        self.e(f"v_bfe_u32 v{x + 6}, v{L}, 4, 1")
        self.e(f"v_lshl_add_u32 v{x + 5}, v{x + 6}, 4, v{x + 5}")
        for jj in (0, 1):
            self.e(f"v_add_u32 v{x + 6}, {8 * jj}, v{x + 4}")
            self.e(f"v_and_b32 v{x + 7}, 3, v{x + 6}")
            self.e(f"v_lshlrev_b32 v{x + 7}, 2, v{x + 7}")
            self.e(f"v_bfe_u32 v{x + 2}, v{x + 6}, 2, 2")
            self.e(f"v_or_b32 v{x + 7}, v{x + 7}, v{x + 2}")
            self.e(f"v_lshrrev_b32 v{x + 2}, 3, v{x + 5}")
            self.e(f"v_xor_b32 v{x + 7}, v{x + 7}, v{x + 2}")
            self.e(f"v_lshlrev_b32 v{x + 7}, 4, v{x + 7}")
            self.e(f"v_lshl_add_u32 v{x + 7}, v{x + 6}, 8, v{x + 7}")
            self.e(f"v_and_b32 v{x + 2}, 7, v{x + 5}")
            self.e(f"v_lshl_add_u32 v{x + 7}, v{x + 2}, 1, v{x + 7}")
            for dt in range(4):
                self.e(f"v_xor_b32 v{F_V_TR + 4 * jj + dt}, {dt << 6}, v{x + 7}")
        self.compute_item_setup()
        self.q_load_f(F_A_QF, Q_SOFFQ)
        self.e(f"s_mov_b32 s{Q_DU}, s{Q_U}")
        self.pending_item_setup()
        self.pending_soffs()
        for m0, ld in self.dma_first(0) + self.dma_second(0):
            self.e(m0)
            self.e(ld)
        self.advance_pending()
        for i in range(64):
            self.e(f"v_accvgpr_write_b32 a{F_A_O + i}, 0")
        self.e("s_waitcnt vmcnt(0)")
        self.e("s_barrier")
        for m in range(F_LA):
            for txt in self.ring_reads(0, m):
                self.e(txt)
        self.e("s_waitcnt lgkmcnt(0)")
        self.e("s_nop 4")

    def text(self):
        self.lines = []
        labs = [self.newlab(f"tile{b}") for b in range(2)]
        lexit = self.newlab("exit")
        self.prologue(lexit)
        self.in_loop = True
        for b in range(2):
            self.lab(labs[b])
            self.emit_body(b, labs[(b + 1) % 2], lexit)
        self.in_loop = False
        self.lab(lexit)
        self.exit()
        n = self.name
        head = ["\t.text", f"\t.globl {n}", "\t.p2align 8", f"\t.type {n},@function", f"{n}:"]
        tail = [
            f".L{n}_end:", f"\t.size {n}, .L{n}_end-{n}", "\t.rodata", "\t.p2align 6",
            f"\t.amdhsa_kernel {n}",
            f"\t\t.amdhsa_group_segment_fixed_size {F_LDS_BYTES}",
            "\t\t.amdhsa_private_segment_fixed_size 0",
            f"\t\t.amdhsa_kernarg_size {ARGS_SIZE}",
            "\t\t.amdhsa_user_sgpr_count 2",
            "\t\t.amdhsa_user_sgpr_kernarg_segment_ptr 1",
            "\t\t.amdhsa_system_sgpr_workgroup_id_x 1",
            "\t\t.amdhsa_system_vgpr_workitem_id 0",
            f"\t\t.amdhsa_next_free_vgpr {F_NV + F_NA}",
            f"\t\t.amdhsa_next_free_sgpr {Q_NSGPR}",
            f"\t\t.amdhsa_accum_offset {F_NV}",
            "\t\t.amdhsa_reserve_vcc 1",
            "\t\t.amdhsa_float_denorm_mode_32 3",
            "\t\t.amdhsa_float_denorm_mode_16_64 3",
            "\t\t.amdhsa_ieee_mode 0",
            "\t\t.amdhsa_dx10_clamp 1",
            "\t.end_amdhsa_kernel",
            "\t.text",
        ]
        return "\n".join(head + self.lines + tail) + "\n"

    def metadata(self):
        return FaDkdv.metadata(self).replace(f"group_segment_fixed_size: {LDS_BYTES}",
                                             f"group_segment_fixed_size: {F_LDS_BYTES}") \
            .replace(f".vgpr_count:     {NV + NA}", f".vgpr_count:     {F_NV + F_NA}") \
            .replace(f".agpr_count:     {NA}", f".agpr_count:     {F_NA}") \
            .replace(".max_flat_workgroup_size: 256", f".max_flat_workgroup_size: {64 * self.NWV}")


class FaFwd8(FaFwd):
    """Eight waves (256 queries) per workgroup, one workgroup per CU: every K/V tile DMA'd into LDS
    feeds twice the queries (half the L2→LDS and HBM traffic per query of the 4-wave kernel);
    two waves per SIMD still overlap one wave's softmax with the other's MFMAs."""
    NWV = 8
    PPW = 2
    QSH = 8


def kernels():
    return [FaDkdv("piamd_fa_dkdv_d128_causal", True), FaDkdv("piamd_fa_dkdv_d128", False),
            FaDq("piamd_fa_dq_d128_causal", True), FaDq("piamd_fa_dq_d128", False),
            FaFwd("piamd_fa_fwd_d128_causal", True), FaFwd("piamd_fa_fwd_d128", False),
            FaFwd8("piamd_fa_fwd8_d128_causal", True), FaFwd8("piamd_fa_fwd8_d128", False)]


def generate() -> str:
    ks = kernels()
    out = ['\t.amdgcn_target "amdgcn-amd-amdhsa--gfx950"', "\t.amdhsa_code_object_version 5"]
    for k in ks:
        out.append(k.text())
    out.append("\t.amdgpu_metadata\n---\namdhsa.kernels:")
    for k in ks:
        out.append(k.metadata().rstrip("\n"))
    out.append("amdhsa.target:   amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n\t.end_amdgpu_metadata")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    text = generate()
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(text)
    else:
        sys.stdout.write(text)
