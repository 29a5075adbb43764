"""Generator of the hand-scheduled gfx950 (CDNA4) bf16 GEMM kernels (``agemm``).

Why assembly: the GEMMs are ~75 % of a GPT training step. The structure that reaches the MFMA
rate on gfx950 — ONE wave per SIMD holding a 128×128 f32 accumulator tile in the 256 AGPRs, all
64-deep operand fragments of a K-block (128 VGPRs) in registers, LDS filled by LDS-DMA
(`buffer_load_dwordx4 … lds`) two blocks ahead into the stage that is being consumed — cannot be
expressed through hipcc: with 512 live registers per lane hipcc either spills or re-orders the
MFMA/DMA/LDS-read interleave and inserts drains (the round-2 HIP kernel `gemm_pipe.hip` reached
0.77-0.87× hipBLASLt, `profiles/gemm_pipe_r2.txt`). Here every instruction is placed by this
generator and every wait is counted by hand.

Kernel (one per (A layout, B layout, epilogue) variant):

* C[M,N] = A·B, bf16 operands, f32 accumulation. A is KC ("K-contiguous", stored [M][K]) or MC
  (stored [K][M]); B is KC (stored [N][K]) or MC (stored [K][N]). Forward and data-gradient
  products of a linear are KC×KC; the weight gradient xᵀ·dy is MC×MC — no transpose kernels.
* workgroup = 4 waves (one per SIMD), 256×256 output tile, wave (wr, wc) owns 128×128 =
  8×8 blocks of `v_mfma_f32_16x16x32_bf16` (operands swapped, Cᵀ-blocks = B·A, so a lane owns
  one output row and 4 consecutive columns: 8-byte bf16 / 16-byte f32 stores).
* K-block = 64. LDS = 2 stages × (A 32 KiB + B 32 KiB) = 128 KiB. Block t lives in stage t%2.
  Iteration t: phase A runs the 64 MFMAs of k-half 0 (fragments X, read during the previous
  iteration) while reading k-half 1 (fragments Y); a barrier then certifies every wave has ALL of
  block t in registers, so phase B issues the 16 LDS-DMAs of block t+2 into the SAME stage while
  running the 64 MFMAs of k-half 1, waits (counted `vmcnt(16)`) for block t+1, barriers, and reads
  its k-half 0 into X. Two barriers per 128 MFMAs; DMA latency budget ≈1.5 iterations.
* LDS images: KC operand = [256 rows][128 B], 16-B chunk c of row r at c ^ ((r>>1)&7)
  (conflict-free `ds_read_b128` for the MFMA lane groups); MC operand = 4 column groups of
  64 × [64 k][128 B] with the 32-B slot XOR ((k>>1)&1 | ((k>>3)&1)<<1) — conflict-free
  `ds_read_b64_tr_b16` (hardware transpose). LDS-DMA writes are lane-linear, so the swizzle sits
  on the per-lane GLOBAL source address; every DMA moves whole 128-B lines.
* Work mapping: bijective XCD remap (blocks b, b+8, … share an XCD and take consecutive tiles),
  group-M tile order (GM m-tiles × all n-tiles), optional split-K (f32 partial planes, reduced by
  `splitk_reduce` in a fixed order).
* Epilogues: bf16 store, f32 store (split-K partials), f32 accumulate (main_grad += ),
  bias + activation with the pre-activation stored as aux (FFN1 forward), C = acc ⊙ act'(aux)
  (FFN2 data gradient fused with the GELU backward). Rows beyond M fall outside the store
  descriptor's range (dropped by the buffer unit); columns beyond N are EXEC-masked.

Every global access is a `buffer_*` op through a descriptor whose range is the operand's extent,
and every address is clamped in range by construction.

Parity: reference `paddle/phi/kernels/funcs/blas/blas_impl.cu.h` (cublas GEMM behind matmul /
linear and their gradients), `paddle/fluid/operators/fused/fused_gemm_epilogue_op.cu:30`
(cublasLt bias / bias+GELU(aux) / dGELU epilogues).

``python gemm_gen.py OUT.s`` writes every variant; `_build.py` assembles and links it into
``_lib/piamd_agemm.hsaco`` (loaded by ``csrc/kernels/agemm_host.hip``).
"""
from __future__ import annotations

import os
import sys

TILE, BK, NW = 256, 64, 4
# ablation builds for measurement only (tools/agemm_ablate.py): nodma / noreads / nomfma / nobar
ABL = set(filter(None, os.environ.get("PIAMD_AGEMM_ABL", "").split(",")))
LDS_BYTES = 2 * 2 * 256 * BK * 2  # 2 stages × (A + B) × 256 × 64 × bf16 = 128 KiB
STAGE_BYTES = 65536
OP_BYTES = 32768

# ---- kernel-argument block (byte offsets; mirrored by struct AgemmArgs in agemm_host.hip) ------
ARGS = [
    ("a", 0, 8), ("b", 8, 8), ("a_bytes", 16, 8), ("b_bytes", 24, 8),
    ("lda_b", 32, 4), ("ldb_b", 36, 4), ("M", 40, 4), ("N", 44, 4),
    ("nk", 48, 4), ("tiles_n", 52, 4), ("nwg", 56, 4), ("ksplit", 60, 4),
    ("tiles_m", 64, 4), ("ntiles", 68, 4), ("rcp_ntiles", 72, 4), ("per_group", 76, 4),
    ("rcp_per_group", 80, 4), ("gm", 84, 4), ("act", 88, 4), ("grid", 92, 4),
    # epilogue block (loaded after the main loop)
    ("c", 96, 8), ("c_bytes", 104, 8), ("ldc_b", 112, 4), ("ldaux_b", 116, 4),
    ("c_part", 120, 8), ("aux", 128, 8), ("aux_bytes", 136, 8), ("bias", 144, 8),
    # work-unit "part" decomposition (loaded at each tile setup): K start = part·kmul (split-K:
    # kmul = nk·64; batched: kmul = 0) and operand base += part·{a,b}_bstride bytes (batched)
    ("kmul", 152, 4), ("pad0", 156, 4), ("a_bstride", 160, 8), ("b_bstride", 168, 8),
    # column-sum partials of the fused dact epilogue ("dgelucs"): f32 [ceil(M/128)][N] (one row per
    # 128-row wave band), byte size for the descriptor range
    ("colsum", 176, 8), ("colsum_bytes", 184, 4), ("pad1", 188, 4),
]
ARGS_SIZE = 192

# ---- SGPR map ------------------------------------------------------------------------------------
S_KARG = 0        # s[0:1]
S_WG = 2          # workgroup id
S_ARG = 4         # s[4:27]: the first 96 argument bytes
S_A, S_B, S_ABYTES, S_BBYTES = 4, 6, 8, 10
S_LDA, S_LDB, S_M, S_N = 12, 13, 14, 15
S_NK, S_TN, S_NWG, S_KSPLIT = 16, 17, 18, 19
S_TM, S_NTILES, S_RCPNT, S_PERGRP, S_RCPPG, S_GM, S_ACT, S_GRID = 20, 21, 22, 23, 24, 25, 26, 27
S_SRDA, S_SRDB = 28, 32            # 4 each
S_SOFFA, S_SOFFB = 36, 44          # 8 each (MC operands)
S_REMA, S_REMB = 52, 54            # 64-bit remaining bytes behind the descriptor base
S_STEPA, S_STEPB = 56, 58          # 64-bit K-block step
S_LDSA, S_LDSB = 60, 62            # per-stage LDS-DMA base of this wave's pieces (2 each)
S_LOOP, S_REM = 64, 65
S_WAVE, S_M0T, S_N0T, S_PART = 66, 67, 68, 69
S_T = 70                           # temps s70..s79
S_E = 80                           # epilogue arguments s80..s93 (loaded once)
S_U0, S_ROUND = 94, 95             # persistent: first work unit, round counter
S_CSRD = 96                        # C descriptor (epilogue)
S_AUXSRD, S_BIASSRD = 40, 44       # fused epilogues (K-contiguous operands: no soffsets in use)
# next tile (persistent): argument SGPRs the kernel never reads after the prologue
S_NM0, S_NN0, S_NPART, S_NVALID = 3, 19, 26, 65
NSGPR = 100

# ---- VGPR map ------------------------------------------------------------------------------------
V_TID, V_LANE = 0, 1
V_DMAA, V_DMAB = 2, 10             # 8 each (KC: one per piece row-group; MC: 2)
V_RBA, V_RBB = 18, 26              # read bases, 8 each (KC: [stage][h] 4; MC: [stage][bq] 8)
V_T = 34                           # temps v34..v47
V_FRAG = 48                        # X: A v48..79, B v80..111; Y: A v112..143, B v144..175
# epilogue registers (relative to the epilogue base: the dead fragments of both sets for the
# one-tile kernel, set Y + v176.. for the persistent kernel whose set X already holds the next
# tile's first fragments): +0..7 offsets, +8..39 values, +40..55 aux / old C, +56..71 bias,
# +72..76 temps (+76 even: a 64-bit pair), +80..82 constants
# +84..87 paired-store offsets, +88..91 the aux pair being assembled, +92..101 constant pairs
# (packed f32 math); loads of old C / aux double-buffer in +40..55 / +56..71 (+40..71 / +72..103
# for f32 C)
E_BIAS, E_TMP, E_CONST, E_PAIR, E_AUXP = 56, 72, 92, 84, 88
ACC_OFF = 224                      # AGPRs follow the VGPRs in the unified file
NVGPR = ACC_OFF + 256


K0, K1 = 0.7978845608028654, 0.044715          # gelu_tanh constants (sqrt(2/pi), 0.044715)
TWO_LOG2E = 2.0 * 1.4426950408889634
# exact (erf) GELU: Φ(x) = 1 − q (x ≥ 0) or q (x < 0), q = ½·poly(t)·exp(−x²/2), t = 1/(1 + p·|x|/√2)
# (Abramowitz–Stegun 7.1.26, |error| ≤ 1.5e-7); constant pairs 0 p/√2, 1..3 ½a5, ½a4, ½a3, 4 1.0,
# 5 ½a2, 6 ½a1, 7 −log2(e)/2
ERF_P = 0.3275911 / 2.0 ** 0.5
ERF_A = (0.254829592, -0.284496736, 1.421413741, -1.453152027, 1.061405429)
ERF_CONSTS = (ERF_P, 0.5 * ERF_A[4], 0.5 * ERF_A[3], 0.5 * ERF_A[2], 1.0, 0.5 * ERF_A[1], 0.5 * ERF_A[0],
              -0.5 * 1.4426950408889634)


def fhex(x):
    import struct
    return "0x%08x" % struct.unpack("<I", struct.pack("<f", x))[0]


def frag(set_, op, blk):
    """First VGPR of fragment `blk` of operand `op` (0 = A, 1 = B) in set X (0) / Y (1)."""
    return V_FRAG + set_ * 64 + op * 32 + blk * 4


def acc(mb, nb):
    return 4 * (mb * 8 + nb)


# ---- layout model (shared with tests/test_agemm_layout_cpu.py) ----------------------------------
def kc_dma(i, w, L):
    """KC operand, wave w, DMA i (0..7), lane L → (tile row, global 16-B chunk), LDS byte."""
    row = 32 * i + 8 * w + (L >> 3)
    g = (L & 7) ^ ((4 * w + (L >> 4)) & 7)
    lds = (4 * i + w) * 1024 + 16 * L
    return row, g, lds


def kc_read(WO, h, blk, l):
    """KC fragment read (ds_read_b128): LDS byte of lane l for block blk, k-half h."""
    r = WO + 16 * blk + (l & 15)
    c = (4 * h + (l >> 4)) ^ ((l >> 1) & 7)
    return r * 128 + c * 16


def mc_f(k):
    return ((k >> 1) & 1) | (((k >> 3) & 1) << 1)


def mc_dma(i, w, L):
    """MC operand ([K][cols]), wave w, DMA i, lane L → (k row, first col), LDS byte."""
    k = 8 * i + (L >> 3)
    c = L & 7
    cg = (((c >> 1) ^ mc_f(k)) << 1) | (c & 1)
    col = 64 * w + 8 * cg
    lds = w * 8192 + i * 1024 + 16 * L
    return k, col, lds


def mc_read(WO, h, blk, j, l):
    """MC fragment read (ds_read_b64_tr_b16 #j): LDS byte supplied by lane l."""
    g, q, p = l >> 4, (l >> 2) & 3, l & 3
    f = ((q >> 1) & 1) | ((g & 1) << 1)
    bq = blk & 3
    base = WO * 128 + (8 * g + q) * 128 + ((bq ^ f) * 32) + 8 * p
    return base + (blk >> 2) * 8192 + h * 4096 + j * 512


# ---- emitter -------------------------------------------------------------------------------------
class Kernel:
    def __init__(self, name, a_kc, b_kc, ek, persistent=False, f16=False):
        self.name, self.a_kc, self.b_kc = name, a_kc, b_kc
        # operand / 16-bit output type: bf16 (default) or IEEE fp16 (same tiles and schedule;
        # MFMA, output conversion and epilogue unpacks differ)
        self.f16 = f16
        self.cvt = "v_cvt_pk_f16_f32" if f16 else "v_cvt_pk_bf16_f32"
        self.mfma_op = "v_mfma_f32_16x16x32_f16" if f16 else "v_mfma_f32_16x16x32_bf16"
        self.persistent = persistent
        self.VE = 112 if persistent else V_FRAG
        self.VBIAS, self.VTMP, self.VCONST = self.VE + E_BIAS, self.VE + E_TMP, self.VE + E_CONST
        # ek: plain kinds (bf16 / f32 / f32acc) or fused: bias[gelu|relu] (pre-activation stored
        # as aux), d{gelu,relu} (C = acc ⊙ act'(aux))
        fused = {"bias": ("bias_act", 0), "biasgelu": ("bias_act", 1), "biasrelu": ("bias_act", 3),
                 "biasgeluerf": ("bias_act", 2),
                 "dgelu": ("dact", 1), "drelu": ("dact", 3), "biasnx": ("bias_act", 0),
                 "dgelucs": ("dact", 1), "drelucs": ("dact", 3)}
        self.ek, self.act = fused.get(ek, (ek, 0))
        # *cs: the dact epilogue also writes per-128-row-band column sums of C (the bias gradient
        # of the layer whose pre-activation this is: FFN1's db1 from the FFN2 data-gradient GEMM)
        self.colsum = ek in ("dgelucs", "drelucs")
        self.VCS = self.VE + 102        # 32 column-sum accumulators (8 blocks × 4 columns), +32 row,
        # +34..37 masked values (≤ v251 in the persistent kernel: accum_offset 256 below)
        self.store_aux = ek != "biasnx"  # biasnx: C = acc + bias, no pre-activation output
        self.NBW = 8                    # 16-column accumulator blocks per wave row
        # resources: LDS bytes, workgroup size, accum_offset, AGPR count
        self.lds_bytes, self.wg_size, self.acc_off, self.n_agpr = LDS_BYTES, 256, ACC_OFF, 256
        if self.colsum:  # the persistent kernel's epilogue registers end at v213: room for 32 more
            self.acc_off = 256
        assert self.ek not in ("bias_act", "dact") or (a_kc and b_kc)  # descriptor SGPRs 40..47
        self.lines = []
        self.nlab = 0

    def e(self, s):
        if ABL:
            m = s.split(" ", 1)[0]
            if (("nodma" in ABL and m == "buffer_load_dwordx4" and s.endswith(" lds"))
                    or ("noreads" in ABL and m.startswith("ds_read"))
                    or ("nobar" in ABL and m == "s_barrier")):
                return
            if "nomfma" in ABL and m.startswith("v_mfma"):
                s = "s_nop 0"
            if ("vload" in ABL or "dsw" in ABL) and m == "buffer_load_dwordx4" and s.endswith(" lds"):
                # register-staged operand path priced without its latency: a plain VMEM load into
                # scratch VGPRs (vload) and/or a ds_write_b128 of a fixed register (dsw)
                i = int(s.split()[1].strip("v,")) % 8
                if "vload" in ABL:
                    self.lines.append(f"\tbuffer_load_dwordx4 v[{180 + 4 * i}:{183 + 4 * i}], "
                                      + s.split(" ", 1)[1][:-4])
                if "dsw" in ABL:  # v220 = lane·16 (set in the prologue): in-range LDS addresses
                    self.lines.append(f"\tds_write_b128 v220, v[216:219] offset:{i * 4096}")
                return
            if "mfma32" in ABL and m.startswith("v_mfma"):
                # 32x32x16 MFMAs (half the count, twice the length) at the same slots
                self.nmf = getattr(self, "nmf", 0) + 1
                if self.nmf % 2 == 0:
                    return
                ops = s.split(" ", 1)[1].split(", ")
                c = 16 * ((self.nmf // 2) % 16)
                s = f"v_mfma_f32_32x32x16_bf16 a[{c}:{c + 15}], {ops[1]}, {ops[2]}, " + (
                    "0" if ops[3] == "0" else f"a[{c}:{c + 15}]")
        self.lines.append("\t" + s)

    def lab(self, s):
        self.lines.append(s + ":")

    def newlab(self, tag):
        self.nlab += 1
        return f".L{self.name}_{tag}_{self.nlab}"

    # -- scalar helpers ---------------------------------------------------------------------------
    def udiv(self, q, r, n, d, rcp_s=None, rcp_v=None):
        """q = n / d, r = n % d (SGPRs; n < 2^24) via an f32 reciprocal (SGPR bits or VGPR) and
        a ±1 integer fix-up."""
        v = V_T
        self.e(f"v_cvt_f32_u32 v{v}, s{n}")
        if rcp_s is not None:
            self.e(f"v_mul_f32 v{v}, s{rcp_s}, v{v}")
        else:
            self.e(f"v_mul_f32 v{v}, v{rcp_v}, v{v}")
        self.e(f"v_cvt_u32_f32 v{v}, v{v}")
        self.e("s_nop 1")
        self.e(f"v_readfirstlane_b32 s{q}, v{v}")
        self.e("s_nop 1")
        t = S_T + 9
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

    def srd_set_records(self, srd, rem):
        self.e(f"s_cmp_eq_u32 s{rem + 1}, 0")
        self.e(f"s_cselect_b32 s{srd + 2}, s{rem}, -1")

    def srd_advance(self, srd, rem, step):
        self.e(f"s_add_u32 s{srd}, s{srd}, s{step}")
        self.e(f"s_addc_u32 s{srd + 1}, s{srd + 1}, s{step + 1}")
        self.e(f"s_sub_u32 s{rem}, s{rem}, s{step}")
        self.e(f"s_subb_u32 s{rem + 1}, s{rem + 1}, s{step + 1}")
        self.srd_set_records(srd, rem)

    # -- prologue ---------------------------------------------------------------------------------
    def prologue(self):
        T = S_T
        self.e(f"s_load_dwordx16 s[{S_ARG}:{S_ARG + 15}], s[0:1], 0x0")
        self.e(f"s_load_dwordx8 s[{S_ARG + 16}:{S_ARG + 23}], s[0:1], 0x40")
        self.e(f"s_load_dwordx8 s[{S_E}:{S_E + 7}], s[0:1], 0x60")       # c, c_bytes, ldc_b, ldaux_b, c_part
        self.e(f"s_load_dwordx4 s[{S_E + 8}:{S_E + 11}], s[0:1], 0x80")  # aux, aux_bytes
        self.e(f"s_load_dwordx2 s[{S_E + 12}:{S_E + 13}], s[0:1], 0x90")  # bias
        self.e(f"v_and_b32 v{V_LANE}, 63, v{V_TID}")
        if "dsw" in ABL:
            self.e(f"v_lshlrev_b32 v220, 4, v{V_LANE}")
        self.e(f"v_lshrrev_b32 v{V_T}, 6, v{V_TID}")
        self.e("s_nop 1")
        self.e(f"v_readfirstlane_b32 s{S_WAVE}, v{V_T}")
        self.e("s_waitcnt lgkmcnt(0)")
        # XCD remap over the launched grid G: u = (x < r ? x*(q+1) : r*(q+1) + (x-r)*q) + b/8,
        # x = b%8, q = G/8, r = G%8 (bijective; blocks sharing an XCD take consecutive units)
        G = S_GRID
        self.e(f"s_and_b32 s{T}, s{S_WG}, 7")
        self.e(f"s_lshr_b32 s{T + 1}, s{G}, 3")
        self.e(f"s_and_b32 s{T + 2}, s{G}, 7")
        self.e(f"s_add_u32 s{T + 3}, s{T + 1}, 1")
        self.e(f"s_mul_i32 s{T + 4}, s{T}, s{T + 3}")
        self.e(f"s_mul_i32 s{T + 5}, s{T + 2}, s{T + 3}")
        self.e(f"s_sub_u32 s{T + 6}, s{T}, s{T + 2}")
        self.e(f"s_mul_i32 s{T + 6}, s{T + 6}, s{T + 1}")
        self.e(f"s_add_u32 s{T + 5}, s{T + 5}, s{T + 6}")
        self.e(f"s_cmp_lt_u32 s{T}, s{T + 2}")
        self.e(f"s_cselect_b32 s{T + 4}, s{T + 4}, s{T + 5}")
        self.e(f"s_lshr_b32 s{T + 6}, s{S_WG}, 3")
        self.e(f"s_add_u32 s{S_U0}, s{T + 4}, s{T + 6}")
        self.e(f"s_mov_b32 s{S_ROUND}, 0")

    def tile_coords(self, u, m0, n0, part):
        """Work unit u (SGPR) → tile origin (rows m0, cols n0) and split-K part: part = u / ntiles,
        tile in group-M order (GM m-tiles × all n-tiles per group)."""
        T = S_T
        self.e(f"s_mov_b32 s{T + 4}, s{u}")
        self.udiv(part, T + 5, T + 4, S_NTILES, rcp_s=S_RCPNT)
        self.udiv(T + 6, T + 7, T + 5, S_PERGRP, rcp_s=S_RCPPG)
        self.e(f"s_mul_i32 s{T + 6}, s{T + 6}, s{S_GM}")          # first_m
        self.e(f"s_sub_u32 s{T + 8}, s{S_TM}, s{T + 6}")
        self.e(f"s_min_u32 s{T + 8}, s{T + 8}, s{S_GM}")          # gm
        self.e(f"v_cvt_f32_u32 v{V_T + 1}, s{T + 8}")
        self.e(f"v_rcp_f32 v{V_T + 1}, v{V_T + 1}")
        self.e("s_nop 0")
        self.udiv(n0, T + 4, T + 7, T + 8, rcp_v=V_T + 1)         # tn = in_g / gm, tm_off
        self.e(f"s_add_u32 s{m0}, s{T + 6}, s{T + 4}")
        self.e(f"s_lshl_b32 s{m0}, s{m0}, 8")
        self.e(f"s_lshl_b32 s{n0}, s{n0}, 8")

    def setup_tile(self, m0, n0, part, full=True):
        """Descriptors and DMA offsets of both operands for the tile at (m0, n0, part); ``full``
        also sets the tile-invariant LDS bases, soffsets and fragment-read bases."""
        T = S_T
        # part decomposition (split-K / batch): kmul → s{T+5}, batch strides → s[T+6:T+9]
        self.e(f"s_load_dword s{T + 5}, s[0:1], 0x98")
        self.e(f"s_load_dwordx4 s[{T + 6}:{T + 9}], s[0:1], 0xa0")
        self.e("s_waitcnt lgkmcnt(0)")
        self.e(f"s_mul_i32 s{T}, s{part}, s{T + 5}")             # K start (elements)
        for op in (0, 1):
            self.setup_operand(op, T, m0 if op == 0 else n0, full, part)

    def setup_operand(self, op, T, t0, full=True, part=None):
        """Descriptor, K step, DMA voffsets, LDS-DMA bases and read bases of operand op; t0: SGPR
        with the tile origin along this operand's rows (A: m0, B: n0); s{T}: K start."""
        kc = self.a_kc if op == 0 else self.b_kc
        ptr = S_A if op == 0 else S_B
        tot = S_ABYTES if op == 0 else S_BBYTES
        ld = S_LDA if op == 0 else S_LDB
        srd = S_SRDA if op == 0 else S_SRDB
        rem = S_REMA if op == 0 else S_REMB
        step = S_STEPA if op == 0 else S_STEPB
        soff = S_SOFFA if op == 0 else S_SOFFB
        ldsb = S_LDSA if op == 0 else S_LDSB
        vd = V_DMAA if op == 0 else V_DMAB
        rb = V_RBA if op == 0 else V_RBB
        lim = S_M if op == 0 else S_N
        opoff = 0 if op == 0 else OP_BYTES
        a, b = T + 1, T + 2                       # 64-bit offset accumulator s[a:b]
        # byte offset of the tile origin + K range start
        if kc:
            self.e(f"s_mul_i32 s{a}, s{t0}, s{ld}")
            self.e(f"s_mul_hi_u32 s{b}, s{t0}, s{ld}")
            self.e(f"s_lshl_b32 s{T + 3}, s{T}, 1")
            self.e(f"s_add_u32 s{a}, s{a}, s{T + 3}")
            self.e(f"s_addc_u32 s{b}, s{b}, 0")
            self.e(f"s_mov_b32 s{step}, {BK * 2}")
            self.e(f"s_mov_b32 s{step + 1}, 0")
        else:
            self.e(f"s_mul_i32 s{a}, s{T}, s{ld}")
            self.e(f"s_mul_hi_u32 s{b}, s{T}, s{ld}")
            self.e(f"s_lshl_b32 s{T + 3}, s{t0}, 1")
            self.e(f"s_add_u32 s{a}, s{a}, s{T + 3}")
            self.e(f"s_addc_u32 s{b}, s{b}, 0")
            self.e(f"s_lshl_b32 s{T + 3}, s{ld}, 6")
            self.e(f"s_mov_b32 s{step}, s{T + 3}")
            self.e(f"s_lshr_b32 s{step + 1}, s{ld}, 26")
        if part is not None:  # batched: + part · bstride (64-bit)
            slo = T + 6 + 2 * op
            self.e(f"s_mul_i32 s{T + 3}, s{part}, s{slo}")
            self.e(f"s_mul_hi_u32 s{T + 4}, s{part}, s{slo}")
            self.e(f"s_add_u32 s{a}, s{a}, s{T + 3}")
            self.e(f"s_addc_u32 s{b}, s{b}, s{T + 4}")
            self.e(f"s_mul_i32 s{T + 3}, s{part}, s{slo + 1}")
            self.e(f"s_add_u32 s{b}, s{b}, s{T + 3}")
        self.e(f"s_add_u32 s{srd}, s{ptr}, s{a}")
        self.e(f"s_addc_u32 s{srd + 1}, s{ptr + 1}, s{b}")
        self.e(f"s_and_b32 s{srd + 1}, s{srd + 1}, 0xffff")
        self.e(f"s_sub_u32 s{rem}, s{tot}, s{a}")
        self.e(f"s_subb_u32 s{rem + 1}, s{tot + 1}, s{b}")
        self.srd_set_records(srd, rem)
        self.e(f"s_mov_b32 s{srd + 3}, 0x20000")
        # LDS-DMA bases of this wave (stage 0 / 1)
        per_wave = 1024 if kc else 8192
        if full:
            self.e(f"s_mul_i32 s{T + 3}, s{S_WAVE}, {per_wave}")
            self.e(f"s_add_u32 s{ldsb}, s{T + 3}, {opoff}")
            self.e(f"s_add_u32 s{ldsb + 1}, s{T + 3}, {opoff + STAGE_BYTES}")
        V, L = V_T, V_LANE
        if kc:
            # g16 = ((L&7) ^ ((4w + (L>>4)) & 7)) * 16 ; rows 32i + 8w + (L>>3) clamped to lim-1-t0
            self.e(f"s_lshl_b32 s{T + 3}, s{S_WAVE}, 2")
            self.e(f"v_lshrrev_b32 v{V}, 4, v{L}")
            self.e(f"v_add_u32 v{V}, s{T + 3}, v{V}")
            self.e(f"v_and_b32 v{V + 1}, 7, v{L}")
            self.e(f"v_xor_b32 v{V}, v{V}, v{V + 1}")
            self.e(f"v_and_b32 v{V}, 7, v{V}")
            self.e(f"v_lshlrev_b32 v{V}, 4, v{V}")                  # g16
            self.e(f"v_lshrrev_b32 v{V + 1}, 3, v{L}")
            self.e(f"s_lshl_b32 s{T + 3}, s{S_WAVE}, 3")
            self.e(f"v_add_u32 v{V + 1}, s{T + 3}, v{V + 1}")       # 8w + (L>>3)
            self.e(f"s_sub_u32 s{T + 4}, s{lim}, s{t0}")
            self.e(f"s_sub_u32 s{T + 4}, s{T + 4}, 1")               # last valid local row
            for i in range(8):
                self.e(f"v_add_u32 v{V + 2}, {32 * i}, v{V + 1}")
                self.e(f"v_min_u32 v{V + 2}, s{T + 4}, v{V + 2}")
                self.e(f"v_mad_u32_u24 v{vd + i}, v{V + 2}, s{ld}, v{V}")
            if not full:
                return
            # read bases [stage][h]
            WO = 128  # rows per wave half; wave offset = 128 * (wr or wc)
            sel = "wr" if op == 0 else "wc"
            self.wave_half(T + 3, sel)
            self.e(f"s_mul_i32 s{T + 3}, s{T + 3}, {WO * 128}")
            self.e(f"v_and_b32 v{V}, 15, v{L}")
            self.e(f"v_lshlrev_b32 v{V}, 7, v{V}")                  # (l&15)*128
            self.e(f"v_add_u32 v{V}, s{T + 3}, v{V}")
            self.e(f"v_lshrrev_b32 v{V + 1}, 1, v{L}")
            self.e(f"v_and_b32 v{V + 1}, 7, v{V + 1}")               # (l>>1)&7
            self.e(f"v_lshrrev_b32 v{V + 2}, 4, v{L}")               # l>>4
            for h in (0, 1):
                self.e(f"v_add_u32 v{V + 3}, {4 * h}, v{V + 2}")
                self.e(f"v_xor_b32 v{V + 3}, v{V + 3}, v{V + 1}")
                self.e(f"v_lshl_add_u32 v{V + 3}, v{V + 3}, 4, v{V}")
                for s in (0, 1):
                    self.e(f"v_add_u32 v{rb + 2 * s + h}, {s * STAGE_BYTES + opoff}, v{V + 3}")
        else:
            # DMA: k row (L>>3) (+8i by soffset), chunk c = L&7,
            # cg = (((c>>1) ^ f) << 1) | (c&1), f = ((L>>4)&1) | ((i&1)<<1); col = 64w + 8cg
            self.e(f"v_lshrrev_b32 v{V}, 4, v{L}")
            self.e(f"v_and_b32 v{V}, 1, v{V}")                       # (L>>4)&1
            self.e(f"v_lshrrev_b32 v{V + 1}, 1, v{L}")
            self.e(f"v_and_b32 v{V + 1}, 3, v{V + 1}")               # c>>1
            self.e(f"v_and_b32 v{V + 2}, 1, v{L}")                   # c&1
            self.e(f"v_lshrrev_b32 v{V + 3}, 3, v{L}")               # k row
            self.e(f"s_lshl_b32 s{T + 3}, s{S_WAVE}, 6")             # 64w
            self.e(f"s_sub_u32 s{T + 4}, s{lim}, s{t0}")
            self.e(f"s_sub_u32 s{T + 4}, s{T + 4}, 8")               # last valid 8-col chunk start
            for par in (0, 1):
                self.e(f"v_xor_b32 v{V + 4}, v{V + 1}, v{V}")
                if par:
                    self.e(f"v_xor_b32 v{V + 4}, 2, v{V + 4}")
                self.e(f"v_lshl_or_b32 v{V + 4}, v{V + 4}, 1, v{V + 2}")   # cg
                self.e(f"v_lshl_add_u32 v{V + 4}, v{V + 4}, 3, s{T + 3}")  # col
                self.e(f"v_min_u32 v{V + 4}, s{T + 4}, v{V + 4}")
                self.e(f"v_lshlrev_b32 v{V + 4}, 1, v{V + 4}")
                self.e(f"v_mad_u32_u24 v{vd + par}, v{V + 3}, s{ld}, v{V + 4}")
            if not full:
                return
            for i in range(8):
                self.e(f"s_mul_i32 s{soff + i}, s{ld}, {8 * i}")
            # read bases [stage][bq]: WO*128 + (8g+q)*128 + ((bq ^ f)*32) + 8p
            sel = "wr" if op == 0 else "wc"
            self.wave_half(T + 3, sel)
            self.e(f"s_mul_i32 s{T + 3}, s{T + 3}, {128 * 128}")
            self.e(f"v_lshrrev_b32 v{V}, 4, v{L}")                   # g
            self.e(f"v_lshrrev_b32 v{V + 1}, 2, v{L}")
            self.e(f"v_and_b32 v{V + 1}, 3, v{V + 1}")               # q
            self.e(f"v_lshl_add_u32 v{V + 2}, v{V}, 3, v{V + 1}")    # 8g+q
            self.e(f"v_lshlrev_b32 v{V + 2}, 7, v{V + 2}")
            self.e(f"v_and_b32 v{V + 3}, 3, v{L}")                   # p
            self.e(f"v_lshl_add_u32 v{V + 2}, v{V + 3}, 3, v{V + 2}")
            self.e(f"v_add_u32 v{V + 2}, s{T + 3}, v{V + 2}")
            self.e(f"v_lshrrev_b32 v{V + 3}, 1, v{V + 1}")           # (q>>1)&1
            self.e(f"v_and_b32 v{V}, 1, v{V}")
            self.e(f"v_lshl_or_b32 v{V + 3}, v{V}, 1, v{V + 3}")     # f
            for bq in range(4):
                self.e(f"v_xor_b32 v{V + 4}, {bq}, v{V + 3}")
                self.e(f"v_lshl_add_u32 v{V + 4}, v{V + 4}, 5, v{V + 2}")
                for s in (0, 1):
                    self.e(f"v_add_u32 v{rb + 4 * s + bq}, {s * STAGE_BYTES + opoff}, v{V + 4}")

    def wave_half(self, dst, sel):
        if sel == "wr":
            self.e(f"s_lshr_b32 s{dst}, s{S_WAVE}, 1")
        else:
            self.e(f"s_and_b32 s{dst}, s{S_WAVE}, 1")

    # -- main-loop building blocks ------------------------------------------------------------------
    def dma_ops(self, stage):
        """The 16 LDS-DMA issues of one K-block (A then B): list of (m0 line, load line, after)."""
        ops = []
        for op in (0, 1):
            kc = self.a_kc if op == 0 else self.b_kc
            srd = S_SRDA if op == 0 else S_SRDB
            ldsb = (S_LDSA if op == 0 else S_LDSB) + stage
            vd = V_DMAA if op == 0 else V_DMAB
            soff = S_SOFFA if op == 0 else S_SOFFB
            for i in range(8):
                if kc:
                    m0 = f"s_add_u32 m0, s{ldsb}, {i * 4096}"
                    ld = (f"global_load_lds_dwordx4 v{vd + i}, s[{srd}:{srd + 1}]" if self.GLDS else
                          f"buffer_load_dwordx4 v{vd + i}, s[{srd}:{srd + 3}], 0 offen lds")
                else:
                    m0 = f"s_add_u32 m0, s{ldsb}, {i * 1024}"
                    ld = f"buffer_load_dwordx4 v{vd + (i & 1)}, s[{srd}:{srd + 3}], s{soff + i} offen lds"
                ops.append((m0, ld, op if i == 7 else None))
        return ops

    def advance(self, op):
        if op == 0:
            self.srd_advance(S_SRDA, S_REMA, S_STEPA)
        else:
            self.srd_advance(S_SRDB, S_REMB, S_STEPB)

    def read_ops(self, set_, stage, h):
        """LDS reads of the 16 fragments of k-half h of `stage` into set `set_` (B first: the
        first MFMA row needs all 8 B fragments)."""
        order = []
        for k in range(8):
            order.append((1, k))
            if k % 2 == 1:
                order.append((0, k // 2))
        for k in range(4, 8):
            order.append((0, k))
        ops = []
        for op, blk in order:
            kc = self.a_kc if op == 0 else self.b_kc
            rb = V_RBA if op == 0 else V_RBB
            d = frag(set_, op, blk)
            if kc:
                ops.append(f"ds_read_b128 v[{d}:{d + 3}], v{rb + 2 * stage + h} offset:{blk * 2048}")
            else:
                base = rb + 4 * stage + (blk & 3)
                off = (blk >> 2) * 8192 + h * 4096
                ops.append(f"ds_read_b64_tr_b16 v[{d}:{d + 1}], v{base} offset:{off}")
                ops.append(f"ds_read_b64_tr_b16 v[{d + 2}:{d + 3}], v{base} offset:{off + 512}")
        return ops

    def mfma(self, set_, mb, nb, zero=False):
        a, b, c = frag(set_, 0, mb), frag(set_, 1, nb), acc(mb, nb)
        src2 = "0" if zero else f"a[{c}:{c + 3}]"
        self.e(f"{self.mfma_op} a[{c}:{c + 3}], v[{b}:{b + 3}], v[{a}:{a + 3}], {src2}")

    # Schedule of one K-block (128 MFMAs; slot k = after MFMA k):
    #   slots 0-15   read Y (k-half 1 of this stage)                    [phase A: MFMAs on X]
    #   slot 24      lgkmcnt(0) + barrier: every wave has this whole block in registers
    #   slots 26-116 16 LDS-DMAs of block t+2 into THIS stage, one per 6 MFMAs (m0 one slot
    #                before); those past BAR2 land under the next iteration (the stage they fill is
    #                read only after the next BAR2)
    #   slot 92      vmcnt(#DMAs of this iteration issued so far) + barrier: block t+1 has landed
    #   slots 93-114 read X (k-half 0 of the other stage)                [phase B: MFMAs on Y]
    #   end          lgkmcnt(0)
    # The DMA issue cost (~60 cycles each among MFMAs, MI355X_MICROARCH.md) is spread over 90
    # MFMAs instead of being bunched.
    # Round 5: DMAs one per 6 MFMAs (26 … 116, past BAR2) instead of one per 4 (26 … 86): each
    # LDS-DMA issue stalls its wave ~60 cycles, so bunched issues left the MFMA pipe idle; with
    # the Y reads done by slot 16 the NT GEMMs run 4.5-5.3 % faster (profiles/gemm_sched_r5.txt)
    Y_END, BAR1, DMA0, DMA_GAP, BAR2, X0, X_END = 16, 24, 26, 6, 92, 93, 115
    # K-contiguous operands by global_load_lds (saddr form; the descriptor's first two dwords are
    # the 64-bit base) instead of buffer_load … lds: A/B of the DMA issue cost (every address is
    # in range by construction; an exhausted stream is rewound onto consumed blocks, never 0)
    GLDS = os.environ.get("PIAMD_AGEMM_GLDS", "0") == "1"
    if os.environ.get("PIAMD_AGEMM_SCHED"):  # schedule sweeps (tools/agemm_sched_sweep.py)
        Y_END, BAR1, DMA0, DMA_GAP, BAR2, X0, X_END = (float(v) if "." in v else int(v) for v in
                                                       os.environ["PIAMD_AGEMM_SCHED"].split(","))

    def dma_slot(self, n):
        """Slot of the n-th of the 16 DMAs of a K-block (DMA_GAP may be fractional)."""
        return self.DMA0 + int(self.DMA_GAP * n)

    def iteration(self, stage, dma, read_next, first=False, vm_extra=0):
        ysl, dsl, xsl = {}, {}, {}
        yreads = self.read_ops(1, stage, 1)
        for r, op in enumerate(yreads):
            ysl.setdefault(r * self.Y_END // len(yreads), []).append(op)
        if dma:
            for n, (m0, ld, adv) in enumerate(self.dma_ops(stage)):
                k = self.dma_slot(n)
                dsl.setdefault(k - 1, []).append(m0)
                dsl.setdefault(k, []).append(ld)
                if adv is not None:
                    dsl.setdefault(k, []).append(("adv", adv))
        if read_next:
            xreads = self.read_ops(0, stage ^ 1, 0)
            for r, op in enumerate(xreads):
                xsl.setdefault(self.X0 + r * (self.X_END - self.X0) // len(xreads), []).append(op)
        for k in range(128):
            if k == self.BAR1:
                self.e("s_waitcnt lgkmcnt(0)")
                if dma:
                    self.e("s_barrier")
            if k == self.BAR2 and read_next:
                # every DMA of this iteration issued before BAR2 may still fly (the rest come later):
                # block t+1 (issued one iteration earlier) is then complete
                nb = sum(1 for n in range(16) if self.dma_slot(n) < self.BAR2) if dma else 0
                self.e(f"s_waitcnt vmcnt({min(63, nb + vm_extra)})")
                self.e("s_barrier")
            kk = k % 64
            self.mfma(k // 64, kk // 8, kk % 8, zero=first and k < 64)
            for op in dsl.get(k, []):
                if isinstance(op, tuple):
                    self.advance(op[1])
                else:
                    self.e(op)
            for op in ysl.get(k, []) + xsl.get(k, []):
                self.e(op)
        if read_next:
            self.e("s_waitcnt lgkmcnt(0)")

    def prime(self):
        """Blocks 0 and 1 of the current tile into stages 0 and 1, then k-half 0 of block 0."""
        for stage in (0, 1):
            for m0, ld, adv in self.dma_ops(stage):
                self.e(m0)
                self.e("s_nop 0")
                self.e(ld)
                if adv is not None:
                    self.advance(adv)
        self.e("s_waitcnt vmcnt(16)")
        self.e("s_barrier")
        for op in self.read_ops(0, 0, 0):
            self.e(op)
        self.e("s_waitcnt lgkmcnt(0)")

    # -- whole kernel ---------------------------------------------------------------------------------
    def body(self):
        """One tile per workgroup (any nk >= 2)."""
        self.prologue()
        self.tile_coords(S_U0, S_M0T, S_N0T, S_PART)
        self.setup_tile(S_M0T, S_N0T, S_PART)
        self.prime()
        # npairs = (nk - 2) >> 1, rem = nk - 2 npairs (2 or 3)
        self.e(f"s_sub_u32 s{S_LOOP}, s{S_NK}, 2")
        self.e(f"s_lshr_b32 s{S_LOOP}, s{S_LOOP}, 1")
        self.e(f"s_lshl_b32 s{S_REM}, s{S_LOOP}, 1")
        self.e(f"s_sub_u32 s{S_REM}, s{S_NK}, s{S_REM}")
        lend, lbeg = self.newlab("loopend"), self.newlab("loop")
        first_done = self.newlab("firstdone")
        # the first pair zero-initialises the accumulators (MFMA with a 0 accumulator input)
        self.e(f"s_cmp_le_i32 s{S_LOOP}, 0")
        self.e(f"s_cbranch_scc1 {first_done}")
        self.iteration(0, True, True, first=True)
        self.iteration(1, True, True)
        self.e(f"s_sub_i32 s{S_LOOP}, s{S_LOOP}, 1")
        self.e(f"s_cmp_le_i32 s{S_LOOP}, 0")
        self.e(f"s_cbranch_scc1 {lend}")
        self.lab(lbeg)
        self.iteration(0, True, True)
        self.iteration(1, True, True)
        self.e(f"s_sub_i32 s{S_LOOP}, s{S_LOOP}, 1")
        self.e(f"s_cmp_gt_i32 s{S_LOOP}, 0")
        self.e(f"s_cbranch_scc1 {lbeg}")
        self.e(f"s_branch {lend}")
        # nk = 2 or 3: no pair ran — zero the accumulators here
        self.lab(first_done)
        for i in range(256):
            self.e(f"v_accvgpr_write_b32 a{i}, 0")
        self.e("s_nop 4")
        self.lab(lend)
        t2, epi = self.newlab("tail2"), self.newlab("epi")
        self.e(f"s_cmp_eq_u32 s{S_REM}, 3")
        self.e(f"s_cbranch_scc0 {t2}")
        self.iteration(0, True, True)
        self.iteration(1, False, True)
        self.iteration(0, False, False)
        self.e(f"s_branch {epi}")
        self.lab(t2)
        self.iteration(0, False, True)
        self.iteration(1, False, False)
        self.lab(epi)
        self.epilogue()
        self.e("s_waitcnt vmcnt(0)")
        self.e("s_endpgm")

    def body_persistent(self):
        """Workgroup w takes work units U0(w) + i·G (G = launched grid), tiles chained through
        the LDS-DMA stream: the last K-block pair of a tile issues the NEXT tile's blocks 0 and 1
        and reads its first fragments, so the epilogue overlaps the next tile's loads. nk even,
        >= 4 (host contract)."""
        self.prologue()
        lend = self.newlab("end")
        self.e(f"s_cmp_ge_u32 s{S_U0}, s{S_NWG}")                     # nwg = total units
        self.e(f"s_cbranch_scc1 {lend}")
        self.tile_coords(S_U0, S_M0T, S_N0T, S_PART)
        self.setup_tile(S_M0T, S_N0T, S_PART)
        self.prime()
        ltile, lbeg, lpend = self.newlab("tile"), self.newlab("loop"), self.newlab("loopend")
        lsecond = self.newlab("second")
        self.iteration(0, True, True, first=True)
        self.e(f"s_branch {lsecond}")
        # later tiles: the previous epilogue's stores are still in flight, older than this
        # iteration's DMAs — count past them instead of draining them
        self.lab(ltile)
        self.iteration(0, True, True, first=True, vm_extra=self.store_count())
        self.lab(lsecond)
        self.iteration(1, True, True)
        self.e(f"s_lshr_b32 s{S_LOOP}, s{S_NK}, 1")
        self.e(f"s_sub_i32 s{S_LOOP}, s{S_LOOP}, 2")
        self.e(f"s_cmp_le_i32 s{S_LOOP}, 0")
        self.e(f"s_cbranch_scc1 {lpend}")
        self.lab(lbeg)
        self.iteration(0, True, True)
        self.iteration(1, True, True)
        self.e(f"s_sub_i32 s{S_LOOP}, s{S_LOOP}, 1")
        self.e(f"s_cmp_gt_i32 s{S_LOOP}, 0")
        self.e(f"s_cbranch_scc1 {lbeg}")
        self.lab(lpend)
        # switch the DMA stream to the next unit (or to an empty descriptor)
        T = S_T
        nxt, nonext, ready = self.newlab("next"), self.newlab("nonext"), self.newlab("ready")
        self.e(f"s_add_u32 s{T + 9}, s{S_ROUND}, 1")
        self.e(f"s_mul_i32 s{T + 9}, s{T + 9}, s{S_GRID}")
        self.e(f"s_add_u32 s{S_NVALID}, s{S_U0}, s{T + 9}")               # next unit
        self.e(f"s_cmp_lt_u32 s{S_NVALID}, s{S_NWG}")
        self.e(f"s_cbranch_scc0 {nonext}")
        self.tile_coords(S_NVALID, S_NM0, S_NN0, S_NPART)
        self.setup_tile(S_NM0, S_NN0, S_NPART, full=False)
        self.e(f"s_mov_b32 s{S_NVALID}, 1")
        self.e(f"s_branch {ready}")
        self.lab(nonext)
        if self.GLDS:  # global_load_lds has no range check: re-read the last two consumed blocks
            for op, srd, kc in ((0, S_SRDA, self.a_kc), (1, S_SRDB, self.b_kc)):
                if kc:
                    self.e(f"s_sub_u32 s{srd}, s{srd}, {2 * BK * 2}")
                    self.e(f"s_subb_u32 s{srd + 1}, s{srd + 1}, 0")
        self.e(f"s_mov_b32 s{S_SRDA + 2}, 0")
        self.e(f"s_mov_b32 s{S_SRDB + 2}, 0")
        self.e(f"s_mov_b32 s{S_REMA}, 0")
        self.e(f"s_mov_b32 s{S_REMA + 1}, 0")
        self.e(f"s_mov_b32 s{S_REMB}, 0")
        self.e(f"s_mov_b32 s{S_REMB + 1}, 0")
        self.e(f"s_mov_b32 s{S_STEPA}, 0")
        self.e(f"s_mov_b32 s{S_STEPA + 1}, 0")
        self.e(f"s_mov_b32 s{S_STEPB}, 0")
        self.e(f"s_mov_b32 s{S_STEPB + 1}, 0")
        self.e(f"s_mov_b32 s{S_NVALID}, 0")
        self.lab(ready)
        self.iteration(0, True, True)
        self.iteration(1, True, True)
        self.epilogue()
        self.e(f"s_cmp_eq_u32 s{S_NVALID}, 0")
        self.e(f"s_cbranch_scc1 {lend}")
        self.e(f"s_mov_b32 s{S_M0T}, s{S_NM0}")
        self.e(f"s_mov_b32 s{S_N0T}, s{S_NN0}")
        self.e(f"s_mov_b32 s{S_PART}, s{S_NPART}")
        self.e(f"s_add_u32 s{S_ROUND}, s{S_ROUND}, 1")
        self.e(f"s_branch {ltile}")
        self.lab(lend)
        self.e("s_waitcnt vmcnt(0)")
        self.e("s_endpgm")

    # -- epilogues --------------------------------------------------------------------------------
    def epilogue(self):
        E, V = S_E, self.VE
        ek = self.ek
        f32 = ek in ("f32", "f32acc")
        es = 4 if f32 else 2
        self.e("s_nop 15")
        self.e("s_nop 15")
        if self.colsum:  # column-sum plane descriptor base / range (waited for before its stores)
            self.e("s_load_dwordx2 s[44:45], s[0:1], 0xb0")
            self.e("s_load_dword s46, s[0:1], 0xb8")
        # C descriptor base = c + part*c_part + m0*ldc_b + n0*es
        T = S_T
        self.e(f"s_mul_i32 s{T}, s{S_PART}, s{E + 6}")
        self.e(f"s_mul_hi_u32 s{T + 1}, s{S_PART}, s{E + 6}")
        self.e(f"s_mul_i32 s{T + 2}, s{S_PART}, s{E + 7}")
        self.e(f"s_add_u32 s{T + 1}, s{T + 1}, s{T + 2}")
        self.e(f"s_mul_i32 s{T + 2}, s{S_M0T}, s{E + 4}")
        self.e(f"s_mul_hi_u32 s{T + 3}, s{S_M0T}, s{E + 4}")
        self.e(f"s_add_u32 s{T}, s{T}, s{T + 2}")
        self.e(f"s_addc_u32 s{T + 1}, s{T + 1}, s{T + 3}")
        self.e(f"s_mul_i32 s{T + 2}, s{S_N0T}, {es}")
        self.e(f"s_add_u32 s{T}, s{T}, s{T + 2}")
        self.e(f"s_addc_u32 s{T + 1}, s{T + 1}, 0")
        srd = S_CSRD
        self.e(f"s_add_u32 s{srd}, s{E}, s{T}")
        self.e(f"s_addc_u32 s{srd + 1}, s{E + 1}, s{T + 1}")
        self.e(f"s_and_b32 s{srd + 1}, s{srd + 1}, 0xffff")
        # records = lim - (part*c_part + tile offset), clamped to [0, 2^32-1], where lim = the end
        # of this part's plane ((part+1)*c_part, at most c_bytes) for split-K / batched launches
        # (rows past M of a plane are dropped instead of landing in the next plane), else c_bytes
        self.e(f"s_add_u32 s{T + 4}, s{S_PART}, 1")
        self.e(f"s_mul_i32 s{T + 2}, s{T + 4}, s{E + 6}")
        self.e(f"s_mul_hi_u32 s{T + 3}, s{T + 4}, s{E + 6}")
        self.e(f"s_mul_i32 s{T + 5}, s{T + 4}, s{E + 7}")
        self.e(f"s_add_u32 s{T + 3}, s{T + 3}, s{T + 5}")
        self.e(f"s_or_b32 s{T + 5}, s{E + 6}, s{E + 7}")
        self.e(f"s_cmp_eq_u32 s{T + 5}, 0")
        self.e(f"s_cselect_b64 s[{T + 2}:{T + 3}], s[{E + 2}:{E + 3}], s[{T + 2}:{T + 3}]")
        self.e(f"s_sub_u32 s{T + 4}, s{E + 2}, s{T + 2}")
        self.e(f"s_subb_u32 s{T + 5}, s{E + 3}, s{T + 3}")          # SCC: c_bytes < lim
        self.e(f"s_cselect_b64 s[{T + 2}:{T + 3}], s[{E + 2}:{E + 3}], s[{T + 2}:{T + 3}]")
        self.e(f"s_sub_u32 s{T + 2}, s{T + 2}, s{T}")
        self.e(f"s_subb_u32 s{T + 3}, s{T + 3}, s{T + 1}")
        self.e(f"s_cmp_eq_u32 s{T + 3}, 0")
        self.e(f"s_cselect_b32 s{srd + 2}, s{T + 2}, -1")
        self.e(f"s_mov_b32 s{srd + 3}, 0x20000")
        if ek in ("bias_act", "dact"):
            # aux descriptor: aux + m0*ldaux_b + n0*2
            self.e(f"s_mul_i32 s{T}, s{S_M0T}, s{E + 5}")
            self.e(f"s_mul_hi_u32 s{T + 1}, s{S_M0T}, s{E + 5}")
            self.e(f"s_lshl_b32 s{T + 2}, s{S_N0T}, 1")
            self.e(f"s_add_u32 s{T}, s{T}, s{T + 2}")
            self.e(f"s_addc_u32 s{T + 1}, s{T + 1}, 0")
            a = S_AUXSRD
            self.e(f"s_add_u32 s{a}, s{E + 8}, s{T}")
            self.e(f"s_addc_u32 s{a + 1}, s{E + 9}, s{T + 1}")
            self.e(f"s_and_b32 s{a + 1}, s{a + 1}, 0xffff")
            self.e(f"s_sub_u32 s{T + 2}, s{E + 10}, s{T}")
            self.e(f"s_subb_u32 s{T + 3}, s{E + 11}, s{T + 1}")
            self.e(f"s_cmp_eq_u32 s{T + 3}, 0")
            self.e(f"s_cselect_b32 s{a + 2}, s{T + 2}, -1")
            self.e(f"s_or_b32 s{T + 2}, s{E + 8}, s{E + 9}")
            self.e(f"s_cmp_eq_u32 s{T + 2}, 0")
            self.e(f"s_cselect_b32 s{a + 2}, 0, s{a + 2}")
            self.e(f"s_mov_b32 s{a + 3}, 0x20000")
        # lane offsets: row (wave row origin + (l&15)), col (wave col origin + 4(l>>4))
        L = V_LANE
        self.wave_origin(T + 4, T + 5)
        self.e(f"v_and_b32 v{V}, 15, v{L}")
        self.e(f"v_add_u32 v{V}, s{T + 4}, v{V}")                    # local row
        self.e(f"v_lshrrev_b32 v{V + 1}, 4, v{L}")
        self.e(f"v_lshl_add_u32 v{V + 1}, v{V + 1}, 2, s{T + 5}")    # local col
        self.e(f"v_mul_lo_u32 v{V + 2}, v{V}, s{E + 4}")
        self.e(f"v_mad_u32_u24 v{V + 2}, v{V + 1}, {es}, v{V + 2}")  # C voffset (mb = 0)
        if ek in ("bias_act", "dact"):
            self.e(f"v_mul_lo_u32 v{V + 3}, v{V}, s{E + 5}")
            self.e(f"v_lshl_add_u32 v{V + 3}, v{V + 1}, 1, v{V + 3}")  # aux voffset
            consts = ERF_CONSTS if self.act == 2 else (K0, K0 * K1, 3 * K0 * K1, TWO_LOG2E, 1.0)
            for i, val in enumerate(consts):
                self.e(f"v_mov_b32 v{self.VCONST + 2 * i}, {fhex(val)}")
                self.e(f"v_mov_b32 v{self.VCONST + 2 * i + 1}, {fhex(val)}")
        if ek == "bias_act":
            # bias descriptor (records 0 when there is no bias: loads return 0)
            b = S_BIASSRD
            self.e(f"s_lshl_b32 s{T}, s{S_N0T}, 1")
            self.e(f"s_add_u32 s{b}, s{E + 12}, s{T}")
            self.e(f"s_addc_u32 s{b + 1}, s{E + 13}, 0")
            self.e(f"s_and_b32 s{b + 1}, s{b + 1}, 0xffff")
            self.e(f"s_sub_u32 s{T + 1}, s{S_N}, s{S_N0T}")
            self.e(f"s_lshl_b32 s{T + 1}, s{T + 1}, 1")
            self.e(f"s_or_b32 s{T + 2}, s{E + 12}, s{E + 13}")
            self.e(f"s_cmp_eq_u32 s{T + 2}, 0")
            self.e(f"s_cselect_b32 s{b + 2}, 0, s{T + 1}")
            self.e(f"s_mov_b32 s{b + 3}, 0x20000")
            self.e(f"v_lshlrev_b32 v{V + 7}, 1, v{V + 1}")
            for nb in range(self.NBW):
                self.e(f"buffer_load_dwordx2 v[{self.VBIAS + 2 * nb}:{self.VBIAS + 2 * nb + 1}], v{V + 7}, s[{b}:{b + 3}], 0 offen offset:{nb * 32}")
            self.e("s_waitcnt vmcnt(0)")
        self.e(f"v_add_u32 v{V + 4}, s{S_N0T}, v{V + 1}")            # global col (nb = 0)
        if not f32:
            # paired stores: lane group g (= l>>4) stores 8 columns at (g&1)·16 + (g>>1)·8
            self.e(f"v_lshrrev_b32 v{V + 7}, 4, v{L}")
            self.e(f"v_and_b32 v{V + E_PAIR + 2}, 1, v{V + 7}")
            self.e(f"v_lshrrev_b32 v{V + 7}, 1, v{V + 7}")
            self.e(f"v_lshlrev_b32 v{V + 7}, 3, v{V + 7}")
            self.e(f"v_lshl_add_u32 v{V + 7}, v{V + E_PAIR + 2}, 4, v{V + 7}")
            self.e(f"v_add_u32 v{V + 7}, s{T + 5}, v{V + 7}")          # paired local col
            self.e(f"v_mul_lo_u32 v{V + E_PAIR}, v{V}, s{E + 4}")
            self.e(f"v_lshl_add_u32 v{V + E_PAIR}, v{V + 7}, 1, v{V + E_PAIR}")
            if ek == "bias_act":
                self.e(f"v_mul_lo_u32 v{V + E_PAIR + 1}, v{V}, s{E + 5}")
                self.e(f"v_lshl_add_u32 v{V + E_PAIR + 1}, v{V + 7}, 1, v{V + E_PAIR + 1}")
        # edge tile in N: per-store EXEC masks
        full = self.newlab("full")
        done = self.newlab("done")
        self.e(f"s_add_u32 s{T + 6}, s{S_N0T}, {TILE}")
        self.e(f"s_cmp_le_u32 s{T + 6}, s{S_N}")
        self.e(f"s_cbranch_scc1 {full}")
        self.store_all(masked=True)
        # EXEC-masked stores may be skipped outright (no lanes): the counted wait of the next
        # tile cannot rely on them, so an edge tile drains its stores here
        self.e("s_waitcnt vmcnt(0)")
        self.e(f"s_branch {done}")
        self.lab(full)
        self.store_all(masked=False)
        self.lab(done)

    def wave_origin(self, r, c):
        """s{r} / s{c} ← this wave's row / column origin in the tile (2×2 waves of 128×128)."""
        self.e(f"s_lshr_b32 s{r}, s{S_WAVE}, 1")
        self.e(f"s_lshl_b32 s{r}, s{r}, 7")
        self.e(f"s_and_b32 s{c}, s{S_WAVE}, 1")
        self.e(f"s_lshl_b32 s{c}, s{c}, 7")

    def accf(self, mb, nb):
        return acc(mb, nb)

    def load_group(self, mb, buf):
        """Issue the epilogue loads of row block mb (old C for accumulate, aux for dact) into
        buffer `buf`; returns the VMEM instruction count."""
        V, E, T, srd = self.VE, S_E, S_T, S_CSRD
        ek = self.ek
        if ek not in ("f32acc", "bf16acc", "dact"):
            return 0
        # row offset of block mb in a temp (the loop's own offsets are per mb)
        if ek == "dact":
            self.e(f"s_mul_i32 s{T + 8}, s{E + 5}, {16 * mb}")
            self.e(f"v_add_u32 v{V + 7}, s{T + 8}, v{V + 3}")
        else:
            self.e(f"s_mul_i32 s{T + 8}, s{E + 4}, {16 * mb}")
            self.e(f"v_add_u32 v{V + 7}, s{T + 8}, v{V + 2}")
        for nb in range(self.NBW):
            if ek == "f32acc":
                d = V + 40 + 32 * buf + 4 * nb
                self.e(f"buffer_load_dwordx4 v[{d}:{d + 3}], v{V + 7}, s[{srd}:{srd + 3}], 0 offen offset:{nb * 64}")
            else:
                d = V + 40 + 16 * buf + 2 * nb
                rs = S_AUXSRD if ek == "dact" else srd
                self.e(f"buffer_load_dwordx2 v[{d}:{d + 1}], v{V + 7}, s[{rs}:{rs + 3}], 0 offen offset:{nb * 32}")
        return self.NBW

    def store_all(self, masked):
        """Per 16-row block (mb): convert / fuse / store the 8 accumulator blocks of the row.
        Full tiles pair blocks (nb, nb+1) with v_permlane16_swap so every lane stores 16 B
        (bf16: half the store instructions; the store tail is issue-bound, MI355X_MICROARCH.md);
        edge tiles store 8 B per block under per-block EXEC masks. Loads (old C, aux) of block
        mb+1 are in flight while block mb is processed; waits are counted exactly."""
        E, V, T = S_E, self.VE, S_T
        ek = self.ek
        srd = S_CSRD
        es = 4 if ek in ("f32", "f32acc") else 2
        paired = not masked and es == 2
        W = V + 8          # working registers
        has_loads = ek in ("f32acc", "bf16acc", "dact")
        issued = []        # VMEM ops in issue order: ("L", mb) loads / ("S", mb) stores
        if has_loads:
            issued += [("L", 0)] * self.load_group(0, 0)
        for mb in range(8):
            if has_loads and mb < 7:
                issued += [("L", mb + 1)] * self.load_group(mb + 1, (mb + 1) % 2)
            if has_loads:
                last = max(i for i, t in enumerate(issued) if t == ("L", mb))
                self.e(f"s_waitcnt vmcnt({min(63, len(issued) - 1 - last)})")
            buf = mb % 2
            if self.colsum:
                # rows past M hold clamped re-reads of valid A rows (loads are clamped in range):
                # the column sums take each row only when m0 + local row + 16·mb < M
                self.e(f"s_add_u32 s{T + 2}, s{S_M0T}, {16 * mb}")
                self.e(f"v_add_u32 v{self.VCS + 32}, s{T + 2}, v{V}")
                self.e(f"v_cmp_gt_u32 s[{T}:{T + 1}], s{S_M}, v{self.VCS + 32}")
            # row voffset for this mb
            self.e(f"s_mul_i32 s{T + 7}, s{E + 4}, {16 * mb}")
            self.e(f"v_add_u32 v{V + 5}, s{T + 7}, v{V + 2}")
            if paired:
                self.e(f"v_add_u32 v{V + E_PAIR + 2}, s{T + 7}, v{V + E_PAIR}")
            if ek == "bias_act":
                self.e(f"s_mul_i32 s{T + 8}, s{E + 5}, {16 * mb}")
                self.e(f"v_add_u32 v{V + 6}, s{T + 8}, v{V + 3}")
                if paired:
                    self.e(f"v_add_u32 v{V + E_PAIR + 3}, s{T + 8}, v{V + E_PAIR + 1}")
            for nb in range(self.NBW):
                c = self.accf(mb, nb)
                d = W + 4 * nb
                for j in range(4):
                    self.e(f"v_accvgpr_read_b32 v{d + j}, a{c + j}")
                if ek == "f32acc":
                    o = V + 40 + 32 * buf + 4 * nb
                    self.e(f"v_pk_add_f32 v[{d}:{d + 1}], v[{o}:{o + 1}], v[{d}:{d + 1}]")
                    self.e(f"v_pk_add_f32 v[{d + 2}:{d + 3}], v[{o + 2}:{o + 3}], v[{d + 2}:{d + 3}]")
                if masked:
                    self.e(f"v_add_u32 v{V + 7}, {nb * 16}, v{V + 4}")
                    self.e(f"v_cmp_gt_u32 vcc, s{S_N}, v{V + 7}")
                    self.e(f"s_and_saveexec_b64 s[{T + 8}:{T + 9}], vcc")
                if es == 4:
                    self.e(f"buffer_store_dwordx4 v[{d}:{d + 3}], v{V + 5}, s[{srd}:{srd + 3}], 0 offen offset:{nb * 64}")
                    issued.append(("S", mb))
                else:
                    if ek == "bias_act":
                        n_st = self.bias_act_vals(d, nb, mb, paired)
                        issued += [("S", mb)] * n_st
                    elif ek == "dact":
                        self.dact_vals(d, V + 40 + 16 * buf + 2 * nb)
                        if self.colsum:
                            cs = self.VCS + 4 * nb
                            tt = self.VCS + 34
                            if mb == 0:
                                for j in range(4):
                                    self.e(f"v_cndmask_b32_e64 v{cs + j}, 0, v{d + j}, s[{T}:{T + 1}]")
                            else:
                                for j in range(4):
                                    self.e(f"v_cndmask_b32_e64 v{tt + j}, 0, v{d + j}, s[{T}:{T + 1}]")
                                self.e(f"v_pk_add_f32 v[{cs}:{cs + 1}], v[{cs}:{cs + 1}], v[{tt}:{tt + 1}]")
                                self.e(f"v_pk_add_f32 v[{cs + 2}:{cs + 3}], v[{cs + 2}:{cs + 3}], v[{tt + 2}:{tt + 3}]")
                    elif ek == "bf16acc":
                        o = V + 40 + 16 * buf + 2 * nb
                        t = self.VTMP + 4
                        for j in (0, 2):
                            self.unpack(t, o + j // 2, 0)
                            self.unpack(t + 1, o + j // 2, 1)
                            self.e(f"v_pk_add_f32 v[{d + j}:{d + j + 1}], v[{t}:{t + 1}], v[{d + j}:{d + j + 1}]")
                    if not paired:
                        self.e(f"{self.cvt} v{d}, v{d}, v{d + 1}")
                        self.e(f"{self.cvt} v{d + 1}, v{d + 2}, v{d + 3}")
                        self.e(f"buffer_store_dwordx2 v[{d}:{d + 1}], v{V + 5}, s[{srd}:{srd + 3}], 0 offen offset:{nb * 32}")
                        issued.append(("S", mb))
                    elif nb % 2 == 1:
                        # blocks nb-1 (in d-4..d-1) and nb (d..d+3) → packed pair q..q+3, swap
                        q = d - 4
                        self.e(f"{self.cvt} v{q}, v{q}, v{q + 1}")
                        self.e(f"{self.cvt} v{q + 1}, v{q + 2}, v{q + 3}")
                        self.e(f"{self.cvt} v{q + 2}, v{d}, v{d + 1}")
                        self.e(f"{self.cvt} v{q + 3}, v{d + 2}, v{d + 3}")
                        self.e("s_nop 1")
                        self.e(f"v_permlane16_swap_b32 v{q}, v{q + 2}")
                        self.e(f"v_permlane16_swap_b32 v{q + 1}, v{q + 3}")
                        self.e(f"buffer_store_dwordx4 v[{q}:{q + 3}], v{V + E_PAIR + 2}, s[{srd}:{srd + 3}], 0 offen offset:{(nb - 1) * 32}")
                        issued.append(("S", mb))
                if masked:
                    self.e("s_mov_b64 exec, -1")
        if self.colsum:
            issued += [("S", 8)] * self.colsum_store()
        self.vm_ops = min(getattr(self, "vm_ops", 10 ** 6), len(issued))

    def colsum_store(self):
        """Column sums of this wave's 128×128 C block: the 8 row blocks were summed per lane during
        the stores (VCS), the 16 rows of a lane group are reduced with row_ror DPP adds (32
        independent registers per step: no DPP read-after-write hazard), and the group leaders
        (lane % 16 == 0) store 4 columns per 16-column block into partial row m0/128 + wave row.
        Returns the store count."""
        V, T, CS = self.VE, S_T, self.VCS
        for sh in (8, 4, 2, 1):
            for r in range(32):
                self.e(f"v_add_f32_dpp v{CS + r}, v{CS + r}, v{CS + r} row_ror:{sh} row_mask:0xf bank_mask:0xf")
        self.e("s_waitcnt lgkmcnt(0)")
        self.e("s_and_b32 s45, s45, 0xffff")
        self.e("s_mov_b32 s47, 0x20000")
        # lane byte offset: ((m0 >> 7) + wave row) · N · 4 + global col · 4
        self.e(f"s_lshr_b32 s{T}, s{S_M0T}, 7")
        self.e(f"s_lshr_b32 s{T + 1}, s{S_WAVE}, 1")
        self.e(f"s_add_u32 s{T}, s{T}, s{T + 1}")
        self.e(f"s_mul_i32 s{T}, s{T}, s{S_N}")
        self.e(f"s_lshl_b32 s{T}, s{T}, 2")
        t0, t1 = self.VTMP, self.VTMP + 1
        self.e(f"v_lshlrev_b32 v{t0}, 2, v{V + 4}")
        self.e(f"v_add_u32 v{t0}, s{T}, v{t0}")
        self.e(f"v_and_b32 v{t1}, 15, v{V_LANE}")
        self.e(f"v_cmp_eq_u32 s[{T + 2}:{T + 3}], 0, v{t1}")          # group leaders
        for nb in range(self.NBW):
            self.e("s_mov_b64 exec, -1")
            self.e(f"v_add_u32 v{t1}, {nb * 16}, v{V + 4}")
            self.e(f"v_cmp_gt_u32 vcc, s{S_N}, v{t1}")
            self.e(f"s_and_b64 exec, vcc, s[{T + 2}:{T + 3}]")
            self.e(f"buffer_store_dwordx4 v[{CS + 4 * nb}:{CS + 4 * nb + 3}], v{t0}, s[44:47], 0 offen offset:{nb * 64}")
        self.e("s_mov_b64 exec, -1")
        return self.NBW

    def store_count(self):
        """VMEM ops the epilogue issues on its shorter path (the next tile's first block-landed
        wait counts past them: they are all younger than the DMAs of the next tile's blocks 0
        and 1). Found by generating the epilogue once into a scratch buffer."""
        if not hasattr(self, "vm_ops"):
            saved = self.lines
            self.lines = []
            self.epilogue()
            self.lines = saved
        return self.vm_ops

    # -- fused activation epilogues -----------------------------------------------------------------
    def trans(self, op):
        """A transcendental op; gfx950 needs one wait state before a VALU consumes its result."""
        self.e(op)
        self.e("s_nop 0")

    def cpair(self, i):
        """Constant pair i: 0 k0, 1 k0·k1, 2 3·k0·k1, 3 2·log2(e), 4 1.0."""
        c = self.VCONST + 2 * i
        return f"v[{c}:{c + 1}]"

    def gelu2(self, x):
        """v[x:x+1] ← gelu_tanh (packed f32): x·(1 − r), r = 1 / (exp(2u) + 1), u = k0·(x + k1·x³)."""
        t = self.VTMP
        X, Tp = f"v[{x}:{x + 1}]", f"v[{t}:{t + 1}]"
        self.e(f"v_pk_mul_f32 {Tp}, {X}, {X}")
        self.e(f"v_pk_fma_f32 {Tp}, {Tp}, {self.cpair(1)}, {self.cpair(0)}")
        self.e(f"v_pk_mul_f32 {Tp}, {Tp}, {X}")
        self.e(f"v_pk_mul_f32 {Tp}, {Tp}, {self.cpair(3)}")
        self.e(f"v_exp_f32 v{t}, v{t}")
        self.trans(f"v_exp_f32 v{t + 1}, v{t + 1}")
        self.e(f"v_pk_add_f32 {Tp}, {Tp}, {self.cpair(4)}")
        self.e(f"v_rcp_f32 v{t}, v{t}")
        self.trans(f"v_rcp_f32 v{t + 1}, v{t + 1}")
        self.e(f"v_pk_fma_f32 {X}, {X}, {Tp}, {X} neg_lo:[1,0,0] neg_hi:[1,0,0]")

    def gelu_erf2(self, x):
        """v[x:x+1] ← exact GELU x·Φ(x) (packed f32; constant pairs ERF_CONSTS)."""
        ta, tb, tc = self.VTMP, self.VTMP + 2, self.VTMP + 4
        X = f"v[{x}:{x + 1}]"
        A, B, C = f"v[{ta}:{ta + 1}]", f"v[{tb}:{tb + 1}]", f"v[{tc}:{tc + 1}]"
        c = self.cpair
        for k in range(2):
            self.e(f"v_max_f32_e64 v{ta + k}, v{x + k}, -v{x + k}")
        self.e(f"v_pk_fma_f32 {A}, {A}, {c(0)}, {c(4)}")
        self.e(f"v_rcp_f32 v{ta}, v{ta}")
        self.trans(f"v_rcp_f32 v{ta + 1}, v{ta + 1}")
        self.e(f"v_pk_fma_f32 {B}, {A}, {c(1)}, {c(2)}")
        self.e(f"v_pk_fma_f32 {B}, {B}, {A}, {c(3)}")
        self.e(f"v_pk_fma_f32 {B}, {B}, {A}, {c(5)}")
        self.e(f"v_pk_fma_f32 {B}, {B}, {A}, {c(6)}")
        self.e(f"v_pk_mul_f32 {B}, {B}, {A}")
        self.e(f"v_pk_mul_f32 {C}, {X}, {X}")
        self.e(f"v_pk_mul_f32 {C}, {C}, {c(7)}")
        self.e(f"v_exp_f32 v{tc}, v{tc}")
        self.trans(f"v_exp_f32 v{tc + 1}, v{tc + 1}")
        self.e(f"v_pk_mul_f32 {B}, {B}, {C}")
        self.e(f"v_pk_add_f32 {A}, {c(4)}, {B} neg_lo:[0,1] neg_hi:[0,1]")
        for k in range(2):
            self.e(f"v_cmp_le_f32 vcc, 0, v{x + k}")
            self.e(f"v_cndmask_b32 v{tb + k}, v{tb + k}, v{ta + k}, vcc")
        self.e(f"v_pk_mul_f32 {X}, {X}, {B}")

    def gelu_grad_mul2(self, y, h):
        """v[y:y+1] ← y · gelu_tanh'(h) (packed): (1−r)(1 + 2h·r·(k0 + 3k0k1·h²))."""
        ta, tb = self.VTMP, self.VTMP + 2
        Y, H = f"v[{y}:{y + 1}]", f"v[{h}:{h + 1}]"
        A, B = f"v[{ta}:{ta + 1}]", f"v[{tb}:{tb + 1}]"
        self.e(f"v_pk_mul_f32 {A}, {H}, {H}")
        self.e(f"v_pk_fma_f32 {B}, {A}, {self.cpair(1)}, {self.cpair(0)}")
        self.e(f"v_pk_fma_f32 {A}, {A}, {self.cpair(2)}, {self.cpair(0)}")
        self.e(f"v_pk_mul_f32 {B}, {B}, {H}")
        self.e(f"v_pk_mul_f32 {B}, {B}, {self.cpair(3)}")
        self.e(f"v_exp_f32 v{tb}, v{tb}")
        self.trans(f"v_exp_f32 v{tb + 1}, v{tb + 1}")
        self.e(f"v_pk_add_f32 {B}, {B}, {self.cpair(4)}")
        self.e(f"v_rcp_f32 v{tb}, v{tb}")
        self.trans(f"v_rcp_f32 v{tb + 1}, v{tb + 1}")
        self.e(f"v_pk_mul_f32 {A}, {A}, {H}")
        self.e(f"v_pk_mul_f32 {A}, {A}, {B}")
        self.e(f"v_pk_add_f32 {B}, {self.cpair(4)}, {B} neg_lo:[0,1] neg_hi:[0,1]")
        self.e(f"v_pk_add_f32 {A}, {A}, {A}")
        self.e(f"v_pk_fma_f32 {A}, {A}, {B}, {B}")
        self.e(f"v_pk_mul_f32 {Y}, {Y}, {A}")

    def unpack(self, dst, src, j):
        """f32 v{dst} ← 16-bit half j%2 of v{src} (bf16: a shift / mask; fp16: a conversion)."""
        if self.f16:
            if j % 2 == 0:
                self.e(f"v_cvt_f32_f16 v{dst}, v{src}")
            else:
                self.e(f"v_cvt_f32_f16_sdwa v{dst}, v{src} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1")
        elif j % 2 == 0:
            self.e(f"v_lshlrev_b32 v{dst}, 16, v{src}")
        else:
            self.e(f"v_and_b32 v{dst}, 0xffff0000, v{src}")

    def bias_act_vals(self, d, nb, mb, paired=False):
        """pre = bf16(acc + bias) → aux; d ← act(pre) (f32, rounded to bf16 by the caller).
        Returns the number of aux store instructions issued."""
        t = self.VTMP + 4
        p = self.VE + E_AUXP + 2 * (nb % 2) if paired else self.VTMP + 6
        for j in (0, 2):
            self.unpack(t, self.VBIAS + 2 * nb + j // 2, 0)
            self.unpack(t + 1, self.VBIAS + 2 * nb + j // 2, 1)
            self.e(f"v_pk_add_f32 v[{d + j}:{d + j + 1}], v[{t}:{t + 1}], v[{d + j}:{d + j + 1}]")
        if not self.store_aux:
            return 0
        self.e(f"{self.cvt} v{p}, v{d}, v{d + 1}")
        self.e(f"{self.cvt} v{p + 1}, v{d + 2}, v{d + 3}")
        n = 0
        if not paired:
            self.e(f"buffer_store_dwordx2 v[{p}:{p + 1}], v{self.VE + 6}, s[{S_AUXSRD}:{S_AUXSRD + 3}], 0 offen offset:{nb * 32}")
            n = 1
        if self.act != 0:
            for j in range(4):
                self.unpack(d + j, p + j // 2, j)
            for j in (0, 2):
                if self.act == 1:
                    self.gelu2(d + j)
                elif self.act == 2:
                    self.gelu_erf2(d + j)
                else:
                    self.e(f"v_max_f32 v{d + j}, 0, v{d + j}")
                    self.e(f"v_max_f32 v{d + j + 1}, 0, v{d + j + 1}")
        if paired and nb % 2 == 1:
            q = self.VE + E_AUXP
            self.e("s_nop 1")
            self.e(f"v_permlane16_swap_b32 v{q}, v{q + 2}")
            self.e(f"v_permlane16_swap_b32 v{q + 1}, v{q + 3}")
            self.e(f"buffer_store_dwordx4 v[{q}:{q + 3}], v{self.VE + E_PAIR + 3}, s[{S_AUXSRD}:{S_AUXSRD + 3}], 0 offen offset:{(nb - 1) * 32}")
            n = 1
        return n

    def dact_vals(self, d, auxreg):
        h = self.VTMP + 4
        for j in (0, 2):
            self.unpack(h, auxreg + j // 2, 0)
            self.unpack(h + 1, auxreg + j // 2, 1)
            if self.act == 1:
                self.gelu_grad_mul2(d + j, h)
            else:
                for k in range(2):
                    self.e(f"v_cmp_lt_f32 vcc, 0, v{h + k}")
                    self.e(f"v_cndmask_b32 v{d + j + k}, 0, v{d + j + k}, vcc")

    # -- text ----------------------------------------------------------------------------------------
    def text(self):
        self.lines = []
        if self.persistent:
            self.body_persistent()
        else:
            self.body()
        n = self.name
        head = [
            "\t.text",
            f"\t.globl {n}",
            "\t.p2align 8",
            f"\t.type {n},@function",
            f"{n}:",
        ]
        tail = [
            f".L{n}_end:",
            f"\t.size {n}, .L{n}_end-{n}",
            "\t.rodata",
            "\t.p2align 6",
            f"\t.amdhsa_kernel {n}",
            f"\t\t.amdhsa_group_segment_fixed_size {self.lds_bytes}",
            "\t\t.amdhsa_private_segment_fixed_size 0",
            f"\t\t.amdhsa_kernarg_size {ARGS_SIZE}",
            "\t\t.amdhsa_user_sgpr_count 2",
            "\t\t.amdhsa_user_sgpr_kernarg_segment_ptr 1",
            "\t\t.amdhsa_system_sgpr_workgroup_id_x 1",
            "\t\t.amdhsa_system_vgpr_workitem_id 0",
            f"\t\t.amdhsa_next_free_vgpr {self.acc_off + self.n_agpr}",
            f"\t\t.amdhsa_next_free_sgpr {NSGPR}",
            f"\t\t.amdhsa_accum_offset {self.acc_off}",
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
        n = self.name
        return f"""  - .args:
      - .offset:         0
        .size:           {ARGS_SIZE}
        .value_kind:     by_value
    .group_segment_fixed_size: {self.lds_bytes}
    .kernarg_segment_align: 8
    .kernarg_segment_size: {ARGS_SIZE}
    .max_flat_workgroup_size: {self.wg_size}
    .name:           {n}
    .private_segment_fixed_size: 0
    .sgpr_count:     {NSGPR + 6}
    .sgpr_spill_count: 0
    .symbol:         {n}.kd
    .vgpr_count:     {self.acc_off + self.n_agpr}
    .agpr_count:     {self.n_agpr}
    .vgpr_spill_count: 0
    .wavefront_size: 64
"""


LAYOUTS = {"nt": (True, True), "tn": (False, False), "nn": (True, False), "tt": (False, True)}
EPILOGUES = ("bf16", "bf16acc", "f32", "f32acc")


FUSED = ("bias", "biasgelu", "biasrelu", "dgelu", "drelu", "biasnx", "biasgeluerf", "dgelucs", "drelucs")


def variants():
    """(name, A K-contiguous, B K-contiguous, epilogue, persistent, fp16). ``_p_`` kernels are the
    persistent ones (nk even and >= 4); the others take one tile per workgroup (any nk >= 2).
    ``_f16`` kernels take IEEE fp16 operands (and write fp16 where the bf16 kernel writes bf16)."""
    for f16 in (False, True):
        sfx = "_f16" if f16 else ""
        for pers in (False, True):
            tag = "p_" if pers else ""
            for lay in ("nt", "tn", "nn", "tt"):
                for ek in EPILOGUES:
                    yield f"piamd_agemm_{tag}{lay}_{ek}{sfx}", LAYOUTS[lay][0], LAYOUTS[lay][1], ek, pers, f16
            for ek in FUSED:  # fused epilogues: forward / data-gradient products (both K-contiguous)
                yield f"piamd_agemm_{tag}nt_{ek}{sfx}", True, True, ek, pers, f16


def this_module():
    """This generator as a module object (also when loaded by path without sys.modules)."""
    import types
    m = sys.modules.get(__name__)
    if m is not None and getattr(m, "Kernel", None) is Kernel:
        return m
    return types.SimpleNamespace(**globals())


def generate() -> str:
    ks = [Kernel(n, a, b, ek, pers, f16) for n, a, b, ek, pers, f16 in variants()]
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
