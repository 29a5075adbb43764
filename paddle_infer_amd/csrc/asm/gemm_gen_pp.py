"""Ping-pong variant of the gfx950 assembly GEMM (``agemm_q``): 8 waves, TWO per SIMD, for the NT
products (A [M][K], B [N][K], both K-contiguous: forward and data-gradient linears).

Why: the 4-wave kernel (`gemm_gen.py`) runs one wave per SIMD, so every LDS-DMA issue (≈60 cycles
among MFMAs, MI355X_MICROARCH.md constants) and every barrier wait idles that SIMD's matrix pipe
— ≈26 % of its cycles (74 % MFMA busy, `profiles/pmc_agemm_nt_vs_tn_r3.txt`). Here the two waves
of a SIMD alternate roles every phase: one runs a 32-MFMA compute phase while its partner reads
the next fragments from LDS and issues its share of the LDS-DMAs; an `s_barrier` swaps them.

Kernel:

* 256×256 output tile per workgroup of 8 waves; wave w owns rows (w&1)·128 … +127 and columns
  (w>>1)·64 … +63: 8×4 blocks of `v_mfma_f32_16x16x32_{bf16,f16}` (operands swapped as in the
  4-wave kernel, so a lane owns one output row and 4 consecutive columns), 128 AGPRs.
* K-block = 32 (one compute phase). LDS ring of 4 stages × (A 16 KiB + B 16 KiB) = 128 KiB; block
  t lives in stage t%4. KC image: [256 rows][64 B], 16-B chunk c of row r at c ^ F((r>>2)&3),
  F(q) = ((q0^q1)<<1)|q1 — conflict-free `ds_read_b128` for the gfx950 lane groups (checked in
  tests/test_agemm_layout_cpu.py). LDS-DMA pieces are 16 rows × 64 B (1 KiB); wave w fills
  pieces w and w+8 of each operand (4 DMAs per K-block per wave).
* Group G0 = waves 0-3, G1 = waves 4-7 (waves w and w+4 share a SIMD). Phase 2t: G0 computes
  block t while G1 reads its block-t fragments and issues its DMAs of block t+3; phase 2t+1: G1
  computes block t while G0 reads block t+1 and issues block t+4. Every load phase ends with a
  counted ``vmcnt(8)`` (two K-blocks of this wave's DMAs stay in flight across the barrier) and
  ``lgkmcnt(0)``; a stage is re-filled only after both groups' reads of it retired.
* Persistent over work units like the 4-wave kernel: the last loop iteration switches the DMA
  stream to the next unit's first blocks (same ring positions, nk32 % 4 == 0), and each group
  writes its 128×64 part of the tile (the 4-wave kernel's epilogues, fused or not) at the head of
  the load phase after its last compute phase, while the partner computes.

Contract (host: `csrc/kernels/agemm_host.hip`): NT layout, K per unit % 128 == 0 and ≥ 256
(nk even ≥ 4 in 64-blocks), everything else as the 4-wave kernel.
"""
from __future__ import annotations

import sys

BKQ = 32                       # K per block (one compute phase)
NSTAGE = 4
QSTAGE = 32768                 # bytes per stage (A 16 KiB + B 16 KiB)
QOP = 16384
QLDS = NSTAGE * QSTAGE         # 128 KiB
# VGPR map (128 architectural VGPRs; AGPRs a0..a127 hold the accumulators)
Q_DMA = 2                      # v2 A piece w, v3 A piece w+8, v4 B piece w, v5 B piece w+8
Q_RB = 6                       # v6 A stages 0/1, v7 A stages 2/3, v8 B 0/1, v9 B 2/3
Q_FRAG = 48                    # A fragments v48..79 (8 × 4), B v80..95 (4 × 4)
Q_VE = 10                      # epilogue frame v10..v117 (the fragments are dead there)
Q_ACC_OFF = 128
S_LDSQ = 60                    # this wave's LDS-DMA base (w·1024)


def qf(q):
    """Row-quad → chunk XOR of the KC image (rows r: q = (r>>2)&3)."""
    q0, q1 = q & 1, (q >> 1) & 1
    return ((q0 ^ q1) << 1) | q1


def q_dma(j, w, L):
    """Piece j (0/1) of wave w, lane L → (tile row, global 16-B chunk, LDS byte in the operand)."""
    p = w + 8 * j
    r = L >> 2
    row = 16 * p + r
    g = (L & 3) ^ qf((r >> 2) & 3)
    return row, g, p * 1024 + 16 * L


def q_read(R0, blk, l):
    """Fragment read (ds_read_b128) of lane l: rows R0 + 16·blk + (l&15), K chunk l>>4 → LDS byte
    in the operand image."""
    r = R0 + 16 * blk + (l & 15)
    c = (l >> 4) ^ qf((r >> 2) & 3)
    return r * 64 + c * 16


S_QOFF = {2: 36, 3: 37, 4: 38, 5: 39, 6: 48}   # SGPRs holding DMA soffsets 64k (k ≥ 2; 0 / 64 inline)


def qoff(k):
    return str(64 * k) if k < 2 else f"s{S_QOFF[k]}"


def make_kernel_pp(gg):
    """The ping-pong kernel class, built on the 4-wave generator module ``gg`` (its prologue, tile
    walk, descriptors and epilogues)."""
    Base = gg.Kernel

    class KPP(Base):
        def __init__(self, name, ek, f16=False, prio=False, dma_first=False):
            super().__init__(name, True, True, ek, persistent=True, f16=f16)
            # schedule options (A/B variants): s_setprio 1 around each compute phase's MFMAs;
            # a load phase issuing its DMAs before its fragment reads
            self.prio, self.dma_first = prio, dma_first
            self.VE = Q_VE
            self.VBIAS, self.VTMP, self.VCONST = self.VE + gg.E_BIAS, self.VE + gg.E_TMP, self.VE + gg.E_CONST
            self.NBW = 4
            self.lds_bytes, self.wg_size, self.acc_off, self.n_agpr = QLDS, 512, Q_ACC_OFF, 128
            assert self.VCONST + 16 <= Q_ACC_OFF
            self.trace = None           # schedule events (tests/test_agemm_layout_cpu.py checker)

        def ev(self, *x):
            if self.trace is not None:
                self.trace.append(x)

        def wait_vm(self, n):
            self.e(f"s_waitcnt vmcnt({min(63, n)})")
            self.ev("vmcnt", min(63, n))

        def wait_lgkm0(self):
            self.e("s_waitcnt lgkmcnt(0)")
            self.ev("lgkm0")

        def barrier(self):
            self.e("s_barrier")
            self.ev("bar")

        def emit_reads(self, stage):
            self.ev("read", stage)
            for r in self.reads(stage):
                self.e(r)

        def emit_dma(self, d):
            m0, ld, stage, k = d
            self.e(m0)
            self.e("s_nop 0")
            self.e(ld)
            self.ev("dma", stage, k)

        def epilogue_ev(self):
            self.epilogue()
            self.ev("epi", self.store_count())

        # -- geometry ------------------------------------------------------------------------------
        def wave_origin(self, r, c):
            self.e(f"s_and_b32 s{r}, s{gg.S_WAVE}, 1")
            self.e(f"s_lshl_b32 s{r}, s{r}, 7")                # (w&1)·128
            self.e(f"s_lshr_b32 s{c}, s{gg.S_WAVE}, 1")
            self.e(f"s_lshl_b32 s{c}, s{c}, 6")                # (w>>1)·64

        def accf(self, mb, nb):
            return 4 * (mb * 4 + nb)

        def fa(self, mb):
            return Q_FRAG + 4 * mb

        def fb(self, nb):
            return Q_FRAG + 32 + 4 * nb

        # -- operand setup (KC only) -----------------------------------------------------------------
        def setup_operand(self, op, T, t0, full=True, part=None):
            ptr = gg.S_A if op == 0 else gg.S_B
            tot = gg.S_ABYTES if op == 0 else gg.S_BBYTES
            ld = gg.S_LDA if op == 0 else gg.S_LDB
            srd = gg.S_SRDA if op == 0 else gg.S_SRDB
            rem = gg.S_REMA if op == 0 else gg.S_REMB
            step = gg.S_STEPA if op == 0 else gg.S_STEPB
            lim = gg.S_M if op == 0 else gg.S_N
            a, b = T + 1, T + 2
            self.e(f"s_mul_i32 s{a}, s{t0}, s{ld}")
            self.e(f"s_mul_hi_u32 s{b}, s{t0}, s{ld}")
            self.e(f"s_lshl_b32 s{T + 3}, s{T}, 1")
            self.e(f"s_add_u32 s{a}, s{a}, s{T + 3}")
            self.e(f"s_addc_u32 s{b}, s{b}, 0")
            self.e(f"s_mov_b32 s{step}, {4 * BKQ * 2}")          # one loop iteration = 4 blocks
            self.e(f"s_mov_b32 s{step + 1}, 0")
            if part is not None:
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
            V, L = gg.V_T, gg.V_LANE
            # DMA voffsets: rows 16(w + 8j) + (L>>2) (clamped), chunk (L&3) ^ F(L>>4)
            self.e(f"v_lshrrev_b32 v{V}, 4, v{L}")                      # q = L>>4
            self.e(f"v_and_b32 v{V + 1}, 1, v{V}")
            self.e(f"v_lshrrev_b32 v{V + 2}, 1, v{V}")                  # q1
            self.e(f"v_xor_b32 v{V + 1}, v{V + 1}, v{V + 2}")
            self.e(f"v_lshl_or_b32 v{V + 1}, v{V + 1}, 1, v{V + 2}")    # F(q)
            self.e(f"v_and_b32 v{V + 2}, 3, v{L}")
            self.e(f"v_xor_b32 v{V + 1}, v{V + 1}, v{V + 2}")
            self.e(f"v_lshlrev_b32 v{V + 1}, 4, v{V + 1}")              # chunk·16
            self.e(f"v_lshrrev_b32 v{V + 2}, 2, v{L}")                  # L>>2
            self.e(f"s_lshl_b32 s{T + 3}, s{gg.S_WAVE}, 4")              # 16w
            self.e(f"v_add_u32 v{V + 2}, s{T + 3}, v{V + 2}")
            self.e(f"s_sub_u32 s{T + 4}, s{lim}, s{t0}")
            self.e(f"s_sub_u32 s{T + 4}, s{T + 4}, 1")                   # last valid local row
            for j in range(2):
                vd = Q_DMA + 2 * op + j
                self.e(f"v_add_u32 v{V + 3}, {128 * j}, v{V + 2}")
                self.e(f"v_min_u32 v{V + 3}, s{T + 4}, v{V + 3}")
                self.e(f"v_mad_u32_u24 v{vd}, v{V + 3}, s{ld}, v{V + 1}")
            if not full:
                return
            if op == 0:
                self.e(f"s_lshl_b32 s{S_LDSQ}, s{gg.S_WAVE}, 10")        # w·1024
            # read base: (R0 + (l&15))·64 + ((l>>4) ^ F(((l&15)>>2)&3))·16 + op·16 KiB
            self.e(f"v_and_b32 v{V}, 15, v{L}")
            self.e(f"v_lshrrev_b32 v{V + 1}, 2, v{V}")                  # q = (l&15)>>2
            self.e(f"v_and_b32 v{V + 2}, 1, v{V + 1}")
            self.e(f"v_lshrrev_b32 v{V + 3}, 1, v{V + 1}")
            self.e(f"v_xor_b32 v{V + 2}, v{V + 2}, v{V + 3}")
            self.e(f"v_lshl_or_b32 v{V + 2}, v{V + 2}, 1, v{V + 3}")    # F(q)
            self.e(f"v_lshrrev_b32 v{V + 3}, 4, v{L}")
            self.e(f"v_xor_b32 v{V + 2}, v{V + 2}, v{V + 3}")
            self.e(f"v_lshlrev_b32 v{V + 2}, 4, v{V + 2}")              # chunk·16
            if op == 0:
                self.e(f"s_and_b32 s{T + 3}, s{gg.S_WAVE}, 1")
                self.e(f"s_lshl_b32 s{T + 3}, s{T + 3}, 7")              # R0 = (w&1)·128
            else:
                self.e(f"s_lshr_b32 s{T + 3}, s{gg.S_WAVE}, 1")
                self.e(f"s_lshl_b32 s{T + 3}, s{T + 3}, 6")              # R0 = (w>>1)·64
            self.e(f"v_add_u32 v{V}, s{T + 3}, v{V}")
            self.e(f"v_lshl_add_u32 v{V}, v{V}, 6, v{V + 2}")
            rb = Q_RB + 2 * op
            self.e(f"v_add_u32 v{rb}, {op * QOP}, v{V}")
            self.e(f"v_add_u32 v{rb + 1}, {op * QOP + 2 * QSTAGE}, v{V}")

        # -- phases ----------------------------------------------------------------------------------
        def compute(self, zero=False):
            self.ev("compute", zero)
            for mb in range(8):
                for nb in range(4):
                    c = self.accf(mb, nb)
                    src2 = "0" if zero else f"a[{c}:{c + 3}]"
                    self.e(f"{self.mfma_op} a[{c}:{c + 3}], v[{self.fb(nb)}:{self.fb(nb) + 3}], "
                           f"v[{self.fa(mb)}:{self.fa(mb) + 3}], {src2}")

        def reads(self, stage):
            """The 12 fragment reads of the block in `stage` (B first: every MFMA row needs all
            four B fragments)."""
            ops = []
            hi, off = stage // 2, (stage % 2) * QSTAGE
            for nb in range(4):
                d = self.fb(nb)
                ops.append(f"ds_read_b128 v[{d}:{d + 3}], v{Q_RB + 2 + hi} offset:{off + 1024 * nb}")
            for mb in range(8):
                d = self.fa(mb)
                ops.append(f"ds_read_b128 v[{d}:{d + 3}], v{Q_RB + hi} offset:{off + 1024 * mb}")
            return ops

        def dmas(self, stage, k):
            """This wave's 4 LDS-DMAs of one block into `stage`, 64·k bytes along K past the
            current descriptors (soffset: an instruction offset would move the LDS address too):
            [(m0 line, load line)]."""
            ops = []
            for op in (0, 1):
                srd = gg.S_SRDA if op == 0 else gg.S_SRDB
                for j in range(2):
                    lds = stage * QSTAGE + op * QOP + j * 8192
                    ops.append((f"s_add_u32 m0, s{S_LDSQ}, {lds}",
                                f"buffer_load_dwordx4 v{Q_DMA + 2 * op + j}, s[{srd}:{srd + 3}], {qoff(k)} offen lds",
                                stage, k))
            return ops

        def load_phase(self, read_stage, dma, vm, pre=None, split=None):
            """Reads of `read_stage` interleaved with the DMAs (list from `dmas`), then the counted
            waits; ``pre`` emits code first (epilogue / next-unit setup); ``split`` = (k, fn): run fn
            before DMA k (descriptor switch between this block's DMAs)."""
            if pre is not None:
                pre()
            rd = self.reads(read_stage)
            self.ev("read", read_stage)
            di = 0
            if self.dma_first and split is None:
                for d in dma:
                    self.emit_dma(d)
                di = len(dma)
            for i, r in enumerate(rd):
                self.e(r)
                if i % 3 == 2 and di < len(dma):
                    if split is not None and split[0] == di:
                        split[1]()
                    self.emit_dma(dma[di])
                    di += 1
            while di < len(dma):
                if split is not None and split[0] == di:
                    split[1]()
                self.emit_dma(dma[di])
                di += 1
            self.wait_vm(vm)
            self.wait_lgkm0()
            self.barrier()

        def compute_phase(self, zero=False):
            if self.prio:
                self.e("s_setprio 1")
            self.compute(zero)
            if self.prio:
                self.e("s_setprio 0")
            self.barrier()

        def advance(self, op):
            (self.srd_advance(gg.S_SRDA, gg.S_REMA, gg.S_STEPA) if op == 0
             else self.srd_advance(gg.S_SRDB, gg.S_REMB, gg.S_STEPB))

        def adv_both(self):
            self.advance(0)
            self.advance(1)
            self.ev("adv")

        # one loop iteration = blocks 4i..4i+3 (stages 0..3)
        def iter_g0(self, first=False, last=False, vmx=(0, 0, 0, 0), switch=None, epi=None):
            if not last:
                self.adv_both()           # descriptors → body i+1 (blocks t+4)
            for j in range(4):
                self.compute_phase(zero=first and j == 0)
                pre = None
                if last and j == 0:
                    pre = switch
                if last and j == 3:
                    pre = epi
                self.load_phase((j + 1) % 4, self.dmas(j, j), 8 + vmx[j], pre=pre)

        def iter_g1(self, first=False, last=False, vmx=(0, 0, 0, 0), switch=None):
            if not first:
                self.adv_both()           # descriptors → body i (blocks t+3 at 192 + 64j)
            for j in range(4):
                if last and j >= 1:
                    dma = self.dmas((j + 3) % 4, j - 1)
                else:
                    dma = self.dmas((j + 3) % 4, 3 + j)
                split = (0, switch) if (last and j == 1) else None
                self.load_phase(j, dma, 8 + vmx[j], split=split)
                self.compute_phase(zero=first and j == 0)

        def next_unit(self):
            """Next work unit → S_NM0/S_NN0/S_NPART and the DMA descriptors (or null descriptors
            when none is left; S_NVALID tells the tail)."""
            T = gg.S_T
            nxt, nonext, ready = self.newlab("next"), self.newlab("nonext"), self.newlab("ready")
            self.e(f"s_add_u32 s{T + 9}, s{gg.S_ROUND}, 1")
            self.e(f"s_mul_i32 s{T + 9}, s{T + 9}, s{gg.S_GRID}")
            self.e(f"s_add_u32 s{gg.S_NVALID}, s{gg.S_U0}, s{T + 9}")
            self.e(f"s_cmp_lt_u32 s{gg.S_NVALID}, s{gg.S_NWG}")
            self.e(f"s_cbranch_scc0 {nonext}")
            self.ev("switch")
            self.tile_coords(gg.S_NVALID, gg.S_NM0, gg.S_NN0, gg.S_NPART)
            self.setup_tile(gg.S_NM0, gg.S_NN0, gg.S_NPART, full=False)
            self.e(f"s_mov_b32 s{gg.S_NVALID}, 1")
            self.e(f"s_branch {ready}")
            self.lab(nonext)
            for r in (gg.S_SRDA + 2, gg.S_SRDB + 2, gg.S_REMA, gg.S_REMA + 1, gg.S_REMB, gg.S_REMB + 1,
                      gg.S_STEPA, gg.S_STEPA + 1, gg.S_STEPB, gg.S_STEPB + 1, gg.S_NVALID):
                self.e(f"s_mov_b32 s{r}, 0")
            self.lab(ready)

        def to_next(self, lend):
            self.e(f"s_cmp_eq_u32 s{gg.S_NVALID}, 0")
            self.e(f"s_cbranch_scc1 {lend}")
            self.e(f"s_mov_b32 s{gg.S_M0T}, s{gg.S_NM0}")
            self.e(f"s_mov_b32 s{gg.S_N0T}, s{gg.S_NN0}")
            self.e(f"s_mov_b32 s{gg.S_PART}, s{gg.S_NPART}")
            self.e(f"s_add_u32 s{gg.S_ROUND}, s{gg.S_ROUND}, 1")

        def loop_counter(self):
            # middle iterations = nk/2 - 2 (nk = 64-blocks; one iteration = 2 of them)
            self.e(f"s_lshr_b32 s{gg.S_LOOP}, s{gg.S_NK}, 1")
            self.e(f"s_sub_i32 s{gg.S_LOOP}, s{gg.S_LOOP}, 2")

        def middle(self, body):
            lbeg, lend = self.newlab("loop"), self.newlab("loopend")
            self.e(f"s_cmp_le_i32 s{gg.S_LOOP}, 0")
            self.e(f"s_cbranch_scc1 {lend}")
            self.lab(lbeg)
            body()
            self.e(f"s_sub_i32 s{gg.S_LOOP}, s{gg.S_LOOP}, 1")
            self.e(f"s_cmp_gt_i32 s{gg.S_LOOP}, 0")
            self.e(f"s_cbranch_scc1 {lbeg}")
            self.lab(lend)

        def prime_g0(self):
            for t in range(4):                       # blocks 0..3
                for d in self.dmas(t, t):
                    self.emit_dma(d)
            self.wait_vm(12)
            self.barrier()
            self.emit_reads(0)
            self.wait_vm(8)
            self.wait_lgkm0()
            self.barrier()

        def prime_g1(self):
            for t in range(3):                       # blocks 0..2
                for d in self.dmas(t, t):
                    self.emit_dma(d)
            self.wait_vm(8)
            self.barrier()
            self.barrier()

        def schedule_trace(self, nk64, ntiles):
            """Event streams of G0 and G1 for ``ntiles`` consecutive units of nk64 64-blocks, in
            execution order (the same emitters as the kernel text; for the CPU schedule checker)."""
            saved, self.lines = self.lines, []
            S = self.store_count()
            out = []
            L = nk64 // 2
            for g in (0, 1):
                self.trace = []
                it = self.iter_g0 if g == 0 else self.iter_g1
                (self.prime_g0 if g == 0 else self.prime_g1)()
                for tile in range(ntiles):
                    vmx = (0, 0, 0, 0) if tile == 0 else ((S, 0, 0, 0) if g == 0 else (S, S, 0, 0))
                    it(first=True, vmx=vmx)
                    for _ in range(L - 2):
                        it()
                    if g == 0:
                        it(last=True, vmx=(0, 0, 0, S), switch=lambda: self.ev("switch"),
                           epi=lambda: self.ev("epi", S))
                    else:
                        it(last=True, switch=lambda: self.ev("switch"))
                        self.ev("epi", S)
                out.append(self.trace)
            self.trace = None
            self.lines = saved
            return out

        def body_persistent(self):
            self.prologue()
            lend = self.newlab("end")
            g1 = self.newlab("g1")
            self.e(f"s_cmp_ge_u32 s{gg.S_U0}, s{gg.S_NWG}")
            self.e(f"s_cbranch_scc1 {lend}")
            self.tile_coords(gg.S_U0, gg.S_M0T, gg.S_N0T, gg.S_PART)
            self.setup_tile(gg.S_M0T, gg.S_N0T, gg.S_PART)
            for k, sr in S_QOFF.items():
                self.e(f"s_mov_b32 s{sr}, {64 * k}")
            S = self.store_count()
            self.e(f"s_cmp_ge_u32 s{gg.S_WAVE}, 4")
            self.e(f"s_cbranch_scc1 {g1}")
            # ---------------- G0 (waves 0-3)
            self.prime_g0()
            ltile0, lsec0 = self.newlab("tile0"), self.newlab("sec0")
            self.iter_g0(first=True)
            self.e(f"s_branch {lsec0}")
            self.lab(ltile0)
            self.iter_g0(first=True, vmx=(S, 0, 0, 0))
            self.lab(lsec0)
            self.loop_counter()
            self.middle(lambda: self.iter_g0())
            self.iter_g0(last=True, vmx=(0, 0, 0, S), switch=self.next_unit, epi=self.epilogue_ev)
            self.to_next(lend)
            self.e(f"s_branch {ltile0}")
            # ---------------- G1 (waves 4-7)
            self.lab(g1)
            self.prime_g1()
            ltile1, lsec1 = self.newlab("tile1"), self.newlab("sec1")
            self.iter_g1(first=True)
            self.e(f"s_branch {lsec1}")
            self.lab(ltile1)
            self.iter_g1(first=True, vmx=(S, S, 0, 0))
            self.lab(lsec1)
            self.loop_counter()
            self.middle(lambda: self.iter_g1())
            self.iter_g1(last=True, switch=self.next_unit)
            self.epilogue_ev()
            self.to_next(lend)
            self.e(f"s_branch {ltile1}")
            self.lab(lend)
            self.e("s_waitcnt vmcnt(0)")
            self.e("s_endpgm")

    return KPP


def variants_pp(gg):
    """NT ping-pong kernels: every plain and fused epilogue, bf16 and fp16; plus schedule A/B
    variants of the plain bf16 kernel (``_v1`` setprio, ``_v2`` DMAs first, ``_v3`` both)."""
    for f16 in (False, True):
        sfx = "_f16" if f16 else ""
        for ek in gg.EPILOGUES + gg.FUSED:
            yield f"piamd_agemm_q_nt_{ek}{sfx}", ek, f16, {}
    for v, kw in ((1, {"prio": True}), (2, {"dma_first": True}), (3, {"prio": True, "dma_first": True})):
        yield f"piamd_agemm_q_nt_bf16_v{v}", "bf16", False, kw


if __name__ == "__main__":
    sys.exit("generated through gemm_gen.py")
