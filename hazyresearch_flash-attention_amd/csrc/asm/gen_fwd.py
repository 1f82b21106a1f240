#!/usr/bin/env python3
"""gen_fwd.py — generator of the hand-scheduled gfx950 FlashAttention forward kernel (head_dim <= 64).

Writes one AMDGPU assembly file (code, kernel descriptor, metadata) for one dtype:

    python gen_fwd.py --dtype bf16 --out fa_fwd_d64_bf16.s

What the kernel computes is the forward of fa_fwd_kernel.h (and of the reference,
csrc/flash_attn/src/fmha_fprop_kernel_1xN.h:453-681): for each (batch, head) and query row,
O = softmax(scale * Q K^T) V over the keys of the row's sequence, and the natural-log LSE.
Non-causal, no dropout: the shapes this kernel serves; the launcher keeps the HIP kernels for
the others. Var-len sequences come through cu_seqlens exactly as in the HIP kernel.

Why a generator: the D=64 forward is VALU-issue bound (per 32x64 score tile: 32 exp, 32 fma,
16 cvt, 18 max3 against 16 MFMAs), so the instruction stream is placed by hand, the way
cdna_hip_programming.md (Appendix B, "4-wave, one-wave-per-SIMD") describes:

  * workgroup = 4 waves = 256 query rows, one wave per SIMD owning the whole register file;
    each wave holds two 32-row query blocks A and B (every K/V fragment read feeds two MFMAs);
  * S^T = K Q^T with v_mfma_f32_32x32x16 (lane = query row), O^T += V^T P^T with P straight
    from registers, V^T fragments by ds_read_b64_tr_b16 (same fragment maps as fa_common.h);
  * per 64-key tile two phases of 20 MFMAs: phase 1 = QK_B(j) + PV_B(j-1) beside block A's
    softmax of tile j, phase 2 = QK_A(j+1) + PV_A(j) beside block B's softmax of tile j;
  * row sums by a 16x16x32 MFMA of the 16-bit P against a 0/1 indicator matrix (4 per tile and
    block, 16-cycle MFMAs) instead of 32 v_add_f32: the sum then covers the rounded P that the
    P.V product uses;
  * K/V tiles HBM -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds) into a 4-slot ring with a
    3-tile prefetch distance, counted vmcnt, one s_barrier per tile;
  * the deferred rescale (T13) of fa_fwd_kernel.h: the running max moves only when a tile max
    passes it by 2^8 (one compare per tile; the rescale itself is an out-of-line block);
  * fillers are distributed over the MFMA gaps by issue cost; a hazard pass inserts the
    gfx950 wait states (measured from hipcc's own hazard recognizer: MFMA 32x32 -> read 12,
    16x16 -> read 8, VALU -> MFMA 2, trans -> VALU 1, VALU -> permlane 2, m0 -> LDS-DMA 1)
    and counted lgkmcnt waits.

Nothing here writes through the scalar data cache: all stores are vector buffer stores.
"""
import argparse
import copy
import math
import os
import sys

# ------------------------------------------------------------------------------------------
# geometry
# ------------------------------------------------------------------------------------------
D = 64                 # head-dim tile: 64 (head_dim in (32, 64], zero-padded by the loads) or 128
                       # (head_dim == 128); configure() sets the dependent constants and registers
BN = 64                # keys per tile
R = 4                  # LDS ring slots (K and V each)
DIST = 3               # DMA prefetch distance in tiles (tile t issues K(t+1+DIST), V(t+DIST))
U = 4                  # loop unroll = lcm(R, 2 register buffers)
TILE = BN * D * 2      # bytes per tile image
KREG = 0
VREG = R * TILE
LDS_BYTES = 2 * R * TILE
VREADS_P1 = True       # V^T fragment reads of tile j in phase 1 (one phase ahead of PV_A(j))
SM_PIPE = False        # software-pipelined fma -> exp -> cvt order inside the softmax
DMA_P2 = False         # all four DMA pieces of a tile in phase 2 (K's with V's)
SPEC = True            # exps against the current max; rescale test branches at the phase end
ORDET = True           # rescale test = top exponent bit of the packed P (any P >= 2) by an OR tree;
#                        the max tree moves into the out-of-line rescale block
ORDET_DELTA = {'bf16': 8.0, 'f16': 4.0}   # a rescale sets m = tile max * c + delta (P <= 2^-delta)
# (f16: P's smallest normal is 2^-14, so a larger delta turns more of a row's small weights subnormal; 4
# instead of round 3's 2 measured C2 -10 % (fewer rescales) at unchanged fp16 errors: DESIGN.md 4.0d)
EXP_LAG = 4            # exp_stream: fma(i) -> exp(i) distance (instructions)
CVT_LAG = 4            # exp_stream: exp -> cvt distance
MC_BANKS = False       # fma reads m*c from one of 4 copies in a VGPR bank other than its S operand
PRESCALE = False       # Q pre-multiplied by c (rounded to the 16-bit type once per block) and S^T seeded
#                        with -m c (16 registers per block): the softmax is exp2(S), no per-element fma
SEED0 = 4096.0         # initial -m c: every tile 0 fires the rescale unless all its scores are < -3968
V_SEED = {'A': 212, 'B': 228}   # PRESCALE: -m c broadcast over the 16 registers of an S^T tile
KFIRST = True          # phase 1: K(t+1) fragment reads ahead of the V^T reads (D = 64)
KFIRST_LO = 2          # softmax-stream position of the first K read with KFIRST
LGKM_XPHASE = True     # counted lgkmcnt waits may count LDS reads of the previous phase
KSPLIT_LAG = 3         # ... each at least this many MFMAs ahead of its QK MFMA
KSPLIT = 3             # K(t+1) fragment reads moved from phase 1 to the start of phase 2 (D = 64)
FIRST_MAX = True       # prologue: tile 0's row max sets the starting shift (no rescale at tile 0)
LAST_UNMASKED = True   # last tile: unmasked copy when every row sees the whole tile
MFMA_ZERO = True       # prologue: O, row sums, V buffer zeroed by MFMAs of a zero operand
ORDET_ANDOR = True     # ORDET: the last P word enters the test by one v_and_or_b32 (mask in V_MTHR)
PHASE_TAIL = 1         # ORDET test issued before the phase's last PHASE_TAIL MFMAs, its branch after them
ORDET_BITOP3 = False   # ORDET: (T | P15) & M by one v_bitop3_b32 instead of v_and + v_and_or: one VALU fewer
#                        per block and tile, measured 0.3-0.4 % SLOWER (profiles/r06/bitop3_ab.txt): A/B only


def soff_walk():
    """SOFF_WALK applies to every form but the persistent forms with the next-block K/V tail
    (PERSIST_KV: D = 96 / 128), whose tail DMAs walk the next block's descriptor sets."""
    return SOFF_WALK and not (PERSIST and PERSIST_KV)


def set_geometry(r, dist):
    """Ring of r slots per tensor, DMA distance dist (<= r - 1: a slot is rewritten only after
    the barrier that follows its last read); the loop unroll is lcm(r, 2)."""
    global R, DIST, U, VREG, LDS_BYTES
    assert 1 <= dist <= r - 1
    R, DIST = r, dist
    U = r * 2 // math.gcd(r, 2)
    VREG = R * TILE
    LDS_BYTES = 2 * R * TILE
NKS = D // 16          # 16-deep k-steps of Q K^T
NDT = D // 32          # 32-wide d-blocks of O^T
NP = D // 32           # 1-KiB LDS-DMA pieces per tensor, tile and wave
ROWB = 2 * D           # bytes per LDS image row
KFB = D // 2           # registers of one K (or V^T) fragment buffer per wave
NBK = NBV = 2          # K / V^T fragment buffers (double-buffered at D = 64)
RESCALE_THR = 8.0      # log2-domain threshold of the deferred rescale (fa_fwd_kernel.h)
OOB = 0x80000000
PROBE = set()          # timing-only variants (tools/asm_variants.py); empty in the product build

# ---- VGPRs (arch)
V_KADDR = 4            # 4: K fragment read address per k-step
V_VADDR = 8            # 4: V^T fragment read address per (dt, half)
V_DMA = 12             # 4: DMA source offsets: K piece 0, K piece 1, V piece 0, V piece 1
V_S = {'A': 16, 'B': 48}        # 32 each: S^T accumulators (2 sub-tiles x 16)
V_P = {'A': 80, 'B': 96}        # 16 each: P as 16-bit B operands
V_MTHR = {'A': 112, 'B': 113}   # rescale threshold m + 2^8/c (raw score units)
V_MC = {'A': 114, 'B': 115}     # m * c (log2 domain)
V_TMP = {'A': 116, 'B': 124}    # 8 each
V_BPA = 132            # ds_bpermute address: alpha of query (l&15)+16(l>>5)  (sum-MFMA lane map)
V_BPL = 133            # ds_bpermute address: row sum of query l&31
V_NEGINF = 134
V_NVREL = {'A': 135, 'B': 164}  # masked tiles: keys of the tile the lane's row may see, minus 4*hi
V_ROW1 = {'A': 165, 'B': 166}   # min(seqlen_k, row + 1 if causal) - 4*hi (per block)
V_OOFF = {'A': 136, 'B': 140}   # 4 each: O store offsets (dt, g)
V_LOFF = {'A': 144, 'B': 145}   # LSE store offset
V_ONEF = 146           # 1.0f
V_LANE = 147
V_ETMP = 148           # 16: rotating exp temporaries of the speculative softmax (S stays intact)
V_MCB = {'A': 168, 'B': 172}    # 4 each (MC_BANKS): copies of m*c in VGPR banks 0..3
NVGPR = 168
# ---- AGPRs
A_O = {'A': 0, 'B': 32}         # O^T accumulators (2 d-blocks x 16)
A_L = {'A': 64, 'B': 68}        # row-sum accumulators (16x16 MFMA C)
A_ONES = 72                     # 0/1 indicator A operand of the row-sum MFMA
A_Q = {'A': 76, 'B': 92}        # Q fragments (B operand of S^T = K Q^T), 4 k-steps x 4
A_KF = 108                      # K fragments [buf 2][st*4+ks] x 4
A_VF = 172                      # V^T fragments [buf 2][dt*4+st*2+s] x 4
NAGPR = 236
O_BASE = False         # Q loads / O stores from one row base + immediates (requires head_dim == D)
QL_VGPR = False        # Q fragments, row sums and the 0/1 indicator in VGPRs (D = 128: AGPRs hold
#                        O, K and V^T fragments, 256, the most an AGPR index reaches)
NWAVES = 4             # waves per workgroup (8: the two-waves-per-SIMD form, configure(64, 8))
BLOCKS = 'AB'          # 32-row query blocks of a wave
NETMP = 16             # rotating exp temporaries
V_ORT = None           # OR-test accumulator (None: V_TMP[X])
V_EPT = None           # epilogue temporaries (None: V_TMP[X])
PRIO4 = False          # 8 waves: s_setprio 1 for waves 4-7 (the SIMD partners dispatched second)
STAGGER = False        # 8 waves: waves 4-7 run half a tile behind (their barrier mid-tile; ring 6)
FIRST_MAX_W8 = False   # 8 waves: FIRST_MAX (tile 0's row max sets the starting shift) as in the 4-wave form
STAGGER_FRAC = 0.5     # STAGGER: the group-1 barrier after this fraction of a phase's MFMAs
PINGPONG = False       # 8 waves (with STAGGER, ring 6): each phase = its MFMAs, then the softmax; the
#                        group-1 barrier between the two, so SIMD partners alternate matrix / vector work


def rq(base):
    """Text and register names of a 4-register Q / row-sum / indicator operand."""
    return vs(base, 4) if QL_VGPR else as_(base, 4)


def rqn(base, n=4):
    return rv(base, n) if QL_VGPR else ra(base, n)


# LDS ring per form: (slots, DMA distance, one barrier per two tiles, persistent K/V tail). D <= 64
# (4 waves): 6 slots (96 KiB), distance 3, a barrier after odd tiles only (a fast wave leads by up
# to two tiles, so a slot is rewritten two tiles after its last read; distance 3 also lets the
# prologue skip its barrier after the K0 reads) and no K/V tail (its seam
# saving measured ~0 once tile 0 stopped taking the rescale; the tail needs nt % R == 0). D = 128
# (32 KiB per slot) and the 8-wave form keep 4 slots, distance 3, a barrier per tile.
GEOMETRY = {(64, 4): (6, 3, True, False), (32, 4): (6, 3, True, False),
            (128, 4): (4, 3, False, True), (96, 4): (4, 3, False, True), (64, 8): (4, 3, False, True)}
D_NAME = 64            # the tile named in the kernel symbol (96: the D = 128 layout computing 96 columns)


def configure(hd, waves=4):
    """The head-dim tile's register map (configure_layout), then its ring geometry (GEOMETRY).
    hd = 96: the D = 128 layout (LDS rows, registers, DMA) with the QK k-steps and PV d-blocks of
    96 columns only (NKS 6, NDT 3); head_dim 80 zeroes Q's k-step 5 and drops the O chunk 80..95."""
    global BAR2, PERSIST_KV, NKS, NDT, D_NAME
    configure_layout(128 if hd == 96 else hd, waves)
    D_NAME = hd
    if hd == 96:
        NKS, NDT = 6, 3
    r, dist, BAR2, PERSIST_KV = GEOMETRY[(hd, waves)]
    set_geometry(r, dist)


def configure_layout(hd, waves=4):
    """Head-dim tile. 64: the layout above (head_dim in (32, 64]). 128 (head_dim == 128): twice the
    k-steps and d-blocks, single K / V^T fragment buffers (the K reads of tile j+1 follow the last
    QK_B(j) MFMA, the V^T reads of tile j follow PV_B(j-1), one phase earlier), Q / O offsets as
    one base + immediates, 128 KiB of LDS ring. 252 VGPRs (Q, row sums, indicator among them) + 256
    AGPRs (O, K and V^T fragments).

    waves=8 (D = 64, head_dim == 64): two waves per SIMD, each owning ONE 32-row block in at most
    256 registers (132 VGPRs + 120 AGPRs). The two register buffers 'A' / 'B' of S and P are then
    the tiles of even / odd index of that block (O, Q, row sums, m are shared): one phase per tile,
    QK(t+1) + PV(t-1) + row sums beside the softmax of tile t; single K / V^T fragment buffers;
    one 1-KiB DMA piece per tensor, tile and wave."""
    global D, NKS, NDT, NP, ROWB, KFB, NBK, NBV, TILE, VREG, LDS_BYTES, O_BASE, VREADS_P1, QL_VGPR
    global V_KADDR, V_VADDR, V_DMA, V_S, V_P, V_MTHR, V_MC, V_TMP, V_BPA, V_BPL, V_NEGINF, V_NVREL, V_ROW1
    global V_OOFF, V_LOFF, V_ONEF, V_LANE, V_ETMP, V_MCB, NVGPR, A_O, A_L, A_ONES, A_Q, A_KF, A_VF, NAGPR
    global NWAVES, BLOCKS, NETMP, V_ORT, V_EPT, EXP_LAG, CVT_LAG
    assert hd in (32, 64, 128) and waves in (4, 8)
    globals().update(_D64)   # the D = 64 layout, then the D = 128 / 8-wave changes
    globals().update(PERSIST=False, KARG_BYTES=168)
    EXP_LAG, CVT_LAG = 4, 4
    if waves == 8:
        assert hd == 64
        NWAVES, BLOCKS, NETMP = 8, 'A', 8
        EXP_LAG, CVT_LAG = 3, 3
        NP, NBK, NBV = 1, 1, 1
        O_BASE, VREADS_P1 = True, False
        V_KADDR, V_VADDR, V_DMA = 4, 8, 12
        V_S, V_P = {'A': 16, 'B': 48}, {'A': 80, 'B': 96}
        V_MTHR = {'A': 112, 'B': 112}
        V_MC = {'A': 113, 'B': 113}
        V_ORT = 114
        V_TMP = dict(V_P)          # rescale temporaries: the P buffer the rescale recomputes anyway
        V_BPA, V_BPL, V_NEGINF = 115, 116, 117
        V_NVREL, V_ROW1 = {'A': 118, 'B': 118}, {'A': 119, 'B': 119}
        V_OOFF, V_LOFF = {'A': 120, 'B': 120}, {'A': 121, 'B': 121}
        V_ONEF, V_LANE, V_ETMP = 122, 123, 124
        V_EPT = V_ETMP
        V_MCB = None
        NVGPR = 132
        A_O, A_L, A_ONES = {'A': 0, 'B': 0}, {'A': 32, 'B': 32}, 36
        A_Q = {'A': 40, 'B': 40}
        A_KF, A_VF = 56, 88
        NAGPR = 120
        return
    NWAVES, BLOCKS, NETMP, V_ORT, V_EPT = 4, 'AB', 16, None, None
    if hd == 64:
        return
    if hd == 32:
        # D = 32 (head_dim <= 32, zero-padded): the D = 64 register map with half-size K / V^T fragment
        # buffers, one O d-block, one 1-KiB DMA piece per tensor, tile and wave (4 KiB tiles)
        D, NKS, NDT, NP, ROWB, KFB = 32, 2, 1, 1, 64, 16
        TILE = BN * D * 2
        VREG = R * TILE
        LDS_BYTES = 2 * R * TILE
        return
    D, NKS, NDT, NP, ROWB, KFB = hd, hd // 16, hd // 32, hd // 32, 2 * hd, hd // 2
    NBK = NBV = 1
    O_BASE, VREADS_P1, QL_VGPR = True, False, True
    TILE = BN * D * 2
    VREG = R * TILE
    LDS_BYTES = 2 * R * TILE
    # S / P first: the prologue's temporaries (v16..v51) live there until QK_A(0)
    V_S, V_P = {'A': 4, 'B': 36}, {'A': 68, 'B': 84}
    V_KADDR, V_VADDR, V_DMA = 100, 108, 116
    V_MTHR, V_MC, V_TMP = {'A': 124, 'B': 125}, {'A': 126, 'B': 127}, {'A': 128, 'B': 136}
    V_BPA, V_BPL, V_NEGINF = 144, 145, 146
    V_NVREL, V_ROW1 = {'A': 147, 'B': 248}, {'A': 249, 'B': 250}
    V_OOFF, V_LOFF = {'A': 148, 'B': 149}, {'A': 150, 'B': 151}
    V_ONEF, V_LANE, V_ETMP = 152, 153, 154
    # VGPRs: Q fragments, row sums and the indicator after the exp temporaries (A_* names kept)
    A_Q, A_L, A_ONES = {'A': 172, 'B': 204}, {'A': 236, 'B': 240}, 244
    V_MCB = None           # no room for MC_BANKS copies at D = 128
    NVGPR = 252
    A_O, A_KF, A_VF = {'A': 0, 'B': 64}, 128, 192
    NAGPR = 256


_D64 = {k: (dict(v) if isinstance(v, dict) else v) for k, v in globals().items()
        if k in ('D', 'NKS', 'NDT', 'NP', 'ROWB', 'KFB', 'NBK', 'NBV', 'TILE', 'VREG', 'LDS_BYTES', 'O_BASE',
                 'VREADS_P1', 'QL_VGPR', 'V_KADDR', 'V_VADDR', 'V_DMA', 'V_S', 'V_P', 'V_MTHR', 'V_MC', 'V_TMP',
                 'V_BPA', 'V_BPL', 'V_NEGINF', 'V_NVREL', 'V_ROW1', 'V_OOFF', 'V_LOFF', 'V_ONEF', 'V_LANE', 'V_ETMP',
                 'V_MCB', 'NVGPR', 'A_O', 'A_L', 'A_ONES', 'A_Q', 'A_KF', 'A_VF', 'NAGPR')}


def epi_regs(X, idx):
    """Epilogue temporaries of block X, output slot idx (d-block, group): 8 fp32 and 4 packed
    words in registers dead by then. D = 64: S_X and P_X. D = 128 (8 slots): S_A..S_B for the fp32
    (both softmaxes are done); the words of block A in P_A then the exp temporaries (P_B still
    feeds the last P_B.V beside it), of block B in P_A..P_B."""
    if D <= 64:
        return V_S[X] + 8 * idx, V_P[X] + 4 * idx
    E = V_S['A'] + 8 * idx
    if X == 'A' and idx >= 4:
        return E, V_ETMP + 4 * (idx - 4)
    return E, V_P['A'] + 4 * idx

# ---- SGPRs
S_KD, S_VD, S_QD, S_OD, S_LD = 8, 12, 16, 20, 24   # buffer descriptors (4 each)
S_KD1, S_VD1 = 80, 84  # second K / V descriptor sets (odd tiles; prologue temporaries before)
# SOFF_WALK (round 6): one K and one V descriptor per block, the tile selected by the SGPR offset of
# the DMA (the raw-buffer range check includes it on gfx950: tools/micro/soffset_probe.hip,
# profiles/r06/soffset_probe.txt), two offsets per tensor (even / odd tiles) each advanced by two
# tiles right before its next use: one SALU per tensor and tile instead of four, in s80..s83
S_KOFF, S_VOFF = (80, 81), (82, 83)
SOFF_WALK = True
S_C, S_THR, S_J, S_NT, S_LAST = 28, 29, 30, 31, 32
S_CAUSAL, S_MAGIC_BH = 33, 34   # kernel arguments: causal flag, ceil(2^32 / (2 nbh))
S_MSTART = 39          # first tile of the masked loop (causal: the diagonal band; else the last tile)
S_KSTEP, S_VSTEP, S_WAVE = 35, 36, 37
S_M0B = 38             # 1024 * wave: this wave's DMA pieces start at piece `wave`
S_ARG = 40             # kernel arguments s[40:75]
S_CU = 76              # cu_seqlens values s[76:79]
S_T = 80               # temporaries s[80:97]
NSGPR = 102


class Inst:
    """One instruction (or an unbreakable group of lines).

    kind: mfma | valu | trans | perm | accr | accw | ds | dma | vload | vstore | salu | m0 |
          smem | wait | nop | br | label | barrier | raw
    cost: issue cycles used by the gap placer. rd / wr: register names ('v12', 'a40', 's3',
    'vcc', 'm0'). rdc: MFMA srcC registers. pipe: MFMA pipe cycles (32 or 16).
    deadline: index of the MFMA (within its phase) that this filler must precede.
    not_before: number of the phase's MFMAs that must be issued before this filler (it overwrites
    their operands: the single-buffered fragments at D = 128).
    """
    __slots__ = ('txt', 'kind', 'cost', 'rd', 'wr', 'rdc', 'pipe', 'deadline', 'lgkm_dst', 'not_before')

    def __init__(self, txt, kind, cost=4, rd=(), wr=(), rdc=(), pipe=0, deadline=None):
        self.txt, self.kind, self.cost = txt, kind, cost
        self.rd, self.wr, self.rdc = frozenset(rd), frozenset(wr), frozenset(rdc)
        self.pipe, self.deadline = pipe, deadline
        self.not_before = None


def rv(base, n=1):
    return [f'v{base + i}' for i in range(n)]


def ra(base, n=1):
    return [f'a{base + i}' for i in range(n)]


def vs(base, n=1):
    return f'v{base}' if n == 1 else f'v[{base}:{base + n - 1}]'


def as_(base, n=1):
    return f'a{base}' if n == 1 else f'a[{base}:{base + n - 1}]'


def V(txt, dst, srcs, kind='valu', cost=4):
    """VALU with VGPR operands given as ints (register numbers) or names."""
    def nm(x):
        return f'v{x}' if isinstance(x, int) else x
    wr = [nm(d) for d in (dst if isinstance(dst, (list, tuple)) else [dst])]
    rd = [nm(s) for s in srcs]
    return Inst(txt, kind, cost, rd=rd, wr=wr)


def salu(txt, rd=(), wr=(), cost=2):
    return Inst(txt, 'salu', cost, rd=rd, wr=wr)


def label(name):
    return Inst(f'{name}:', 'label', 0)


def raw(txt, cost=0):
    return Inst(txt, 'raw', cost)


class Gen:
    def __init__(self, dtype):
        assert dtype in ('bf16', 'f16')
        self.dtype = dtype
        self.mf32 = 'v_mfma_f32_32x32x16_bf16' if dtype == 'bf16' else 'v_mfma_f32_32x32x16_f16'
        self.mf16 = 'v_mfma_f32_16x16x32_bf16' if dtype == 'bf16' else 'v_mfma_f32_16x16x32_f16'
        self.cvt = 'v_cvt_pk_bf16_f32' if dtype == 'bf16' else 'v_cvt_pk_f16_f32'
        self.one2 = 0x3F803F80 if dtype == 'bf16' else 0x3C003C00
        self.nlabel = 0
        self.name = f'fa_fwd_d{D_NAME}{"w8" if NWAVES == 8 else ""}{"p" if PERSIST else ""}_{dtype}_asm'

    def lab(self, stem):
        self.nlabel += 1
        return f'.L{stem}_{self.nlabel}'

    # ------------------------------------------------------------------ MFMA groups
    def qk(self, X, t):
        """S_X^T = K(t) Q_X^T: 2 sub-tiles x 4 k-steps (K fragment buffer t % 2)."""
        out = []
        S, Q = V_S[X], A_Q[X]
        for st in range(2):
            acc = S + 16 * st
            for ks in range(NKS):
                kf = A_KF + KFB * (t % NBK) + 4 * (st * NKS + ks)
                seed = PRESCALE and ks == 0
                c = (vs(V_SEED[X], 16) if seed else '0') if ks == 0 else vs(acc, 16)
                out.append(Inst(f'{self.mf32} {vs(acc, 16)}, {as_(kf, 4)}, {rq(Q + 4 * ks)}, {c}', 'mfma', 8,
                                rd=ra(kf, 4) + rqn(Q + 4 * ks) + (rv(V_SEED[X], 16) if seed else []),
                                wr=rv(acc, 16), rdc=rv(acc, 16) if ks else (), pipe=32))
        return out

    def pv_sum(self, X, t):
        """O_X^T += V^T(t) P_X^T (8 MFMAs) interleaved with the 4 row-sum MFMAs.
        Returns (list, {frag index: position in list})."""
        out, use = [], {}
        O, P, L = A_O[X], V_P[X], A_L[X]
        sums = []
        for st in range(2):
            for s in range(2):
                p = P + 4 * (st * 2 + s)
                sums.append(Inst(f'{self.mf16} {rq(L)}, {rq(A_ONES)}, {vs(p, 4)}, {rq(L)}', 'mfma', 8,
                                 rd=rqn(A_ONES) + rv(p, 4), wr=rqn(L), rdc=rqn(L), pipe=16))
        si = 0
        for dt in range(NDT):
            for st in range(2):
                for s in range(2):
                    f = dt * 4 + st * 2 + s
                    vf = A_VF + KFB * (t % NBV) + 4 * f
                    p = P + 4 * (st * 2 + s)
                    acc = O + 16 * dt
                    use[f] = len(out)
                    out.append(Inst(f'{self.mf32} {as_(acc, 16)}, {as_(vf, 4)}, {vs(p, 4)}, {as_(acc, 16)}', 'mfma', 8,
                                    rd=ra(vf, 4) + rv(p, 4), wr=ra(acc, 16), rdc=ra(acc, 16), pipe=32))
                if si < 4 and 'nosum' not in PROBE:
                    out.append(sums[si])
                    si += 1
        if 'nosum' not in PROBE:
            out += sums[si:]     # D = 32: one d-block leaves two row-sum MFMAs
        return out, use

    # ------------------------------------------------------------------ LDS reads / DMA
    def kreads(self, t):
        """K(t) fragments from ring slot t % R into buffer t % 2 (8 x ds_read_b128)."""
        out = []
        if 'nolds' in PROBE:
            return out
        slot = KREG + (t % R) * TILE
        for st in range(2):
            for ks in range(NKS):
                kf = A_KF + KFB * (t % NBK) + 4 * (st * NKS + ks)
                out.append(Inst(f'ds_read_b128 {as_(kf, 4)}, v{V_KADDR + ks} offset:{slot + st * 32 * ROWB}', 'ds', 2,
                                rd=[f'v{V_KADDR + ks}'], wr=ra(kf, 4)))
        return out

    def vreads(self, t):
        """V(t)^T fragments from ring slot t % R into buffer t % 2 (16 x ds_read_b64_tr_b16).
        Returns list of (frag, inst)."""
        out = []
        if 'nolds' in PROBE:
            return out
        slot = VREG + (t % R) * TILE
        for dt in range(NDT):
            for st in range(2):
                for s in range(2):
                    f = dt * 4 + st * 2 + s
                    vf = A_VF + KFB * (t % NBV) + 4 * f
                    for half in range(2):
                        addr = V_VADDR + dt * 2 + half
                        off = slot - VREG + (32 * st + 16 * s) * ROWB   # VREG is in the address VGPR
                        out.append((f, Inst(f'ds_read_b64_tr_b16 {as_(vf + 2 * half, 2)}, v{addr} offset:{off}', 'ds', 2,
                                            rd=[f'v{addr}'], wr=ra(vf + 2 * half, 2))))
        return out

    def dma(self, kind, t):
        if 'nodma' in PROBE:
            return []
        return self._dma(kind, t)

    def _dma(self, kind, t, nxt=False, walk_only=False):
        """This wave's two 1-KiB pieces of the K or V tile t (LDS-DMA into ring slot t % R).
        Tile t reads through descriptor set t % 2. Each set walks the sequence two tiles at a
        time: right before its next use its base advances by 128 rows and num_records shrinks by
        the same bytes, saturating at 0, so rows past the end (and every tile past the last) read
        as zeros whatever the SGPR-offset range-check rule is. Updating the set used two tiles
        ago (not the one a DMA just read) keeps the SALU writes off SGPRs an in-flight LDS-DMA
        still reads (measured -4 % against a walk right behind the DMA)."""
        out = []
        region = KREG if kind == 'K' else VREG
        step = S_KSTEP if kind == 'K' else S_VSTEP          # 2 tiles of bytes
        if soff_walk() and not nxt:
            desc = S_KD if kind == 'K' else S_VD
            off = (S_KOFF if kind == 'K' else S_VOFF)[t % 2]
            dregs = [f's{desc + i}' for i in range(4)] + [f's{off}']
            if t >= 2 and 'nowalk' not in PROBE:
                out.append(salu(f's_add_u32 s{off}, s{off}, s{step}', rd=[f's{off}', f's{step}'], wr=[f's{off}', 'scc']))
            if walk_only:
                return out
            for i in range(NP):
                m0 = region + (t % R) * TILE + 1024 * NWAVES * i   # + 1024 * wave (S_M0B)
                voff = V_DMA + (0 if kind == 'K' else NP) + i
                out.append(Inst(f's_add_u32 m0, s{S_M0B}, {m0}', 'm0', 2, rd=[f's{S_M0B}'], wr=['m0', 'scc']))
                out.append(Inst(f'buffer_load_dwordx4 v{voff}, s[{desc}:{desc + 3}], s{off} offen lds', 'dma', 16,
                                rd=[f'v{voff}', 'm0'] + dregs))
            return out
        desc = (S_KD if t % 2 == 0 else S_KD1) if kind == 'K' else (S_VD if t % 2 == 0 else S_VD1)
        if nxt:     # the next block's sets (persistent form's tail: t = the next block's tile)
            desc = S_NXD[kind][t % 2]
        dregs = [f's{desc + i}' for i in range(4)]
        if t >= 2 and 'nowalk' not in PROBE:
            st = f's{step}'
            out.append(salu(f's_add_u32 s{desc}, s{desc}, {st}', rd=[dregs[0], st], wr=[dregs[0], 'scc']))
            out.append(salu(f's_addc_u32 s{desc + 1}, s{desc + 1}, 0', rd=[dregs[1], 'scc'], wr=[dregs[1], 'scc']))
            out.append(salu(f's_sub_u32 s{desc + 2}, s{desc + 2}, {st}', rd=[dregs[2], st], wr=[dregs[2], 'scc']))
            out.append(salu(f's_cselect_b32 s{desc + 2}, 0, s{desc + 2}', rd=[dregs[2], 'scc'], wr=[dregs[2]]))
        if walk_only:
            return out
        for i in range(NP):
            m0 = region + (t % R) * TILE + 1024 * NWAVES * i   # + 1024 * wave (S_M0B)
            voff = V_DMA + (0 if kind == 'K' else NP) + i
            out.append(Inst(f's_add_u32 m0, s{S_M0B}, {m0}', 'm0', 2, rd=[f's{S_M0B}'], wr=['m0', 'scc']))
            out.append(Inst(f'buffer_load_dwordx4 v{voff}, s[{desc}:{desc + 3}], 0 offen lds', 'dma', 16,
                            rd=[f'v{voff}', 'm0'] + dregs))
        return out

    # ------------------------------------------------------------------ softmax of one tile
    def mc_reg(self, X, sreg, mc):
        """The m*c register an fma with S operand v{sreg} reads: m*c itself, or with MC_BANKS
        the copy two VGPR banks away from the S operand (no read-port conflict)."""
        if not MC_BANKS:
            return mc
        return next(c for c in range(V_MCB[X], V_MCB[X] + 4) if c % 4 == (sreg % 4 + 2) % 4)

    def exp_stream(self, X, mc, ortest=False, shift=None):
        """P_X = cvt(exp2(S_X c - mc)) through the 16 rotating temporaries: fma(i) at step i,
        exp(i) at step i + EXP_LAG, cvt of pair q at step 2q + 1 + EXP_LAG + CVT_LAG (every
        consumer several instructions behind its producer; temporary i % 16 is free again before
        element i + 16 needs it). ortest: also the ORDET rescale test over the packed P (an OR
        chain behind the cvts, then vcc = lanes holding some P >= 2: bit 14 of either half is
        the top exponent bit of a bf16 / f16 >= 2, and of inf / NaN)."""
        S, P, E = V_S[X], V_P[X], V_ETMP
        assert EXP_LAG + CVT_LAG + 1 < NETMP
        steps = []
        for i in range(32):
            e = E + i % NETMP
            if PRESCALE and shift is None:
                # S^T = K Q~^T - m c already: the exp reads the accumulator
                steps.append((i + EXP_LAG, 1, V(f'v_exp_f32 v{e}, v{S + i}', e, [S + i], kind='trans', cost=8)))
                continue
            if PRESCALE:    # rescale recompute: exp2(S - shift)
                steps.append((i, 0, V(f'v_sub_f32 v{e}, v{S + i}, v{shift}', e, [S + i, shift])))
            else:
                m = self.mc_reg(X, S + i, mc)
                steps.append((i, 0, Inst(f'v_fma_f32 v{e}, v{S + i}, s{S_C}, -v{m}', 'valu', 4,
                                         rd=[f'v{S + i}', f's{S_C}', f'v{m}'], wr=[f'v{e}'])))
            steps.append((i + EXP_LAG, 1, V(f'v_exp_f32 v{e}, v{e}', e, [e], kind='trans', cost=8)))
        cvt_at = {}
        for q in range(16):
            a, b = E + (2 * q) % NETMP, E + (2 * q + 1) % NETMP
            cvt_at[q] = 2 * q + 1 + EXP_LAG + CVT_LAG
            steps.append((cvt_at[q], 2, V(f'{self.cvt} v{P + q}, v{a}, v{b}', P + q, [a, b])))
        if ortest:
            T = V_TMP[X] if V_ORT is None else V_ORT
            last = 14 if ORDET_ANDOR else 15
            groups = [(0, 1, 2)] + [(2 * k + 1, 2 * k + 2) for k in range(1, 7)] + ([] if ORDET_ANDOR else [(15,)])
            for gi, grp in enumerate(groups):
                srcs = ([] if gi == 0 else [T]) + [P + q for q in grp]
                op = 'v_or3_b32' if len(srcs) == 3 else 'v_or_b32'
                steps.append((cvt_at[max(grp)] + 3, 3, V(f'{op} v{T}, ' + ', '.join(f'v{r}' for r in srcs), T, srcs)))
            end = cvt_at[last] + 3
            if ORDET_BITOP3 and ORDET_ANDOR:
                # (T | P15) & M in one v_bitop3_b32 (table 0xa8: S0 | S1, and S2), M = 0x40004000 in V_MTHR
                end = cvt_at[15] + 3
                M = V_MTHR[X]
                steps.append((end, 3, Inst(f'v_bitop3_b32 v{T}, v{T}, v{P + 15}, v{M} bitop3:0xa8', 'valu', 4,
                                           rd=[f'v{P + 15}', f'v{M}', f'v{T}'], wr=[f'v{T}'])))
                steps.append((end + 2, 3, V(f'v_cmp_ne_u32 vcc, 0, v{T}', 'vcc', [T])))
                return [x for _, _, x in sorted(steps, key=lambda z: (z[0], z[1]))]
            steps.append((end + 1, 3, V(f'v_and_b32 v{T}, 0x40004000, v{T}', T, [T])))
            if ORDET_ANDOR:
                # the last P word joins after the mask: (P15 & M) | T, M = 0x40004000 in V_MTHR
                # (unused by the OR test): one dependent step between the last cvt and the compare
                end = cvt_at[15] + 3
                M = V_MTHR[X]
                steps.append((end, 3, Inst(f'v_and_or_b32 v{T}, v{P + 15}, v{M}, v{T}', 'valu', 4,
                                           rd=[f'v{P + 15}', f'v{M}', f'v{T}'], wr=[f'v{T}'])))
            steps.append((end + 2, 3, V(f'v_cmp_ne_u32 vcc, 0, v{T}', 'vcc', [T])))
        return [x for _, _, x in sorted(steps, key=lambda z: (z[0], z[1]))]

    def max_ops(self, X):
        """Row max of S_X (4 v_max3 chains, merge, lane pair (l, l^32)) and the rescale test
        (vcc = lanes whose tile max passed the threshold)."""
        S, T, mthr = V_S[X], V_TMP[X], V_MTHR[X]
        chains = []
        for k in range(4):
            c = [S + 8 * k + e for e in range(8)]
            t = T + k
            chains.append([V(f'v_max3_f32 v{t}, v{c[0]}, v{c[1]}, v{c[2]}', t, c[0:3]),
                           V(f'v_max3_f32 v{t}, v{t}, v{c[3]}, v{c[4]}', t, [t, c[3], c[4]]),
                           V(f'v_max3_f32 v{t}, v{t}, v{c[5]}, v{c[6]}', t, [t, c[5], c[6]]),
                           V(f'v_max_f32 v{t}, v{t}, v{c[7]}', t, [t, c[7]])])
        out = [chains[k][st] for st in range(4) for k in range(4)]
        out += [V(f'v_max3_f32 v{T + 4}, v{T}, v{T + 1}, v{T + 2}', T + 4, [T, T + 1, T + 2]),
                V(f'v_max_f32 v{T + 4}, v{T + 4}, v{T + 3}', T + 4, [T + 4, T + 3]),
                V(f'v_mov_b32 v{T + 5}, v{T + 4}', T + 5, [T + 4]),
                Inst(f'v_permlane32_swap_b32 v{T + 4}, v{T + 5}', 'perm', 4,
                     rd=[f'v{T + 4}', f'v{T + 5}'], wr=[f'v{T + 4}', f'v{T + 5}']),
                V(f'v_max_f32 v{T + 6}, v{T + 4}, v{T + 5}', T + 6, [T + 4, T + 5]),
                V(f'v_cmp_gt_f32 vcc, v{T + 6}, v{mthr}', 'vcc', [T + 6, mthr])]
        if 'nomax' in PROBE:     # timing probe: a test that never fires
            out[-1] = V(f'v_cmp_gt_f32 vcc, v{V_NEGINF}, v{mthr}', 'vcc', [V_NEGINF, mthr])
        return out

    def softmax_spec(self, X, masked, rescue):
        """Speculative form: the exps run against the current m while the max tree runs
        beside them (no dependence between the two), and the rescale test branches only at the
        end of the phase, when its vcc is long known; the rare rescale block then moves m,
        scales O and the row sums and recomputes P from the untouched S."""
        S, P, T = V_S[X], V_P[X], V_TMP[X]
        mthr, mc = V_MTHR[X], V_MC[X]
        out = []
        if masked:
            for i in range(32):
                st, r = divmod(i, 16)
                kofs = 32 * st + (r & 3) + 8 * (r >> 2)
                out.append(V(f'v_cmp_lt_i32 vcc, {kofs}, v{V_NVREL[X]}', 'vcc', [V_NVREL[X]]))
                out.append(Inst(f'v_cndmask_b32 v{S + i}, v{V_NEGINF}, v{S + i}, vcc', 'valu', 4,
                                rd=[f'v{V_NEGINF}', f'v{S + i}', 'vcc'], wr=[f'v{S + i}']))
        if ORDET:
            out += probe_filter(self.exp_stream(X, mc, ortest=True), keep_last=True)
        else:
            ex = self.exp_stream(X, mc)
            mx = self.max_ops(X)
            ex, mx = probe_filter(ex), probe_filter(mx, keep_last=True)
            # max ops spread over the first 70 % of the exp stream
            out += merge(ex, [(i, x) for i, x in zip(spread(len(mx), 2, int(len(ex) * 0.7)), mx)])
        resc, ret = self.lab(f'resc{X}'), self.lab(f'ret{X}')
        touched = [f'v{mc}', f'v{mthr}'] + rv(T, 8) + ra(A_O[X], D // 2) + rqn(A_L[X]) + rv(V_ETMP, NETMP) + rv(P, 16)
        if MC_BANKS:
            touched += rv(V_MCB[X], 4)
        if PRESCALE:
            touched += rv(V_SEED[X], 16)
        out.append(Inst(f's_cbranch_vccnz {resc}\n{ret}:', 'br', 4, rd=['vcc'] + touched, wr=touched))
        if PRESCALE:
            assert ORDET
            rb = self.rescale_block_seed(X, resc, ret)
            rb[-2:-2] = self.exp_stream(X, mc, shift=T + 7)   # recompute P = exp2(S - shift)
        else:
            rb = self.rescale_block_or(X, resc, ret) if ORDET else self.rescale_block(X, resc, ret)
            rb[-2:-2] = self.exp_stream(X, mc)       # recompute P with the new m (before the s_nop 2)
        rescue.append(rb)
        if 'nofill' in PROBE:
            out = []
            rescue.pop()
        return out

    def softmax(self, X, masked, rescue):
        if SPEC:
            return self.softmax_spec(X, masked, rescue)
        return self.softmax_serial(X, masked, rescue)

    def softmax_serial(self, X, masked, rescue):
        """Block X's softmax of the tile in S_X: [mask], max tree, deferred-rescale test
        (branch to an out-of-line block), exp2(s c - m c), conversion into P_X.
        rescue: list that receives the out-of-line rescale block."""
        S, P, T = V_S[X], V_P[X], V_TMP[X]
        mthr, mc = V_MTHR[X], V_MC[X]
        out = []
        if masked:
            for i in range(32):
                st, r = divmod(i, 16)
                kofs = 32 * st + (r & 3) + 8 * (r >> 2)
                out.append(V(f'v_cmp_lt_i32 vcc, {kofs}, v{V_NVREL[X]}', 'vcc', [V_NVREL[X]]))
                out.append(Inst(f'v_cndmask_b32 v{S + i}, v{V_NEGINF}, v{S + i}, vcc', 'valu', 4,
                                rd=[f'v{V_NEGINF}', f'v{S + i}', 'vcc'], wr=[f'v{S + i}']))
        # max tree: 4 chains of v_max3 (ILP 4), then merge, then the lane pair (l, l^32)
        chains = []
        for k in range(4):
            c = [S + 8 * k + e for e in range(8)]
            t = T + k
            chains.append([V(f'v_max3_f32 v{t}, v{c[0]}, v{c[1]}, v{c[2]}', t, c[0:3]),
                           V(f'v_max3_f32 v{t}, v{t}, v{c[3]}, v{c[4]}', t, [t, c[3], c[4]]),
                           V(f'v_max3_f32 v{t}, v{t}, v{c[5]}, v{c[6]}', t, [t, c[5], c[6]]),
                           V(f'v_max_f32 v{t}, v{t}, v{c[7]}', t, [t, c[7]])])
        for step in range(4):
            for k in range(4):
                out.append(chains[k][step])
        if 'nomax' in PROBE:
            out = [x for x in out if not x.txt.startswith(('v_max', 'v_cmp_lt'))]
        out.append(V(f'v_max3_f32 v{T + 4}, v{T}, v{T + 1}, v{T + 2}', T + 4, [T, T + 1, T + 2]))
        out.append(V(f'v_max_f32 v{T + 4}, v{T + 4}, v{T + 3}', T + 4, [T + 4, T + 3]))
        out.append(V(f'v_mov_b32 v{T + 5}, v{T + 4}', T + 5, [T + 4]))
        out.append(Inst(f'v_permlane32_swap_b32 v{T + 4}, v{T + 5}', 'perm', 4,
                        rd=[f'v{T + 4}', f'v{T + 5}'], wr=[f'v{T + 4}', f'v{T + 5}']))
        out.append(V(f'v_max_f32 v{T + 6}, v{T + 4}, v{T + 5}', T + 6, [T + 4, T + 5]))
        out.append(V(f'v_cmp_gt_f32 vcc, v{T + 6}, v{mthr}', 'vcc', [T + 6, mthr]))
        if 'nomax' in PROBE:
            out += [V(f'v_max_f32 v{T + 6}, v{S}, v{S + 1}', T + 6, [S, S + 1]),
                    V(f'v_cmp_gt_f32 vcc, v{T + 6}, v{mthr}', 'vcc', [T + 6, mthr])]
            out = [x for x in out if not (x.txt.startswith('v_cmp_gt_f32') and x is not out[-1])]
        resc, ret = self.lab(f'resc{X}'), self.lab(f'ret{X}')
        # branch and its return label form one unbreakable group
        # (it also carries the registers the out-of-line block touches, so the scheduler keeps
        # their readers after it and anything unrelated may move across it)
        touched = [f'v{mc}', f'v{mthr}'] + rv(T, 8) + ra(A_O[X], D // 2) + rqn(A_L[X])
        out.append(Inst(f's_cbranch_vccnz {resc}\n{ret}:', 'br', 4, rd=['vcc'] + touched, wr=touched))
        rescue.append(self.rescale_block(X, resc, ret))
        # exp2(s * c - m * c), converted pairwise into the 16-bit P operand
        if SM_PIPE:
            # fma(i) at step i, exp(i) at step i + 4, cvt of pair q at step 2q + 9: every
            # dependent instruction sits 4+ instructions behind its producer
            steps = []
            for i in range(32):
                a = S + i
                steps.append((i, 0, Inst(f'v_fma_f32 v{a}, v{a}, s{S_C}, -v{mc}', 'valu', 4,
                                         rd=[f'v{a}', f's{S_C}', f'v{mc}'], wr=[f'v{a}'])))
                steps.append((i + 4, 1, V(f'v_exp_f32 v{a}, v{a}', a, [a], kind='trans', cost=8)))
            for q in range(16):
                steps.append((2 * q + 9, 2, V(f'{self.cvt} v{P + q}, v{S + 2 * q}, v{S + 2 * q + 1}', P + q,
                                              [S + 2 * q, S + 2 * q + 1])))
            out += [x for _, _, x in sorted(steps, key=lambda z: (z[0], z[1]))]
        for q in ([] if SM_PIPE else range(16)):
            a, b = S + 2 * q, S + 2 * q + 1
            out.append(Inst(f'v_fma_f32 v{a}, v{a}, s{S_C}, -v{mc}', 'valu', 4, rd=[f'v{a}', f's{S_C}', f'v{mc}'],
                            wr=[f'v{a}']))
            out.append(Inst(f'v_fma_f32 v{b}, v{b}, s{S_C}, -v{mc}', 'valu', 4, rd=[f'v{b}', f's{S_C}', f'v{mc}'],
                            wr=[f'v{b}']))
            out.append(V(f'v_exp_f32 v{a}, v{a}', a, [a], kind='trans', cost=8))
            out.append(V(f'v_exp_f32 v{b}, v{b}', b, [b], kind='trans', cost=8))
            if q >= 1:
                out.append(V(f'{self.cvt} v{P + q - 1}, v{S + 2 * q - 2}, v{S + 2 * q - 1}', P + q - 1,
                             [S + 2 * q - 2, S + 2 * q - 1]))
        if not SM_PIPE:
            out.append(V(f'{self.cvt} v{P + 15}, v{S + 30}, v{S + 31}', P + 15, [S + 30, S + 31]))
        if 'expmov' in PROBE:     # price the transcendental beyond a plain VALU op
            for x in out:
                if x.txt.startswith('v_exp_f32'):
                    x.txt = x.txt.replace('v_exp_f32', 'v_mov_b32')
                    x.kind, x.cost = 'valu', 4
        drop = {'noexp': 'v_exp', 'nofma': 'v_fma', 'nocvt': 'v_cvt'}
        for k, pre in drop.items():
            if k in PROBE:
                out = [x for x in out if not x.txt.startswith(pre)]
        if 'nofill' in PROBE:
            out = []
            rescue.pop()
        return out

    def rescale_block(self, X, resc, ret):
        """Out-of-line: lanes whose tile max passed the threshold move m (alpha = 2^(mc_old -
        mc_new)), O_X and the row sums are scaled by alpha (the row-sum accumulator holds
        query (l&15) + 16 (l>>5) in lane l: alpha is permuted to it)."""
        T, mthr, mc = V_TMP[X], V_MTHR[X], V_MC[X]
        O, L = A_O[X], A_L[X]
        b = [label(resc), raw('s_nop 4')]
        b.append(V(f'v_mul_f32 v{T + 7}, v{T + 6}, s{S_C}', T + 7, [T + 6]))
        b.append(V(f'v_sub_f32 v{T}, v{mc}, v{T + 7}', T, [mc, T + 7]))
        b.append(V(f'v_exp_f32 v{T}, v{T}', T, [T], kind='trans'))
        b.append(V(f'v_add_f32 v{T + 1}, s{S_THR}, v{T + 6}', T + 1, [T + 6]))
        b.append(Inst(f'v_cndmask_b32 v{T}, v{V_ONEF}, v{T}, vcc', 'valu', rd=[f'v{V_ONEF}', f'v{T}', 'vcc'],
                      wr=[f'v{T}']))
        b.append(Inst(f'v_cndmask_b32 v{mc}, v{mc}, v{T + 7}, vcc', 'valu', rd=[f'v{mc}', f'v{T + 7}', 'vcc'],
                      wr=[f'v{mc}']))
        b.append(Inst(f'v_cndmask_b32 v{mthr}, v{mthr}, v{T + 1}, vcc', 'valu', rd=[f'v{mthr}', f'v{T + 1}', 'vcc'],
                      wr=[f'v{mthr}']))
        b += self.scale_acc(X)
        b.append(raw('s_nop 2'))
        b.append(raw(f's_branch {ret}'))
        return b

    def rescale_block_or(self, X, resc, ret):
        """Out-of-line rescale of the ORDET test: the tile max (max tree) sets m*c = max*c + delta
        on the lanes where that passes the current m*c (alpha = 2^(mc_old - mc_new)), O_X and the
        row sums are scaled by alpha, and P is recomputed (appended by the caller)."""
        T, mc = V_TMP[X], V_MC[X]
        b = [label(resc), raw('s_nop 4')]
        b += self.max_ops(X)[:-1]                   # v{T+6} = tile max of the query (raw units)
        b.append(V(f'v_mul_f32 v{T + 7}, s{S_C}, v{T + 6}', T + 7, [T + 6]))
        b.append(V(f'v_add_f32 v{T + 7}, {ORDET_DELTA[self.dtype]!r}, v{T + 7}', T + 7, [T + 7]))
        b.append(V(f'v_cmp_gt_f32 vcc, v{T + 7}, v{mc}', 'vcc', [T + 7, mc]))
        b.append(V(f'v_sub_f32 v{T}, v{mc}, v{T + 7}', T, [mc, T + 7]))
        b.append(V(f'v_exp_f32 v{T}, v{T}', T, [T], kind='trans'))
        b.append(Inst(f'v_cndmask_b32 v{T}, v{V_ONEF}, v{T}, vcc', 'valu', rd=[f'v{V_ONEF}', f'v{T}', 'vcc'],
                      wr=[f'v{T}']))
        b.append(Inst(f'v_cndmask_b32 v{mc}, v{mc}, v{T + 7}, vcc', 'valu', rd=[f'v{mc}', f'v{T + 7}', 'vcc'],
                      wr=[f'v{mc}']))
        b += self.scale_acc(X)
        b.append(raw('s_nop 2'))
        b.append(raw(f's_branch {ret}'))
        return b

    def rescale_block_seed(self, X, resc, ret):
        """Out-of-line rescale of the PRESCALE form: S holds s~ - m c, so its tile max T6 is the
        excess over the current m c; lanes with T6 + delta > 0 move m c up by shift = T6 + delta
        (P <= 2^-delta afterwards), O and the row sums are scaled by 2^-shift, the S^T seed
        registers follow m c, and P is recomputed as exp2(S - shift) (appended by the caller)."""
        T, mc = V_TMP[X], V_MC[X]
        b = [label(resc), raw('s_nop 4')]
        b += self.max_ops(X)[:-1]                   # v{T+6} = tile max of S (s~ - m c)
        b.append(V(f'v_add_f32 v{T + 7}, {ORDET_DELTA[self.dtype]!r}, v{T + 6}', T + 7, [T + 6]))
        b.append(V(f'v_cmp_lt_f32 vcc, 0, v{T + 7}', 'vcc', [T + 7]))
        b.append(Inst(f'v_cndmask_b32 v{T + 7}, 0, v{T + 7}, vcc', 'valu', rd=[f'v{T + 7}', 'vcc'], wr=[f'v{T + 7}']))
        b.append(V(f'v_sub_f32 v{T}, 0, v{T + 7}', T, [T + 7]))
        b.append(V(f'v_exp_f32 v{T}, v{T}', T, [T], kind='trans'))
        b.append(V(f'v_add_f32 v{mc}, v{mc}, v{T + 7}', mc, [mc, T + 7]))
        b += [V(f'v_sub_f32 v{r}, v{r}, v{T + 7}', r, [r, T + 7]) for r in range(V_SEED[X], V_SEED[X] + 16)]
        b += self.scale_acc(X)
        b.append(raw('s_nop 2'))
        b.append(raw(f's_branch {ret}'))
        return b

    def first_max(self):
        """FIRST_MAX (prologue, after QK_A(0)): QK_B(0) into S_B as well, then per block the
        row max of tile 0 sets the starting shift (m c = max c + delta, as the rescale block
        would, O and the row sums being zero): tile 0 then passes the ORDET test instead of always
        taking the out-of-line rescale. PRESCALE: the seeds and S_A(0) (already seeded) move by
        the shift, S_B(0) is recomputed by tile 0's QK_B with the new seed. Only when tile 0 is
        unmasked for every row (S_MSTART > 0): a masked first tile keeps the initial state (the
        max over keys a row may not see could shift its P out of range)."""
        # (8 waves: one block per wave, S_A(0) only; its QK(1) runs in phase 0)
        out = self.qk('B', 0) if NWAVES == 4 else []
        out.append(Inst(f's_cmp_lg_u32 s{S_MSTART}, 0', 'salu', 2, rd=[f's{S_MSTART}']))
        out.append(Inst('s_cselect_b64 s[96:97], -1, 0', 'salu', 2, wr=['s96', 's97']))
        for X in BLOCKS:
            T, mc = V_TMP[X], V_MC[X]
            out += self.max_ops(X)[:-1]            # v{T+6}: tile max of S_X
            if PRESCALE:
                # S holds s~ - m c: T6 + delta is the shift (> 0: m c starts at -SEED0)
                out.append(V(f'v_add_f32 v{T + 7}, {ORDET_DELTA[self.dtype]!r}, v{T + 6}', T + 7, [T + 6]))
                out.append(Inst(f'v_cndmask_b32 v{T + 7}, 0, v{T + 7}, s[96:97]', 'valu', 4,
                                rd=[f'v{T + 7}', 's96', 's97'], wr=[f'v{T + 7}']))
                out.append(V(f'v_add_f32 v{mc}, v{mc}, v{T + 7}', mc, [mc, T + 7]))
                out += [V(f'v_sub_f32 v{r}, v{r}, v{T + 7}', r, [r, T + 7]) for r in range(V_SEED[X], V_SEED[X] + 16)]
                if X == 'A':
                    out += [V(f'v_sub_f32 v{r}, v{r}, v{T + 7}', r, [r, T + 7]) for r in range(V_S['A'], V_S['A'] + 32)]
            else:
                out.append(V(f'v_mul_f32 v{T + 7}, s{S_C}, v{T + 6}', T + 7, [T + 6]))
                out.append(V(f'v_add_f32 v{T + 7}, {ORDET_DELTA[self.dtype]!r}, v{T + 7}', T + 7, [T + 7]))
                out.append(Inst(f'v_cndmask_b32 v{mc}, v{mc}, v{T + 7}, s[96:97]', 'valu', 4,
                                rd=[f'v{mc}', f'v{T + 7}', 's96', 's97'], wr=[f'v{mc}']))
                if MC_BANKS:
                    out += [V(f'v_mov_b32 v{c}, v{mc}', c, [mc]) for c in range(V_MCB[X], V_MCB[X] + 4)]
        return out

    def scale_acc(self, X):
        """Rescale tail: m*c copies (MC_BANKS), O_X and the row sums times alpha (v{T})."""
        T, mc = V_TMP[X], V_MC[X]
        O, L = A_O[X], A_L[X]
        b = []
        if MC_BANKS:
            b += [V(f'v_mov_b32 v{c}, v{mc}', c, [mc]) for c in range(V_MCB[X], V_MCB[X] + 4)]
        for r in range(D // 2):
            t = T + 2 + (r % 4)
            b.append(Inst(f'v_accvgpr_read_b32 v{t}, a{O + r}', 'accr', rd=[f'a{O + r}'], wr=[f'v{t}']))
            b.append(V(f'v_mul_f32 v{t}, v{t}, v{T}', t, [t, T]))
            b.append(Inst(f'v_accvgpr_write_b32 a{O + r}, v{t}', 'accw', rd=[f'v{t}'], wr=[f'a{O + r}']))
        b.append(Inst(f'ds_bpermute_b32 v{T + 1}, v{V_BPA}, v{T}', 'ds', 2, rd=[f'v{V_BPA}', f'v{T}'], wr=[f'v{T + 1}']))
        for r in range(4):
            t = T + 2 + r
            if QL_VGPR:
                b.append(V(f'v_mul_f32 v{L + r}, v{L + r}, v{T + 1}', L + r, [L + r, T + 1]))
                continue
            b.append(Inst(f'v_accvgpr_read_b32 v{t}, a{L + r}', 'accr', rd=[f'a{L + r}'], wr=[f'v{t}']))
            b.append(V(f'v_mul_f32 v{t}, v{t}, v{T + 1}', t, [t, T + 1]))
            b.append(Inst(f'v_accvgpr_write_b32 a{L + r}, v{t}', 'accw', rd=[f'v{t}'], wr=[f'a{L + r}']))
        return b

    # ------------------------------------------------------------------ epilogue of a block
    def epilogue(self, X):
        """Normalise O_X by the row sum, store O (16-B stores after a permlane32 pair swap,
        T21) and the LSE = (m c + log2 l) ln 2; an empty row (l == 0) gets 0 and -inf."""
        S, T, mc = V_S[X], (V_TMP[X] if V_EPT is None else V_EPT), V_MC[X]
        O, L = A_O[X], A_L[X]
        e = []
        if QL_VGPR:
            e.append(V(f'v_mov_b32 v{T}, v{L}', T, [L]))
        else:
            e.append(Inst(f'v_accvgpr_read_b32 v{T}, a{L}', 'accr', rd=[f'a{L}'], wr=[f'v{T}']))
        e.append(Inst(f'ds_bpermute_b32 v{T + 1}, v{V_BPL}, v{T}', 'ds', 2, rd=[f'v{V_BPL}', f'v{T}'], wr=[f'v{T + 1}']))
        e.append(V(f'v_rcp_f32 v{T + 2}, v{T + 1}', T + 2, [T + 1], kind='trans', cost=8))
        e.append(V(f'v_cmp_nlg_f32 vcc, 0, v{T + 1}', 'vcc', [T + 1]))
        e.append(Inst(f'v_cndmask_b32 v{T + 2}, v{T + 2}, v{V_ONEF}, vcc', 'valu', rd=[f'v{T + 2}', f'v{V_ONEF}', 'vcc'],
                      wr=[f'v{T + 2}']))
        e.append(V(f'v_log_f32 v{T + 3}, v{T + 1}', T + 3, [T + 1], kind='trans', cost=8))
        e.append(V(f'v_add_f32 v{T + 3}, v{T + 3}, v{mc}', T + 3, [T + 3, mc]))
        e.append(V(f'v_mul_f32 v{T + 3}, 0x3f317218, v{T + 3}', T + 3, [T + 3]))
        e.append(Inst(f'v_cndmask_b32 v{T + 3}, v{T + 3}, v{V_NEGINF}, vcc', 'valu', rd=[f'v{T + 3}', f'v{V_NEGINF}', 'vcc'],
                      wr=[f'v{T + 3}']))
        if 'noepi' not in PROBE:     # timing probe: no LSE / O stores (the store tail's price)
            e.append(Inst(f'buffer_store_dword v{T + 3}, v{V_LOFF[X]}, s[{S_LD}:{S_LD + 3}], 0 offen', 'vstore', 8,
                          rd=[f'v{T + 3}', f'v{V_LOFF[X]}']))
        for dt in range(NDT):
            for gi, g in enumerate((0, 2)):
                # registers 4g..4g+7 of d-block dt hold d = 8g + 4hi + 0..3 and 8(g+1) + 4hi + 0..3
                base = O + 16 * dt + 4 * g
                E, Wb = epi_regs(X, dt * 2 + gi)   # 8 fp32 temps, 4 packed words (dead registers)
                for k in range(8):
                    e.append(Inst(f'v_accvgpr_read_b32 v{E + k}, a{base + k}', 'accr', rd=[f'a{base + k}'],
                                  wr=[f'v{E + k}']))
                for k in range(8):
                    e.append(V(f'v_mul_f32 v{E + k}, v{E + k}, v{T + 2}', E + k, [E + k, T + 2]))
                # a0 -> Wb+0 (regs 0,1), a1 -> Wb+1 (2,3), b0 -> Wb+2 (4,5), b1 -> Wb+3 (6,7)
                for k in range(4):
                    e.append(V(f'{self.cvt} v{Wb + k}, v{E + 2 * k}, v{E + 2 * k + 1}', Wb + k,
                               [E + 2 * k, E + 2 * k + 1]))
                # swap(a0, b0), swap(a1, b1): lanes 0-31 then hold d = 8g..8g+7 and lanes 32-63
                # d = 8(g+1)..8(g+1)+7, in store order {a0', a1', b0', b1'} = Wb..Wb+3
                e.append(Inst(f'v_permlane32_swap_b32 v{Wb + 0}, v{Wb + 2}', 'perm', 4, rd=[f'v{Wb}', f'v{Wb + 2}'],
                              wr=[f'v{Wb}', f'v{Wb + 2}']))
                e.append(Inst(f'v_permlane32_swap_b32 v{Wb + 1}, v{Wb + 3}', 'perm', 4, rd=[f'v{Wb + 1}', f'v{Wb + 3}'],
                              wr=[f'v{Wb + 1}', f'v{Wb + 3}']))
                if O_BASE:   # one row base + immediate (head_dim == D)
                    oreg, oimm = V_OOFF[X], f' offset:{16 * (4 * dt + g)}'
                else:
                    oreg, oimm = V_OOFF[X] + dt * 2 + gi, ''
                if D_NAME == 96 and dt == 2 and g == 2:
                    # columns 80..95: dropped for head_dim 80 (the offset pushed past num_records)
                    e += [Inst('s_cmp_gt_u32 s74, 80', 'salu', 2, rd=['s74']),
                          Inst('s_cselect_b32 s96, 0, 0x80000000', 'salu', 2, wr=['s96']),
                          V(f'v_or_b32 v{T + 4}, s96, v{oreg}', T + 4, [oreg])]
                    oreg = T + 4
                if 'noepi' not in PROBE:
                    e.append(Inst(f'buffer_store_dwordx4 {vs(Wb, 4)}, v{oreg}, s[{S_OD}:{S_OD + 3}], 0 offen{oimm}',
                                  'vstore', 8, rd=rv(Wb, 4) + [f'v{oreg}']))
        return e

    # ------------------------------------------------------------------ phases
    @staticmethod
    def tail_test(sm, mf):
        """PHASE_TAIL: the rescale test (and everything before it in the fill) is issued before
        the phase's last PHASE_TAIL MFMAs and the branch after them, so the compare's latency
        runs under those MFMAs instead of stalling the branch."""
        if PHASE_TAIL and len(sm) >= 2 and sm[-1].kind == 'br' and len(mf) > PHASE_TAIL:
            sm[-2].deadline = len(mf) - PHASE_TAIL
            sm[-1].not_before = len(mf)

    def phase1(self, t, masked=False, last=False, rescue=None, kv_next=False):
        """Tile t, phase 1: QK_B(t) + PV_B(t-1) + row sums beside block A's softmax of tile t,
        K(t+1) fragment reads and the K(t+1+DIST) DMA."""
        qkb = self.qk('B', t)
        mf = qkb + self.pv_sum('B', t - 1)[0]
        sm = self.softmax('A', masked, rescue)
        self.tail_test(sm, mf)
        side = [] if last else self.kreads(t + 1)
        if KSPLIT and NBK == 2:
            side = side[:len(side) - KSPLIT]     # the rest go to phase 2 (kreads_late)
        k_lo = 16
        if NBK == 1:
            # one K buffer: the reads of K(t+1) overwrite what QK_B(t) reads; they go behind its
            # last MFMA, in the part of the softmax stream that lands there
            for x in side:
                x.not_before = len(qkb)
            k_lo = len(sm) * sum(m.pipe for m in qkb) // sum(m.pipe for m in mf) + 2
        if VREADS_P1:
            vr = [x for _, x in self.vreads(t)]
            # KFIRST: K(t+1) (needed by the first MFMA of phase 2) before the V^T reads, so the
            # counted wait at phase 2's start covers only the K reads, issued early in the phase
            side = side + vr if KFIRST and NBK == 2 else vr + side
            if KFIRST and NBK == 2:
                k_lo = KFIRST_LO
        dma = [] if (last or DMA_P2) else self.dma('K', t + 1 + DIST)
        if kv_next:     # tail tile t (block tile nt - 4 + t) loads K(nt + t) = the next block's K(t)
            dma = self._dma('K', t, nxt=True)
        fill = merge(sm, [(i, x) for i, x in zip(spread(len(side), k_lo, len(sm) - 4), side)] +
                     [(i, x) for i, x in zip(spread(len(dma), 6, len(sm) - 10), dma)])
        return [mark()] + place(mf, fill)

    def phase2(self, t, masked=False, last=False, rescue=None, kv_next=False):
        """Tile t, phase 2: QK_A(t+1) + PV_A(t) + row sums beside block B's softmax of tile t,
        V(t) fragment reads (deadline: 3 MFMAs before their P.V MFMA) and the V(t+DIST) DMA."""
        qk = [] if last else self.qk('A', t + 1)
        pv, use = self.pv_sum('A', t)
        mf = qk + pv
        sm = self.softmax('B', masked, rescue)
        self.tail_test(sm, mf)
        vr = []
        for f, ins in ([] if VREADS_P1 else self.vreads(t)):
            ins.deadline = max(0, len(qk) + use[f] - 3)
            vr.append(ins)
        dma = [] if last else self.dma('V', t + DIST)
        if kv_next:     # V(nt - 1 + t): this block's last V tile, then the next block's V(t - 1)
            dma = self.dma('V', t + DIST) if t == 0 else self._dma('V', t - 1, nxt=True)
        if DMA_P2 and not last:
            dma = self.dma('K', t + 1 + DIST) + dma
        # the V reads go early (two per softmax instruction pair), the DMA pieces in the middle
        kl = []
        if KSPLIT and NBK == 2 and not last:
            # KSPLIT: the last K(t+1) fragment reads (sub-tile 1) open this phase, each issued at
            # least 3 MFMAs before QK_A(t+1)'s MFMA that reads it
            rd = self.kreads(t + 1)
            for j, x in enumerate(rd[len(rd) - KSPLIT:]):
                x.deadline = max(0, len(rd) - KSPLIT + j - KSPLIT_LAG)
                kl.append(x)
        fill = merge(sm, [(i, x) for i, x in enumerate(kl)] +
                     [(i, x) for i, x in zip(spread(len(vr), 1, 56), vr)] +
                     [(i, x) for i, x in zip(spread(len(dma), 30, len(sm) - 10), dma)])
        return [mark()] + place(mf, fill)

    def phase_w8(self, t, masked=False, last=False, rescue=None):
        """8-wave form, tile t (one 32-row block per wave; 'A'/'B' = register buffers of even/odd
        tiles): QK(t+1) + PV(t-1) + row sums beside the softmax of tile t. The single K buffer
        takes K(t+2) behind the QK MFMAs that read K(t+1); the single V^T buffer takes V(t)
        behind the P.V MFMA that read each fragment of V(t-1). DMA: K(t+1+DIST), V(t+DIST)."""
        X, Y, Z = par(t), par(t + 1), par(t - 1)
        qk = [] if last else self.qk(Y, t + 1)
        pv, use = self.pv_sum(Z, t - 1)
        mf = qk + pv
        sm = self.softmax(X, masked, rescue)
        kr = [] if last else self.kreads(t + 2)
        for x in kr:
            x.not_before = len(qk)
        vr = []
        for f, ins in self.vreads(t):
            ins.not_before = len(qk) + use[f] + 1
            vr.append(ins)
        dma = [] if last else self.dma('K', t + 1 + DIST) + self.dma('V', t + DIST)
        # the rescale branch (end of the softmax stream) scales the O and row sums that this
        # phase's PV(t-1) MFMAs accumulate into: it follows every MFMA of the phase
        br = sm[-1] if sm and sm[-1].kind == 'br' else None
        body = sm[:-1] if br else sm
        n = len(body)
        if PINGPONG:
            # matrix segment: the MFMAs with the DMA pieces and the K(t+2) reads (behind QK(t+1))
            # in their gaps; vector segment: the softmax with the V^T(t) reads spread over it (every
            # P.V MFMA that read V^T(t-1) is issued by then). Waves 4-7 take their barrier between
            # the two segments (tile_body), so each SIMD pairs one wave's MFMAs with its partner's
            # softmax.
            for x in vr:
                x.not_before = None
            vseg = merge(body, [(i, x) for i, x in zip(spread(len(vr), 2, max(3, n - 8)), vr)])
            if br:
                vseg.append(br)
            if vseg:
                vseg[0].not_before = len(mf)
            return [mark()] + place(mf, dma + kr + vseg)
        k_lo = n * len(qk) // max(1, len(mf)) + 1
        fill = merge(body, [(i, x) for i, x in zip(spread(len(kr), k_lo, n * 3 // 4), kr)] +
                     [(i, x) for i, x in zip(spread(len(dma), 4, n // 2), dma)])
        # the V^T reads follow their P.V MFMAs (second half of the phase): after the softmax
        fill += vr
        if br:
            br.not_before = len(mf)
            fill.append(br)
        return [mark()] + place(mf, fill)


def par(t):
    """Register buffer ('A' even / 'B' odd) of tile t in the 8-wave form."""
    return 'A' if t % 2 == 0 else 'B'


def mark():
    return Inst('', 'mark', 0)


def probe_filter(xs, keep_last=False):
    """Timing probes (--probe): drop or cheapen one instruction class of the softmax stream.
    keep_last keeps the final instruction (the rescale test) so control flow stays intact."""
    drop = {'noexp': 'v_exp', 'nofma': 'v_fma', 'nocvt': 'v_cvt', 'nomax': 'v_max'}
    tail = xs[-1:] if keep_last else []
    body = xs[:-1] if keep_last else list(xs)
    for k, pre in drop.items():
        if k in PROBE:
            body = [x for x in body if not x.txt.startswith(pre)]
    if 'expmov' in PROBE:
        for x in body:
            if x.txt.startswith('v_exp_f32'):
                x.txt, x.kind, x.cost = x.txt.replace('v_exp_f32', 'v_mov_b32'), 'valu', 4
    if 'noor' in PROBE and tail and tail[0].txt.startswith('v_cmp_ne_u32 vcc, 0,'):
        # timing probe: no OR-tree rescale test (a compare that never fires)
        body = [x for x in body if not x.txt.startswith(('v_or3_b32', 'v_or_b32', 'v_and_b32'))]
        r = tail[0].txt.split()[-1]
        tail = [V(f'v_cmp_gt_u32 vcc, 0, {r}', 'vcc', [r])]
    if 'nobrdep' in PROBE and tail and tail[0].txt.startswith('v_cmp_ne_u32 vcc, 0,'):
        # timing probe: the OR tree stays, the branch tests a register it does not produce
        tail = [V(f'v_cmp_gt_u32 vcc, 0, v{V_ONEF}', 'vcc', [V_ONEF])]
    return body + tail


def spread(n, lo, hi):
    """n positions spread evenly over [lo, hi)."""
    if n == 0:
        return []
    hi = max(hi, lo + 1)
    return [lo + (hi - lo) * k // n for k in range(n)]


def merge(base, extra):
    """Insert (position, inst) pairs into the list `base` (position = index in base before
    which the extra instruction goes; stable for equal positions)."""
    out = []
    extra = sorted(extra, key=lambda p: p[0])
    k = 0
    for i, x in enumerate(base):
        while k < len(extra) and extra[k][0] <= i:
            out.append(extra[k][1])
            k += 1
        out.append(x)
    out.extend(x for _, x in extra[k:])
    return out


def place(mfmas, fillers, window=10):
    if 'nomfma' in PROBE:
        mfmas = []
    """Distribute the filler sequence over the gaps after each MFMA in proportion to the MFMA
    pipe cycles; a filler with a deadline k is issued before MFMA k. Within that, a small list
    scheduler may issue a later independent filler first when the next one would need wait
    states (e.g. the permlane after the max tree)."""
    M = len(mfmas)
    if M == 0:
        return schedule_run([], list(fillers), window)
    total = sum(f.cost for f in fillers)
    pipe = [m.pipe for m in mfmas]
    P = float(sum(pipe))
    out, acc, cum = [], 0.0, 0
    rest = list(fillers)
    for g in range(-1, M):
        if g >= 0:
            out.append(mfmas[g])
            cum += pipe[g]
        target = total * cum / P if g >= 0 else 0.0
        if g == M - 1:
            target = float('inf')
        # every filler up to the last one whose deadline is g + 1 must be issued now
        forced = -1
        for i, f in enumerate(rest):
            if f.deadline is not None and f.deadline <= g + 1:
                forced = i
        take = 0
        a2 = acc
        while take < len(rest) and (take <= forced or a2 + rest[take].cost * 0.5 <= target):
            nb = rest[take].not_before
            if nb is not None and nb > g + 1:
                break     # must follow MFMA nb-1 (not issued yet): in-order stream waits
            a2 += rest[take].cost
            take += 1
        chunk, rest = rest[:take], rest[take:]
        acc = a2
        out = schedule_run(out, chunk, window)
    return out


def conflicts(a, b):
    """True if a and b may not be swapped (register dependences or control flow)."""
    if a.kind in ('label', 'mark') or b.kind in ('label', 'mark'):
        return True
    ra_, wa = a.rd | a.rdc, a.wr
    rb_, wb = b.rd | b.rdc, b.wr
    return bool(wa & rb_ or wb & ra_ or wa & wb)


def schedule_run(out, chunk, window):
    """Append `chunk` (in order, but a filler may be issued ahead of at most `window` others it
    does not depend on) to `out`, preferring fillers that need no wait states now."""
    chunk = list(chunk)
    while chunk:
        pick = 0
        if need_now(out, chunk[0]) > 0:
            for j in range(1, min(window, len(chunk))):
                c = chunk[j]
                if any(conflicts(chunk[i], c) for i in range(j)):
                    continue
                if need_now(out, c) == 0:
                    pick = j
                    break
        out.append(chunk.pop(pick))
    return out


def need_now(out, x, lookback=16):
    """Wait states x would need if issued after `out` (writers within the last instructions)."""
    need, dist = 0, 0
    regs = set(x.rd) | set(x.rdc)
    if x.kind == 'dma':
        regs.add('m0')
    for w in reversed(out[-lookback:]):
        if w.kind in ('label', 'mark'):
            continue
        for reg in regs & w.wr:
            need = max(need, need_states(w, x, reg) - dist)
        dist += states_of(w)
    return need


# ------------------------------------------------------------------------------------------
# hazard pass: wait states and counted waits along explicit control-flow paths
# ------------------------------------------------------------------------------------------
VALU_KINDS = ('valu', 'trans', 'perm', 'accr', 'accw', 'rfl')


def states_of(x):
    if x.kind in ('label', 'mark', 'wait'):
        return 0
    if x.kind in ('nop', 'raw') and x.txt.startswith('s_nop'):
        return int(x.txt.split()[1]) + 1
    if x.kind == 'raw' and (x.txt.startswith('s_waitcnt') or x.txt.endswith(':')):
        return 0
    return 1


def need_states(w, r, reg):
    """Minimum distance (in issued states; 1 = back to back) from writer w to reader r of reg:
    the gfx950 wait states hipcc's hazard recognizer inserts, plus one."""
    if w.kind == 'mfma':
        if r.kind == 'mfma' and reg in r.rdc and w.wr == r.wr:
            return 0                                   # same-accumulator chain
        return 13 if w.pipe == 32 else 9               # s_nop 11 / s_nop 7
    if w.kind in VALU_KINDS:
        if reg.startswith('s') and r.kind in ('salu', 'm0', 'smem', 'dma', 'vload', 'vstore', 'br'):
            return 6
        if r.kind == 'mfma' or r.kind == 'perm':
            return 3                                   # s_nop 1
        if r.kind == 'rfl':
            return 2                                   # s_nop 0 (v_readfirstlane / v_readlane)
        if w.kind == 'trans' and r.kind in VALU_KINDS:
            return 2                                   # s_nop 0
        return 0
    if w.kind == 'm0' and r.kind == 'dma':
        return 2
    return 0


def parse_wait(txt):
    """(vmcnt, lgkmcnt) limits of an s_waitcnt text (None = unconstrained)."""
    vm = lg = None
    for part in txt.replace(',', ' ').split()[1:]:
        if part.startswith('vmcnt('):
            vm = int(part[6:-1])
        elif part.startswith('lgkmcnt('):
            lg = int(part[8:-1])
    return vm, lg


def analyse(path):
    """path: list of (block_list, index) references in execution order. Returns the list of
    (block_list, index, Inst) insertions needed before the instruction at that index."""
    ins = []
    last_w = {}          # reg -> (state position, writer Inst)
    pos = 0
    lgkm = []            # outstanding DS / SMEM ops: (Inst, regs, phase_id)
    vm = []              # outstanding vector-memory ops: (Inst, regs)
    phase = 0
    for blk, i in path:
        x = blk[i]
        if x.kind == 'mark':
            phase += 1
            continue
        if x.kind in ('raw', 'wait') and x.txt.startswith('s_waitcnt'):
            v_lim, l_lim = parse_wait(x.txt)
            if l_lim is not None:
                lgkm = lgkm[len(lgkm) - l_lim:] if l_lim < len(lgkm) else lgkm
                if l_lim == 0:
                    lgkm = []
            if v_lim is not None:
                vm = vm[len(vm) - v_lim:] if v_lim < len(vm) else vm
                if v_lim == 0:
                    vm = []
            continue
        if x.kind == 'raw' and x.txt.startswith('s_barrier'):
            pos += 1
            continue
        regs = set(x.rd) | set(x.rdc)
        touch = regs | set(x.wr)
        # counted waits for outstanding LDS / vector-memory results
        pre = []
        k_l = max((k for k, (_, rr, _) in enumerate(lgkm) if rr & touch), default=-1)
        if x.kind in ('ds', 'smem') and len(lgkm) >= 15:
            k_l = max(k_l, 0)
        if k_l >= 0:
            younger = len(lgkm) - 1 - k_l
            in_phase = sum(1 for (_, _, ph) in lgkm if ph == phase)
            # counts reach back across phase marks only with LGKM_XPHASE (every control-flow path
            # into the phase is enumerated, so the younger count is exact on each); the hardware
            # counter holds at most 15
            n = min(younger, 15) if LGKM_XPHASE else min(younger, in_phase)
            if any(o.kind == 'smem' for (o, _, _) in lgkm[:k_l + 1]):
                n = 0
            pre.append(Inst(f's_waitcnt lgkmcnt({n})', 'wait', 0))
            lgkm = lgkm[len(lgkm) - n:] if n else []
        k_v = max((k for k, (_, rr) in enumerate(vm) if rr & touch), default=-1)
        if k_v >= 0:
            n = len(vm) - 1 - k_v
            pre.append(Inst(f's_waitcnt vmcnt({n})', 'wait', 0))
            vm = vm[len(vm) - n:] if n else []
        # wait states
        need = 0
        for reg in regs:
            if reg in last_w:
                wp, w = last_w[reg]
                need = max(need, need_states(w, x, reg) - (pos - wp))
        if x.kind == 'dma' and 'm0' in last_w:
            wp, w = last_w['m0']
            need = max(need, need_states(w, x, 'm0') - (pos - wp))
        if need > 0:
            pre.append(Inst(f's_nop {need - 1}', 'nop', 4 * need))
            pos += need
        for p in pre:
            ins.append((blk, i, p))
        pos += states_of(x)
        for reg in x.wr:
            last_w[reg] = (pos - 1, x)
        if x.kind in ('ds', 'smem'):
            lgkm.append((x, set(x.wr), phase))
        elif x.kind in ('dma', 'vload', 'vstore'):
            vm.append((x, set(x.wr)))
    return ins


def apply_insertions(ins):
    # one wait / nop of each sort per position: the strictest of the requests (a position can be
    # reached along several paths or twice along one)
    best = {}
    for blk, i, p in ins:
        key = (id(blk), i, p.txt.split()[0] + (p.txt.split('(')[0] if p.kind == 'wait' else ''))
        if key not in best:
            best[key] = (blk, i, p)
        else:
            q = best[key][2]
            if p.kind == 'nop':
                if int(p.txt.split()[1]) > int(q.txt.split()[1]):
                    best[key] = (blk, i, p)
            else:
                if int(p.txt.split('(')[1][:-1]) < int(q.txt.split('(')[1][:-1]):
                    best[key] = (blk, i, p)
    ins = list(best.values())
    by_blk = {}
    for blk, i, p in ins:
        by_blk.setdefault(id(blk), (blk, []))[1].append((i, p))
    for blk, lst in by_blk.values():
        grouped = {}
        for i, p in lst:
            grouped.setdefault(i, []).append(p)
        for i in sorted(grouped, reverse=True):
            blk[i:i] = grouped[i]
    return len(ins)


def fix_paths(paths, max_iter=400):
    """Insert waits / nops until every path is clean (paths are rebuilt after each change,
    since insertions move block indices)."""
    total = 0
    for _ in range(max_iter):
        changed = 0
        for mk in paths:      # every path once per sweep (each rebuilt after the previous insertions)
            ins = analyse(mk())
            if ins:
                changed += apply_insertions(ins)
        total += changed
        if not changed:
            return total
    raise RuntimeError('hazard pass did not converge')


def refs(blk):
    return [(blk, i) for i in range(len(blk))]


# ------------------------------------------------------------------------------------------
# the kernel program
# ------------------------------------------------------------------------------------------
def S(txt, rd=(), wr=(), kind='salu'):
    return Inst(txt, kind, 2, rd=rd, wr=wr)


def xfun(dst, r, t1, t2):
    """x(r) of the LDS swizzle (fa_common.h Swz<D>): D = 64: u = (r>>1)&7, x = ((u&1)<<2)|(u>>1);
    D = 128: x = ((r&3)<<2)|((r>>2)&3)."""
    if D == 32:
        return [V(f'v_bfe_u32 v{dst}, v{r}, 2, 2', dst, [r])]
    lo = (1, 1) if D == 64 else (0, 2)
    return [V(f'v_bfe_u32 v{t1}, v{r}, {lo[0]}, {lo[1]}', t1, [r]),
            V(f'v_lshlrev_b32 v{t1}, 2, v{t1}', t1, [t1]),
            V(f'v_bfe_u32 v{t2}, v{r}, 2, 2', t2, [r]),
            V(f'v_or_b32 v{dst}, v{t1}, v{t2}', dst, [t1, t2])]


def make_desc(d, ptr, start, rs, hs_lo, hs_hi, seqlen):
    """Buffer descriptor s[d:d+3] for one (sequence, head): base = ptr + start*rs + h*hs (64-bit),
    num_records = seqlen*rs bytes (rows past the sequence read as zero / drop their stores)."""
    h = S_T + 9
    return [S(f's_mul_i32 s92, s{start}, s{rs}'), S(f's_mul_hi_u32 s93, s{start}, s{rs}'),
            S(f's_add_u32 s{d}, s{ptr}, s92'), S(f's_addc_u32 s{d + 1}, s{ptr + 1}, s93'),
            S(f's_mul_i32 s92, s{h}, s{hs_lo}'), S(f's_mul_hi_u32 s93, s{h}, s{hs_lo}'),
            S(f's_mul_i32 s94, s{h}, s{hs_hi}'), S('s_add_u32 s93, s93, s94'),
            S(f's_add_u32 s{d}, s{d}, s92'), S(f's_addc_u32 s{d + 1}, s{d + 1}, s93'),
            S(f's_mul_i32 s{d + 2}, s{seqlen}, s{rs}'), S(f's_mov_b32 s{d + 3}, 0x00020000')]


WAVE_MODE = 'late'


def wave_id_insts():
    """Wave index within the workgroup (tid >> 6) into an SGPR. (gfx950: a v_readfirstlane
    right behind the VALU that wrote its source reads the stale VGPR: the hazard pass keeps
    them 2 states apart, as hipcc's s_nop 0 does.)"""
    return [V('v_lshrrev_b32 v1, 6, v0', 1, [0]),
            Inst(f'v_readfirstlane_b32 s{S_WAVE}, v1', 'rfl', rd=['v1'], wr=[f's{S_WAVE}'])]


def sec(name):
    """Section marker inside the prologue list (prologue_sections splits on them)."""
    return Inst(name, 'sec', 0)


PRO_ORDER = ('args', 'decode', 'decode_map', 'decode_wait', 'wave', 'state', 'soffinit', 'state2', 'lanes', 'rows',
             'qload', 'dma', 'lanes_lds', 'lanes2', 'qscale', 'zero', 'start')


PRO_ORDER_R5 = ('args', 'decode', 'decode_map', 'decode_wait', 'wave', 'state', 'soffinit', 'state2', 'lanes',
                'lanes_lds', 'rows', 'lanes2', 'qload', 'dma', 'qscale', 'zero', 'start')   # round 5 (--proorder 0)
PRO_ORDER_LANES_FIRST = ('args', 'decode', 'decode_map', 'wave', 'lanes', 'lanes_lds', 'decode_wait', 'state',
                         'soffinit', 'state2', 'rows', 'lanes2', 'qload', 'dma', 'qscale', 'zero', 'start')  # --proorder 2


def prologue(g):
    """The one-block prologue: its sections in PRO_ORDER (the per-lane address setup, which needs no
    decoded value, between the decode's cu_seqlens loads and their first use)."""
    sc = split_sections(prologue_sections(g))
    assert set(sc) == set(PRO_ORDER), sorted(sc)
    return sum((sc[k] for k in PRO_ORDER), [])


def prologue_sections(g):
    """Kernel arguments, (q-block, head, batch) of this workgroup (XCD-aware order as
    fa_fwd_kernel.h), sequence bounds, buffer descriptors, per-lane addresses, Q loads, the first
    DMAs, zeroed accumulators, and QK_A of tile 0."""
    a = S_ARG   # s40 q, s42 k, s44 v, s46 o, s48 lse, s50 cu_q, s52 cu_k, s54 q_hs, s56 k_hs, s58 v_hs,
    #             s60 o_hs, s62 q_rs, s63 k_rs, s64 v_rs, s65 o_rs, s66 nheads, s67 lse row bytes, s68 c,
    #             s69 thr, s70 nqb, s71 nwg, s72 magic(nqb), s73 magic(nheads), s74 head_dim
    p = []
    p.append(Inst('s_load_dwordx16 s[40:55], s[0:1], 0x0', 'smem', 2, wr=[f's{i}' for i in range(40, 56)]))
    p.append(Inst('s_load_dwordx16 s[56:71], s[0:1], 0x40', 'smem', 2, wr=[f's{i}' for i in range(56, 72)]))
    p.append(Inst('s_load_dwordx4 s[72:75], s[0:1], 0x80', 'smem', 2, wr=[f's{i}' for i in range(72, 76)]))
    p.append(Inst(f's_load_dword s{S_CAUSAL}, s[0:1], 0x90', 'smem', 2, wr=[f's{S_CAUSAL}']))
    p.append(Inst(f's_load_dword s{S_MAGIC_BH}, s[0:1], 0x94', 'smem', 2, wr=[f's{S_MAGIC_BH}']))
    # causal XCD groups: s98 per = G nqb (0: global order), s99 magic(per), s100 G, s101 magic(G)
    p.append(Inst('s_load_dwordx2 s[98:99], s[0:1], 0x98', 'smem', 2, wr=['s98', 's99']))
    p.append(Inst('s_load_dwordx2 s[100:101], s[0:1], 0xa0', 'smem', 2, wr=['s100', 's101']))
    p.append(raw('s_waitcnt lgkmcnt(0)'))
    if WAVE_MODE == 'early':
        p += wave_id_insts()
    p.append(sec('decode'))
    # L = x + nqb (y + H z); Lp = xcd q8 + min(xcd, r8) + (L >> 3); bh = Lp / nqb; b = bh / H
    p += [S('s_mul_i32 s80, s66, s4'), S('s_add_u32 s80, s80, s3'), S('s_mul_i32 s80, s80, s70'),
          S('s_add_u32 s80, s80, s2'), sec('decode_map'),
          S('s_and_b32 s81, s80, 7'), S('s_lshr_b32 s82, s71, 3'), S('s_and_b32 s83, s71, 7'),
          S('s_mul_i32 s84, s81, s82'), S('s_min_u32 s85, s81, s83'), S('s_add_u32 s84, s84, s85'),
          S('s_lshr_b32 s85, s80, 3'), S('s_add_u32 s84, s84, s85'),
          S('s_lshl_b32 s85, s84, 1'), S('s_mul_hi_u32 s86, s85, s72'),
          S('s_mul_i32 s87, s86, s70'), S('s_sub_u32 s87, s84, s87')]
    # (the persistent form runs non-causal grids only: the causal block orders below are not in it;
    # there s98..s101 hold its own state)
    p += [] if PERSIST else [
          # causal: global heaviest-first order, rank = L / nbh (s75 = nbh), bh = L - rank nbh,
          # qb = nqb - 1 - rank (the last q-blocks see the most keys)
          S('s_lshl_b32 s85, s80, 1'), S(f's_mul_hi_u32 s81, s85, s{S_MAGIC_BH}'),
          S('s_mul_i32 s82, s81, s75'), S('s_sub_u32 s82, s80, s82'),
          S('s_sub_u32 s83, s70, 1'), S('s_sub_u32 s83, s83, s81'),
          # ... or, when the host gave a group size (s98 = per = G nqb > 0), XCD groups as the HIP
          # kernels (fa_common.h xcd_grouped with full groups): i = L >> 3 on XCD x = L & 7, grp =
          # i / per, w = i % per, rank = w / G, bh = x (nbh / 8) + grp G + w % G
          S('s_lshr_b32 s90, s80, 3'), S('s_lshl_b32 s91, s90, 1'), S('s_mul_hi_u32 s91, s91, s99'),
          S('s_mul_i32 s92, s91, s98'), S('s_sub_u32 s92, s90, s92'),
          S('s_lshl_b32 s93, s92, 1'), S('s_mul_hi_u32 s93, s93, s101'),
          S('s_mul_i32 s94, s93, s100'), S('s_sub_u32 s94, s92, s94'),
          S('s_mul_i32 s95, s91, s100'), S('s_add_u32 s94, s94, s95'),
          S('s_lshr_b32 s95, s75, 3'), S('s_and_b32 s90, s80, 7'), S('s_mul_i32 s95, s95, s90'),
          S('s_add_u32 s94, s94, s95'),
          S('s_sub_u32 s95, s70, 1'), S('s_sub_u32 s95, s95, s93'),
          S('s_cmp_lg_u32 s98, 0'), S('s_cselect_b32 s82, s94, s82'), S('s_cselect_b32 s83, s95, s83'),
          S(f's_cmp_lg_u32 s{S_CAUSAL}, 0'), S('s_cselect_b32 s86, s82, s86'), S('s_cselect_b32 s87, s83, s87')]
    p += [S('s_lshl_b32 s85, s86, 1'), S('s_mul_hi_u32 s88, s85, s73'),
          S('s_mul_i32 s89, s88, s66'), S('s_sub_u32 s89, s86, s89'),
          S('s_lshl_b32 s90, s88, 2'),
          S('s_add_u32 s92, s50, s90'), S('s_addc_u32 s93, s51, 0'),
          Inst('s_load_dwordx2 s[76:77], s[92:93], 0x0', 'smem', 2, wr=['s76', 's77']),
          S('s_add_u32 s94, s52, s90'), S('s_addc_u32 s95, s53, 0'),
          Inst('s_load_dwordx2 s[78:79], s[94:95], 0x0', 'smem', 2, wr=['s78', 's79'])]
    # the cu_seqlens loads' wait is a section of its own: the one-block prologue (prologue(), PRO_ORDER)
    # runs the per-lane address setup between the loads and this wait (the SALU helper S() does not
    # list its registers, so the hazard pass cannot place it); the persistent decodes add it after
    # every copy of decode_map
    p += [sec('decode_wait'), raw('s_waitcnt lgkmcnt(0)')]
    p.append(sec('wave'))
    if WAVE_MODE != 'early':
        p += wave_id_insts()
    p.append(sec('state'))
    p += [S('s_sub_u32 s77, s77, s76'), S('s_sub_u32 s79, s79, s78'),
          S('s_lshl_b32 s90, s87, 8'), S('s_cmp_ge_u32 s90, s77'), raw('s_cbranch_scc1 .Lend')]
    # descriptors: K, V, Q, O, LSE
    p += make_desc(S_KD, 42, 78, 63, 56, 57, 79)
    p += make_desc(S_VD, 44, 78, 64, 58, 59, 79)
    p += make_desc(S_QD, 40, 76, 62, 54, 55, 77)
    p += make_desc(S_OD, 46, 76, 65, 60, 61, 77)
    p += [S('s_mul_i32 s92, s88, s66'), S('s_add_u32 s92, s92, s89'),
          S('s_mul_i32 s93, s92, s67'), S('s_mul_hi_u32 s94, s92, s67'),
          S(f's_add_u32 s{S_LD}, s48, s93'), S(f's_addc_u32 s{S_LD + 1}, s49, s94'),
          S(f's_lshl_b32 s{S_LD + 2}, s77, 2'), S(f's_mov_b32 s{S_LD + 3}, 0x00020000')]
    p += [S(f's_mov_b32 s{S_C}, s68'), S(f's_mov_b32 s{S_THR}, s{68 if PRESCALE else 69}'),
          S(f's_add_u32 s{S_NT}, s79, 63'), S(f's_lshr_b32 s{S_NT}, s{S_NT}, 6'),
          # causal: the q-block's rows end at 256 (qb + 1), so 4 (qb + 1) tiles at most, and the
          # diagonal band (masked loop) starts at tile 4 qb
          S('s_add_u32 s96, s87, 1'), S('s_lshl_b32 s96, s96, 2'), S(f's_min_u32 s97, s{S_NT}, s96'),
          S(f's_cmp_lg_u32 s{S_CAUSAL}, 0'), S(f's_cselect_b32 s{S_NT}, s97, s{S_NT}'),
          S(f's_sub_u32 s{S_LAST}, s{S_NT}, 1'), S(f's_mov_b32 s{S_J}, 0'),
          S('s_lshl_b32 s96, s87, 2'), S(f's_min_u32 s97, s96, s{S_LAST}'),
          S(f's_cmp_lg_u32 s{S_CAUSAL}, 0'), S(f's_cselect_b32 s{S_MSTART}, s97, s{S_LAST}'),
          S(f's_lshl_b32 s{S_KSTEP}, s63, 7'), S(f's_lshl_b32 s{S_VSTEP}, s64, 7'),
          S(f's_lshl_b32 s{S_M0B}, s{S_WAVE}, 10')]
    # SOFF_WALK: the DMA offsets of tiles 0 and 1; else second descriptor sets (odd tiles): one tile
    # (64 rows) further, num_records saturating
    # (own section: the persistent form with CARRY_DECODE places it after the next block's decode,
    # whose temporaries include s80..s83)
    p.append(sec('soffinit'))
    if soff_walk():
        p += [S(f's_mov_b32 s{S_KOFF[0]}, 0'), S(f's_lshl_b32 s{S_KOFF[1]}, s63, 6'),
              S(f's_mov_b32 s{S_VOFF[0]}, 0'), S(f's_lshl_b32 s{S_VOFF[1]}, s64, 6')]
    p.append(sec('state2'))
    for d0, d1, rs in ((S_KD, S_KD1, 63), (S_VD, S_VD1, 64)) if not soff_walk() else ():
        p += [S(f's_lshl_b32 s96, s{rs}, 6'),
              S(f's_add_u32 s{d1}, s{d0}, s96'), S(f's_addc_u32 s{d1 + 1}, s{d0 + 1}, 0'),
              S(f's_sub_u32 s{d1 + 2}, s{d0 + 2}, s96'), S(f's_cselect_b32 s{d1 + 2}, 0, s{d1 + 2}'),
              S(f's_mov_b32 s{d1 + 3}, s{d0 + 3}')]
    # ---- per-lane constants
    p.append(sec('lanes'))
    L = V_LANE
    p += [V(f'v_and_b32 v{L}, 63, v0', L, [0]), V('v_and_b32 v16, 31, v0', 16, [0]),
          V('v_bfe_u32 v17, v0, 5, 1', 17, [0]), V('v_bfe_u32 v18, v0, 2, 2', 18, [0]),
          V('v_and_b32 v19, 3, v0', 19, [0]), V('v_bfe_u32 v20, v0, 4, 1', 20, [0])]
    p += [V(f'v_mov_b32 v{V_NEGINF}, 0xff800000', V_NEGINF, []), V(f'v_mov_b32 v{V_ONEF}, 1.0', V_ONEF, []),
          V('v_mov_b32 v31, 0x80000000', 31, []), V('v_mov_b32 v32, 0', 32, [])]
    # DMA source offsets: pieces `wave + 4i` of a tile; lane l -> row RPP p + l/LPR, slot l%LPR
    # (RPP = rows per 1-KiB piece, LPR = 16-B chunks per row)
    lpr = D // 8
    rpp = 1024 // ROWB
    p += [V(f'v_lshrrev_b32 v33, {lpr.bit_length() - 1}, v{L}', 33, [L]), V(f'v_and_b32 v34, {lpr - 1}, v{L}', 34, [L]),
          S(f's_lshl_b32 s97, s{S_WAVE}, {rpp.bit_length() - 1}')]
    for i in range(NP):
        p += [S(f's_add_u32 s96, s97, {NWAVES * rpp * i}'), V('v_add_u32 v35, s96, v33', 35, [33])]
        p += xfun(36, 35, 37, 38)
        p += [V('v_xor_b32 v36, v34, v36', 36, [34, 36]), V('v_lshlrev_b32 v37, 3, v36', 37, [36]),
              V('v_cmp_gt_u32 vcc, s74, v37', 'vcc', [37]),
              V('v_mul_lo_u32 v38, v35, s63', 38, [35]), V('v_lshl_add_u32 v38, v36, 4, v38', 38, [36, 38]),
              Inst(f'v_cndmask_b32 v{V_DMA + i}, v31, v38, vcc', 'valu', rd=['v31', 'v38', 'vcc'], wr=[f'v{V_DMA + i}']),
              V('v_mul_lo_u32 v38, v35, s64', 38, [35]), V('v_lshl_add_u32 v38, v36, 4, v38', 38, [36, 38]),
              Inst(f'v_cndmask_b32 v{V_DMA + NP + i}, v31, v38, vcc', 'valu', rd=['v31', 'v38', 'vcc'],
                   wr=[f'v{V_DMA + NP + i}'])]
    # K / V^T fragment read addresses (LDS), needed from the first LDS reads on: own section, so that a
    # prologue order may issue the Q loads and first DMAs before it (PRO_ORDER)
    p.append(sec('lanes_lds'))
    p += xfun(21, 16, 22, 23)
    rsh = ROWB.bit_length() - 1     # log2 of the LDS row bytes
    for ks in range(NKS):   # K fragment reads: row l32, chunk 2ks + hi
        p += [V(f'v_add_u32 v22, {2 * ks}, v17', 22, [17]), V('v_xor_b32 v22, v22, v21', 22, [22, 21]),
              V('v_lshlrev_b32 v22, 4, v22', 22, [22]), V(f'v_lshl_add_u32 v{V_KADDR + ks}, v16, {rsh}, v22', V_KADDR + ks, [16, 22])]
    # V^T tr reads: row 4hi + qq + 8 half, column 32 dt + 16 grp + 4 pp
    p += [V('v_lshl_add_u32 v24, v17, 2, v18', 24, [17, 18]), V('v_lshrrev_b32 v25, 1, v19', 25, [19]),
          V('v_lshl_add_u32 v25, v20, 1, v25', 25, [20, 25]), V('v_and_b32 v26, 1, v19', 26, [19]),
          V('v_lshlrev_b32 v26, 3, v26', 26, [26])]
    for half in range(2):
        p += [V(f'v_add_u32 v27, {8 * half}, v24', 27, [24])] + xfun(28, 27, 29, 30)
        for dt in range(NDT):
            p += [V(f'v_add_u32 v29, {4 * dt}, v25', 29, [25]), V('v_xor_b32 v29, v29, v28', 29, [29, 28]),
                  V('v_lshl_or_b32 v29, v29, 4, v26', 29, [29, 26]),
                  V(f'v_lshl_add_u32 v{V_VADDR + dt * 2 + half}, v27, {rsh}, v29', V_VADDR + dt * 2 + half, [27, 29]),
                  V(f'v_add_u32 v{V_VADDR + dt * 2 + half}, {VREG}, v{V_VADDR + dt * 2 + half}',
                    V_VADDR + dt * 2 + half, [V_VADDR + dt * 2 + half])]
    # Q load offsets (v43..v50), O store offsets, LSE offsets of blocks A (rows +0) and B (+32)
    p.append(sec('rows'))
    p += [S(f's_lshl_b32 s93, s{S_WAVE}, {(32 * len(BLOCKS)).bit_length() - 1}'), S('s_add_u32 s93, s93, s90')]
    # (O_BASE, head_dim == D: one row base per block, the chunk offsets as immediates)
    qoff = {'A': 43, 'B': 47} if not O_BASE else {'A': V_P['A'], 'B': V_P['A'] + 1}
    for X, xo in (('A', 0), ('B', 32))[:len(BLOCKS)]:
        p += [V('v_add_u32 v39, s93, v16', 39, [16])]
        if xo:
            p += [V(f'v_add_u32 v39, {xo}, v39', 39, [39])]
        # keys this lane's row may see: min(seqlen_k, row + 1 if causal), minus 4 hi (the mask
        # compares register key offsets without the 4 hi of their lane half)
        p += [V('v_add_u32 v40, 1, v39', 40, [39]),
              V(f'v_cmp_ne_u32 vcc, s{S_CAUSAL}, v32', 'vcc', [32]),
              Inst('v_cndmask_b32 v40, v31, v40, vcc', 'valu', rd=['v31', 'v40', 'vcc'], wr=['v40']),
              V('v_min_u32 v40, s79, v40', 40, [40]), V('v_lshlrev_b32 v41, 2, v17', 41, [17]),
              V(f'v_sub_u32 v{V_ROW1[X]}, v40, v41', V_ROW1[X], [40, 41])]
        if O_BASE:
            p += [V('v_mul_lo_u32 v42, v39, s62', 42, [39]),
                  V(f'v_lshl_add_u32 v{qoff[X]}, v17, 4, v42', qoff[X], [17, 42]),
                  V('v_mul_lo_u32 v42, v39, s65', 42, [39]),
                  V(f'v_lshl_add_u32 v{V_OOFF[X]}, v17, 4, v42', V_OOFF[X], [17, 42])]
        for ks in ([] if O_BASE else range(NKS)):
            p += [V(f'v_add_u32 v40, {2 * ks}, v17', 40, [17]), V('v_lshlrev_b32 v41, 3, v40', 41, [40]),
                  V('v_cmp_gt_u32 vcc, s74, v41', 'vcc', [41]),
                  V('v_mul_lo_u32 v42, v39, s62', 42, [39]), V('v_lshl_add_u32 v42, v40, 4, v42', 42, [40, 42]),
                  Inst(f'v_cndmask_b32 v{qoff[X] + ks}, v31, v42, vcc', 'valu', rd=['v31', 'v42', 'vcc'],
                       wr=[f'v{qoff[X] + ks}'])]
        for dt in ([] if O_BASE else range(NDT)):
            for gi, gg in enumerate((0, 2)):
                p += [V(f'v_add_u32 v40, {4 * dt + gg}, v17', 40, [17]), V('v_lshlrev_b32 v41, 3, v40', 41, [40]),
                      V('v_cmp_gt_u32 vcc, s74, v41', 'vcc', [41]),
                      V('v_mul_lo_u32 v42, v39, s65', 42, [39]), V('v_lshl_add_u32 v42, v40, 4, v42', 42, [40, 42]),
                      Inst(f'v_cndmask_b32 v{V_OOFF[X] + dt * 2 + gi}, v31, v42, vcc', 'valu',
                           rd=['v31', 'v42', 'vcc'], wr=[f'v{V_OOFF[X] + dt * 2 + gi}'])]
        p += [V('v_cmp_eq_u32 vcc, 0, v17', 'vcc', [17]), V('v_lshlrev_b32 v42, 2, v39', 42, [39]),
              Inst(f'v_cndmask_b32 v{V_LOFF[X]}, v31, v42, vcc', 'valu', rd=['v31', 'v42', 'vcc'],
                   wr=[f'v{V_LOFF[X]}'])]
    # ds_bpermute addresses and the 0/1 indicator of the row-sum MFMA
    p.append(sec('lanes2'))
    p += [V(f'v_and_b32 v40, 15, v{L}', 40, [L]), V(f'v_lshrrev_b32 v41, 5, v{L}', 41, [L]),
          V('v_lshl_or_b32 v41, v41, 4, v40', 41, [41, 40]), V(f'v_lshlrev_b32 v{V_BPA}, 2, v41', V_BPA, [41]),
          V(f'v_bfe_u32 v41, v{L}, 4, 1', 41, [L]), V('v_lshl_add_u32 v41, v41, 5, v40', 41, [41, 40]),
          V(f'v_lshlrev_b32 v{V_BPL}, 2, v41', V_BPL, [41]),
          V(f'v_bfe_u32 v41, v{L}, 4, 1', 41, [L]), V(f'v_bfe_u32 v42, v{L}, 3, 1', 42, [L]),
          V('v_cmp_eq_u32 vcc, v41, v42', 'vcc', [41, 42]), V(f'v_mov_b32 v51, {g.one2:#x}', 51, []),
          Inst('v_cndmask_b32 v51, v32, v51, vcc', 'valu', rd=['v32', 'v51', 'vcc'], wr=['v51'])]
    if QL_VGPR:
        p += [V(f'v_mov_b32 v{A_ONES + r}, v51', A_ONES + r, [51]) for r in range(4)]
    else:
        p += [Inst(f'v_accvgpr_write_b32 a{A_ONES + r}, v51', 'accw', rd=['v51'], wr=[f'a{A_ONES + r}']) for r in range(4)]
    # Q fragments ('nopro' timing probe: no Q loads and no first DMAs, the prologue burst's price)
    p.append(sec('qload'))
    if D_NAME == 96 and 'nopro' not in PROBE:
        # head_dim 80: Q's k-step 5 (columns 80..95: another head's, or past the tensor) loads
        # through an offset pushed past num_records (zeros)
        p += [Inst('s_cmp_gt_u32 s74, 80', 'salu', 2, rd=['s74']),
              Inst('s_cselect_b32 s96, 0, 0x80000000', 'salu', 2, wr=['s96'])]
        p += [V(f'v_or_b32 v{V_P["A"] + 2 + i}, s96, v{qoff[X]}', V_P['A'] + 2 + i, [qoff[X]])
              for i, X in enumerate(BLOCKS)]
    for X in ([] if 'nopro' in PROBE else BLOCKS):
        for ks in range(NKS):
            q = A_Q[X] + 4 * ks
            qr, qi = (qoff[X], f' offset:{32 * ks}') if O_BASE else (qoff[X] + ks, '')
            if D_NAME == 96 and ks == 5:
                qr = V_P['A'] + 2 + BLOCKS.index(X)
            p.append(Inst(f'buffer_load_dwordx4 {rq(q)}, v{qr}, s[{S_QD}:{S_QD + 3}], 0 offen{qi}', 'vload', 8,
                          rd=[f'v{qr}'], wr=rqn(q)))
    # first DMAs: K0, [K1 V0], [K2 V1], [K3 V2] (tile t of the loop issues K(t+1+DIST), V(t+DIST))
    p.append(sec('dma'))
    if 'nopro' in PROBE:     # Q = 0 (S = 0: one rescale at tile 0, as always, then none)
        p += [Inst(f'v_accvgpr_write_b32 a{A_Q[X] + r}, 0', 'accw', wr=[f'a{A_Q[X] + r}'])
              for X in BLOCKS for r in range(4 * NKS)] if not QL_VGPR else []
    if 'nopro' not in PROBE:
        p += g.dma('K', 0)
        for t in range(DIST - (1 if defer_dma() else 0)):
            p += g.dma('K', t + 1) + g.dma('V', t)
    # zero O, row sums, the V fragment buffer PV_B(-1) reads and P_B (PV_B(-1) of tile 0 adds
    # nothing); m = -inf
    # PRESCALE: Q~ = Q c right after Q landed (the hazard pass counts the wait past the DMAs just
    # issued), while the first K/V tiles are in flight
    p.append(sec('qscale'))
    p += q_prescale(g)
    p.append(sec('zero'))
    if QL_VGPR:     # row sums in VGPRs (D = 128 layout)
        p += [V(f'v_mov_b32 v{r}, 0', r, []) for r in range(A_L['A'], A_L['B'] + 4)]
    vf1 = A_VF + KFB * ((-1) % NBV)
    # O (and, below D = 128, the row sums) in AGPRs from a0
    o_regs = D if QL_VGPR else A_ONES
    if not MFMA_ZERO:
        p += [Inst(f'v_accvgpr_write_b32 a{r}, v32', 'accw', rd=['v32'], wr=[f'a{r}']) for r in range(o_regs)]
        p += [Inst(f'v_accvgpr_write_b32 a{vf1 + r}, v32', 'accw', rd=['v32'], wr=[f'a{vf1 + r}'])
              for r in range(KFB)]
        p += [V(f'v_mov_b32 v{r}, 0', r, []) for r in range(V_P['B'], V_P['B'] + 16)]
    else:
        # P_B = 0 first; then O, the row sums and the V fragment buffer PV_B(-1) reads are MFMA
        # products of that zero with C = 0 (16 / 4 AGPRs per instruction instead of one)
        p += [V(f'v_mov_b32 v{r}, 0', r, []) for r in range(V_P['B'], V_P['B'] + 16)]
        z = V_P['B']
        for lo, n in ((0, o_regs), (vf1, KFB)):
            r = lo
            while r < lo + n:
                if lo + n - r >= 16 and r % 16 == 0:
                    p.append(Inst(f'{g.mf32} {as_(r, 16)}, {vs(z, 4)}, {vs(z, 4)}, 0', 'mfma', 8,
                                  rd=rv(z, 4), wr=ra(r, 16), pipe=32))
                    r += 16
                elif lo + n - r >= 4 and r % 4 == 0:
                    p.append(Inst(f'{g.mf16} {as_(r, 4)}, {vs(z, 4)}, {vs(z, 4)}, 0', 'mfma', 8,
                                  rd=rv(z, 4), wr=ra(r, 4), pipe=16))
                    r += 4
                else:
                    p.append(Inst(f'v_accvgpr_write_b32 a{r}, v32', 'accw', rd=['v32'], wr=[f'a{r}']))
                    r += 1
    p += [V(f'v_mov_b32 v{r}, v{V_NEGINF}', r, [V_NEGINF]) for r in (V_MC['A'], V_MC['B'])]
    # V_MTHR: the max test's threshold, or with ORDET the OR test's mask (ORDET_ANDOR)
    p += [V(f'v_mov_b32 v{r}, 0x40004000', r, []) if ORDET else V(f'v_mov_b32 v{r}, v{V_NEGINF}', r, [V_NEGINF])
          for r in sorted({V_MTHR['A'], V_MTHR['B']})]
    if PRESCALE:
        p += [V(f'v_mov_b32 v{r}, {-SEED0!r}', r, []) for r in (V_MC['A'], V_MC['B'])]
        p += [V(f'v_mov_b32 v{r}, {SEED0!r}', r, []) for X in BLOCKS for r in range(V_SEED[X], V_SEED[X] + 16)]
    if MC_BANKS:
        p += [V(f'v_mov_b32 v{r}, v{V_NEGINF}', r, [V_NEGINF]) for r in range(V_MCB['A'], V_MCB['B'] + 4)]
    p.append(sec('start'))
    p += [S(f's_cmp_eq_u32 s{S_NT}, 0'), raw('s_cbranch_scc1 .Lempty')]
    # K0, K1, V0 (and Q) landed: all but the 8 youngest pieces
    # (8 waves: phase 0 reads K2 as well: K0 K1 V0 K2 landed, all but the 3 youngest pieces)
    p += [raw(f's_waitcnt vmcnt({3 if NWAVES == 8 else start_pieces()})')]
    p += [raw('s_barrier')]
    if defer_dma() and 'nopro' not in PROBE:
        # DEFER_DMA: the prologue's last DMA tile (K(DIST), V(DIST-1)) goes out after the barrier
        p += g.dma('K', DIST) + g.dma('V', DIST - 1)
    p += stamp(STAMP_V + 12) if 'stamps' in PROBE else []
    p += pstamp(PS_V + 4)
    # every wave reads K0 before any wave passes the next barrier when the loop's first DMA into K0's
    # slot (tile R - 1 - DIST) comes before its first barrier (after tile 0, or tile 1 with BAR2):
    # R 4 / DIST 3 (tile 0 DMAs K4 into slot 0) needs this one, R 6 / DIST 3 with BAR2 does not
    kbar = [raw('s_barrier')] if R - 1 - DIST < (2 if BAR2 else 1) or NWAVES == 8 else []
    p += g.kreads(0) + [raw('s_waitcnt lgkmcnt(0)')] + kbar + g.qk('A', 0)
    if FIRST_MAX and ORDET and (NWAVES == 4 or FIRST_MAX_W8):
        p += g.first_max()
    if NWAVES == 8:
        # K1 into the single K buffer behind QK(0) (phase 0 runs QK(1))
        p += [raw('s_nop 3')] + g.kreads(1)
        if PRIO4:
            p += [S(f's_cmp_lt_u32 s{S_WAVE}, 4'), raw('s_cbranch_scc1 .Lprio_done'), raw('s_setprio 1'),
                  label('.Lprio_done')]
    p += [raw('s_nop 7'), raw('s_nop 3')]
    return p


def q_prescale(g, src=None):
    """PRESCALE: Q~ = rne16(Q c) in place (AGPR fragments of every block, after they landed), or
    from the VGPRs of `src` [(vgpr, agpr), ...] into the AGPRs (the persistent form's prefetched
    next Q): per register the two 16-bit halves widened to fp32, multiplied by c, packed back. The
    per-register chains run 8 at a time, interleaved, so no op waits on its predecessor."""
    if not PRESCALE:
        return []
    if 'noqs' in PROBE:     # timing probe: Q copied unscaled (the pre-scale's price)
        return [Inst(f'v_accvgpr_write_b32 a{q}, v{vq}', 'accw', rd=[f'v{vq}'], wr=[f'a{q}']) for vq, q in (src or [])]
    pairs = src or [(None, A_Q[X] + r) for X in BLOCKS for r in range(4 * NKS)]
    chains = []
    for k, (vq, q) in enumerate(pairs):
        if True:
            # P registers: free (P_B is zeroed later); lo:hi an even-aligned pair (v_pk_mul_f32)
            lo, hi, a = (V_P['A'] + (k % 8) * 4 + j for j in range(3))
            if vq is None:
                c = [Inst(f'v_accvgpr_read_b32 v{a}, a{q}', 'accr', rd=[f'a{q}'], wr=[f'v{a}'])]
            else:
                c, a = [], vq
                a_out = V_P['A'] + (k % 8) * 4 + 3
            if g.dtype == 'bf16':
                c += [V(f'v_lshlrev_b32 v{lo}, 16, v{a}', lo, [a]), V(f'v_and_b32 v{hi}, 0xffff0000, v{a}', hi, [a])]
            else:
                c += [V(f'v_cvt_f32_f16 v{lo}, v{a}', lo, [a]), V(f'v_lshrrev_b32 v{hi}, 16, v{a}', hi, [a]),
                      V(f'v_cvt_f32_f16 v{hi}, v{hi}', hi, [hi])]
            o = a if vq is None else a_out
            # (s[S_C:S_C+1] = (c, c) with PRESCALE: S_THR holds c, the max test that reads it is off)
            c += [Inst(f'v_pk_mul_f32 v[{lo}:{hi}], v[{lo}:{hi}], s[{S_C}:{S_C + 1}]', 'valu', 4,
                       rd=[f'v{lo}', f'v{hi}', f's{S_C}', f's{S_C + 1}'], wr=[f'v{lo}', f'v{hi}']),
                  V(f'{g.cvt} v{o}, v{lo}, v{hi}', o, [lo, hi]),
                  Inst(f'v_accvgpr_write_b32 a{q}, v{o}', 'accw', rd=[f'v{o}'], wr=[f'a{q}'])]
            chains.append(c)
    res = []
    for base in range(0, len(chains), 8):
        grp = chains[base:base + 8]
        for j in range(max(len(c) for c in grp)):
            res += [c[j] for c in grp if j < len(c)]
    return res


def split_sections(lst):
    out, cur = {'args': []}, 'args'
    for x in lst:
        if x.kind == 'sec':
            cur = x.txt
            out[cur] = []
        else:
            out[cur].append(x)
    return out


# ---- persistent form (PERSIST): one workgroup per CU walks logical blocks L = P, P + G, P + 2G, ...
# (the same XCD-aware block order as the one-block-per-workgroup launch), and prefetches the next
# block's Q fragments into spare VGPRs while the current block runs, so that only the first block
# of a workgroup pays the Q part of the prologue's load burst (probe 'nopro': the burst is ~15 %
# of the north star's time).
# Code placement of the main loop (MI355X_MICROARCH.md, two waves per SIMD, item 8: hand-written
# streams are sensitive to shifts of 4 mod 8 bytes): LOOP_SHIFT 4-byte s_nop 0 between the loop's
# 64-B alignment and its label (run once, on entry)
LOOP_SHIFT = 0
PERSIST = False
S_L, S_G, S_QPF = 99, 100, 101      # logical block, grid size, "next Q prefetched" flag
S_NQD = 4                           # next block's Q descriptor s[4:7] (1-D grid: s3, s4 unused)
S_NQB = 3                           # next block's q-block index
V_QN = 168                          # next Q fragments: v168.. (16 per block, A_Q layout)
V_QNOFF = 200                       # next Q lane offsets (4 per block)
V_TID = 208                         # workitem id kept across blocks
NVGPR_PERSIST = 212
S_NXD = {'K': (88, 92), 'V': (76, 4)}   # next block's K / V descriptor sets (even, odd tiles), tail only
S_TAIL = 7                           # tile index where the tail starts (nt - 4), or -1


def tail_blocks(g, rescue):
    """Persistent form, block tiles nt-4 .. nt-1 (loop positions 0..3, nt % 4 == 0): the main loop's
    and the last tile's code with the DMAs redirected to the next block's K0..K3 / V0..V2 (ring slots
    0..3, as its prologue would have loaded them), then .Lseam with s101 = 2."""
    b = [label('.Ltail')] + tail_desc()
    for t in range(3):
        b += g.phase1(t, rescue=rescue, kv_next=True) + g.phase2(t, rescue=rescue, kv_next=True)
        b += [raw(f's_waitcnt vmcnt({tile_vmcnt()})'), raw('s_barrier'), S(f's_add_u32 s{S_J}, s{S_J}, 1')]
    b += pstamp(PS_V + 6) + nvrel_insts()
    b += g.phase1(3, masked=True, last=True, rescue=rescue, kv_next=True)
    b += g.phase2(3, masked=True, last=True, rescue=rescue, kv_next=True)
    b += [mark()] + place(g.pv_sum('B', 3)[0], g.epilogue('A'))
    b += [mark()] + g.epilogue('B')
    b += [S('s_mov_b32 s101, 2'), raw('s_branch .Lseam')]
    return b


def set_prescale(on):
    """PRESCALE on/off (D = 64, 4 waves): the seed registers raise the VGPR count."""
    global PRESCALE, NVGPR
    if on:
        assert D in (32, 64) and NWAVES == 4 and ORDET
        NVGPR = max(NVGPR, V_SEED['B'] + 16)
    PRESCALE = on


def product_prescale(dtype, hd, waves, persist):
    """The shipped setting (build.py, tests): no form is pre-scaled since round 5. PRESCALE scores
    carry the rounding of Q c to the input type (|error| <= 2^-9 c sum_d |q_d k_d| for bf16, 2^-11
    for fp16); on a ragged batch with 1..5-key sequences and at softmax_scale 1.0 it broke the LSE
    tolerance (up to 16x) and the reference's 2x rule on dV (1.5x bf16, 1.75x fp16) where the
    fp32-exact forms pass (tools/r05/prescale_diag.py). It stays a generator switch
    (--prescale 1) for A/B only."""
    return hd == 64 and waves == 4 and (persist or dtype == 'f16') and PRESCALE_PRODUCT.get(dtype, False)


PRESCALE_PRODUCT = {'bf16': False, 'f16': False}


def set_persist(on):
    """Persistent form on/off (D = 64, 4 waves): 8 more kernel-argument bytes (grid size at 168),
    registers up to V_TID."""
    global PERSIST, KARG_BYTES, NVGPR, V_TID, PERSIST_Q, N_STORES, V_MCB
    if on:
        assert NWAVES == 4
        if MC_BANKS:
            # the m*c copies move out of the next-Q registers (v168..) to v212.. (PRESCALE's seeds)
            assert not PRESCALE and D <= 64
            V_MCB = {'A': 212, 'B': 216}
        # D = 128: Q, row sums and the indicator fill the VGPRs (no room for the next Q): K/V tail
        # only, the workitem id in the last free VGPR
        PERSIST_Q = D <= 64
        V_TID = 208 if PERSIST_Q else 251
        NVGPR = max(NVGPR, NVGPR_PERSIST if PERSIST_Q else V_TID + 1)
        N_STORES = len(BLOCKS) * (1 + 2 * NDT)
        KARG_BYTES = 176
    else:
        KARG_BYTES = 168
    PERSIST = on


def prologue_persist(g):
    """Blocks of the persistent prologue: (pro_a, pb1, qcopy, qload, pb2)."""
    sc = split_sections(prologue_sections(g))
    ps_ptr = [raw(f's_load_dwordx2 s[96:97], s[0:1], {KARG_BYTES - 8:#x}'), raw('s_waitcnt lgkmcnt(0)'),
              raw(f'v_mov_b32 v{PS_V}, s96'), raw(f'v_mov_b32 v{PS_V + 1}, s97')] if 'pstamps' in PROBE else []
    pro_a = sc['args'] + ps_ptr + [Inst('s_load_dword s100, s[0:1], 0xa8', 'smem', 2, wr=['s100']),
                          raw('s_waitcnt lgkmcnt(0)'),
                          S('s_mov_b32 s99, s2'), S('s_mov_b32 s101, 0'), S('s_mov_b32 s98, 0'),
                          V(f'v_mov_b32 v{V_TID}, v0', V_TID, [0])]
    pro_a += sc['wave'] + sc['lanes'] + sc['lanes_lds'] + sc['lanes2']
    # next block (clamped to the last one: its decode stays in range) -> Q descriptor s[4:7], q-block s3
    nxt = [S('s_add_u32 s80, s99, s100'), S('s_sub_u32 s81, s71, 1'), S('s_min_u32 s80, s80, s81')]
    nxt += sc['decode_map'] + [raw('s_waitcnt lgkmcnt(0)')]
    nxt += [S('s_sub_u32 s77, s77, s76'), S(f's_mov_b32 s{S_NQB}, s87'),
            S('s_mov_b32 s0, s78'), S('s_sub_u32 s1, s79, s78'), S('s_mov_b32 s2, s89')]
    nxt += make_desc(S_NQD, 40, 76, 62, 54, 55, 77)
    lanes_t = [V(f'v_and_b32 v16, 31, v{V_TID}', 16, [V_TID]), V(f'v_bfe_u32 v17, v{V_TID}, 5, 1', 17, [V_TID]),
               V('v_mov_b32 v31, 0x80000000', 31, []), V('v_mov_b32 v32, 0', 32, [])]
    dec2 = [S('s_mov_b32 s80, s99')] + [copy.copy(x) for x in sc['decode_map']] + [raw('s_waitcnt lgkmcnt(0)')]
    if 'dec3' in PROBE:     # timing probe: the current block's decode twice (the price of one decode)
        dec2 = dec2 + [S('s_mov_b32 s80, s99')] + [copy.copy(x) for x in sc['decode_map']] + [raw('s_waitcnt lgkmcnt(0)')]
    if carry_decode():
        # the block's sequence bounds and (b, h, q-block) come from the previous decode of this block
        # (the previous block's `nxt`, or for a workgroup's first block pro_a, or the .Lend path): no
        # second decode with its cu_seqlens loads per block; `nxt` runs after the row offsets
        restore = [S('s_mov_b32 s76, s84'), S('s_add_u32 s77, s84, s85'), S('s_mov_b32 s78, s0'),
                   S('s_add_u32 s79, s0, s1'), S(f's_mov_b32 s87, s{S_NQB}'), S('s_mov_b32 s88, s86'),
                   S('s_mov_b32 s89, s2')]
        if 'dec3' in PROBE:     # timing probe: one more decode of this block (the price of a decode)
            restore = [S('s_mov_b32 s80, s99')] + [copy.copy(x) for x in sc['decode_map']] + \
                [raw('s_waitcnt lgkmcnt(0)')] + restore
        pro_a += [S('s_mov_b32 s80, s99')] + [copy.copy(x) for x in sc['decode_map']] + \
            [raw('s_waitcnt lgkmcnt(0)')] + carry_save()
        if DMA_FIRST:
            # the block's first DMAs go out before the next block's decode (pb2): its cu_seqlens
            # round trip runs under their latency. The decode's temporaries include the DMA offsets
            # s80..s83, which a VGPR lane stash keeps across it.
            pb1 = [label('.Lblock')] + pstamp(PS_V + 2) + restore + sc['state'] + sc['state2'] + lanes_t + \
                sc['rows'] + sc['soffinit'] + pstamp(PS_V + 4, 'pstA') + \
                ([S('s_cmp_eq_u32 s101, 0'), raw('s_cbranch_scc1 .Lqload')] if PERSIST_Q else [])
            assert V_TID < V_STASH < NVGPR_PERSIST <= NVGPR, 'V_STASH: a spare VGPR of the persistent map'
            stash = [Inst(f'v_writelane_b32 v{V_STASH}, s{80 + i}, {i}', 'valu', rd=[f's{80 + i}'], wr=[f'v{V_STASH}'])
                     for i in range(4)]
            unstash = [Inst(f'v_readlane_b32 s{80 + i}, v{V_STASH}, {i}', 'rfl', rd=[f'v{V_STASH}'], wr=[f's{80 + i}'])
                       for i in range(4)]
            nxt_late = stash + nxt + carry_save(after_nxt=True) + unstash
        else:
            pb1 = [label('.Lblock')] + pstamp(PS_V + 2) + restore + sc['state'] + sc['state2'] + lanes_t + \
                sc['rows'] + nxt + carry_save(after_nxt=True) + sc['soffinit'] + pstamp(PS_V + 4, 'pstA') + \
                ([S('s_cmp_eq_u32 s101, 0'), raw('s_cbranch_scc1 .Lqload')] if PERSIST_Q else [])
    nxt_late = nxt_late if carry_decode() and DMA_FIRST else []
    if not carry_decode():
        pb1 = [label('.Lblock')] + pstamp(PS_V + 2) + nxt + dec2 + \
            sc['state'] + sc['soffinit'] + sc['state2'] + lanes_t + \
            sc['rows'] + pstamp(PS_V + 4, 'pstA') + ([S('s_cmp_eq_u32 s101, 0'), raw('s_cbranch_scc1 .Lqload')] if PERSIST_Q else [])
    qcopy = [Inst(f'v_accvgpr_write_b32 a{A_Q[X] + r}, v{V_QN + 16 * xi + r}', 'accw',
                  rd=[f'v{V_QN + 16 * xi + r}'], wr=[f'a{A_Q[X] + r}'])
             for xi, X in enumerate(BLOCKS) for r in range(16)] + [raw('s_branch .Lqdone')]
    qcopy_late = []
    if PRESCALE:
        # the prefetched Q is scaled on its way into the AGPRs (no AGPR pass at .Lqdone), after this
        # block's first DMAs are issued: its ~800 cycles run under their latency (QCOPY_LATE)
        qc = q_prescale(g, src=[(V_QN + 16 * xi + r, A_Q[X] + r) for xi, X in enumerate(BLOCKS)
                                for r in range(16)])
        if QCOPY_LATE:
            qcopy, qcopy_late = [raw('s_branch .Lqdone')], qc
        else:
            qcopy = qc + [raw('s_branch .Lqdone')]
    if not PERSIST_Q:
        qcopy = []
    qload = [label('.Lqload')] + sc['qload']
    # next Q lane offsets (the 'rows' section's Q part with the next q-block's row base), then its loads
    pf = [S(f's_lshl_b32 s93, s{S_WAVE}, 6'), S(f's_lshl_b32 s90, s{S_NQB}, 8'), S('s_add_u32 s93, s93, s90')]
    for xi, (X, xo) in enumerate((('A', 0), ('B', 32)) if PERSIST_Q else ()):
        pf += [V('v_add_u32 v39, s93, v16', 39, [16])] + ([V(f'v_add_u32 v39, {xo}, v39', 39, [39])] if xo else [])
        pf += [V('v_mul_lo_u32 v38, v39, s62', 38, [39])]     # row base: one multiply per block
        for ks in range(NKS):
            o = V_QNOFF + 4 * xi + ks
            pf += [V(f'v_add_u32 v40, {2 * ks}, v17', 40, [17]), V('v_lshlrev_b32 v41, 3, v40', 41, [40]),
                   V('v_cmp_gt_u32 vcc, s74, v41', 'vcc', [41]),
                   V('v_lshl_add_u32 v42, v40, 4, v38', 42, [40, 38]),
                   Inst(f'v_cndmask_b32 v{o}, v31, v42, vcc', 'valu', rd=['v31', 'v42', 'vcc'], wr=[f'v{o}'])]
    for xi, X in enumerate(BLOCKS if PERSIST_Q else ''):
        for ks in range(NKS):
            q, o = V_QN + 16 * xi + 4 * ks, V_QNOFF + 4 * xi + ks
            pf.append(Inst(f'buffer_load_dwordx4 {vs(q, 4)}, v{o}, s[{S_NQD}:{S_NQD + 3}], 0 offen', 'vload', 8,
                           rd=[f'v{o}'], wr=rv(q, 4)))
    pf.append(S('s_mov_b32 s101, 1'))
    # tail start (PERSIST_KV): nt - 4 when nt % 4 == 0 and a next block exists, else never (-1)
    pf += [S(f's_sub_u32 s{S_TAIL}, s{S_NT}, 4'), S(f's_and_b32 s96, s{S_NT}, 3'), S('s_cmp_lg_u32 s96, 0'),
           S(f's_cselect_b32 s{S_TAIL}, -1, s{S_TAIL}'), S(f's_cmp_lt_u32 s{S_NT}, 4'),
           S(f's_cselect_b32 s{S_TAIL}, -1, s{S_TAIL}'), S(f's_add_u32 s96, s{S_L}, s{S_G}'), S('s_cmp_ge_u32 s96, s71'),
           S(f's_cselect_b32 s{S_TAIL}, -1, s{S_TAIL}')]
    if not PERSIST_KV:
        pf.append(S(f's_mov_b32 s{S_TAIL}, -1'))
    nq = len(BLOCKS) * NKS if PERSIST_Q else 0

    def start_with_wait(n):
        st = [copy.copy(x) for x in sc['start']]
        i = next(k for k, x in enumerate(st) if x.txt.startswith('s_waitcnt vmcnt('))
        # 'nostartwait' timing probe: no wait for the block's first K/V tiles (wrong results, the
        # price of their latency at the block start)
        st[i] = raw(f's_waitcnt vmcnt({63 if "nostartwait" in PROBE else n})')
        return st
    # the first wait waits for Q, K0, K1, V0: younger are K2 V1 K3 V2 (8 pieces) and the next Q's loads
    qs = ([S('s_cmp_lg_u32 s101, 0'), raw('s_cbranch_scc1 .Lqsdone')] + sc['qscale'] + [label('.Lqsdone')]
          if PRESCALE else [])
    qcb = qfb = None
    if qcopy_late:
        # later blocks: the prefetched Q, scaled (qcb); the first block, s101 == 0: Q~ in place (qfb).
        # Separate blocks, so that the hazard pass walks each on its own path (build: pb2 parts)
        qs = [S('s_cmp_eq_u32 s101, 0'), raw('s_cbranch_scc1 .Lqfirst')]
        qcb = qcopy_late + [raw('s_branch .Lqsdone')]
        qfb = [label('.Lqfirst')] + sc['qscale']
    # 'pstB' probe: the loop-start stamp at .Lqdone, which the first block (after its Q loads) and every
    # later block (after the next-Q copy) pass. (Round 4 stamped inside the later blocks' copy only, so
    # the first block of every workgroup never wrote it: the negative round-0 prologues of
    # profiles/r04_pstamps/pstamps_r04f/h.)
    pb2 = [label('.Lqdone')] + pstamp(PS_V + 4, 'pstB') + [S('s_cmp_eq_u32 s101, 2'), raw('s_cbranch_scc1 .Lkvpf')] + \
        sc['dma'] + nxt_late + qs + pf + \
        sc['zero'] + start_with_wait(start_pieces() + nq)
    if qcb is not None:
        # pb2 as [head up to the branch, the copy, the first-block scale, the rest from .Lqsdone]
        i = len(pb2) - len(pf) - len(sc['zero']) - len(sc['start'])
        pb2 = [pb2[:i], qcb, qfb, [label('.Lqsdone')] + pb2[i:]]
    else:
        pb2 = [pb2]
    # K0..K3 / V0..V2 came from the previous block's tail: the descriptor sets only walk as the
    # prologue's DMAs would have; younger than K0 K1 V0 are the tail's last 8 pieces, this
    # block's 2 x 5 O / LSE stores per wave and the next Q's loads
    walk = g._dma('K', 2, walk_only=True) + g._dma('K', 3, walk_only=True) + g._dma('V', 2, walk_only=True)
    pb2k = [label('.Lkvpf')] + walk + [copy.copy(x) for x in pf] + [copy.copy(x) for x in sc['zero']] + \
        start_with_wait(4 * NP + N_STORES + nq) + [raw('s_branch .Lloop')]
    return pro_a, pb1, qcopy, qload, pb2, pb2k


N_STORES = 10         # LSE + O stores per wave of the epilogue (D = 64: 2 x (1 + 4); set_persist)
CARRY_DECODE = True   # persistent form: a block's decode carried from the previous block's next-block decode
DMA_FIRST = True      # persistent carry form: the block's first DMAs before the next block's decode
V_STASH = 209         # DMA_FIRST: lanes 0..3 keep the SGPR DMA offsets s80..s83 across the decode


def carry_decode():
    """CARRY_DECODE applies to the persistent forms without the next-block K/V tail (D = 64): the
    tail's descriptor code (tail_desc) uses s3 as a temporary."""
    return CARRY_DECODE and PERSIST and not PERSIST_KV and soff_walk()


def carry_save(after_nxt=False):
    """Carry registers of the next block's decode: s0 k start, s1 seqlen_k, s2 head, s3 (S_NQB) q-block,
    s84 q start, s85 seqlen_q, s86 batch (free from the block's decode to the next block's restore:
    the loop keeps only its DMA offsets in s80..s83). `nxt` already leaves s0..s3 and s77 = seqlen_q."""
    out = [S('s_mov_b32 s84, s76'), S('s_mov_b32 s86, s88')]
    if after_nxt:
        return out + [S('s_mov_b32 s85, s77')]
    return out + [S('s_sub_u32 s85, s77, s76'), S(f's_mov_b32 s{S_NQB}, s87'), S('s_mov_b32 s0, s78'),
                  S('s_sub_u32 s1, s79, s78'), S('s_mov_b32 s2, s89')]
PERSIST_Q = True      # persistent form: next-block Q prefetch (D = 64 only)
QCOPY_LATE = True     # persistent PRESCALE: the next-Q copy + scale after the block's first DMAs
BAR2 = False          # main loop: one barrier per two tiles (needs R >= 6, DIST >= 3, even unroll)
PERSIST_KV = True     # persistent form: the tail streams the next block's K0..K3 / V0..V2


def tail_desc():
    """The next block's K / V descriptor sets (tile 0 and tile 1 of its sequence) from s0 = its first
    key row, s1 = seqlen_k, s2 = head (make_desc + the odd-tile sets of the prologue); temps s3, s29,
    s31 (unused by the loop)."""
    out = []
    for kind, ptr, rs, hs in (('K', 42, 63, 56), ('V', 44, 64, 58)):
        d0, d1 = S_NXD[kind]
        out += [S(f's_mul_i32 s3, s0, s{rs}'), S(f's_mul_hi_u32 s29, s0, s{rs}'),
                S(f's_add_u32 s{d0}, s{ptr}, s3'), S(f's_addc_u32 s{d0 + 1}, s{ptr + 1}, s29'),
                S(f's_mul_i32 s3, s2, s{hs}'), S(f's_mul_hi_u32 s29, s2, s{hs}'), S(f's_mul_i32 s31, s2, s{hs + 1}'),
                S('s_add_u32 s29, s29, s31'),
                S(f's_add_u32 s{d0}, s{d0}, s3'), S(f's_addc_u32 s{d0 + 1}, s{d0 + 1}, s29'),
                S(f's_mul_i32 s{d0 + 2}, s1, s{rs}'), S(f's_mov_b32 s{d0 + 3}, 0x00020000'),
                S(f's_lshl_b32 s3, s{rs}, 6'),
                S(f's_add_u32 s{d1}, s{d0}, s3'), S(f's_addc_u32 s{d1 + 1}, s{d0 + 1}, 0'),
                S(f's_sub_u32 s{d1 + 2}, s{d0 + 2}, s3'), S(f's_cselect_b32 s{d1 + 2}, 0, s{d1 + 2}'),
                S(f's_mov_b32 s{d1 + 3}, s{d0 + 3}')]
    return out


def dump_block(regs):
    """Debug only (gen_fwd.py --dump): workgroup (0,0,0) stores the listed registers of every
    wave into the O buffer as raw dwords [wave][reg][lane] (64-bit global stores), then ends."""
    n = len(regs)
    A0, A1, T = 140, 141, 142      # address pair and data temp (V_OOFF of block B: unused here)
    b = [raw('s_waitcnt vmcnt(0) lgkmcnt(0)'), raw('s_nop 15'), raw('s_nop 15'),
         S('s_or_b32 s96, s2, s3'), S('s_or_b32 s96, s96, s4'), S('s_cmp_eq_u32 s96, 0'),
         raw('s_cbranch_scc1 .Ldump_go'), raw('s_endpgm'), label('.Ldump_go'),
         S(f's_mul_i32 s96, s{S_WAVE}, {n * 256}'), raw('s_nop 3'),
         V(f'v_lshlrev_b32 v{A0}, 2, v{V_LANE}', A0, [V_LANE]),
         V(f'v_add_u32 v{A0}, s96, v{A0}', A0, [A0]),
         V(f'v_mov_b32 v{A1}, s47', A1, []),
         Inst(f'v_add_co_u32 v{A0}, vcc, s46, v{A0}', 'valu', rd=[f'v{A0}'], wr=[f'v{A0}', 'vcc']),
         Inst(f'v_addc_co_u32 v{A1}, vcc, 0, v{A1}, vcc', 'valu', rd=[f'v{A1}', 'vcc'], wr=[f'v{A1}', 'vcc']),
         raw('s_nop 3')]
    for i, r in enumerate(regs):
        src = r
        if r.startswith('a'):
            b.append(Inst(f'v_accvgpr_read_b32 v{T}, {r}', 'accr', rd=[r], wr=[f'v{T}']))
            b.append(raw('s_nop 3'))
            src = f'v{T}'
        b.append(raw(f'global_store_dword v[{A0}:{A1}], {src}, off offset:{(i % 8) * 256}'))
        b.append(raw('s_waitcnt vmcnt(0)'))
        b.append(raw('s_nop 3'))
        if i % 8 == 7:
            b.append(Inst(f'v_add_co_u32 v{A0}, vcc, 0x800, v{A0}', 'valu', rd=[f'v{A0}'], wr=[f'v{A0}', 'vcc']))
            b.append(Inst(f'v_addc_co_u32 v{A1}, vcc, 0, v{A1}, vcc', 'valu', rd=[f'v{A1}', 'vcc'], wr=[f'v{A1}', 'vcc']))
            b.append(raw('s_nop 3'))
    b += [raw('s_waitcnt vmcnt(0)'), raw('s_endpgm')]
    return b


DUMP = None   # (point, [registers]) set by --dump
LOOP_BLOCKS = set()   # ids of the main-loop and masked-loop tile blocks (the nolgkm / novm probes' scope)

# 'stamps' probe (tools/asm_wg_timeline.py, D = 64 only): s_memrealtime (100 MHz) at kernel entry
# (v168:169), after the prologue's first barrier (v180:181), at the last tile's entry (v170:171)
# and after the final store drain (v172:173); HW_ID / XCC_ID, the workgroup ids s2..s4 and the
# wave index; lane 0 claims a 64-byte record with a vector atomic on the counter at the pointer
# in the 8 kernel-argument bytes after KARG_BYTES and writes the record with vector stores.
STAMP_V = 168


def stamp(lo):
    # 'stampcyc': shader-clock cycles (s_memtime) instead of the 100 MHz real-time counter
    clk = 's_memtime' if 'stampcyc' in PROBE else 's_memrealtime'
    return [raw(f'{clk} s[96:97]'), raw('s_waitcnt lgkmcnt(0)'),
            raw(f'v_mov_b32 v{lo}, s96'), raw(f'v_mov_b32 v{lo + 1}, s97')]


def stamp_entry():
    if 'stamps' not in PROBE:
        return []
    b = STAMP_V
    return stamp(b) + [raw('s_getreg_b32 s96, hwreg(HW_REG_HW_ID)'), raw('s_getreg_b32 s97, hwreg(HW_REG_XCC_ID)'),
                       raw(f'v_mov_b32 v{b + 6}, s96'), raw(f'v_mov_b32 v{b + 7}, s97'),
                       raw(f'v_mov_b32 v{b + 8}, s2'), raw(f'v_mov_b32 v{b + 9}, s3'), raw(f'v_mov_b32 v{b + 10}, s4')]


def stamp_exit():
    if 'stamps' not in PROBE:
        return []
    b = STAMP_V
    return stamp(b + 4) + [
        raw(f's_load_dwordx2 s[98:99], s[0:1], {KARG_BYTES - 8:#x}'), raw('s_waitcnt lgkmcnt(0)'),
        raw(f'v_mov_b32 v{b + 11}, s{S_WAVE}'), raw('s_mov_b64 exec, 1'),
        raw(f'v_mov_b32 v{b + 14}, 1'), raw(f'v_mov_b32 v{b + 15}, 0'),
        raw(f'global_atomic_add v{b + 14}, v{b + 15}, v{b + 14}, s[98:99] sc0'), raw('s_waitcnt vmcnt(0)'),
        raw(f'v_lshlrev_b32 v{b + 14}, 6, v{b + 14}'), raw(f'v_add_u32 v{b + 14}, 64, v{b + 14}'), raw('s_nop 1'),
        raw(f'global_store_dwordx4 v{b + 14}, v[{b}:{b + 3}], s[98:99]'),
        raw(f'global_store_dwordx4 v{b + 14}, v[{b + 4}:{b + 7}], s[98:99] offset:16'),
        raw(f'global_store_dwordx4 v{b + 14}, v[{b + 8}:{b + 11}], s[98:99] offset:32'),
        raw(f'global_store_dwordx2 v{b + 14}, v[{b + 12}:{b + 13}], s[98:99] offset:48'),
        raw('s_waitcnt vmcnt(0)')]


# 'pstamps' probe (tools/asm_pstamps.py, persistent D = 64 form): per (block, wave) four s_memtime
# stamps -- block entry (.Lblock), loop start (after the start barrier), last-tile entry, seam --
# stored by lane 0 as a 32-byte record at [ptr + 32 (4 L + wave)]; ptr = the 8 kernel-argument bytes
# after KARG_BYTES - 8, kept in v244:245 (v244..v255 are free in the persistent form).
PS_V = 244


def pstamp(lo, at=None):
    """at: 'pstA' (after the block's decode and row offsets) / 'pstB' (after the Q copy): the
    loop-start stamp moved there by the probe of that name (prologue split)."""
    if 'pstamps' not in PROBE:
        return []
    if lo == PS_V + 4 and (at or 'start') not in PROBE and ('pstA' in PROBE or 'pstB' in PROBE):
        return []
    if at is not None and at not in PROBE:
        return []
    clk = 's_memrealtime' if 'pstrt' in PROBE else 's_memtime'    # pstrt: the global 100 MHz clock
    return [raw(f'{clk} s[96:97]'), raw('s_waitcnt lgkmcnt(0)'), raw(f'v_mov_b32 v{lo}, s96'),
            raw(f'v_mov_b32 v{lo + 1}, s97')]


def pstamp_store():
    if 'pstamps' not in PROBE:
        return []
    b = PS_V
    return pstamp(b + 8) + [
        raw(f's_lshl_b32 s96, s{S_L}, 2'), raw(f's_add_u32 s96, s96, s{S_WAVE}'), raw('s_lshl_b32 s96, s96, 5'),
        raw(f'v_add_co_u32 v{b + 10}, vcc, s96, v{b}'), raw(f'v_addc_co_u32 v{b + 11}, vcc, 0, v{b + 1}, vcc'),
        raw('s_mov_b64 s[96:97], exec'), raw('s_mov_b64 exec, 1'), raw('s_nop 1'),
        raw(f'global_store_dwordx4 v[{b + 10}:{b + 11}], v[{b + 2}:{b + 5}], off'),
        raw(f'global_store_dwordx4 v[{b + 10}:{b + 11}], v[{b + 6}:{b + 9}], off offset:16'),
        raw('s_mov_b64 exec, s[96:97]')]


def nvrel_insts():
    """Per-block key limits of a masked tile: NVREL_X = ROW1_X - 64 j."""
    return [S(f's_lshl_b32 s96, s{S_J}, 6')] + \
           [V(f'v_subrev_u32 v{V_NVREL[X]}, s96, v{V_ROW1[X]}', V_NVREL[X], [V_ROW1[X]]) for X in BLOCKS]


def tile_vmcnt():
    """vmcnt of the wait before each tile's barrier: the 4-wave form needs K(t+2), V(t+1) in LDS
    for the next tile (all but the DMAs of the last DIST - 1 tiles); the 8-wave form reads K(t+2)
    one tile earlier (all but this tile's two pieces)."""
    return 2 * NP * (DIST - 2) if NWAVES == 8 else pieces_wait()


def bar2_vmcnt():
    """BAR2 (main loop barrier after odd tiles only): the barrier after tile t publishes the data of
    tiles t+1 and t+2 (K(t+3), V(t+2) and older): the DMAs of the last DIST - 2 tiles may stay in
    flight. Slot reuse needs a ring of 6 (a fast wave may lead by up to two tiles)."""
    return min(2 * NP, 4) * (DIST - 2)


def start_pieces():
    """DMA pieces that may still be in flight at the prologue's barrier: pieces_wait(), or with
    BAR2 one tile fewer (no barrier after tile 0: tile 1's K(2), V(1) must be published here);
    DEFER_DMA: the last prologue tile is not issued yet."""
    n = pieces_wait() - (min(2 * NP, 4) if BAR2 else 0)
    return n - 2 * NP if defer_dma() else n


DEFER_DMA = True      # 4 waves, D <= 64: the prologue's last DMA tile after its barrier


def defer_dma():
    """DEFER_DMA applies where the prologue's barrier already waits for every earlier piece: the
    4-wave D <= 64 forms (BAR2, ring 6, distance 3: start_pieces() is exactly that tile's pieces)."""
    return DEFER_DMA and NWAVES == 4 and D <= 64 and BAR2 and pieces_wait() - min(2 * NP, 4) == 2 * NP


def pieces_wait():
    """4-wave form: DMA pieces that may stay in flight when the next tile starts: the last DIST - 1
    tiles' (2 NP each; D = 32 has NP = 1 and needs exactly this). At D = 128 (NP = 4) the stricter
    4 (DIST - 1) stays: measured even against 2 NP (DIST - 1) (tools/wait_ab.sh)."""
    return min(2 * NP, 4) * (DIST - 1)


def tile_phases(g, t, **kw):
    if NWAVES == 8:
        return g.phase_w8(t, **kw)
    return g.phase1(t, **kw) + g.phase2(t, **kw)


def stagger_split(lst):
    """STAGGER (8 waves): a phase's instruction list cut after its first half of MFMAs, and the
    count of LDS-DMA pieces in the first part (the group-1 barrier's vmcnt)."""
    mf = [i for i, x in enumerate(lst) if x.kind == 'mfma']
    k = max(1, min(len(mf) - 1, round(len(mf) * STAGGER_FRAC)))
    cut = mf[k - 1] + 1
    if PINGPONG:
        # between the matrix and the vector segment: after the last MFMA and the fillers placed
        # in its gap that are not softmax (DMA, K reads, SALU)
        cut = mf[-1] + 1
        while cut < len(lst) and lst[cut].kind in ('dma', 'm0', 'salu', 'ds') and lst[cut].txt.startswith(
                ('buffer_load', 's_add_u32 m0', 's_add', 's_sub', 's_addc', 's_cselect', 'ds_read_b128')):
            cut += 1
    return lst[:cut], lst[cut:], sum(1 for x in lst[:cut] if x.kind == 'dma')


def tile_body(g, t, sfx, **kw):
    """One tile's phases and its barrier. Group 0 (sfx ''): phases, wait, barrier. Group 1 of the
    STAGGER form (sfx '_g1', waves 4-7): the barrier in the middle of the phase, so these waves run
    half a tile behind their SIMD partners (MI355X_MICROARCH.md "Two waves per SIMD" item 9). At the
    group-1 barrier of tile t every DMA piece of tiles < t has landed (vmcnt = the pieces issued
    before it in this phase), as at the group-0 barrier; the 6-slot ring keeps every slot a DMA
    rewrites at least two tiles behind the half-tile-late reads (configure_stagger)."""
    ph = tile_phases(g, t, **kw)
    if not sfx:
        return ph + [raw(f's_waitcnt vmcnt({tile_vmcnt()})'), raw('s_barrier')]
    a, b, n = stagger_split(ph)
    return a + [raw(f's_waitcnt vmcnt({n})'), raw('s_barrier')] + b


def masked_tile(g, t, rescue, sfx=''):
    """Loop position t of the masked loop: tiles from S_MSTART (the causal diagonal band) up to
    the last one, which exits to .Llast{t}."""
    blk = [label(f'.Lmask{sfx}{t}'), S(f's_cmp_eq_u32 s{S_J}, s{S_LAST}'), raw(f's_cbranch_scc1 .Llast{sfx}{t}')]
    blk += nvrel_insts()
    blk += tile_body(g, t, sfx, masked=True, rescue=rescue)
    blk += [S(f's_add_u32 s{S_J}, s{S_J}, 1')]
    if t == U - 1:
        blk.append(raw(f's_branch .Lmask{sfx}0'))
    return blk


def last_tile(g, t, rescue, masked=True, sfx=''):
    """Tile t = nt - 1 (position t of the unrolled loop): masked softmax of both blocks, no
    next-tile reads or DMA, then P.V of block B and the two epilogues. LAST_UNMASKED: the masked
    form first tests whether any lane's row sees fewer than all 64 keys of the tile and otherwise
    branches to the unmasked copy (masked=False, .LlastU{t}: key counts that are multiples of 64
    skip 128 compare/select pairs per block)."""
    if not masked:
        b = [label(f'.LlastU{sfx}{t}')]
    else:
        b = [label(f'.Llast{sfx}{t}')] + (stamp(STAMP_V + 2) if 'stamps' in PROBE else []) + pstamp(PS_V + 6) + nvrel_insts()
        if LAST_UNMASKED:
            # masked key offsets reach 59 (32 st + 3 + 24): a lane needs the mask iff NVREL < 60
            # (no temporaries: the 8-wave form keeps the previous tile's P in V_TMP)
            nv = sorted({V_NVREL[X] for X in BLOCKS})
            for i, r in enumerate(nv):
                b.append(V(f'v_cmp_gt_i32 vcc, 60, v{r}', 'vcc', [r]))
                last = i == len(nv) - 1
                b.append(Inst(f's_cbranch_vccz .LlastU{sfx}{t}' if last else f's_cbranch_vccnz .LlastM{sfx}{t}', 'br', 4,
                              rd=['vcc']))
            if len(nv) > 1:
                b.append(label(f'.LlastM{sfx}{t}'))
    b += tile_phases(g, t, masked=masked, last=True, rescue=rescue)
    if NWAVES == 8:
        b += [mark()] + place(g.pv_sum(par(t), t)[0], [])
        b += [mark()] + g.epilogue('A')
    else:
        b += [mark()] + place(g.pv_sum('B', t)[0], g.epilogue('A'))
        b += [mark()] + g.epilogue('B')
    if PERSIST:
        b.append(raw('s_branch .Lseam'))
    else:
        b += [raw('s_waitcnt vmcnt(0)')] + stamp_exit() + [raw('s_endpgm')]
    return b


def build(g):
    rescue = []
    if PERSIST:
        pro_a, pb1, qcopy, qload, pb2, pb2k = prologue_persist(g)
        pro = pro_a + pb1 + qload + sum(pb2, [])       # (only for the DUMP hook below)
    else:
        pro = stamp_entry() + prologue(g)
    if DUMP and DUMP[0] == 'pro':
        pro += dump_block(DUMP[1])
    tiles = []
    if STAGGER:
        assert NWAVES == 8 and not PERSIST
        # waves 4-7 branch to their own copy of the loops (the barrier mid-tile: tile_body)
        pro += [S(f's_cmp_ge_u32 s{S_WAVE}, 4'), raw('s_cbranch_scc1 .Lloop_g1')]
    for t in range(U):
        blk = []
        if t == 0:
            blk.append(raw('.p2align 6'))
            blk += [raw('s_nop 0')] * LOOP_SHIFT      # placement probe: the loop stream 4 B per nop later
            blk.append(label('.Lloop'))
        if PERSIST and PERSIST_KV and t == 0:
            blk += [S(f's_cmp_eq_u32 s{S_J}, s{S_TAIL}'), raw('s_cbranch_scc1 .Ltail')]
        blk += [S(f's_cmp_ge_u32 s{S_J}, s{S_MSTART}'), raw(f's_cbranch_scc1 .Lmask{t}')]
        if NWAVES == 8:
            blk += tile_body(g, t, '', rescue=rescue)
            blk += [S(f's_add_u32 s{S_J}, s{S_J}, 1')]
            if t == U - 1:
                blk.append(raw('s_branch .Lloop'))
            tiles.append(blk)
            continue
        else:
            blk += g.phase1(t, rescue=rescue)
            if DUMP and DUMP[0] == 'p1' and t == 0:
                blk += dump_block(DUMP[1])
            blk += g.phase2(t, rescue=rescue)
            if DUMP and DUMP[0] == 'p2' and t == 0:
                blk += dump_block(DUMP[1])
        if 'nobar' not in PROBE and (not BAR2 or t % 2 == 1):
            blk += [raw(f's_waitcnt vmcnt({bar2_vmcnt() if BAR2 else tile_vmcnt()})'), raw('s_barrier')]
        blk += [S(f's_add_u32 s{S_J}, s{S_J}, 1')]
        if t == U - 1:
            blk.append(raw('s_branch .Lloop'))
        tiles.append(blk)
    masks = [masked_tile(g, t, rescue) for t in range(U)]
    LOOP_BLOCKS.clear()
    LOOP_BLOCKS.update(id(b) for b in tiles + masks)
    lasts = [last_tile(g, t, rescue) for t in range(U)]
    lastsu = [last_tile(g, t, rescue, masked=False) for t in range(U)] if LAST_UNMASKED else []
    tiles1, masks1, lasts1, lastsu1 = [], [], [], []
    if STAGGER:
        for t in range(U):
            blk = [raw('.p2align 6')] + [raw('s_nop 0')] * LOOP_SHIFT + [label('.Lloop_g1')] if t == 0 else []
            blk += [S(f's_cmp_ge_u32 s{S_J}, s{S_MSTART}'), raw(f's_cbranch_scc1 .Lmask_g1{t}')]
            blk += tile_body(g, t, '_g1', rescue=rescue) + [S(f's_add_u32 s{S_J}, s{S_J}, 1')]
            if t == U - 1:
                blk.append(raw('s_branch .Lloop_g1'))
            tiles1.append(blk)
        masks1 = [masked_tile(g, t, rescue, sfx='_g1') for t in range(U)]
        lasts1 = [last_tile(g, t, rescue, sfx='_g1') for t in range(U)]
        lastsu1 = [last_tile(g, t, rescue, masked=False, sfx='_g1') for t in range(U)] if LAST_UNMASKED else []

    def last_paths(t, lasts=lasts, lastsu=lastsu):
        """The last tile at loop position t: the masked form, and (LAST_UNMASKED) its test then
        the unmasked copy."""
        out = [lambda: refs(lasts[t])]
        if LAST_UNMASKED:
            ib = next(i for i, x in enumerate(lasts[t]) if x.txt.startswith('s_cbranch_vccz'))
            out.append(lambda: [(lasts[t], k) for k in range(ib + 1)] + refs(lastsu[t]))
        return out
    empty = [label('.Lempty')] + sum(([mark()] + g.epilogue(X) for X in BLOCKS), []) + \
            ([raw('s_waitcnt vmcnt(0)'), raw('s_branch .Lseam')] if PERSIST else [raw('s_waitcnt vmcnt(0)'), raw('s_endpgm')])
    # (PERSIST: an empty key set may follow a tail that prefetched its (zero-length) K/V: drain before
    # the next block's DMAs reuse the ring. The loop's own past-the-end DMAs of a block without a tail
    # read nothing (num_records 0: zero-filled, no memory access) and were issued a tile or more
    # before the seam; every GPU form test mixes both kinds of seams.)
    end = [label('.Lend'), raw('s_endpgm')]
    if PERSIST:
        # .Lend (q-block past its sequence: nothing prefetched) and .Lseam (after a block): next block
        lend_dec = []
        if carry_decode():
            # a q-block past its sequence skipped `nxt`: decode the next block here
            lend_dec = [S('s_add_u32 s80, s99, s100'), S('s_sub_u32 s81, s71, 1'), S('s_min_u32 s80, s80, s81')] + \
                [x for x in split_sections(prologue_sections(g))['decode_map']] + [raw('s_waitcnt lgkmcnt(0)')] + \
                carry_save()
        end = [label('.Lend'), S(f's_mov_b32 s{S_QPF}, 0')] + lend_dec + [label('.Lseam')] + pstamp_store() + [
               S(f's_add_u32 s{S_L}, s{S_L}, s{S_G}'), S(f's_cmp_ge_u32 s{S_L}, s71'), raw('s_cbranch_scc1 .Ldone'),
               raw('s_barrier'), raw('s_branch .Lblock')]
        done = [label('.Ldone'), raw('s_waitcnt vmcnt(0)'), raw('s_endpgm')]
        # a block past its sequence: the previous tail's DMAs must land before this slot reuse
        end.insert(1, raw('s_waitcnt vmcnt(0)'))
        tail = tail_blocks(g, rescue) if PERSIST_KV else []
    # control-flow paths for the hazard pass
    paths = []
    def seq(blks):
        return sum((refs(b) for b in blks), [])
    if PERSIST:
        # pb2 parts: one block, or [head, next-Q copy, first-block Q scale, rest] (QCOPY_LATE)
        p2_first = lambda: sum((refs(b) for b in (pb2[:1] + pb2[2:] if len(pb2) > 1 else pb2)), [])
        p2_next = lambda: sum((refs(b) for b in (pb2[:2] + pb2[3:] if len(pb2) > 1 else pb2)), [])
        first = lambda: refs(pro_a) + refs(pb1) + refs(qload) + p2_first()
        qsel = qcopy if PERSIST_Q else qload
        # a finished block reaches the next one at .Lseam (the .Lend entry above it drains vmcnt, .Lseam does not)
        iseam = next(i for i, x in enumerate(end) if x.kind == 'label' and x.txt.startswith('.Lseam'))
        seam = lambda: [(end, k) for k in range(iseam, len(end))]
        nxt = lambda: seam() + refs(pb1) + refs(qsel) + p2_next()
        lend = next(i for i, x in enumerate(pb1) if x.txt.endswith('.Lend'))
        paths.append(lambda: first() + seq(tiles) + seq(tiles))
        for t in range(U):
            paths.append(lambda t=t: first() + seq(tiles) + seq(tiles[:t]) + seq(masks[t:]) + seq(masks))
            for lp in last_paths(t):
                paths.append(lambda t=t, lp=lp: first() + seq(tiles) + seq(masks) + seq(masks[:t]) + lp() + nxt() +
                             seq(tiles))
            # the masked loop (causal band / last tile) entered after only t main tiles of the block's first
            # round, and its last tile reached directly (blocks of fewer than U tiles)
            paths.append(lambda t=t: first() + seq(tiles[:t]) + seq(masks[t:]) + seq(masks))
            for lp in last_paths(t):
                paths.append(lambda t=t, lp=lp: first() + seq(tiles[:t]) + [(masks[t], k) for k in range(3)] + lp() +
                             nxt() + seq(tiles))
        paths.append(lambda: first() + refs(empty) + nxt() + seq(tiles))
        paths.append(lambda: refs(pro_a) + [(pb1, k) for k in range(lend + 1)] + refs(end) + refs(pb1) + refs(qload) +
                     p2_first() + seq(tiles))
        ikv = next(i for i, x in enumerate(pb2[0]) if x.txt.endswith('.Lkvpf'))
        nxt_from_tail = lambda: seam() + refs(pb1) + refs(qsel) + [(pb2[0], k) for k in range(ikv + 1)] + refs(pb2k)
        if PERSIST_KV:
            itail = next(i for i, x in enumerate(tiles[0]) if x.txt.endswith('.Ltail'))
            for_tail = lambda: first() + seq(tiles) + [(tiles[0], k) for k in range(itail + 1)] + refs(tail)
            paths.append(lambda: for_tail() + nxt_from_tail() + seq(tiles) + seq(tiles))
            # a block of exactly 4 tiles enters the tail at its first tile
            tail_now = lambda: first() + [(tiles[0], k) for k in range(itail + 1)] + refs(tail)
            paths.append(lambda: tail_now() + nxt_from_tail() + seq(tiles) + seq(tiles))
            paths.append(lambda: for_tail() + nxt_from_tail() + [(tiles[0], k) for k in range(itail + 1)] + refs(tail))
    else:
        paths.append(lambda: refs(pro) + seq(tiles) + seq(tiles))
        for t in range(U):
            # main loop -> masked loop entered at position t -> a full masked round
            paths.append(lambda t=t: refs(pro) + seq(tiles) + seq(tiles[:t]) + seq(masks[t:]) + seq(masks))
            # masked loop -> last tile at position t
            for lp in last_paths(t):
                paths.append(lambda t=t, lp=lp: refs(pro) + seq(tiles) + seq(masks) + seq(masks[:t]) + lp())
            # the masked loop entered after only t main tiles (causal band from tile t < U), and its last
            # tile reached directly (fewer than U tiles)
            paths.append(lambda t=t: refs(pro) + seq(tiles[:t]) + seq(masks[t:]) + seq(masks))
            for lp in last_paths(t):
                paths.append(lambda t=t, lp=lp: refs(pro) + seq(tiles[:t]) + [(masks[t], k) for k in range(3)] + lp())
        paths.append(lambda: refs(pro) + refs(empty))
        if STAGGER:
            # group 1 (waves 4-7): the same paths through its own loop copies
            for tl, ms, ls, lu in ((tiles1, masks1, lasts1, lastsu1),):
                paths.append(lambda: refs(pro) + seq(tl) + seq(tl))
                for t in range(U):
                    paths.append(lambda t=t: refs(pro) + seq(tl) + seq(tl[:t]) + seq(ms[t:]) + seq(ms))
                    for lp in last_paths(t, ls, lu):
                        paths.append(lambda t=t, lp=lp: refs(pro) + seq(tl) + seq(ms) + seq(ms[:t]) + lp())
                    paths.append(lambda t=t: refs(pro) + seq(tl[:t]) + seq(ms[t:]) + seq(ms))
                    for lp in last_paths(t, ls, lu):
                        paths.append(lambda t=t, lp=lp: refs(pro) + seq(tl[:t]) + [(ms[t], k) for k in range(3)] + lp())
    # rescale blocks entered from their branch: the 40 instructions before it, the block, the rest
    def resc_path(rb):
        ret = rb[-1].txt.split()[-1]
        for blk in tiles + masks + lasts + lastsu + tiles1 + masks1 + lasts1 + lastsu1 + \
                ([tail] if PERSIST and tail else []):
            for i, x in enumerate(blk):
                if x.kind == 'br' and x.txt.endswith(f'{ret}:'):
                    lo = max(0, i - 40)
                    return [(blk, k) for k in range(lo, i + 1)] + refs(rb) + [(blk, k) for k in range(i + 1, min(len(blk), i + 60))]
        raise RuntimeError('rescale return not found')
    for rb in rescue:
        paths.append(lambda rb=rb: resc_path(rb))
    if PERSIST:
        n = fix_paths(paths)
        return [pro_a, pb1, qcopy, qload] + pb2 + tiles + masks + lasts + lastsu + [empty, end, done, pb2k] + \
            ([tail] if tail else []) + rescue, n
    n = fix_paths(paths)
    blocks = [pro] + tiles + masks + lasts + lastsu + tiles1 + masks1 + lasts1 + lastsu1 + [empty, end] + rescue
    return blocks, n


def emit(g, blocks):
    name = g.name
    if 'nolgkm' in PROBE or 'novm' in PROBE:
        # timing probes: the counted waits of the main-loop tiles only (never the prologue's, which
        # cover the scalar loads of kernel arguments and cu_seqlens: without them the descriptors
        # are built from stale SGPRs and the kernel faults -- a persistent-form probe run of round 6
        # did exactly that when this stripped every block but the first)
        for blk in blocks:
            if id(blk) not in LOOP_BLOCKS:
                continue
            assert not any(x.kind == 'smem' for x in blk)
            blk[:] = [x for x in blk if not (x.txt.startswith('s_waitcnt') and
                                             (('nolgkm' in PROBE and 'lgkmcnt' in x.txt) or
                                              ('novm' in PROBE and 'vmcnt' in x.txt and 'lgkm' not in x.txt)))]
    lines = ['.amdgcn_target "amdgcn-amd-amdhsa--gfx950"', '.amdhsa_code_object_version 5', '.text',
             f'.globl {name}', '.p2align 8', f'.type {name},@function', f'{name}:']
    for blk in blocks:
        for x in blk:
            if x.kind == 'mark' or not x.txt:
                continue
            if x.kind == 'label' or x.txt.startswith('.p2align'):
                lines.append(x.txt)
            else:
                for ln in x.txt.split('\n'):
                    lines.append(ln if ln.endswith(':') else '\t' + ln)
    lines += ['.Lfunc_end:', f'\t.size {name}, .Lfunc_end-{name}', '',
              '.rodata', '.p2align 6', f'.amdhsa_kernel {name}',
              f'\t.amdhsa_group_segment_fixed_size {LDS_BYTES}',
              '\t.amdhsa_private_segment_fixed_size 0',
              f'\t.amdhsa_kernarg_size {KARG_BYTES}',
              '\t.amdhsa_user_sgpr_count 2',
              '\t.amdhsa_user_sgpr_kernarg_segment_ptr 1',
              '\t.amdhsa_system_sgpr_workgroup_id_x 1',
              '\t.amdhsa_system_sgpr_workgroup_id_y 1',
              '\t.amdhsa_system_sgpr_workgroup_id_z 1',
              '\t.amdhsa_system_vgpr_workitem_id 0',
              f'\t.amdhsa_next_free_vgpr {NVGPR + NAGPR}',
              f'\t.amdhsa_next_free_sgpr {NSGPR}',
              f'\t.amdhsa_accum_offset {NVGPR}',
              '\t.amdhsa_reserve_vcc 1',
              '\t.amdhsa_float_denorm_mode_32 3',
              '\t.amdhsa_float_denorm_mode_16_64 3',
              '\t.amdhsa_dx10_clamp 1',
              '\t.amdhsa_ieee_mode 0',
              '.end_amdhsa_kernel', '',
              '.amdgpu_metadata', '---', 'amdhsa.kernels:',
              f'  - .agpr_count: {NAGPR}',
              '    .args:', '      - .offset: 0', f'        .size: {KARG_BYTES}', '        .value_kind: by_value',
              f'    .group_segment_fixed_size: {LDS_BYTES}',
              '    .kernarg_segment_align: 8', f'    .kernarg_segment_size: {KARG_BYTES}',
              f'    .max_flat_workgroup_size: {64 * NWAVES}', f'    .name: {name}',
              '    .private_segment_fixed_size: 0', f'    .sgpr_count: {NSGPR + 2}',
              f'    .symbol: {name}.kd', f'    .vgpr_count: {NVGPR + NAGPR}', '    .wavefront_size: 64',
              'amdhsa.target: amdgcn-amd-amdhsa--gfx950', 'amdhsa.version:', '  - 1', '  - 2', '...',
              '.end_amdgpu_metadata', '']
    return '\n'.join(lines)


KARG_BYTES = 168


def expand_regs(spec):
    out = []
    for part in spec.split(','):
        if '-' in part:
            f = part[0]
            lo, hi = part[1:].split('-')
            hi = hi.lstrip('vas')
            out += [f'{f}{i}' for i in range(int(lo), int(hi) + 1)]
        elif part:
            out.append(part)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'f16'])
    ap.add_argument('--hd', type=int, default=64, choices=[32, 64, 96, 128], help='head-dim tile')
    ap.add_argument('--waves', type=int, default=4, choices=[4, 8], help='waves per workgroup (8: D = 64 only)')
    ap.add_argument('--prio4', type=int, default=None, help='8 waves: s_setprio 1 for waves 4-7')
    ap.add_argument('--stagger', type=int, default=0, help='8 waves: waves 4-7 half a tile behind (ring 6)')
    ap.add_argument('--fmax8', type=int, default=0, help="8 waves: tile 0's row max sets the starting shift")
    ap.add_argument('--sfrac', type=float, default=None, help='STAGGER: group-1 barrier after this fraction of the MFMAs')
    ap.add_argument('--pingpong', type=int, default=0, help='8 waves: matrix / vector segments alternating between SIMD partners')
    ap.add_argument('--lag8', default=None, help='8 waves: EXP_LAG,CVT_LAG')
    ap.add_argument('--persist', type=int, default=0, help='persistent workgroups: next-block K/V tail (and next-Q prefetch at D = 64), 4 waves')
    ap.add_argument('--out', required=True)
    ap.add_argument('--stats', action='store_true')
    ap.add_argument('--dump', default=None, help='debug: point:reg,reg,... (pro|p1|p2)')
    ap.add_argument('--probe', default='', help='timing-only variant switches, comma separated')
    ap.add_argument('--ring', type=int, default=None)
    ap.add_argument('--qlate', type=int, default=None, help='persistent: Q copy + scale after the first DMAs')
    ap.add_argument('--bar2', type=int, default=None, help='main-loop barrier after odd tiles only (with --ring 6 --dist 4)')
    ap.add_argument('--kvtail', type=int, default=None, help='persistent form: stream the next block K/V in the tail')
    ap.add_argument('--dist', type=int, default=None)
    ap.add_argument('--vp1', type=int, default=None)
    ap.add_argument('--smpipe', type=int, default=None)
    ap.add_argument('--dmap2', type=int, default=None)
    ap.add_argument('--spec', type=int, default=None)
    ap.add_argument('--ordet', type=int, default=None)
    ap.add_argument('--lag', default=None, help='EXP_LAG,CVT_LAG')
    ap.add_argument('--mcbanks', type=int, default=None)
    ap.add_argument('--kfirst', type=int, default=None, help='K(t+1) reads first in phase 1 (value: first position)')
    ap.add_argument('--prescale', type=int, default=None, help='Q pre-scaled by c, S^T seeded with -m c (D = 64, 4 waves)')
    ap.add_argument('--xphase', type=int, default=None, help='counted lgkmcnt waits across phase marks')
    ap.add_argument('--kslag', type=int, default=None, help='KSPLIT reads: MFMAs ahead of their use')
    ap.add_argument('--ksplit', type=int, default=None, help='K reads moved into phase 2')
    ap.add_argument('--fmax', type=int, default=None, help="tile 0's row max sets the starting shift")
    ap.add_argument('--lastu', type=int, default=None, help='unmasked copy of the last tile')
    ap.add_argument('--mzero', type=int, default=None, help='prologue zeroing by MFMAs (D <= 64)')
    ap.add_argument('--andor', type=int, default=None, help='ORDET: last P word joins the test by v_and_or_b32')
    ap.add_argument('--ptail', type=int, default=None, help='rescale test before the last N MFMAs of its phase')
    ap.add_argument('--shift', type=int, default=None, help='loop code placement: N 4-byte s_nop 0 after its alignment')
    ap.add_argument('--soff', type=int, default=None, help='DMA tiles by the SGPR offset of one descriptor (SOFF_WALK)')
    ap.add_argument('--carry', type=int, default=None, help="persistent: a block's decode carried from the previous block")
    ap.add_argument('--bitop3', type=int, default=None, help='ORDET test: (T | P15) & M by one v_bitop3_b32')
    ap.add_argument('--proorder', type=int, default=None, help='one-block prologue: 0 = round-5 section order')
    ap.add_argument('--fdelta', type=float, default=None, help='f16: the rescale delta (P <= 2^-delta after a rescale)')
    ap.add_argument('--defer', type=int, default=None, help="prologue: the last DMA tile after the barrier")
    ap.add_argument('--dmafirst', type=int, default=None, help="persistent: the block's first DMAs before the next decode")
    args = ap.parse_args()
    global LOOP_SHIFT, SOFF_WALK
    if args.shift is not None:
        LOOP_SHIFT = args.shift
    if args.soff is not None:
        SOFF_WALK = bool(args.soff)
    global CARRY_DECODE
    if args.carry is not None:
        CARRY_DECODE = bool(args.carry)
    global ORDET_BITOP3
    if args.bitop3 is not None:
        ORDET_BITOP3 = bool(args.bitop3)
    if args.fdelta is not None:
        ORDET_DELTA['f16'] = args.fdelta
    global DEFER_DMA
    if args.defer is not None:
        DEFER_DMA = bool(args.defer)
    global DMA_FIRST
    if args.dmafirst is not None:
        DMA_FIRST = bool(args.dmafirst)
    global PRO_ORDER
    if args.proorder is not None:
        PRO_ORDER = {0: PRO_ORDER_R5, 1: PRO_ORDER, 2: PRO_ORDER_LANES_FIRST}[args.proorder]
    global DUMP
    if args.dump:
        pt, regs = args.dump.split(':')
        DUMP = (pt, expand_regs(regs))
    PROBE.update(x for x in args.probe.split(',') if x)
    configure(args.hd, args.waves)
    global VREADS_P1, SM_PIPE
    if args.ring or args.dist:
        set_geometry(args.ring or R, args.dist or DIST)
    global BAR2, PERSIST_KV, QCOPY_LATE
    if args.qlate is not None:
        QCOPY_LATE = bool(args.qlate)
    if args.bar2 is not None:
        BAR2 = bool(args.bar2)
        assert not BAR2 or (R >= 6 and DIST >= 3 and U % 2 == 0)
    if args.kvtail is not None:
        PERSIST_KV = bool(args.kvtail)
    if args.vp1 is not None:
        VREADS_P1 = bool(args.vp1)
    if args.smpipe is not None:
        SM_PIPE = bool(args.smpipe)
    global DMA_P2, SPEC
    if args.spec is not None:
        SPEC = bool(args.spec)
    if args.dmap2 is not None:
        DMA_P2 = bool(args.dmap2)
    global ORDET, EXP_LAG, CVT_LAG, MC_BANKS, NVGPR
    if args.ordet is not None:
        ORDET = bool(args.ordet)
    # (--lag and --mcbanks tune the 4-wave softmax stream; the 8-wave form keeps its own settings)
    if args.lag and NWAVES == 4:
        EXP_LAG, CVT_LAG = (int(x) for x in args.lag.split(','))
    if args.mcbanks is not None and NWAVES == 4 and V_MCB is not None:
        MC_BANKS = bool(args.mcbanks)
    global KFIRST, KFIRST_LO, LGKM_XPHASE, PRESCALE, PHASE_TAIL
    if args.ptail is not None:
        PHASE_TAIL = args.ptail
    global ORDET_ANDOR, MFMA_ZERO, LAST_UNMASKED, FIRST_MAX
    if args.fmax is not None:
        FIRST_MAX = bool(args.fmax)
    global KSPLIT
    if args.ksplit is not None:
        KSPLIT = args.ksplit
    global KSPLIT_LAG
    if args.kslag is not None:
        KSPLIT_LAG = args.kslag
    if args.lastu is not None:
        LAST_UNMASKED = bool(args.lastu)
    if args.mzero is not None:
        MFMA_ZERO = bool(args.mzero)
    if args.andor is not None:
        ORDET_ANDOR = bool(args.andor)
    prescale = product_prescale(args.dtype, args.hd, args.waves, bool(args.persist)) if args.prescale is None else bool(args.prescale)
    if args.kfirst is not None:
        KFIRST, KFIRST_LO = args.kfirst > 0, max(0, args.kfirst)
    if args.xphase is not None:
        LGKM_XPHASE = bool(args.xphase)
    global PRIO4, STAGGER
    if args.prio4 is not None:
        PRIO4 = bool(args.prio4)
    if args.stagger and NWAVES == 8:     # (ignored by the 4-wave forms: variant-library builds)
        STAGGER = True
    global FIRST_MAX_W8, STAGGER_FRAC
    if args.fmax8 and NWAVES == 8:
        FIRST_MAX_W8 = True
    if args.sfrac is not None:
        STAGGER_FRAC = args.sfrac
    if args.lag8 and NWAVES == 8:
        EXP_LAG, CVT_LAG = (int(x) for x in args.lag8.split(','))
        set_geometry(6, 3)
    global PINGPONG
    if args.pingpong and NWAVES == 8:
        PINGPONG = STAGGER = True
        set_geometry(6, 3)
    set_persist(bool(args.persist))
    set_prescale(prescale)
    if MC_BANKS:
        NVGPR = max(NVGPR, V_MCB['B'] + 4)
    global KARG_BYTES
    if 'pstamps' in PROBE:
        assert args.hd in (32, 64) and PERSIST and NVGPR <= PS_V
        NVGPR = 256
        KARG_BYTES += 8
    if 'stamps' in PROBE:
        assert args.hd == 64 and not PERSIST and (not PRESCALE or V_SEED['A'] >= STAMP_V + 16)
        NVGPR = max(NVGPR, STAMP_V + 16)
        KARG_BYTES += 8
    g = Gen(args.dtype)
    blocks, n = build(g)
    txt = emit(g, blocks)
    with open(args.out, 'w') as f:
        f.write(txt)
    if args.stats:
        print(f'{args.out}: {sum(len(b) for b in blocks)} items, {n} waits/nops inserted')


if __name__ == '__main__':
    main()
