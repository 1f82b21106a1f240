"""CPU check of the hand-scheduled assembly forward (csrc/asm/gen_fwd.py) in the functional
simulator tools/asm_sim.py: the generated instruction stream, run one workgroup at a time with
the MFMA / LDS fragment maps of the MI355X guide, must reproduce the fp32 oracle
(oracle/attention_ref.py, restating tests/test_flash_attn.py:115-159 of the reference) on small
var-len cases, including the masked last tile, empty key sets and the rescale path. The GPU tests
(tests/test_flash_attn.py, -m gpu) run the same kernel on the hardware."""
import math
import os
import struct
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd", "csrc", "asm"))

import asm_sim  # noqa: E402
import gen_fwd  # noqa: E402
from oracle.attention_ref import attention_ref  # noqa: E402

_TXT = {}


def _kernel(dtype, hd=64, waves=4, persist=False, prescale=None):
    """prescale: None = the product setting of build.py for this form (gen_fwd.product_prescale)."""
    if prescale is None:
        prescale = gen_fwd.product_prescale(dtype, hd, waves, persist)
    key = (dtype, hd, waves, persist, prescale)
    if key not in _TXT:
        gen_fwd.configure(hd, waves)
        try:
            gen_fwd.set_persist(persist)
            gen_fwd.set_prescale(prescale)
            g = gen_fwd.Gen(dtype)
            blocks, _ = gen_fwd.build(g)
            _TXT[key] = gen_fwd.emit(g, blocks)
        finally:
            gen_fwd.set_prescale(False)
            gen_fwd.set_persist(False)
            gen_fwd.configure(64)
    return _TXT[key]


def _run(lens_q, lens_k, H, D, dtype, scale=None, seed=0, causal=False, waves=4, grid=None, prescale=None, hd=None):
    """grid: the persistent form's workgroup count (each walks blocks L, L + grid, ...); hd: the
    tile (default: the one fa_asm.cpp picks for head_dim D)."""
    rng = np.random.default_rng(seed)
    cv = asm_sim.bf16_bits if dtype == "bf16" else asm_sim.f16_bits
    B, tq, tk = len(lens_q), sum(lens_q), sum(lens_k)
    q = cv(rng.standard_normal((tq, H, D)).astype(np.float32)).astype(np.uint16)
    k = cv(rng.standard_normal((tk, H, D)).astype(np.float32)).astype(np.uint16)
    v = cv(rng.standard_normal((tk, H, D)).astype(np.float32)).astype(np.uint16)
    mem = asm_sim.Memory()
    pq, pk, pv = mem.alloc(q), mem.alloc(k), mem.alloc(v)
    po = mem.alloc(np.zeros((tq, H, D), np.uint16))
    maxq = max(lens_q)
    lse_stride = max((maxq + 15) // 16 * 16, 16)
    pl = mem.alloc(np.full((B, H, lse_stride), 7.0, np.float32))
    cq = np.concatenate([[0], np.cumsum(lens_q)]).astype(np.int32)
    ck = np.concatenate([[0], np.cumsum(lens_k)]).astype(np.int32)
    pcq, pck = mem.alloc(cq), mem.alloc(ck)
    scale = D ** -0.5 if scale is None else scale
    c = np.float32(scale * 1.4426950408889634)
    nqb = (maxq + 255) // 256
    mg = lambda d: ((1 << 32) + 2 * d - 1) // (2 * d)
    per = grp = 0
    if causal and (H * B) % 8 == 0:     # fa_asm.cpp's group choice
        nh, want = H * B // 8, (64 + nqb - 1) // nqb
        grp = max(c for c in range(1, min(nh, want) + 1) if nh % c == 0)
        per = grp * nqb
    karg = struct.pack("<7Q4Q4I2I2f2I2I2I2I4I", pq, pk, pv, po, pl, pcq, pck, D * 2, D * 2, D * 2, D * 2,
                       H * D * 2, H * D * 2, H * D * 2, H * D * 2, H, lse_stride * 4, c, np.float32(8.0 / c),
                       nqb, nqb * H * B, mg(nqb), mg(H), D, H * B, int(causal), mg(H * B),
                       per, mg(per) if per else 0, grp, mg(grp) if grp else 0)
    if grid:
        karg += struct.pack("<2I", grid, 0)
    pa = mem.alloc(np.frombuffer(karg, np.uint8))
    if hd is None:
        hd = 128 if D > 96 else 96 if D > 64 else 64 if D > 32 else 32
    if prescale is None:
        prescale = gen_fwd.product_prescale(dtype, hd, waves, bool(grid))
    asm_sim.Sim(_kernel(dtype, hd, waves, bool(grid), prescale), dtype).run(
        (grid, 1, 1) if grid else (nqb, H, B), pa, mem)
    o = asm_sim.from16(mem.get(po).view(np.uint16).astype(np.uint32), dtype).reshape(tq, H, D)
    lse = mem.get(pl).view(np.float32).reshape(B, H, lse_stride)
    to = lambda x: torch.from_numpy(asm_sim.from16(x.astype(np.uint32), dtype))
    qf, kf, vf = to(q), to(k), to(v)
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float16
    for b in range(B):
        sq, sk = slice(cq[b], cq[b + 1]), slice(ck[b], ck[b + 1])
        o_b = torch.from_numpy(o[sq])
        if lens_k[b] == 0:
            assert torch.count_nonzero(o_b) == 0
            assert np.all(lse[b, :, :lens_q[b]] == -np.inf)
            continue
        # the reference's own oracle at fp32 and at the input precision (the 2x rule of
        # tests/test_flash_attn.py:407-409)
        args = (qf[sq][None], kf[sk][None], vf[sk][None])
        ref = attention_ref(*args, upcast=True, causal=causal)[0][0] if scale == D ** -0.5 else None
        cmask = torch.triu(torch.ones(lens_q[b], lens_k[b], dtype=torch.bool), 1) if causal else None
        if ref is None:
            s = torch.einsum("qhd,khd->hqk", qf[sq].double(), kf[sk].double()) * scale
            if causal:
                s = s.masked_fill(cmask, float("-inf"))
            ref = torch.einsum("hqk,khd->qhd", torch.softmax(s, -1), vf[sk].double()).float()
            base = 4e-3
            if prescale:
                # the PyTorch low-precision baseline at this scale: scores rounded to the input type
                # (as attention_ref(upcast=False) rounds its einsum output), softmax, P V
                s_lo = s.to(tdt).double()
                lo = torch.einsum("hqk,khd->qhd", torch.softmax(s_lo, -1).to(tdt).double(), vf[sk].double()).float()
                base = max(base, (lo - ref).abs().max().item())
        else:
            lo = attention_ref(*(x.to(tdt) for x in args), upcast=False, causal=causal)[0][0].float()
            base = (lo - ref).abs().max().item()
        assert (o_b - ref).abs().max().item() <= 2 * base + 1e-4, (b, (o_b - ref).abs().max().item(), base)
        s = torch.einsum("qhd,khd->hqk", qf[sq].double(), kf[sk].double()) * scale
        if causal:
            s = s.masked_fill(cmask, float("-inf"))
        ref_lse = torch.logsumexp(s, -1).numpy()
        # the row sums cover the 16-bit-rounded P (what multiplies V): up to 2^-8 relative in the
        # sum, so the LSE is within 4e-3; the PRESCALE form's scores carry the
        # rounding of Q c to the input type: its bound is twice the LSE error of scores rounded
        # to the input type (the low-precision baseline above)
        tol = 4e-3
        if prescale:
            tol = max(tol, 2 * np.abs(torch.logsumexp(s.to(tdt).double(), -1).numpy() - ref_lse).max())
        assert np.abs(lse[b, :, :lens_q[b]] - ref_lse).max() < tol


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("lens_q,lens_k,H,D", [
    ([130], [200], 1, 64),            # 3 full tiles + a masked one, rows past the block end
    ([257, 40], [33, 190], 2, 64),    # var-len, two q-blocks, single masked tile
    ([70], [700], 1, 64),             # 11 tiles: every unrolled loop position and its last-tile exit
    ([40, 64], [0, 65], 1, 48),       # empty key set (zeros, -inf), head_dim < 64 zero-padded
])
def test_asm_forward_in_simulator(lens_q, lens_k, H, D, dtype):
    _run(lens_q, lens_k, H, D, dtype)


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("lens_q,lens_k", [
    ([130], [200]),                   # 3 full tiles + a masked one
    ([70, 33], [700, 0]),             # 11 tiles (every loop position, last-tile exit); empty key set
])
def test_asm_forward_d128_in_simulator(lens_q, lens_k, dtype):
    """The head_dim = 128 kernel (single-buffered K / V^T fragments, Q and row sums in VGPRs)."""
    _run(lens_q, lens_k, 1, 128, dtype)


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("lens_q,lens_k", [
    ([300], [300]),                   # two q-blocks: the diagonal band (masked loop) of each, LPT order
    ([70, 600], [130, 520]),          # var-len, Sq != Sk (top-left aligned), unequal band positions
])
def test_asm_forward_causal_in_simulator(lens_q, lens_k, D):
    _run(lens_q, lens_k, 1, D, "bf16", causal=True)


def test_asm_forward_causal_xcd_groups_in_simulator():
    """8 (batch, head) pairs: the XCD-grouped causal order (every workgroup still covers its own
    q-block exactly once)."""
    _run([300] * 4, [300] * 4, 2, 64, "bf16", causal=True)


def test_asm_forward_rescale_path_in_simulator():
    """A large softmax scale makes later tiles pass the running max by more than 2^8: the
    out-of-line rescale block (O, row sums and the permuted alpha) runs past tile 0."""
    _run([70], [300], 1, 64, "bf16", scale=3.0)


@pytest.mark.parametrize("dtype,hd,waves,persist", [
    (dt, hd, w, p) for dt in ("bf16", "f16") for hd, w, p in ((64, 4, False), (128, 4, False), (64, 8, False))] + [
    ("bf16", 64, 4, True), ("bf16", 128, 4, True), ("bf16", 32, 4, False)])   # (f16 persistent: build.py assembles it)
def test_generated_kernel_assembles(dtype, hd, waves, persist, tmp_path):
    """The simulator does not check encodings (register alignment, gfx950 operand forms): the
    product kernels must also assemble for gfx950, as build.py does."""
    import subprocess
    llvm = "/opt/rocm/lib/llvm/bin/clang"
    if not os.path.exists(llvm):
        pytest.skip("no ROCm LLVM")
    s = tmp_path / "k.s"
    s.write_text(_kernel(dtype, hd, waves, persist))
    r = subprocess.run([llvm, "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c", str(s),
                        "-o", str(tmp_path / "k.o")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.parametrize("lens_q,lens_k,causal,dtype", [
    ([130], [200], False, "bf16"),            # 3 full tiles + a masked one, rows past the block end
    ([257, 40], [33, 190], False, "bf16"),    # var-len, two q-blocks, single masked tile
    ([70], [700], False, "bf16"),             # 11 tiles: every unrolled loop position and its last-tile exit
    ([70], [700], False, "f16"),              # (fp16: its own rescale delta)
    ([40, 64], [0, 65], False, "bf16"),       # empty key set (zeros, -inf)
    ([300], [300], True, "bf16"),             # causal: the diagonal band of two q-blocks
])
def test_asm_forward_w8_in_simulator(lens_q, lens_k, causal, dtype):
    """The two-waves-per-SIMD form (8 waves, one 32-row block per wave, head_dim == 64)."""
    _run(lens_q, lens_k, 1, 64, dtype, causal=causal, waves=8)


def test_asm_forward_w8_rescale_path_in_simulator():
    """The 8-wave form's rescale block runs after the phase's P.V MFMAs into the same O."""
    _run([70], [300], 1, 64, "bf16", scale=3.0, waves=8)


@pytest.mark.parametrize("lens_q,lens_k,H,D,grid,dtype", [
    ([130], [200], 3, 64, 1, "bf16"),             # one workgroup walks all 3 blocks (next-Q prefetch each time)
    ([257, 40], [33, 190], 2, 64, 3, "bf16"),     # var-len, 3 workgroups over 8 blocks: empty q-blocks (.Lend)
    ([70, 300], [700, 0], 2, 48, 2, "bf16"),      # 11 tiles, empty key set, head_dim < 64 (masked Q chunks)
    ([300, 200], [512, 256], 2, 64, 1, "bf16"),   # nt = 8 and 4: the tail streams the next block's K/V tiles
    ([300, 200], [512, 256], 2, 64, 1, "f16"),
    ([300, 100], [512, 320], 2, 64, 3, "bf16"),   # tails into a next block with nt % 4 != 0, and into an empty q-block
])
def test_asm_forward_persistent_in_simulator(lens_q, lens_k, H, D, grid, dtype):
    """The persistent form (one workgroup walks blocks L, L + grid, ...; the next block's Q is
    prefetched into spare VGPRs and copied at the seam; a block past its sequence skips to the next)."""
    _run(lens_q, lens_k, H, D, dtype, grid=grid)


@pytest.mark.parametrize("lens_q,lens_k,H,grid", [
    ([300, 200], [512, 256], 2, 1),       # nt = 8 and 4: the tail streams the next block's K/V tiles
    ([300, 100], [512, 320], 2, 3),       # tails into a block with nt % 4 != 0 and into an empty q-block
])
def test_asm_forward_persistent_d128_in_simulator(lens_q, lens_k, H, grid):
    """The persistent form at head_dim = 128 (K/V tail only: Q stays in VGPRs, no next-Q prefetch)."""
    _run(lens_q, lens_k, H, 128, "bf16", grid=grid)


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("lens_q,lens_k,H,D", [
    ([130], [200], 1, 32),            # 3 full tiles + a masked one
    ([70, 33], [700, 0], 1, 32),      # 11 tiles (every loop position, last-tile exit); empty key set
    ([257, 40], [33, 190], 2, 16),    # head_dim 16 zero-padded into the D = 32 tile; var-len
])
def test_asm_forward_d32_in_simulator(lens_q, lens_k, H, D, dtype):
    """The head_dim <= 32 tile (one O d-block, 4-KiB K / V tiles, two 16-deep k-steps)."""
    _run(lens_q, lens_k, H, D, dtype)


def test_asm_forward_d32_causal_and_persistent_in_simulator():
    _run([300], [300], 1, 32, "bf16", causal=True)
    _run([300, 200], [512, 256], 2, 24, "bf16", grid=2)


@pytest.mark.parametrize("lens_q,lens_k,H,D,grid,dtype,causal,scale", [
    ([130], [200], 1, 64, None, "bf16", False, None),       # one-block form: 3 full tiles + a masked one
    ([70], [700], 1, 64, None, "f16", False, None),         # 11 tiles, fp16 (its own rescale delta)
    ([40, 64], [0, 65], 1, 48, None, "bf16", False, None),  # empty key set, head_dim < 64
    ([300], [300], 1, 64, None, "bf16", True, None),        # causal band
    ([70], [300], 1, 64, None, "bf16", False, 3.0),         # forced rescales past tile 0
    ([300, 200], [512, 256], 2, 64, 1, "bf16", False, None),  # persistent: K/V tail, next-Q copy at the seam
    ([300, 100], [512, 320], 2, 64, 3, "f16", False, None),   # persistent: tails, empty q-block, fp16
])
def test_asm_forward_prescaled_in_simulator(lens_q, lens_k, H, D, grid, dtype, causal, scale):
    """The PRESCALE form (Q~ = Q c rounded once per block, S^T seeded with -m c, softmax exp2(S))."""
    _run(lens_q, lens_k, H, D, dtype, scale=scale, causal=causal, grid=grid, prescale=True)


def _run_text(txt, lens_q, lens_k, H, D, dtype, mode="lazy"):
    """_run with a given kernel text (the product kernel cache bypassed)."""
    saved = dict(_TXT)
    hd = 128 if D > 96 else 96 if D > 64 else 64 if D > 32 else 32
    _TXT.clear()
    _TXT[(dtype, hd, 4, False, gen_fwd.product_prescale(dtype, hd, 4, False))] = txt
    orig = asm_sim.Sim.__init__

    def init(self, asm_text, dtype="bf16", soff_checked=True, **kw):
        orig(self, asm_text, dtype, soff_checked, mode=mode)
    asm_sim.Sim.__init__ = init
    try:
        _run(lens_q, lens_k, H, D, dtype)
    finally:
        asm_sim.Sim.__init__ = orig
        _TXT.clear()
        _TXT.update(saved)


def test_simulator_catches_the_round3_d32_wait_bug():
    """the D=32 tile's round-3 hardware bug -- a tile-end vmcnt sized for two DMA pieces
    per tensor and tile when the D=32 tile issues one -- lets the next tile read ring slots whose DMA
    has not landed. With lazy completion the simulator reads the stale slot and the result is wrong;
    the correct count passes."""
    gen_fwd.configure(32)
    try:
        g = gen_fwd.Gen("bf16")
        good = gen_fwd.emit(g, gen_fwd.build(g)[0])
        fixed = gen_fwd.pieces_wait
        gen_fwd.pieces_wait = lambda: 4 * (gen_fwd.DIST - 1)     # the round-3 count
        try:
            g = gen_fwd.Gen("bf16")
            bad = gen_fwd.emit(g, gen_fwd.build(g)[0])
        finally:
            gen_fwd.pieces_wait = fixed
    finally:
        gen_fwd.configure(64)
    assert good != bad
    _run_text(good, [70], [700], 1, 32, "bf16")
    with pytest.raises(AssertionError):
        _run_text(bad, [70], [700], 1, 32, "bf16")


def test_simulator_catches_a_missing_wait_state():
    """Removing the wait state between the VALU that writes the wave index and the v_readfirstlane
    that reads it (round 3: three faulting dumps) raises HazardError in the simulator."""
    txt = _kernel("bf16")
    lines = txt.split("\n")
    i = next(k for k, ln in enumerate(lines) if ln.strip().startswith("v_readfirstlane_b32"))
    assert lines[i - 1].strip().startswith("s_nop"), lines[i - 2:i + 1]
    bad = "\n".join(lines[:i - 1] + lines[i:])
    with pytest.raises(asm_sim.HazardError):
        _run_text(bad, [130], [200], 1, 64, "bf16")


@pytest.mark.parametrize("lens_q,lens_k,H,D,grid,causal", [
    ([300, 200], [512, 256], 2, 96, None, False),    # one-block, two sequences
    ([130], [300], 2, 80, None, False),              # head_dim 80: Q k-step 5 zeroed, O columns 80..95 dropped
    ([257, 100], [700, 190], 2, 80, None, True),     # causal band
    ([300, 200], [512, 256], 2, 96, 2, False),       # persistent, K/V tail into the next block
    ([300, 40], [640, 0], 2, 80, 3, False),          # persistent, empty key set, head_dim 80
])
def test_asm_forward_d96_in_simulator(lens_q, lens_k, H, D, grid, causal):
    """The D = 96 tile (D = 128 layout, 6 k-steps and 3 d-blocks) at head_dim 96 and 80."""
    _run(lens_q, lens_k, H, D, "bf16", causal=causal, grid=grid, hd=96)


def test_simulator_catches_a_wave_dependent_barrier():
    """A barrier that one wave skips (a wave-dependent branch around it) desynchronises the hardware's
    barrier counting; the simulator counts each wave's barriers and raises HazardError."""
    txt = _kernel("bf16")
    lines = txt.split("\n")
    i = next(k for k, ln in enumerate(lines) if ln.strip() == "s_barrier")
    bad = "\n".join(lines[:i] + [f"\ts_cmp_eq_u32 s{gen_fwd.S_WAVE}, 0", "\ts_cbranch_scc1 .Lskipbar_t",
                                 lines[i], ".Lskipbar_t:"] + lines[i + 1:])
    with pytest.raises(asm_sim.HazardError):
        _run_text(bad, [130], [200], 1, 64, "bf16")
