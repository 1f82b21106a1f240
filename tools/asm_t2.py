"""asm_t2.py — bisect the assembly forward's prologue on the GPU: run the first N items of
gen_fwd.prologue(), then store a set of SGPR / VGPR values with the minimal store sequence of
asm_t1.py (which is known to work). Debug only."""
import ctypes, os, subprocess, sys, struct
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd", "csrc", "asm"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_fwd as G
import asm_sim

SREGS = ['s2', 's3', 's4', 's37', 's76', 's77', 's78', 's79', 's86', 's87', 's88', 's89', 's90',
         's8', 's9', 's10', 's11', 's20', 's21', 's22', 's46', 's47', 's31', 's38']

def build(cut, out_dir):
    g = G.Gen('bf16')
    pro = G.prologue(g)
    # the hazard pass on the cut prologue + probe tail
    body = pro[:cut]
    tail = [G.raw('s_waitcnt vmcnt(0) lgkmcnt(0)'), G.raw('s_nop 7'),
            G.raw('s_mov_b32 s84, s46'), G.raw('s_and_b32 s85, s47, 0xffff'), G.raw('s_mov_b32 s86, 65536'),
            G.raw('s_mov_b32 s87, 0x00020000'), G.raw('v_lshlrev_b32 v2, 2, v0'), G.raw('s_nop 4')]
    for i, r in enumerate(SREGS):
        tail += [G.raw(f'v_mov_b32 v3, {r}'), G.raw('s_nop 2'),
                 G.raw(f'buffer_store_dword v3, v2, s[84:87], 0 offen offset:{(i % 4) * 1024}')]
        if i % 4 == 3:
            tail += [G.raw('s_waitcnt vmcnt(0)'), G.raw('v_add_u32 v2, 4096, v2'), G.raw('s_nop 2')]
    tail += [G.raw('s_waitcnt vmcnt(0)'), G.raw('s_endpgm')]
    blk = body + tail
    G.fix_paths([lambda: G.refs(blk)])
    txt = G.emit(g, [blk, [G.label('.Lend'), G.raw('s_endpgm'), G.label('.Lempty'), G.raw('s_endpgm')]])
    s = os.path.join(out_dir, f't2_{cut}.s'); open(s, 'w').write(txt)
    subprocess.check_call(["/opt/rocm/lib/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                           "-mcpu=gfx950", "-c", s, "-o", s[:-2] + ".o"])
    subprocess.check_call(["/opt/rocm/lib/llvm/bin/ld.lld", "-shared", s[:-2] + ".o", "-o", s[:-2] + ".hsaco"])
    return txt, open(s[:-2] + ".hsaco", "rb").read()

def inputs(sq=64, sk=64, H=1, Dh=64):
    rng = np.random.default_rng(0)
    q = asm_sim.bf16_bits(rng.standard_normal((sq, H, Dh)).astype(np.float32)).astype(np.uint16)
    k = asm_sim.bf16_bits(rng.standard_normal((sk, H, Dh)).astype(np.float32)).astype(np.uint16)
    v = asm_sim.bf16_bits(rng.standard_normal((sk, H, Dh)).astype(np.float32)).astype(np.uint16)
    return q, k, v, np.array([0, sq], np.int32), np.array([0, sk], np.int32)

def karg(pq, pk, pv, po, pl, pcq, pck, H=1, Dh=64, lse_stride=64, nqb=1):
    mg = lambda d: ((1 << 32) + 2 * d - 1) // (2 * d)
    c = np.float32(Dh ** -0.5 * 1.4426950408889634)
    return struct.pack("<7Q4Q4I2I2f2I2I2I", pq, pk, pv, po, pl, pcq, pck, Dh * 2, Dh * 2, Dh * 2, Dh * 2,
                       H * Dh * 2, H * Dh * 2, H * Dh * 2, H * Dh * 2, H, lse_stride * 4, c, np.float32(8.0 / c),
                       nqb, nqb * H, mg(nqb), mg(H), Dh, 0)

def main():
    cut = int(sys.argv[1])
    if len(sys.argv) > 3:
        G.WAVE_MODE = sys.argv[3]
    out = os.path.join(ROOT, "gpurun_out"); os.makedirs(out, exist_ok=True)
    txt, image = build(cut, out)
    q, k, v, cq, ck = inputs()
    # simulator
    mem = asm_sim.Memory()
    P = [mem.alloc(x) for x in (q, k, v)]
    po = mem.alloc(np.zeros(65536, np.uint8)); pl = mem.alloc(np.zeros(256, np.float32))
    pcq, pck = mem.alloc(cq), mem.alloc(ck)
    pa = mem.alloc(np.frombuffer(karg(*P, po, pl, pcq, pck), np.uint8))
    asm_sim.Sim(txt).run((1, 1, 1), pa, mem)
    simr = mem.get(po).view(np.uint32)
    if len(sys.argv) > 2 and sys.argv[2] == 'sim':
        print('sim only'); return
    import torch
    dev = torch.device('cuda', 0)
    T = [torch.from_numpy(x.view(np.int16)).to(dev) for x in (q, k, v)]
    to = torch.zeros(65536, dtype=torch.uint8, device=dev); tl = torch.zeros(256, device=dev)
    tcq, tck = torch.from_numpy(cq).to(dev), torch.from_numpy(ck).to(dev)
    kb = karg(*[t.data_ptr() for t in T], to.data_ptr(), tl.data_ptr(), tcq.data_ptr(), tck.data_ptr())
    libs = [ln.split()[-1] for ln in open("/proc/self/maps").read().split("\n") if "libamdhip64" in ln]
    hip = ctypes.CDLL(libs[0])
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    img = ctypes.create_string_buffer(image, len(image))
    assert hip.hipModuleLoadData(ctypes.byref(mod), img) == 0
    assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, b"fa_fwd_d64_bf16_asm") == 0
    kbuf = ctypes.create_string_buffer(kb, len(kb)); size = ctypes.c_size_t(len(kb))
    extra = (ctypes.c_void_p * 5)(1, ctypes.addressof(kbuf), 2, ctypes.addressof(size), 3)
    torch.cuda.synchronize()
    assert hip.hipModuleLaunchKernel(fn, 1, 1, 1, 256, 1, 1, 0, ctypes.c_void_p(0), None, extra) == 0
    torch.cuda.synchronize()
    gr = to.cpu().numpy().view(np.uint32)
    for i, r in enumerate(SREGS):
        blk, sub = divmod(i, 4)
        base = blk * 1024 + sub * 256
        gv, sv = gr[base:base + 256], simr[base:base + 256]
        flag = '' if (gv == sv).all() else '   <-- DIFF'
        print(f'{G.WAVE_MODE} cut {cut} {r}: gpu {hex(int(gv[0]))} {hex(int(gv[64]))} sim {hex(int(sv[0]))} {hex(int(sv[64]))}{flag}')

main()
