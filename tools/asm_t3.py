"""asm_t3.py — probe VALU -> SGPR writes (v_readfirstlane / v_readlane) on gfx950. Debug only."""
import ctypes, os, subprocess, sys, struct
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd", "csrc", "asm"))
import gen_fwd as G

def build(out_dir):
    g = G.Gen('bf16')
    R = G.raw
    b = [R('s_load_dwordx16 s[40:55], s[0:1], 0x0'), R('s_waitcnt lgkmcnt(0)'),
         R('s_mov_b32 s84, s46'), R('s_and_b32 s85, s47, 0xffff'), R('s_mov_b32 s86, 65536'),
         R('s_mov_b32 s87, 0x00020000'), R('v_lshlrev_b32 v2, 2, v0'),
         R('v_lshrrev_b32 v1, 6, v0'), R('s_nop 4')]
    def st(src, slot):
        return [R(f'v_mov_b32 v3, {src}'), R('s_nop 2'),
                R(f'buffer_store_dword v3, v2, s[84:87], 0 offen offset:{slot * 1024 % 4096}')] + \
               ([R('v_add_u32 v2, 4096, v2'), R('s_nop 2')] if slot % 4 == 3 else [])
    b += [R('v_readfirstlane_b32 s37, v1'), R('s_nop 4')] + st('s37', 0)
    b += [R('v_readlane_b32 s38, v1, 0'), R('s_nop 4')] + st('s38', 1)
    b += [R('v_readfirstlane_b32 s5, v1'), R('s_nop 4')] + st('s5', 2)
    b += [R('s_mov_b32 s90, 77'), R('s_nop 1')] + st('s90', 3)
    b += [R('s_nop 15')] * 8 + st('s37', 4) + st('v1', 5)
    b += [R('s_mov_b32 s37, 55'), R('s_nop 1')] + st('s37', 6)
    b += [R('v_readfirstlane_b32 s37, v1'), R('s_waitcnt vmcnt(0)'), R('s_nop 7'), R('s_nop 7')] + st('s37', 7)
    b += [R('s_waitcnt vmcnt(0)'), R('s_endpgm')]
    txt = G.emit(g, [b])
    s = os.path.join(out_dir, 't3.s'); open(s, 'w').write(txt)
    subprocess.check_call(["/opt/rocm/lib/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                           "-mcpu=gfx950", "-c", s, "-o", s[:-2] + ".o"])
    subprocess.check_call(["/opt/rocm/lib/llvm/bin/ld.lld", "-shared", s[:-2] + ".o", "-o", s[:-2] + ".hsaco"])
    return open(s[:-2] + ".hsaco", "rb").read()

def main():
    out = os.path.join(ROOT, "gpurun_out"); os.makedirs(out, exist_ok=True)
    image = build(out)
    if len(sys.argv) > 1:
        print('built'); return
    import torch
    dev = torch.device('cuda', 0)
    to = torch.zeros(65536, dtype=torch.uint8, device=dev)
    kb = struct.pack('<7Q4Q4I2I2f2I2I2I', 0, 0, 0, to.data_ptr(), 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0.0, 0.0, 0, 0, 0, 0, 0, 0)
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
    r = to.cpu().numpy().view(np.uint32)
    names = ['rfl s37', 'readlane s38', 'rfl s5', 's_mov s90=77', 's37 later', 'v1', 's_mov s37=55', 'rfl s37 + waits']
    for i, n in enumerate(names):
        base = (i // 4) * 1024 + (i % 4) * 256
        print(f'{n:18s}', [hex(int(r[base + 64 * w])) for w in range(4)])

main()
