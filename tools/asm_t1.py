"""asm_t1.py — minimal assembly-kernel probe of the launch machinery (kernel descriptor, kernarg
loads, workgroup ids, buffer stores), built with gen_fwd.emit. Debug only."""
import ctypes, os, subprocess, sys, struct
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd", "csrc", "asm"))
import gen_fwd as G

def build(out_dir):
    g = G.Gen('bf16')
    body = [G.raw('s_load_dwordx16 s[40:55], s[0:1], 0x0'), G.raw('s_waitcnt lgkmcnt(0)'),
            # descriptor on the o pointer (kernarg offset 24 = s[46:47]), 4096 bytes
            G.raw('s_mov_b32 s84, s46'), G.raw('s_and_b32 s85, s47, 0xffff'), G.raw('s_mov_b32 s86, 4096'),
            G.raw('s_mov_b32 s87, 0x00020000'),
            G.raw('v_and_b32 v1, 63, v0'), G.raw('v_lshlrev_b32 v2, 2, v0'),   # byte offset 4*tid
            G.raw('v_mov_b32 v3, s2'), G.raw('v_add_u32 v3, v3, v0'),
            G.raw('s_nop 4'),
            G.raw('buffer_store_dword v3, v2, s[84:87], 0 offen'),
            G.raw('v_mov_b32 v4, s40'), G.raw('s_nop 4'),
            G.raw('buffer_store_dword v4, v2, s[84:87], 0 offen offset:1024'),
            G.raw('s_waitcnt vmcnt(0)'), G.raw('s_endpgm')]
    txt = G.emit(g, [body])
    s = os.path.join(out_dir, 't1.s'); open(s, 'w').write(txt)
    subprocess.check_call([f"/opt/rocm/lib/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                           "-mcpu=gfx950", "-c", s, "-o", s[:-2] + ".o"])
    subprocess.check_call(["/opt/rocm/lib/llvm/bin/ld.lld", "-shared", s[:-2] + ".o", "-o", s[:-2] + ".hsaco"])
    return open(s[:-2] + ".hsaco", "rb").read()

def main():
    out = os.path.join(ROOT, "gpurun_out"); os.makedirs(out, exist_ok=True)
    image = build(out)
    if len(sys.argv) > 1 and sys.argv[1] == '--build-only':
        print('built'); return
    import torch
    dev = torch.device('cuda', 0)
    to = torch.zeros(4096, dtype=torch.uint8, device=dev)
    kb = struct.pack('<7Q4Q4I2I2f2I2I2I', 0x1234, 0, 0, to.data_ptr(), 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0.0, 0.0, 0, 0, 0, 0, 0, 0)
    libs = [ln.split()[-1] for ln in open("/proc/self/maps").read().split("\n") if "libamdhip64" in ln]
    hip = ctypes.CDLL(libs[0])
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    img = ctypes.create_string_buffer(image, len(image))
    print('load', hip.hipModuleLoadData(ctypes.byref(mod), img))
    print('getfn', hip.hipModuleGetFunction(ctypes.byref(fn), mod, b"fa_fwd_d64_bf16_asm"))
    kbuf = ctypes.create_string_buffer(kb, len(kb)); size = ctypes.c_size_t(len(kb))
    extra = (ctypes.c_void_p * 5)(1, ctypes.addressof(kbuf), 2, ctypes.addressof(size), 3)
    torch.cuda.synchronize()
    print('launch', hip.hipModuleLaunchKernel(fn, 1, 1, 1, 256, 1, 1, 0, ctypes.c_void_p(0), None, extra), flush=True)
    torch.cuda.synchronize()
    r = to.cpu().numpy().view(np.uint32)
    print('tid+wgx', r[:8].tolist(), r[250:256].tolist(), 'kernarg[0]', hex(int(r[256])), hex(int(r[300])))

main()
