"""issue_probe.py — cycles per loop iteration of synthetic one-wave-per-SIMD MFMA loops on gfx950,
to price the memory instructions of the attention forward's tile (LDS-DMA pieces against
register-staged loads + ds_write, LDS fragment reads, barriers) beside MFMAs and softmax-like VALU.

Each variant is an assembly kernel (generated here, assembled with the ROCm clang, loaded with
hipModuleLoadData): 256 workgroups of 4 waves (one per SIMD: 512 registers per lane, 96 KiB LDS),
every wave runs `iters` iterations of one body and stores its s_memtime delta. The body is
`nm` v_mfma_f32_32x32x16_bf16 (4 accumulator chains) with the fillers of each gap given by a spec.

    python tools/micro/issue_probe.py [--iters 400] [--variants base,dma2,...]

Variant spec: comma-free tokens joined by '+': fill=<letters> (per MFMA gap: E exp, F fma,
C cvt_pk, O or3), dma=<n> (LDS-DMA pieces per iteration), gld=<n> (buffer_load_dwordx4 to VGPRs),
dsw=<n> (ds_write_b128), dsr=<n> (ds_read_b128), tr=<n> (ds_read_b64_tr_b16), bar (s_barrier per
iteration), s16=<n> (16x16x32 MFMAs appended), stream (sources walk 16 KiB per iteration through
a 4 MiB window per workgroup instead of re-reading one 16 KiB tile).
"""
import argparse
import ctypes
import os
import struct
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LLVM = "/opt/rocm/lib/llvm/bin"

FILL = {
    'E': 'v_exp_f32 v{d}, v{s}',
    'F': 'v_fma_f32 v{d}, v{s}, s20, -v{t}',
    'C': 'v_cvt_pk_bf16_f32 v{d}, v{s}, v{t}',
    'O': 'v_or3_b32 v{d}, v{s}, v{t}, v{s}',
    'M': 'v_max3_f32 v{d}, v{s}, v{t}, v{s}',
}


def parse(spec):
    o = dict(fill='', dma=0, gld=0, dsw=0, dsr=0, tr=0, bar=False, s16=0, stream=False, nm=16, mwait=-1)
    for tok in spec.split('+'):
        if not tok or tok == 'base':
            continue
        if '=' in tok:
            k, v = tok.split('=')
            o[k] = v if k == 'fill' else int(v)
        else:
            o[tok] = True
    return o


def body(o):
    """One iteration: list of instruction lines."""
    nm, fill = o['nm'], o['fill']
    mem = []
    for i in range(o['dma']):
        mem.append([f's_add_u32 m0, s21, {1024 * (i % 16)}', 's_nop 0',
                    f'buffer_load_dwordx4 v60, s[8:11], s30 offen offset:{(i % 4) * 1024} lds'])
    for i in range(o['gld']):
        r = 64 + 4 * (i % 8)
        mem.append([f'buffer_load_dwordx4 v[{r}:{r + 3}], v60, s[8:11], s30 offen offset:{(i % 4) * 1024}'])
    for i in range(o['dsw']):
        r = 96 + 4 * (i % 4)
        mem.append([f'ds_write_b128 v61, v[{r}:{r + 3}] offset:{32768 + 1024 * (i % 16)}'])
    for i in range(o['dsr']):
        mem.append([f'ds_read_b128 a[{64 + 4 * (i % 16)}:{67 + 4 * (i % 16)}], v62 offset:{2048 * (i % 8)}'])
    for i in range(o['tr']):
        mem.append([f'ds_read_b64_tr_b16 a[{128 + 2 * (i % 32)}:{129 + 2 * (i % 32)}], v63 offset:{512 * (i % 32)}'])
    # spread memory ops over the gaps
    gaps = [[] for _ in range(nm)]
    for k, m in enumerate(mem):
        gaps[(k * nm) // max(1, len(mem))].extend(m)
    lines = []
    fi = 0
    for g in range(nm):
        acc = 16 * (g % 4)
        c = f'v[{acc}:{acc + 15}]'
        lines.append(f'v_mfma_f32_32x32x16_bf16 {c}, a[0:3], a[4:7], {c}')
        for ch in fill:
            d = 160 + fi % 32
            s = 200 + (fi + 7) % 32
            t = 200 + (fi + 13) % 32
            lines.append(FILL[ch].format(d=d, s=s, t=t))
            fi += 1
        lines += gaps[g]
    for k in range(o['s16']):
        lines.append('v_mfma_f32_16x16x32_bf16 a[32:35], a[0:3], a[4:7], a[32:35]')
    if o['stream']:
        lines += ['s_add_u32 s30, s30, 16384', 's_and_b32 s30, s30, 0x3fffff']
    vm = o['mwait']
    if vm < 0:
        vm = 2 * (o['dma'] + o['gld'])   # two iterations in flight
    lines.append(f's_waitcnt vmcnt({min(vm, 63)}) lgkmcnt(0)')
    if o['bar']:
        lines.append('s_barrier')
    return lines


def kernel(name, o, iters):
    L = ['.amdgcn_target "amdgcn-amd-amdhsa--gfx950"', '.amdhsa_code_object_version 5', '.text',
         f'.globl {name}', '.p2align 8', f'.type {name},@function', f'{name}:']
    # args: s[0:1] -> {src ptr, out ptr}
    L += ['s_load_dwordx4 s[12:15], s[0:1], 0x0', 's_waitcnt lgkmcnt(0)',
          # src descriptor: base = src + wg * 4 MiB, num_records 4 MiB
          's_lshl_b32 s16, s2, 22', 's_add_u32 s8, s12, s16', 's_addc_u32 s9, s13, 0',
          's_mov_b32 s10, 0x400000', 's_mov_b32 s11, 0x00020000',
          's_mov_b32 s20, 0x3e000000', 's_mov_b32 s30, 0',
          'v_lshrrev_b32 v1, 6, v0', 's_nop 1', 'v_readfirstlane_b32 s22, v1',
          's_lshl_b32 s21, s22, 10',                      # m0 base: 1 KiB per wave
          'v_and_b32 v2, 63, v0', 'v_lshlrev_b32 v60, 4, v2',   # 16 B per lane
          'v_lshlrev_b32 v61, 4, v2', 'v_lshlrev_b32 v62, 4, v2', 'v_lshlrev_b32 v63, 3, v2',
          'v_cvt_f32_u32 v3, v0', 'v_mul_f32 v3, 0x3a83126f, v3']
    for r in range(8):
        L.append(f'v_accvgpr_write_b32 a{r}, v3')
    for r in list(range(160, 192)) + list(range(200, 232)):
        L.append(f'v_mov_b32 v{r}, v3')
    for r in range(64):
        L.append(f'v_mov_b32 v{r}, 0' if r not in (60, 61, 62, 63) else 's_nop 0')
    L += ['s_mov_b32 s23, 0', 's_barrier', 's_memtime s[24:25]', 's_waitcnt lgkmcnt(0)', '.Lloop:']
    L += ['\t' + x for x in body(o)]
    L += ['s_add_u32 s23, s23, 1', f's_cmp_lt_u32 s23, {iters}', 's_cbranch_scc1 .Lloop',
          's_waitcnt vmcnt(0) lgkmcnt(0)',
          's_memtime s[26:27]', 's_waitcnt lgkmcnt(0)',
          's_sub_u32 s26, s26, s24', 's_subb_u32 s27, s27, s25',
          # out[wg * 4 + wave] (8 bytes), lane 0 only
          's_lshl_b32 s28, s2, 2', 's_add_u32 s28, s28, s22', 's_lshl_b32 s28, s28, 3',
          'v_mov_b32 v4, s26', 'v_mov_b32 v5, s27', 'v_mov_b32 v6, s28',
          # a sink of every accumulator chain and filler (keeps nothing dead)
          's_mov_b64 exec, 1', 's_nop 1',
          'global_store_dwordx2 v6, v[4:5], s[14:15]', 's_waitcnt vmcnt(0)', 's_endpgm']
    L += ['.Lfunc_end:', f'\t.size {name}, .Lfunc_end-{name}', '', '.rodata', '.p2align 6',
          f'.amdhsa_kernel {name}', '\t.amdhsa_group_segment_fixed_size 98304',
          '\t.amdhsa_private_segment_fixed_size 0', '\t.amdhsa_kernarg_size 16',
          '\t.amdhsa_user_sgpr_count 2', '\t.amdhsa_user_sgpr_kernarg_segment_ptr 1',
          '\t.amdhsa_system_sgpr_workgroup_id_x 1', '\t.amdhsa_system_vgpr_workitem_id 0',
          '\t.amdhsa_next_free_vgpr 512', '\t.amdhsa_next_free_sgpr 48', '\t.amdhsa_accum_offset 256',
          '\t.amdhsa_reserve_vcc 1', '\t.amdhsa_ieee_mode 0', '.end_amdhsa_kernel', '',
          '.amdgpu_metadata', '---', 'amdhsa.kernels:', '  - .agpr_count: 256', '    .args:',
          '      - .offset: 0', '        .size: 16', '        .value_kind: by_value',
          '    .group_segment_fixed_size: 98304', '    .kernarg_segment_align: 8',
          '    .kernarg_segment_size: 16', '    .max_flat_workgroup_size: 256', f'    .name: {name}',
          '    .private_segment_fixed_size: 0', '    .sgpr_count: 50', f'    .symbol: {name}.kd',
          '    .vgpr_count: 512', '    .wavefront_size: 64', 'amdhsa.target: amdgcn-amd-amdhsa--gfx950',
          'amdhsa.version:', '  - 1', '  - 2', '...', '.end_amdgpu_metadata', '']
    return '\n'.join(L)


def build(tag, o, iters, out_dir):
    name = 'probe_' + ''.join(c if c.isalnum() else '_' for c in tag)
    s = os.path.join(out_dir, name + '.s')
    open(s, 'w').write(kernel(name, o, iters))
    subprocess.check_call([f'{LLVM}/clang', '-x', 'assembler', '-target', 'amdgcn-amd-amdhsa', '-mcpu=gfx950', '-c',
                           s, '-o', s[:-2] + '.o'])
    subprocess.check_call([f'{LLVM}/ld.lld', '-shared', s[:-2] + '.o', '-o', s[:-2] + '.hsaco'])
    return open(s[:-2] + '.hsaco', 'rb').read(), name


DEFAULT = ('base;fill=EFFF;fill=EFFF+dma=2;fill=EFFF+dma=4;fill=EFFF+gld=2+dsw=2;fill=EFFF+gld=4+dsw=4;'
           'fill=EFFF+gld=4;fill=EFFF+dsw=4;fill=EFFF+dsr=8;fill=EFFF+tr=16;fill=EFFF+dsr=8+tr=16;'
           'fill=EFFF+dsr=8+tr=16+dma=4;fill=EFFF+dsr=8+tr=16+gld=4+dsw=4;fill=EFFF+bar;'
           'fill=EFFF+dsr=8+tr=16+dma=4+stream;fill=EFFF+dsr=8+tr=16+gld=4+dsw=4+stream')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=400)
    ap.add_argument('--variants', default=DEFAULT, help="';'-separated specs")
    ap.add_argument('--build-only', action='store_true')
    args = ap.parse_args()
    out = os.path.join(ROOT, 'gpurun_out', 'issue_probe')
    os.makedirs(out, exist_ok=True)
    specs = args.variants.split(';')
    imgs = {sp: build(sp, parse(sp), args.iters, out) for sp in specs}
    if args.build_only:
        print(f'built {len(imgs)} variants in {out}')
        return
    import torch
    dev = torch.device('cuda', 0)
    src = torch.randn(256 * (4 << 20) // 4, device=dev)
    cyc = torch.zeros(256 * 4, dtype=torch.int64, device=dev)
    libs = [ln.split()[-1] for ln in open('/proc/self/maps').read().split('\n') if 'libamdhip64' in ln]
    hip = ctypes.CDLL(libs[0])
    kb = struct.pack('<2Q', src.data_ptr(), cyc.data_ptr())
    kbuf = ctypes.create_string_buffer(kb, len(kb))
    size = ctypes.c_size_t(len(kb))
    extra = (ctypes.c_void_p * 5)(1, ctypes.addressof(kbuf), 2, ctypes.addressof(size), 3)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    keep = []
    for sp in specs:
        img, name = imgs[sp]
        mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
        buf = ctypes.create_string_buffer(img, len(img))
        keep.append(buf)
        assert hip.hipModuleLoadData(ctypes.byref(mod), buf) == 0
        assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, name.encode()) == 0
        res = []
        for rep in range(4):
            assert hip.hipModuleLaunchKernel(fn, 256, 1, 1, 256, 1, 1, 0, stream, None, extra) == 0
            torch.cuda.synchronize()
            if rep:
                res.append(cyc.double().median().item() / args.iters)
        o = parse(sp)
        print(f'{sp:60s} {np.median(res):8.1f} cyc/iter  ({np.median(res) / o["nm"]:6.2f} per MFMA gap)', flush=True)


if __name__ == '__main__':
    main()
