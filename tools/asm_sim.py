"""asm_sim.py — functional simulator of the generated gfx950 assembly kernel (test infrastructure).

Executes the instruction subset csrc/asm/gen_fwd.py emits, one workgroup at a time, with the
fragment layouts of the MI355X guide (cdna_hip_programming.md §3):

  v_mfma_f32_32x32x16: A[i = l&31][k = 8(l>>5)+j], B[k = 8(l>>5)+j][n = l&31],
                       C reg r -> C[(r&3) + 8(r>>2) + 4(l>>5)][l&31]
  v_mfma_f32_16x16x32: A[i = l&15][k = 8(l>>4)+j], B[k = 8(l>>4)+j][n = l&15],
                       C reg r -> C[4(l>>4) + r][l&15]
  ds_read_b64_tr_b16:  in each 16-lane group, lane 4q+p gives the address of row q, columns
                       4p..4p+3; lane i receives column i of rows 0..3
  v_permlane32_swap:   lanes 32..63 of vdst <-> lanes 0..31 of src

Waves run round-robin between s_barriers. Buffer range checks include the SGPR offset (`soff_checked`).

Completion of memory operations (mode `lazy`, the default): every vector-memory operation (loads,
LDS-DMA, stores) and every LDS / SMEM operation is queued per wave in issue order and takes effect
(registers or LDS written) only when an `s_waitcnt vmcnt(N)` / `lgkmcnt(N)` of that wave forces it
(the latest point the hardware allows), or at s_endpgm: a consumer that the generator's counted
waits do not cover reads the OLD contents and the result is wrong. Mode `eager` applies every
operation at issue instead (an LDS-DMA that overwrites a ring slot other waves still read then
shows up). Register hazards: `check_hazards` raises HazardError when an instruction reads a
register closer to its writer than the gfx950 wait states allow (MFMA 32x32 result 12 states,
16x16 8, VALU -> MFMA operand 2, transcendental -> VALU 1, VALU -> v_readfirstlane 1,
VALU -> v_permlane 2); s_nop N counts N + 1 states, s_waitcnt none.

Usage (tests/test_asm_sim.py): Sim(asm_text).run(grid, kernarg_bytes, memory).
"""
import re
import struct

import numpy as np

F32 = np.float32


def bf16_bits(x):
    """fp32 array -> bf16 bits (round to nearest even)."""
    u = np.asarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF
    return r.astype(np.uint32)


def f16_bits(x):
    return np.asarray(x, dtype=np.float32).astype(np.float16).view(np.uint16).astype(np.uint32)


def from16(bits, dtype):
    bits = np.asarray(bits, dtype=np.uint32) & 0xFFFF
    if dtype == 'bf16':
        return (bits << 16).astype(np.uint32).view(np.float32)
    return bits.astype(np.uint16).view(np.float16).astype(np.float32)


class Memory:
    """Flat device memory: named numpy byte buffers at fake addresses."""

    def __init__(self):
        self.bufs = []       # (base, bytearray-like np.uint8)
        self.next = 0x10000000

    def alloc(self, arr):
        data = np.frombuffer(np.ascontiguousarray(arr).tobytes(), dtype=np.uint8).copy()
        base = self.next
        self.next += (len(data) + 0xFFFFF) // 0x100000 * 0x100000 + 0x100000
        self.bufs.append((base, data))
        return base

    def find(self, addr, n):
        for base, data in self.bufs:
            if base <= addr and addr + n <= base + len(data):
                return data, addr - base
        raise MemoryError(f'access outside every allocation: {addr:#x} +{n}')

    def read(self, addr, n):
        d, o = self.find(addr, n)
        return d[o:o + n]

    def write(self, addr, b):
        d, o = self.find(addr, len(b))
        d[o:o + len(b)] = b

    def get(self, base):
        for b, data in self.bufs:
            if b == base:
                return data
        raise KeyError(base)


_RANGE = re.compile(r'^([vas])\[(\d+):(\d+)\]$')
_ONE = re.compile(r'^([vas])(\d+)$')


class Wave:
    def __init__(self, nv, na, wave_id, wg):
        self.v = np.zeros((nv, 64), dtype=np.uint32)
        self.a = np.zeros((256, 64), dtype=np.uint32)
        self.s = np.zeros(110, dtype=np.uint64)
        self.vcc = np.zeros(64, dtype=bool)
        self.scc = False
        self.m0 = 0
        self.pc = 0
        self.done = False
        self.vmq = []        # pending vector-memory completions (callables), issue order
        self.lgq = []        # pending LDS / SMEM completions
        self.state = 0       # issued wait states (hazard checks)
        self.wr = {}         # register -> (state after the writer, writer class, writer dst range)
        self.pend = {}       # register -> pc of the queued load that will write it (lazy mode)
        self.v[0] = np.arange(64, dtype=np.uint32) + 64 * wave_id
        self.s[2], self.s[3], self.s[4] = wg


class HazardError(RuntimeError):
    pass


# minimum distance in issued states from a writer class to a reader class (1 = back to back)
_NEED = {('mfma32', None): 13, ('mfma16', None): 9, ('valu', 'mfma'): 3, ('trans', 'mfma'): 3,
         ('trans', 'valu'): 2, ('trans', 'trans'): 2, ('trans', 'rfl'): 2, ('trans', 'perm'): 3,
         ('valu', 'rfl'): 2, ('valu', 'perm'): 3}
_TRANS = ('v_exp_f32', 'v_log_f32', 'v_rcp_f32')


class Sim:
    def __init__(self, asm_text, dtype='bf16', soff_checked=True, mode='lazy', check_hazards=True):
        self.dtype = dtype
        self.soff_checked = soff_checked
        assert mode in ('lazy', 'eager')
        self.mode, self.check_hazards = mode, check_hazards
        self.races = []      # lazy mode: (read pc, reading wave, DMA issue pc, issuing wave) of stale LDS reads
        lines = asm_text.split('\n')
        start = next(i for i, ln in enumerate(lines) if re.match(r'^fa_fwd_\w+:$', ln))
        end = next(i for i, ln in enumerate(lines) if ln.startswith('.Lfunc_end'))
        self.prog, self.labels = [], {}
        for ln in lines[start + 1:end]:
            ln = ln.split(';')[0].strip()
            if not ln or ln.startswith('.p2align') or ln.startswith('.size'):
                continue
            if ln.endswith(':'):
                self.labels[ln[:-1]] = len(self.prog)
                continue
            op, _, rest = ln.partition(' ')
            args = [x.strip() for x in self._split(rest)] if rest else []
            self.prog.append((op, args))
        m = re.search(r'\.amdhsa_accum_offset (\d+)', asm_text)
        self.nv = int(m.group(1))
        self.lds_bytes = int(re.search(r'\.amdhsa_group_segment_fixed_size (\d+)', asm_text).group(1))
        self.nwaves = int(re.search(r'\.max_flat_workgroup_size: (\d+)', asm_text).group(1)) // 64
        self.count = {}

    @staticmethod
    def _split(rest):
        out, depth, cur = [], 0, ''
        for ch in rest:
            if ch == '[':
                depth += 1
            elif ch == ']':
                depth -= 1
            if ch == ',' and depth == 0:
                out.append(cur)
                cur = ''
            else:
                cur += ch
        out.append(cur)
        # trailing modifiers separated by spaces ("0 offen lds", "v4 offset:8192")
        res = []
        for x in out:
            parts = x.strip().split()
            res.extend(parts)
        return res

    # ---------------------------------------------------------------- operand access
    def regs(self, w, name):
        """(file, start, count) of a register operand."""
        m = _RANGE.match(name)
        if m:
            f, lo, hi = m.group(1), int(m.group(2)), int(m.group(3))
            return f, lo, hi - lo + 1
        m = _ONE.match(name)
        if m:
            return m.group(1), int(m.group(2)), 1
        raise ValueError(name)

    def vread(self, w, name):
        """32-bit per-lane value of a VALU source operand (uint32[64])."""
        neg = False
        if name.startswith('-'):
            neg, name = True, name[1:]
        if name == 'vcc':
            raise ValueError('vcc as data')
        m = _ONE.match(name)
        if m:
            f, i = m.group(1), int(m.group(2))
            if f == 'v':
                val = w.v[i].copy()
            elif f == 'a':
                val = w.a[i].copy()
            else:
                val = np.full(64, int(w.s[i]) & 0xFFFFFFFF, dtype=np.uint32)
        else:
            val = np.full(64, self.const(name), dtype=np.uint32)
        if neg:
            val = (val ^ np.uint32(0x80000000)).astype(np.uint32)
        return val

    def fread(self, w, name):
        return self.vread(w, name).view(np.float32)

    @staticmethod
    def const(tok):
        if re.match(r'^-?\d+\.\d+$', tok):
            return struct.unpack('<I', struct.pack('<f', float(tok)))[0]
        v = int(tok, 0)
        return v & 0xFFFFFFFF

    def vwrite(self, w, name, val):
        f, i, n = self.regs(w, name)
        val = np.asarray(val)
        if val.dtype != np.uint32:
            val = val.astype(np.float32).view(np.uint32) if val.dtype.kind == 'f' else val.astype(np.uint32)
        if f == 'v':
            w.v[i] = val
        elif f == 'a':
            w.a[i] = val
        else:
            raise ValueError(name)

    def sread(self, w, tok):
        m = _ONE.match(tok)
        if m and m.group(1) == 's':
            return int(w.s[int(m.group(2))]) & 0xFFFFFFFF
        if tok == 'm0':
            return w.m0
        if tok == 'scc':
            return int(w.scc)
        return self.const(tok)

    def swrite(self, w, tok, val):
        if tok == 'm0':
            w.m0 = val & 0xFFFFFFFF
            return
        m = _ONE.match(tok)
        w.s[int(m.group(2))] = val & 0xFFFFFFFF

    def block(self, w, name):
        """(n x 64) uint32 block of a register range."""
        f, i, n = self.regs(w, name)
        src = w.v if f == 'v' else w.a
        return src[i:i + n]

    # ---------------------------------------------------------------- run
    def run(self, grid, karg, mem, max_steps=50_000_000):
        gx, gy, gz = grid
        for z in range(gz):
            for y in range(gy):
                for x in range(gx):
                    self.run_wg((x, y, z), karg, mem, max_steps)

    def run_wg(self, wg, karg, mem, max_steps):
        self.mem, self.karg = mem, karg
        self.lds = np.zeros(self.lds_bytes, dtype=np.uint8)
        self.lds_pend = np.full(self.lds_bytes, -1, dtype=np.int64)   # lazy: issue pc * 16 + wave of a pending DMA
        waves = [Wave(self.nv, 256, i, wg) for i in range(self.nwaves)]
        for i, w in enumerate(waves):
            w.id = i
        for w in waves:
            w.s[0] = karg & 0xFFFFFFFF
            w.s[1] = karg >> 32
        steps = 0
        nbar = [0] * len(waves)
        while not all(w.done for w in waves):
            for w in waves:
                while not w.done:
                    op, args = self.prog[w.pc]
                    w.pc += 1
                    steps += 1
                    if steps > max_steps:
                        raise RuntimeError('step limit')
                    self.count[op] = self.count.get(op, 0) + 1
                    if op == 's_barrier':
                        nbar[w.id] += 1
                        break
                    self.exec(w, op, args)
        # every wave of the workgroup must pass the same number of barriers (a wave-dependent branch
        # around a barrier desynchronises the hardware's barrier counting)
        if len(set(nbar)) != 1:
            raise HazardError(f'workgroup {wg}: waves passed different numbers of barriers {nbar}')

    # ---------------------------------------------------------------- semantics
    # ---------------------------------------------------------------- completion queues / hazards
    def _defer(self, w, q, fn, dst=None):
        """Queue a completion; dst: destination register operand (lazy mode tracks it as pending)."""
        if self.mode == 'eager':
            fn()
            return
        regs = self._reg_list(dst) if dst else []
        pc = w.pc - 1
        for r in regs:
            w.pend[r] = pc

        def run(fn=fn, regs=regs, pc=pc):
            fn()
            for r in regs:
                if w.pend.get(r) == pc:
                    del w.pend[r]
        q.append(run)

    @staticmethod
    def _drain(q, n):
        while len(q) > n:
            q.pop(0)()

    def _reg_list(self, name):
        m = _RANGE.match(name) or _ONE.match(name)
        if not m or m.group(1) not in ('v', 'a'):
            return []
        f, lo = m.group(1), int(m.group(2))
        hi = int(m.group(3)) if m.lastindex == 3 else lo
        return [(f, i) for i in range(lo, hi + 1)]

    def _hazard(self, w, op, a):
        """Check the operand reads of `op` against their writers, then record its writes."""
        if op.startswith('v_mfma'):
            rk = 'mfma'
            reads = [(x, 'ab') for x in a[1:3]] + ([(a[3], 'c')] if a[3] != '0' else [])
            dst = a[0]
        elif op in ('v_readfirstlane_b32', 'v_readlane_b32'):
            rk, reads, dst = 'rfl', [(a[1], None)], None
        elif op.startswith('v_permlane'):
            rk, reads, dst = 'perm', [(a[0], None), (a[1], None)], a[0]
        elif op.startswith('v_cmp'):
            rk, reads, dst = 'valu', [(x, None) for x in a[1:]], None
        elif op.startswith('v_'):
            rk = 'trans' if op in _TRANS else 'valu'
            reads, dst = [(x.lstrip('-'), None) for x in a[1:]], a[0]
        else:
            return
        for name, role in reads:
            for reg in self._reg_list(name):
                if reg not in w.wr:
                    continue
                st, wk, wdst = w.wr[reg]
                if wk.startswith('mfma'):
                    if rk == 'mfma' and role == 'c' and wdst == a[0]:
                        continue            # same-accumulator chain
                    need = _NEED[(wk, None)]
                else:
                    need = _NEED.get((wk, rk), 1)
                if w.state - st + 1 < need:
                    raise HazardError(f'{op} {",".join(a)} reads {reg[0]}{reg[1]} {w.state - st + 1} states after '
                                      f'its {wk} writer (needs {need}) at pc {w.pc - 1}')
        if dst is not None:
            wk = ('mfma32' if '32x32' in op else 'mfma16') if rk == 'mfma' else ('trans' if rk == 'trans' else 'valu')
            for reg in self._reg_list(dst):
                w.wr[reg] = (w.state + 1, wk, dst)

    def exec(self, w, op, a):
        if op == 's_nop':
            w.state += int(a[0], 0) + 1
            return
        if op == 's_waitcnt':
            for part in a:
                if part.startswith('vmcnt('):
                    self._drain(w.vmq, int(part[6:-1]))
                elif part.startswith('lgkmcnt('):
                    self._drain(w.lgq, int(part[8:-1]))
            return
        if w.pend:
            for x in a:
                for r in self._reg_list(x.lstrip('-')):
                    if r in w.pend:
                        self.races.append((w.pc - 1, w.id, w.pend[r], w.id))
                        break
        if self.check_hazards:
            self._hazard(w, op, a)
        w.state += 1
        if op == 's_setprio':
            return
        if op == 's_endpgm':
            self._drain(w.vmq, 0)
            self._drain(w.lgq, 0)
            w.done = True
            return
        if op == 's_branch':
            w.pc = self.labels[a[0]]
            return
        if op == 's_cbranch_scc1':
            if w.scc:
                w.pc = self.labels[a[0]]
            return
        if op == 's_cbranch_vccnz':
            if w.vcc.any():
                w.pc = self.labels[a[0]]
            return
        if op == 's_cbranch_vccz':
            if not w.vcc.any():
                w.pc = self.labels[a[0]]
            return
        if op.startswith('s_load_dword'):
            n = {'s_load_dword': 1, 's_load_dwordx2': 2, 's_load_dwordx4': 4, 's_load_dwordx16': 16}[op]
            f, i, cnt = self.regs(w, a[0])
            _, b, _ = self.regs(w, a[1])
            addr = (int(w.s[b]) | (int(w.s[b + 1]) << 32)) + int(a[2], 0)
            data = np.frombuffer(self.mem.read(addr, 4 * n).tobytes(), dtype=np.uint32).copy()

            def done(w=w, i=i, n=n, data=data):
                w.s[i:i + n] = data
            self._defer(w, w.lgq, done)
            return
        if op.startswith('s_'):
            return self.salu(w, op, a)
        if op.startswith('v_mfma'):
            return self.mfma(w, op, a)
        if op.startswith('ds_'):
            return self.ds(w, op, a)
        if op.startswith('buffer_'):
            return self.buf(w, op, a)
        if op == 'global_store_dword':
            _, i, _ = self.regs(w, a[0])
            addr = w.v[i].astype(np.uint64) | (w.v[i + 1].astype(np.uint64) << 32)
            off = self._offset(a)
            data = self.vread(w, a[1])
            for l in range(64):
                self.mem.write(int(addr[l]) + off, np.frombuffer(data[l:l + 1].tobytes(), dtype=np.uint8))
            self._defer(w, w.vmq, lambda: None)
            return
        return self.valu(w, op, a)

    def salu(self, w, op, a):
        d = a[0]
        if op == 's_cselect_b64':       # 64-bit lane mask (constants -1 / 0 or an SGPR pair)
            f, lo, n = self.regs(w, d)
            src = a[1] if w.scc else a[2]
            m = _RANGE.match(src)
            if m:
                v = [int(w.s[int(m.group(2))]), int(w.s[int(m.group(2)) + 1])]
            else:
                c = int(src, 0) & 0xFFFFFFFFFFFFFFFF
                v = [c & 0xFFFFFFFF, c >> 32]
            w.s[lo], w.s[lo + 1] = v[0] & 0xFFFFFFFF, v[1] & 0xFFFFFFFF
            return
        x = self.sread(w, a[1]) if len(a) > 1 else 0
        y = self.sread(w, a[2]) if len(a) > 2 else 0
        M = 0xFFFFFFFF
        if op == 's_mov_b32':
            r = x
        elif op == 's_add_u32':
            t = x + y
            w.scc = t > M
            r = t
        elif op == 's_addc_u32':
            t = x + y + int(w.scc)
            w.scc = t > M
            r = t
        elif op == 's_sub_u32':
            w.scc = y > x
            r = (x - y) & M
        elif op == 's_mul_i32':
            r = (x * y) & M
        elif op == 's_mul_hi_u32':
            r = (x * y) >> 32
        elif op == 's_or_b32':
            r = x | y
            w.scc = r != 0
        elif op == 's_and_b32':
            r = x & y
            w.scc = r != 0
        elif op == 's_lshr_b32':
            r = x >> (y & 31)
            w.scc = r != 0
        elif op == 's_lshl_b32':
            r = (x << (y & 31)) & M
            w.scc = r != 0
        elif op == 's_min_u32':
            r = min(x, y)
        elif op == 's_cselect_b32':
            r = x if w.scc else y
        elif op == 's_cmp_ge_u32':
            w.scc = self.sread(w, a[0]) >= x
            return
        elif op == 's_cmp_eq_u32':
            w.scc = self.sread(w, a[0]) == x
            return
        elif op == 's_cmp_lt_u32':
            w.scc = self.sread(w, a[0]) < x
            return
        elif op == 's_cmp_gt_u32':
            w.scc = self.sread(w, a[0]) > x
            return
        elif op == 's_cmp_lg_u32':
            w.scc = self.sread(w, a[0]) != x
            return
        else:
            raise NotImplementedError(op)
        self.swrite(w, d, r & M)

    def valu(self, w, op, a):
        U = np.uint32
        if op == 'v_readfirstlane_b32':
            self.swrite(w, a[0], int(self.vread(w, a[1])[0]))
            return
        if op == 'v_readlane_b32':
            self.swrite(w, a[0], int(self.vread(w, a[1])[self.sread(w, a[2]) & 63]))
            return
        if op == 'v_writelane_b32':
            d = self.vread(w, a[0])
            d[self.sread(w, a[2]) & 63] = self.sread(w, a[1])
            self.vwrite(w, a[0], d)
            return
        if op.startswith('v_cmp_'):
            kind = op[6:]
            if kind.endswith('_e32'):
                kind = kind[:-4]
            x, y = a[1], a[2]
            if kind.endswith('f32'):
                p, q = self.fread(w, x), self.fread(w, y)
                c = kind[:-4]
                res = {'gt': p > q, 'lt': p < q, 'nlg': ~((p < q) | (p > q))}[c]
            elif kind.endswith('i32'):
                p, q = self.vread(w, x).view(np.int32), self.vread(w, y).view(np.int32)
                res = {'lt': p < q, 'gt': p > q, 'eq': p == q}[kind[:-4]]
            else:
                p, q = self.vread(w, x), self.vread(w, y)
                res = {'gt': p > q, 'eq': p == q, 'lt': p < q, 'ne': p != q}[kind[:-4]]
            w.vcc = np.asarray(res, dtype=bool)
            return
        if op == 'v_pk_mul_f32':      # 64-bit operands: two fp32 lanes, default op_sel
            halves = lambda tok: (lambda f, lo, n: [f'{f}{lo}', f'{f}{lo + 1}'])(*self.regs(w, tok))
            (d0, d1), (x0, x1), (y0, y1) = halves(a[0]), halves(a[1]), halves(a[2])
            with np.errstate(all='ignore'):
                r0 = (self.fread(w, x0) * self.fread(w, y0)).astype(np.float32)
                r1 = (self.fread(w, x1) * self.fread(w, y1)).astype(np.float32)
            self.vwrite(w, d0, r0.view(U))
            self.vwrite(w, d1, r1.view(U))
            return
        if op == 'v_cndmask_b32':
            s0, s1 = self.vread(w, a[1]), self.vread(w, a[2])
            mask = w.vcc
            if len(a) > 3 and a[3] != 'vcc':    # SGPR-pair lane mask
                _, lo, _ = self.regs(w, a[3])
                bits = int(w.s[lo]) | (int(w.s[lo + 1]) << 32)
                mask = np.array([(bits >> l) & 1 for l in range(64)], dtype=bool)
            self.vwrite(w, a[0], np.where(mask, s1, s0).astype(U))
            return
        if op == 'v_permlane32_swap_b32':
            d, s = self.vread(w, a[0]), self.vread(w, a[1])
            nd, ns = d.copy(), s.copy()
            nd[32:] = s[:32]
            ns[:32] = d[32:]
            self.vwrite(w, a[0], nd)
            self.vwrite(w, a[1], ns)
            return
        if op == 'v_accvgpr_write_b32' or op == 'v_accvgpr_read_b32' or op == 'v_mov_b32':
            self.vwrite(w, a[0], self.vread(w, a[1]))
            return
        if op in ('v_cvt_pk_bf16_f32', 'v_cvt_pk_f16_f32'):
            cv = bf16_bits if op == 'v_cvt_pk_bf16_f32' else f16_bits
            lo, hi = cv(self.fread(w, a[1])), cv(self.fread(w, a[2]))
            self.vwrite(w, a[0], (lo | (hi << 16)).astype(U))
            return
        if op in ('v_add_co_u32', 'v_addc_co_u32'):
            x, y = self.vread(w, a[2]).astype(np.uint64), self.vread(w, a[3]).astype(np.uint64)
            t = x + y + (w.vcc.astype(np.uint64) if op == 'v_addc_co_u32' else 0)
            w.vcc = t > 0xFFFFFFFF
            self.vwrite(w, a[0], (t & 0xFFFFFFFF).astype(U))
            return
        if op == 'v_bitop3_b32':
            # D = BITOP3(S0, S1, S2, table): bit i of the table is the result for the source bits
            # (S0 << 2) | (S1 << 1) | S2 = i (LLVM's encoding: (a | b) & c with S0 = a, S1 = b, S2 = c is 0xa8)
            x0, x1, x2 = (self.vread(w, x) for x in a[1:4])
            tbl = int(a[4].split(':')[1], 0)
            r = np.zeros(64, dtype=U)
            for i in range(8):
                if tbl >> i & 1:
                    r |= (x0 if i & 4 else ~x0) & (x1 if i & 2 else ~x1) & (x2 if i & 1 else ~x2)
            self.vwrite(w, a[0], r.astype(U))
            return
        src = [self.vread(w, x) for x in a[1:]]
        f = [s.view(np.float32) for s in src]
        with np.errstate(all='ignore'):
            if op == 'v_lshrrev_b32':
                r = src[1] >> (src[0] & 31)
            elif op == 'v_lshlrev_b32':
                r = src[1] << (src[0] & 31)
            elif op == 'v_and_b32':
                r = src[0] & src[1]
            elif op == 'v_or_b32':
                r = src[0] | src[1]
            elif op == 'v_or3_b32':
                r = src[0] | src[1] | src[2]
            elif op == 'v_and_or_b32':
                r = (src[0] & src[1]) | src[2]
            elif op == 'v_xor_b32':
                r = src[0] ^ src[1]
            elif op == 'v_bfe_u32':
                r = (src[0] >> (src[1] & 31)) & ((np.uint64(1) << src[2].astype(np.uint64)) - 1).astype(U)
            elif op == 'v_add_u32':
                r = (src[0].astype(np.uint64) + src[1]).astype(np.uint64) & 0xFFFFFFFF
            elif op == 'v_sub_u32':
                r = (src[0].astype(np.int64) - src[1].astype(np.int64)) & 0xFFFFFFFF
            elif op == 'v_subrev_u32':
                r = (src[1].astype(np.int64) - src[0].astype(np.int64)) & 0xFFFFFFFF
            elif op == 'v_min_u32':
                r = np.minimum(src[0], src[1])
            elif op == 'v_min_i32':
                r = np.minimum(src[0].view(np.int32), src[1].view(np.int32)).view(U)
            elif op == 'v_lshl_add_u32':
                r = ((src[0].astype(np.uint64) << src[1].astype(np.uint64)) + src[2]) & 0xFFFFFFFF
            elif op == 'v_lshl_or_b32':
                r = ((src[0].astype(np.uint64) << src[1].astype(np.uint64)) | src[2]) & 0xFFFFFFFF
            elif op == 'v_mul_lo_u32':
                r = (src[0].astype(np.uint64) * src[1].astype(np.uint64)) & 0xFFFFFFFF
            elif op == 'v_max3_f32':
                r = np.maximum(np.maximum(f[0], f[1]), f[2])
            elif op == 'v_max_f32':
                r = np.maximum(f[0], f[1])
            elif op == 'v_fma_f32':
                r = (f[0].astype(np.float64) * f[1] + f[2]).astype(np.float32)
            elif op == 'v_mul_f32':
                r = (f[0] * f[1]).astype(np.float32)
            elif op == 'v_add_f32':
                r = (f[0] + f[1]).astype(np.float32)
            elif op == 'v_sub_f32':
                r = (f[0] - f[1]).astype(np.float32)
            elif op == 'v_cvt_f32_f16':
                r = (src[0] & 0xFFFF).astype(np.uint16).view(np.float16).astype(np.float32)
            elif op == 'v_exp_f32':
                r = np.exp2(f[0]).astype(np.float32)
            elif op == 'v_log_f32':
                r = np.log2(f[0]).astype(np.float32)
            elif op == 'v_rcp_f32':
                r = (np.float32(1.0) / f[0]).astype(np.float32)
            else:
                raise NotImplementedError(op)
        r = np.asarray(r)
        if r.dtype.kind == 'f':
            r = r.astype(np.float32).view(U)
        self.vwrite(w, a[0], r.astype(U))

    def mfma(self, w, op, a):
        dt = 'bf16' if op.endswith('bf16') else 'f16'
        big = '32x32x16' in op
        A = self.block(w, a[1])
        B = self.block(w, a[2])
        lane = np.arange(64)

        def unpack(blk):   # (4, 64) regs -> (64, 8) fp32 elements
            e = np.zeros((64, 8), dtype=np.float32)
            for r in range(4):
                e[:, 2 * r] = from16(blk[r] & 0xFFFF, dt)
                e[:, 2 * r + 1] = from16(blk[r] >> 16, dt)
            return e
        ea, eb = unpack(A), unpack(B)
        if big:
            Am = np.zeros((32, 16), dtype=np.float64)
            Bm = np.zeros((16, 32), dtype=np.float64)
            for j in range(8):
                Am[lane & 31, 8 * (lane >> 5) + j] = ea[:, j]
                Bm[8 * (lane >> 5) + j, lane & 31] = eb[:, j]
            n = 16
            rows = lambda r: (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
            cols = lane & 31
        else:
            Am = np.zeros((16, 32), dtype=np.float64)
            Bm = np.zeros((32, 16), dtype=np.float64)
            for j in range(8):
                Am[lane & 15, 8 * (lane >> 4) + j] = ea[:, j]
                Bm[8 * (lane >> 4) + j, lane & 15] = eb[:, j]
            n = 4
            rows = lambda r: 4 * (lane >> 4) + r
            cols = lane & 15
        Cm = Am @ Bm
        if a[3] == '0':
            Cin = np.zeros((n, 64), dtype=np.float32)
        else:
            Cin = self.block(w, a[3]).view(np.float32)
        out = np.zeros((n, 64), dtype=np.float32)
        for r in range(n):
            out[r] = (Cin[r].astype(np.float64) + Cm[rows(r), cols]).astype(np.float32)
        f, i, cnt = self.regs(w, a[0])
        dst = w.v if f == 'v' else w.a
        dst[i:i + cnt] = out.view(np.uint32)

    def _offset(self, a):
        for x in a:
            if x.startswith('offset:'):
                return int(x[7:])
        return 0

    def ds(self, w, op, a):
        off = self._offset(a)
        if op == 'ds_bpermute_b32':
            addr = self.vread(w, a[1])
            src = self.vread(w, a[2])
            val = src[(addr // 4) % 64].copy()
            self._defer(w, w.lgq, lambda w=w, d=a[0], val=val: self.vwrite(w, d, val), a[0])
            return
        addr = self.vread(w, a[1]).astype(np.int64) + off
        f, i, cnt = self.regs(w, a[0])
        dst = w.v if f == 'v' else w.a
        if self.mode == 'lazy':
            span = 16 if op == 'ds_read_b128' else 8
            for l in range(64):
                p = self.lds_pend[addr[l]:addr[l] + span]
                if (p >= 0).any():
                    q = int(p[p >= 0][0])
                    self.races.append((w.pc - 1, w.id, q // 16, q % 16))
                    break
        if op == 'ds_read_b128':
            out = np.zeros((4, 64), dtype=np.uint32)
            for l in range(64):
                b = self.lds[addr[l]:addr[l] + 16]
                out[:, l] = np.frombuffer(b.tobytes(), dtype=np.uint32)

            def done(dst=dst, i=i, out=out):
                dst[i:i + 4] = out
            self._defer(w, w.lgq, done, a[0])
            return
        if op == 'ds_read_b64_tr_b16':
            out = np.zeros((2, 64), dtype=np.uint32)
            for g in range(4):
                for li in range(16):
                    vals = []
                    for q in range(4):
                        src = 16 * g + 4 * q + li // 4
                        b = self.lds[addr[src] + 2 * (li % 4): addr[src] + 2 * (li % 4) + 2]
                        vals.append(int(b[0]) | (int(b[1]) << 8))
                    out[0, 16 * g + li] = vals[0] | (vals[1] << 16)
                    out[1, 16 * g + li] = vals[2] | (vals[3] << 16)

            def done(dst=dst, i=i, out=out):
                dst[i:i + 2] = out
            self._defer(w, w.lgq, done, a[0])
            return
        raise NotImplementedError(op)

    def buf(self, w, op, a):
        off = self._offset(a)
        if op.startswith('buffer_load'):
            lds = 'lds' in a
            if lds:
                vo, srd, so = a[0], a[1], a[2]
            else:
                dst, vo, srd, so = a[0], a[1], a[2], a[3]
        else:
            src, vo, srd, so = a[0], a[1], a[2], a[3]
        _, d0, _ = self.regs(w, srd)
        base = int(w.s[d0]) | ((int(w.s[d0 + 1]) & 0xFFFF) << 32)
        nrec = int(w.s[d0 + 2])
        voff = self.vread(w, vo).astype(np.int64)
        soff = self.sread(w, so)
        n = {'buffer_load_dwordx4': 16, 'buffer_store_dwordx4': 16, 'buffer_store_dword': 4}[op]
        chk = voff + off + (soff if self.soff_checked else 0)
        ok = (voff & 0x80000000) == 0
        ok &= chk + n <= nrec
        addr = base + voff + off + soff
        if op == 'buffer_load_dwordx4':
            data = [self.mem.read(int(addr[l]), 16).copy() if ok[l] else np.zeros(16, dtype=np.uint8)
                    for l in range(64)]
            if lds:
                m0 = w.m0
                if self.mode == 'lazy':
                    self.lds_pend[m0:m0 + 1024] = (w.pc - 1) * 16 + w.id

                def done(m0=m0, data=data):
                    for l in range(64):
                        self.lds[m0 + 16 * l:m0 + 16 * l + 16] = data[l]
                    self.lds_pend[m0:m0 + 1024] = -1
            else:
                f, i, cnt = self.regs(w, dst)
                tgt = w.v if f == 'v' else w.a

                def done(tgt=tgt, i=i, data=data):
                    for l in range(64):
                        tgt[i:i + 4, l] = np.frombuffer(data[l].tobytes(), dtype=np.uint32)
            self._defer(w, w.vmq, done, None if lds else dst)
            return
        f, i, cnt = self.regs(w, src)
        srcr = w.v if f == 'v' else w.a
        for l in range(64):
            if ok[l]:
                words = srcr[i:i + n // 4, l].astype(np.uint32)
                self.mem.write(int(addr[l]), np.frombuffer(words.tobytes(), dtype=np.uint8))
        self._defer(w, w.vmq, lambda: None)     # stores count in vmcnt (applied at issue)
