#!/usr/bin/env python3
"""Small functional emulator of gfx950 wave64 execution for the instruction subset of the generated
asm bodies (tools/gen_tw_kernel.py transforms, tools/gen_pbs_kernel.py blind rotation).  Checks the
data path's logic on the CPU — not hazards or timing, which only the GPU run can.  Several waves of
one workgroup share LDS and run round-robin between s_barrier instructions.

  python tools/asm_emu.py            # runs the transform bodies on one random polynomial vs the oracle
"""
import os
import re
import sys

import numpy as np

M32 = np.uint64(0xFFFFFFFF)
LANES = 64
SH = np.arange(32, dtype=np.uint64)


def _bits(word):
    w = np.array([word & 0xFFFFFFFF, word >> 32], dtype=np.uint64)
    return np.concatenate([((w[0] >> SH) & np.uint64(1)), ((w[1] >> SH) & np.uint64(1))]).astype(bool)


def _word(m):
    b = m.astype(np.uint64)
    return int((b[:32] << SH).sum()) | (int((b[32:] << SH).sum()) << 32)


class Wave:
    def __init__(self, ops, mem, lds=None, lds_bytes=65536):
        self.v = np.zeros((256, LANES), dtype=np.uint64)   # 32-bit values kept in uint64
        self.s = np.zeros(128, dtype=np.uint64)
        self.exec = np.ones(LANES, dtype=bool)
        self.lds = lds if lds is not None else np.zeros(lds_bytes // 8, dtype=np.uint64)
        self.mem = mem          # dict base_address -> np.uint64 array (global memory regions)
        self.ops = ops          # operand name -> text
        self.scc = 0

    # ---- operand parsing ----------------------------------------------------------------------
    @staticmethod
    def vreg(tok):
        m = re.fullmatch(r"v(\d+)", tok)
        return int(m.group(1)) if m else None

    @staticmethod
    def vpair(tok):
        m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
        return int(m.group(1)) if m else None

    @staticmethod
    def spair(tok):
        m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
        return int(m.group(1)) if m else None

    VCC = 106  # vcc_lo / vcc_hi are s106 / s107

    def mask(self, tok):
        b = self.VCC if tok == "vcc" else self.spair(tok)
        if b is None:
            raise ValueError(tok)
        return _bits(int(self.s[b]) | (int(self.s[b + 1]) << 32))

    def set_mask(self, tok, m):
        m = m & self.exec  # a VALU lane-mask write clears the bits of inactive lanes
        word = _word(m)
        b = self.spair(tok)
        self.s[b] = np.uint64(word & 0xFFFFFFFF)
        self.s[b + 1] = np.uint64(word >> 32)

    def src32(self, tok):
        r = self.vreg(tok)
        if r is not None:
            return self.v[r].copy()
        m = re.fullmatch(r"s(\d+)", tok)
        if m:
            return np.full(LANES, self.s[int(m.group(1))], dtype=np.uint64)
        return np.full(LANES, np.uint64(int(tok, 0) & 0xFFFFFFFF), dtype=np.uint64)

    def src64(self, tok):
        b = self.vpair(tok)
        if b is not None:
            return self.v[b] | (self.v[b + 1] << np.uint64(32))
        sb = self.spair(tok)
        if sb is not None:
            return np.full(LANES, self.s[sb] | (self.s[sb + 1] << np.uint64(32)), dtype=np.uint64)
        return np.full(LANES, np.uint64(int(tok, 0) & 0xFFFFFFFFFFFFFFFF), dtype=np.uint64)

    def wv(self, r, val):
        self.v[r] = np.where(self.exec, val & M32, self.v[r])

    def wv64(self, b, val):
        self.wv(b, val & M32)
        self.wv(b + 1, val >> np.uint64(32))

    # ---- execution ------------------------------------------------------------------------------
    def load(self, lines):
        self.prog, self.labels = [], {}
        for line in lines:
            line = line.strip()
            for k, v in self.ops.items():
                line = line.replace(f"%[{k}]", v)
            line = line.replace("%=", "0")
            if not line or line.startswith("s_nop") or line.startswith("s_waitcnt"):
                continue
            if line.endswith(":"):
                self.labels[line[:-1]] = len(self.prog)
                continue
            mn, _, rest = line.partition(" ")
            args = [a.strip() for a in re.split(r",(?![^\[]*\])", rest)] if rest else []
            fn = getattr(self, "op_" + mn, None)
            if fn is None:
                raise NotImplementedError(mn)
            self.prog.append((fn, args, mn))
        self.pc = 0

    def steps(self):
        """Generator: runs to the end, yielding at every s_barrier."""
        while self.pc < len(self.prog):
            fn, args, mn = self.prog[self.pc]
            self.pc += 1
            if mn == "s_barrier":
                yield
                continue
            fn(args)

    def run(self, lines):
        self.load(lines)
        for _ in self.steps():
            pass

    # VALU
    def op_v_mov_b32(self, a):
        self.wv(self.vreg(a[0]), self.src32(a[1]))

    def op_v_mov_b64(self, a):
        self.wv64(self.vpair(a[0]), self.src64(a[1]))

    def op_v_mov_b32_dpp(self, a):
        src = self.src32(a[1].split()[0])
        perm = [int(x) for x in re.search(r"quad_perm:\[(.*?)\]", a[1]).group(1).split(",")]
        idx = np.array([(l & ~3) + perm[l & 3] for l in range(LANES)])
        self.wv(self.vreg(a[0]), src[idx])

    def op_v_lshlrev_b32(self, a):
        self.wv(self.vreg(a[0]), (self.src32(a[2]) << (self.src32(a[1]) & np.uint64(31))) & M32)

    def op_v_lshrrev_b32(self, a):
        self.wv(self.vreg(a[0]), self.src32(a[2]) >> (self.src32(a[1]) & np.uint64(31)))

    def op_v_ashrrev_i32(self, a):
        x = self.src32(a[2]).astype(np.int64)
        x = np.where(x >= 2 ** 31, x - 2 ** 32, x)
        self.wv(self.vreg(a[0]), (x >> (self.src32(a[1]).astype(np.int64) & 31)).astype(np.uint64) & M32)

    def op_v_lshlrev_b64(self, a):
        self.wv64(self.vpair(a[0]), self.src64(a[2]) << (self.src32(a[1]) & np.uint64(63)))

    def op_v_lshrrev_b64(self, a):
        self.wv64(self.vpair(a[0]), self.src64(a[2]) >> (self.src32(a[1]) & np.uint64(63)))

    def op_v_add_u32(self, a):
        self.wv(self.vreg(a[0]), (self.src32(a[1]) + self.src32(a[2])) & M32)

    def op_v_subrev_u32(self, a):
        self.wv(self.vreg(a[0]), (self.src32(a[2]) - self.src32(a[1])) & M32)

    def op_v_and_b32(self, a):
        self.wv(self.vreg(a[0]), self.src32(a[1]) & self.src32(a[2]))

    def op_v_or_b32(self, a):
        self.wv(self.vreg(a[0]), self.src32(a[1]) | self.src32(a[2]))

    def op_v_xor_b32(self, a):
        self.wv(self.vreg(a[0]), self.src32(a[1]) ^ self.src32(a[2]))

    def op_v_mul_u32_u24(self, a):
        x, y = self.src32(a[1]) & np.uint64(0xFFFFFF), self.src32(a[2]) & np.uint64(0xFFFFFF)
        self.wv(self.vreg(a[0]), (x * y) & M32)

    def op_v_bfe_u32(self, a):
        x, off, w = self.src32(a[1]), self.src32(a[2]) & np.uint64(31), self.src32(a[3]) & np.uint64(31)
        self.wv(self.vreg(a[0]), (x >> off) & ((np.uint64(1) << w) - np.uint64(1)))

    def op_v_bfe_i32(self, a):
        x, off, w = self.src32(a[1]), self.src32(a[2]) & np.uint64(31), self.src32(a[3]) & np.uint64(31)
        f = ((x >> off) & ((np.uint64(1) << w) - np.uint64(1))).astype(np.int64)
        sign = (f >> (w.astype(np.int64) - 1)) & 1
        f = np.where((w > 0) & (sign == 1), f - (np.int64(1) << w.astype(np.int64)), f)
        self.wv(self.vreg(a[0]), f.astype(np.uint64) & M32)

    def op_v_sub_u32(self, a):
        self.wv(self.vreg(a[0]), (self.src32(a[1]) - self.src32(a[2])) & M32)

    def op_v_cmp_ge_u64_e64(self, a):
        self.set_mask(a[0], self.src64(a[1]) >= self.src64(a[2]))

    def op_v_bfi_b32(self, a):
        m = self.src32(a[1])
        self.wv(self.vreg(a[0]), (m & self.src32(a[2])) | (~m & M32 & self.src32(a[3])))

    def op_v_cmp_eq_u32_e64(self, a):
        self.set_mask(a[0], self.src32(a[1]) == self.src32(a[2]))

    def op_v_cmp_le_u32_e64(self, a):
        self.set_mask(a[0], self.src32(a[1]) <= self.src32(a[2]))

    def op_v_mad_u64_u32(self, a):
        x, y, z = self.src32(a[2]), self.src32(a[3]), self.src64(a[4])
        prod = x * y
        s = prod + z
        self.wv64(self.vpair(a[0]), s)
        self.set_mask(a[1], s < z)

    def op_v_mad_i64_i32(self, a):
        x, y = self.src32(a[2]).astype(np.int64), self.src32(a[3]).astype(np.int64)
        x = np.where(x >= 2 ** 31, x - 2 ** 32, x)
        y = np.where(y >= 2 ** 31, y - 2 ** 32, y)
        prod = (x * y).astype(np.uint64)          # |x y| < 2^62: exact, then two's complement
        self.wv64(self.vpair(a[0]), prod + self.src64(a[4]))
        self.set_mask(a[1], np.zeros(LANES, dtype=bool))  # overflow flag: unused (junk destination)

    def _carry_op(self, a, fn):
        x, y = self.src32(a[2]).astype(np.int64), self.src32(a[3]).astype(np.int64)
        cin = self.mask(a[4]).astype(np.int64) if len(a) > 4 else np.zeros(LANES, dtype=np.int64)
        res, co = fn(x, y, cin)
        self.wv(self.vreg(a[0]), res.astype(np.uint64) & M32)
        self.set_mask(a[1], co)

    def op_v_add_co_u32_e64(self, a):
        self._carry_op(a, lambda x, y, c: (x + y, (x + y) >> 32 != 0))

    def op_v_addc_co_u32_e64(self, a):
        self._carry_op(a, lambda x, y, c: (x + y + c, (x + y + c) >> 32 != 0))

    def op_v_sub_co_u32_e64(self, a):
        self._carry_op(a, lambda x, y, c: ((x - y) & 0xFFFFFFFF, x - y < 0))

    def op_v_subb_co_u32_e64(self, a):
        self._carry_op(a, lambda x, y, c: ((x - y - c) & 0xFFFFFFFF, x - y - c < 0))

    def op_v_cndmask_b32_dpp(self, a):
        # VOP2 select with a DPP source: D = VCC ? src1 : dpp(src0); a[3] = "vcc quad_perm:[...] ..."
        src = self.src32(a[1])
        perm = [int(x) for x in re.search(r"quad_perm:\[(.*?)\]", a[3]).group(1).split(",")]
        idx = np.array([(l & ~3) + perm[l & 3] for l in range(LANES)])
        self.wv(self.vreg(a[0]), np.where(self.mask("vcc"), self.src32(a[2]), src[idx]))

    def op_v_permlane32_swap_b32(self, a):
        # half-wave exchange: lanes 32-63 of vdst <-> lanes 0-31 of vsrc (whole registers, EXEC all ones)
        d, s_ = self.vreg(a[0]), self.vreg(a[1])
        lo = self.v[s_][:32].copy()
        self.v[s_][:32] = self.v[d][32:]
        self.v[d][32:] = lo

    def op_v_cndmask_b32_e64(self, a):
        m = self.mask(a[3])
        self.wv(self.vreg(a[0]), np.where(m, self.src32(a[2]), self.src32(a[1])))

    # SALU
    def s_src(self, tok):
        m = re.fullmatch(r"s(\d+)", tok)
        if m:
            return int(self.s[int(m.group(1))])
        return int(tok, 0) & 0xFFFFFFFF

    def s_set(self, tok, val):
        self.s[int(tok[1:])] = np.uint64(val & 0xFFFFFFFF)

    def op_s_mov_b32(self, a):
        val = self.s_src(a[1])
        if a[0] == "exec_lo":
            self.exec[:32] = _bits(val)[:32]
        elif a[0] == "exec_hi":
            self.exec[32:] = _bits(val)[:32]
        else:
            self.s_set(a[0], val)

    def op_s_mov_b64(self, a):
        if a[0] == "vcc":
            v = int(a[1], 0) if not a[1].startswith("s[") else (int(self.s[self.spair(a[1])]) |
                                                                 (int(self.s[self.spair(a[1]) + 1]) << 32))
            self.s[self.VCC], self.s[self.VCC + 1] = np.uint64(v & 0xFFFFFFFF), np.uint64((v >> 32) & 0xFFFFFFFF)
        elif a[1] == "exec":
            word = _word(self.exec)
            b = self.spair(a[0])
            self.s[b], self.s[b + 1] = np.uint64(word & 0xFFFFFFFF), np.uint64(word >> 32)
        elif a[0] == "exec":
            self.exec = self.mask(a[1])
        else:
            raise NotImplementedError(a)

    def _set_exec_or(self, a, m):
        """SALU write of EXEC (the EXEC-masked arithmetic of gen_tw_kernel); True when a[0] is exec."""
        if a[0] != "exec":
            return False
        self.exec = m
        self.scc = int(m.any())
        return True

    def op_s_not_b64(self, a):
        if self._set_exec_or(a, ~self.mask(a[1])):
            return
        word = _word(~self.mask(a[1]))
        b = self.VCC if a[0] == "vcc" else self.spair(a[0])
        self.s[b], self.s[b + 1] = np.uint64(word & 0xFFFFFFFF), np.uint64(word >> 32)
        self.scc = int(word != 0)

    def op_s_or_b64(self, a):
        if self._set_exec_or(a, self.mask(a[1]) | self.mask(a[2])):
            return
        word = _word(self.mask(a[1]) | self.mask(a[2]))
        b = self.spair(a[0])
        self.s[b], self.s[b + 1] = np.uint64(word & 0xFFFFFFFF), np.uint64(word >> 32)
        self.scc = int(word != 0)

    def op_s_andn2_b64(self, a):
        word = _word(self.mask(a[1]) & ~self.mask(a[2]))
        b = self.spair(a[0])
        self.s[b], self.s[b + 1] = np.uint64(word & 0xFFFFFFFF), np.uint64(word >> 32)
        self.scc = int(word != 0)

    def op_s_add_u32(self, a):
        x = self.s_src(a[1]) + self.s_src(a[2])
        self.s_set(a[0], x)
        self.scc = x >> 32

    def op_s_addc_u32(self, a):
        x = self.s_src(a[1]) + self.s_src(a[2]) + self.scc
        self.s_set(a[0], x)
        self.scc = x >> 32

    def op_s_sub_u32(self, a):
        x = self.s_src(a[1]) - self.s_src(a[2])
        self.s_set(a[0], x)
        self.scc = int(x < 0)

    def op_s_and_b32(self, a):
        x = self.s_src(a[1]) & self.s_src(a[2])
        self.s_set(a[0], x)
        self.scc = int(x != 0)

    def op_s_lshl_b32(self, a):
        x = (self.s_src(a[1]) << (self.s_src(a[2]) & 31)) & 0xFFFFFFFF
        self.s_set(a[0], x)
        self.scc = int(x != 0)

    def op_s_lshr_b32(self, a):
        x = self.s_src(a[1]) >> (self.s_src(a[2]) & 31)
        self.s_set(a[0], x)
        self.scc = int(x != 0)

    def op_s_cmp_eq_u32(self, a):
        self.scc = int(self.s_src(a[0]) == self.s_src(a[1]))

    def op_s_cbranch_scc1(self, a):
        if self.scc:
            self.pc = self.labels[a[0]]

    def op_s_branch(self, a):
        self.pc = self.labels[a[0]]

    def op_s_barrier(self, a):
        pass

    def op_s_load_dwordx2(self, a):
        b = self.spair(a[1])
        addr = int(self.s[b]) | (int(self.s[b + 1]) << 32)
        arr, i = self._mem(addr + int(a[2], 0))
        val = int(arr[i])
        d = self.spair(a[0])
        self.s[d], self.s[d + 1] = np.uint64(val & 0xFFFFFFFF), np.uint64(val >> 32)

    # memory
    def _mem(self, addr):
        for base, arr in self.mem.items():
            if base <= addr < base + arr.size * 8:
                return arr, (addr - base) // 8
        raise IndexError(hex(addr))

    def _gaddr(self, voff, tok):
        parts = tok.split()
        off = int(parts[1].split(":")[1]) if len(parts) > 1 else 0
        b = self.spair(parts[0])
        base = int(self.s[b]) | (int(self.s[b + 1]) << 32)
        addrs = voff.astype(np.uint64) + np.uint64(base + off)
        lo = int(addrs[self.exec].min()) if self.exec.any() else base
        arr, i0 = self._mem(lo)
        region = lo - i0 * 8
        idx = ((addrs - np.uint64(region)) // np.uint64(8)).astype(np.int64)
        if self.exec.any() and int(idx[self.exec].max()) >= arr.size:
            raise IndexError("global access crosses a region")
        return arr, idx

    def op_global_load_dwordx2(self, a):
        arr, idx = self._gaddr(self.src32(a[1]), a[2])
        vals = np.where(self.exec, arr[np.where(self.exec, idx, 0)], np.uint64(0))
        self.wv64(self.vpair(a[0]), vals)

    def op_global_store_dwordx2(self, a):
        arr, idx = self._gaddr(self.src32(a[0]), a[2])
        vals = self.src64(a[1])
        arr[idx[self.exec]] = vals[self.exec]

    def op_ds_write_b64(self, a):
        parts = a[1].split()
        off = int(parts[1].split(":")[1]) if len(parts) > 1 else 0
        addr = (self.src32(a[0]) + np.uint64(off)).astype(np.int64)
        if (addr[self.exec] % 8).any():
            raise ValueError("unaligned ds_write_b64")
        self.lds[addr[self.exec] // 8] = self.src64(parts[0])[self.exec]

    def op_ds_read_b64(self, a):
        parts = a[1].split()
        off = int(parts[1].split(":")[1]) if len(parts) > 1 else 0
        addr = (self.src32(parts[0]) + np.uint64(off)).astype(np.int64)
        self.wv64(self.vpair(a[0]), self.lds[np.where(self.exec, addr, 0) // 8])


def body_lines(hdr, name, prefix="MI_TW_BODY_"):
    txt = open(hdr).read()
    start = txt.index(f"#define {prefix}{name.upper()}(")
    end = txt.index(":: __VA_ARGS__", start)
    return [m.group(1) for m in re.finditer(r'"(.*?)\\n"', txt[start:end])]


def run_body(hdr, name, poly, twist_tab, fwd=True, out_of_place=False, mem_extra=None, ops_extra=None, out_init=None,
             w1x=None):
    """Emulate one wave (wave 0 of a workgroup) of the transform body on one polynomial.  out_of_place: the body
    writes another buffer (%[o_lo] / %[o_hi], the key-conversion body), which is returned.  mem_extra / ops_extra:
    more memory regions (base address -> u64 array) and operand bindings (the MAC-fused inverse's term bases).
    out_init: the %[o_*] buffer's initial contents (the Ntt64View add_backward bodies read and write it); the call then
    returns (data, out).  w1x (default: the generator's FWD_W1X for forward bodies, i.e. names starting "fwd"): the
    forward's W1x lane-pair layout (lane = i + 32 j0) and its transpose addresses, as ntt64_tw_device.hpp computes them."""
    data = np.array(poly, dtype=np.uint64).copy()
    tw = np.array(twist_tab, dtype=np.uint64)
    GB, TB, OB = 0x100000000, 0x200000000, 0x300000000
    out = np.zeros_like(data) if out_init is None else np.array(out_init, dtype=np.uint64).copy()
    mem = {GB: data, TB: tw, OB: out}
    lane = np.arange(LANES, dtype=np.uint64)
    par, i = lane & np.uint64(1), lane >> np.uint64(1)
    S = 0
    ops = {"g_lo": f"{GB & 0xFFFFFFFF}", "g_hi": f"{GB >> 32}", "tw_lo": f"{TB & 0xFFFFFFFF}", "tw_hi": f"{TB >> 32}",
           "o_lo": f"{OB & 0xFFFFFFFF}", "o_hi": f"{OB >> 32}"}
    w = Wave(None, mem)
    vin = {"l8": lane * 8, "t1w": S + (lane & 31) * 8, "t1r": S + (i * 34 + par) * 8, "lwo": par * 128,
           "t2wl": S + ((i & 15) * 66 + 33 * par) * 8, "t2wh": S + ((i & 15) * 66 + 31 * par + 1) * 8,
           "t2r": S + (lane ^ (lane >> np.uint64(5))) * 8, "t4w": S + ((i & 15) * 66 + par) * 8, "t4r": S + lane * 8,
           "t1x": S + (lane + (lane >> np.uint64(5))) * 8, "t1y": S + ((i & 15) * 66 + 33 * par) * 8}
    if w1x is None:
        import gen_tw_kernel as _T
        w1x = (_T.FWD_W1X and name.startswith("fwd")) or (_T.INV_W1X and name.startswith("inv"))
    if w1x:  # lane = i + 32 j0 (gen_tw_kernel NTT_ADDR_W1X; the inverse's W1'' pair bit j5 likewise)
        par, i = lane >> np.uint64(5), lane & np.uint64(31)
        vin.update({"t1r": S + (i * 33 + par) * 8, "lwo": par * 128,
                    "t2wl": S + ((i & 15) * 65 + 33 * par) * 8, "t2wh": S + ((i & 15) * 65 + 31 * par + 1) * 8,
                    "t4w": S + ((i & 15) * 65 + par) * 8, "t1y": S + ((i & 15) * 66 + 33 * par) * 8})
    for k, (name_, val) in enumerate(vin.items()):
        w.v[200 + k] = val.astype(np.uint64)   # outside the body's v8..v127
        ops[name_] = f"v{200 + k}"
    lw = TB + 2048 * 8
    # an SGPR pair no body clobbers (the key-conversion body owns s94..s101)
    w.s[104], w.s[105] = np.uint64(lw & 0xFFFFFFFF), np.uint64(lw >> 32)
    ops["lw"] = "s[104:105]"
    if mem_extra:
        mem.update(mem_extra)
    if ops_extra:
        ops.update(ops_extra)
    w.ops = ops
    w.run(body_lines(hdr, name))
    if out_init is not None:
        return data, out
    return out if out_of_place else data


def _lds_with_lane_pair_tables(tab, N, stride=None):
    """Workgroup LDS as pbs_tw.hip lays it out: 2 exchange buffers of `stride` u64 (default N), then the 32 forward
    lane-pair twiddles (tab[N:N+32]) and the W1'' inverse's 32 last-DIT-stage twiddles, entry m + 16 par =
    2^(-3 (2 m + par) mod 192) (the plan's fourth table region, c_api.cpp)."""
    P = 0xFFFFFFFF00000001
    st = stride or N
    lds = np.zeros(2 * st + 64, dtype=np.uint64)
    t = np.array(tab, dtype=np.uint64)
    lds[2 * st:2 * st + 32] = t[N:N + 32]
    lds[2 * st + 32:2 * st + 64] = [pow(2, (192 - 3 * (2 * m + par) % 192) % 192, P)
                                    for par in range(2) for m in range(16)]
    return lds


def pbs_lds_stride(hdr, which="PBS"):
    """MI_PBS_LDS_STRIDE (MI_EXT_LDS_STRIDE: which="EXT") of a generated pbs_tw_body.hpp (u64 per wave buffer)."""
    m = re.search(r"#define MI_%s_LDS_STRIDE (\d+)" % which, open(hdr).read())
    return int(m.group(1)) if m else 2048


def run_pbs(hdr, lwe, lut, bsk, tab, base_log, n_lwe, name="bnf_l1", acc0=None):
    """Emulate the 2-wave workgroup of the blind-rotation body (tools/gen_pbs_kernel.py) on one LWE
    ciphertext.  bsk: n x 2 x 2 x N NTT-domain key (N^-1 folded in), tab: the plan's twist tables
    [fwd | lane-pair | inverse | lane-pair].  Returns the accumulator (2 x N) the body leaves in LDS.
    Solinas bodies (name "sol_l1"): lwe holds the pre-switched mask, acc0 (2 x N) the rotated LUT the
    wrapper leaves in LDS."""
    N = 2048
    LB, UB, KB, TB = 0x100000000, 0x200000000, 0x300000000, 0x400000000
    mem = {LB: np.array(lwe, dtype=np.uint64), UB: np.array(lut, dtype=np.uint64).reshape(-1),
           KB: np.array(bsk, dtype=np.uint64).reshape(-1), TB: np.array(tab, dtype=np.uint64)}
    st = pbs_lds_stride(hdr)
    lds = _lds_with_lane_pair_tables(tab, N, st)
    if acc0 is not None:
        a0 = np.array(acc0, dtype=np.uint64).reshape(2, N)
        for w in range(2):
            lds[w * st:w * st + N] = a0[w]
    lines = body_lines(hdr, name, "MI_PBS_BODY_")
    waves = []
    for w in range(2):
        ops = {"lane": "v0", "S": str(w * st * 8), "SP": str((1 - w) * st * 8),
               "lut_lo": str((UB + w * N * 8) & 0xFFFFFFFF), "lut_hi": str((UB + w * N * 8) >> 32),
               "gown_lo": str((KB + 3 * w * N * 8) & 0xFFFFFFFF), "gown_hi": str((KB + 3 * w * N * 8) >> 32),
               "gpar_lo": str((KB + (2 - w) * N * 8) & 0xFFFFFFFF), "gpar_hi": str((KB + (2 - w) * N * 8) >> 32),
               "lwe_lo": str(LB & 0xFFFFFFFF), "lwe_hi": str(LB >> 32), "n": str(n_lwe),
               "tab_lo": str(TB & 0xFFFFFFFF), "tab_hi": str(TB >> 32), "bl": str(base_log), "LW": str(2 * st * 8)}
        wv = Wave(ops, mem, lds=lds)
        wv.v[0] = np.arange(LANES, dtype=np.uint64)
        wv.load(lines)
        waves.append(wv.steps())
    live = [True, True]
    while any(live):
        for k in range(2):
            if live[k]:
                try:
                    next(waves[k])
                except StopIteration:
                    live[k] = False
    return np.stack([lds[w * st:w * st + N] for w in range(2)]).copy()


def run_ext(hdr, glwe, out, ggsw, tab, base_log, cmux=False, sol=False):
    """Emulate the 2-wave external-product / CMUX body on one GLWE pair (glwe, out: 2 x N, updated
    in place and returned); ggsw: 2 x 2 x N Raw NTT key; tab: [fwd | inverse | inverse * N^-1]."""
    N = 2048
    GB, OB, KB, TB = 0x100000000, 0x200000000, 0x300000000, 0x400000000
    g = np.array(glwe, dtype=np.uint64).reshape(-1).copy()
    o = np.array(out, dtype=np.uint64).reshape(-1).copy()
    mem = {GB: g, OB: o, KB: np.array(ggsw, dtype=np.uint64).reshape(-1), TB: np.array(tab, dtype=np.uint64)}
    st = pbs_lds_stride(hdr, "EXT")
    lds = _lds_with_lane_pair_tables(tab, N, st)
    kind = "sol" if sol else "bnf"
    lines = body_lines(hdr, f"cmux_{kind}_l1" if cmux else f"ext_{kind}_l1", "MI_PBS_BODY_")
    waves = []
    for w in range(2):
        lo = lambda a: str(a & 0xFFFFFFFF)
        hi = lambda a: str(a >> 32)
        ops = {"lane": "v0", "S": str(w * st * 8), "SP": str((1 - w) * st * 8),
               "glwe_lo": lo(GB + w * N * 8), "glwe_hi": hi(GB + w * N * 8),
               "out_lo": lo(OB + w * N * 8), "out_hi": hi(OB + w * N * 8),
               "gown_lo": lo(KB + 3 * w * N * 8), "gown_hi": hi(KB + 3 * w * N * 8),
               "gpar_lo": lo(KB + (2 - w) * N * 8), "gpar_hi": hi(KB + (2 - w) * N * 8),
               "tab_lo": lo(TB), "tab_hi": hi(TB), "bl": str(base_log), "LW": str(2 * st * 8)}
        wv = Wave(ops, mem, lds=lds)
        wv.v[0] = np.arange(LANES, dtype=np.uint64)
        wv.load(lines)
        waves.append(wv.steps())
    live = [True, True]
    while any(live):
        for k in range(2):
            if live[k]:
                try:
                    next(waves[k])
                except StopIteration:
                    live[k] = False
    return g.reshape(2, N), o.reshape(2, N)


if __name__ == "__main__":
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
    import random
    import oracle as O
    P = 0xFFFFFFFF00000001
    here = os.path.dirname(os.path.abspath(__file__))
    hdr = sys.argv[1] if len(sys.argv) > 1 else os.path.join(here, "..", "tfhe-rs-main_modified_amd", "csrc",
                                                             "ntt64_tw_body.hpp")
    plan = O.Plan.try_new(2048, P)
    tw = [int(v) for v in plan.twid]
    br = lambda x, b: int(format(x, f"0{b}b")[::-1], 2)
    psi = tw[br(1, 11)]
    tab = []
    for i_ in range(32):
        rho = pow(psi, 2 * br(i_, 5) + 1, P)
        tab += [pow(rho, j, P) for j in range(64)]
    omega = pow(psi, 64, P)
    cyc5 = [pow(omega, br(g, 5), P) for g in range(32)]
    random.seed(3)
    x = [random.randrange(P) for _ in range(2048)]
    got = run_body(hdr, "fwd", x, tab + cyc5)
    want = plan.fwd(np.array(x, dtype=np.uint64))
    bad = np.nonzero(got != want)[0]
    print("fwd mismatches:", len(bad), bad[:16])
    # inverse: untwist table rho_i^-j and the inverse lane-pair twiddles
    itab = []
    for i_ in range(32):
        rinv = pow(pow(psi, 2 * br(i_, 5) + 1, P), P - 2, P)
        itab += [pow(rinv, j, P) for j in range(64)]
    icyc5 = [pow(pow(omega, br(g, 5), P), P - 2, P) for g in range(32)]
    y = [int(v) for v in want]
    got_i = run_body(hdr, "inv", y, itab + icyc5)
    want_i = plan.inv(np.array(y, dtype=np.uint64))
    bad = np.nonzero(got_i != want_i)[0]
    print("inv mismatches:", len(bad), bad[:16])
