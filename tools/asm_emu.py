#!/usr/bin/env python3
"""Tiny functional emulator (one wave64) for the instruction subset the generated twisted-NTT
bodies use (tools/gen_tw_kernel.py).  Checks the data path's logic on the CPU — not hazards or
timing, which only the GPU run can.

  python tools/asm_emu.py            # runs the forward body on one random polynomial vs the oracle
"""
import os
import re
import sys

import numpy as np

M32 = np.uint64(0xFFFFFFFF)
LANES = 64


class Wave:
    def __init__(self, ops, mem, lds_bytes=65536):
        self.v = np.zeros((256, LANES), dtype=np.uint64)   # 32-bit values kept in uint64
        self.s = np.zeros(128, dtype=np.uint64)
        self.exec = np.ones(LANES, dtype=bool)
        self.vcc = np.zeros(LANES, dtype=bool)
        self.lds = np.zeros(lds_bytes // 8, dtype=np.uint64)
        self.mem = mem          # dict base_address -> np.uint64 array (global memory regions)
        self.ops = ops          # operand name -> value

    # ---- operand parsing ----------------------------------------------------------------------
    def vreg(self, tok):
        m = re.fullmatch(r"v(\d+)", tok)
        return int(m.group(1)) if m else None

    def vpair(self, tok):
        m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
        return int(m.group(1)) if m else None

    def spair(self, tok):
        m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
        return int(m.group(1)) if m else None

    def mask(self, tok):
        if tok == "vcc":
            return self.vcc.copy()
        b = self.spair(tok)
        if b is None:
            raise ValueError(tok)
        word = int(self.s[b]) | (int(self.s[b + 1]) << 32)
        return np.array([(word >> l) & 1 for l in range(LANES)], dtype=bool)

    def set_mask(self, tok, m):
        m = m & self.exec | (self.mask(tok) & ~self.exec) if tok != "vcc" else m
        word = 0
        for l in range(LANES):
            if m[l]:
                word |= 1 << l
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
        val = int(tok, 0)
        return np.full(LANES, np.uint64(val & 0xFFFFFFFF), dtype=np.uint64)

    def src64(self, tok):
        b = self.vpair(tok)
        if b is not None:
            return self.v[b] | (self.v[b + 1] << np.uint64(32))
        val = int(tok, 0)
        return np.full(LANES, np.uint64(val & 0xFFFFFFFFFFFFFFFF), dtype=np.uint64)

    def wv(self, r, val):
        self.v[r] = np.where(self.exec, val & M32, self.v[r])

    def wv64(self, b, val):
        self.wv(b, val & M32)
        self.wv(b + 1, val >> np.uint64(32))

    # ---- execution ------------------------------------------------------------------------------
    def run(self, lines):
        for line in lines:
            line = line.strip()
            if not line or line.startswith("s_nop") or line.startswith("s_waitcnt"):
                continue
            for k, v in self.ops.items():
                line = line.replace(f"%[{k}]", v)
            mn, _, rest = line.partition(" ")
            args = [a.strip() for a in re.split(r",(?![^\[]*\])", rest)] if rest else []
            getattr(self, "op_" + mn.replace(".", "_"), None) or self.unknown(mn)
            getattr(self, "op_" + mn)(args)

    def unknown(self, mn):
        raise NotImplementedError(mn)

    # VALU
    def op_v_mov_b32(self, a):
        self.wv(self.vreg(a[0]), self.src32(a[1]))

    def op_v_mov_b32_dpp(self, a):
        src = self.src32(a[1].split()[0])
        perm = [int(x) for x in re.search(r"quad_perm:\[(.*?)\]", a[1]).group(1).split(",")]
        out = np.array([src[(l & ~3) + perm[l & 3]] for l in range(LANES)], dtype=np.uint64)
        self.wv(self.vreg(a[0]), out)

    def op_v_lshlrev_b32(self, a):
        self.wv(self.vreg(a[0]), (self.src32(a[2]) << (self.src32(a[1]) & np.uint64(31))) & M32)

    def op_v_lshrrev_b32(self, a):
        self.wv(self.vreg(a[0]), self.src32(a[2]) >> (self.src32(a[1]) & np.uint64(31)))

    def op_v_lshlrev_b64(self, a):
        self.wv64(self.vpair(a[0]), self.src64(a[2]) << (self.src32(a[1]) & np.uint64(63)))

    def op_v_lshrrev_b64(self, a):
        self.wv64(self.vpair(a[0]), self.src64(a[2]) >> (self.src32(a[1]) & np.uint64(63)))

    def op_v_mad_u64_u32(self, a):
        x, y, z = self.src32(a[2]), self.src32(a[3]), self.src64(a[4])
        full = [int(x[l]) * int(y[l]) + int(z[l]) for l in range(LANES)]
        self.wv64(self.vpair(a[0]), np.array([f & 0xFFFFFFFFFFFFFFFF for f in full], dtype=np.uint64))
        self.set_mask(a[1], np.array([f >> 64 != 0 for f in full]))

    def _carry_op(self, a, fn):
        x, y = self.src32(a[2]), self.src32(a[3])
        cin = self.mask(a[4]).astype(np.uint64) if len(a) > 4 else np.zeros(LANES, dtype=np.uint64)
        res, co = fn(x.astype(np.int64), y.astype(np.int64), cin.astype(np.int64))
        self.wv(self.vreg(a[0]), (res.astype(np.uint64)) & M32)
        self.set_mask(a[1], co)

    def op_v_add_co_u32_e64(self, a):
        self._carry_op(a, lambda x, y, c: (x + y, (x + y) >> 32 != 0))

    def op_v_addc_co_u32_e64(self, a):
        self._carry_op(a, lambda x, y, c: (x + y + c, (x + y + c) >> 32 != 0))

    def op_v_sub_co_u32_e64(self, a):
        self._carry_op(a, lambda x, y, c: ((x - y) & 0xFFFFFFFF, x - y < 0))

    def op_v_subb_co_u32_e64(self, a):
        self._carry_op(a, lambda x, y, c: ((x - y - c) & 0xFFFFFFFF, x - y - c < 0))

    def op_v_cndmask_b32_e64(self, a):
        m = self.mask(a[3])
        self.wv(self.vreg(a[0]), np.where(m, self.src32(a[2]), self.src32(a[1])))

    # SALU
    def op_s_mov_b32(self, a):
        val = self.s_src(a[1])
        if a[0] == "exec_lo":
            for l in range(32):
                self.exec[l] = bool((val >> l) & 1)
        elif a[0] == "exec_hi":
            for l in range(32):
                self.exec[32 + l] = bool((val >> l) & 1)
        else:
            self.s[int(a[0][1:])] = np.uint64(val)

    def s_src(self, tok):
        m = re.fullmatch(r"s(\d+)", tok)
        if m:
            return int(self.s[int(m.group(1))])
        return int(tok, 0) & 0xFFFFFFFF

    def op_s_mov_b64(self, a):
        if a[1] == "exec":
            word = sum(1 << l for l in range(LANES) if self.exec[l])
            b = self.spair(a[0])
            self.s[b], self.s[b + 1] = np.uint64(word & 0xFFFFFFFF), np.uint64(word >> 32)
        elif a[0] == "exec":
            self.exec = self.mask(a[1])
        else:
            raise NotImplementedError(a)

    def op_s_or_b64(self, a):
        m = self.mask(a[1]) | self.mask(a[2])
        word = sum(1 << l for l in range(LANES) if m[l])
        b = self.spair(a[0])
        self.s[b], self.s[b + 1] = np.uint64(word & 0xFFFFFFFF), np.uint64(word >> 32)

    def op_s_add_u32(self, a):
        x = self.s_src(a[1]) + self.s_src(a[2])
        self.s[int(a[0][1:])] = np.uint64(x & 0xFFFFFFFF)
        self.scc = x >> 32

    def op_s_addc_u32(self, a):
        x = self.s_src(a[1]) + self.s_src(a[2]) + self.scc
        self.s[int(a[0][1:])] = np.uint64(x & 0xFFFFFFFF)
        self.scc = x >> 32

    # memory
    def _addr(self, voff, sbase, off):
        b = self.spair(sbase)
        base = int(self.s[b]) | (int(self.s[b + 1]) << 32)
        return [base + int(voff[l]) + off for l in range(LANES)]

    def _mem(self, addr):
        for base, arr in self.mem.items():
            if base <= addr < base + arr.size * 8:
                return arr, (addr - base) // 8
        raise IndexError(hex(addr))

    def op_global_load_dwordx2(self, a):
        parts = a[2].split()
        off = int(parts[1].split(":")[1]) if len(parts) > 1 else 0
        addrs = self._addr(self.src32(a[1]), parts[0], off)
        vals = np.zeros(LANES, dtype=np.uint64)
        for l in range(LANES):
            if self.exec[l]:
                arr, i = self._mem(addrs[l])
                vals[l] = arr[i]
        self.wv64(self.vpair(a[0]), vals)

    def op_global_store_dwordx2(self, a):
        parts = a[2].split()
        off = int(parts[1].split(":")[1]) if len(parts) > 1 else 0
        addrs = self._addr(self.src32(a[0]), parts[0], off)
        vals = self.src64(a[1])
        for l in range(LANES):
            if self.exec[l]:
                arr, i = self._mem(addrs[l])
                arr[i] = vals[l]

    def op_ds_write_b64(self, a):
        parts = a[1].split()
        off = int(parts[1].split(":")[1]) if len(parts) > 1 else 0
        addr = self.src32(a[0])
        vals = self.src64(parts[0])
        for l in range(LANES):
            if self.exec[l]:
                self.lds[(int(addr[l]) + off) // 8] = vals[l]

    def op_ds_read_b64(self, a):
        parts = a[1].split()
        off = int(parts[1].split(":")[1]) if len(parts) > 1 else 0
        addr = self.src32(parts[0])
        vals = np.array([self.lds[(int(addr[l]) + off) // 8] for l in range(LANES)], dtype=np.uint64)
        self.wv64(self.vpair(a[0]), vals)


def body_lines(hdr, name):
    txt = open(hdr).read()
    start = txt.index(f"#define MI_TW_BODY_{name.upper()}(")
    end = txt.index(":: __VA_ARGS__", start)
    return [m.group(1) for m in re.finditer(r'"(.*?)\\n"', txt[start:end])]


def run_body(hdr, name, poly, twist_tab, fwd=True):
    """Emulate one wave (wave 0 of a workgroup) on one polynomial."""
    data = np.array(poly, dtype=np.uint64).copy()
    tw = np.array(twist_tab, dtype=np.uint64)
    GB, TB = 0x100000000, 0x200000000
    mem = {GB: data, TB: tw}
    lane = np.arange(LANES, dtype=np.uint64)
    par, i = lane & np.uint64(1), lane >> np.uint64(1)
    S = 0
    ops = {"g_lo": f"{GB & 0xFFFFFFFF}", "g_hi": f"{GB >> 32}", "tw_lo": f"{TB & 0xFFFFFFFF}", "tw_hi": f"{TB >> 32}"}
    w = Wave(None, mem)
    vin = {"l8": lane * 8, "t1w": S + (lane & 31) * 8, "t1r": S + (i * 34 + par) * 8, "lwo": par * 128,
           "t2wl": S + ((i & 15) * 66 + 33 * par) * 8, "t2wh": S + ((i & 15) * 66 + 31 * par + 1) * 8,
           "t2r": S + (lane ^ (lane >> np.uint64(5))) * 8, "t4w": S + ((i & 15) * 66 + par) * 8, "t4r": S + lane * 8}
    for k, (name_, val) in enumerate(vin.items()):
        w.v[200 + k] = val.astype(np.uint64)   # outside the body's v8..v127
        ops[name_] = f"v{200 + k}"
    # lw: SGPR pair at s[100:101]
    lw = TB + 2048 * 8
    w.s[100], w.s[101] = np.uint64(lw & 0xFFFFFFFF), np.uint64(lw >> 32)
    ops["lw"] = "s[100:101]"
    # the body writes s22:23 <- exec; 'ops' substitution
    w.ops = ops
    w.scc = 0
    w.run(body_lines(hdr, name))
    return data


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
