#!/usr/bin/env python3
"""Generate tfhe-rs-main_modified_amd/csrc/ntt64_tw_asm.hpp: hand-scheduled gfx950 stages of the
twisted N = 2048 Goldilocks transform (ntt64_tw.hip).

Each generated function runs one radix-2 stage (16 butterflies per lane) on the 32 coefficients a
lane holds, pinned at v[64:127] (x[r] = v[64+2r : 65+2r]), with twiddles 2^e known per register at
generation time (tables from ntt64_tw_tables.hpp / tools/gen_tw_tables.py).

Arithmetic (p = 2^64 - 2^32 + 1, EPS = 2^32 - 1; values are "semi": any u64 standing for x mod p):
  shift multiply, canonical result t (x * 2^S = +-t):
    A (1 <= E <= 32):  L = x << E, H = x_hi >> (32-E); R = L + H*EPS (mad, carry c);
                       t = (c | R >= p) ? R + EPS : R      (U = R + EPS by a mad, its carry = R >= p)
    B (32 < E < 64):   z = x * 2^(E-32) as in A but only folded once (semi), then z * 2^32 =
                       (0 : z_lo) + z_hi * EPS (mad) and canonical select as in A
    C (64 <= E < 96):  2^E = -2^-K (K = 96 - E): t' = (x >> K) + u - u*2^32, u = x_lo << (32-K),
                       + p on borrow; the sign flips the butterfly
    E = 0:             canonical copy
  CT (forward):  a' = a + t, b' = a - t  (a semi, t canonical: one fold each, never two)
  GS (inverse):  b -> canonical first; a' = a + b, d = a - b, b' = +-tmul(d)
Carries live in per-slot SGPR pairs (VOP3b forms cost the same as VCC forms on gfx950: 4.6 cycles,
tools/valu_probe.hip), so independent butterflies interleave; the list scheduler pads every
VALU-written SGPR read by a VALU with 2 wait states (what hipcc itself inserts on gfx950).

Usage: python tools/gen_tw_asm.py > tfhe-rs-main_modified_amd/csrc/ntt64_tw_asm.hpp
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

DATA = 64          # x[r] at v[DATA + 2r : DATA + 2r + 1]
SCR = 32           # scratch slots: v[SCR + 8k .. SCR + 8k + 7]
NSLOT = 4
SGB = 40           # SGPR carry pairs: s[SGB + 8k ..] four pairs per slot
JUNK = 72          # s[72:73] junk carry-out


def xr(r):
    return f"v{DATA + 2 * r}", f"v{DATA + 2 * r + 1}", f"v[{DATA + 2 * r}:{DATA + 2 * r + 1}]"


class Slot:
    def __init__(self, k):
        b = SCR + 8 * k
        self.v = [f"v{b + i}" for i in range(8)]
        self.P = [f"v[{b + 2 * i}:{b + 2 * i + 1}]" for i in range(4)]
        sb = SGB + 8 * k
        self.c = [f"s[{sb + 2 * i}:{sb + 2 * i + 1}]" for i in range(4)]


J = f"s[{JUNK}:{JUNK + 1}]"


def pair_regs(p):
    a, b = p[2:-1].split(":")
    return [f"v{a}", f"v{b}"]


class Op:
    __slots__ = ("text", "reads", "writes", "salu", "cost", "preds", "succs", "prio", "sgpr_reads", "bf")

    def __init__(self, text, reads, writes, bf):
        self.text, self.bf = text, bf
        self.reads, self.writes = set(), set()
        for r in reads:
            self.reads.update(pair_regs(r) if r.startswith("v[") else [r])
        for w in writes:
            self.writes.update(pair_regs(w) if w.startswith("v[") else [w])
        m = text.split()[0]
        self.salu = m.startswith("s_")
        self.cost = 0.0 if self.salu else (2.3 if m in ("v_mov_b32", "v_lshrrev_b32", "v_lshlrev_b32") else 4.5)
        self.preds, self.succs = set(), set()
        self.sgpr_reads = {r for r in self.reads if r.startswith("s[")}
        self.prio = 0.0


def E(ops, bf, text, reads, writes):
    ops.append(Op(text, reads, writes, bf))


# ---- sequences ---------------------------------------------------------------------------------
def tmul(ops, bf, S, xlo, xhi, xp, sl, tlo, thi):
    """canonical t (into tlo/thi) with x * 2^S = (neg ? -t : t); returns neg."""
    e = S % 96
    neg = (S >= 96) != (e >= 64)
    v, P, c = sl.v, sl.P, sl.c
    if e == 0:
        E(ops, bf, f"v_mad_u64_u32 {P[0]}, {c[1]}, -1, 1, {xp}", [xp], [P[0], c[1]])
        E(ops, bf, f"v_cndmask_b32_e64 {tlo}, {xlo}, {v[0]}, {c[1]}", [xlo, v[0], c[1]], [tlo])
        E(ops, bf, f"v_cndmask_b32_e64 {thi}, {xhi}, {v[1]}, {c[1]}", [xhi, v[1], c[1]], [thi])
        return neg
    if e < 64:
        r = e if e <= 32 else e - 32
        E(ops, bf, f"v_lshlrev_b64 {P[0]}, {r}, {xp}", [xp], [P[0]])
        if r == 32:
            h = xhi
        else:
            h = v[4]
            E(ops, bf, f"v_lshrrev_b32 {h}, {32 - r}, {xhi}", [xhi], [h])
        E(ops, bf, f"v_mad_u64_u32 {P[1]}, {c[0]}, {h}, -1, {P[0]}", [h, P[0]], [P[1], c[0]])
        src = P[1]
        if e > 32:
            # z = R + c*EPS (semi), then z * 2^32 = (0 : z_lo) + z_hi * EPS
            E(ops, bf, f"v_cndmask_b32_e64 {v[4]}, 0, -1, {c[0]}", [c[0]], [v[4]])
            E(ops, bf, f"v_mad_u64_u32 {P[0]}, {J}, {v[4]}, 1, {P[1]}", [v[4], P[1]], [P[0]])
            E(ops, bf, f"v_mov_b32 {v[6]}, 0", [], [v[6]])
            E(ops, bf, f"v_mov_b32 {v[7]}, {v[0]}", [v[0]], [v[7]])
            E(ops, bf, f"v_mad_u64_u32 {P[1]}, {c[0]}, {v[1]}, -1, {P[3]}", [v[1], P[3]], [P[1], c[0]])
        E(ops, bf, f"v_mad_u64_u32 {P[0]}, {c[1]}, -1, 1, {src}", [src], [P[0], c[1]])
        E(ops, bf, f"s_or_b64 {c[1]}, {c[1]}, {c[0]}", [c[1], c[0]], [c[1], "scc"])
        E(ops, bf, f"v_cndmask_b32_e64 {tlo}, {v[2]}, {v[0]}, {c[1]}", [v[2], v[0], c[1]], [tlo])
        E(ops, bf, f"v_cndmask_b32_e64 {thi}, {v[3]}, {v[1]}, {c[1]}", [v[3], v[1], c[1]], [thi])
        return neg
    K = 96 - e
    E(ops, bf, f"v_lshrrev_b64 {P[0]}, {K}, {xp}", [xp], [P[0]])
    if K == 32:
        u = xlo
    else:
        u = v[4]
        E(ops, bf, f"v_lshlrev_b32 {u}, {32 - K}, {xlo}", [xlo], [u])
    E(ops, bf, f"v_mad_u64_u32 {P[1]}, {J}, {u}, 1, {P[0]}", [u, P[0]], [P[1]])
    E(ops, bf, f"v_sub_co_u32_e64 {v[3]}, {c[0]}, {v[3]}, {u}", [v[3], u], [v[3], c[0]])
    E(ops, bf, f"v_cndmask_b32_e64 {v[5]}, 0, -1, {c[0]}", [c[0]], [v[5]])
    E(ops, bf, f"v_addc_co_u32_e64 {tlo}, {c[1]}, {v[2]}, 0, {c[0]}", [v[2], c[0]], [tlo, c[1]])
    E(ops, bf, f"v_addc_co_u32_e64 {thi}, {J}, {v[3]}, {v[5]}, {c[1]}", [v[3], v[5], c[1]], [thi])
    return neg


def add_part1(ops, bf, sl, alo, ahi, tlo, thi):
    v, P, c = sl.v, sl.P, sl.c
    E(ops, bf, f"v_add_co_u32_e64 {v[0]}, {c[2]}, {alo}, {tlo}", [alo, tlo], [v[0], c[2]])
    E(ops, bf, f"v_addc_co_u32_e64 {v[1]}, {c[3]}, {ahi}, {thi}, {c[2]}", [ahi, thi, c[2]], [v[1], c[3]])


def add_part2(ops, bf, sl, dp):
    v, P, c = sl.v, sl.P, sl.c
    E(ops, bf, f"v_cndmask_b32_e64 {v[5]}, 0, -1, {c[3]}", [c[3]], [v[5]])
    E(ops, bf, f"v_mad_u64_u32 {dp}, {J}, {v[5]}, 1, {P[0]}", [v[5], P[0]], [dp])


def sub_seq(ops, bf, sl, dlo, dhi, alo, ahi, tlo, thi):
    """d = a - t (+ p on borrow): a semi, t canonical -> semi."""
    v, c = sl.v, sl.c
    E(ops, bf, f"v_sub_co_u32_e64 {dlo}, {c[0]}, {alo}, {tlo}", [alo, tlo], [dlo, c[0]])
    E(ops, bf, f"v_subb_co_u32_e64 {dhi}, {c[1]}, {ahi}, {thi}, {c[0]}", [ahi, thi, c[0]], [dhi, c[1]])
    E(ops, bf, f"v_cndmask_b32_e64 {v[4]}, 0, -1, {c[1]}", [c[1]], [v[4]])
    E(ops, bf, f"v_addc_co_u32_e64 {dlo}, {c[0]}, {dlo}, 0, {c[1]}", [dlo, c[1]], [dlo, c[0]])
    E(ops, bf, f"v_addc_co_u32_e64 {dhi}, {J}, {dhi}, {v[4]}, {c[0]}", [dhi, v[4], c[0]], [dhi])


def ct(ops, bf, sl, ra, rb, S):
    alo, ahi, ap = xr(ra)
    blo, bhi, bp = xr(rb)
    v = sl.v
    tlo, thi = v[2], v[3]
    neg = tmul(ops, bf, S, blo, bhi, bp, sl, tlo, thi)
    # t in v2:v3.  non-neg: a' = a + t, b' = a - t ; neg: a' = a - t, b' = a + t
    add_part1(ops, bf, sl, alo, ahi, tlo, thi)
    if not neg:
        sub_seq(ops, bf, sl, blo, bhi, alo, ahi, tlo, thi)
        add_part2(ops, bf, sl, ap)
    else:
        sub_seq(ops, bf, sl, alo, ahi, alo, ahi, tlo, thi)  # reads a before add_part2 writes b
        add_part2(ops, bf, sl, bp)


def gs(ops, bf, sl, ra, rb, S):
    alo, ahi, ap = xr(ra)
    blo, bhi, bp = xr(rb)
    v, P, c = sl.v, sl.P, sl.c
    # cb = canon(b) into v2:v3
    E(ops, bf, f"v_mad_u64_u32 {P[3]}, {c[1]}, -1, 1, {bp}", [bp], [P[3], c[1]])
    E(ops, bf, f"v_cndmask_b32_e64 {v[2]}, {blo}, {v[6]}, {c[1]}", [blo, v[6], c[1]], [v[2]])
    E(ops, bf, f"v_cndmask_b32_e64 {v[3]}, {bhi}, {v[7]}, {c[1]}", [bhi, v[7], c[1]], [v[3]])
    add_part1(ops, bf, sl, alo, ahi, v[2], v[3])            # s = a + cb -> v0:v1
    sub_seq(ops, bf, sl, blo, bhi, alo, ahi, v[2], v[3])     # d = a - cb -> b
    add_part2(ops, bf, sl, ap)                               # a' = s (+EPS)
    neg = tmul(ops, bf, S, blo, bhi, bp, sl, blo, bhi)       # b' = tmul(d)
    if neg:
        E(ops, bf, f"v_sub_co_u32_e64 {blo}, {sl.c[2]}, 1, {blo}", [blo], [blo, sl.c[2]])
        E(ops, bf, f"v_subb_co_u32_e64 {bhi}, {J}, -1, {bhi}, {sl.c[2]}", [bhi, sl.c[2]], [bhi])


# ---- scheduling ----------------------------------------------------------------------------------
def schedule(ops):
    last_w, readers = {}, {}
    for op in ops:
        for r in op.reads:
            if r in last_w:
                op.preds.add(last_w[r])
        for w in op.writes:
            if w in (J,):
                continue
            if w in last_w:
                op.preds.add(last_w[w])
            for rd in readers.get(w, []):
                if rd is not op:
                    op.preds.add(rd)
        for r in op.reads:
            readers.setdefault(r, []).append(op)
        for w in op.writes:
            if w in (J,):
                continue
            last_w[w] = op
            readers[w] = []
    for op in ops:
        for p in op.preds:
            p.succs.add(op)
    for op in reversed(ops):
        op.prio = op.cost + max((s.prio for s in op.succs), default=0.0)
    # SGPR producer tracking for hazards
    producer = {}
    last = {}
    for op in ops:
        for r in op.sgpr_reads:
            if r in last:
                producer[(op, r)] = last[r]
        for w in op.writes:
            if w.startswith("s["):
                last[w] = op
    done, out, issued = set(), [], {}
    remaining = list(ops)
    slot = 0
    while remaining:
        best = None
        for op in remaining:
            if not all(p in done for p in op.preds):
                continue
            ok = True
            for r in op.sgpr_reads:
                pr = producer.get((op, r))
                if pr is not None and not pr.salu:
                    need = 2 if op.salu else 3
                    if slot - issued[pr] < need:
                        ok = False
                        break
            if not ok:
                continue
            key = (op.prio, -op.bf)
            if best is None or key > bkey:
                best, bkey = op, key
        if best is None:
            out.append("s_nop 0")
            slot += 1
            continue
        out.append(best.text)
        issued[best] = slot
        slot += 1
        done.add(best)
        remaining.remove(best)
    # merge nops
    res, run = [], 0
    for l in out + ["<end>"]:
        if l == "s_nop 0":
            run += 1
            continue
        while run:
            n = min(run, 8)
            res.append(f"s_nop {n - 1}")
            run -= n
        if l != "<end>":
            res.append(l)
    return res


def stage(kind, dist, exps):
    """kind 'ct'/'gs'; dist = register distance; exps[g] for group g = r // (2*dist)."""
    ops = []
    slots = [Slot(k) for k in range(NSLOT)]
    bf = 0
    for r in range(32):
        if r & dist:
            continue
        S = exps[r // (2 * dist)]
        (ct if kind == "ct" else gs)(ops, bf, slots[bf % NSLOT], r, r + dist, S)
        bf += 1
    lines = schedule(ops)
    nvalu = sum(1 for l in lines if l.startswith("v_"))
    nsalu = sum(1 for l in lines if l.startswith("s_") and not l.startswith("s_nop"))
    nnop = sum(int(l.split()[1]) + 1 for l in lines if l.startswith("s_nop"))
    return lines, nvalu, nsalu, nnop


def cfun(name, lines, stats):
    outs = ", ".join(f'"+{{v[{DATA + 2 * r}:{DATA + 2 * r + 1}]}}"(x[{r}])' for r in range(32))
    clob = [f'"v{SCR + i}"' for i in range(8 * NSLOT)] + [f'"s{SGB + i}"' for i in range(8 * NSLOT)]
    clob += [f'"s{JUNK}"', f'"s{JUNK + 1}"', '"scc"']
    body = "\n".join(f'      "{l}\\n"' for l in lines)
    return (f"// {stats}\n__device__ __forceinline__ void {name}(u64 (&x)[32]) {{\n  asm volatile(\n{body}\n"
            f"      : {outs}\n      :\n      : {', '.join(clob)});\n}}\n")


def main():
    import importlib.util
    here = os.path.dirname(os.path.abspath(__file__))
    hdr = os.path.join(here, "..", "tfhe-rs-main_modified_amd", "csrc", "ntt64_tw_tables.hpp")
    tabs = {}
    cur = None
    for line in open(hdr):
        line = line.strip()
        if line.startswith("constexpr int"):
            cur = line.split()[2].split("[")[0]
            tabs[cur] = []
        elif cur and line.startswith("{"):
            tabs[cur].append([int(t) for t in line.strip("{},").split(",")])
        elif line.startswith("};"):
            cur = None
    out = ["// GENERATED by tools/gen_tw_asm.py — do not edit.  Hand-scheduled gfx950 stages of the twisted",
           "// N = 2048 Goldilocks transform; x[r] pinned at v[%d + 2r], scratch v%d..v%d, s%d..s%d." %
           (DATA, SCR, SCR + 8 * NSLOT - 1, SGB, JUNK + 1),
           "#pragma once", "#include <stdint.h>", "namespace mi { namespace twasm {", "typedef uint64_t u64;", ""]
    total = 0
    for name, kind, tab, order in (("g1_fwd", "ct", "G1_FWD", range(5)), ("cyc_fwd", "ct", "CYC_FWD", range(5)),
                                   ("g1_inv", "gs", "G1_INV", range(4, -1, -1)),
                                   ("cyc_inv", "gs", "CYC_INV", range(4, -1, -1))):
        for s in order:
            lines, nv, ns, nn = stage(kind, 16 >> s, tabs[tab][s])
            total += nv
            out.append(cfun(f"{name}_{s}", lines, f"{name} stage {s}: {nv} VALU, {ns} SALU, {nn} nop states"))
    out.append("}  // namespace twasm\n}  // namespace mi\n")
    print("\n".join(out))
    print(f"// total VALU in stage blocks: {total}", file=sys.stderr)


if __name__ == "__main__":
    main()
