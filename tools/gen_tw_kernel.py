#!/usr/bin/env python3
"""Generate tfhe-rs-main_modified_amd/csrc/ntt64_tw_body.hpp: the whole data path of the twisted
N = 2048 Goldilocks transform (ntt64_tw.hip) as ONE hand-scheduled gfx950 asm body per direction.

The compiler keeps no data registers: the body owns v8..v127 (64 of them hold the 32 coefficients
of the lane, the rest are scratch) and s20..s99; C++ only passes addresses.  See ntt64_tw.hip for
the factorisation and the layouts; tools/gen_tw_tables.py for the exponent tables.

Data path (forward):
  LOAD  W0 rows (512-B coalesced)          -> G1 stages (CT, shift twiddles, compile-time per register)
  TWIST x *= rho_i^j (table, general multiply)
  T1    W0 -> W1 through LDS (two 8 KiB halves split by j, row stride 34)
  CYC   stages q = 0..4 (CT, shift twiddles)
  LAST  regroup lane pairs (DPP) -> stage q = 5 with a per-lane twiddle -> canonical
  T2    W1' -> W0 through LDS (halves split by i, row stride 66, column swizzle j ^ (j >> 5))
  STORE W0 rows
Inverse: LOAD, T1, regroup + first GS stage + regroup back, CYC_INV, T4 (W1 -> W0), UNTWIST, G1_INV,
canonical, STORE.

Usage: python tools/gen_tw_kernel.py > tfhe-rs-main_modified_amd/csrc/ntt64_tw_body.hpp
"""
import os
import sys

# ------------------------------------------------------------------------------------------------
# register budget
VLO, VHI = 8, 128            # v8..v127 owned by the body (v0..v7: compiler / address inputs)
# SGPRs: s20:21 odd-lane mask, s22:23 saved exec, s24:25 junk carry, s36..s77 carry pairs (3 per slot,
# up to 7 slots), s78..s93 row-group bases.  s32..s35 are left alone (stack/frame registers).
SG0 = 36
JUNK = "s[24:25]"
SGPR_CLOBBER = list(range(20, 32)) + list(range(36, 94))


def pv(b):
    return f"v[{b}:{b + 1}]"


class Op:
    __slots__ = ("text", "reads", "writes", "kind", "cost", "preds", "succs", "prio", "idx", "mask_reads")

    def __init__(self, text, reads, writes, kind="valu"):
        self.text, self.kind = text, kind
        self.reads, self.writes = set(), set()
        self.mask_reads = set()
        for r in reads:
            self.reads.update(expand(r))
        for w in writes:
            self.writes.update(expand(w))
        m = (text[1] if isinstance(text, list) else text).split()[0]
        if kind == "salu":
            self.cost = 0.0
        elif m in ("v_mov_b32", "v_lshrrev_b32", "v_lshlrev_b32") or kind == "dpp":
            self.cost = 2.3
        else:
            self.cost = 4.5
        self.preds, self.succs = set(), set()
        self.prio = 0.0


def expand(r):
    if r.startswith("v[") or r.startswith("s["):
        a, b = r[2:-1].split(":")
        return [f"{r[0]}{i}" for i in range(int(a), int(b) + 1)]
    return [r]


class Seg:
    """A list of ops in sequential program order, list-scheduled with gfx950 hazard padding:
    VALU write of an SGPR -> VALU read: 2 wait states; -> SALU read: 1; VALU write of a VGPR ->
    DPP read of it: 2 wait states."""

    def __init__(self):
        self.ops = []

    def add(self, text, reads=(), writes=(), kind="valu"):
        self.ops.append(Op(text, reads, writes, kind))

    def add_masked(self, set_line, set_reads, text, reads=(), writes=()):
        """One VALU instruction under EXEC = a lane mask the SALU `set_line` writes from the SGPR pairs `set_reads`
        (carry / borrow masks of earlier VALU ops), EXEC restored to the saved full mask right after.  Scheduled as one
        unit; the SALU read of the mask obeys the VALU-write -> SALU-read wait state.  Back-to-back masked units drop
        the restore between them (masked_peephole)."""
        op = Op([set_line, text, EXEC_RESTORE], list(reads) + list(set_reads), writes)
        for r in set_reads:
            op.mask_reads.update(expand(r))
        self.ops.append(op)

    def schedule(self):
        ops = self.ops
        last_w, readers = {}, {}
        for op in ops:
            for r in op.reads:
                if r in last_w:
                    op.preds.add(last_w[r])
            for w in op.writes:
                if w in ("s24", "s25"):
                    continue
                if w in last_w:
                    op.preds.add(last_w[w])
                for rd in readers.get(w, []):
                    if rd is not op:
                        op.preds.add(rd)
            for r in op.reads:
                readers.setdefault(r, []).append(op)
            for w in op.writes:
                if w in ("s24", "s25"):
                    continue
                last_w[w] = op
                readers[w] = []
        for op in ops:
            for p in op.preds:
                p.succs.add(op)
        for op in reversed(ops):
            op.prio = op.cost + max((s.prio for s in op.succs), default=0.0)
        # producers of each read register (for hazards)
        prod = {}
        lw = {}
        for op in ops:
            for r in op.reads:
                if r in lw:
                    prod[(op, r)] = lw[r]
            for w in op.writes:
                lw[w] = op
        done, out, issued = set(), [], {}
        remaining = list(ops)
        slot = 0
        while remaining:
            best = None
            for op in remaining:
                if not all(p in done for p in op.preds):
                    continue
                ok = True
                for r in op.reads:
                    p = prod.get((op, r))
                    if p is None or p.kind == "salu":
                        continue
                    if r[0] == "s" or r == "vcc":
                        need = 2 if op.kind == "salu" else 3
                        if r in op.mask_reads:  # a VALU-written carry mask read by the SALU that sets EXEC
                            need = max(2, MASK_LATENCY)
                    elif op.kind == "dpp":
                        need = 3
                    else:
                        continue
                    if slot - issued[p] < need:
                        ok = False
                        break
                if not ok:
                    continue
                key = (op.prio, -op.idx)
                if best is None or key > bkey:
                    best, bkey = op, key
            if best is None:
                out.append("s_nop 0")
                slot += 1
                continue
            if isinstance(best.text, list):
                out.extend(best.text)
            else:
                out.append(best.text)
            issued[best] = slot
            slot += 1
            done.add(best)
            remaining.remove(best)
        return merge_nops(masked_peephole(out))

    def emit_in_order(self):
        out = []
        for op in self.ops:
            out.extend(op.text if isinstance(op.text, list) else [op.text])
        return out


def masked_peephole(lines):
    """Drop an EXEC restore that the next instruction overwrites (two masked units back to back)."""
    res = []
    for i, l in enumerate(lines):
        if l == EXEC_RESTORE and i + 1 < len(lines) and lines[i + 1].split(" ")[1:2] == ["exec,"]:
            continue
        res.append(l)
    return res


def merge_nops(lines):
    res, run = [], 0
    for l in lines + ["<end>"]:
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


# ------------------------------------------------------------------------------------------------
class Slot:
    """8 scratch VGPRs (4 pairs) + 3 SGPR carry pairs."""

    def __init__(self, vbase, sbase):
        self.v = [f"v{vbase + i}" for i in range(8)]
        self.P = [pv(vbase + 2 * i) for i in range(4)]
        self.c = [f"s[{sbase + 2 * i}:{sbase + 2 * i + 1}]" for i in range(3)]


class MulSlot:
    """12 scratch VGPRs (6 aligned pairs: vbase.. contiguous, or an explicit register list) for a general
    multiply + 2 SGPR carry pairs."""

    def __init__(self, vbase, sbase, regs=None):
        regs = regs if regs is not None else list(range(vbase, vbase + 12))
        assert len(regs) == 12 and all(regs[2 * i] % 2 == 0 and regs[2 * i + 1] == regs[2 * i] + 1 for i in range(6))
        self.v = [f"v{r}" for r in regs]
        self.P = [pv(regs[2 * i]) for i in range(6)]
        self.c = [f"s[{sbase + 2 * i}:{sbase + 2 * i + 1}]" for i in range(2)]


def X(dmap, r):
    b = dmap[r]
    return f"v{b}", f"v{b + 1}", pv(b)


def tmul(sg, S, xlo, xhi, xp, sl, tlo, thi):
    """canonical t (tlo:thi) with x * 2^S = (neg ? -t : t)."""
    e = S % 96
    neg = (S >= 96) != (e >= 64)
    v, P, c = sl.v, sl.P, sl.c
    if e == 0:
        sg.add(f"v_mad_u64_u32 {P[0]}, {c[1]}, -1, 1, {xp}", [xp], [P[0], c[1]])
        sg.add(f"v_cndmask_b32_e64 {tlo}, {xlo}, {v[0]}, {c[1]}", [xlo, v[0], c[1]], [tlo])
        sg.add(f"v_cndmask_b32_e64 {thi}, {xhi}, {v[1]}, {c[1]}", [xhi, v[1], c[1]], [thi])
        return neg
    if e < 64:
        r = e if e <= 32 else e - 32
        sg.add(f"v_lshlrev_b64 {P[0]}, {r}, {xp}", [xp], [P[0]])
        if r == 32:
            h = xhi
        else:
            h = v[4]
            sg.add(f"v_lshrrev_b32 {h}, {32 - r}, {xhi}", [xhi], [h])
        sg.add(f"v_mad_u64_u32 {P[1]}, {c[0]}, {h}, -1, {P[0]}", [h, P[0]], [P[1], c[0]])
        if e > 32:
            times_2_32(sg, sl)
        sg.add(f"v_mad_u64_u32 {P[0]}, {c[1]}, -1, 1, {P[1]}", [P[1]], [P[0], c[1]])
        sg.add(f"s_or_b64 {c[1]}, {c[1]}, {c[0]}", [c[1], c[0]], [c[1], "scc"], "salu")
        sg.add(f"v_cndmask_b32_e64 {tlo}, {v[2]}, {v[0]}, {c[1]}", [v[2], v[0], c[1]], [tlo])
        sg.add(f"v_cndmask_b32_e64 {thi}, {v[3]}, {v[1]}, {c[1]}", [v[3], v[1], c[1]], [thi])
        return neg
    K = 96 - e
    sg.add(f"v_lshrrev_b64 {P[0]}, {K}, {xp}", [xp], [P[0]])
    if K == 32:
        u = xlo
    else:
        u = v[4]
        sg.add(f"v_lshlrev_b32 {u}, {32 - K}, {xlo}", [xlo], [u])
    sg.add(f"v_mad_u64_u32 {P[1]}, {JUNK}, {u}, 1, {P[0]}", [u, P[0]], [P[1], JUNK])
    sg.add(f"v_sub_co_u32_e64 {v[3]}, {c[0]}, {v[3]}, {u}", [v[3], u], [v[3], c[0]])
    sg.add(f"v_cndmask_b32_e64 {v[5]}, 0, -15, {c[0]}", [c[0]], [v[5]])
    tp = pair_of(tlo, thi)
    sg.add(f"v_mad_i64_i32 {tp}, {JUNK}, {v[5]}, s{S_X15}, {P[1]}", [v[5], P[1]], [tp, tlo, thi, JUNK])
    return neg


def times_2_32_r2(sg, sl):
    """The r2 form of times_2_32 (carry folded first, then the (y_lo : 0) pair by two moves), kept for A/B runs."""
    v, P, c = sl.v, sl.P, sl.c
    sg.add(f"v_cndmask_b32_e64 {v[4]}, 0, -1, {c[0]}", [c[0]], [v[4]])
    sg.add(f"v_mad_u64_u32 {P[0]}, {JUNK}, {v[4]}, 1, {P[1]}", [v[4], P[1]], [P[0], JUNK])
    sg.add(f"v_mov_b32 {v[6]}, 0", [], [v[6]])
    sg.add(f"v_mov_b32 {v[7]}, {v[0]}", [v[0]], [v[7]])
    sg.add(f"v_mad_u64_u32 {P[1]}, {c[0]}, {v[1]}, -1, {P[3]}", [v[1], P[3]], [P[1], c[0]])


def times_2_32(sg, sl):
    """P1 <- y 2^32 mod p (not canonical, carry in c0) for y = P1 + c0 2^64 (the unfolded result of a shift, carry
    in c0): y 2^32 = P1_lo 2^32 + P1_hi 2^64 + c0 2^96 = (P1_lo : 0) + P1_hi EPS - c0.  The -c0 goes into the high
    word: (P1_lo - c0 : 0) + (P1_hi + c0') EPS with the borrow b of P1_lo - c0 and c0' = c0 & ~b, since EPS - 2^32 = -1
    (and when P1_lo = 0 the word wraps to 2^32 - 1 with b set: (2^32 - 1) 2^32 = -1 + p).  P1_hi + c0' never wraps
    (y < 2^63 whenever c0 is set).  5 VALU + 1 SALU instead of folding the carry first (cndmask + mad) and moving
    y_lo into a (y_lo : 0) pair."""
    if not CLASS1_FOLD:
        return times_2_32_r2(sg, sl)
    v, P, c = sl.v, sl.P, sl.c
    sg.add(f"v_mov_b32 {v[6]}, 0", [], [v[6]])
    sg.add(f"v_subb_co_u32_e64 {v[7]}, {c[1]}, {v[2]}, 0, {c[0]}", [v[2], c[0]], [v[7], c[1]])
    sg.add(f"s_andn2_b64 {c[0]}, {c[0]}, {c[1]}", [c[0], c[1]], [c[0], "scc"], "salu")
    sg.add(f"v_addc_co_u32_e64 {v[4]}, {JUNK}, {v[3]}, 0, {c[0]}", [v[3], c[0]], [v[4], JUNK])
    sg.add(f"v_mad_u64_u32 {P[1]}, {c[0]}, {v[4]}, -1, {P[3]}", [v[4], P[3]], [P[1], c[0]])


def add_part1(sg, sl, alo, ahi, tlo, thi):
    v, c = sl.v, sl.c
    sg.add(f"v_add_co_u32_e64 {v[0]}, {c[2]}, {alo}, {tlo}", [alo, tlo], [v[0], c[2]])
    sg.add(f"v_addc_co_u32_e64 {v[1]}, {c[2]}, {ahi}, {thi}, {c[2]}", [ahi, thi, c[2]], [v[1], c[2]])


def add_part2(sg, sl, dp):
    v, P, c = sl.v, sl.P, sl.c
    sg.add(f"v_cndmask_b32_e64 {v[5]}, 0, -1, {c[2]}", [c[2]], [v[5]])
    sg.add(f"v_mad_u64_u32 {dp}, {JUNK}, {v[5]}, 1, {P[0]}", [v[5], P[0]], [dp, JUNK])


def pair_of(lo, hi):
    a, b = int(lo[1:]), int(hi[1:])
    assert b == a + 1 and a % 2 == 0, (lo, hi)
    return pv(a)


def minus_eps(sg, m, c, dp):
    """dp <- dp - EPS where the SGPR mask c is set (a borrow: + p mod 2^64): m = c ? -15 : 0, then
    dp += m * 0x11111111 (signed 32 x 32 + 64).  EXEC_MASK: one masked v_mad_i64_i32 (m unused)."""
    if EXEC_MASK:
        minus_eps_masked(sg, c, dp)
        return
    sg.add(f"v_cndmask_b32_e64 {m}, 0, -15, {c}", [c], [m])
    sg.add(f"v_mad_i64_i32 {dp}, {JUNK}, {m}, s{S_X15}, {dp}", [m, dp], [dp, JUNK])


def sub_seq(sg, sl, dlo, dhi, alo, ahi, tlo, thi):
    v, c = sl.v, sl.c
    sg.add(f"v_sub_co_u32_e64 {dlo}, {c[0]}, {alo}, {tlo}", [alo, tlo], [dlo, c[0]])
    sg.add(f"v_subb_co_u32_e64 {dhi}, {c[1]}, {ahi}, {thi}, {c[0]}", [ahi, thi, c[0]], [dhi, c[1]])
    minus_eps(sg, v[4], c[1], pair_of(dlo, dhi))


def ct_core(sg, sl, a, b, neg, tsrc=None):
    """t in sl.v2:v3 (or tsrc) canonical; a, b = (lo, hi, pair)."""
    if EXEC_MASK:
        if tsrc:
            assert tsrc == (b[0], b[1]), tsrc
            return ct_x(sg, sl, a, b, 96 if neg else 0, b_canon=True)
        return ct_core_x(sg, sl, a, b, neg, (sl.v[2], sl.v[3]))
    alo, ahi, ap = a
    blo, bhi, bp = b
    tlo, thi = tsrc if tsrc else (sl.v[2], sl.v[3])
    # t may alias b (tsrc: twiddle +-1 on a canonical b): the sum reads it first, and the subtraction that overwrites
    # b reads each word of it in the instruction that writes that word, so no copy is needed (the list scheduler
    # keeps the sum's reads ahead of the overwrite: a write waits for every earlier reader of its register)
    if tsrc and ALIAS_COPY:  # r2 form (tools/variant_probe A/B)
        sg.add(f"v_mov_b32 {sl.v[2]}, {tlo}", [tlo], [sl.v[2]])
        sg.add(f"v_mov_b32 {sl.v[3]}, {thi}", [thi], [sl.v[3]])
        tlo, thi = sl.v[2], sl.v[3]
    add_part1(sg, sl, alo, ahi, tlo, thi)
    if not neg:
        sub_seq(sg, sl, blo, bhi, alo, ahi, tlo, thi)
        add_part2(sg, sl, ap)
    else:
        sub_seq(sg, sl, alo, ahi, alo, ahi, tlo, thi)
        add_part2(sg, sl, bp)


def ct_core_canon(sg, sl, a, b, neg):
    """ct_core for a canonical a and the canonical t in sl.v2:v3, with canonical outputs: the difference of
    two canonical values needs only the borrow fix (sub_seq), and their sum is canonical after one select
    between s and U = s + EPS (U when the add carried, s + 2^64 = U mod p, or when U carried, s >= p)."""
    if EXEC_MASK:
        return ct_core_x(sg, sl, a, b, neg, (sl.v[2], sl.v[3]), canon_out=True)
    alo, ahi, ap = a
    blo, bhi, bp = b
    v, P, c = sl.v, sl.P, sl.c
    tlo, thi = v[2], v[3]
    add_part1(sg, sl, alo, ahi, tlo, thi)                 # s = a + t in P0, carry c2
    if not neg:
        sub_seq(sg, sl, blo, bhi, alo, ahi, tlo, thi)      # b = a - t
        dlo, dhi = alo, ahi
    else:
        sub_seq(sg, sl, alo, ahi, alo, ahi, tlo, thi)      # a = a - t (t stands for -w b)
        dlo, dhi = blo, bhi
    sg.add(f"v_mad_u64_u32 {P[3]}, {c[0]}, -1, 1, {P[0]}", [P[0]], [P[3], c[0]])
    sg.add(f"s_or_b64 {c[0]}, {c[0]}, {c[2]}", [c[0], c[2]], [c[0], "scc"], "salu")
    sg.add(f"v_cndmask_b32_e64 {dlo}, {v[0]}, {v[6]}, {c[0]}", [v[0], v[6], c[0]], [dlo])
    sg.add(f"v_cndmask_b32_e64 {dhi}, {v[1]}, {v[7]}, {c[0]}", [v[1], v[7], c[0]], [dhi])


def ct(sg, sl, a, b, S):
    if EXEC_MASK:
        return ct_x(sg, sl, a, b, S)
    neg = tmul(sg, S, b[0], b[1], b[2], sl, sl.v[2], sl.v[3])
    ct_core(sg, sl, a, b, neg)


def gs_core(sg, sl, a, b):
    """a' = a + b, b <- a - b (both semi in, semi out); b canonicalised first."""
    alo, ahi, ap = a
    blo, bhi, bp = b
    v, P, c = sl.v, sl.P, sl.c
    sg.add(f"v_mad_u64_u32 {P[3]}, {c[1]}, -1, 1, {bp}", [bp], [P[3], c[1]])
    sg.add(f"v_cndmask_b32_e64 {v[2]}, {blo}, {v[6]}, {c[1]}", [blo, v[6], c[1]], [v[2]])
    sg.add(f"v_cndmask_b32_e64 {v[3]}, {bhi}, {v[7]}, {c[1]}", [bhi, v[7], c[1]], [v[3]])
    add_part1(sg, sl, alo, ahi, v[2], v[3])
    sub_seq(sg, sl, blo, bhi, alo, ahi, v[2], v[3])
    add_part2(sg, sl, ap)


def gs(sg, sl, a, b, S, ac=False, bc=False):
    """GS butterfly (a, b) -> (a + b, (a - b) w), w = 2^S; ac / bc: whether a / b are known canonical.

    The subtraction needs a canonical subtrahend and the sign of w decides which operand that is:
    (a - b) w = (b - a) |w| when w < 0, so the subtrahend is b for w > 0 and a for w < 0.  That operand is
    canonicalised in place when it is not known canonical (a + b only needs one canonical operand, the
    same one), so the new b is always the canonical, positive tmul magnitude: no negation is ever
    emitted.  When both inputs are canonical the sum is made canonical too (one select after the add:
    +1 VALU, and the next stage needs no canonicalisation).  Returns (new a canonical, new b canonical)."""
    if EXEC_MASK:
        return gs_x(sg, sl, a, b, S, ac, bc)
    alo, ahi, ap = a
    blo, bhi, bp = b
    v, P, c = sl.v, sl.P, sl.c
    e = S % 96
    neg = (S >= 96) != (e >= 64)
    if ac and bc:
        add_part1(sg, sl, alo, ahi, blo, bhi)              # s = a + b in P0, carry c2
        if neg:
            sub_seq(sg, sl, blo, bhi, blo, bhi, alo, ahi)  # d = b - a
        else:
            sub_seq(sg, sl, blo, bhi, alo, ahi, blo, bhi)  # d = a - b
        sg.add(f"v_mad_u64_u32 {P[3]}, {c[0]}, -1, 1, {P[0]}", [P[0]], [P[3], c[0]])
        sg.add(f"s_or_b64 {c[0]}, {c[0]}, {c[2]}", [c[0], c[2]], [c[0], "scc"], "salu")
        sg.add(f"v_cndmask_b32_e64 {alo}, {v[0]}, {v[6]}, {c[0]}", [v[0], v[6], c[0]], [alo])
        sg.add(f"v_cndmask_b32_e64 {ahi}, {v[1]}, {v[7]}, {c[0]}", [v[1], v[7], c[0]], [ahi])
        tmul(sg, S, blo, bhi, bp, sl, blo, bhi)
        return True, True
    sub_a = neg  # subtrahend: a when w < 0 (d = b - a), b otherwise (d = a - b)
    if sub_a and not ac:
        canon(sg, sl, a)
    if not sub_a and not bc:
        canon(sg, sl, b)
    if sub_a:
        add_part1(sg, sl, blo, bhi, alo, ahi)          # s = b + a (a canonical)
        sub_seq(sg, sl, blo, bhi, blo, bhi, alo, ahi)  # d = b - a
    else:
        add_part1(sg, sl, alo, ahi, blo, bhi)          # s = a + b (b canonical)
        sub_seq(sg, sl, blo, bhi, alo, ahi, blo, bhi)  # d = a - b
    add_part2(sg, sl, ap)
    tmul(sg, S, blo, bhi, bp, sl, blo, bhi)  # |w| d, canonical; the sign is absorbed by the orientation
    return False, True


def scaled_ct(sg, sl, dmap, ra, rb, S, mode, scales, canon):
    """CT butterfly on logical registers (ra, rb), twiddle 2^S, inputs carrying the scales (ea, eb) (register r holds
    2^scales[r] times its value).  Mode 0: t = 2^(S + ea - eb) b, outputs a + t / a - t of scale ea.  Mode 1:
    t = 2^(eb - S - ea) a, outputs t + b = 2^(eb - S) (a + 2^S b) to position ra and b - t = -2^(eb - S) (a - 2^S b)
    to position rb (scale eb - S + 96), each into the register of its position (under EXEC_MASK the two logical
    registers swap their physical ones instead)."""
    ea, eb = scales[ra], scales[rb]
    a, b = X(dmap, ra), X(dmap, rb)
    if mode == 0:
        m = (S + ea - eb) % 192
        if m % 96 == 0 and canon[rb]:
            ct_core(sg, sl, a, b, m >= 96, tsrc=(b[0], b[1]))
        else:
            ct(sg, sl, a, b, m)
        scales[ra] = scales[rb] = ea % 192
    elif EXEC_MASK:  # the masked primitives write the sum into their first operand: the logical registers swap
        m = (eb - S - ea) % 192
        if m % 96 == 0 and canon[ra]:
            ct_core(sg, sl, b, a, m >= 96, tsrc=(a[0], a[1]))
        else:
            ct(sg, sl, b, a, m)
        dmap[ra], dmap[rb] = dmap[rb], dmap[ra]
    else:
        # ct_core's neg flag exchanges which register receives the sum: with it flipped, b + t lands in a's register
        # and b - t in b's, so the register map is unchanged (the PBS bodies' fixed MAC / inverse layout needs that)
        m = (eb - S - ea) % 192
        if m % 96 == 0 and canon[ra]:
            ct_core(sg, sl, b, a, m < 96, tsrc=(a[0], a[1]))
        else:
            neg = tmul(sg, m, a[0], a[1], a[2], sl, sl.v[2], sl.v[3])
            ct_core(sg, sl, b, a, not neg)
        scales[ra] = (eb - S) % 192
        scales[rb] = (eb - S + 96) % 192
    canon[ra] = canon[rb] = False


def gmul(sg, ms, x, wlo, whi, olo, ohi, zero_hi=True):
    """o = x * w canonical (x semi, w canonical), general 64x64 multiply (17 VALU; 15 with
    zero_hi=False, when the caller keeps the slot's Z1h / Z2h at 0 across a run of multiplies)."""
    xlo, xhi, _ = x
    v, P, c = ms.v, ms.P, ms.c
    PA, PB, PC, PD, Z1, Z2 = P
    A0, A1, B0, B1, C0, C1, D0, D1, Z1l, Z1h, Z2l, Z2h = v
    if EXEC_MASK:
        # the same product; R = T + H0 EPS goes straight into o (every read of x is earlier), the borrow fix and
        # the canonicalising select are EXEC-masked single instructions (13 VALU)
        op = pair_of(olo, ohi)
        if zero_hi:
            sg.add(f"v_mov_b32 {Z1h}, 0", [], [Z1h])
            sg.add(f"v_mov_b32 {Z2h}, 0", [], [Z2h])
        sg.add(f"v_mad_u64_u32 {PA}, {JUNK}, {xlo}, {wlo}, 0", [xlo, wlo], [PA, JUNK])
        sg.add(f"v_mov_b32 {Z1l}, {A1}", [A1], [Z1l])
        sg.add(f"v_mad_u64_u32 {PB}, {JUNK}, {xlo}, {whi}, {Z1}", [xlo, whi, Z1], [PB, JUNK])
        sg.add(f"v_mov_b32 {Z2l}, {B0}", [B0], [Z2l])
        sg.add(f"v_mov_b32 {Z1l}, {B1}", [B1], [Z1l])
        sg.add(f"v_mad_u64_u32 {PC}, {JUNK}, {xhi}, {wlo}, {Z2}", [xhi, wlo, Z2], [PC, JUNK])
        sg.add(f"v_mad_u64_u32 {PD}, {JUNK}, {xhi}, {whi}, {Z1}", [xhi, whi, Z1], [PD, JUNK])
        sg.add(f"v_mad_u64_u32 {PB}, {JUNK}, {C1}, 1, {PD}", [C1, PD], [PB, JUNK])          # H = D + C.hi
        sg.add(f"v_sub_co_u32_e64 {D0}, {c[0]}, {A0}, {B1}", [A0, B1], [D0, c[0]])          # T = L - H1
        sg.add(f"v_subb_co_u32_e64 {D1}, {c[1]}, {C0}, 0, {c[0]}", [C0, c[0]], [D1, c[1]])
        minus_eps_masked(sg, c[1], PD)
        sg.add(f"v_mad_u64_u32 {op}, {c[0]}, {B0}, -1, {PD}", [B0, PD], [op, c[0]])         # R = T + H0 EPS
        sg.add(f"v_mad_u64_u32 {PC}, {c[1]}, -1, 1, {op}", [op], [PC, c[1]])                # U = R + EPS
        mov64_masked(sg, ("or", c[1], c[0]), op, PC)
        return
    if zero_hi:
        sg.add(f"v_mov_b32 {Z1h}, 0", [], [Z1h])
        sg.add(f"v_mov_b32 {Z2h}, 0", [], [Z2h])
    sg.add(f"v_mad_u64_u32 {PA}, {JUNK}, {xlo}, {wlo}, 0", [xlo, wlo], [PA, JUNK])
    sg.add(f"v_mov_b32 {Z1l}, {A1}", [A1], [Z1l])
    sg.add(f"v_mad_u64_u32 {PB}, {JUNK}, {xlo}, {whi}, {Z1}", [xlo, whi, Z1], [PB, JUNK])
    sg.add(f"v_mov_b32 {Z2l}, {B0}", [B0], [Z2l])
    sg.add(f"v_mov_b32 {Z1l}, {B1}", [B1], [Z1l])
    sg.add(f"v_mad_u64_u32 {PC}, {JUNK}, {xhi}, {wlo}, {Z2}", [xhi, wlo, Z2], [PC, JUNK])
    sg.add(f"v_mad_u64_u32 {PD}, {JUNK}, {xhi}, {whi}, {Z1}", [xhi, whi, Z1], [PD, JUNK])
    sg.add(f"v_mad_u64_u32 {PB}, {JUNK}, {C1}, 1, {PD}", [C1, PD], [PB, JUNK])          # H = D + C.hi
    sg.add(f"v_sub_co_u32_e64 {D0}, {c[0]}, {A0}, {B1}", [A0, B1], [D0, c[0]])          # T = L - H1
    sg.add(f"v_subb_co_u32_e64 {D1}, {c[1]}, {C0}, 0, {c[0]}", [C0, c[0]], [D1, c[1]])
    minus_eps(sg, Z2l, c[1], PD)
    sg.add(f"v_mad_u64_u32 {PA}, {c[0]}, {B0}, -1, {PD}", [B0, PD], [PA, c[0]])         # R = T + H0 EPS
    sg.add(f"v_mad_u64_u32 {PC}, {c[1]}, -1, 1, {PA}", [PA], [PC, c[1]])                # U = R + EPS
    sg.add(f"s_or_b64 {c[1]}, {c[1]}, {c[0]}", [c[1], c[0]], [c[1], "scc"], "salu")
    sg.add(f"v_cndmask_b32_e64 {olo}, {A0}, {C0}, {c[1]}", [A0, C0, c[1]], [olo])
    sg.add(f"v_cndmask_b32_e64 {ohi}, {A1}, {C1}, {c[1]}", [A1, C1, c[1]], [ohi])


def canon(sg, sl, x):
    xlo, xhi, xp = x
    v, P, c = sl.v, sl.P, sl.c
    if EXEC_MASK:
        sg.add(f"v_mad_u64_u32 {P[0]}, {c[1]}, -1, 1, {xp}", [xp], [P[0], c[1]])
        mov64_masked(sg, c[1], xp, P[0])
        return
    sg.add(f"v_mad_u64_u32 {P[0]}, {c[1]}, -1, 1, {xp}", [xp], [P[0], c[1]])
    sg.add(f"v_cndmask_b32_e64 {xlo}, {xlo}, {v[0]}, {c[1]}", [xlo, v[0], c[1]], [xlo])
    sg.add(f"v_cndmask_b32_e64 {xhi}, {xhi}, {v[1]}, {c[1]}", [xhi, v[1], c[1]], [xhi])


# ------------------------------------------------------------------------------------------------
# The scale plan (r5, tools/tw_scale_plan.py): the forward's in-register butterfly networks carry power-of-two scales
# that the twist table absorbs, so each butterfly may multiply whichever input makes the cheaper shift class.  The
# plan's table side (ntt64_tw_tables.hpp TW_G1_OUT_SCALE / TW_CYC_IN_SCALE) is generated from the same JSON.
SCALE_PLAN = True
_PLAN = None


def scale_plan():
    global _PLAN
    if not SCALE_PLAN:
        return None
    if _PLAN is None:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import tw_scale_plan
        _PLAN = tw_scale_plan.load()
    return _PLAN


# ------------------------------------------------------------------------------------------------
# EXEC-masked arithmetic (r5).  Every conditional step of the Goldilocks arithmetic (fold a carry: + EPS; fix a
# borrow: - EPS; canonicalise: select x + EPS) was a VALU select (v_cndmask on the carry mask, 4.3 cycles per 32-bit
# word) feeding a multiply-add, or a pair of selects.  Here the carry mask goes into EXEC through the SALU (off the
# VALU issue path) and the step is ONE VALU instruction on the lanes that need it: a fold or a borrow fix is one
# v_mad (4.6 instead of 8.9 cycles), a select one v_mov_b64 (4.2 instead of 8.6).  Every result is written in
# place, so the butterflies also need no sum / difference temporaries.  The arithmetic is unchanged: same values,
# lane by lane (the emulator tests and the GPU parity tests check it).
EXEC_MASK = False  # measured slower on MI355X (r5, tools/variant_probe): see DESIGN.md §4
MASK_LATENCY = 2   # list-scheduler slots between a VALU carry write and the SALU EXEC write that reads it


def cond_exec(cond):
    """(SALU line writing EXEC, SGPR pairs it reads) for cond = an SGPR pair, ("or", c1, c0) or ("not", c)."""
    if isinstance(cond, tuple):
        if cond[0] == "or":
            return f"s_or_b64 exec, {cond[1]}, {cond[2]}", [cond[1], cond[2]]
        return f"s_not_b64 exec, {cond[1]}", [cond[1]]
    return f"s_mov_b64 exec, {cond}", [cond]


def mov64_masked(sg, cond, dst, src):
    """dst <- src (u64 pairs) on the lanes of cond."""
    line, sr = cond_exec(cond)
    sg.add_masked(line, sr, f"v_mov_b64 {dst}, {src}", [src, dst], [dst])


def plus_eps_masked(sg, cond, dp):
    """dp += EPS on the lanes of cond (the fold of a carry out of bit 64: 2^64 = EPS mod p)."""
    line, sr = cond_exec(cond)
    sg.add_masked(line, sr, f"v_mad_u64_u32 {dp}, {JUNK}, -1, 1, {dp}", [dp], [dp, JUNK])


def minus_eps_masked(sg, cond, dp):
    """dp -= EPS on the lanes of cond (a borrow out of bit 64: d - 2^64 = d - EPS mod p); -15 * 0x11111111 = -EPS."""
    line, sr = cond_exec(cond)
    sg.add_masked(line, sr, f"v_mad_i64_i32 {dp}, {JUNK}, -15, s{S_X15}, {dp}", [dp], [dp, JUNK])


def tmul_x(sg, S, x, sl, T, copy_u=False):
    """T (an aligned pair, may be x itself) <- canonical t with x * 2^S = (neg ? -t : t); returns neg.  Scratch: the
    slot's P0, v4 and (class 1) P3, carry pairs c0 / c1.  The raw product goes straight into T, so x may be T: every
    read of x precedes the first write of T in program order (the scheduler keeps that order)."""
    xlo, xhi, xp = x
    tlo, thi = T
    tp = pair_of(tlo, thi)
    e = S % 96
    neg = (S >= 96) != (e >= 64)
    v, P, c = sl.v, sl.P, sl.c
    if e == 0:
        if tp == xp:
            canon(sg, sl, x)
        else:
            sg.add(f"v_mad_u64_u32 {tp}, {c[1]}, -1, 1, {xp}", [xp], [tp, c[1]])   # T = x + EPS
            mov64_masked(sg, ("not", c[1]), tp, xp)                                # x < p: T = x
        return neg
    if e < 64:
        r = e if e <= 32 else e - 32
        sg.add(f"v_lshlrev_b64 {P[0]}, {r}, {xp}", [xp], [P[0]])
        if r == 32:
            h = xhi
        else:
            h = v[4]
            sg.add(f"v_lshrrev_b32 {h}, {32 - r}, {xhi}", [xhi], [h])
        sg.add(f"v_mad_u64_u32 {tp}, {c[0]}, {h}, -1, {P[0]}", [h, P[0]], [tp, c[0]])   # x 2^r = T + c0 2^64
        if e > 32:
            # y = x 2^r folded (T < (2^32 - 1)^2 when c0: no second wrap), then y 2^32 = (y_lo << 32) + y_hi EPS
            plus_eps_masked(sg, c[0], tp)
            sg.add(f"v_lshlrev_b64 {P[3]}, 32, {tp}", [tp], [P[3]])
            sg.add(f"v_mad_u64_u32 {tp}, {c[0]}, {thi}, -1, {P[3]}", [thi, P[3]], [tp, c[0]])
        sg.add(f"v_mad_u64_u32 {P[0]}, {c[1]}, -1, 1, {tp}", [tp], [P[0], c[1]])        # U = T + EPS
        mov64_masked(sg, ("or", c[1], c[0]), tp, P[0])                                  # canonical: U if a carry
        return neg
    K = 96 - e
    sg.add(f"v_lshrrev_b64 {P[0]}, {K}, {xp}", [xp], [P[0]])
    if K == 32 and tp != xp:
        u = xlo
    else:
        u = v[4]
        if K == 32:
            sg.add(f"v_mov_b32 {u}, {xlo}", [xlo], [u])
        else:
            sg.add(f"v_lshlrev_b32 {u}, {32 - K}, {xlo}", [xlo], [u])
    sg.add(f"v_mad_u64_u32 {tp}, {JUNK}, {u}, 1, {P[0]}", [u, P[0]], [tp, JUNK])
    sg.add(f"v_sub_co_u32_e64 {thi}, {c[0]}, {thi}, {u}", [thi, u], [thi, c[0]])
    minus_eps_masked(sg, c[0], tp)
    return neg


def ct_core_x(sg, sl, a, b, neg, t, canon_out=False):
    """In-place CT butterfly with the canonical t (= w b, or its negation when neg): not neg: b <- a - t, a <- a + t;
    neg: b <- a + t, a <- a - t.  The destination of the first result is dead (its value is in t), so nothing needs a
    temporary.  canon_out (a canonical): both outputs canonical (the sum by a select between s and s + EPS)."""
    alo, ahi, ap = a
    blo, bhi, bp = b
    tlo, thi = t
    c = sl.c
    S, D = (b, a) if neg else (a, b)

    def diff(dst):
        sg.add(f"v_sub_co_u32_e64 {dst[0]}, {c[0]}, {alo}, {tlo}", [alo, tlo], [dst[0], c[0]])
        sg.add(f"v_subb_co_u32_e64 {dst[1]}, {c[1]}, {ahi}, {thi}, {c[0]}", [ahi, thi, c[0]], [dst[1], c[1]])
        minus_eps_masked(sg, c[1], dst[2])

    def add(dst):
        sg.add(f"v_add_co_u32_e64 {dst[0]}, {c[2]}, {alo}, {tlo}", [alo, tlo], [dst[0], c[2]])
        sg.add(f"v_addc_co_u32_e64 {dst[1]}, {c[2]}, {ahi}, {thi}, {c[2]}", [ahi, thi, c[2]], [dst[1], c[2]])
        if canon_out:
            P3 = sl.P[3]
            sg.add(f"v_mad_u64_u32 {P3}, {c[0]}, -1, 1, {dst[2]}", [dst[2]], [P3, c[0]])
            mov64_masked(sg, ("or", c[0], c[2]), dst[2], P3)
        else:
            plus_eps_masked(sg, c[2], dst[2])

    # the dead destination first (b, whose value t carries), then the other one in place
    if neg:
        add(S)
        diff(D)
    else:
        diff(D)
        add(S)


def ct_x(sg, sl, a, b, S, b_canon=False):
    """CT butterfly (a, b) with twiddle 2^S: t = 2^S b canonical in the slot's P1, then ct_core_x."""
    t = (sl.v[2], sl.v[3])
    if S % 96 == 0 and b_canon:
        sg.add(f"v_mov_b64 {sl.P[1]}, {b[2]}", [b[2]], [sl.P[1]])
        neg = S >= 96
    else:
        neg = tmul_x(sg, S, b, sl, t)
    ct_core_x(sg, sl, a, b, neg, t)


def gs_x(sg, sl, a, b, S, ac=False, bc=False):
    """EXEC-masked gs (same contract): the difference goes to the slot's P1, the sum into a in place, then
    b <- |w| (difference) canonical (tmul_x from P1 into b)."""
    alo, ahi, ap = a
    blo, bhi, bp = b
    c, P = sl.c, sl.P
    dl, dh, dpair = sl.v[2], sl.v[3], P[1]
    e = S % 96
    neg = (S >= 96) != (e >= 64)
    both = ac and bc
    if not both:
        if neg and not ac:
            canon(sg, sl, a)
        if not neg and not bc:
            canon(sg, sl, b)
    # difference (the subtrahend is canonical): a - b, or b - a when the twiddle is negative
    m, s_ = (b, a) if neg else (a, b)
    sg.add(f"v_sub_co_u32_e64 {dl}, {c[0]}, {m[0]}, {s_[0]}", [m[0], s_[0]], [dl, c[0]])
    sg.add(f"v_subb_co_u32_e64 {dh}, {c[1]}, {m[1]}, {s_[1]}, {c[0]}", [m[1], s_[1], c[0]], [dh, c[1]])
    minus_eps_masked(sg, c[1], dpair)
    # sum into a in place
    sg.add(f"v_add_co_u32_e64 {alo}, {c[2]}, {alo}, {blo}", [alo, blo], [alo, c[2]])
    sg.add(f"v_addc_co_u32_e64 {ahi}, {c[2]}, {ahi}, {bhi}, {c[2]}", [ahi, bhi, c[2]], [ahi, c[2]])
    if both:
        sg.add(f"v_mad_u64_u32 {P[3]}, {c[0]}, -1, 1, {ap}", [ap], [P[3], c[0]])
        mov64_masked(sg, ("or", c[0], c[2]), ap, P[3])
    else:
        plus_eps_masked(sg, c[2], ap)
    tmul_x(sg, S, (dl, dh, dpair), sl, (blo, bhi))
    return both, True


# ------------------------------------------------------------------------------------------------
class Body:
    def __init__(self, tabs):
        self.tabs = tabs
        self.lines = []
        self.nvalu = 0
        # the per-block tally (tools/valu_cost.py --blocks): `tag` names the block being emitted; blocks[tag] holds its
        # lines, bfly[(tag, exponent mod 192)] the lines of each butterfly of a stage before scheduling
        self.tag = "setup"
        self.blocks, self.bfly = {}, {}

    def out(self, lines):
        self.lines += lines
        self.nvalu += sum(1 for l in lines if l.startswith("v_"))
        self.blocks.setdefault(self.tag, []).extend(lines)

    def raw(self, *lines):
        self.out(list(lines))

    # slots from a list of free 8-register blocks
    @staticmethod
    def slots(free_blocks, n=None):
        sl = []
        for i, b in enumerate(free_blocks[: n or len(free_blocks)]):
            sl.append(Slot(b, SG0 + 6 * i))
        return sl

    def stage(self, kind, dist, exps, dmap, free_blocks, canon=None, by_reg=False, group_waits=None, modes=None,
              scales=None):
        """canon: list of 32 flags (logical registers known canonical), updated in place.  The twiddle
        exponent of the butterfly on registers (r, r + dist) is exps[r // (2 dist)] (one per group, the
        natural-in CT / GS stages), or exps[r] with by_reg (one per position, the DIT stages).
        modes / scales (CT only, the scale plan of tools/tw_scale_plan.py): scales[r] is the power-of-two exponent
        logical register r carries (updated in place); butterfly k of the stage multiplies b (mode 0) or a (mode 1),
        see scaled_ct."""
        sg = Seg()
        slots = self.slots(free_blocks)
        bf = 0
        if canon is None:
            canon = [False] * 32
        for r in range(32):
            if r & dist:
                continue
            if group_waits and bf % 4 == 0:  # flush the previous group, wait for the next group's rows
                for i, op in enumerate(sg.ops):
                    op.idx = i
                self.out(sg.schedule())
                self.raw(group_waits[bf // 4])
                sg = Seg()
            S = exps[r] if by_reg else exps[r // (2 * dist)]
            sl = slots[bf % len(slots)]
            a, b = X(dmap, r), X(dmap, r + dist)
            n0 = len(sg.ops)
            if kind == "ct" and modes is not None:
                scaled_ct(sg, sl, dmap, r, r + dist, S, modes[bf], scales, canon)
            elif kind == "ct":
                if S % 96 == 0 and canon[r + dist]:
                    ct_core(sg, sl, a, b, S >= 96, tsrc=(b[0], b[1]))
                else:
                    ct(sg, sl, a, b, S)
                canon[r] = canon[r + dist] = False
            else:
                canon[r], canon[r + dist] = gs(sg, sl, a, b, S, canon[r], canon[r + dist])
            self.bfly.setdefault((self.tag, S % 192), []).append(
                [t for op in sg.ops[n0:] for t in (op.text if isinstance(op.text, list) else [op.text])])
            bf += 1
        for i, op in enumerate(sg.ops):
            op.idx = i
        self.out(sg.schedule())

    def mulrows(self, dmap, rows, wregs, mslots, zero_hi=True):
        """x[r] = x[r] * w (general), w in wregs[k] (pair base)."""
        sg = Seg()
        for k, r in enumerate(rows):
            ms = mslots[k % len(mslots)]
            x = X(dmap, r)
            wb = wregs[k]
            gmul(sg, ms, x, f"v{wb}", f"v{wb + 1}", x[0], x[1], zero_hi)
        for i, op in enumerate(sg.ops):
            op.idx = i
        self.out(sg.schedule())


def load_tables():
    here = os.path.dirname(os.path.abspath(__file__))
    hdr = os.path.join(here, "..", "tfhe-rs-main_modified_amd", "csrc", "ntt64_tw_tables.hpp")
    tabs, cur = {}, None
    for line in open(hdr):
        line = line.strip()
        if line.startswith("constexpr int"):
            cur = line.split()[2].split("[")[0]
            tabs[cur] = []
        elif cur and line.startswith("{"):
            tabs[cur].append([int(t) for t in line.strip("{},").split(",")])
        elif line.startswith("};"):
            cur = None
    return tabs


# SGPR map (beyond the carry pairs s20..s75 of up to 7 slots)
S_GB = 78    # s[78:85]: data row-group bases g + 4096 m, m = 0..3
S_TB = 86    # s[86:93]: table bases
S_PAR = 20   # s[20:21]: odd-lane mask
S_X15 = 27   # s27 = 0x11111111 = EPS / 15: d - EPS = d + (-15) * 0x11111111 in one v_mad_i64_i32
S_EXE = 22   # s[22:23]: saved exec
EXEC_RESTORE = f"s_mov_b64 exec, s[{S_EXE}:{S_EXE + 1}]"


def bases(body, reg_g, dst):
    for m in range(4):
        body.raw(f"s_add_u32 s{dst + 2 * m}, {reg_g}[0], {4096 * m}")
    # (replaced below by proper lo/hi handling)


def gen_bases(src, dst):
    """dst pairs = src + 4096 m; src is an asm operand name for an SGPR pair."""
    lines = []
    for m in range(4):
        lines.append(f"s_add_u32 s{dst + 2 * m}, %[{src}_lo], {4096 * m}")
        lines.append(f"s_addc_u32 s{dst + 2 * m + 1}, %[{src}_hi], 0")
    return lines


# cache-policy bits appended to the data row loads / stores (gfx950: "nt", "sc0", "sc1").  Stores carry sc0 sc1
# (system scope): tools/variant_probe measured the forward 2.0 % and the 4-wave inverse 3.9 % faster per launch
# (back-to-back launches, so the dependent-launch gap is included: fewer dirty L2 lines to write back at the kernel
# boundary), sc1 alone about half of that, nt sc1 10 % slower; loads keep the default policy (nt loads were slower)
LOAD_POLICY = ""
STORE_POLICY = " sc0 sc1"
# Two instruction cuts were tried in r3 and are OFF: tools/variant_probe timed them in one process against the r2 bodies
# (profiles/r3/variant_probe_r3_changes.txt): the forward with both is 1.2 % slower (58.6 vs 57.9 us per 8192-poly
# launch) although it issues 2.8 % fewer VALU cycles by the model; the inverse is unchanged.  Dropping the two moves puts
# the subtraction right behind the add on the same registers, and the fold puts an SALU op inside the carry chain, so
# both lengthen the dependent chains the 4 resident waves per SIMD must hide.
ALIAS_COPY = True    # copy a +-1-twiddle operand before the subtraction overwrites it (2 moves; False saves them)
CLASS1_FOLD = False  # class-1 shifts: True folds the first carry into the 2^32 step (times_2_32) instead
INV_CYC_DIT = True   # inverse cyclic blocks by decimation in time (dit_exps); False: the GS form
PROGRESSIVE = True   # forward: start the first stage as the data rows arrive (4 waits) instead of one vmcnt(0):
                     # 0.6 % faster (tools/variant_probe); the same per row in the inverse's T1 was 0.8 % slower
PROGRESSIVE_INV = False
FWD_STORE = "t2"     # forward output: "t2" LDS transpose to W0 + coalesced rows; "x2" / "x4": each lane stores its
                     # 32 consecutive outputs from the lane-pair layout directly (8- / 16-byte stores, %[pso])


def load_rows(dmap, base, voff="%[l8]"):
    out = []
    for r in range(32):
        out.append(f"global_load_dwordx2 {pv(dmap[r])}, {voff}, s[{base + 2 * (r // 8)}:{base + 2 * (r // 8) + 1}] "
                   f"offset:{512 * (r % 8)}{LOAD_POLICY}")
    return out


def store_rows(dmap, base):
    out = []
    for r in range(32):
        out.append(f"global_store_dwordx2 %[l8], {pv(dmap[r])}, s[{base + 2 * (r // 8)}:{base + 2 * (r // 8) + 1}] "
                   f"offset:{512 * (r % 8)}{STORE_POLICY}")
    return out


EXEC_LO = [f"s_mov_b32 exec_hi, 0"]          # lanes 0..31 (assumes exec was all ones)
EXEC_HI = [f"s_mov_b32 exec_lo, 0", f"s_mov_b32 exec_hi, -1"]


def exec_block_half(ad, h):
    """EXEC = the lanes of blocks i in [16 h, 16 h + 16): lanes 32 h .. 32 h + 31 in the lane-pair layouts 2 i + par,
    lanes 16 h .. 16 h + 15 and 32 + 16 h .. 47 + 16 h in the W1x layouts i + 32 par (assumes exec was all ones)."""
    if getattr(ad, "w1x", False):
        m = "0xffff" if h == 0 else "0xffff0000"
        return [f"s_mov_b32 exec_lo, {m}", f"s_mov_b32 exec_hi, {m}"]
    return EXEC_LO if h == 0 else EXEC_HI
EXEC_ALL = [f"s_mov_b64 exec, s[{S_EXE}:{S_EXE + 1}]"]


class Addr:
    """Where the transform cores find their per-lane LDS addresses and tables: asm operand names in
    the standalone transform kernel, fixed registers inside bigger bodies (tools/gen_pbs_kernel.py)."""

    def __init__(self, tw_load, **regs):
        self.tw_load = tw_load    # (batch bt, row k, dst pair base) -> load line of table row 8 bt + k
        self.tw_wait = "s_waitcnt vmcnt(0)"
        self.tw_wait_n = lambda n: f"s_waitcnt vmcnt({n})"   # at most n younger table loads outstanding
        # (dst pair base, table entry k) -> load line of the lane's pair-stage twiddle k (+16 odd lanes)
        self.lw_load = lambda dst, k: f"global_load_dwordx2 {pv(dst)}, {self.lwo}, {self.lw} offset:{8 * k}"
        self.lw_wait = None   # wait after the lane-pair twiddle loads (None: tw_wait)
        self.__dict__.update(regs)


NTT_ADDR = Addr(lambda bt, k, dst: f"global_load_dwordx2 {pv(dst)}, %[l8], s[{S_TB + 2 * bt}:{S_TB + 2 * bt + 1}] "
                                   f"offset:{512 * k}",
                **{n: f"%[{n}]" for n in ("t1w", "t1r", "t2wl", "t2wh", "t2r", "t4w", "t4r", "lwo", "lw", "t1x", "t1y")})

# The forward's W1x layout (r6): the lane pair of block i is lanes i and i + 32 (lane = i + 32 j0) instead of 2 i and
# 2 i + 1, so the lane-pair stage's regroup is two v_permlane32_swap_b32 per register pair (a half-wave exchange,
# 8.2 cycles each) instead of four DPP moves and four selects (34.8 cycles).  Its transposes: T1 with row stride 33
# (reads at (i 33 + j0 + 2 q) 8: conflict-free for both 32-lane groups), T2 with row stride 65 and the halves split by
# i < 16 (lanes 0-15 and 32-47).  The per-lane addresses come from the kernel wrapper (ntt64_tw_device.hpp tw_body:
# i = lane & 31, j0 = lane >> 5); the odd-lane mask s[S_PAR] becomes the upper half-wave.
FWD_W1X = True
INV_W1X = True   # the standalone inverse bodies' W1'' blocks in the same half-wave pairing (lane = i + 32 j5)
NTT_ADDR_W1X = Addr(NTT_ADDR.tw_load, w1x=True,
                    **{n: f"%[{n}]" for n in ("t1w", "t1r", "t2wl", "t2wh", "t2r", "t4w", "t4r", "lwo", "lw", "t1x", "t1y")})


def par_mask(ad):
    """s[S_PAR:S_PAR+1] = the lanes holding the odd member of each lane pair."""
    if getattr(ad, "w1x", False):
        return [f"s_mov_b32 s{S_PAR}, 0", f"s_mov_b32 s{S_PAR + 1}, -1"]
    return [f"s_mov_b32 s{S_PAR}, 0xaaaaaaaa", f"s_mov_b32 s{S_PAR + 1}, 0xaaaaaaaa"]


FULL_STRIDE = 66  # row stride (u64) of the one-pass transposes of a wave with a 16.5 KiB LDS buffer (ad.full_t)


def t1_full(body, dmap, ad, written=False):
    """W0 -> W1 in one pass through a 32 x 66 (u64) LDS tile: lane j writes its 32 rows at i 66 + j (%[tfw] = S + 8 lane,
    row in the offset field), lane 2 i + j0 reads element j = 2 q + j0 of row i into register q (%[tfb] = S + 8 (66 i + j0),
    q in the offset field).  Both sides conflict-free (the reads' 64-bank pattern is 4 i + 2 j0).  For waves that own
    16.5 KiB of LDS (the blind rotation); the 8.5 KiB standalone waves run the two-half t1.  The data stays in the same
    registers (every write has landed before the first read)."""
    L = [] if written else t1_full_writes(dmap, ad, range(32))
    L.append("s_waitcnt lgkmcnt(0)")
    L += [f"ds_read_b64 {pv(dmap[q])}, {ad.tfb} offset:{q * 16}" for q in range(32)]
    L.append("s_waitcnt lgkmcnt(0)")
    body.raw(*L)
    return list(dmap)


def t1_full_writes(dmap, ad, rows):
    return [f"ds_write_b64 {ad.tfw}, {pv(dmap[r])} offset:{r * FULL_STRIDE * 8}" for r in rows]


# The one-pass transposes of the blind rotation overlap their LDS traffic with the neighbouring multiplies: the forward's
# T1 writes each twist batch's 8 rows right after they are multiplied, the inverse's W1'' -> W0 writes each half of the
# lane-pair DIT stage's registers as soon as that half is done, and the untwist's batches wait only for the rows they use.
# Built at the end of round 3 and emulator-exact (its waits are not emulated: checked by reasoning only).  One-box A/B:
# BNF 35.2 k vs 35.3 k PBS/s (noise of +-1.5 k between repeats), Solinas equal (profiles/r3/pbs_progressive_full_t_ab/):
# no measurable gain, not GPU-parity-tested, so off and the bodies stay byte-identical to the measured ones.
PROGRESSIVE_FULL_T = False


def t1(body, dmap, ybase, newhi, ad=NTT_ADDR, row_waits=None):
    """W0 -> W1 (split by j half).  Returns the new dmap (x[q] in y for q < 16, x[16+q] at newhi).
    row_waits: a wait line before each first-half row write (rows written as their loads land)."""
    if getattr(ad, "full_t", False):
        assert row_waits is None
        return t1_full(body, dmap, ad)
    L = []
    st = 33 if getattr(ad, "w1x", False) else 34  # row stride (u64): conflict-free reads in either lane-pair layout
    L += [f"s_mov_b32 exec_lo, -1", f"s_mov_b32 exec_hi, 0"]
    for r in range(32):
        if row_waits:
            L.append(row_waits[r])
        L.append(f"ds_write_b64 {ad.t1w}, {pv(dmap[r])} offset:{r * st * 8}")
    L += EXEC_ALL
    for q in range(16):
        L.append(f"ds_read_b64 {pv(ybase + 2 * q)}, {ad.t1r} offset:{2 * q * 8}")
    L += [f"s_mov_b32 exec_lo, 0", f"s_mov_b32 exec_hi, -1"]
    for r in range(32):
        L.append(f"ds_write_b64 {ad.t1w}, {pv(dmap[r])} offset:{r * st * 8}")
    L += EXEC_ALL
    L.append("s_waitcnt lgkmcnt(0)")
    for q in range(16):
        L.append(f"ds_read_b64 {pv(newhi + 2 * q)}, {ad.t1r} offset:{2 * q * 8}")
    L.append("s_waitcnt lgkmcnt(0)")
    body.raw(*L)
    return [ybase + 2 * q for q in range(16)] + [newhi + 2 * q for q in range(16)]


def t_iw0(body, dmap, pairs, ybase, newhi, ad=NTT_ADDR):
    """W1 (pairs=False) or W1' (pairs=True) -> W0, halves split by i (row stride 66).  The first half's 16 rows land
    in registers no data occupies (ybase.. when free; the renamed pairs of REGROUP_DPP_SELECT may sit there)."""
    ydst = [ybase + 2 * r for r in range(16)]
    if any(d + o in range(ybase, ybase + 32) for d in dmap for o in (0, 1)):
        free = [b + 2 * j for b in free_blocks_except(dmap) for j in range(4) if not newhi <= b < newhi + 32]
        assert len(free) >= 16, free
        ydst = free[:16]
    L = []
    w1x = getattr(ad, "w1x", False)
    rs = 65 if w1x else 66  # row stride (u64) of the W0 side
    for h in range(2):
        if w1x:  # the half of blocks i < 16 (h = 0) is lanes 0-15 and 32-47
            m = "0xffff" if h == 0 else "0xffff0000"
            L += [f"s_mov_b32 exec_lo, {m}", f"s_mov_b32 exec_hi, {m}"]
        else:
            L += ([f"s_mov_b32 exec_lo, -1", f"s_mov_b32 exec_hi, 0"] if h == 0 else
                  [f"s_mov_b32 exec_lo, 0", f"s_mov_b32 exec_hi, -1"])
        for k in range(32):
            if pairs:
                if k < 16:
                    L.append(f"ds_write_b64 {ad.t2wl}, {pv(dmap[k])} offset:{2 * k * 8}")
                else:
                    L.append(f"ds_write_b64 {ad.t2wh}, {pv(dmap[k])} offset:{2 * (k - 16) * 8}")
            else:
                L.append(f"ds_write_b64 {ad.t4w}, {pv(dmap[k])} offset:{2 * k * 8}")
        L += EXEC_ALL
        if h == 1:
            L.append("s_waitcnt lgkmcnt(0)")
        dst = ydst if h == 0 else [newhi + 2 * r for r in range(16)]
        rb = ad.t2r if pairs else ad.t4r
        for r in range(16):
            L.append(f"ds_read_b64 {pv(dst[r])}, {rb} offset:{r * rs * 8}")
    L.append("s_waitcnt lgkmcnt(0)")
    body.raw(*L)
    return ydst + [newhi + 2 * r for r in range(16)]


# The lane-pair regroup as two VOP2 selects per 32-bit word with a DPP partner-lane source (v_cndmask_b32_dpp, VCC set
# by the SALU) instead of two DPP moves and two selects; the second slot's new value goes to a fresh register pair
# (renamed in dmap) so neither select overwrites a value the partner lane still has to read.
REGROUP_DPP_SELECT = False


def regroup(sg, dmap, k, tmp, to_pairs, k2=None, w1x=False):
    """W1 <-> W1' for register pair (k, k2 = k+16) of this lane and its partner (lane ^ 1).
    to_pairs: even lane ends with (a_k, b_k), odd lane with (a_{k2}, b_{k2}).
    back:     even lane ends with (a_k, a_{k2}), odd lane with (b_k, b_{k2}).
    With REGROUP_DPP_SELECT the k2 slot moves to the pair tmp[0:2] (dmap updated) and the returned register base is
    the one it left, free for the caller's next temporary; otherwise returns None."""
    kk2 = k + 16 if k2 is None else k2
    lo0, hi0, p0 = X(dmap, k)
    lo1, hi1, p1 = X(dmap, kk2)
    if w1x:
        # W1x (lane = i + 32 par): one half-wave exchange per word moves the lower lanes' x[k2] up and the upper
        # lanes' x[k] down — the same permutation in both directions (it is an involution)
        sg.add(f"v_permlane32_swap_b32 {lo0}, {lo1}", [lo0, lo1], [lo0, lo1], "dpp")
        sg.add(f"v_permlane32_swap_b32 {hi0}, {hi1}", [hi0, hi1], [hi0, hi1], "dpp")
        return None
    T0, T1, U0, U1 = tmp
    par = f"s[{S_PAR}:{S_PAR + 1}]"
    dpp = "quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
    if REGROUP_DPP_SELECT:
        # both directions move the same values: the k2 slot of an even lane takes its partner's k slot, the k slot of an
        # odd lane its partner's k2 slot (VOP2 select: D = VCC ? src1 : dpp(src0))
        old = dmap[kk2]
        sg.add(f"s_mov_b64 vcc, {par}", [par], ["vcc"], "salu")
        sg.add(f"v_cndmask_b32_dpp {T0}, {lo0}, {lo1}, vcc {dpp}", [lo0, lo1, "vcc"], [T0], "dpp")
        sg.add(f"v_cndmask_b32_dpp {T1}, {hi0}, {hi1}, vcc {dpp}", [hi0, hi1, "vcc"], [T1], "dpp")
        sg.add(f"s_not_b64 vcc, {par}", [par], ["vcc", "scc"], "salu")
        sg.add(f"v_cndmask_b32_dpp {lo0}, {lo1}, {lo0}, vcc {dpp}", [lo1, lo0, "vcc"], [lo0], "dpp")
        sg.add(f"v_cndmask_b32_dpp {hi0}, {hi1}, {hi0}, vcc {dpp}", [hi1, hi0, "vcc"], [hi0], "dpp")
        dmap[kk2] = int(T0[1:])
        return old
    if EXEC_MASK:
        # both directions: T = partner's x[k], U = partner's x[k2] (four DPP moves, all lanes), then the odd lanes take
        # x[k] <- U and the even lanes x[k2] <- T, each one EXEC-masked 64-bit move instead of two selects
        sg.add(f"v_mov_b32_dpp {T0}, {lo0} {dpp}", [lo0], [T0], "dpp")
        sg.add(f"v_mov_b32_dpp {T1}, {hi0} {dpp}", [hi0], [T1], "dpp")
        sg.add(f"v_mov_b32_dpp {U0}, {lo1} {dpp}", [lo1], [U0], "dpp")
        sg.add(f"v_mov_b32_dpp {U1}, {hi1} {dpp}", [hi1], [U1], "dpp")
        mov64_masked(sg, par, p0, pair_of(U0, U1))
        mov64_masked(sg, ("not", par), p1, pair_of(T0, T1))
        return None
    if to_pairs:
        # T = partner x[k], U = partner x[k+16]; even: x[k+16] <- T ; odd: x[k] <- U
        sg.add(f"v_mov_b32_dpp {T0}, {lo0} {dpp}", [lo0], [T0], "dpp")
        sg.add(f"v_mov_b32_dpp {T1}, {hi0} {dpp}", [hi0], [T1], "dpp")
        sg.add(f"v_mov_b32_dpp {U0}, {lo1} {dpp}", [lo1], [U0], "dpp")
        sg.add(f"v_mov_b32_dpp {U1}, {hi1} {dpp}", [hi1], [U1], "dpp")
        sg.add(f"v_cndmask_b32_e64 {lo0}, {lo0}, {U0}, {par}", [lo0, U0, par], [lo0])
        sg.add(f"v_cndmask_b32_e64 {hi0}, {hi0}, {U1}, {par}", [hi0, U1, par], [hi0])
        sg.add(f"v_cndmask_b32_e64 {lo1}, {T0}, {lo1}, {par}", [T0, lo1, par], [lo1])
        sg.add(f"v_cndmask_b32_e64 {hi1}, {T1}, {hi1}, {par}", [T1, hi1, par], [hi1])
    else:
        # even holds (a_k, b_k) -> wants (a_k, a_{k+16}) ; odd holds (a_{k+16}, b_{k+16}) -> (b_k, b_{k+16})
        sg.add(f"v_mov_b32_dpp {T0}, {lo0} {dpp}", [lo0], [T0], "dpp")   # partner's first
        sg.add(f"v_mov_b32_dpp {T1}, {hi0} {dpp}", [hi0], [T1], "dpp")
        sg.add(f"v_mov_b32_dpp {U0}, {lo1} {dpp}", [lo1], [U0], "dpp")   # partner's second
        sg.add(f"v_mov_b32_dpp {U1}, {hi1} {dpp}", [hi1], [U1], "dpp")
        # even: x[k+16] <- T (partner a_{k+16}) ; odd: x[k] <- U (partner b_k)
        sg.add(f"v_cndmask_b32_e64 {lo1}, {T0}, {lo1}, {par}", [T0, lo1, par], [lo1])
        sg.add(f"v_cndmask_b32_e64 {hi1}, {T1}, {hi1}, {par}", [T1, hi1, par], [hi1])
        sg.add(f"v_cndmask_b32_e64 {lo0}, {lo0}, {U0}, {par}", [lo0, U0, par], [lo0])
        sg.add(f"v_cndmask_b32_e64 {hi0}, {hi0}, {U1}, {par}", [hi0, U1, par], [hi0])


def free_blocks_except(dmap, extra_busy=()):
    busy = set()
    for b in dmap:
        busy.update((b, b + 1))
    busy.update(extra_busy)
    blocks = []
    for b in range(VLO, VHI, 8):
        if not any(x in busy for x in range(b, b + 8)):
            blocks.append(b)
    return blocks


def slot_view(m, c23):
    """CT/GS scratch view over a general-multiply slot (used after / around its multiply)."""
    sl = Slot.__new__(Slot)
    sl.v = m.v[0:8]
    sl.P = [m.P[0], m.P[1], m.P[2], m.P[3]]
    sl.c = [m.c[0], m.c[1], c23[0]]
    return sl


def shift_class(e):
    """tmul code path of an exponent e = S % 96: 0 (e <= 32), 1 (32 < e < 64), 2 (64 <= e < 96)."""
    return 0 if e <= 32 else (1 if e < 64 else 2)


def lane_tmul_applies(Se, So):
    """Whether tmul_lane covers the lane pair (even lanes x 2^Se, odd lanes x 2^So): one code path and
    one sign for both lanes, and a per-lane shift amount that is never out of range (r >= 1 in class 1)."""
    ee, eo = Se % 96, So % 96
    neg = lambda S, e: (S >= 96) != (e >= 64)
    if shift_class(ee) != shift_class(eo) or neg(Se, ee) != neg(So, eo):
        return False
    if shift_class(ee) == 0:
        return max(ee, eo) < 32  # v_bfe width r must stay below 32
    return shift_class(ee) != 1 or min(ee, eo) > 32


def tmul_lane(sg, S_even, S_odd, x, sl, tlo, thi, par3, amt):
    """tmul with a lane-dependent exponent (even lanes S_even, odd lanes S_odd = S_even +- 3): the
    compile-time code path of the common class with VGPR shift amounts built from par3 = 3 (lane & 1).
    Same VALU count as tmul plus two full-rate adds; returns the common sign flag."""
    xlo, xhi, xp = x
    v, P, c = sl.v, sl.P, sl.c
    e0, e1 = S_even % 96, S_odd % 96
    assert lane_tmul_applies(S_even, S_odd) and abs(e1 - e0) == 3, (S_even, S_odd)
    neg = (S_even >= 96) != (e0 >= 64)
    A0, A1 = amt
    op_up = "v_add_u32" if e1 > e0 else "v_sub_u32"      # amount grows with the exponent
    op_dn = "v_sub_u32" if e1 > e0 else "v_add_u32"
    cls = shift_class(e0)
    if EXEC_MASK:
        tp = pair_of(tlo, thi)
        if cls in (0, 1):
            r0, w0 = (e0, 32 - e0) if cls == 0 else (e0 - 32, 64 - e0)
            sg.add(f"{op_up} {A0}, {r0}, {par3}", [par3], [A0])
            sg.add(f"{op_dn} {A1}, {w0}, {par3}", [par3], [A1])
            sg.add(f"v_lshlrev_b64 {P[0]}, {A0}, {xp}", [A0, xp], [P[0]])
            if cls == 0:
                sg.add(f"v_bfe_u32 {v[4]}, {xhi}, {A1}, {A0}", [xhi, A1, A0], [v[4]])
            else:
                sg.add(f"v_lshrrev_b32 {v[4]}, {A1}, {xhi}", [A1, xhi], [v[4]])
            sg.add(f"v_mad_u64_u32 {tp}, {c[0]}, {v[4]}, -1, {P[0]}", [v[4], P[0]], [tp, c[0]])
            if cls == 1:
                plus_eps_masked(sg, c[0], tp)
                sg.add(f"v_lshlrev_b64 {P[3]}, 32, {tp}", [tp], [P[3]])
                sg.add(f"v_mad_u64_u32 {tp}, {c[0]}, {thi}, -1, {P[3]}", [thi, P[3]], [tp, c[0]])
            sg.add(f"v_mad_u64_u32 {P[0]}, {c[1]}, -1, 1, {tp}", [tp], [P[0], c[1]])
            mov64_masked(sg, ("or", c[1], c[0]), tp, P[0])
            return neg
        sg.add(f"{op_dn} {A0}, {96 - e0}, {par3}", [par3], [A0])
        sg.add(f"{op_up} {A1}, {e0 - 64}, {par3}", [par3], [A1])
        sg.add(f"v_lshrrev_b64 {P[0]}, {A0}, {xp}", [A0, xp], [P[0]])
        sg.add(f"v_lshlrev_b32 {v[4]}, {A1}, {xlo}", [A1, xlo], [v[4]])
        sg.add(f"v_mad_u64_u32 {tp}, {JUNK}, {v[4]}, 1, {P[0]}", [v[4], P[0]], [tp, JUNK])
        sg.add(f"v_sub_co_u32_e64 {thi}, {c[0]}, {thi}, {v[4]}", [thi, v[4]], [thi, c[0]])
        minus_eps_masked(sg, c[0], tp)
        return neg
    if cls == 0:
        # r = e, h = top r bits of x_hi (v_bfe: width 0 gives 0, so r = 0 needs no special case)
        sg.add(f"{op_up} {A0}, {e0}, {par3}", [par3], [A0])
        sg.add(f"{op_dn} {A1}, {32 - e0}, {par3}", [par3], [A1])
        sg.add(f"v_lshlrev_b64 {P[0]}, {A0}, {xp}", [A0, xp], [P[0]])
        sg.add(f"v_bfe_u32 {v[4]}, {xhi}, {A1}, {A0}", [xhi, A1, A0], [v[4]])
        sg.add(f"v_mad_u64_u32 {P[1]}, {c[0]}, {v[4]}, -1, {P[0]}", [v[4], P[0]], [P[1], c[0]])
        sg.add(f"v_mad_u64_u32 {P[0]}, {c[1]}, -1, 1, {P[1]}", [P[1]], [P[0], c[1]])
        sg.add(f"s_or_b64 {c[1]}, {c[1]}, {c[0]}", [c[1], c[0]], [c[1], "scc"], "salu")
        sg.add(f"v_cndmask_b32_e64 {tlo}, {v[2]}, {v[0]}, {c[1]}", [v[2], v[0], c[1]], [tlo])
        sg.add(f"v_cndmask_b32_e64 {thi}, {v[3]}, {v[1]}, {c[1]}", [v[3], v[1], c[1]], [thi])
    elif cls == 1:
        # r = e - 32 >= 1: y = x 2^r folded once, then y 2^32 = y_lo 2^32 + y_hi eps
        sg.add(f"{op_up} {A0}, {e0 - 32}, {par3}", [par3], [A0])
        sg.add(f"{op_dn} {A1}, {64 - e0}, {par3}", [par3], [A1])
        sg.add(f"v_lshlrev_b64 {P[0]}, {A0}, {xp}", [A0, xp], [P[0]])
        sg.add(f"v_lshrrev_b32 {v[4]}, {A1}, {xhi}", [A1, xhi], [v[4]])
        sg.add(f"v_mad_u64_u32 {P[1]}, {c[0]}, {v[4]}, -1, {P[0]}", [v[4], P[0]], [P[1], c[0]])
        times_2_32(sg, sl)
        sg.add(f"v_mad_u64_u32 {P[0]}, {c[1]}, -1, 1, {P[1]}", [P[1]], [P[0], c[1]])
        sg.add(f"s_or_b64 {c[1]}, {c[1]}, {c[0]}", [c[1], c[0]], [c[1], "scc"], "salu")
        sg.add(f"v_cndmask_b32_e64 {tlo}, {v[2]}, {v[0]}, {c[1]}", [v[2], v[0], c[1]], [tlo])
        sg.add(f"v_cndmask_b32_e64 {thi}, {v[3]}, {v[1]}, {c[1]}", [v[3], v[1], c[1]], [thi])
    else:
        # K = 96 - e in [3, 32]: x 2^-K = (x >> K) + u - u 2^32, u = low K bits of x moved to the top of a word
        sg.add(f"{op_dn} {A0}, {96 - e0}, {par3}", [par3], [A0])
        sg.add(f"{op_up} {A1}, {e0 - 64}, {par3}", [par3], [A1])
        sg.add(f"v_lshrrev_b64 {P[0]}, {A0}, {xp}", [A0, xp], [P[0]])
        sg.add(f"v_lshlrev_b32 {v[4]}, {A1}, {xlo}", [A1, xlo], [v[4]])
        sg.add(f"v_mad_u64_u32 {P[1]}, {JUNK}, {v[4]}, 1, {P[0]}", [v[4], P[0]], [P[1], JUNK])
        sg.add(f"v_sub_co_u32_e64 {v[3]}, {c[0]}, {v[3]}, {v[4]}", [v[3], v[4]], [v[3], c[0]])
        sg.add(f"v_cndmask_b32_e64 {v[5]}, 0, -15, {c[0]}", [c[0]], [v[5]])
        tp = pair_of(tlo, thi)
        sg.add(f"v_mad_i64_i32 {tp}, {JUNK}, {v[5]}, s{S_X15}, {P[1]}", [v[5], P[1]], [tp, tlo, thi, JUNK])
    return neg


def pair_stage_gmul_ks(tabs, fwd):
    """Butterflies of the lane-pair stage that need a table twiddle (no common shift path)."""
    E = tabs["CYC_FWD" if fwd else "CYC_INV"][5]
    return [k for k in range(16) if not lane_tmul_applies(E[k], E[k + 16])]


def pair_stage(B, dmap, fwd, ad=NTT_ADDR, tabs=None, pre=None, busy=()):
    """Cyclic stage q = 5 on lane pairs: regroup W1 -> W1' (DPP), then butterfly k of lane 2i + par uses
    the twiddle w_g = 2^E[g], g = k + 16 par (E = the exponent row of the stage).  Where both lanes'
    exponents share one code path the multiply is a shift-twiddle tmul with per-lane shift amounts
    (tmul_lane); elsewhere a general multiply by the table value (entry g of the 32-entry table).
    Forward: CT then canonical outputs (layout stays W1' for T2); inverse: GS then regroup back to W1."""
    if tabs is None:
        tabs = load_tables()
    E = tabs["CYC_FWD" if fwd else "CYC_INV"][5]
    regs = []
    for b in free_blocks_except(dmap, busy):
        regs += list(range(b, b + 8))
    assert len(regs) >= (48 if busy else 49), len(regs)
    wb = regs[0:16]
    tmps = [regs[16:20], regs[20:24]]
    msl = [MulSlot(0, SG0, regs[24:36]), MulSlot(0, SG0 + 6, regs[36:48])]
    c23 = [(f"s[{SG0 + 4}:{SG0 + 5}]",), (f"s[{SG0 + 10}:{SG0 + 11}]",)]
    # the lane-parity shift offset: the top register of the reserved block (its twiddles use the bottom)
    par3 = f"v{busy[-1]}" if busy else f"v{regs[48]}"
    assert not pre or all(r + 1 < busy[-1] for r in pre.values())
    B.raw(f"v_cndmask_b32_e64 {par3}, 0, 3, s[{S_PAR}:{S_PAR + 1}]")
    if pre:
        B.raw(ad.lw_wait or ad.tw_wait)  # the preloaded twiddles (issued stages ago: normally no stall)
    for half in range(2):
        ks = list(range(8 * half, 8 * half + 8))
        gm = [(i, k) for i, k in enumerate(ks) if not lane_tmul_applies(E[k], E[k + 16]) and not (pre and k in pre)]
        if gm:
            B.raw(*[ad.lw_load(wb[2 * i], k) for i, k in gm], ad.lw_wait or ad.tw_wait, "s_nop 1")
        sg = Seg()
        for i, k in enumerate(ks):
            tmp = [f"v{r}" for r in tmps[i % 2]]
            m = msl[i % 2]
            sl = slot_view(m, c23[i % 2])
            lane = lane_tmul_applies(E[k], E[k + 16])
            wlo, whi = f"v{wb[2 * i]}", f"v{wb[2 * i] + 1}"
            if pre and k in pre:  # twiddle loaded earlier, latency hidden behind the previous stages
                wlo, whi = f"v{pre[k]}", f"v{pre[k] + 1}"
            freed = regroup(sg, dmap, k, tmp, True, w1x=getattr(ad, "w1x", False))
            if freed is not None:
                tmps[i % 2][0:2] = [freed, freed + 1]
            a, b = X(dmap, k), X(dmap, k + 16)
            if fwd:
                # last stage: canonical outputs from a canonical a (3 VALU) and a canonicalising add /
                # borrow-fixed subtract (12 VALU per butterfly instead of 14 for add, sub and two canons)
                canon(sg, sl, a)
                if lane:
                    neg = tmul_lane(sg, E[k], E[k + 16], b, sl, sl.v[2], sl.v[3], par3, (wlo, whi))
                    ct_core_canon(sg, sl, a, b, neg)
                else:
                    # t = b * w into the slot's Z1 pair, then CT with t viewed as v2:v3
                    gmul(sg, m, b, wlo, whi, m.v[8], m.v[9])
                    ct_sl = Slot.__new__(Slot)
                    ct_sl.v = [m.v[0], m.v[1], m.v[8], m.v[9], m.v[4], m.v[5], m.v[6], m.v[7]]
                    ct_sl.P = [m.P[0], None, None, m.P[3]]
                    ct_sl.c = sl.c
                    ct_core_canon(sg, ct_sl, a, b, False)
            else:
                # inputs are canonical (loaded data), so either may be the subtrahend: a' = a + b and
                # d = a - b, or d = b - a when the shift twiddle is negative (the product stays positive)
                e0 = E[k] % 96
                swap = lane and ((E[k] >= 96) != (e0 >= 64))
                add_part1(sg, sl, a[0], a[1], b[0], b[1])
                if swap:
                    sub_seq(sg, sl, b[0], b[1], b[0], b[1], a[0], a[1])
                else:
                    sub_seq(sg, sl, b[0], b[1], a[0], a[1], b[0], b[1])
                add_part2(sg, sl, a[2])
                if lane:
                    tmul_lane(sg, E[k], E[k + 16], b, sl, b[0], b[1], par3, (wlo, whi))
                else:
                    gmul(sg, m, b, wlo, whi, b[0], b[1])
                freed = regroup(sg, dmap, k, [f"v{r}" for r in tmps[i % 2]], False, w1x=getattr(ad, "w1x", False))
                if freed is not None:
                    tmps[i % 2][0:2] = [freed, freed + 1]
        for j, op in enumerate(sg.ops):
            op.idx = j
        B.out(sg.schedule())


def store_raw(dmap):
    return store_rows(dmap, S_GB) + ["s_waitcnt vmcnt(0)"]


def twist_rows(B, dmap, ad, bufs, ms, contiguous=True, regs=None, first_loaded=False, before_batch=None,
               after_batch=None):
    """x[r] *= table row r (general multiplies) for the 32 registers, in 4 batches of 8 rows; the next
    batch's 8 table rows are loaded into the other buffer before this batch multiplies, so the table
    latency (L2 or LDS) hides behind the multiplies.  The slots' zero addend halves are set once.
    before_batch / after_batch (bt): extra lines before / after batch bt's multiplies (the progressive one-pass
    transposes: a wait for the rows an LDS read brings, the LDS writes of the rows just multiplied)."""
    B.raw(*[f"v_mov_b32 {m.v[z]}, 0" for m in ms for z in (9, 11)])
    buf = (lambda i, k: bufs[i] + 2 * k) if contiguous else (lambda i, k: regs[16 * i + 2 * k])
    if not first_loaded:
        B.raw(*[ad.tw_load(0, k, buf(0, k)) for k in range(8)])
    for bt in range(4):
        if bt + 1 < 4:
            B.raw(*[ad.tw_load(bt + 1, k, buf((bt + 1) % 2, k)) for k in range(8)], ad.tw_wait_n(8))
        else:
            B.raw(ad.tw_wait)
        if before_batch:
            B.raw(*before_batch(bt))
        B.mulrows(dmap, list(range(8 * bt, 8 * bt + 8)), [buf(bt % 2, k) for k in range(8)], ms, zero_hi=False)
        if after_batch:
            B.raw(*after_batch(bt))


def fwd_core(B, tabs, dmap, ad=NTT_ADDR, stop=None, prefetch=False, first_stage=0):
    """Forward transform of the W0 data in dmap (must be v64..v127); returns the output dmap (W0,
    canonical).  With `stop`, returns early (debug bodies).  `prefetch` (the standalone kernel, whose
    waves run in lockstep so a wait on a table load is not covered by other waves): the first twist
    batch is loaded before the G1 stages into v8..v23 and the lane-pair table twiddles right after T1,
    each load's latency hidden behind the stages in between (one or two fewer scratch slots there)."""
    busy = tuple(range(8, 24)) if prefetch else ()
    if prefetch:
        B.raw(*[ad.tw_load(0, k, 8 + 2 * k) for k in range(8)])
    fb = free_blocks_except(dmap, busy)
    plan = scale_plan()
    g1_scales = [0] * 32
    for s in range(first_stage, 5):  # first_stage 1: the caller ran stage 0 (the PBS bodies' signed digits)
        gw = None
        if s == 0 and PROGRESSIVE and prefetch:  # rows issued as pairs (k, k + 16), then the 8 twist-row loads
            gw = [f"s_waitcnt vmcnt({40 - 8 * (g + 1)})" for g in range(4)]
        modes = plan["fwd_g1"]["modes"][16 * s:16 * s + 16] if plan else None
        B.tag = f"G1 stage {s}"
        B.stage("ct", 16 >> s, tabs["G1_FWD"][s], dmap, fb, group_waits=gw, modes=modes,
                scales=g1_scales if plan else None)
    if plan:
        assert g1_scales == [v % 192 for v in plan["fwd_g1"]["out_scales"]], "G1 scales differ from the plan's"
    if stop == "g1":
        return dmap
    # twist: 4 batches of 8 rows; table rows double-buffered in v8..v23 / v48..v63 (batch bt + 1
    # loads while batch bt multiplies), 2 multiply slots in v24..v47
    prog = getattr(ad, "full_t", False) and PROGRESSIVE_FULL_T
    after = (lambda bt: t1_full_writes(dmap, ad, range(8 * bt, 8 * bt + 8))) if prog else None
    B.tag = "twist"
    twist_rows(B, dmap, ad, [8, 48], [MulSlot(24 + 12 * i, SG0 + 6 * i) for i in range(2)], first_loaded=prefetch,
               after_batch=after)
    if stop == "twist":
        return dmap
    B.tag = "T1 transpose"
    dmap = t1_full(B, dmap, ad, written=True) if prog else t1(B, dmap, 8, 64, ad)
    if stop == "t1":
        return dmap
    pre, busy = None, ()
    if prefetch:
        gks = pair_stage_gmul_ks(tabs, True)
        fb0 = free_blocks_except(dmap)
        pre = {k: fb0[0] + 2 * i for i, k in enumerate(gks)}
        busy = tuple(range(fb0[0], fb0[0] + 8))
        B.raw(*[ad.lw_load(r, k) for k, r in pre.items()])
    fb = free_blocks_except(dmap, busy)
    cf = [True] * 32  # twist outputs are canonical
    cyc_scales = list(plan["fwd_cyc"]["in_scales"]) if plan else None
    for q in range(5):
        B.tag = f"cyclic stage {q}"
        B.stage("ct", 16 >> q, tabs["CYC_FWD"][q], dmap, fb, cf, modes=plan["fwd_cyc"]["modes"][16 * q:16 * q + 16]
                if plan else None, scales=cyc_scales)
    if plan:
        assert all(v % 192 == 0 for v in cyc_scales), "the cyclic blocks' outputs must be unscaled"
    if stop == "cyc":
        return dmap
    B.tag = "lane-pair stage"
    pair_stage(B, dmap, True, ad, tabs, pre, busy)
    if stop == "last":
        return dmap
    B.tag = "T2 transpose"
    dmap = t_iw0(B, dmap, True, 96, 64, ad)
    B.tag = "store"
    return dmap


def gen_fwd(tabs, stop=None):
    B = Body(tabs)
    dmap = [64 + 2 * r for r in range(32)]
    B.raw(f"s_mov_b64 s[{S_EXE}:{S_EXE + 1}], exec", f"s_mov_b32 s{S_X15}, 0x11111111")
    B.raw(*gen_bases("g", S_GB), *gen_bases("tw", S_TB))
    ad = NTT_ADDR_W1X if FWD_W1X else NTT_ADDR
    B.raw(*par_mask(ad))
    if PROGRESSIVE and not stop:
        rows = load_rows(dmap, S_GB)
        B.raw(*[rows[r] for k in range(16) for r in (k, k + 16)])
    else:
        B.raw(*load_rows(dmap, S_GB), "s_waitcnt vmcnt(0)")
    if FWD_STORE != "t2" and not stop:
        dmap = fwd_core(B, tabs, dmap, ad, stop="last", prefetch=True)
        B.raw(*direct_stores(dmap, FWD_STORE))
        return B
    dmap = fwd_core(B, tabs, dmap, ad, stop=stop, prefetch=True)
    if stop:
        B.raw(*store_raw(dmap))
        return B
    B.raw(*store_rows(dmap, S_GB))  # no final vmcnt wait: the wave may retire while its stores drain
    return B


S_OB = 94      # s[94:101]: output row-group bases (the key-conversion body writes another buffer)
S_H31 = 28     # s28 = 0x80000000 (a VOP3 operand cannot be a 32-bit literal on gfx950)
MS_SGPRS = list(range(S_OB, S_OB + 8))


def modswitch_native(sg, sl, x):
    """x <- (x p + 2^63) >> 64, the native-modulus switch into Z_p of the key conversion (ntt64.rs:166-178,
    lwe_bootstrap_key_conversion.rs:294-365, in_width 64).  With x = x_hi 2^32 + x_lo and p = 2^64 - 2^32 + 1:
    x p + 2^63 = x 2^64 + (x + 2^63 - x_lo 2^32) - x_hi 2^64, so the result is x - x_hi + c1 - b2 with
    c1 = carry(x_hi + 2^31) and b2 = borrow((x_hi + 2^31) mod 2^32 - x_lo); no intermediate wraps and the result
    is canonical (x = 2^64 - 1 gives p - 1).  8 carry ops."""
    xlo, xhi, _ = x
    v, c = sl.v, sl.c
    t = v[0]
    sg.add(f"v_add_co_u32_e64 {t}, {c[0]}, {xhi}, s{S_H31}", [xhi, f"s{S_H31}"], [t, c[0]])
    sg.add(f"v_sub_co_u32_e64 {t}, {c[1]}, {t}, {xlo}", [t, xlo], [t, c[1]])
    sg.add(f"v_sub_co_u32_e64 {xlo}, {c[2]}, {xlo}, {xhi}", [xlo, xhi], [xlo, c[2]])
    sg.add(f"v_subb_co_u32_e64 {xhi}, {c[2]}, {xhi}, 0, {c[2]}", [xhi, c[2]], [xhi, c[2]])
    sg.add(f"v_addc_co_u32_e64 {xlo}, {c[2]}, {xlo}, 0, {c[0]}", [xlo, c[0]], [xlo, c[2]])
    sg.add(f"v_addc_co_u32_e64 {xhi}, {c[2]}, {xhi}, 0, {c[2]}", [xhi, c[2]], [xhi, c[2]])
    sg.add(f"v_subb_co_u32_e64 {xlo}, {c[2]}, {xlo}, 0, {c[1]}", [xlo, c[1]], [xlo, c[2]])
    sg.add(f"v_subb_co_u32_e64 {xhi}, {c[2]}, {xhi}, 0, {c[2]}", [xhi, c[2]], [xhi, c[2]])


def gen_fwd_ms64(tabs):
    """Key conversion body: rows of a standard-domain key (native 2^64 torus) -> modswitch into Z_p -> forward
    transform -> rows of another buffer (bases %[o_lo] / %[o_hi]).  With the plan's N^-1-scaled twist table the
    output is also normalised (the twist multiplies every element exactly once)."""
    B = Body(tabs)
    dmap = [64 + 2 * r for r in range(32)]
    B.raw(f"s_mov_b64 s[{S_EXE}:{S_EXE + 1}], exec", f"s_mov_b32 s{S_X15}, 0x11111111",
          f"s_mov_b32 s{S_H31}, 0x80000000")
    B.raw(*gen_bases("g", S_GB), *gen_bases("tw", S_TB), *gen_bases("o", S_OB))
    ad = NTT_ADDR_W1X if FWD_W1X else NTT_ADDR
    B.raw(*par_mask(ad))
    B.raw(*load_rows(dmap, S_GB), "s_waitcnt vmcnt(0)")
    sg = Seg()
    sls = B.slots(free_blocks_except(dmap))
    for r in range(32):
        modswitch_native(sg, sls[r % len(sls)], X(dmap, r))
    for i, op in enumerate(sg.ops):
        op.idx = i
    B.out(sg.schedule())
    dmap = fwd_core(B, tabs, dmap, ad, prefetch=True)
    B.raw(*store_rows(dmap, S_OB))
    return B


def direct_stores(dmap, mode):
    """After the lane-pair stage lane 2 i + par holds (x[k], x[k+16]) = outputs 64 i + 32 par + 2 k, + 1
    (k < 16): store them straight from registers at %[pso] = 512 i + 256 par (bytes) + 16 k."""
    out = []
    if mode == "x2":
        for k in range(16):
            out.append(f"global_store_dwordx2 %[pso], {pv(dmap[k])}, s[{S_GB}:{S_GB + 1}] offset:{16 * k}")
            out.append(f"global_store_dwordx2 %[pso], {pv(dmap[k + 16])}, s[{S_GB}:{S_GB + 1}] offset:{16 * k + 8}")
        return out
    busy = set()
    for b in dmap:
        busy.update((b, b + 1))
    quads = [q for q in range(VLO, VHI, 4) if not any(r in busy for r in range(q, q + 4))]
    assert len(quads) >= 4, quads
    for k in range(16):
        q = quads[k % len(quads)]
        out.append(f"v_mov_b64 v[{q}:{q + 1}], {pv(dmap[k])}")
        out.append(f"v_mov_b64 v[{q + 2}:{q + 3}], {pv(dmap[k + 16])}")
        out.append(f"global_store_dwordx4 %[pso], v[{q}:{q + 3}], s[{S_GB}:{S_GB + 1}] offset:{16 * k}")
    return out


INV_PRE_LW = 40          # v40..v43: the inverse lane-pair table twiddles, loaded with the data
INV_PRE_TW = 40          # v40..v55: the first untwist batch, loaded during the lane-pair stage


def dit_exps(s):
    """Exponents of DIT stage s = 1..5 of the inverse cyclic blocks (register distance 2^(s-1), storage
    bit s of j = 2 reg + j0), indexed by the butterfly's first register r.

    The inverse of the natural-in / bit-reversed-out cyclic DFT (omega = 8) is computed from its
    bit-reversed input by decimation in time: stage s joins j and j + 2^s with the twiddle
    w = omega^-(k 64 / 2^(s+1)), k = j mod 2^s, so CT butterflies need no canonical inputs (GS ones need a
    canonical subtrahend).  k holds the lane bit j0, so the odd lanes' twiddle would differ from the even
    lanes' by omega^-(64 / 2^(s+1)) at every stage; instead the odd lanes enter stage 1 scaled by the
    product of those factors over the stages to come, sigma(j) = omega^-bitrev5(j >> 1), which the first
    (lane-pair) stage applies as a GS butterfly with exactly the CYC_INV[5] twiddles (a scale common to a
    butterfly's two inputs passes through it; the factor pending for bit s is used up at stage s, so the
    outputs come out unscaled).  Every lane then uses the even-lane twiddle: k = 2 (r mod 2^(s-1))."""
    d = 1 << (s - 1)
    return [(-3 * (64 >> s) * (r % d)) % 192 for r in range(32)]


INV_W1PP = True  # standalone inverse: cyclic blocks in the W1'' layout (t1_w1pp / dit_exps_pp / pair_stage_dit)


def inv_last_exp(r):
    """Twiddle exponent of the last DIT stage (j, j + 32) of the inverse cyclic blocks, k = j mod 32 = r."""
    return (-3 * r) % 192


def dit_exps_pp(s):
    """DIT stage s = 0..4 of the inverse cyclic blocks in W1'' (register r = j & 31, distance 2^s):
    w = omega^-(k 64 / 2^(s+1)), k = r mod 2^s, compile-time per register (the lane bit j5 is not in k)."""
    return [(-3 * (32 >> s) * (r % (1 << s))) % 192 for r in range(32)]


def t1_w1pp(body, dmap, dst, ad=NTT_ADDR):
    """W0 (lane = j, register = block i) -> W1'' (lane = 2 i + j5, register r = j & 31) through LDS, halves split
    by i: every lane writes rows i = 16 h .. 16 h + 15 at (i & 15) 66 + j + (j >> 5) (%[t1x]); lanes 32 h .. 32 h + 31
    (blocks 16 h ..) read their 32 values at (i & 15) 66 + 33 j5 + r (%[t1y]).  Rows 16.. stay live in half 0, so
    `dst` may reuse only the registers of rows 0..15.  Conflict-free both ways (tools/lds_layout_check.py)."""
    L = []
    for h in range(2):
        for rho in range(16):
            L.append(f"ds_write_b64 {ad.t1x}, {pv(dmap[16 * h + rho])} offset:{rho * 66 * 8}")
        L.append("s_waitcnt lgkmcnt(0)")
        L += exec_block_half(ad, h)
        for r in range(32):
            L.append(f"ds_read_b64 {pv(dst[r])}, {ad.t1y} offset:{r * 8}")
        L += EXEC_ALL
        L.append("s_waitcnt lgkmcnt(0)")
    body.raw(*L)
    return list(dst)


def t_w1pp_w0_full_writes(dmap, ad, regs):
    return [f"ds_write_b64 {ad.tfb}, {pv(dmap[R])} offset:{(2 * (R >> 1) + 32 * (R & 1)) * 8}" for R in regs]


# waits of the untwist batches on the progressive W1'' -> W0 reads (LDS completes in order; lgkmcnt saturates at 15):
# batch bt multiplies rows 8 bt .. 8 bt + 7
UNTWIST_ROW_WAITS = ["s_waitcnt lgkmcnt(15)", "s_waitcnt lgkmcnt(15)", "s_waitcnt lgkmcnt(8)", "s_waitcnt lgkmcnt(0)"]


def t_w1pp_w0(body, dmap, ybase, newhi, ad=NTT_ADDR, written=False, reads_pending=False):
    """After pair_stage_dit lane 2 i + par holds output n = 2 m + par + 32 q in register 2 m + q: -> W0 through
    LDS, halves split by i (rows (i & 15) 66, columns n + (n >> 5)); reads at %[t1x] + 66 rho.  ad.full_t: one pass
    through the 32 x 66 tile of t1_full (writes at %[tfb] + 2 m + 32 q, reads at %[tfw] + 66 i), the rows landing in
    the registers of dmap."""
    if getattr(ad, "full_t", False):
        L = [] if written else t_w1pp_w0_full_writes(dmap, ad, range(32))
        L.append("s_waitcnt lgkmcnt(0)")
        L += [f"ds_read_b64 {pv(dmap[i])}, {ad.tfw} offset:{i * FULL_STRIDE * 8}" for i in range(32)]
        if not reads_pending:
            L.append("s_waitcnt lgkmcnt(0)")
        body.raw(*L)
        return list(dmap)
    L = []
    rs = 65 if getattr(ad, "w1x", False) else 66  # W1x: an odd row stride keeps the 16-lane write groups conflict-free
    for h in range(2):
        L += exec_block_half(ad, h)
        for R in range(32):
            off = 2 * (R >> 1) + 33 * (R & 1)
            L.append(f"ds_write_b64 {ad.t4w}, {pv(dmap[R])} offset:{off * 8}")
        L += EXEC_ALL
        L.append("s_waitcnt lgkmcnt(0)")
        dst = ybase if h == 0 else newhi
        for rho in range(16):
            L.append(f"ds_read_b64 {pv(dst + 2 * rho)}, {ad.t1x} offset:{rho * rs * 8}")
        L.append("s_waitcnt lgkmcnt(0)")
    body.raw(*L)
    return [ybase + 2 * r for r in range(16)] + [newhi + 2 * r for r in range(16)]


def pair_stage_dit_gmul_ms():
    return [m for m in range(16) if not lane_tmul_applies(inv_last_exp(2 * m), inv_last_exp(2 * m + 1))]


def pair_stage_dit(B, dmap, ad, pre, busy, after_half=None):
    """Last DIT stage of the inverse cyclic blocks in W1'': j and j + 32 sit in the two lanes of a pair (register
    r = j & 31).  Regroup registers (2 m, 2 m + 1) across the pair (even lane: elements 2 m, 2 m + 32; odd lane:
    2 m + 1, 2 m + 33), then a CT butterfly whose twiddle exponent differs by 3 between the lanes (tmul_lane), or
    a general multiply by the lane's table value (entry m + 16 par of the inverse's DIT table, preloaded into
    `pre`[m]).  Outputs: register 2 m + q holds n = 2 m + par + 32 q."""
    regs = []
    for b in free_blocks_except(dmap, busy):
        regs += list(range(b, b + 8))
    assert len(regs) >= 40, len(regs)
    tmps = [regs[0:4], regs[4:8]]
    amts = [regs[8:10], regs[10:12]]
    msl = [MulSlot(0, SG0, regs[16:28]), MulSlot(0, SG0 + 6, regs[28:40])]  # explicit lists: free blocks need not be contiguous
    c23 = [(f"s[{SG0 + 4}:{SG0 + 5}]",), (f"s[{SG0 + 10}:{SG0 + 11}]",)]
    par3 = f"v{regs[12]}"
    B.raw(f"v_cndmask_b32_e64 {par3}, 0, 3, s[{S_PAR}:{S_PAR + 1}]")
    if pre:
        B.raw(ad.lw_wait or ad.tw_wait)
    for half in range(2):
        sg = Seg()
        for i, m in enumerate(range(8 * half, 8 * half + 8)):
            tmp = [f"v{r}" for r in tmps[i % 2]]
            mm = msl[i % 2]
            sl = slot_view(mm, c23[i % 2])
            Se, So = inv_last_exp(2 * m), inv_last_exp(2 * m + 1)
            freed = regroup(sg, dmap, 2 * m, tmp, True, k2=2 * m + 1, w1x=getattr(ad, "w1x", False))
            if freed is not None:
                tmps[i % 2][0:2] = [freed, freed + 1]
            a, b = X(dmap, 2 * m), X(dmap, 2 * m + 1)
            if lane_tmul_applies(Se, So):
                neg = tmul_lane(sg, Se, So, b, sl, sl.v[2], sl.v[3], par3, tuple(f"v{r}" for r in amts[i % 2]))
                ct_core(sg, sl, a, b, neg)
            else:
                gmul(sg, mm, b, f"v{pre[m]}", f"v{pre[m] + 1}", mm.v[8], mm.v[9])
                ct_sl = Slot.__new__(Slot)
                ct_sl.v = [mm.v[0], mm.v[1], mm.v[8], mm.v[9], mm.v[4], mm.v[5], mm.v[6], mm.v[7]]
                ct_sl.P = [mm.P[0], None, None, mm.P[3]]
                ct_sl.c = sl.c
                ct_core(sg, ct_sl, a, b, False)
        for j, op in enumerate(sg.ops):
            op.idx = j
        B.out(sg.schedule())
        if after_half:
            B.raw(*after_half(half))


def w1p_as_w1pp(dmap):
    """The forward's output layout after its lane-pair stage (W1': lane 2 i + par, register R < 16 holds output
    64 i + 32 par + 2 R, register R + 16 the next one) is W1'' (lane 2 i + j5, register r = j & 31) up to a renaming
    of registers: r = 2 (R mod 16) + [R >= 16].  So a consumer that keeps the NTT-domain data in registers (the PBS
    step: forward -> MAC -> inverse) needs neither the forward's T2 nor the inverse's T1''."""
    return [dmap[(r >> 1) + 16 * (r & 1)] for r in range(32)]


def inv_cyc_w1pp(B, dmap, ad, dst=None, pre_base=72, ybase=96, newhi=64, w1p_in=False):
    """W0 data -> T1'' -> DIT stages 0..4 in registers -> the lane-pair DIT stage -> W0.  The lane-pair stage's
    table twiddles load right after T1'' (into pre_base..), five stages ahead of their use.  Register plan
    (standalone defaults; the PBS bodies pass their own): `dst` (32 pairs) may reuse only rows 0..15 of `dmap`,
    pre_base.. (8 registers) must be free of `dst`, and `ybase` (the first output half) must be free of `dst`.
    w1p_in: `dmap` already holds the data in the forward's W1' layout (no T1'', see w1p_as_w1pp)."""
    if w1p_in:
        dmap = w1p_as_w1pp(dmap)
    else:
        assert not getattr(ad, "full_t", False)
        B.tag = "T1'' transpose"
        dmap = t1_w1pp(B, dmap, dst or [8 + 2 * r for r in range(32)], ad)
    ms = pair_stage_dit_gmul_ms()
    pre = {m: pre_base + 2 * i for i, m in enumerate(ms)}
    assert len(ms) <= 4
    busy = tuple(range(pre_base, pre_base + 8))
    assert not set(busy) & {r for b in dmap for r in (b, b + 1)}
    B.raw(*[ad.lw_load(r, m) for m, r in pre.items()])
    fb = free_blocks_except(dmap, busy)
    cf = [True] * 32  # loaded data is canonical
    for s in range(5):
        B.tag = f"cyclic stage {s}"
        B.stage("ct", 1 << s, dit_exps_pp(s), dmap, fb, cf, by_reg=True)
    prog = getattr(ad, "full_t", False) and PROGRESSIVE_FULL_T
    after = (lambda h: t_w1pp_w0_full_writes(dmap, ad, range(16 * h, 16 * h + 16))) if prog else None
    B.tag = "lane-pair stage"
    pair_stage_dit(B, dmap, ad, pre, busy, after_half=after)
    assert getattr(ad, "full_t", False) or not set(range(ybase, ybase + 32)) & {r for b in dmap for r in (b, b + 1)}
    B.tag = "T2'' transpose"
    return t_w1pp_w0(B, dmap, ybase, newhi, ad, written=prog, reads_pending=prog)


def inv_core(B, tabs, dmap, ad=NTT_ADDR, prefetch=False, row_waits=None, w1pp=False, w1pp_regs=None, g1_busy=(),
             before_g1=()):
    """Inverse transform of the W0 data in dmap; returns the output dmap (W0, canonical).  g1_busy / before_g1: registers
    the G1 stages leave alone and lines emitted right before them (the external-product bodies' out-row loads).  `prefetch`
    (standalone kernel, see fwd_core): the caller has loaded the lane-pair table twiddles into
    v40..v43 with the data; the first untwist batch is loaded into v40..v55 after the lane-pair stage
    and stays there through the cyclic stages and T4 (the one register range free in both layouts)."""
    if w1pp:
        dmap = inv_cyc_w1pp(B, dmap, ad, **(w1pp_regs or {}))
        prefetch, busy = False, ()
    else:
        dmap = t1(B, dmap, 8, 64, ad, row_waits)
        gks = pair_stage_gmul_ks(tabs, False)
        pre = {k: INV_PRE_LW + 2 * i for i, k in enumerate(gks)} if prefetch else None
        pair_stage(B, dmap, False, ad, tabs, pre, tuple(range(INV_PRE_LW, INV_PRE_LW + 8)) if prefetch else ())
        busy = tuple(range(INV_PRE_TW, INV_PRE_TW + 16)) if prefetch else ()
        if prefetch:
            B.raw(*[ad.tw_load(0, k, INV_PRE_TW + 2 * k) for k in range(8)])
        fb = free_blocks_except(dmap, busy)
        cf = [False] * 32
        if INV_CYC_DIT:
            for s in range(1, 6):
                B.stage("ct", 1 << (s - 1), dit_exps(s), dmap, fb, cf, by_reg=True)
        else:  # r2 form (GS, canonical subtrahends), kept for tools/variant_probe A/B runs
            for q in range(4, -1, -1):
                B.stage("gs", 16 >> q, tabs["CYC_INV"][q], dmap, fb, cf)
        dmap = t_iw0(B, dmap, False, 96, 64, ad)
    # untwist: table rows and multiply slots in the registers the data does not occupy
    B.tag = "untwist"
    free = free_blocks_except(dmap, busy)
    regs = []
    for b in free:
        regs += list(range(b, b + 8))
    if prefetch:
        assert len(regs) >= 40, len(regs)
        tregs = list(range(INV_PRE_TW, INV_PRE_TW + 16)) + regs[0:16]
        ms = [MulSlot(0, SG0, regs[16:28]), MulSlot(0, SG0 + 6, regs[28:40])]
        twist_rows(B, dmap, ad, None, ms, contiguous=False, regs=tregs, first_loaded=True)
    else:
        assert len(regs) >= 56, len(regs)
        prog = w1pp and getattr(ad, "full_t", False) and PROGRESSIVE_FULL_T  # the W1'' -> W0 reads are still landing
        twist_rows(B, dmap, ad, [regs[0], regs[16]], [MulSlot(0, SG0 + 6 * i, regs[32 + 12 * i:44 + 12 * i]) for i in range(2)],
                   contiguous=False, regs=regs, before_batch=(lambda bt: [UNTWIST_ROW_WAITS[bt]]) if prog else None)
    B.raw(*before_g1)
    fb = free_blocks_except(dmap, tuple(g1_busy))
    cf = [True] * 32  # untwist outputs are canonical
    for s in range(4, -1, -1):
        B.tag = f"G1 stage {s}"
        B.stage("gs", 16 >> s, tabs["G1_INV"][s], dmap, fb, cf)
    B.tag = "canonicalise + store"
    sg = Seg()
    sls = B.slots(fb)
    for k, r in enumerate([r for r in range(32) if not cf[r]]):
        canon(sg, sls[k % len(sls)], X(dmap, r))
    for j, op in enumerate(sg.ops):
        op.idx = j
    B.out(sg.schedule())
    return dmap


def gen_inv(tabs, stop=None):
    B = Body(tabs)
    dmap = [64 + 2 * r for r in range(32)]
    B.raw(f"s_mov_b64 s[{S_EXE}:{S_EXE + 1}], exec", f"s_mov_b32 s{S_X15}, 0x11111111")
    B.raw(*gen_bases("g", S_GB), *gen_bases("tw", S_TB))
    ad = NTT_ADDR_W1X if INV_W1X and INV_W1PP else NTT_ADDR
    B.raw(*par_mask(ad))
    if INV_W1PP:
        B.raw(*load_rows(dmap, S_GB), "s_waitcnt vmcnt(0)")
        dmap = inv_core(B, tabs, dmap, ad, w1pp=True)
        B.raw(*store_rows(dmap, S_GB))
        return B
    gks = pair_stage_gmul_ks(tabs, False)
    B.raw(*load_rows(dmap, S_GB), *[NTT_ADDR.lw_load(INV_PRE_LW + 2 * i, k) for i, k in enumerate(gks)])
    rw = None
    if PROGRESSIVE_INV:  # row r is written to LDS once it has landed (the pair twiddles are waited for later)
        rw = [f"s_waitcnt vmcnt({32 + len(gks) - 1 - r})" for r in range(32)]
    else:
        B.raw("s_waitcnt vmcnt(0)")
    dmap = inv_core(B, tabs, dmap, prefetch=True, row_waits=rw)
    B.raw(*store_rows(dmap, S_GB))  # no final vmcnt wait: the wave may retire while its stores drain
    return B


# ---- the MAC-fused inverse of the large-N blind rotation (pbs_large.hip, r5) ------------------------------------------
# One CMUX step at N > 2048 runs the forward on the (k + 1) l digit polynomials, the MAC with the step's GGSW, then the
# inverse on the k + 1 products; with the split transform the inverse starts with the 2048-block bodies.  This body
# forms its block of the product on load, y = sum_q d_q . G_q over the L = l (k + 1) digit / GGSW rows of the block
# (update_with_fmadd, ntt64_pbs.rs:683-702 / ntt64_bnf_pbs.rs:707-726), then runs the standalone inverse on it and
# stores y: the separate MAC pass (the product written and read back) disappears.
# Each product term is 4 v_mad_u64_u32 into three 64-bit column accumulators (bits 0, 32, 64) whose carries are
# counted (4 v_addc), one reduction per row at the end (as pbs_large.hip Acc128).  The term loads stream through a ring
# of 4-VGPR buffers (digit pair, GGSW pair) issued MAC_RING terms ahead.
S_MB = 64        # s[64 ..]: term base pairs, the digits' D_q then the GGSW's G_q (2 L pairs; L <= 8: up to s95)
MAC_LS = (2, 3, 4, 6, 8)   # generated term counts: l (k + 1) for k = 1, l = 1..4 and k = 2, l = 1..2
MAC_VHI = 128    # VGPR ceiling of the bodies (168: a longer ring at 3 waves per SIMD)


def mac_ring(vhi):
    """Ring buffer bases (4 VGPRs each: digit pair, GGSW pair) and the slot's base: v8..v63 (+ v128..vhi-1)."""
    slot = 52
    bufs = [8 + 4 * k for k in range(11)] + [128 + 4 * k for k in range((vhi - 128) // 4)]
    return bufs, slot


def mac_row(sg, L, bufs_of_terms, slot, out):
    """Seg ops of one row: y = sum_q x_q w_q (x, w in the term buffers), reduced into the pair `out`, canonical."""
    A0, A32, A64 = slot, slot + 2, slot + 4
    n0, n32, n64 = f"v{slot + 6}", f"v{slot + 7}", f"v{slot + 8}"
    c = [f"s[{36 + 2 * i}:{37 + 2 * i}]" for i in range(4)]
    f = [f"s[{44 + 2 * i}:{45 + 2 * i}]" for i in range(10)]
    v = lambda r: f"v{r}"
    for q, X in enumerate(bufs_of_terms):
        x0, x1, w0, w1 = v(X), v(X + 1), v(X + 2), v(X + 3)
        if q == 0:
            sg.add(f"v_mad_u64_u32 {pv(A0)}, {JUNK}, {x0}, {w0}, 0", [x0, w0], [pv(A0), JUNK])
            sg.add(f"v_mad_u64_u32 {pv(A32)}, {JUNK}, {x0}, {w1}, 0", [x0, w1], [pv(A32), JUNK])
            sg.add(f"v_mad_u64_u32 {pv(A64)}, {JUNK}, {x1}, {w1}, 0", [x1, w1], [pv(A64), JUNK])
            sg.add(f"v_mad_u64_u32 {pv(A32)}, {c[2]}, {x1}, {w0}, {pv(A32)}", [x1, w0, pv(A32)], [pv(A32), c[2]])
            sg.add(f"v_cndmask_b32_e64 {n32}, 0, 1, {c[2]}", [c[2]], [n32])
            continue
        first = q == 1  # n0 / n64 start from this term's carries
        sg.add(f"v_mad_u64_u32 {pv(A0)}, {c[0]}, {x0}, {w0}, {pv(A0)}", [x0, w0, pv(A0)], [pv(A0), c[0]])
        sg.add(f"v_mad_u64_u32 {pv(A32)}, {c[1]}, {x0}, {w1}, {pv(A32)}", [x0, w1, pv(A32)], [pv(A32), c[1]])
        sg.add(f"v_mad_u64_u32 {pv(A64)}, {c[3]}, {x1}, {w1}, {pv(A64)}", [x1, w1, pv(A64)], [pv(A64), c[3]])
        sg.add(f"v_mad_u64_u32 {pv(A32)}, {c[2]}, {x1}, {w0}, {pv(A32)}", [x1, w0, pv(A32)], [pv(A32), c[2]])
        sg.add(f"v_addc_co_u32_e64 {n0}, {JUNK}, {0 if first else n0}, 0, {c[0]}", [c[0]] + ([] if first else [n0]),
               [n0, JUNK])
        sg.add(f"v_addc_co_u32_e64 {n32}, {JUNK}, {n32}, 0, {c[1]}", [n32, c[1]], [n32, JUNK])
        sg.add(f"v_addc_co_u32_e64 {n64}, {JUNK}, {0 if first else n64}, 0, {c[3]}", [c[3]] + ([] if first else [n64]),
               [n64, JUNK])
        sg.add(f"v_addc_co_u32_e64 {n32}, {JUNK}, {n32}, 0, {c[2]}", [n32, c[2]], [n32, JUNK])
    # S = A0 + A32 2^32 + (A64 + n0) 2^64 + n32 2^96 + n64 2^128 -> lo = A0 (64), hi = A64 (64), top = n64:
    a0l, a0h, a32l, a32h, a64l, a64h = v(A0), v(A0 + 1), v(A32), v(A32 + 1), v(A64), v(A64 + 1)
    sg.add(f"v_add_co_u32_e64 {a0h}, {f[0]}, {a0h}, {a32l}", [a0h, a32l], [a0h, f[0]])
    sg.add(f"v_addc_co_u32_e64 {a64l}, {f[1]}, {a64l}, {a32h}, {f[0]}", [a64l, a32h, f[0]], [a64l, f[1]])
    sg.add(f"v_addc_co_u32_e64 {a64h}, {f[2]}, {a64h}, {n32}, {f[1]}", [a64h, n32, f[1]], [a64h, f[2]])
    sg.add(f"v_addc_co_u32_e64 {n64}, {JUNK}, {n64}, 0, {f[2]}", [n64, f[2]], [n64, JUNK])
    sg.add(f"v_add_co_u32_e64 {a64l}, {f[3]}, {a64l}, {n0}", [a64l, n0], [a64l, f[3]])
    sg.add(f"v_addc_co_u32_e64 {a64h}, {f[4]}, {a64h}, 0, {f[3]}", [a64h, f[3]], [a64h, f[4]])
    sg.add(f"v_addc_co_u32_e64 {n64}, {JUNK}, {n64}, 0, {f[4]}", [n64, f[4]], [n64, JUNK])
    # with hi = hh 2^32 + hl, 2^64 = EPS, 2^96 = -1, 2^128 = -2^32: S = lo - (top 2^32 + hh) + hl EPS.  D = lo - (top:hh)
    # (into A32); a borrow adds 2^64 = EPS too many: D - EPS (top <= L + 1, so D >= 2^64 - 2^36 there: no wrap)
    sg.add(f"v_sub_co_u32_e64 {a32l}, {f[5]}, {a0l}, {a64h}", [a0l, a64h], [a32l, f[5]])
    sg.add(f"v_subb_co_u32_e64 {a32h}, {f[6]}, {a0h}, {n64}, {f[5]}", [a0h, n64, f[5]], [a32h, f[6]])
    minus_eps(sg, n0, f[6], pv(A32))
    # R = D + hl EPS (carry: R + 2^64 = R + EPS), U = R + EPS; canonical = (carry(R) | carry(U)) ? U : R
    o = pv(out)
    sg.add(f"v_mad_u64_u32 {o}, {f[7]}, {a64l}, -1, {pv(A32)}", [a64l, pv(A32)], [o, f[7]])
    sg.add(f"v_mad_u64_u32 {pv(A0)}, {f[8]}, -1, 1, {o}", [o], [pv(A0), f[8]])
    sg.add(f"s_or_b64 {f[9]}, {f[7]}, {f[8]}", [f[7], f[8]], [f[9]], kind="salu")
    sg.add(f"v_cndmask_b32_e64 v{out}, v{out}, {a0l}, {f[9]}", [f"v{out}", a0l, f[9]], [f"v{out}"])
    sg.add(f"v_cndmask_b32_e64 v{out + 1}, v{out + 1}, {a0h}, {f[9]}", [f"v{out + 1}", a0h, f[9]], [f"v{out + 1}"])


def mac_phase(B, L, dmap, vhi=MAC_VHI, bufs=None, after_row=None):
    """Rows 0..31 of y = sum_q d_q G_q into dmap (W0: lane j of row r = element 64 r + j of the block).  Term (r, q)
    loads d_q row r from %[d] + q %[dstep] and G_q row r from %[gg] + q %[gstep] (bytes).  bufs / after_row (the
    wave-specialised producer): another term ring, and lines emitted after each row (its hand-off write)."""
    assert 2 <= L <= 8 and S_MB + 4 * L <= 96
    if bufs is None:
        bufs, slot = mac_ring(vhi)
    else:
        slot = mac_ring(vhi)[1]
    ring = len(bufs)
    dq = lambda q: S_MB + 2 * q
    gq = lambda q: S_MB + 2 * L + 2 * q
    sp = lambda b: f"s[{b}:{b + 1}]"
    lines = [f"s_mov_b32 s{dq(0)}, %[d_lo]", f"s_mov_b32 s{dq(0) + 1}, %[d_hi]",
             f"s_mov_b32 s{gq(0)}, %[gg_lo]", f"s_mov_b32 s{gq(0) + 1}, %[gg_hi]"]
    for q in range(1, L):
        lines += [f"s_add_u32 s{dq(q)}, s{dq(q - 1)}, %[dstep]", f"s_addc_u32 s{dq(q) + 1}, s{dq(q - 1) + 1}, 0",
                  f"s_add_u32 s{gq(q)}, s{gq(q - 1)}, %[gstep]", f"s_addc_u32 s{gq(q) + 1}, s{gq(q - 1) + 1}, 0"]
    B.raw(*lines)
    total = 32 * L

    def issue(t):
        r, q = divmod(t, L)
        out = []
        if q == 0 and r % 8 == 0 and r:  # next row group: every term base 4096 bytes on
            for b in [dq(i) for i in range(L)] + [gq(i) for i in range(L)]:
                out += [f"s_add_u32 s{b}, s{b}, 0x1000", f"s_addc_u32 s{b + 1}, s{b + 1}, 0"]
        X = bufs[t % ring]
        off = 512 * (r % 8)
        out += [f"global_load_dwordx2 {pv(X)}, %[l8], {sp(dq(q))} offset:{off}{LOAD_POLICY}",
                f"global_load_dwordx2 {pv(X + 2)}, %[l8], {sp(gq(q))} offset:{off}{LOAD_POLICY}"]
        return out

    issued = min(ring, total)
    B.raw(*[l for t in range(issued) for l in issue(t)])
    for r in range(32):
        last = r * L + L - 1
        B.raw(f"s_waitcnt vmcnt({2 * (issued - last - 1)})")
        sg = Seg()
        mac_row(sg, L, [bufs[(r * L + q) % ring] for q in range(L)], slot, dmap[r])
        for j, op in enumerate(sg.ops):
            op.idx = j
        B.out(sg.schedule())
        nxt = min(issued + L, total)
        B.raw(*[l for t in range(issued, nxt) for l in issue(t)])
        issued = nxt
        if after_row:
            B.raw(*after_row(r))


def gen_inv_mac(tabs, L, vhi=MAC_VHI):
    B = Body(tabs)
    dmap = [64 + 2 * r for r in range(32)]
    B.raw(f"s_mov_b64 s[{S_EXE}:{S_EXE + 1}], exec", f"s_mov_b32 s{S_X15}, 0x11111111")
    mac_phase(B, L, dmap, vhi)
    B.raw(*gen_bases("g", S_GB), *gen_bases("tw", S_TB))
    ad = NTT_ADDR_W1X if INV_W1X else NTT_ADDR
    B.raw(*par_mask(ad))
    assert INV_W1PP
    dmap = inv_core(B, tabs, dmap, ad, w1pp=True)
    B.raw(*store_rows(dmap, S_GB))
    return B


# The wave-specialised form (r5 probe, not emitted into the library: measured 2-5 % slower than the fused kernel): a two-wave workgroup loops over units; its producer wave
# forms unit u's block of y (mac_phase) while its consumer wave runs the inverse of unit u - 1, so the MAC's memory
# phase and the inverse's issue phase overlap inside every SIMD (the dispatcher puts two producers and two consumers on
# each SIMD, tools/placement_probe.hip) instead of running in lockstep across the device.  Hand-off through the
# workgroup's 16 KiB LDS buffer (row r, lane j at %[yw] + 512 r, %[yw] = buffer + 8 lane); the consumer's transposes
# use a second region.  Per unit both waves execute two s_barriers: (1) the rows are written, (2) the consumer has read
# them (the producer writes the next unit's rows only after it).
WS_LS = (4, 6)   # l (k + 1) of the 3_3 and 4_4 shapes (k = 1, l = 2 / 3); other L keep ntt_tw_inv_mac_kernel


WS_OUT = (124, 126)   # the producer's row results alternate between these pairs (each row's hand-off write reads one)


def emit(name, body, ops_in, sgpr_extra=(), vhi=None):
    clob = ([f'"v{i}"' for i in range(VLO, vhi or VHI)] + [f'"s{i}"' for i in list(SGPR_CLOBBER) + list(sgpr_extra)] +
            ['"scc"', '"memory"'] + (['"vcc"'] if REGROUP_DPP_SELECT else []))
    text = "\n".join(f'      "{l}\\n"' for l in body.lines)
    return (f"// {name}: {body.nvalu} VALU, {len(body.lines)} lines\n"
            f"#define MI_TW_BODY_{name.upper()}(...) asm volatile(\\\n" +
            "\\\n".join(f'      "{l}\\n"' for l in body.lines) +
            f"\\\n      :: __VA_ARGS__ \\\n      : {', '.join(clob)})\n")


def main():
    tabs = load_tables()
    f, i = gen_fwd(tabs), gen_inv(tabs)
    print("// GENERATED by tools/gen_tw_kernel.py — do not edit.  Whole-data-path asm bodies of the twisted")
    print("// N = 2048 Goldilocks transform (ntt64_tw.hip).  Owns v8..v127, s20..s31 + s36..s93, exec (restored).")
    print("#pragma once")
    print(emit("fwd", f, None))
    print(emit("inv", i, None))
    print(emit("fwd_ms64", gen_fwd_ms64(tabs), None, MS_SGPRS))
    for L in MAC_LS:
        print(emit(f"inv_mac{L}", gen_inv_mac(tabs, L), None, range(94, max(94, S_MB + 4 * L)), MAC_VHI))
    print(f"// fwd {f.nvalu} VALU, inv {i.nvalu} VALU", file=sys.stderr)


if __name__ == "__main__":
    main()
