#!/usr/bin/env python3
"""Generate hand-scheduled gfx950 inline-asm Goldilocks butterflies (csrc/gl_asm.hpp).

Why: the N = 2048 transform is VALU-issue bound.  On gfx950 a wave64 VOP1/VOP2 instruction
issues in 2 cycles, a VOP3 one (incl. every 64-bit op and `v_mad_u64_u32`) in ~4-4.6, so the
butterfly is written with VCC-carry VOP2 chains around the four 32x32->64 `v_mad_u64_u32`
partial products, and kept fully canonical (outputs in [0, p)), which makes it bit-identical
to the reference whatever the schedule.

Arithmetic (p = 2^64 - 2^32 + 1, EPS = 2^32 - 1; 2^64 = EPS, 2^96 = -1 mod p):
  mul   t = b*w: 128-bit (L, H) by 4 mads; T = L - H1 (-EPS on borrow);
        R = T + H0*EPS (mad, carry c2); t = (c2 | R+EPS carries) ? R + EPS : R      -> t < p
  add   a + t = a - (p - t), + p on borrow                                          -> < p
  sub   a - t, + p on borrow                                                        -> < p
CT (forward, generic_solinas.rs:449-481):  (a, b) -> (a + b*w, a - b*w)
GS (inverse, generic_solinas.rs:483-514):  (a, b) -> (a + b, (a - b)*w)

Scheduling: the butterflies of one block are list-scheduled together (critical path first).
VCC is one shared resource: a VCC value must be consumed before another op may overwrite it,
and every VALU read of VCC / an SGPR written by a VALU needs 2 wait states (gfx950 hazard, as
hipcc itself pads); gaps no independent instruction can fill get `s_nop`.

Usage: python tools/gen_gl_asm.py > tfhe-rs-main_modified_amd/csrc/gl_asm.hpp
"""
import sys

VOP3 = {"v_mad_u64_u32"}


class Op:
    def __init__(self, bf, idx, text, reads, writes):
        self.bf, self.idx, self.text = bf, idx, text
        self.reads, self.writes = set(reads), set(writes)
        self.mnemonic = text.split()[0]
        self.salu = self.mnemonic.startswith("s_")
        self.preds = set()
        self.succs = set()
        self.vcc_src = None  # op whose VCC value this op reads
        self.sgpr_src = {}   # sgpr reg -> producing op
        self.cost = 0 if self.salu else (4.6 if self.mnemonic in VOP3 else 2.0)
        self.prio = 0.0


def regs_of(pairs):
    out = []
    for p in pairs:
        out.append(p)
    return out


class Block:
    """Butterflies scheduled together.  Register names: symbolic per butterfly, resolved later."""

    def __init__(self):
        self.ops = []

    def add_seq(self, bf, seq):
        last_w = {}
        readers = {}
        for i, (text, reads, writes) in enumerate(seq):
            op = Op(bf, i, text, reads, writes)
            for r in op.reads:
                if r in last_w:
                    op.preds.add(last_w[r])
                    if r == "vcc":
                        op.vcc_src = last_w[r]
                    elif r.startswith("sC"):
                        op.sgpr_src[r] = last_w[r]
            for w in op.writes:
                if w == "sJ":
                    continue
                if w in last_w:
                    op.preds.add(last_w[w])  # WAW
                for rd in readers.get(w, []):
                    if rd is not op:
                        op.preds.add(rd)  # WAR
            for r in op.reads:
                readers.setdefault(r, []).append(op)
            for w in op.writes:
                if w == "sJ":
                    continue
                last_w[w] = op
                readers[w] = []
            self.ops.append(op)
        for op in self.ops:
            for p in op.preds:
                p.succs.add(op)

    def schedule(self):
        # priority: longest cost path to the end
        order = list(reversed(self.ops))
        for op in order:
            op.prio = op.cost + max((s.prio for s in op.succs), default=0.0)
        done, out = set(), []
        slot = 0
        issued_at = {}
        vcc_val = None          # op whose value VCC holds
        vcc_pending = {}        # producer -> set of readers not yet issued
        for op in self.ops:
            if op.vcc_src is not None:
                vcc_pending.setdefault(op.vcc_src, set()).add(op)
        remaining = list(self.ops)
        while remaining:
            best = None
            for op in remaining:
                if not all(p in done for p in op.preds):
                    continue
                if op.vcc_src is not None:
                    if vcc_val is not op.vcc_src:
                        continue
                    gap = slot - issued_at[op.vcc_src]
                    need = 1 if op.vcc_src.salu else (2 if op.salu else 3)
                    if gap < need:
                        continue
                ok = True
                for r, src in op.sgpr_src.items():
                    gap = slot - issued_at[src]
                    need = 2 if op.salu else 3
                    if gap < need:
                        ok = False
                if not ok:
                    continue
                if "vcc" in op.writes and vcc_val is not None and vcc_pending.get(vcc_val):
                    if not (op.vcc_src is vcc_val and vcc_pending[vcc_val] == {op}):
                        continue
                key = (op.vcc_src is not None, op.prio, -op.bf)
                if best is None or key > bestkey:
                    best, bestkey = op, key
            if best is None:
                out.append("s_nop 0")
                slot += 1
                continue
            out.append(best.text)
            issued_at[best] = slot
            slot += 1
            done.add(best)
            remaining.remove(best)
            if best.vcc_src is not None:
                vcc_pending[best.vcc_src].discard(best)
            if "vcc" in best.writes:
                vcc_val = best
        return out


# ---------------------------------------------------------------------------------------------
def mul_seq(x0, x1, w0, w1, t0, t1, R):
    """t = x*w canonical.  R: dict of pinned reg names for this butterfly."""
    PA, PAh, PB, PBh, PC, PCh, PD, PDh = R["PA"], R["PAh"], R["PB"], R["PBh"], R["PC"], R["PCh"], R["PD"], R["PDh"]
    Z1, Z1h, Z2, Z2h = R["Z1"], R["Z1h"], R["Z2"], R["Z2h"]
    pA, pB, pC, pD, pZ1, pZ2 = R["pA"], R["pB"], R["pC"], R["pD"], R["pZ1"], R["pZ2"]
    C2 = R["C2"]
    s = []
    s.append((f"v_mov_b32 {Z1h}, 0", [], [Z1h]))
    s.append((f"v_mov_b32 {Z2h}, 0", [], [Z2h]))
    s.append((f"v_mad_u64_u32 {pA}, sJ, {x0}, {w0}, 0", [x0, w0], [PA, PAh, "sJ"]))
    s.append((f"v_mov_b32 {Z1}, {PAh}", [PAh], [Z1]))
    s.append((f"v_mad_u64_u32 {pB}, sJ, {x0}, {w1}, {pZ1}", [x0, w1, Z1, Z1h], [PB, PBh, "sJ"]))
    s.append((f"v_mov_b32 {Z2}, {PB}", [PB], [Z2]))
    s.append((f"v_mov_b32 {Z1}, {PBh}", [PBh], [Z1]))
    s.append((f"v_mad_u64_u32 {pC}, sJ, {x1}, {w0}, {pZ2}", [x1, w0, Z2, Z2h], [PC, PCh, "sJ"]))
    s.append((f"v_mad_u64_u32 {pD}, sJ, {x1}, {w1}, {pZ1}", [x1, w1, Z1, Z1h], [PD, PDh, "sJ"]))
    s.append((f"v_add_co_u32_e32 {PD}, vcc, {PCh}, {PD}", [PCh, PD], [PD, "vcc"]))
    s.append((f"v_addc_co_u32_e32 {PDh}, vcc, 0, {PDh}, vcc", [PDh, "vcc"], [PDh, "vcc"]))
    # T = L - H1 (L = PA.lo : PC.lo), into PB
    s.append((f"v_sub_co_u32_e32 {PB}, vcc, {PA}, {PDh}", [PA, PDh], [PB, "vcc"]))
    s.append((f"v_subbrev_co_u32_e32 {PBh}, vcc, 0, {PC}, vcc", [PC, "vcc"], [PBh, "vcc"]))
    s.append((f"v_cndmask_b32_e64 {Z2}, 0, %[ff], vcc", ["vcc"], [Z2]))
    s.append((f"v_sub_co_u32_e32 {PB}, vcc, {PB}, {Z2}", [PB, Z2], [PB, "vcc"]))
    s.append((f"v_subbrev_co_u32_e32 {PBh}, vcc, 0, {PBh}, vcc", [PBh, "vcc"], [PBh, "vcc"]))
    # R = T + H0*EPS -> PA, carry c2
    s.append((f"v_mad_u64_u32 {pA}, {C2}, {PD}, -1, {pB}", [PD, PB, PBh], [PA, PAh, C2]))
    s.append((f"v_add_co_u32_e32 {PC}, vcc, -1, {PA}", [PA], [PC, "vcc"]))
    s.append((f"v_addc_co_u32_e32 {PCh}, vcc, 0, {PAh}, vcc", [PAh, "vcc"], [PCh, "vcc"]))
    s.append((f"s_or_b64 vcc, vcc, {C2}", ["vcc", C2], ["vcc"]))
    s.append((f"v_cndmask_b32_e64 {t0}, {PA}, {PC}, vcc", [PA, PC, "vcc"], [t0]))
    s.append((f"v_cndmask_b32_e64 {t1}, {PAh}, {PCh}, vcc", [PAh, PCh, "vcc"], [t1]))
    return s


def modsub_seq(d0, d1, a0, a1, b0, b1, M):
    """d = a - b mod p (canonical inputs); M: scratch 32-bit."""
    return [
        (f"v_sub_co_u32_e32 {d0}, vcc, {a0}, {b0}", [a0, b0], [d0, "vcc"]),
        (f"v_subb_co_u32_e32 {d1}, vcc, {a1}, {b1}, vcc", [a1, b1, "vcc"], [d1, "vcc"]),
        (f"v_cndmask_b32_e64 {M}, 0, %[ff], vcc", ["vcc"], [M]),
        (f"v_addc_co_u32_e32 {d0}, vcc, 0, {d0}, vcc", [d0, "vcc"], [d0, "vcc"]),
        (f"v_addc_co_u32_e32 {d1}, vcc, {M}, {d1}, vcc", [M, d1, "vcc"], [d1, "vcc"]),
    ]


def neg_seq(n0, n1, t0, t1):
    """n = p - t (t canonical -> n in (0, p])."""
    return [
        (f"v_sub_co_u32_e32 {n0}, vcc, 1, {t0}", [t0], [n0, "vcc"]),
        (f"v_subb_co_u32_e32 {n1}, vcc, -1, {t1}, vcc", [t1, "vcc"], [n1, "vcc"]),
    ]


def ct_seq(k, R):
    a0, a1, b0, b1, w0, w1 = (f"%[a0_{k}]", f"%[a1_{k}]", f"%[b0_{k}]", f"%[b1_{k}]", f"%[w0_{k}]", f"%[w1_{k}]")
    s = mul_seq(b0, b1, w0, w1, R["PD"], R["PDh"], R)
    t0, t1 = R["PD"], R["PDh"]
    s += neg_seq(R["PB"], R["PBh"], t0, t1)
    s += modsub_seq(b0, b1, a0, a1, t0, t1, R["Z2"])        # b' = a - t
    s += modsub_seq(a0, a1, a0, a1, R["PB"], R["PBh"], R["Z1"])  # a' = a - (p - t) = a + t
    return s


def gs_seq(k, R):
    a0, a1, b0, b1, w0, w1 = (f"%[a0_{k}]", f"%[a1_{k}]", f"%[b0_{k}]", f"%[b1_{k}]", f"%[w0_{k}]", f"%[w1_{k}]")
    s = neg_seq(R["PB"], R["PBh"], b0, b1)                     # n = p - b
    s += modsub_seq(b0, b1, a0, a1, b0, b1, R["Z2"])          # d = a - b (in b)
    s += modsub_seq(a0, a1, a0, a1, R["PB"], R["PBh"], R["Z1"])  # a' = a + b
    s += mul_seq(b0, b1, w0, w1, b0, b1, R)                   # b' = d * w
    return s


def merge_nops(lines):
    out, run = [], 0
    for l in lines + ["<end>"]:
        if l == "s_nop 0":
            run += 1
            continue
        while run > 0:
            n = min(run, 8)
            out.append(f"s_nop {n - 1}")
            run -= n
        if l != "<end>":
            out.append(l)
    return out


def pinned(k, vbase, sbase):
    v = vbase + 12 * k
    R = {}
    for name, off in (("A", 0), ("B", 2), ("C", 4), ("D", 6), ("Z1", 8), ("Z2", 10)):
        lo, hi = v + off, v + off + 1
        key = "P" + name if name in "ABCD" else name
        R[key] = f"v{lo}"
        R[key + "h"] = f"v{hi}"
        R["p" + name] = f"v[{lo}:{hi}]"
    R["C2"] = f"s[{sbase + 2 * k}:{sbase + 2 * k + 1}]"
    return R


def emit(fname, kind, nb, vbase, sbase, junk, wshared):
    blk = Block()
    regs = []
    for k in range(nb):
        R = pinned(k, vbase, sbase)
        seq = ct_seq(k, R) if kind == "ct" else gs_seq(k, R)
        # rename sC / C2 for hazard tracking
        fixed = []
        for text, reads, writes in seq:
            reads = ["sC%d" % k if r == R["C2"] else r for r in reads]
            writes = ["sC%d" % k if w == R["C2"] else w for w in writes]
            fixed.append((text.replace("sJ", f"s[{junk}:{junk + 1}]"), reads, writes))
        blk.add_seq(k, fixed)
        regs += [R[x] for x in ("PA", "PAh", "PB", "PBh", "PC", "PCh", "PD", "PDh", "Z1", "Z1h", "Z2", "Z2h")]
    lines = merge_nops(blk.schedule())
    nops = sum(int(l.split()[1]) + 1 for l in lines if l.startswith("s_nop"))
    nvalu = sum(1 for l in lines if l.startswith("v_"))
    cyc = sum(4.6 if l.startswith("v_mad") else (2.0 if l.startswith("v_") else 0) for l in lines)
    args = []
    for k in range(nb):
        args += [f"u32& a0_{k}", f"u32& a1_{k}", f"u32& b0_{k}", f"u32& b1_{k}"]
    for k in range(nb):
        if wshared and k > 0:
            continue
        args += [f"u32 w0_{k}", f"u32 w1_{k}"]
    outs = []
    for k in range(nb):
        outs += [f'[a0_{k}] "+v"(a0_{k})', f'[a1_{k}] "+v"(a1_{k})', f'[b0_{k}] "+v"(b0_{k})', f'[b1_{k}] "+v"(b1_{k})']
    ins = []
    for k in range(nb):
        src = 0 if wshared else k
        ins += [f'[w0_{k}] "v"(w0_{src})', f'[w1_{k}] "v"(w1_{src})']
    ins.append('[ff] "v"(0xFFFFFFFFu)')
    clob = [f'"{r}"' for r in regs]
    for k in range(nb):
        clob += [f'"s{sbase + 2 * k}"', f'"s{sbase + 2 * k + 1}"']
    clob += [f'"s{junk}"', f'"s{junk + 1}"', '"vcc"', '"scc"']
    body = "\n".join(f'      "{l}\\n"' for l in lines)
    return (f"// {kind.upper()} x{nb}{' (shared twiddle)' if wshared else ''}: {nvalu} VALU ({cyc:.1f} issue cycles), "
            f"{nops} wait states of s_nop padding\n"
            f"__device__ __forceinline__ void {fname}({', '.join(args)}) {{\n"
            f"  asm volatile(\n{body}\n"
            f"      : {', '.join(outs)}\n"
            f"      : {', '.join(ins)}\n"
            f"      : {', '.join(clob)});\n}}\n")


def main():
    vbase = int(sys.argv[1]) if len(sys.argv) > 1 else 80
    sbase, junk = 80, 78
    out = ["// GENERATED by tools/gen_gl_asm.py — do not edit.  Hand-scheduled gfx950 Goldilocks butterflies.",
           "// Pinned scratch: v%d..v%d, s%d..s%d (declared clobbered)." % (vbase, vbase + 12 * 4 - 1, junk, sbase + 7),
           "#pragma once", "#include <stdint.h>", "namespace mi { namespace glasm {", "typedef uint32_t u32;", ""]
    for kind in ("ct", "gs"):
        for nb in (1, 2, 4):
            out.append(emit(f"{kind}{nb}", kind, nb, vbase, sbase, junk, False))
    out.append("}  // namespace glasm\n}  // namespace mi\n")
    print("\n".join(out))


if __name__ == "__main__":
    main()
