#!/usr/bin/env python3
"""Generate csrc/ntt64_tile_asm.hpp: the forward top-pass arithmetic of the large-N blind rotation's fused rotation +
decomposition pass at K = 5 (pbs_large.hip large_rotdec_tile<5, BNF, ONLY>: the 4_4 shape) as list-scheduled gfx950
asm, r5.  (The K = 2 column pass of 3_3 measured slower as asm — its block-twist values must be resident before the
block starts — and stays compiled C++.)

Compiled C++ spends ~906 VALU per level per wave in the K = 5 tile (64-bit compares for every carry, canonical adds and
subtracts, a general 128-bit reduction per shift twiddle); the butterflies and the block-twist multiply here are
tools/gen_tw_kernel.py's primitives (class-specialised shift multiplies `tmul`, lazy CT cores `ct_core`, the 15-VALU
general multiply `gmul`), with the values bound to fixed VGPR pairs through explicit register constraints
("+{v[a:a+1]}"), so the compiler places the digits there and no copies are needed.

The arithmetic is the transform's first top stages at s0 = 0 (tower twiddles 2^(3 bitrev5(2^s + g)), SURVEY F6,
prime64.rs:166-177), then the block twist (launch_ntt_split, element e times blk_fwd[e]); outputs canonical.

  python tools/gen_tile_asm.py > tfhe-rs-main_modified_amd/csrc/ntt64_tile_asm.hpp
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_tw_kernel as T  # noqa: E402
from gen_tw_kernel import MulSlot, Seg, Slot, canon, ct, gmul, gs, pv  # noqa: E402

XB = 64          # x[k] at v[XB + 2k : XB + 2k + 1]
TB_K5 = 80      # the twist values tw[k] (ONLY passes)
SC_K5 = 96      # scratch: 3 Slots (8 VGPRs each) / 2 MulSlots (12 each) share this block
SG = 36          # SGPR carry pairs s36 .. s53 (3 per Slot; the MulSlots reuse the first 4 pairs)
S_X15 = T.S_X15  # s27 = 0x11111111 (minus_eps), set inside every block


def bitrev5(i):
    return int(format(i, "05b")[::-1], 2)


def tower_exp(s, g, fwd=True):
    """mi_arith.hpp tower_exp(fwd, s, g): stage s, group g of the first five stages -> 2^(3 bitrev5) (forward) or its
    inverse 2^(192 - 3 bitrev5)."""
    r = 3 * bitrev5((1 << s) + g)
    return r if fwd else (192 - r) % 192


def X(k):
    b = XB + 2 * k
    return f"v{b}", f"v{b + 1}", pv(b)


def sched(sg):
    for i, op in enumerate(sg.ops):
        op.idx = i
    return sg.schedule()


def stages_text(pairs_by_stage, scratch):
    """Lines for a list of stages; each stage a list of (register a, register b, exponent) CT butterflies (lazy
    outputs: any 64-bit representative)."""
    slots = [Slot(scratch + 8 * i, SG + 6 * i) for i in range(3)]
    lines = []
    for st in pairs_by_stage:
        sg = Seg()
        for i, (a, b, e) in enumerate(st):
            ct(sg, slots[i % 3], X(a), X(b), e)
        lines += sched(sg)
    return lines


def twist_text(n, tb, scratch):
    """x[k] <- x[k] * tw[k] for k < n, canonical (x any 64-bit value, tw canonical)."""
    ms = [MulSlot(scratch + 12 * i, SG + 4 * i) for i in range(2)]
    sg = Seg()
    for k in range(n):
        x = X(k)
        gmul(sg, ms[k % 2], x, f"v{tb + 2 * k}", f"v{tb + 2 * k + 1}", x[0], x[1])
    return sched(sg)


def tile5_stages(W, phase):
    """The K = 5 cooperative tile (ntt64_tile.hpp): lane (wave W, column c) holds 8 rows; phase A rows W + 4 k, stages
    0..2 (pair distance d / 4 in k); phase B rows 8 W + k, stages 3..4 (distance d)."""
    K, RPT = 5, 8
    out = []
    for S in ((0, 1, 2) if phase == "a" else (3, 4)):
        d = 1 << (K - 1 - S)
        dk = d // 4 if phase == "a" else d
        st = []
        for k in range(RPT):
            if k & dk:
                continue
            row = (W + 4 * k) if phase == "a" else (RPT * W + k)
            st.append((k, k + dk, tower_exp(S, row >> (K - S))))
        out.append(st)
    return out


def gs_stages_text(pairs_by_stage, scratch, canon_in=True, canon_out=True):
    """GS stages (a, b) -> (a + b, (a - b) 2^e) on canonical inputs (the generator's gs keeps both outputs canonical
    then); with canon_out every output is canonical at the end."""
    slots = [Slot(scratch + 8 * i, SG + 6 * i) for i in range(3)]
    flags = {}
    lines = []
    for st in pairs_by_stage:
        sg = Seg()
        for i, (a, b, e) in enumerate(st):
            flags[a], flags[b] = gs(sg, slots[i % 3], X(a), X(b), e, flags.get(a, canon_in), flags.get(b, canon_in))
        lines += sched(sg)
    if canon_out and not all(flags.values()):
        sg = Seg()
        for i, r in enumerate(r for r, f in flags.items() if not f):
            canon(sg, slots[i % 3], X(r))
        lines += sched(sg)
    return lines


def tile5_inv_stages(W, phase):
    """The inverse K = 5 tile (ntt64_tile.hpp phase_b<5, false> then phase_a<5, false>): phase B stages 4, 3 on rows
    8 W + k (distance d), phase A stages 2, 1, 0 on rows W + 4 k (distance d / 4); GS with the inverse tower twiddles."""
    K, RPT = 5, 8
    out = []
    for S in ((4, 3) if phase == "b" else (2, 1, 0)):
        d = 1 << (K - 1 - S)
        dk = d if phase == "b" else d // 4
        st = []
        for k in range(RPT):
            if k & dk:
                continue
            row = (RPT * W + k) if phase == "b" else (W + 4 * k)
            st.append((k, k + dk, tower_exp(S, row >> (K - S), fwd=False)))
        out.append(st)
    return out


def emit_fn(name, lines, n_x, tb, scratch, n_scratch):
    xs = ", ".join(f'"+{{v[{XB + 2 * k}:{XB + 2 * k + 1}]}}"(x[{k}])' for k in range(n_x))
    ins = ", ".join(f'"{{v[{tb + 2 * k}:{tb + 2 * k + 1}]}}"(tw[{k}])' for k in range(n_x)) if tb else ""
    clob = ([f'"v{i}"' for i in range(scratch, scratch + n_scratch)] +
            [f'"s{i}"' for i in list(range(SG, SG + 18)) + [24, 25, S_X15]] + ['"scc"'])
    body = "\n".join(f'      "{l}\\n"' for l in [f"s_mov_b32 s{S_X15}, 0x11111111"] + lines)
    nvalu = sum(1 for l in lines if l.startswith("v_"))
    args = f"u64 (&x)[{n_x}]" + (f", const u64 (&tw)[{n_x}]" if tb else "")
    return (f"// {nvalu} VALU\n"
            f"__device__ __forceinline__ void {name}({args}) {{\n"
            f"  asm volatile(\n{body}\n      : {xs}\n      : {ins}\n      : {', '.join(clob)});\n}}\n")


def main():
    out = ["// GENERATED by tools/gen_tile_asm.py — do not edit.  The large-N blind rotation's forward top-pass",
           "// arithmetic (pbs_large.hip): CT stages with the tower's shift twiddles and the block twist, asm on fixed",
           "// VGPR pairs (explicit register constraints).  Outputs of the *_tw functions are canonical.",
           "#pragma once", "#include <stdint.h>", "namespace mi {", "namespace tile_asm {", "typedef uint64_t u64;", ""]
    for W in range(4):
        out.append(emit_fn(f"k5_fwd_a_w{W}", stages_text(tile5_stages(W, "a"), SC_K5), 8, None, SC_K5, 24))
        lines = stages_text(tile5_stages(W, "b"), SC_K5) + twist_text(8, TB_K5, SC_K5)
        out.append(emit_fn(f"k5_fwd_b_tw_w{W}", lines, 8, TB_K5, SC_K5, 24))
        # (the inverse tile of the accumulating last top pass as asm, tile5_inv_stages / gs_stages_text, measured
        # slower in r5 and is not emitted: the library runs the compiled stages there)
    out += ["}  // namespace tile_asm", "}  // namespace mi"]
    print("\n".join(out))


if __name__ == "__main__":
    main()
