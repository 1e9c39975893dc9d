#!/usr/bin/env python3
"""Issue-cycle model of the generated asm bodies: instruction mix x per-instruction issue cost.

Costs are the MI355X measurements of tools/valu_probe.hip (cycles per wave-instruction per SIMD,
8 waves/SIMD of independent instructions).  The model is what bench.py's
"valu_bound" reports against: cycles per polynomial pass (transform) or per CMUX step (PBS body).

  python tools/valu_cost.py        -> JSON {"fwd", "inv": cycles per polynomial pass; "pbs_step", "pbs_sol_step": per wave
                                      per CMUX step; "ext_bnf": per wave per external product}
  python tools/valu_cost.py --blocks -> the N = 2048 bodies' per-block table (markdown): VALU, modelled cycles and
                                      butterflies per block, and per stage the VALU per butterfly by twiddle exponent
                                      (mod 192; 2 is a primitive 192nd root of unity mod p, so exponent e is the shift
                                      by e bits, e mod 96 = 0 a plus/minus one, 48 the 2^48 = -2^-48... class)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

COST = {  # cycles per wave-instruction (tools/valu_probe.hip on MI355X)
    "v_add_u32": 2.35, "v_sub_u32": 2.34, "v_subrev_u32": 2.34, "v_xor_b32": 2.35, "v_mov_b32": 2.36,
    "v_lshrrev_b32": 2.32, "v_lshlrev_b32": 2.32, "v_not_b32": 2.33, "v_and_b32": 2.35, "v_or_b32": 2.35,
    "v_ashrrev_i32": 2.35,
    "v_add3_u32": 4.26, "v_alignbit_b32": 4.30, "v_cndmask_b32_e64": 4.31, "v_mad_u64_u32": 4.56,
    "v_mad_i64_i32": 4.56, "v_lshl_add_u64": 4.22, "v_mov_b64": 4.21, "v_lshrrev_b64": 4.24,
    "v_lshlrev_b64": 4.24, "v_mul_hi_u32": 4.29, "v_mul_lo_u32": 4.31, "v_mul_u32_u24": 4.27,
    "v_bfe_u32": 4.28, "v_bfe_i32": 4.28, "v_cmp_eq_u32_e64": 4.52, "v_cmp_ge_u64_e64": 4.56, "v_bfi_b32": 4.28, "v_perm_b32": 4.27, "v_cmp_le_u32_e64": 4.52,
    "v_add_co_u32_e64": 4.56, "v_addc_co_u32_e64": 4.57, "v_sub_co_u32_e64": 4.57, "v_subb_co_u32_e64": 4.57,
    "v_mov_b32_dpp": 4.3, "v_permlane32_swap_b32": 8.2,
}


def cycles(lines):
    tot, unknown = 0.0, {}
    for l in lines:
        if not l.startswith("v_"):
            continue
        op = l.split()[0]
        if op not in COST:
            unknown[op] = unknown.get(op, 0) + 1
            tot += 4.3
        else:
            tot += COST[op]
    return tot, unknown


def blocks_table():
    import gen_tw_kernel as T
    tabs = T.load_tables()
    out = ["# Per-block VALU of the N = 2048 twisted transform bodies (tools/valu_cost.py --blocks)", "",
           f"W1x layout: forward {T.FWD_W1X}, inverse {T.INV_W1X}.  VALU = wave instructions, cycles = the issue model "
           "(tools/valu_probe.hip costs).  Butterfly rows: VALU of one butterfly as generated (before scheduling; "
           "canonicalisation folded into the stage that needs it).", ""]
    for name, body in (("forward", T.gen_fwd(tabs)), ("inverse", T.gen_inv(tabs))):
        out += [f"## {name}: {body.nvalu} VALU, {cycles(body.lines)[0]:.0f} cycles", "",
                "| block | VALU | cycles | butterflies | VALU / butterfly |", "|---|---:|---:|---:|---:|"]
        for tag, lines in body.blocks.items():
            nb = sum(len(v) for (t, _), v in body.bfly.items() if t == tag)
            nv = sum(1 for l in lines if l.startswith("v_"))
            out.append(f"| {tag} | {nv} | {cycles(lines)[0]:.0f} | {nb or ''} | {f'{nv / nb:.1f}' if nb else ''} |")
        out += ["", f"### {name}: VALU per butterfly by stage and twiddle exponent (mod 192)", "",
                "| stage | exponent | butterflies | VALU each (min-max) | cycles each (mean) |", "|---|---:|---:|---:|---:|"]
        for (tag, e), bl in sorted(body.bfly.items(), key=lambda kv: (list(body.blocks).index(kv[0][0]), kv[0][1])):
            nv = [sum(1 for l in b if l.startswith("v_")) for b in bl]
            cy = sum(cycles(b)[0] for b in bl) / len(bl)
            out.append(f"| {tag} | {e} | {len(bl)} | {min(nv)}-{max(nv)} | {cy:.1f} |")
        out.append("")
    return "\n".join(out)


def main():
    if "--blocks" in sys.argv:
        print(blocks_table())
        return
    import gen_pbs_kernel as P
    import gen_tw_kernel as T
    tabs = T.load_tables()
    out = {}
    for name, body in (("fwd", T.gen_fwd(tabs)), ("inv", T.gen_inv(tabs))):
        out[name], unk = cycles(body.lines)
        out[name + "_valu"] = body.nvalu
        if unk:
            out[name + "_unpriced"] = unk
    for name, body in (("pbs_step", P.gen_pbs(tabs)), ("pbs_sol_step", P.gen_pbs(tabs, sol=True)),
                       ("ext_bnf", P.gen_ext(tabs, False))):
        out[name], unk = cycles(body.lines)
        out[name + "_valu"] = body.nvalu
        if unk:
            out[name + "_unpriced"] = unk
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in out.items()}))


if __name__ == "__main__":
    main()
