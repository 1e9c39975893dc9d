#!/usr/bin/env python3
"""Generate tfhe-rs-main_modified_amd/csrc/ntt64_view_body.hpp: the Ntt64View conversions of tfhe-rs
(tfhe/src/core_crypto/commons/math/ntt/ntt64.rs:89-266) fused into the twisted N = 2048 Goldilocks bodies of
tools/gen_tw_kernel.py, one hand-scheduled gfx950 asm body each.

Forward side (standard-domain rows in, NTT-domain rows out to another buffer; the wave reads its whole polynomial
before it writes, so the two buffers may be the same):
  FWD_COPY    forward / forward_normalized (ntt64.rs:89-108): copy + Plan::fwd (the normalised form is the same body
              on the plan's N^-1-scaled twist table: the twist multiplies every element exactly once)
  FWD_POW2    forward_from_power_of_two_modulus (ntt64.rs:166-177, 201-214): x -> ((x >> (64 - w)) p + 2^(w-1)) >> w,
              computed as the native switch (x' p + 2^63) >> 64 of x' = x with its low 64 - w bits cleared (the two
              are equal: x' = (x >> (64 - w)) 2^(64 - w)), so one body serves every width (the mask in %[m_lo] / %[m_hi])
  FWD_DECOMP  forward_from_decomp (ntt64.rs:221-240): x -> x + p (wrapping) where x is negative as an i64, i.e.
              x - EPS for x >= 2^63 (always canonical), x otherwise
Inverse side (the NTT-domain rows at %[g_*] are inverted in place, as Plan::inv on the reference's `ntt` buffer, and
added into the standard-domain rows at %[o_*]):
  INV_ADDP    add_backward (ntt64.rs:110-131): standard = wrapping_add_custom_mod(standard, inv(ntt), p), canonical
              inputs -> canonical (a + b) mod p
  INV_ADD64   add_backward_on_power_of_two_modulus at w = 64 (ntt64.rs:184-197, 244-266): ntt = ((v << 64) | p >> 1) / p
              (the OR is an add here: p >> 1 < 2^64), standard += ntt wrapping; q = v + v_hi + [v_lo EPS + p/2 - v_hi
              >= p], the PBS bodies' 6-VALU form (tools/gen_pbs_kernel.py modswitch_acc).  Other widths run the
              generic epilogue kernel (csrc/ntt64_view.hip).

Usage: python tools/gen_view_kernel.py > tfhe-rs-main_modified_amd/csrc/ntt64_view_body.hpp
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_tw_kernel as T  # noqa: E402
from gen_tw_kernel import (JUNK, MS_SGPRS, S_EXE, S_GB, S_H31, S_OB, S_PAR, S_TB, S_X15, Body, Seg, X,  # noqa: E402
                           emit, free_blocks_except, fwd_core, gen_bases, inv_core, load_rows, minus_eps,
                           modswitch_native, pv, store_rows)


def _prologue(B, ad, extra=()):
    B.raw(f"s_mov_b64 s[{S_EXE}:{S_EXE + 1}], exec", f"s_mov_b32 s{S_X15}, 0x11111111",
          f"s_mov_b32 s{S_H31}, 0x80000000", *extra)
    B.raw(*gen_bases("g", S_GB), *gen_bases("tw", S_TB), *gen_bases("o", S_OB))
    B.raw(*T.par_mask(ad))


def _sched(B, sg):
    for i, op in enumerate(sg.ops):
        op.idx = i
    B.out(sg.schedule())


def conv_pow2(sg, sl, x):
    """x <- the switch into Z_p of x's top w bits (ntt64.rs:166-177): clear the low 64 - w bits (mask operands), then
    the native switch (x p + 2^63) >> 64 (gen_tw_kernel.modswitch_native)."""
    xlo, xhi, _ = x
    sg.add(f"v_and_b32 {xlo}, %[m_lo], {xlo}", [xlo], [xlo])
    sg.add(f"v_and_b32 {xhi}, %[m_hi], {xhi}", [xhi], [xhi])
    modswitch_native(sg, sl, x)


def conv_decomp(sg, sl, x):
    """x <- x + p (wrapping) for x negative as an i64 (ntt64.rs:231-238): x - EPS when x >= 2^63 (s28 = 2^31)."""
    xlo, xhi, xp = x
    c = sl.c[0]
    sg.add(f"v_cmp_le_u32_e64 {c}, s{S_H31}, {xhi}", [xhi], [c])
    minus_eps(sg, sl.v[0], c, xp)


def gen_fwd_view(tabs, kind):
    """Standard rows (%[g_*]) -> conversion -> forward transform -> NTT rows (%[o_*])."""
    B = Body(tabs)
    dmap = [64 + 2 * r for r in range(32)]
    ad = T.NTT_ADDR_W1X if T.FWD_W1X else T.NTT_ADDR
    _prologue(B, ad)
    if kind == "copy" and T.PROGRESSIVE:  # as gen_fwd: stage 0 starts as the row pairs (k, k + 16) land
        rows = load_rows(dmap, S_GB)
        B.raw(*[rows[r] for k in range(16) for r in (k, k + 16)])
    else:
        B.raw(*load_rows(dmap, S_GB), "s_waitcnt vmcnt(0)")
    if kind != "copy":
        sg = Seg()
        sls = B.slots(free_blocks_except(dmap))
        for r in range(32):
            (conv_pow2 if kind == "pow2" else conv_decomp)(sg, sls[r % len(sls)], X(dmap, r))
        _sched(B, sg)
    dmap = fwd_core(B, tabs, dmap, ad, prefetch=True)
    B.raw(*store_rows(dmap, S_OB))  # no final vmcnt wait: the wave may retire while its stores drain
    return B


# epilogue registers of the inverse bodies: after inv_core the data sits in v64..v127, v8..v63 are free
BUF_A, BUF_B = 8, 24     # two 8-row buffers of standard-domain rows (16 VGPRs each)
V_C7F = 63               # 0x7fffffff, the high word of p / 2 (a VOP3 carry op reads one SGPR at most: the carry)
EPI_SLOTS = (40, 48)     # the epilogue's scratch slots (8 VGPRs + 3 SGPR carry pairs each)


def std_rows(buf, bt, load):
    """Load (or store) standard-domain rows 8 bt .. 8 bt + 7 into (from) the pairs buf, buf + 2, ..."""
    out = []
    for k in range(8):
        base = f"s[{S_OB + 2 * bt}:{S_OB + 2 * bt + 1}]"
        if load:
            out.append(f"global_load_dwordx2 {pv(buf + 2 * k)}, %[l8], {base} offset:{512 * k}{T.LOAD_POLICY}")
        else:
            out.append(f"global_store_dwordx2 %[l8], {pv(buf + 2 * k)}, {base} offset:{512 * k}{T.STORE_POLICY}")
    return out


def ms_p_to_2_64(sg, sl, x):
    """x <- ((x << 64) | p >> 1) / p for canonical x (ntt64.rs:184-197 at w = 64), in place: q = x + x_hi + c with
    c = [x_lo EPS + (p / 2 - x_hi) >= p] (carry of the mad, or of + EPS after it)."""
    xlo, xhi, _ = x
    v, P, c = sl.v, sl.P, sl.c
    sg.add(f"v_sub_co_u32_e64 {v[0]}, {c[0]}, s{S_H31}, {xhi}", [xhi], [v[0], c[0]])
    sg.add(f"v_subb_co_u32_e64 {v[1]}, {JUNK}, v{V_C7F}, 0, {c[0]}", [c[0], f"v{V_C7F}"], [v[1], JUNK])
    sg.add(f"v_mad_u64_u32 {P[1]}, {c[1]}, {xlo}, -1, {P[0]}", [xlo, P[0]], [P[1], c[1]])
    sg.add(f"v_mad_u64_u32 {P[2]}, {c[2]}, -1, 1, {P[1]}", [P[1]], [P[2], c[2]])
    sg.add(f"s_or_b64 {c[1]}, {c[1]}, {c[2]}", [c[1], c[2]], [c[1], "scc"], "salu")
    sg.add(f"v_addc_co_u32_e64 {xlo}, {c[2]}, {xlo}, {xhi}, {c[1]}", [xlo, xhi, c[1]], [xlo, c[2]])
    sg.add(f"v_addc_co_u32_e64 {xhi}, {JUNK}, {xhi}, 0, {c[2]}", [xhi, c[2]], [xhi, JUNK])


def add_into(sg, sl, a, x, modp):
    """a <- a + x: mod p canonical (both canonical: wrapping_add_custom_mod, unsigned.rs:174-187) or wrapping."""
    alo, ahi = f"v{a}", f"v{a + 1}"
    xlo, xhi, _ = x
    v, P, c = sl.v, sl.P, sl.c
    if not modp:
        sg.add(f"v_add_co_u32_e64 {alo}, {c[0]}, {alo}, {xlo}", [alo, xlo], [alo, c[0]])
        sg.add(f"v_addc_co_u32_e64 {ahi}, {JUNK}, {ahi}, {xhi}, {c[0]}", [ahi, xhi, c[0]], [ahi, JUNK])
        return
    # s = a + x (carry c0), U = s + EPS (carry c1); the sum mod p is U when either carried (s + 2^64 = U mod p, or
    # s >= p), else s
    sg.add(f"v_add_co_u32_e64 {v[0]}, {c[0]}, {alo}, {xlo}", [alo, xlo], [v[0], c[0]])
    sg.add(f"v_addc_co_u32_e64 {v[1]}, {c[0]}, {ahi}, {xhi}, {c[0]}", [ahi, xhi, c[0]], [v[1], c[0]])
    sg.add(f"v_mad_u64_u32 {P[1]}, {c[1]}, -1, 1, {P[0]}", [P[0]], [P[1], c[1]])
    sg.add(f"s_or_b64 {c[1]}, {c[1]}, {c[0]}", [c[1], c[0]], [c[1], "scc"], "salu")
    sg.add(f"v_cndmask_b32_e64 {alo}, {v[0]}, {v[2]}, {c[1]}", [v[0], v[2], c[1]], [alo])
    sg.add(f"v_cndmask_b32_e64 {ahi}, {v[1]}, {v[3]}, {c[1]}", [v[1], v[3], c[1]], [ahi])


def gen_inv_view(tabs, kind):
    """NTT rows (%[g_*]) -> inverse transform -> [switch to 2^64] -> stored back to %[g_*] and added into the
    standard rows (%[o_*])."""
    B = Body(tabs)
    dmap = [64 + 2 * r for r in range(32)]
    ad = T.NTT_ADDR_W1X if T.INV_W1X else T.NTT_ADDR
    _prologue(B, ad)
    B.raw(*load_rows(dmap, S_GB), "s_waitcnt vmcnt(0)")
    dmap = inv_core(B, tabs, dmap, ad, w1pp=True)
    busy = {r for b in dmap for r in (b, b + 1)}
    assert not busy & set(range(8, 64)), "the epilogue expects the inverse's output in v64..v127"
    slots = B.slots(list(EPI_SLOTS))
    # the first two batches of standard rows load while the switch and the ntt stores issue
    B.raw(*std_rows(BUF_A, 0, True), *std_rows(BUF_B, 1, True))
    if kind == "add64":
        B.raw(f"v_mov_b32 v{V_C7F}, 0x7fffffff", f"s_mov_b32 s{S_H31}, 0x80000000")  # inv_core's scratch held both
        sg = Seg()
        for r in range(32):
            ms_p_to_2_64(sg, slots[r % len(slots)], X(dmap, r))
        _sched(B, sg)
    B.raw(*store_rows(dmap, S_GB))  # ntt <- inv(ntt) (switched), as the reference leaves its buffer
    for half in range(2):
        B.raw("s_waitcnt vmcnt(0)")  # loads and stores share vmcnt and need not complete in order
        for j, buf in enumerate((BUF_A, BUF_B)):
            bt = 2 * half + j
            sg = Seg()
            for k in range(8):
                add_into(sg, slots[k % len(slots)], buf + 2 * k, X(dmap, 8 * bt + k), kind == "addp")
            _sched(B, sg)
            B.raw(*std_rows(buf, bt, False))
        if half == 0:  # x2 stores read their data at issue: the buffers may be reloaded right away
            B.raw(*std_rows(BUF_A, 2, True), *std_rows(BUF_B, 3, True))
    return B


BODIES = [("fwd_copy", lambda t: gen_fwd_view(t, "copy")), ("fwd_pow2", lambda t: gen_fwd_view(t, "pow2")),
          ("fwd_decomp", lambda t: gen_fwd_view(t, "decomp")), ("inv_addp", lambda t: gen_inv_view(t, "addp")),
          ("inv_add64", lambda t: gen_inv_view(t, "add64"))]


def main():
    tabs = T.load_tables()
    print("// GENERATED by tools/gen_view_kernel.py — do not edit.  The Ntt64View conversions (ntt64.rs:89-266) fused")
    print("// into the twisted N = 2048 bodies (ntt64_view.hip).  Owns v8..v127, s20..s31 + s36..s101, exec (restored).")
    print("#pragma once")
    for name, gen in BODIES:
        B = gen(tabs)
        print(emit(name, B, None, MS_SGPRS))
        print(f"// {name} {B.nvalu} VALU", file=sys.stderr)


if __name__ == "__main__":
    main()
