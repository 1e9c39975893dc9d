#!/usr/bin/env python3
"""Generate tfhe-rs-main_modified_amd/csrc/pbs_tw_body.hpp: the whole blind-rotation loop of the
BNF programmable bootstrap (level 1) as ONE hand-scheduled gfx950 asm body per wave, built on the
twisted transform cores of tools/gen_tw_kernel.py.

Reference: tfhe/src/core_crypto/algorithms/lwe_programmable_bootstrapping/ntt64_bnf_pbs.rs:208-726
(blind_rotate_ntt64_bnf_assign_mem_optimized -> cmux -> add_external_product_ntt64_bnf_assign).

Work split: one workgroup = 2 waves = one LWE ciphertext.  Wave w owns GLWE polynomial w of the
accumulator (32 coefficients per lane, W0 layout: element 64 r + lane in register pair r) for the
whole loop, in v128..v191.  Per CMUX step i (a_i = ms(lwe[i]) != 0):
  ROT     acc -> own LDS buffer; ct1[e] = +-acc[(e - a) mod N] - acc[e]     (monomial mul + cmux diff)
  DECOMP  level-1 signed decomposition of ct1 (decomposer.rs:156-185, iter.rs:131-151), into [0, p)
  FWD     twisted forward transform (fwd_core)
  MAC     own transform -> own LDS buffer, barrier, partner's rows from its buffer:
          y_w = x_w * G[w][w] + x_{1-w} * G[1-w][w] (mod p, canonical; key pre-multiplied by N^-1)
  INV     twisted inverse transform (inv_core)
  MS      q = v + floor((v EPS + p/2) / p) = v + v_hi + [v_lo EPS + p/2 - v_hi >= p]  (ntt64.rs:184-197)
          acc += q (wrapping)
The step's GGSW rows are prefetched (two 4-row chunks ahead) into v208..v239 while the rotation and
the forward transform run.  At the end acc goes to the wave's LDS buffer in natural order; the C++
wrapper (pbs_tw.hip) does the final rotation by -ms(b) and the sample extraction.

Register map (the body owns v8..v255, s20..s31, s36..s93):
  v8..v127 transform data + scratch, v128..v191 acc, v192..v195 lane*8 + 4096 m (row-group offsets),
  v196..v203 per-lane LDS addresses of the transposes, v204 S, v205 partner exchange address,
  v206 rotation offset, v207 0x7fffffff, v208..v239 GGSW prefetch, v240..v247 partner rows.
The external-product / CMUX bodies (r6) use a second map below v168 (set_regmap / mac_ext): no accumulator held
through the step, the fixed registers in v128..v163, the GGSW chunks in the forward's free scratch, the partner
exchange in 16-row halves; three waves per SIMD.

Usage: python tools/gen_pbs_kernel.py > tfhe-rs-main_modified_amd/csrc/pbs_tw_body.hpp
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_tw_kernel as T  # noqa: E402
from gen_tw_kernel import (JUNK, SG0, Addr, Body, MulSlot, Seg, X, free_blocks_except,  # noqa: E402
                           minus_eps, pv)

ACC = 128
VOFF = 192
V_T1W, V_T1R, V_LWO, V_T2WL, V_T2WH, V_T2R, V_T4W, V_T4R = range(196, 204)
V_S, V_PX, V_U8, V_HHI = 204, 205, 206, 207
GBUF, PBUF = 208, 240

S_SH, S_BM1, S_HALF, S_K1, S_FULL = 26, 28, 29, 30, 31   # s27: T.S_X15
S_TWF, S_TWI, S_GOWN, S_GPAR, S_LWE = 78, 80, 82, 84, 86
S_CNT, S_AMS, S_A, S_R8, S_HLO = 88, 89, 90, 92, 93
S_PHALF = 94   # s[94:95] (Solinas bodies): p / 2 + 1, the sign threshold of the non-native decomposition
SGPR_CLOBBER = list(range(20, 32)) + list(range(36, 94))
SGPR_CLOBBER_SOL = SGPR_CLOBBER + [94, 95]
STEP_BYTES = 4 * 2048 * 8   # one level-1 GGSW (2 x 2 polynomials)


def sp(b):
    return f"s[{b}:{b + 1}]"


V_T1X = 249   # the W1'' inverse's transpose address S + 8 (lane + (lane >> 5)); its read address equals V_T2WL


def addr_for(tab):
    return Addr(lambda bt, k, dst: f"global_load_dwordx2 {pv(dst)}, v{VOFF + bt}, {sp(tab)} offset:{512 * k}",
                t1w=f"v{V_T1W}", t1r=f"v{V_T1R}", t2wl=f"v{V_T2WL}", t2wh=f"v{V_T2WH}", t2r=f"v{V_T2R}",
                t4w=f"v{V_T4W}", t4r=f"v{V_T4R}", lwo=f"v{V_LWO}", lw=sp(tab), t1x=f"v{V_T1X}", t1y=f"v{V_T2WL}")


# The blind-rotation bodies own 16.5 KiB of LDS per wave (PBS_LDS_STRIDE u64): their forward T1 and inverse W1'' -> W0
# transposes run in one pass through a 32 x 66 tile (gen_tw_kernel.t1_full) instead of two lane halves with exec flips
# and three waits.  V_TB = S + 8 (66 (lane >> 1) + (lane & 1)); the tile's other address is V_T4R = S + 8 lane.
PBS_FULL_T = True
PBS_LDS_STRIDE = 32 * 66 if PBS_FULL_T else 2048   # u64 per wave buffer (pbs_tw.hip MI_PBS_LDS_STRIDE)
V_TB = 250
# the lane-pair twiddles (32 forward + the inverse's 32 last-DIT-stage twiddles of the W1'' layout) live in the
# workgroup's LDS (copied by pbs_tw.hip at kernel start): lookups at LDS instead of L2 latency.
# V_LWL = table base + 128 * (lane & 1).
V_LWL = 248


def build_addrs():
    """The transform cores' address objects for the current register map (set_regmap)."""
    global FWD_ADDR, INV_ADDR, FWD_ADDR_P, INV_ADDR_P
    FWD_ADDR, INV_ADDR = addr_for(S_TWF), addr_for(S_TWI)
    FWD_ADDR_P, INV_ADDR_P = addr_for(S_TWF), addr_for(S_TWI)
    for a in (FWD_ADDR_P, INV_ADDR_P):
        a.full_t, a.tfw, a.tfb = PBS_FULL_T, f"v{V_T4R}", f"v{V_TB}"
    for a in (FWD_ADDR, FWD_ADDR_P):
        a.lw_load = lambda dst, k: f"ds_read_b64 {pv(dst)}, v{V_LWL} offset:{8 * k}"
    for a in (INV_ADDR, INV_ADDR_P):
        a.lw_load = lambda dst, k: f"ds_read_b64 {pv(dst)}, v{V_LWL} offset:{256 + 8 * k}"
    for a in (FWD_ADDR, INV_ADDR, FWD_ADDR_P, INV_ADDR_P):
        a.lw_wait = "s_waitcnt lgkmcnt(0)"


build_addrs()

# The external-product / CMUX bodies' register map (r6, EXT_VGPRS): everything below v168, so three waves fit per SIMD
# (512 / 168) instead of two.  The 32 out rows are not held through the step (they are read at the end, 16 rows at a
# time, into the registers the inverse leaves free), the GGSW chunks land in the scratch the forward leaves free (two
# multiply slots instead of four), and the fixed registers pack into v128..v163.
EXT_VGPRS = 168
_PBS_MAP = dict(VOFF=192, V_T1W=196, V_T1R=197, V_LWO=198, V_T2WL=199, V_T2WH=200, V_T2R=201, V_T4W=202, V_T4R=203,
                V_S=204, V_PX=205, V_U8=206, V_HHI=207, GBUF=208, PBUF=240, V_LWL=248, V_T1X=249, V_TB=250)
_EXT_MAP = dict(VOFF=128, V_T1W=132, V_T1R=133, V_LWO=134, V_T2WL=135, V_T2WH=136, V_T2R=137, V_T4W=138, V_T4R=139,
                V_S=140, V_PX=141, V_U8=142, V_HHI=143, V_LWL=144, V_T1X=145, V_TB=146, PBUF=148, GBUF=96)
EXT_PBUF2 = 156   # the partner rows' second buffer (MAC_PARTNER_AHEAD) in the ext map
EXT_LDS_STRIDE = 1088   # u64 per wave: the half-wave transposes (32 x 34, 16 x 66) and a 16-row exchange half


def set_regmap(ext):
    globals().update(_EXT_MAP if ext else _PBS_MAP)
    build_addrs()


def sched(B, sg):
    for i, op in enumerate(sg.ops):
        op.idx = i
    B.out(sg.schedule())


def prologue(B):
    B.raw(f"s_mov_b64 s[{T.S_EXE}:{T.S_EXE + 1}], exec",
          f"s_mov_b32 s{T.S_PAR}, 0xaaaaaaaa", f"s_mov_b32 s{T.S_PAR + 1}, 0xaaaaaaaa",
          f"s_mov_b32 s{T.S_X15}, 0x11111111",
          f"s_mov_b32 s{S_TWF}, %[tab_lo]", f"s_mov_b32 s{S_TWF + 1}, %[tab_hi]",
          f"s_add_u32 s{S_TWI}, %[tab_lo], {2080 * 8}", f"s_addc_u32 s{S_TWI + 1}, %[tab_hi], 0",
          f"s_mov_b32 s{S_GOWN}, %[gown_lo]", f"s_mov_b32 s{S_GOWN + 1}, %[gown_hi]",
          f"s_mov_b32 s{S_GPAR}, %[gpar_lo]", f"s_mov_b32 s{S_GPAR + 1}, %[gpar_hi]",
          # base-log constants: 31 - B, B - 1, 2^(B-1), 2^32 - 2^B + 1
          f"s_sub_u32 s{S_SH}, 31, %[bl]",
          f"s_lshl_b32 s{S_HALF}, 1, %[bl]",
          f"s_mov_b32 s{S_K1}, s{S_HALF}",
          f"s_sub_u32 s{S_BM1}, %[bl], 1",
          f"s_lshr_b32 s{S_HALF}, s{S_HALF}, 1",
          f"s_mov_b32 s{S_HLO}, 0x80000000",
          # per-lane addresses
          f"v_lshlrev_b32 v{VOFF}, 3, %[lane]",
          f"v_add_u32 v{VOFF + 1}, 0x1000, v{VOFF}",
          f"v_add_u32 v{VOFF + 2}, 0x2000, v{VOFF}",
          f"v_add_u32 v{VOFF + 3}, 0x3000, v{VOFF}",
          f"v_mov_b32 v{V_S}, %[S]",
          f"v_add_u32 v{V_PX}, %[SP], v{VOFF}",
          f"v_add_u32 v{V_T4R}, %[S], v{VOFF}",
          f"v_mov_b32 v{V_HHI}, 0x7fffffff",
          "v_and_b32 v8, 31, %[lane]", "v_lshlrev_b32 v8, 3, v8", f"v_add_u32 v{V_T1W}, %[S], v8",
          "v_and_b32 v9, 1, %[lane]", "v_lshrrev_b32 v10, 1, %[lane]",
          "v_mul_u32_u24 v11, 34, v10", "v_add_u32 v11, v11, v9", "v_lshlrev_b32 v11, 3, v11",
          f"v_add_u32 v{V_T1R}, %[S], v11",
          "v_and_b32 v12, 15, v10", "v_mul_u32_u24 v12, 0x42, v12",
          "v_mul_u32_u24 v13, 33, v9", "v_add_u32 v13, v12, v13", "v_lshlrev_b32 v13, 3, v13",
          f"v_add_u32 v{V_T2WL}, %[S], v13",
          "v_mul_u32_u24 v14, 31, v9", "v_add_u32 v14, v12, v14", "v_add_u32 v14, 1, v14",
          "v_lshlrev_b32 v14, 3, v14", f"v_add_u32 v{V_T2WH}, %[S], v14",
          "v_lshrrev_b32 v15, 5, %[lane]", "v_xor_b32 v15, %[lane], v15", "v_lshlrev_b32 v15, 3, v15",
          f"v_add_u32 v{V_T2R}, %[S], v15",
          "v_add_u32 v16, v12, v9", "v_lshlrev_b32 v16, 3, v16", f"v_add_u32 v{V_T4W}, %[S], v16",
          f"v_lshlrev_b32 v{V_LWO}, 7, v9", f"v_add_u32 v{V_LWO}, 0x4000, v{V_LWO}",
          f"v_lshlrev_b32 v{V_LWL}, 7, v9", f"v_add_u32 v{V_LWL}, %[LW], v{V_LWL}",
          "v_lshrrev_b32 v17, 5, %[lane]", "v_add_u32 v17, %[lane], v17", "v_lshlrev_b32 v17, 3, v17",
          f"v_add_u32 v{V_T1X}, %[S], v17",
          "v_mul_u32_u24 v18, 66, v10", "v_add_u32 v18, v18, v9", "v_lshlrev_b32 v18, 3, v18",
          f"v_add_u32 v{V_TB}, %[S], v18")


def load_rows(dst, base):
    return [f"global_load_dwordx2 {pv(dst + 2 * r)}, v{VOFF + r // 8}, {sp(base)} offset:{512 * (r % 8)}"
            for r in range(32)]


def store_rows(src, base):
    return [f"global_store_dwordx2 v{VOFF + r // 8}, {pv(src + 2 * r)}, {sp(base)} offset:{512 * (r % 8)}{T.STORE_POLICY}"
            for r in range(32)]


def load_rows_sub(dst, base, rows):
    return [f"global_load_dwordx2 {pv(dst + 2 * q)}, v{VOFF + r // 8}, {sp(base)} offset:{512 * (r % 8)}"
            for q, r in enumerate(rows)]


def store_rows_sub(src, base, rows):
    return [f"global_store_dwordx2 v{VOFF + r // 8}, {pv(src + 2 * q)}, {sp(base)} offset:{512 * (r % 8)}{T.STORE_POLICY}"
            for q, r in enumerate(rows)]


def gload(c):
    """GGSW rows of MAC chunk c (rows 4c..4c+3) of this step into prefetch buffer c % 2."""
    out = []
    base = GBUF + 16 * (c % 2)
    for k in range(4):
        r = 4 * c + k
        out.append(f"global_load_dwordx2 {pv(base + 2 * k)}, v{VOFF + r // 8}, {sp(S_GOWN)} offset:{512 * (r % 8)}")
        out.append(f"global_load_dwordx2 {pv(base + 8 + 2 * k)}, v{VOFF + r // 8}, {sp(S_GPAR)} offset:{512 * (r % 8)}")
    return out


def slots_at(bases):
    return [T.Slot(b, SG0 + 6 * i) for i, b in enumerate(bases)]


def decompose(sg, sl, xl, xh, signed=False):
    """Level-1 signed decomposition of the native u64 (xl, xh) in place (closest representable +
    one balanced digit, decomposer.rs:156-185 + iter.rs:131-151), mapped into [0, p) (ntt64.rs:231-238).
    With t = the top B + 1 bits of x (rounding bit last) the reference's digit is
    sext_B(((t + 1) >> 1) mod 2^B), except t == 2^B (res == 2^(B-1) with a clear rounding bit, the
    one tie that is not balanced), where it is +2^(B-1) = -sext_B(...).  The signed digit d becomes
    d mod p as the sign-extended pair (d, d >> 31) plus (-15 [d < 0]) * 0x11111111 = -EPS [d < 0]."""
    v, c = sl.v, sl.c
    t, s, nd, m = v[1], v[2], v[3], v[4]
    sg.add(f"v_lshrrev_b32 {t}, s{S_SH}, {xh}", [xh], [t])
    sg.add(f"v_add_u32 {s}, 1, {t}", [t], [s])
    sg.add(f"v_bfe_i32 {xl}, {s}, 1, %[bl]", [s], [xl])
    sg.add(f"v_cmp_eq_u32_e64 {c[2]}, s{S_K1}, {t}", [t], [c[2]])
    sg.add(f"v_sub_u32 {nd}, 0, {xl}", [xl], [nd])
    sg.add(f"v_cndmask_b32_e64 {xl}, {xl}, {nd}, {c[2]}", [xl, nd, c[2]], [xl])
    if signed:  # the signed digit in xl only: stage0_signed consumes it
        return
    sg.add(f"v_ashrrev_i32 {xh}, 31, {xl}", [xl], [xh])
    sg.add(f"v_and_b32 {m}, -15, {xh}", [xh], [m])
    xp = pv(int(xl[1:]))
    sg.add(f"v_mad_i64_i32 {xp}, {JUNK}, {m}, s{T.S_X15}, {xp}", [m, xl, xh], [xl, xh, JUNK])


def decompose_sol(sg, sl, xl, xh, signed=False):
    """Level-1 signed decomposition of x in [0, p] modulo the Solinas prime, in place, mapped into
    [0, p): TensorSignedDecompositionLendingIterNonNative (iter.rs:623-745) with one level.  The sign is
    s = x >= p / 2 + 1 (div_ceil), the magnitude |x| = s ? p - x : x < 2^63, the rounded state
    (closest_abs_nonnative, decomposer.rs:521-548) ((|x| >> (63 - B)) + 1) >> 1 <= 2^(B-1), so the one
    level's digit is that state itself (decompose_one_level never carries here); the signed digit
    d = s ? -state : state becomes d mod p as in `decompose` (x = p decomposes like 0)."""
    v, c = sl.v, sl.c
    nl, nh, t = v[1], v[2], v[3]
    sg.add(f"v_cmp_ge_u64_e64 {c[2]}, {T.pv(int(xl[1:]))}, s[{S_PHALF}:{S_PHALF + 1}]", [xl, xh], [c[2]])
    sg.add(f"v_sub_co_u32_e64 {nl}, {c[0]}, 1, {xl}", [xl], [nl, c[0]])
    sg.add(f"v_subb_co_u32_e64 {nh}, {JUNK}, -1, {xh}, {c[0]}", [xh, c[0]], [nh, JUNK])
    sg.add(f"v_cndmask_b32_e64 {nh}, {xh}, {nh}, {c[2]}", [xh, nh, c[2]], [nh])       # |x| high word
    sg.add(f"v_lshrrev_b32 {t}, s{S_SH}, {nh}", [nh], [t])                          # top B + 1 bits
    sg.add(f"v_add_u32 {t}, 1, {t}", [t], [t])
    sg.add(f"v_lshrrev_b32 {t}, 1, {t}", [t], [t])                                  # state = digit
    sg.add(f"v_sub_u32 {nl}, 0, {t}", [t], [nl])
    sg.add(f"v_cndmask_b32_e64 {xl}, {t}, {nl}, {c[2]}", [t, nl, c[2]], [xl])
    if signed:
        return
    sg.add(f"v_ashrrev_i32 {xh}, 31, {xl}", [xl], [xh])
    m = v[4]
    sg.add(f"v_and_b32 {m}, -15, {xh}", [xh], [m])
    xp = pv(int(xl[1:]))
    sg.add(f"v_mad_i64_i32 {xp}, {JUNK}, {m}, s{T.S_X15}, {xp}", [m, xl, xh], [xl, xh, JUNK])


def stage0_signed(B, tabs, dmap, rows=range(16)):
    """The forward's first stage (registers r, r + 16, twiddle 2^48) straight from the signed level-1 digits the
    decomposition leaves in the low words (|d| < 2^31), instead of mapping each digit into [0, p) and running a
    general shift-class butterfly.  With bh = d_b >> 16 (arithmetic) and T = (d_b mod 2^16) 2^48 (high word
    d_b << 16, low word 0): d_b 2^48 = T + bh 2^64 = T + bh EPS (mod p), so a + d_b 2^48 = S0 + T and
    a - d_b 2^48 = S1 - T with S0 = d_a + bh EPS = sext(d_a - bh) + bh 2^32 and S1 = d_a - bh EPS =
    sext(d_a + bh) - bh 2^32 (|S| < 2^47), each made canonical (S < 0: S - EPS mod 2^64 = S + p).  T < p, so
    a' = S0 + T (one carry fix) and b' = S1 - T (one borrow fix) need only high-word arithmetic: 16 VALU, 12 of
    them single-rate 32-bit ops, per butterfly, and no digit is ever mapped into [0, p) on its own."""
    assert all(e == 48 for e in tabs["G1_FWD"][0]), "stage 0 twiddle is not 2^48"
    sg = Seg()
    sls = B.slots(free_blocks_except(dmap))
    for r in rows:
        sl = sls[r % len(sls)]
        v, c = sl.v, sl.c
        al, ah, ap = X(dmap, r)
        bl, bh, bp = X(dmap, r + 16)
        hb, th, m0, m1 = v[0], v[1], v[2], v[3]
        sg.add(f"v_ashrrev_i32 {hb}, 16, {bl}", [bl], [hb])                      # bh = d_b >> 16
        sg.add(f"v_lshlrev_b32 {th}, 16, {bl}", [bl], [th])                      # T high word
        sg.add(f"v_add_u32 {bl}, {al}, {hb}", [al, hb], [bl])                    # S1 = sext(d_a + bh) - bh 2^32
        sg.add(f"v_sub_u32 {al}, {al}, {hb}", [al, hb], [al])                    # S0 = sext(d_a - bh) + bh 2^32
        sg.add(f"v_ashrrev_i32 {bh}, 31, {bl}", [bl], [bh])
        sg.add(f"v_sub_u32 {bh}, {bh}, {hb}", [bh, hb], [bh])
        sg.add(f"v_ashrrev_i32 {ah}, 31, {al}", [al], [ah])
        sg.add(f"v_add_u32 {ah}, {ah}, {hb}", [ah, hb], [ah])
        for (lo, hi, pair, m) in ((al, ah, ap, m0), (bl, bh, bp, m1)):            # S < 0: S + p
            sg.add(f"v_ashrrev_i32 {m}, 31, {hi}", [hi], [m])
            sg.add(f"v_and_b32 {m}, -15, {m}", [m], [m])
            sg.add(f"v_mad_i64_i32 {pair}, {JUNK}, {m}, s{T.S_X15}, {pair}", [m, lo, hi], [lo, hi, JUNK])
        sg.add(f"v_sub_co_u32_e64 {bh}, {c[0]}, {bh}, {th}", [bh, th], [bh, c[0]])   # b' = S1 - T
        minus_eps(sg, v[4], c[0], bp)
        sg.add(f"v_add_co_u32_e64 {ah}, {c[1]}, {ah}, {th}", [ah, th], [ah, c[1]])   # a' = S0 + T
        sg.add(f"v_cndmask_b32_e64 {v[5]}, 0, -1, {c[1]}", [c[1]], [v[5]])
        sg.add(f"v_mad_u64_u32 {ap}, {JUNK}, {v[5]}, 1, {ap}", [v[5], al, ah], [al, ah, JUNK])
    sched(B, sg)


# the rotation's 32 LDS reads issued together (one exposed LDS round trip instead of two): emulator-exact, but BNF
# 35.9 k -> 35.2 k PBS/s in a one-box A/B (profiles/r3/pbs_rot_all_reads_ab/): off
ROT_ALL_READS = False


def rotate_decompose(B, sol=False):
    """dmap v64..v127 <- decompose(+-acc[(e - a) mod N] - acc[e]); Solinas bodies negate and subtract
    modulo p (polynomial_wrapping_monic_monomial_mul_assign_custom_mod, then the CMUX difference)."""
    B.raw(f"s_and_b32 s{S_R8}, s{S_AMS}, 0x7ff", f"s_lshl_b32 s{S_R8}, s{S_R8}, 3",
          f"s_lshr_b32 s{S_FULL}, s{S_AMS}, 11", f"s_sub_u32 s{S_FULL}, 0, s{S_FULL}",
          f"v_subrev_u32 v{V_U8}, s{S_R8}, v{VOFF}")
    B.raw(*[f"ds_write_b64 v{V_T4R}, {pv(ACC + 2 * r)} offset:{512 * r}" for r in range(32)])
    if ROT_ALL_READS:
        # all 32 source addresses (v8..v39), all 32 reads in flight, then half 0 computes while half 1 lands
        sg = Seg()
        for r in range(32):
            a = f"v{8 + r}"
            sg.add(f"v_add_u32 {a}, {512 * r}, v{V_U8}", [f"v{V_U8}"], [a])
            sg.add(f"v_and_b32 {a}, 0x3ff8, {a}", [a], [a])
            sg.add(f"v_add_u32 {a}, %[S], {a}", [a], [a])
        sched(B, sg)
        B.raw(*[f"ds_read_b64 {pv(64 + 2 * r)}, v{8 + r}" for r in range(32)])
    for h in range(2):
        rows = list(range(16 * h, 16 * h + 16))
        if ROT_ALL_READS:
            B.raw("s_waitcnt lgkmcnt(15)" if h == 0 else "s_waitcnt lgkmcnt(0)")  # (in order: <= 15 left = rows 0..16)
        else:
            sg = Seg()
            for q, r in enumerate(rows):
                a = f"v{8 + q}"
                sg.add(f"v_add_u32 {a}, {512 * r}, v{V_U8}", [f"v{V_U8}"], [a])
                sg.add(f"v_and_b32 {a}, 0x3ff8, {a}", [a], [a])
                sg.add(f"v_add_u32 {a}, %[S], {a}", [a], [a])
            sched(B, sg)
            B.raw(*[f"ds_read_b64 {pv(64 + 2 * r)}, v{8 + q}" for q, r in enumerate(rows)], "s_waitcnt lgkmcnt(0)")
        sg = Seg()
        sls = slots_at([8, 16, 24, 32, 40, 48, 56])
        for q, r in enumerate(rows):
            sl = sls[q % len(sls)]
            v, c = sl.v, sl.c
            xl, xh = f"v{64 + 2 * r}", f"v{65 + 2 * r}"
            al, ah = f"v{ACC + 2 * r}", f"v{ACC + 2 * r + 1}"
            m = v[0]
            sg.add(f"v_add_u32 {m}, {512 * r}, v{V_U8}", [f"v{V_U8}"], [m])
            sg.add(f"v_ashrrev_i32 {m}, 31, {m}", [m], [m])
            sg.add(f"v_xor_b32 {m}, s{S_FULL}, {m}", [m], [m])
            if sol:
                # m = -1: p - x (p for x = 0, which later decomposes like 0); then - acc mod p
                nl, nh = v[6], v[7]
                sg.add(f"v_sub_co_u32_e64 {nl}, {c[0]}, 1, {xl}", [xl], [nl, c[0]])
                sg.add(f"v_subb_co_u32_e64 {nh}, {JUNK}, -1, {xh}, {c[0]}", [xh, c[0]], [nh, JUNK])
                sg.add(f"v_bfi_b32 {xl}, {m}, {nl}, {xl}", [m, nl, xl], [xl])
                sg.add(f"v_bfi_b32 {xh}, {m}, {nh}, {xh}", [m, nh, xh], [xh])
                sg.add(f"v_sub_co_u32_e64 {xl}, {c[0]}, {xl}, {al}", [xl, al], [xl, c[0]])
                sg.add(f"v_subb_co_u32_e64 {xh}, {c[1]}, {xh}, {ah}, {c[0]}", [xh, ah, c[0]], [xh, c[1]])
                minus_eps(sg, v[5], c[1], pv(int(xl[1:])))
                decompose_sol(sg, sl, xl, xh, signed=True)
                continue
            sg.add(f"v_xor_b32 {xl}, {m}, {xl}", [m, xl], [xl])
            sg.add(f"v_xor_b32 {xh}, {m}, {xh}", [m, xh], [xh])
            sg.add(f"v_sub_co_u32_e64 {xl}, {c[0]}, {xl}, {m}", [xl, m], [xl, c[0]])
            sg.add(f"v_subb_co_u32_e64 {xh}, {JUNK}, {xh}, {m}, {c[0]}", [xh, m, c[0]], [xh, JUNK])
            sg.add(f"v_sub_co_u32_e64 {xl}, {c[1]}, {xl}, {al}", [xl, al], [xl, c[1]])
            sg.add(f"v_subb_co_u32_e64 {xh}, {JUNK}, {xh}, {ah}, {c[1]}", [xh, ah, c[1]], [xh, JUNK])
            decompose(sg, sl, xl, xh, signed=True)
        sched(B, sg)


def prod128(sg, ms, x, wlo, whi):
    """Full 128-bit x * w (x, w < 2^64) in multiply slot ms: low 64 bits in (A0, C0) = ms.v[0], ms.v[4],
    high 64 bits in the PB pair (ms.v[2:3]).  The slot's Z1h / Z2h must hold 0 (set once per MAC)."""
    xlo, xhi, _ = x
    v, P = ms.v, ms.P
    PA, PB, PC, PD, Z1, Z2 = P
    A1, B0, B1, C1, Z1l, Z2l = v[1], v[2], v[3], v[5], v[8], v[10]
    sg.add(f"v_mad_u64_u32 {PA}, {JUNK}, {xlo}, {wlo}, 0", [xlo, wlo], [PA, JUNK])             # A = xl wl
    sg.add(f"v_mov_b32 {Z1l}, {A1}", [A1], [Z1l])
    sg.add(f"v_mad_u64_u32 {PB}, {JUNK}, {xlo}, {whi}, {Z1}", [xlo, whi, Z1], [PB, JUNK])      # B = xl wh + A1
    sg.add(f"v_mov_b32 {Z2l}, {B0}", [B0], [Z2l])
    sg.add(f"v_mov_b32 {Z1l}, {B1}", [B1], [Z1l])
    sg.add(f"v_mad_u64_u32 {PC}, {JUNK}, {xhi}, {wlo}, {Z2}", [xhi, wlo, Z2], [PC, JUNK])      # C = xh wl + B0
    sg.add(f"v_mad_u64_u32 {PD}, {JUNK}, {xhi}, {whi}, {Z1}", [xhi, whi, Z1], [PD, JUNK])      # D = xh wh + B1
    sg.add(f"v_mad_u64_u32 {PB}, {JUNK}, {C1}, 1, {PD}", [C1, PD], [PB, JUNK])                # H = D + C1


def mac2(sg, m1, m2, x, g1, p, g2):
    """x <- (x * g1 + p * g2) mod p, canonical, with ONE reduction: both 128-bit products are summed
    exactly (carry c out of bit 128; 2^128 = -2^32 mod p), then reduced as in gmul:
    L + H0 * EPS - H1 - c * 2^32 (2^64 = EPS, 2^96 = -1).  33 VALU instead of 2 x 17 + 5."""
    prod128(sg, m1, x, *g1)
    prod128(sg, m2, p, *g2)
    a, b = m1.v, m2.v
    ca, cb = m1.c[0], m1.c[1]
    cs = m2.c[0]
    # (s0, s1, s2, s3) = (A0, C0, H) + (A0', C0', H'), carry out of bit 128 in cs
    sg.add(f"v_add_co_u32_e64 {a[0]}, {cs}, {a[0]}, {b[0]}", [a[0], b[0]], [a[0], cs])
    sg.add(f"v_addc_co_u32_e64 {a[4]}, {cs}, {a[4]}, {b[4]}, {cs}", [a[4], b[4], cs], [a[4], cs])
    sg.add(f"v_addc_co_u32_e64 {a[2]}, {cs}, {a[2]}, {b[2]}, {cs}", [a[2], b[2], cs], [a[2], cs])
    sg.add(f"v_addc_co_u32_e64 {a[3]}, {cs}, {a[3]}, {b[3]}, {cs}", [a[3], b[3], cs], [a[3], cs])
    c2 = a[6]
    sg.add(f"v_cndmask_b32_e64 {c2}, 0, 1, {cs}", [cs], [c2])
    # T = (s0, s1) - (s3 + c * 2^32); a borrow adds p (T - EPS mod 2^64, no second wrap: T >= 2^64 - 2^33)
    T = m2.P[3]
    t0, t1 = b[6], b[7]
    sg.add(f"v_sub_co_u32_e64 {t0}, {ca}, {a[0]}, {a[3]}", [a[0], a[3]], [t0, ca])
    sg.add(f"v_subb_co_u32_e64 {t1}, {cb}, {a[4]}, {c2}, {ca}", [a[4], c2, ca], [t1, cb])
    minus_eps(sg, b[10], cb, T)
    # R = T + s2 * EPS, U = R + EPS; canonical result = (carry(R) | carry(U)) ? U : R
    PA, PC = m1.P[0], m1.P[2]
    sg.add(f"v_mad_u64_u32 {PA}, {ca}, {a[2]}, -1, {T}", [a[2], T], [PA, ca])
    sg.add(f"v_mad_u64_u32 {PC}, {cb}, -1, 1, {PA}", [PA], [PC, cb])
    sg.add(f"s_or_b64 {cb}, {cb}, {ca}", [cb, ca], [cb, "scc"], "salu")
    xlo, xhi, _ = x
    sg.add(f"v_cndmask_b32_e64 {xlo}, {a[0]}, {a[4]}, {cb}", [a[0], a[4], cb], [xlo])
    sg.add(f"v_cndmask_b32_e64 {xhi}, {a[1]}, {a[5]}, {cb}", [a[1], a[5], cb], [xhi])


# The partner's rows of MAC chunk c + 1 are read while chunk c multiplies (a second 4-row buffer in the registers the
# multiply slots leave free), so each chunk waits only for its GGSW rows, not for an LDS round trip as well.
MAC_PARTNER_AHEAD = True


def mac(B, dmap):
    B.raw(*[f"ds_write_b64 v{V_T4R}, {pv(dmap[r])} offset:{512 * r}" for r in range(32)],
          "s_waitcnt lgkmcnt(0)", "s_barrier")
    free = free_blocks_except(dmap)
    regs = []
    for b in free:
        regs += list(range(b, b + 8))
    ms = [MulSlot(regs[12 * i], SG0 + 6 * i) for i in range(4)]
    # the zero high halves of the product addends, set once for the whole MAC (prod128)
    B.raw(*[f"v_mov_b32 {m.v[z]}, 0" for m in ms for z in (9, 11)])
    ahead = MAC_PARTNER_AHEAD and len(regs) >= 56
    pbufs = [PBUF, regs[48]] if ahead else [PBUF]
    assert not ahead or regs[48:56] == list(range(regs[48], regs[48] + 8)), regs
    pread = lambda c: [f"ds_read_b64 {pv(pbufs[c % len(pbufs)] + 2 * k)}, v{V_PX} offset:{512 * (4 * c + k)}"
                       for k in range(4)]
    if ahead:
        B.raw(*pread(0))
    for c in range(8):
        if ahead:
            # chunk c's partner rows were issued a chunk ago: allow the next chunk's 4 reads to stay in flight
            nxt = pread(c + 1) if c + 1 < 8 else []
            B.raw(*nxt, f"s_waitcnt vmcnt({8 if c < 7 else 0}) lgkmcnt({len(nxt)})")
        else:
            B.raw(*pread(c), f"s_waitcnt vmcnt({8 if c < 7 else 0}) lgkmcnt(0)")
        pb = pbufs[c % len(pbufs)]
        sg = Seg()
        gb = GBUF + 16 * (c % 2)
        for k in range(4):
            r = 4 * c + k
            m1, m2 = ms[(2 * k) % 4], ms[(2 * k + 1) % 4]
            x = X(dmap, r)
            pl, ph = f"v{pb + 2 * k}", f"v{pb + 2 * k + 1}"
            mac2(sg, m1, m2, x, (f"v{gb + 2 * k}", f"v{gb + 2 * k + 1}"), (pl, ph, pv(pb + 2 * k)),
                 (f"v{gb + 8 + 2 * k}", f"v{gb + 9 + 2 * k}"))
        sched(B, sg)
        if c + 2 < 8:
            B.raw(*gload(c + 2))
    B.raw("s_barrier")


def mac_ext(B, dmap):
    """The MAC of the ext-map bodies (set_regmap(True)): the exchange with the partner wave in two halves of 16 rows
    (8 KiB of LDS per wave instead of 16), the GGSW chunks double-buffered in the forward's free scratch (GBUF = v96),
    two multiply slots in v40..v63, the partner rows in PBUF / EXT_PBUF2.  dmap: the forward's W1' output in
    v8..v39 + v64..v95 (the non-full_t transposes)."""
    assert dmap == [8 + 2 * q for q in range(16)] + [64 + 2 * q for q in range(16)], dmap
    ms = [MulSlot(40, SG0), MulSlot(52, SG0 + 6)]
    B.raw(*gload(0), *gload(1))
    B.raw(*[f"v_mov_b32 {m.v[z]}, 0" for m in ms for z in (9, 11)])
    pbufs = [PBUF, EXT_PBUF2]
    pread = lambda c: [f"ds_read_b64 {pv(pbufs[c % 2] + 2 * k)}, v{V_PX} offset:{512 * (4 * (c % 4) + k)}"
                       for k in range(4)]
    for h in range(2):
        if h:  # the partner has read this wave's first half
            B.raw("s_barrier")
        B.raw(*[f"ds_write_b64 v{V_T4R}, {pv(dmap[16 * h + q])} offset:{512 * q}" for q in range(16)],
              "s_waitcnt lgkmcnt(0)", "s_barrier", *pread(4 * h))
        for c in range(4 * h, 4 * h + 4):
            nxt = pread(c + 1) if c + 1 < 4 * h + 4 else []
            B.raw(*nxt, f"s_waitcnt vmcnt({8 if c < 7 else 0}) lgkmcnt({len(nxt)})")
            pb = pbufs[c % 2]
            sg = Seg()
            gb = GBUF + 16 * (c % 2)
            for k in range(4):
                r = 4 * c + k
                m1, m2 = ms
                x = X(dmap, r)
                pl, ph = f"v{pb + 2 * k}", f"v{pb + 2 * k + 1}"
                mac2(sg, m1, m2, x, (f"v{gb + 2 * k}", f"v{gb + 2 * k + 1}"), (pl, ph, pv(pb + 2 * k)),
                     (f"v{gb + 8 + 2 * k}", f"v{gb + 9 + 2 * k}"))
            sched(B, sg)
            if c + 2 < 8:
                B.raw(*gload(c + 2))
    B.raw("s_barrier")


def w1pp_regs(dmap):
    """Register plan of the W1'' inverse after the MAC (dmap: rows 0..15 at v96.., rows 16..31 at v64..): the
    transposed data in v8..v63 + the first four pairs of rows 0..15, the lane-pair twiddles in v64..v71 (rows
    16.. are in LDS by then), the output's first half in v64.. and its second in v96.."""
    assert dmap == [96 + 2 * r for r in range(16)] + [64 + 2 * r for r in range(16)], dmap
    return dict(dst=[8 + 2 * r for r in range(28)] + [96 + 2 * r for r in range(4)], pre_base=64, ybase=64, newhi=96)


def modswitch_acc(B, dmap, rows=range(32), acc=None, sls=None):
    """acc += ms_{p -> 2^64}(y) for the rows of y (dmap); acc[r] at `acc` + 2 q for the q-th row (default ACC + 2 r)."""
    sg = Seg()
    sls = sls or B.slots(free_blocks_except(dmap))
    for q, r in enumerate(rows):
        sl = sls[q % len(sls)]
        v, P, c = sl.v, sl.P, sl.c
        vl, vh, _ = X(dmap, r)
        a = ACC + 2 * r if acc is None else acc + 2 * q
        al, ah = f"v{a}", f"v{a + 1}"
        sg.add(f"v_sub_co_u32_e64 {v[0]}, {c[0]}, s{S_HLO}, {vh}", [vh], [v[0], c[0]])
        sg.add(f"v_subb_co_u32_e64 {v[1]}, {JUNK}, v{V_HHI}, 0, {c[0]}", [c[0]], [v[1], JUNK])
        sg.add(f"v_mad_u64_u32 {P[1]}, {c[1]}, {vl}, -1, {P[0]}", [vl, P[0]], [P[1], c[1]])
        sg.add(f"v_mad_u64_u32 {P[2]}, {c[2]}, -1, 1, {P[1]}", [P[1]], [P[2], c[2]])
        sg.add(f"s_or_b64 {c[1]}, {c[1]}, {c[2]}", [c[1], c[2]], [c[1], "scc"], "salu")
        sg.add(f"v_addc_co_u32_e64 {v[6]}, {c[2]}, {vl}, {vh}, {c[1]}", [vl, vh, c[1]], [v[6], c[2]])
        sg.add(f"v_addc_co_u32_e64 {v[7]}, {JUNK}, {vh}, 0, {c[2]}", [vh, c[2]], [v[7], JUNK])
        sg.add(f"v_add_co_u32_e64 {al}, {c[0]}, {al}, {v[6]}", [al, v[6]], [al, c[0]])
        sg.add(f"v_addc_co_u32_e64 {ah}, {JUNK}, {ah}, {v[7]}, {c[0]}", [ah, v[7], c[0]], [ah, JUNK])
    sched(B, sg)


def add_acc_sol(B, dmap, rows=range(32), acc=None, sls=None):
    """acc <- acc + y mod p, canonical (both canonical): ntt64.rs:244-266 add_backward, custom modulus."""
    sg = Seg()
    sls = sls or B.slots(free_blocks_except(dmap))
    for q, r in enumerate(rows):
        sl = sls[q % len(sls)]
        v, P, c = sl.v, sl.P, sl.c
        vl, vh, _ = X(dmap, r)
        a = ACC + 2 * r if acc is None else acc + 2 * q
        al, ah = f"v{a}", f"v{a + 1}"
        sg.add(f"v_add_co_u32_e64 {v[0]}, {c[0]}, {al}, {vl}", [al, vl], [v[0], c[0]])
        sg.add(f"v_addc_co_u32_e64 {v[1]}, {c[0]}, {ah}, {vh}, {c[0]}", [ah, vh, c[0]], [v[1], c[0]])
        sg.add(f"v_mad_u64_u32 {P[1]}, {c[1]}, -1, 1, {P[0]}", [P[0]], [P[1], c[1]])
        sg.add(f"s_or_b64 {c[1]}, {c[1]}, {c[0]}", [c[1], c[0]], [c[1], "scc"], "salu")
        sg.add(f"v_cndmask_b32_e64 {al}, {v[0]}, {v[2]}, {c[1]}", [v[0], v[2], c[1]], [al])
        sg.add(f"v_cndmask_b32_e64 {ah}, {v[1]}, {v[3]}, {c[1]}", [v[1], v[3], c[1]], [ah])
    sched(B, sg)


# The blind-rotation step keeps the NTT-domain data in registers from the forward's lane-pair stage to the inverse's
# DIT stages: the MAC runs in the forward's W1' layout (the exchange with the partner wave is lane-linear in any
# layout) and the inverse starts from it (gen_tw_kernel.w1p_as_w1pp), so the step does no T2 and no T1'' transpose.
# The key the body reads is then the private copy in that order (row R, lane L of polynomial position 64 R + L holds
# NTT-domain coefficient tw_key_index(64 R + L); pbs_tw.hip prepare_tw_key builds it).
PBS_W1P = True
# the blind-rotation loop keeps one register map across its steps, which the renaming of the DPP-select regroup would
# break: its bodies keep the DPP-move regroup
T.REGROUP_DPP_SELECT = False


def tw_key_index(pos):
    """NTT-domain coefficient index (the reference's order) that the key copy of the W1' step holds at position pos."""
    R, L = pos >> 6, pos & 63
    return 64 * (L >> 1) + 32 * (L & 1) + 2 * (R & 15) + (R >> 4)


def fwd_mac_inv(B, tabs, dmap0, w1p, full_t=False, ext=False, inv_kw=None):
    """Forward transform (its stage 0 already run), the MAC with the partner wave and the inverse; returns the output
    dmap (W0, canonical).  w1p: the MAC and the inverse's input stay in the forward's W1' layout (PBS_W1P).  ext: the
    ext-map MAC (mac_ext)."""
    if w1p:
        fa, ia = (FWD_ADDR_P, INV_ADDR_P) if full_t else (FWD_ADDR, INV_ADDR)
        dmap = T.fwd_core(B, tabs, dmap0, fa, first_stage=1, stop="last")
        (mac_ext if ext else mac)(B, dmap)
        assert dmap == ([64 + 2 * q for q in range(32)] if full_t else
                        [8 + 2 * q for q in range(16)] + [64 + 2 * q for q in range(16)]), dmap
        return T.inv_core(B, tabs, dmap, ia, w1pp=True, w1pp_regs=dict(w1p_in=True, pre_base=40, ybase=96, newhi=64),
                          **(inv_kw or {}))
    dmap = T.fwd_core(B, tabs, dmap0, FWD_ADDR, first_stage=1)
    mac(B, dmap)
    return T.inv_core(B, tabs, dmap, INV_ADDR, w1pp=True, w1pp_regs=w1pp_regs(dmap))


def gen_pbs(tabs, sol=False):
    """BNF (sol=False): native ciphertexts, ms computed here from the raw mask, acc from the LUT rows.
    Solinas (sol=True, ntt64_pbs.rs:213-286): the mask arrives pre-switched (lwe = the switched values,
    0 skipped), acc starts from the wave's LDS buffer (the wrapper rotated the LUT by -ms(b) there)."""
    B = Body(tabs)
    prologue(B)
    B.raw(f"s_mov_b32 s{S_LWE}, %[lwe_lo]", f"s_mov_b32 s{S_LWE + 1}, %[lwe_hi]", f"s_mov_b32 s{S_CNT}, %[n]")
    if sol:
        B.raw(f"s_mov_b32 s{S_PHALF}, 0x80000001", f"s_mov_b32 s{S_PHALF + 1}, 0x7fffffff")
        B.raw(*[f"ds_read_b64 {pv(ACC + 2 * r)}, v{V_T4R} offset:{512 * r}" for r in range(32)],
              "s_waitcnt lgkmcnt(0)")
    else:
        B.raw(f"s_mov_b32 s{S_A}, %[lut_lo]", f"s_mov_b32 s{S_A + 1}, %[lut_hi]")
        B.raw(*load_rows(ACC, S_A), "s_waitcnt vmcnt(0)")    # acc <- LUT polynomial of this wave
    ms = ([f"s_and_b32 s{S_AMS}, s{S_A}, 0xfff"] if sol else     # pre-switched, in [0, 2N)
          [f"s_add_u32 s{S_AMS}, s{S_A + 1}, 0x80000",            # ms(a) = (a + 2^51) >> 52 (log_mod 12)
           f"s_lshr_b32 s{S_AMS}, s{S_AMS}, 20"])
    B.raw("Lpbs_top_%=:",
          f"s_cmp_eq_u32 s{S_CNT}, 0",
          "s_cbranch_scc1 Lpbs_end_%=",
          f"s_load_dwordx2 {sp(S_A)}, {sp(S_LWE)}, 0x0",
          f"s_add_u32 s{S_LWE}, s{S_LWE}, 8", f"s_addc_u32 s{S_LWE + 1}, s{S_LWE + 1}, 0",
          f"s_sub_u32 s{S_CNT}, s{S_CNT}, 1",
          "s_waitcnt lgkmcnt(0)",
          *ms,
          f"s_cmp_eq_u32 s{S_AMS}, 0",
          "s_cbranch_scc1 Lpbs_skip_%=")
    B.raw(*gload(0), *gload(1))
    rotate_decompose(B, sol)
    stage0_signed(B, tabs, [64 + 2 * r for r in range(32)])
    dmap = fwd_mac_inv(B, tabs, [64 + 2 * r for r in range(32)], PBS_W1P, full_t=PBS_W1P and PBS_FULL_T)
    if sol:
        add_acc_sol(B, dmap)
    else:
        modswitch_acc(B, dmap)
    B.raw("Lpbs_skip_%=:",
          f"s_add_u32 s{S_GOWN}, s{S_GOWN}, {STEP_BYTES}", f"s_addc_u32 s{S_GOWN + 1}, s{S_GOWN + 1}, 0",
          f"s_add_u32 s{S_GPAR}, s{S_GPAR}, {STEP_BYTES}", f"s_addc_u32 s{S_GPAR + 1}, s{S_GPAR + 1}, 0",
          "s_branch Lpbs_top_%=",
          "Lpbs_end_%=:")
    B.raw(*[f"ds_write_b64 v{V_T4R}, {pv(ACC + 2 * r)} offset:{512 * r}" for r in range(32)],
          "s_waitcnt lgkmcnt(0)")
    return B


# the external product / CMUX bodies: the same W1' step (with the one-pass transposes of PBS_FULL_T) on a GGSW permuted
# into the body's order per call (pbs_tw.hip launch_ext_tw: the caller's Raw / Normalize GGSW stays in the reference's
# order).  One-box A/Bs: without the one-pass transposes +0.5 % (profiles/r3/ext_w1p_ab/: the per-call reorder launch
# costs about what the two skipped transposes saved), with them 27.70 -> 28.02 M products/s, +1.2 %
# (profiles/r3/ext_w1p_full_t_ab/)
EXT_W1P = True


def gen_ext(tabs, cmux, sol=False):
    """One external product (cmux=False: out += GGSW . glwe) or CMUX (glwe -= out, then
    out += GGSW . glwe), level 1; wave w handles polynomial w of one GLWE pair.  BNF (native GLWEs, Raw
    GGSW) or Solinas (sol: GLWEs mod p, Normalize GGSW, ntt64_pbs.rs:553-702).  Built on the ext register map
    (set_regmap(True): below v168, 8.5 KiB of LDS per wave)."""
    set_regmap(True)
    try:
        return _gen_ext(tabs, cmux, sol)
    finally:
        set_regmap(False)


def _gen_ext(tabs, cmux, sol):
    B = Body(tabs)
    prologue(B)
    S_GL, S_OUT = S_LWE, S_A
    if sol:
        B.raw(f"s_mov_b32 s{S_PHALF}, 0x80000001", f"s_mov_b32 s{S_PHALF + 1}, 0x7fffffff")
    else:
        # the GGSW is the reference's Raw NTT key: N^-1 comes from the third table (untwist * N^-1)
        B.raw(f"s_add_u32 s{S_TWI}, %[tab_lo], {2 * 2080 * 8}", f"s_addc_u32 s{S_TWI + 1}, %[tab_hi], 0")
    B.raw(f"s_mov_b32 s{S_GL}, %[glwe_lo]", f"s_mov_b32 s{S_GL + 1}, %[glwe_hi]",
          f"s_mov_b32 s{S_OUT}, %[out_lo]", f"s_mov_b32 s{S_OUT + 1}, %[out_hi]")
    dmap0 = [64 + 2 * r for r in range(32)]
    sls7 = slots_at([8, 16, 24, 32, 40, 48, 56])
    sls3 = slots_at([40, 48, 56])   # beside the glwe rows (v64..) and a 16-row half of the out rows (v8..v39)
    dec = decompose_sol if sol else decompose
    if cmux:  # ct1 -= ct0 (ntt64_bnf_pbs.rs:683-705 wrapping; ntt64_pbs.rs:669-680 mod p), the out rows 16 at a time
        B.raw(*load_rows(64, S_GL))
        for h in range(2):
            rows = range(16 * h, 16 * h + 16)
            B.raw(*load_rows_sub(8, S_OUT, rows), "s_waitcnt vmcnt(0)")
            sg = Seg()
            for q, r in enumerate(rows):
                sl = sls3[q % len(sls3)]
                xl, xh = f"v{64 + 2 * r}", f"v{65 + 2 * r}"
                al, ah = f"v{8 + 2 * q}", f"v{9 + 2 * q}"
                if sol:
                    sg.add(f"v_sub_co_u32_e64 {xl}, {sl.c[0]}, {xl}, {al}", [xl, al], [xl, sl.c[0]])
                    sg.add(f"v_subb_co_u32_e64 {xh}, {sl.c[1]}, {xh}, {ah}, {sl.c[0]}", [xh, ah, sl.c[0]],
                           [xh, sl.c[1]])
                    minus_eps(sg, sl.v[5], sl.c[1], pv(64 + 2 * r))
                else:
                    sg.add(f"v_sub_co_u32_e64 {xl}, {sl.c[1]}, {xl}, {al}", [xl, al], [xl, sl.c[1]])
                    sg.add(f"v_subb_co_u32_e64 {xh}, {JUNK}, {xh}, {ah}, {sl.c[1]}", [xh, ah, sl.c[1]], [xh, JUNK])
            sched(B, sg)
        B.raw(*store_rows(64, S_GL))
        sg = Seg()
        for r in range(32):
            dec(sg, sls7[r % len(sls7)], f"v{64 + 2 * r}", f"v{65 + 2 * r}", signed=True)
        sched(B, sg)
        stage0_signed(B, tabs, dmap0)
    else:
        # the GLWE rows in butterfly-pair order (r, r + 16); the decomposition and the first forward stage run in 4
        # groups of 4 pairs as their rows arrive (loads return in issue order)
        rows = load_rows(64, S_GL)
        B.raw(*[rows[q] for k in range(16) for q in (k, k + 16)])
        for g in range(4):
            B.raw(f"s_waitcnt vmcnt({32 - 8 * (g + 1)})")
            sg = Seg()
            for k in range(4 * g, 4 * g + 4):
                for r in (k, k + 16):
                    dec(sg, sls7[r % len(sls7)], f"v{64 + 2 * r}", f"v{65 + 2 * r}", signed=True)
            sched(B, sg)
            stage0_signed(B, tabs, dmap0, rows=range(4 * g, 4 * g + 4))
    # out += y, 16 rows at a time: rows 0..15 (y in v96..) through v8..v39, loaded while the inverse's G1 stages run
    # (which keep to v40..v63 for their scratch), then rows 16..31 (y in v64..) through v96..v127
    dmap = fwd_mac_inv(B, tabs, dmap0, EXT_W1P, full_t=False, ext=True,
                       inv_kw=dict(g1_busy=range(8, 40), before_g1=load_rows_sub(8, S_OUT, range(16))))
    assert dmap == [96 + 2 * r for r in range(16)] + [64 + 2 * r for r in range(16)], dmap
    for h, base in ((0, 8), (1, 96)):
        rows = list(range(16 * h, 16 * h + 16))
        B.raw(*(load_rows_sub(base, S_OUT, rows) if h else []), "s_waitcnt vmcnt(0)")
        (add_acc_sol if sol else modswitch_acc)(B, dmap, rows, base, sls3)
        B.raw(*store_rows_sub(base, S_OUT, rows))  # no final wait: the wave retires while its stores drain
    return B


def emit(name, body, sgprs=SGPR_CLOBBER, vgprs=256):
    clob = ([f'"v{i}"' for i in range(8, vgprs)] + [f'"s{i}"' for i in sgprs] + ['"scc"', '"memory"'] +
            (['"vcc"'] if T.REGROUP_DPP_SELECT else []))
    return (f"// {name}: {body.nvalu} VALU, {len(body.lines)} lines\n"
            f"#define MI_PBS_BODY_{name.upper()}(...) asm volatile(\\\n" +
            "\\\n".join(f'      "{l}\\n"' for l in body.lines) +
            f"\\\n      :: __VA_ARGS__ \\\n      : {', '.join(clob)})\n")


def main():
    tabs = T.load_tables()
    b = gen_pbs(tabs)
    print("// GENERATED by tools/gen_pbs_kernel.py — do not edit.  Level-1 blind-rotation loops, external products")
    print("// and CMUXes (BNF and Solinas) as asm bodies per wave (pbs_tw.hip).  Own v8..v255, s20..s31 + s36..s93")
    print("// (+ s94..s95 in the Solinas bodies), exec (restored).")
    print("#pragma once")
    print(f"#define MI_PBS_W1P {int(PBS_W1P)}  // blind rotation reads its key in the W1' order (tw_key_index)")
    print(f"#define MI_EXT_W1P {int(EXT_W1P)}  // external product / CMUX read their GGSW in the W1' order")
    print(f"#define MI_PBS_LDS_STRIDE {PBS_LDS_STRIDE}  // u64 per wave LDS buffer of the blind-rotation bodies")
    print(f"#define MI_EXT_LDS_STRIDE {EXT_LDS_STRIDE}  // u64 per wave LDS buffer of the external-product bodies")
    print(f"#define MI_EXT_VGPRS {EXT_VGPRS}  // the external-product bodies use v0..v{EXT_VGPRS - 1} (3 waves per SIMD)")
    print(emit("bnf_l1", b))
    e, c = gen_ext(tabs, False), gen_ext(tabs, True)
    print(emit("ext_bnf_l1", e, vgprs=EXT_VGPRS))
    print(emit("cmux_bnf_l1", c, vgprs=EXT_VGPRS))
    bs = gen_pbs(tabs, sol=True)
    es, cs = gen_ext(tabs, False, sol=True), gen_ext(tabs, True, sol=True)
    print(emit("sol_l1", bs, SGPR_CLOBBER_SOL))
    print(emit("ext_sol_l1", es, SGPR_CLOBBER_SOL, EXT_VGPRS))
    print(emit("cmux_sol_l1", cs, SGPR_CLOBBER_SOL, EXT_VGPRS))
    print(f"// pbs step {b.nvalu} VALU, ext {e.nvalu}, cmux {c.nvalu}; Solinas pbs step {bs.nvalu}, ext {es.nvalu}, "
          f"cmux {cs.nvalu}", file=sys.stderr)


if __name__ == "__main__":
    main()
