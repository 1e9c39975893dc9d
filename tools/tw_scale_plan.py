#!/usr/bin/env python3
"""Scale plan of the twisted N = 2048 transform's in-register butterfly networks (r5).

Every element of a lane may carry a power-of-two scale through the shift-twiddle stages: register r holds
2^s_r * (true value), s_r mod 192 (2^96 = -1 mod p, 2^192 = 1).  A CT butterfly (a, b; twiddle 2^w) on inputs of
scales (ea, eb) multiplies ONE input by a power of two and adds / subtracts:
  mode 0: t = 2^(w + ea - eb) * b, outputs a + t, a - t, both of scale ea;
  mode 1: t = 2^(eb - w - ea) * a, outputs t + b (position a) and b - t (position b, i.e. -(a - w b)), scale eb - w
          (the sign is a +96 on the exponent).
The multiplier's exponent class decides the cost (tools/gen_tw_kernel.py tmul: 0 mod 96 = a copy or a canonicalisation,
32 < e < 64 = the expensive class-1 sequence, else ~6 VALU).  The twist (forward) and the untwist (inverse) are general
multiplies by a per-element table value, so any scale the network leaves at its free end is absorbed by the plan's
twist table at no cost:
  forward G1  (5 stages, inputs = loaded data, scale 0; outputs free -> the twist table divides them out),
  forward CYC (the 5 in-register stages of the cyclic blocks; inputs free -> the twist table multiplies them in;
               outputs scale 0 for the unchanged lane-pair stage),
  inverse G1  (5 GS stages after the untwist; inputs free -> the untwist table; outputs scale 0, canonical).
The search is a seeded simulated annealing over the per-butterfly modes and the free-end scales, pricing each
butterfly with the measured issue costs of tools/valu_cost.py; the result is committed as tools/tw_scale_plan.json,
which tools/gen_tw_kernel.py (the bodies) and tools/gen_tw_tables.py (the C++ scale tables) both read.

  python tools/tw_scale_plan.py            -> rewrites tools/tw_scale_plan.json and prints the modelled savings
"""
import json
import math
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PLAN_PATH = os.path.join(HERE, "tw_scale_plan.json")
SALU = 1.5  # measured issue cost of an SALU instruction among the bodies' VALU stream (profiles/r5/session3)


def align_cost(m, t_canon):
    """Issue cycles of t = 2^m x, canonical (gen_tw_kernel.tmul / the ALIAS_COPY path for +-1)."""
    e = m % 96
    if e == 0:
        return 4.72 if t_canon else 13.2
    if e <= 32:
        return (22.0 if e == 32 else 24.3) + SALU
    if e < 64:
        return 42.45 + SALU
    return 22.2 if e == 64 else 24.56


CT_BASE = 35.7          # add + fold, sub + borrow fix (gen_tw_kernel.ct_core)
GS_BASE = 41.8 + SALU   # add, sub + borrow fix, canonicalising select of the sum (both inputs canonical)


def tables():
    sys.path.insert(0, HERE)
    import gen_tw_kernel as T
    return T.load_tables(), T


def ct_network(kind):
    tabs, T = tables()
    st = []
    if kind == "fwd_g1":
        for s in range(5):
            d = 16 >> s
            st.append([(r, r + d, tabs["G1_FWD"][s][r // (2 * d)]) for r in range(32) if not r & d])
    elif kind == "fwd_cyc":
        for q in range(5):
            d = 16 >> q
            st.append([(r, r + d, tabs["CYC_FWD"][q][r // (2 * d)]) for r in range(32) if not r & d])
    elif kind == "inv_dit":  # the W1'' inverse's in-register DIT stages (gen_tw_kernel.dit_exps_pp, by register)
        for q in range(5):
            d = 1 << q
            e = T.dit_exps_pp(q)
            st.append([(r, r + d, e[r]) for r in range(32) if not r & d])
    elif kind == "inv_g1":
        for s in range(4, -1, -1):
            d = 16 >> s
            st.append([(r, r + d, tabs["G1_INV"][s][r // (2 * d)]) for r in range(32) if not r & d])
    return st


def eval_ct(net, inp, modes, canon_in):
    """(cost, output scales) of a CT network; modes[k] in {0, 1} for butterfly k in stage order."""
    e, canon, cost, k = list(inp), list(canon_in), 0.0, 0
    for st in net:
        ne, nc = list(e), list(canon)
        for ra, rb, w in st:
            ea, eb = e[ra], e[rb]
            if modes[k] == 0:
                m, s, tc, sb = w + ea - eb, ea, canon[rb], 0
            else:  # the difference comes out negated (b - t): +96
                m, s, tc, sb = eb - w - ea, eb - w, canon[ra], 96
            cost += align_cost(m, tc) + CT_BASE
            ne[ra] = s % 192
            ne[rb] = (s + sb) % 192
            nc[ra] = nc[rb] = False
            k += 1
        e, canon = ne, nc
    return cost, e


def eval_gs(net, inp, modes, xs):
    """(cost, output scales) of the GS network of the inverse (a' = a + b, b' = 2^w (a - b)); every value canonical.
    modes[k]: 0 aligns b to a (t = 2^(ea - eb) b), 1 aligns a to b; xs[k]: the exponent the difference is multiplied
    by (0: none, its scale then carries the deferred twiddle)."""
    e, cost, k = list(inp), 0.0, 0
    for st in net:
        ne = list(e)
        for ra, rb, w in st:
            ea, eb = e[ra], e[rb]
            if modes[k] == 0:
                m, s = ea - eb, ea
            else:
                m, s = eb - ea, eb
            cost += (0.0 if m % 96 == 0 else align_cost(m, True)) + GS_BASE
            x = xs[k]
            if x % 192:
                cost += align_cost(x, True)
            ne[ra] = s % 192
            ne[rb] = (s - w + x) % 192
            k += 1
        e = ne
    return cost, e


def anneal(cost_fn, n_modes, free_in, iters, seed, fixed_modes=(), gs=False):
    rnd = random.Random(seed)
    inp, modes, xs = [0] * 32, [0] * n_modes, [0] * n_modes
    if gs:  # start from the current design: twiddle on the difference, scales 0
        xs = list(GS_START)

    cur = cost_fn(inp, modes, xs)
    best = (cur, list(inp), list(modes), list(xs))
    for it in range(iters):
        temp = max(0.3, 40.0 * (1 - it / iters))
        ni, nm, nx = list(inp), list(modes), list(xs)
        r = rnd.random()
        if free_in and r < 0.35:
            ni[rnd.randrange(32)] = 3 * rnd.randrange(64)
        elif gs and r < 0.7:
            nx[rnd.randrange(n_modes)] = 3 * rnd.randrange(64)
        else:
            j = rnd.randrange(n_modes)
            if j in fixed_modes:
                continue
            nm[j] ^= 1
        c = cost_fn(ni, nm, nx)
        if c <= cur or rnd.random() < math.exp((cur - c) / temp):
            inp, modes, xs, cur = ni, nm, nx, c
            if c < best[0]:
                best = (c, list(ni), list(nm), list(nx))
    return best


GS_START = []


def solve(iters=120000, seeds=4):
    global GS_START
    plan = {}
    big = 1.0e4
    # forward G1: inputs 0 (loaded, canonical), outputs free; stage 0 stays mode 0 (the PBS bodies' signed-digit stage 0)
    net = ct_network("fwd_g1")
    fn = lambda inp, m, x: eval_ct(net, [0] * 32, m, [True] * 32)[0]
    base = fn(None, [0] * 80, None)
    best = min(anneal(fn, 80, False, iters, s, fixed_modes=set(range(16))) for s in range(seeds))
    out = eval_ct(net, [0] * 32, best[2], [True] * 32)[1]
    plan["fwd_g1"] = {"modes": best[2], "out_scales": out, "cost": best[0], "base": base}
    # forward CYC: inputs free (twist), outputs 0 (the lane-pair stage); inputs canonical (twist outputs)
    net_c = ct_network("fwd_cyc")

    def fn_c(inp, m, x):
        c, e = eval_ct(net_c, inp, m, [True] * 32)
        return c + big * sum(1 for v in e if v % 192)

    base_c = fn_c([0] * 32, [0] * 80, None)
    best_c = min(anneal(fn_c, 80, True, iters, 10 + s) for s in range(seeds))
    assert best_c[0] < big, "forward CYC plan leaves a scaled output"
    plan["fwd_cyc"] = {"modes": best_c[2], "in_scales": best_c[1], "cost": best_c[0], "base": base_c}
    # inverse DIT (the W1'' cyclic blocks, r5): inputs 0 (loaded, canonical), outputs free -> the untwist table; the
    # lane-pair DIT stage between passes each register's scale through (its two inputs come from one register)
    net_d = ct_network("inv_dit")
    fn_d = lambda inp, m, x: eval_ct(net_d, [0] * 32, m, [True] * 32)[0]
    base_d = fn_d(None, [0] * 80, None)
    best_d = min(anneal(fn_d, 80, False, iters, 30 + s) for s in range(seeds))
    out_d = eval_ct(net_d, [0] * 32, best_d[2], [True] * 32)[1]
    plan["inv_dit"] = {"modes": best_d[2], "out_scales": out_d, "cost": best_d[0], "base": base_d}
    # inverse G1 (GS): inputs free (untwist), outputs 0
    net_g = ct_network("inv_g1")
    GS_START = [w for st in net_g for (_, _, w) in st]

    def fn_g(inp, m, x):
        c, e = eval_gs(net_g, inp, m, x)
        return c + big * sum(1 for v in e if v % 192)

    base_g = fn_g([0] * 32, [0] * 80, GS_START)
    best_g = min(anneal(fn_g, 80, True, iters, 20 + s, gs=True) for s in range(seeds))
    assert best_g[0] < big, "inverse G1 plan leaves a scaled output"
    plan["inv_g1"] = {"modes": best_g[2], "diff_exps": best_g[3], "in_scales": best_g[1], "cost": best_g[0],
                      "base": base_g}
    return plan


def load():
    with open(PLAN_PATH) as f:
        return json.load(f)


def main():
    plan = solve()
    for k, v in plan.items():
        print(f"{k}: modelled {v['base']:.0f} -> {v['cost']:.0f} cycles per wave", file=sys.stderr)
    with open(PLAN_PATH, "w") as f:
        json.dump(plan, f, indent=None, separators=(",", ":"))
        f.write("\n")


if __name__ == "__main__":
    main()
