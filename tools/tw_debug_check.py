#!/usr/bin/env python3
"""Host side of tools/tw_debug.hip: writes the input (4 polys + twist table) and, given the dump,
compares every phase's registers with a Python model of the twisted transform."""
import os, random, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import oracle as O

P = 0xFFFFFFFF00000001
N = 2048
plan = O.Plan.try_new(N, P)
tw = [int(v) for v in plan.twid]
def br(x, b): return int(format(x, f"0{b}b")[::-1], 2) if b else 0
psi = tw[br(1, 11)]
omega = pow(psi, 64, P)
def twc(mp, g): return pow(omega, (64 // (2 * mp)) * br(g, mp.bit_length() - 1), P)
tables = []
for i in range(32):
    rho = pow(psi, 2 * br(i, 5) + 1, P)
    tables += [pow(rho, j, P) for j in range(64)]
CYC5 = [twc(32, g) for g in range(32)]

def model(x):
    a = list(x); t = N; m = 1; st = {}
    while m < 32:
        t //= 2
        for i in range(m):
            w = tw[m + i]
            for j in range(2 * i * t, 2 * i * t + t):
                u, v = a[j], a[j + t] * w % P
                a[j], a[j + t] = (u + v) % P, (u - v) % P
        m *= 2
    st["g1"] = list(a)
    a = [a[e] * tables[e] % P for e in range(N)]
    st["twist"] = list(a)
    for i in range(32):
        blk = a[64 * i: 64 * i + 64]
        tt = 64; mp = 1
        while mp < 64:
            tt //= 2
            for g in range(mp):
                w = twc(mp, g)
                for j in range(2 * g * tt, 2 * g * tt + tt):
                    u, v = blk[j], blk[j + tt] * w % P
                    blk[j], blk[j + tt] = (u + v) % P, (u - v) % P
            if mp == 16:
                st.setdefault("cyc", [0] * N)
                st["cyc"][64 * i: 64 * i + 64] = list(blk)
            mp *= 2
        a[64 * i: 64 * i + 64] = blk
    st["last"] = list(a)
    return st

def unpack(dump, layout):
    """dump[64 r + lane] -> element index -> value"""
    out = {}
    for r in range(32):
        for lane in range(64):
            v = int(dump[64 * r + lane])
            if layout == "W0":
                e = 64 * r + lane
            elif layout == "W1":
                i, j0 = lane >> 1, lane & 1
                e = 64 * i + 2 * r + j0
            else:  # W1'
                i, p = lane >> 1, lane & 1
                j = (2 * r + 32 * p) if r < 16 else (2 * (r - 16) + 1 + 32 * p)
                e = 64 * i + j
            out[e] = v
    return out

if sys.argv[1] == "gen":
    random.seed(5)
    x = [random.randrange(P) for _ in range(4 * N)]
    arr = np.array(x + tables + CYC5, dtype=np.uint64)
    arr.tofile(sys.argv[2])
else:
    x = [int(v) for v in np.fromfile(sys.argv[2], dtype=np.uint64)[:4 * N]]
    dump = np.fromfile(sys.argv[3], dtype=np.uint64).reshape(5, 4, N)
    for wv in range(1):
        st = model(x[wv * N:(wv + 1) * N])
        for s, (name, lay) in enumerate([("g1", "W0"), ("twist", "W0"), ("twist", "W1"), ("cyc", "W1"), ("last", "W1'")]):
            got = unpack(dump[s][wv], lay)
            bad = [e for e in range(N) if got[e] % P != st[name][e]]
            print(f"stage {s} ({name}, {lay}): {len(bad)} mismatches", bad[:12])
