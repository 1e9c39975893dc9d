"""Exhaustive bank-conflict check of the f64-FFT transpose-2 LDS layout (csrc/fft64_pbs.hip t2slot) under the
MI355X lane-group / bank rules of MI355X_MICROARCH.md §LDS: ds_read_b128 = 4 non-contiguous 16-lane groups,
banks (a/4) mod 64; ds_write_b128 = 8 contiguous 8-lane groups, banks (a/4) mod 32.  Prints every
(permutation of k2, row stride, XOR selector) candidate that is conflict-free for the forward write / read and
the inverse write / read; the kernel uses ('swap', 17, no XOR).  CPU only."""
import itertools
RD128 = [[*range(0,4),*range(12,16),*range(20,28)],[*range(4,12),*range(16,20),*range(28,32)],
         [*range(32,36),*range(44,48),*range(52,60)],[*range(36,44),*range(48,52),*range(60,64)]]
WR128 = [list(range(8*i, 8*i+8)) for i in range(8)]
def conflict_free(addr_fn, groups, mod):
    # addr_fn(lane) -> slot (16 B units); conflict-free iff slots distinct mod (banks/4)
    for grp in groups:
        s = [addr_fn(l) for l in grp]
        # identical addresses broadcast
        seen = {}
        for a in s:
            b = a % mod
            if b in seen and seen[b] != a: return False
            seen[b] = a
    return True
def ok(slot):
    # A: fwd write: lane L writes reg k2 at slot(L,k2)
    for k2 in range(16):
        if not conflict_free(lambda L: slot(L, k2), WR128, 8): return False
    # B: fwd read: lane=4k1+c reads (L=4k1+jj, k2=4c+g)
    for g in range(4):
        for jj in range(4):
            f = lambda l: slot(4*(l>>2)+jj, 4*(l&3)+g)
            if not conflict_free(f, RD128, 16): return False
            if not conflict_free(f, WR128, 8): return False   # C: inverse write, same addresses
    for k2 in range(16):
        if not conflict_free(lambda L: slot(L, k2), RD128, 16): return False  # D: inverse read
    return True
sigmas = {"id": lambda k: k, "swap": lambda k: ((k >> 2) | (k << 2)) & 15}
found = []
for sname, sig in sigmas.items():
    for S in (16, 17, 20, 24):
        for sel in itertools.product([None,0,1,2,3,4,5], repeat=4):
            def h(L, sel=sel):
                v = 0
                for i, a in enumerate(sel):
                    if a is not None: v |= ((L >> a) & 1) << i
                return v
            slot = lambda L, k2, S=S, h=h, sig=sig: S*L + (sig(k2) ^ h(L))
            if ok(slot):
                found.append((sname, S, sel))
print(len(found)); print(found[:10])
