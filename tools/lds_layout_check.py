"""Bank-conflict check of the f64-FFT transpose LDS layout (csrc/fft64_pbs.hip: element (lane L, register r) at
slot ROW * L + r, 16-byte slots) under the MI355X lane-group / bank rules of MI355X_MICROARCH.md §LDS:
ds_read_b128 = 4 non-contiguous 16-lane groups, banks (a/4) mod 64; ds_write_b128 = 8 contiguous 8-lane
groups, banks (a/4) mod 32.  The transpose swaps lane bits 0..3 with the register bits inside each 16-lane
row: forward write (lane L, register r) -> forward read (lane L reads register j from lane 16 (L >> 4) + j,
slot of register L & 15); the inverse uses the same two address patterns the other way round.  Prints each
candidate row stride with its conflict count; the kernel uses ROW = 17.  CPU only."""
RD128 = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)],
         [*range(32, 36), *range(44, 48), *range(52, 60)], [*range(36, 44), *range(48, 52), *range(60, 64)]]
WR128 = [list(range(8 * i, 8 * i + 8)) for i in range(8)]


def conflicts(addr_fn, groups, mod):
    """number of lane groups whose slots collide mod (banks / 4) at different addresses (same address broadcasts)"""
    bad = 0
    for grp in groups:
        seen = {}
        for a in (addr_fn(l) for l in grp):
            if seen.setdefault(a % mod, a) != a:
                bad += 1
                break
    return bad


def count(row):
    slot = lambda L, r: row * L + r
    bad = 0
    for r in range(16):  # forward write / inverse read
        f = lambda L, r=r: slot(L, r)
        bad += conflicts(f, WR128, 8) + conflicts(f, RD128, 16)
    for j in range(16):  # forward read / inverse write
        f = lambda L, j=j: slot(16 * (L >> 4) + j, L & 15)
        bad += conflicts(f, RD128, 16) + conflicts(f, WR128, 8)
    return bad


if __name__ == "__main__":
    for row in (16, 17, 18, 20):
        print(f"ROW {row}: {count(row)} conflicting lane groups")
