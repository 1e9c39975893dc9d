"""Seeded TFHE key generation / encryption / decryption for the PBS tests (numpy, host only).

Restates the *semantics* of the reference's encryption (reference paths relative to
/root/reference/tfhe/src/core_crypto) so ciphertexts decrypt correctly through both the oracle
and the GPU PBS; the random streams are our own (numpy PCG64), so only functional results and
oracle-vs-engine parity on identical inputs are compared, never ciphertext bytes vs the reference.

  * binary LWE / GLWE secret keys        (algorithms/lwe_secret_key_generation.rs, glwe_...)
  * GLWE encryption  b = sum a_i * s_i + m + e  (negacyclic, mod 2^64)   (glwe_encryption.rs)
  * GGSW encryption factor -m << (64 - j*B); rows r<k: s_r * factor, last row: -factor at X^0
                                          (ggsw_encryption.rs:20-45, 318-375)
  * PBS LUT                               (lwe_programmable_bootstrapping/mod.rs:24-75)
"""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def uniform_u64(g, shape):
    return g.integers(0, 2**64, size=shape, dtype=np.uint64)


def tuniform(g, shape, bound_log2):
    """Small signed noise in [-2^b, 2^b] as wrapping u64 (TUniform-shaped support)."""
    v = g.integers(-(1 << bound_log2), (1 << bound_log2) + 1, size=shape, dtype=np.int64)
    return v.astype(np.uint64)


def binary_key(g, size):
    return g.integers(0, 2, size=size, dtype=np.uint64)


def add_q(a, b, q=0):
    """(a + b) mod q for canonical inputs; q = 0 means wrapping mod 2^64."""
    with np.errstate(over="ignore"):
        s = a + b
        if not q:
            return s
        carry = s < a
        return np.where(carry | (s >= np.uint64(q)), s - np.uint64(q), s)


def sub_q(a, b, q=0):
    with np.errstate(over="ignore"):
        d = a - b
        if not q:
            return d
        return np.where(a < b, d + np.uint64(q), d)


def neg_q(a, q=0):
    return sub_q(np.zeros_like(a), a, q)


def negacyclic_mul_binary(a, s, q=0):
    """(a * s) mod (X^N + 1), coefficients mod q (q = 0: mod 2^64), s a {0,1} polynomial."""
    n = a.shape[-1]
    out = np.zeros_like(a)
    for j in np.nonzero(s)[0]:
        j = int(j)
        if j == 0:
            out = add_q(out, a, q)
        else:
            out[..., j:] = add_q(out[..., j:], a[..., : n - j], q)
            out[..., :j] = sub_q(out[..., :j], a[..., n - j:], q)
    return out


def uniform_q(g, shape, q=0):
    return uniform_u64(g, shape) if not q else g.integers(0, q, size=shape, dtype=np.uint64)


def noise_q(g, shape, noise_log2, q=0):
    e = tuniform(g, shape, noise_log2)
    if not q:
        return e
    neg = (e.astype(np.int64) < 0)
    return np.where(neg, e + np.uint64(q), e)  # -x -> q - x


def glwe_encrypt(g, plaintext, glwe_sk, noise_log2, q=0):
    """plaintext (N,) -> GLWE (k+1, N) under glwe_sk (k, N): b = sum a_i s_i + m + e (mod q)."""
    k, n = glwe_sk.shape
    mask = uniform_q(g, (k, n), q)
    body = plaintext.copy()
    for i in range(k):
        body = add_q(body, negacyclic_mul_binary(mask[i], glwe_sk[i], q), q)
    body = add_q(body, noise_q(g, n, noise_log2, q), q)
    return np.concatenate([mask, body[None, :]], axis=0)


def glwe_decrypt(ct, glwe_sk, q=0):
    k = glwe_sk.shape[0]
    body = ct[k].copy()
    for i in range(k):
        body = sub_q(body, negacyclic_mul_binary(ct[i], glwe_sk[i], q), q)
    return body


def ggsw_encrypt(g, m, glwe_sk, base_log, level, noise_log2, q=0):
    """GGSW(m) -> (level, k+1, k+1, N), highest level first (ntt_ggsw_ciphertext.rs:176-192).
    factor = -m * 2^(64 - B*j) (mod q): ggsw_encryption.rs:20-45 (native and non-native summands)."""
    k, n = glwe_sk.shape
    mod = q if q else 2**64
    out = np.zeros((level, k + 1, k + 1, n), np.uint64)
    for li in range(level):
        j = level - li  # DecompositionLevel(level_count - i)
        factor = (-(int(m)) * (1 << (64 - base_log * j))) % mod
        for r in range(k + 1):
            if r < k:  # s_r * factor (slice_wrapping_scalar_mul_assign[_custom_mod])
                pt = np.array([(int(v) * factor) % mod for v in glwe_sk[r]], dtype=np.uint64)
            else:
                pt = np.zeros(n, np.uint64)
                pt[0] = np.uint64((-factor) % mod)
            out[li, r] = glwe_encrypt(g, pt, glwe_sk, noise_log2, q)
    return out


def bsk_gen(g, lwe_sk, glwe_sk, base_log, level, noise_log2, q=0):
    return np.stack([ggsw_encrypt(g, int(b), glwe_sk, base_log, level, noise_log2, q) for b in lwe_sk])


def lwe_encrypt(g, pt, lwe_sk, noise_log2, q=0):
    n = lwe_sk.size
    mod = q if q else 2**64
    a = uniform_q(g, n, q)
    e = int(tuniform(g, 1, noise_log2)[0].astype(np.int64))
    b = (sum(int(x) for x, s in zip(a, lwe_sk) if s) + int(pt) + e) % mod
    return np.concatenate([a, np.array([b], np.uint64)])


def lwe_decrypt(ct, lwe_sk, q=0):
    mod = q if q else 2**64
    return (int(ct[-1]) - sum(int(x) for x, s in zip(ct[:-1], lwe_sk) if s)) % mod


def glwe_sk_as_lwe_sk(glwe_sk):
    return glwe_sk.reshape(-1)


def pbs_lut(n, k, msg_mod, delta, f, q=0):
    """generate_programmable_bootstrap_glwe_lut (lwe_programmable_bootstrapping/mod.rs:24-75)."""
    box = n // msg_mod
    acc = np.zeros(n, np.uint64)
    for i in range(msg_mod):
        acc[i * box:(i + 1) * box] = np.uint64((f(i) * delta) % (q if q else 2**64))
    half = box // 2
    acc[:half] = neg_q(acc[:half], q)
    acc = np.roll(acc, -half)
    lut = np.zeros((k + 1, n), np.uint64)
    lut[k] = acc
    return lut


def decode(pt, delta, msg_mod, q=0):
    """divide_round(pt, delta) mod 2*msg_mod (padding bit kept); mod-q plaintexts are centred first."""
    v = int(pt)
    if q and v > q // 2:
        v -= q
    d = (v + delta // 2) // delta
    return d % (2 * msg_mod)


def lwe_encrypt_batch(g, pts, lwe_sk, noise_log2):
    """Native-modulus LWE encryptions of a vector of plaintexts: rows (a, <a, s> + m + e) mod 2^64."""
    pts = np.asarray(pts, dtype=np.uint64)
    a = uniform_u64(g, (pts.size, lwe_sk.size))
    with np.errstate(over="ignore"):
        b = (a * lwe_sk[None, :]).sum(axis=1, dtype=np.uint64) + pts + tuniform(g, pts.size, noise_log2)
    return np.concatenate([a, b[:, None]], axis=1)


def ksk_gen(g, in_sk, out_sk, base_log, level, noise_log2):
    """LWE keyswitch key (in_dim, level, out_dim + 1): block i, entry li encrypts
    s_in[i] << (64 - base_log * (level - li)) under out_sk (lwe_keyswitch_key_generation.rs:169-199)."""
    pts = np.array([(int(s) << (64 - base_log * (level - li))) % 2**64 for s in in_sk for li in range(level)],
                   dtype=np.uint64)
    return lwe_encrypt_batch(g, pts, out_sk, noise_log2).reshape(in_sk.size, level, out_sk.size + 1)


def lwe_decrypt_batch(cts, lwe_sk):
    with np.errstate(over="ignore"):
        return cts[..., -1] - (cts[..., :-1] * lwe_sk).sum(axis=-1, dtype=np.uint64)


def bsk_gen_native_l1(g, lwe_sk, glwe_sk, base_log, noise_log2):
    """bsk_gen for native 2^64 ciphertexts, k = 1, level 1, with every GGSW row's mask product computed in
    one vectorised pass (ggsw_encryption.rs:20-45 summands).  Test infrastructure only."""
    n_lwe, n = lwe_sk.size, glwe_sk.shape[1]
    masks = uniform_u64(g, (n_lwe * 2, n))
    prod = negacyclic_mul_binary(masks, glwe_sk[0]).reshape(n_lwe, 2, n)
    factor = ((-(lwe_sk.astype(object)) * (1 << (64 - base_log))) % 2**64).astype(np.uint64)  # -b * 2^(64-B)
    pt = np.zeros((n_lwe, 2, n), np.uint64)
    with np.errstate(over="ignore"):
        pt[:, 0] = factor[:, None] * glwe_sk[0][None, :]
        pt[:, 1, 0] = np.uint64(0) - factor
        body = prod + pt + noise_q(g, (n_lwe, 2, n), noise_log2)
    bsk = np.zeros((n_lwe, 1, 2, 2, n), np.uint64)
    bsk[:, 0, :, 0] = masks.reshape(n_lwe, 2, n)
    bsk[:, 0, :, 1] = body
    return bsk


def polymul_binary_fast(oracle, a, s, q=0, threads=16):
    """(a * s) mod (X^N + 1) for every polynomial of `a` (..., N) and one binary polynomial s (N,), coefficients
    mod q (q = 0: mod 2^64), through the oracle's Solinas-prime transform (test infrastructure: the large-N key
    generation of the shape tests).  q = p: one exact product mod p.  Native: a = a_0 + a_1 2^32 with 32-bit limbs;
    each limb product's coefficients are in (-N 2^32, N 2^32), inside (-p/2, p/2) for N <= 2^30, so the prime
    product lifted to a signed integer is exact; the limbs recombine mod 2^64."""
    P = 0xFFFFFFFF00000001
    n = a.shape[-1]
    plan = oracle.Plan.try_new(n, P)
    flat = np.ascontiguousarray(a.reshape(-1, n), dtype=np.uint64)
    s_hat = np.broadcast_to(plan.fwd(np.asarray(s, dtype=np.uint64)), flat.shape).copy()

    def prime_product(x):
        return plan.inv(plan.mul_assign_normalize(plan.fwd(x, threads=threads), s_hat), threads=threads)

    if q:
        assert q == P
        return prime_product(flat).reshape(a.shape)
    out = np.zeros_like(flat)
    with np.errstate(over="ignore"):
        for t in range(2):
            v = prime_product((flat >> np.uint64(32 * t)) & np.uint64(0xFFFFFFFF))
            v = np.where(v > np.uint64(P // 2), v - np.uint64(P), v)  # signed lift, as u64 mod 2^64
            out += v << np.uint64(32 * t)
    return out.reshape(a.shape)


def bsk_gen_fast(g, oracle, lwe_sk, glwe_sk, base_log, level, noise_log2, q=0):
    """Standard-domain bootstrap key (n_lwe, level, k+1, k+1, N) with the semantics of ggsw_encrypt / bsk_gen
    (ggsw_encryption.rs:20-45, 318-375; highest level first), every mask product computed in one batched pass
    (polymul_binary_fast) so N = 8192 / 65536 keys generate in seconds.  Test infrastructure only."""
    n_lwe = lwe_sk.size
    k, n = glwe_sk.shape
    mod = q if q else 2**64
    masks = uniform_q(g, (n_lwe, level, k + 1, k, n), q)
    body = noise_q(g, (n_lwe, level, k + 1, n), noise_log2, q)
    for i in range(k):
        body = add_q(body, polymul_binary_fast(oracle, np.ascontiguousarray(masks[..., i, :]), glwe_sk[i], q), q)
    # plaintexts: factor = -b 2^(64 - B j) (mod q); row r < k: s_r * factor (s_r binary: factor where s_r = 1),
    # row k: -factor at X^0
    for li in range(level):
        j = level - li
        f1 = (-(1 << (64 - base_log * j))) % mod                       # the factor of a key bit b = 1
        fac = np.where(lwe_sk.astype(bool), np.uint64(f1), np.uint64(0))  # (n_lwe,)
        for r in range(k):
            pt = np.where(glwe_sk[r].astype(bool)[None, :], fac[:, None], np.uint64(0))
            body[:, li, r] = add_q(body[:, li, r], pt, q)
        nf = np.where(lwe_sk.astype(bool), np.uint64((-f1) % mod), np.uint64(0))
        body[:, li, k, 0] = add_q(body[:, li, k, 0], nf, q)
    bsk = np.zeros((n_lwe, level, k + 1, k + 1, n), np.uint64)
    bsk[..., :k, :] = masks
    bsk[..., k, :] = body
    return bsk


def ksk32_gen(g, in_sk, out_sk, base_log, level, noise_log2, out_mod_log=32):
    """LweKeyswitchKey<Vec<u32>> of output modulus 2^out_mod_log (values in the MSBs, as the reference encodes a
    non-native power of two): block i, entry li encrypts s_in[i] << (32 - base_log * (level - li)) under out_sk
    (lwe_keyswitch_key_generation.rs:169-199 at OutputScalar = u32).  Test infrastructure only."""
    in_dim, out_dim = in_sk.size, out_sk.size
    scale = np.uint32(1 << (32 - out_mod_log)) if out_mod_log < 32 else np.uint32(1)
    pts = np.array([(int(s) << (32 - base_log * (level - li))) % 2**32 for s in in_sk for li in range(level)],
                   dtype=np.uint32)
    mask = g.integers(0, 1 << out_mod_log, size=(pts.size, out_dim), dtype=np.uint64).astype(np.uint32) * scale
    noise = (g.integers(-(1 << noise_log2), 1 << noise_log2, size=pts.size, dtype=np.int64)
             .astype(np.uint32) * scale)
    with np.errstate(over="ignore"):
        body = (mask.astype(np.uint64) * out_sk.astype(np.uint64)).sum(axis=1).astype(np.uint32) + pts + noise
    return np.concatenate([mask, body[:, None]], axis=1).reshape(in_dim, level, out_dim + 1)


def lwe32_decrypt_batch(cts, lwe_sk):
    with np.errstate(over="ignore"):
        return (cts[..., -1].astype(np.uint64) - (cts[..., :-1].astype(np.uint64) * lwe_sk).sum(axis=-1)) \
            .astype(np.uint32)
