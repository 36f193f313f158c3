"""CPU restatement of the engine's random-linear-combination scalar derivation -- TEST
INFRASTRUCTURE ONLY (imported by tests/, never by the product path).

Reference semantics: lighthouse's `verify_signature_sets` (the batch verify SURVEY.md §8a-7 adopts)
draws one fresh non-zero 64-bit scalar per set from `rand::thread_rng()` -- ChaCha12 keyed from the
OS (rand 0.8) -- with `RAND_BITS = 64` (copied into the reference at src/crypto/impls/blst.rs:12).
The engine (safestakeoperator_amd/csrc/ssb_units.h) keeps that shape: a 256-bit key per batch call
from getrandom(), and share i's scalar = the first 64 bits of the ChaCha12 block (key, counter i,
nonce "SSB-RLC1"), forced odd.  In the deterministic test mode the key is splitmix64 of the
caller's seed.  This module restates both so tests can (a) pin the device function against the
RFC 8439 ChaCha block function and (b) compute the scalars a deterministic batch uses, which is
what an attacker would need to build shares that cancel in the combination.
"""
M32 = 0xFFFFFFFF
M64 = 0xFFFFFFFFFFFFFFFF
SIGMA = (0x61707865, 0x3320646E, 0x79622D32, 0x6B206574)   # "expand 32-byte k"
NONCE = (0x2D425353, 0x31434C52)                            # "SSB-", "RLC1" (little-endian words)


def _rotl(x, r):
    return ((x << r) | (x >> (32 - r))) & M32


def _qr(x, a, b, c, d):
    x[a] = (x[a] + x[b]) & M32; x[d] = _rotl(x[d] ^ x[a], 16)
    x[c] = (x[c] + x[d]) & M32; x[b] = _rotl(x[b] ^ x[c], 12)
    x[a] = (x[a] + x[b]) & M32; x[d] = _rotl(x[d] ^ x[a], 8)
    x[c] = (x[c] + x[d]) & M32; x[b] = _rotl(x[b] ^ x[c], 7)


def chacha_block(state16, rounds):
    """The ChaCha block function (RFC 8439 §2.3) on a 16-word state: `rounds` rounds (20 in the
    RFC, 12 here), then the feed-forward addition."""
    x = list(state16)
    for _ in range(rounds // 2):
        _qr(x, 0, 4, 8, 12); _qr(x, 1, 5, 9, 13); _qr(x, 2, 6, 10, 14); _qr(x, 3, 7, 11, 15)
        _qr(x, 0, 5, 10, 15); _qr(x, 1, 6, 11, 12); _qr(x, 2, 7, 8, 13); _qr(x, 3, 4, 9, 14)
    return [(a + b) & M32 for a, b in zip(x, state16)]


def chacha12_u64(key8, i):
    """ssb_units.h chacha12_u64: words 0, 1 of ChaCha12(key, 64-bit counter i, nonce "SSB-RLC1")."""
    st = list(SIGMA) + list(key8) + [i & M32, (i >> 32) & M32] + list(NONCE)
    out = chacha_block(st, 12)
    return out[0] | (out[1] << 32)


def rlc_scalar_odd(key8, i):
    return chacha12_u64(key8, i) | 1


def splitmix64_at(seed, j):
    z = (seed + 0x9E3779B97F4A7C15 * (j + 1)) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def key_from_seed(seed):
    """ssb_units.h rlc_key_from_seed: the deterministic-mode key."""
    k = []
    for j in range(4):
        z = splitmix64_at(seed & M64, j)
        k += [z & M32, z >> 32]
    return k


def deterministic_scalars(seed, n):
    key = key_from_seed(seed)
    return [rlc_scalar_odd(key, i) for i in range(n)]


def round1_scalars(seed, n):
    """The round-1 engine's public scalars, splitmix64(seed ^ golden*(i+1)) | 1 (what a crafted
    pair against the old default seed 0x5AFE57A4E was built from)."""
    out = []
    for i in range(n):
        z = (seed ^ ((0x9E3779B97F4A7C15 * (i + 1)) & M64)) & M64
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        z ^= z >> 31
        out.append((z or 1) | 1)
    return out
