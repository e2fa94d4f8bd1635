"""Client-side helpers (key generation, LWE encryption/decryption) through the C ABI.

They follow the reference's rules (binary keys, Marsaglia-polar Gaussian noise, GGSW rows of
ggsw_encryption.rs:116-150, KSK levels L..1 of lwe_keyswitch_key_generation.rs:109) with a seeded
xoshiro256** stream instead of the reference's AES-CTR CSPRNG.
"""
from __future__ import annotations

import os

import numpy as np

from . import _lib
from ._lib import u64p


def _ptr(a):
    return a.ctypes.data_as(u64p)


def gen_binary_key(seed: int, stream: int, length: int) -> np.ndarray:
    k = np.zeros(length, dtype=np.uint64)
    _lib.call("tfhe_mi355_client_gen_binary_key", seed, stream, _ptr(k), length)
    return k


def gen_bootstrap_key(seed, lwe_sk, glwe_sk, glwe_dimension, polynomial_size, base_log, level, std_dev,
                      threads: int = 0) -> np.ndarray:
    lwe_sk = np.ascontiguousarray(lwe_sk, dtype=np.uint64)
    glwe_sk = np.ascontiguousarray(glwe_sk, dtype=np.uint64)
    k, N = glwe_dimension, polynomial_size
    bsk = np.empty(len(lwe_sk) * level * (k + 1) * (k + 1) * N, dtype=np.uint64)
    if threads <= 0:
        threads = min(16, os.cpu_count() or 1)
    _lib.call("tfhe_mi355_client_gen_bootstrap_key", seed, _ptr(lwe_sk), len(lwe_sk), _ptr(glwe_sk), k, N,
              base_log, level, std_dev, _ptr(bsk), threads)
    return bsk


def gen_multi_bit_bootstrap_key(seed, lwe_sk, glwe_sk, glwe_dimension, polynomial_size, base_log, level,
                                grouping_factor, std_dev, threads: int = 0) -> np.ndarray:
    """[n/g][2^g][L][k+1][k+1][N] (lwe_multi_bit_bootstrap_key_generation.rs:87-173)."""
    lwe_sk = np.ascontiguousarray(lwe_sk, dtype=np.uint64)
    glwe_sk = np.ascontiguousarray(glwe_sk, dtype=np.uint64)
    k, N, g = glwe_dimension, polynomial_size, grouping_factor
    bsk = np.empty((len(lwe_sk) // g) * (1 << g) * level * (k + 1) * (k + 1) * N, dtype=np.uint64)
    if threads <= 0:
        threads = min(16, os.cpu_count() or 1)
    _lib.call("tfhe_mi355_client_gen_multi_bit_bootstrap_key", seed, _ptr(lwe_sk), len(lwe_sk), _ptr(glwe_sk),
              k, N, base_log, level, g, std_dev, _ptr(bsk), threads)
    return bsk


def gen_keyswitch_key(seed, in_sk, out_sk, base_log, level, std_dev) -> np.ndarray:
    in_sk = np.ascontiguousarray(in_sk, dtype=np.uint64)
    out_sk = np.ascontiguousarray(out_sk, dtype=np.uint64)
    ksk = np.empty(len(in_sk) * level * (len(out_sk) + 1), dtype=np.uint64)
    _lib.call("tfhe_mi355_client_gen_keyswitch_key", seed, _ptr(in_sk), len(in_sk), _ptr(out_sk), len(out_sk),
              base_log, level, std_dev, _ptr(ksk))
    return ksk


def gen_packing_keyswitch_key(seed, in_sk, glwe_sk, glwe_dimension, polynomial_size, base_log, level, std_dev,
                              threads: int = 0) -> np.ndarray:
    """LWE -> GLWE packing KSK [in][level][(k+1)N] (lwe_packing_keyswitch_key_generation.rs:74-149)."""
    in_sk = np.ascontiguousarray(in_sk, dtype=np.uint64)
    glwe_sk = np.ascontiguousarray(glwe_sk, dtype=np.uint64)
    k, N = glwe_dimension, polynomial_size
    out = np.empty(len(in_sk) * level * (k + 1) * N, dtype=np.uint64)
    _lib.call("tfhe_mi355_client_gen_packing_keyswitch_key", seed, _ptr(in_sk), len(in_sk), _ptr(glwe_sk), k, N,
              base_log, level, std_dev, _ptr(out), threads)
    return out


def _seed_parts(seed: int):
    return seed & 0xFFFFFFFFFFFFFFFF, (seed >> 64) & 0xFFFFFFFFFFFFFFFF


def csprng_mask_words(compression_seed: int, first_word: int, count: int) -> np.ndarray:
    """Mask words of a seeded key: word w = LE u64 of AES-CTR stream bytes [1 + 8w, 9 + 8w)."""
    out = np.empty(count, dtype=np.uint64)
    lo, hi = _seed_parts(compression_seed)
    _lib.call("tfhe_mi355_client_csprng_mask_words", lo, hi, first_word, count, _ptr(out))
    return out


def gen_seeded_bootstrap_key(noise_seed, compression_seed: int, lwe_sk, glwe_sk, glwe_dimension, polynomial_size,
                             base_log, level, std_dev, threads: int = 0) -> np.ndarray:
    """SeededLweBootstrapKey bodies [n][L][k+1][N]; masks = the AES-CTR stream of compression_seed."""
    lwe_sk = np.ascontiguousarray(lwe_sk, dtype=np.uint64)
    glwe_sk = np.ascontiguousarray(glwe_sk, dtype=np.uint64)
    k, N = glwe_dimension, polynomial_size
    out = np.empty(len(lwe_sk) * level * (k + 1) * N, dtype=np.uint64)
    lo, hi = _seed_parts(compression_seed)
    _lib.call("tfhe_mi355_client_gen_seeded_bootstrap_key", noise_seed, lo, hi, _ptr(lwe_sk), len(lwe_sk),
              _ptr(glwe_sk), k, N, base_log, level, std_dev, _ptr(out), threads)
    return out


def gen_seeded_keyswitch_key(noise_seed, compression_seed: int, in_sk, out_sk, base_log, level,
                             std_dev) -> np.ndarray:
    """SeededLweKeyswitchKey bodies [in_dim][L]."""
    in_sk = np.ascontiguousarray(in_sk, dtype=np.uint64)
    out_sk = np.ascontiguousarray(out_sk, dtype=np.uint64)
    out = np.empty(len(in_sk) * level, dtype=np.uint64)
    lo, hi = _seed_parts(compression_seed)
    _lib.call("tfhe_mi355_client_gen_seeded_keyswitch_key", noise_seed, lo, hi, _ptr(in_sk), len(in_sk),
              _ptr(out_sk), len(out_sk), base_log, level, std_dev, _ptr(out))
    return out


def lwe_encrypt(seed, sk, plaintexts, std_dev) -> np.ndarray:
    sk = np.ascontiguousarray(sk, dtype=np.uint64)
    pts = np.ascontiguousarray(plaintexts, dtype=np.uint64).ravel()
    cts = np.empty((len(pts), len(sk) + 1), dtype=np.uint64)
    _lib.call("tfhe_mi355_client_lwe_encrypt", seed, _ptr(sk), len(sk), _ptr(pts), len(pts), std_dev, _ptr(cts))
    return cts


def lwe_decrypt(sk, cts) -> np.ndarray:
    sk = np.ascontiguousarray(sk, dtype=np.uint64)
    cts = np.ascontiguousarray(cts, dtype=np.uint64).reshape(-1, len(sk) + 1)
    pts = np.empty(cts.shape[0], dtype=np.uint64)
    _lib.call("tfhe_mi355_client_lwe_decrypt", _ptr(sk), len(sk), _ptr(cts), cts.shape[0], _ptr(pts))
    return pts


def decode(plaintexts, delta: int) -> np.ndarray:
    """shortint decrypt_message_and_carry rounding (shortint/client_key/mod.rs:281-302)."""
    d = np.asarray(plaintexts, dtype=np.uint64)
    rb = np.uint64(delta >> 1)
    rounding = (d & rb) << np.uint64(1)
    return (d + rounding) // np.uint64(delta)
