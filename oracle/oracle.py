"""ctypes wrapper over liboracle_pbs.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker (or the timed CPU baseline).  The product path never imports it.

Every function follows a reference function; the file:line citations are in pbs_oracle.c.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_pbs.so")
_lib = None

u64p = ctypes.POINTER(ctypes.c_uint64)
u32p = ctypes.POINTER(ctypes.c_uint32)
f64p = ctypes.POINTER(ctypes.c_double)


def build(force: bool = False) -> str:
    """Compile the oracle with its own Makefile (gcc)."""
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < max(
        os.path.getmtime(os.path.join(_HERE, f))
        for f in os.listdir(_HERE)
        if f.endswith(".c")
    ):
        subprocess.run(["make", "-C", _HERE, "-B"], check=True, capture_output=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_closest_representable.restype = ctypes.c_uint64
        L.orc_closest_representable.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
        L.orc_decompose.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, u64p]
        L.orc_f64_to_i64.restype = ctypes.c_int64
        L.orc_f64_to_i64.argtypes = [ctypes.c_double]
        L.orc_pbs_modulus_switch.restype = ctypes.c_uint64
        L.orc_pbs_modulus_switch.argtypes = [ctypes.c_uint64, ctypes.c_int]
        L.orc_fft_supported.argtypes = [ctypes.c_int]
        L.orc_fft_product.argtypes = [ctypes.c_int, u64p, u64p, u64p]
        L.orc_fft_roundtrip.argtypes = [ctypes.c_int, u64p, u64p]
        L.orc_fft_complex.argtypes = [ctypes.c_int, f64p, f64p, ctypes.c_int]
        L.orc_negacyclic_mul_u64.argtypes = [ctypes.c_int, u64p, u64p, u64p]
        L.orc_gen_binary_key.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, u64p]
        L.orc_gen_bsk.argtypes = [ctypes.c_uint64, u64p, ctypes.c_int, u64p, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                  u64p, ctypes.c_int]
        L.orc_gen_ksk.argtypes = [ctypes.c_uint64, u64p, ctypes.c_int, u64p, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_double, u64p]
        L.orc_lwe_encrypt_batch.argtypes = [ctypes.c_uint64, u64p, ctypes.c_int, u64p,
                                            ctypes.c_size_t, ctypes.c_double, u64p]
        L.orc_lwe_decrypt_batch.argtypes = [u64p, ctypes.c_int, u64p, ctypes.c_size_t, u64p]
        L.orc_fill_accumulator.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           u64p, u64p]
        L.orc_fbsk_create.restype = ctypes.c_void_p
        L.orc_fbsk_create.argtypes = [u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int]
        L.orc_fbsk_destroy.argtypes = [ctypes.c_void_p]
        L.orc_fbsk_copy.argtypes = [ctypes.c_void_p, f64p]
        L.orc_mb_fbsk_copy.argtypes = [ctypes.c_void_p, f64p]
        L.orc_pbs_batch.argtypes = [ctypes.c_void_p, u64p, u64p, u64p, u32p, ctypes.c_size_t,
                                    ctypes.c_int]
        L.orc_blind_rotate_batch.argtypes = [ctypes.c_void_p, u64p, u64p, u64p, u32p, ctypes.c_size_t,
                                             ctypes.c_int]
        L.orc_keyswitch_batch.argtypes = [u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, u64p, u64p, ctypes.c_size_t]
        L.orc_mono_spectrum.argtypes = [ctypes.c_int, ctypes.c_uint32, f64p]
        L.orc_fft_forward_integer.argtypes = [ctypes.c_int, u64p, f64p]
        L.orc_pos_freq.argtypes = [ctypes.c_int, ctypes.c_int]
        L.orc_gen_pksk.argtypes = [ctypes.c_uint64, u64p, ctypes.c_int, u64p, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_double, u64p]
        L.orc_packing_keyswitch_batch.argtypes = [u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                  ctypes.c_int, u64p, u64p, ctypes.c_size_t]
        L.orc_glwe_poly_mul.argtypes = [ctypes.c_int, ctypes.c_int, u64p, ctypes.c_size_t, u64p,
                                        ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, u64p]
        L.orc_aes128_expand.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint8)]
        L.orc_aes128_encrypt.argtypes = [ctypes.POINTER(ctypes.c_uint8), ctypes.c_char_p,
                                         ctypes.POINTER(ctypes.c_uint8)]
        L.orc_csprng_bytes.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t,
                                       ctypes.POINTER(ctypes.c_uint8)]
        L.orc_seeded_mask_words.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, u64p]
        L.orc_decompress_seeded_bsk.argtypes = [ctypes.c_uint64, ctypes.c_uint64, u64p, ctypes.c_size_t,
                                                ctypes.c_int, ctypes.c_int, ctypes.c_int, u64p]
        L.orc_decompress_seeded_ksk.argtypes = [ctypes.c_uint64, ctypes.c_uint64, u64p, ctypes.c_size_t,
                                                ctypes.c_int, ctypes.c_int, u64p]
        L.orc_negacyclic_mul_add_exact.argtypes = [ctypes.c_int, u64p, u64p, u64p]
        L.orc_exact_pbs_batch.argtypes = [u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, u64p, u64p, u64p, u32p, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.c_int]
        L.orc_exact_mb_pbs_batch.argtypes = [u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, u64p, u64p, u64p, u32p, ctypes.c_size_t,
                                             ctypes.c_int, ctypes.c_int]
        if hasattr(L, "orc_mb_pbs_batch"):
            L.orc_mb_fbsk_create.restype = ctypes.c_void_p
            L.orc_mb_fbsk_create.argtypes = [u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int]
            L.orc_mb_fbsk_destroy.argtypes = [ctypes.c_void_p]
            L.orc_mb_pbs_batch.argtypes = [ctypes.c_void_p, u64p, u64p, u64p, u32p,
                                           ctypes.c_size_t, ctypes.c_int]
            L.orc_gen_mb_bsk.argtypes = [ctypes.c_uint64, u64p, ctypes.c_int, u64p, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_double, u64p, ctypes.c_int]
        _lib = L
    return _lib


def _p(a: np.ndarray, t=u64p):
    return a.ctypes.data_as(t)


def _u64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint64)


# ---- scalar helpers ----------------------------------------------------------------------
def closest_representable(x: int, base_log: int, level: int) -> int:
    return lib().orc_closest_representable(x, base_log, level)


def decompose(x: int, base_log: int, level: int) -> list[int]:
    out = np.zeros(level, dtype=np.uint64)
    lib().orc_decompose(x, base_log, level, _p(out))
    return [int(v) for v in out]


def f64_to_i64(x: float) -> int:
    return lib().orc_f64_to_i64(x)


def pbs_modulus_switch(x: int, log2n: int) -> int:
    return lib().orc_pbs_modulus_switch(x, log2n)


# ---- FFT hooks ---------------------------------------------------------------------------
def fft_product(a_torus: np.ndarray, b_int: np.ndarray) -> np.ndarray:
    a, b = _u64(a_torus), _u64(b_int)
    out = np.zeros_like(a)
    assert lib().orc_fft_product(len(a), _p(a), _p(b), _p(out)) == 0
    return out


def fft_roundtrip(a: np.ndarray) -> np.ndarray:
    a = _u64(a)
    out = np.zeros_like(a)
    assert lib().orc_fft_roundtrip(len(a), _p(a), _p(out)) == 0
    return out


def fft_complex(z: np.ndarray, inverse: bool = False) -> np.ndarray:
    zin = np.ascontiguousarray(z, dtype=np.complex128)
    out = np.zeros_like(zin)
    assert lib().orc_fft_complex(len(zin), zin.ctypes.data_as(f64p), out.ctypes.data_as(f64p),
                                 int(inverse)) == 0
    return out


def negacyclic_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a, b = _u64(a), _u64(b)
    out = np.zeros_like(a)
    lib().orc_negacyclic_mul_u64(len(a), _p(a), _p(b), _p(out))
    return out


def negacyclic_mul_add_exact(a: np.ndarray, b: np.ndarray, out: np.ndarray | None = None) -> np.ndarray:
    """out + a * b in (Z/2^64)[X]/(X^N+1) by Karatsuba (the exact PBS's product)."""
    a, b = _u64(a), _u64(b)
    out = np.zeros_like(a) if out is None else _u64(out).copy()
    lib().orc_negacyclic_mul_add_exact(len(a), _p(a), _p(b), _p(out))
    return out


def exact_pbs(bsk, n, k, N, base_log, level, cts, luts, lut_idx=None, threads=8, glwe_out=False) -> np.ndarray:
    """FFT-free PBS (blind rotation + sample extraction, or the accumulators with glwe_out) with
    exact negacyclic products over the STANDARD-domain BSK (pbs_oracle.c 'FFT-free exact PBS')."""
    bsk = _u64(bsk)
    x = _u64(cts).reshape(-1, n + 1)
    L = _u64(luts)
    if L.ndim == 1:
        L = L.reshape(1, -1)
    out = np.zeros((x.shape[0], (k + 1) * N if glwe_out else k * N + 1), dtype=np.uint64)
    idx = None
    if lut_idx is not None:
        idx = np.ascontiguousarray(lut_idx, dtype=np.uint32)
    lib().orc_exact_pbs_batch(_p(bsk), n, k, N, base_log, level, _p(x), _p(out), _p(L),
                              _p(idx, u32p) if idx is not None else None, x.shape[0], threads, int(glwe_out))
    return out


def exact_mb_pbs(bsk, n, k, N, base_log, level, g, cts, luts, lut_idx=None, threads=8, glwe_out=False) -> np.ndarray:
    """FFT-free multi-bit PBS: exact standard-domain keybundles and exact external products
    (pbs_oracle.c 'exact multi-bit PBS'), deterministic group order."""
    bsk = _u64(bsk)
    x = _u64(cts).reshape(-1, n + 1)
    L = _u64(luts)
    if L.ndim == 1:
        L = L.reshape(1, -1)
    out = np.zeros((x.shape[0], (k + 1) * N if glwe_out else k * N + 1), dtype=np.uint64)
    idx = None
    if lut_idx is not None:
        idx = np.ascontiguousarray(lut_idx, dtype=np.uint32)
    lib().orc_exact_mb_pbs_batch(_p(bsk), n, k, N, base_log, level, g, _p(x), _p(out), _p(L),
                                 _p(idx, u32p) if idx is not None else None, x.shape[0], threads, int(glwe_out))
    return out


# ---- keys / encryption -------------------------------------------------------------------
def binary_key(seed: int, stream: int, length: int) -> np.ndarray:
    k = np.zeros(length, dtype=np.uint64)
    lib().orc_gen_binary_key(seed, stream, length, _p(k))
    return k


def gen_bsk(seed, lwe_sk, glwe_sk, k, N, base_log, level, std, threads=8) -> np.ndarray:
    n = len(lwe_sk)
    bsk = np.zeros(n * level * (k + 1) * (k + 1) * N, dtype=np.uint64)
    lib().orc_gen_bsk(seed, _p(_u64(lwe_sk)), n, _p(_u64(glwe_sk)), k, N, base_log, level,
                      std, _p(bsk), threads)
    return bsk


def gen_ksk(seed, in_sk, out_sk, base_log, level, std) -> np.ndarray:
    ksk = np.zeros(len(in_sk) * level * (len(out_sk) + 1), dtype=np.uint64)
    lib().orc_gen_ksk(seed, _p(_u64(in_sk)), len(in_sk), _p(_u64(out_sk)), len(out_sk),
                      base_log, level, std, _p(ksk))
    return ksk


def lwe_encrypt(seed, sk, plaintexts, std) -> np.ndarray:
    pts = _u64(plaintexts)
    n = len(sk)
    cts = np.zeros((len(pts), n + 1), dtype=np.uint64)
    lib().orc_lwe_encrypt_batch(seed, _p(_u64(sk)), n, _p(pts), len(pts), std, _p(cts))
    return cts


def lwe_decrypt(sk, cts) -> np.ndarray:
    cts = _u64(cts)
    n = len(sk)
    cts2 = cts.reshape(-1, n + 1)
    pts = np.zeros(cts2.shape[0], dtype=np.uint64)
    lib().orc_lwe_decrypt_batch(_p(_u64(sk)), n, _p(cts2), cts2.shape[0], _p(pts))
    return pts


def fill_accumulator(N, k, msg_mod, carry_mod, f) -> np.ndarray:
    p = msg_mod * carry_mod
    fv = _u64([f(i) for i in range(p)])
    acc = np.zeros((k + 1) * N, dtype=np.uint64)
    lib().orc_fill_accumulator(N, k, msg_mod, carry_mod, _p(fv), _p(acc))
    return acc


# ---- PBS / KS ----------------------------------------------------------------------------
_simd = None


def simd_variant() -> str:
    """'v4' (AVX-512, 8 lanes) when the host has avx512f+avx512dq, else 'v3' (AVX2, 4 lanes)."""
    flags = set()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("flags"):
                flags = set(line.split(":", 1)[1].split())
                break
    except OSError:
        pass
    return "v4" if {"avx512f", "avx512dq"} <= flags else "v3"


def simd_lib():
    """libpbs_simd_<v>.so: the CPU baseline's SIMD-across-ciphertexts build of the oracle PBS."""
    global _simd
    if _simd is None:
        path = os.path.join(_HERE, f"libpbs_simd_{simd_variant()}.so")
        if not os.path.exists(path):
            build(force=True)
        L = ctypes.CDLL(path)
        L.simd_width.restype = ctypes.c_int
        L.simd_pbs_batch.restype = ctypes.c_int
        L.simd_pbs_batch.argtypes = [f64p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     u64p, u64p, u64p, u32p, ctypes.c_size_t, ctypes.c_int]
        L.simd_keyswitch_batch.argtypes = [u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, u64p, u64p,
                                           ctypes.c_size_t]
        L.simd_mb_pbs_batch.restype = ctypes.c_int
        L.simd_mb_pbs_batch.argtypes = [f64p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, u64p, u64p, u64p, u32p, ctypes.c_size_t, ctypes.c_int]
        _simd = L
    return _simd


def keyswitch_simd(ksk, in_dim, out_dim, base_log, level, cts) -> np.ndarray:
    """orc keyswitch through the SIMD build (vectorised AXPY, bit-identical): the CPU baseline's KS."""
    ksk = _u64(ksk)
    x = _u64(cts).reshape(-1, in_dim + 1)
    out = np.zeros((x.shape[0], out_dim + 1), dtype=np.uint64)
    simd_lib().simd_keyswitch_batch(_p(ksk), in_dim, out_dim, base_log, level, _p(x), _p(out), x.shape[0])
    return out


class FourierBsk:
    """fbsk = Fourier BSK built with the oracle FFT (lwe_bootstrap_key_conversion.rs)."""

    def __init__(self, bsk, n, k, N, base_log, level):
        self.n, self.k, self.N, self.base_log, self.level = n, k, N, base_log, level
        self._bsk = _u64(bsk)
        self.h = lib().orc_fbsk_create(_p(self._bsk), n, k, N, base_log, level)
        assert self.h

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_fbsk_destroy(self.h)
            self.h = None

    def fourier(self) -> np.ndarray:
        out = np.zeros(self.n * self.level * (self.k + 1) ** 2 * self.N // 2, dtype=np.complex128)
        lib().orc_fbsk_copy(self.h, out.ctypes.data_as(f64p))
        return out

    def pbs(self, lwe_in, luts, lut_idx=None, threads=8) -> np.ndarray:
        lwe_in = _u64(lwe_in).reshape(-1, self.n + 1)
        luts = _u64(luts)
        cnt = lwe_in.shape[0]
        out = np.zeros((cnt, self.k * self.N + 1), dtype=np.uint64)
        idx = None
        if lut_idx is not None:
            idx = np.ascontiguousarray(lut_idx, dtype=np.uint32)
        lib().orc_pbs_batch(self.h, _p(lwe_in), _p(out), _p(luts),
                            idx.ctypes.data_as(u32p) if idx is not None else None, cnt, threads)
        return out

    def pbs_simd(self, lwe_in, luts, lut_idx=None, threads=8) -> np.ndarray:
        """Same PBS as `pbs` through pbs_simd.c (W ciphertexts per SIMD register, bit-identical):
        the CPU baseline's throughput form."""
        lwe_in = _u64(lwe_in).reshape(-1, self.n + 1)
        luts = _u64(luts)
        if getattr(self, "_fourier", None) is None:
            self._fourier = self.fourier()
        cnt = lwe_in.shape[0]
        out = np.zeros((cnt, self.k * self.N + 1), dtype=np.uint64)
        idx = None
        if lut_idx is not None:
            idx = np.ascontiguousarray(lut_idx, dtype=np.uint32)
        rc = simd_lib().simd_pbs_batch(self._fourier.ctypes.data_as(f64p), self.n, self.k, self.N, self.base_log,
                                       self.level, _p(lwe_in), _p(out), _p(luts),
                                       idx.ctypes.data_as(u32p) if idx is not None else None, cnt, threads)
        assert rc == 0, "pbs_simd: unsupported polynomial size"
        return out

    def blind_rotate(self, lwe_in, luts, lut_idx=None, threads=8) -> np.ndarray:
        """bootstrap_without_sample_extract: the accumulators [count][(k+1)N]."""
        lwe_in = _u64(lwe_in).reshape(-1, self.n + 1)
        luts = _u64(luts)
        cnt = lwe_in.shape[0]
        out = np.zeros((cnt, (self.k + 1) * self.N), dtype=np.uint64)
        idx = None
        if lut_idx is not None:
            idx = np.ascontiguousarray(lut_idx, dtype=np.uint32)
        lib().orc_blind_rotate_batch(self.h, _p(lwe_in), _p(out), _p(luts),
                                     idx.ctypes.data_as(u32p) if idx is not None else None, cnt, threads)
        return out


def mono_spectrum(N: int, d: int) -> np.ndarray:
    """Closed-form spectrum of X^d in FFT position order (multi-bit keybundle monomials)."""
    out = np.zeros(N // 2, dtype=np.complex128)
    assert lib().orc_mono_spectrum(N, d, out.ctypes.data_as(f64p)) == 0
    return out


def fft_forward_integer(x) -> np.ndarray:
    x = _u64(x)
    out = np.zeros(x.size // 2, dtype=np.complex128)
    assert lib().orc_fft_forward_integer(x.size, _p(x), out.ctypes.data_as(f64p)) == 0
    return out


def pos_freq(N: int) -> np.ndarray:
    return np.array([lib().orc_pos_freq(N, P) for P in range(N // 2)], dtype=np.int64)


def gen_mb_bsk(seed, lwe_sk, glwe_sk, k, N, base_log, level, g, std, threads=8) -> np.ndarray:
    """Standard multi-bit BSK [n/g][2^g][L][k+1][k+1][N] (lwe_multi_bit_bootstrap_key_generation.rs)."""
    lwe_sk, glwe_sk = _u64(lwe_sk), _u64(glwe_sk)
    n = lwe_sk.size
    out = np.zeros((n // g) * (1 << g) * level * (k + 1) ** 2 * N, dtype=np.uint64)
    lib().orc_gen_mb_bsk(seed, _p(lwe_sk), n, _p(glwe_sk), k, N, base_log, level, g, std, _p(out),
                         threads)
    return out


class MultiBitFourierBsk:
    """Multi-bit Fourier BSK + deterministic multi-bit PBS
    (lwe_multi_bit_programmable_bootstrapping.rs:548-828, 1035-1128)."""

    def __init__(self, bsk, n, k, N, base_log, level, g):
        self.n, self.k, self.N, self.base_log, self.level, self.g = n, k, N, base_log, level, g
        self._bsk = _u64(bsk)
        self.h = lib().orc_mb_fbsk_create(_p(self._bsk), n, k, N, base_log, level, g)
        assert self.h

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_mb_fbsk_destroy(self.h)
            self.h = None

    def fourier(self) -> np.ndarray:
        npoly = (self.n // self.g << self.g) * self.level * (self.k + 1) ** 2
        out = np.zeros(npoly * self.N // 2, dtype=np.complex128)
        lib().orc_mb_fbsk_copy(self.h, out.ctypes.data_as(f64p))
        return out

    def pbs(self, lwe_in, luts, lut_idx=None, threads=8) -> np.ndarray:
        lwe_in = _u64(lwe_in).reshape(-1, self.n + 1)
        luts = _u64(luts)
        cnt = lwe_in.shape[0]
        out = np.zeros((cnt, self.k * self.N + 1), dtype=np.uint64)
        idx = None
        if lut_idx is not None:
            idx = np.ascontiguousarray(lut_idx, dtype=np.uint32)
        lib().orc_mb_pbs_batch(self.h, _p(lwe_in), _p(out), _p(luts),
                               idx.ctypes.data_as(u32p) if idx is not None else None, cnt, threads)
        return out

    def pbs_simd(self, lwe_in, luts, lut_idx=None, threads=8) -> np.ndarray:
        """Same multi-bit PBS through pbs_simd.c (W ciphertexts per SIMD register, bit-identical)."""
        lwe_in = _u64(lwe_in).reshape(-1, self.n + 1)
        luts = _u64(luts)
        if getattr(self, "_fourier", None) is None:
            self._fourier = self.fourier()
        cnt = lwe_in.shape[0]
        out = np.zeros((cnt, self.k * self.N + 1), dtype=np.uint64)
        idx = None
        if lut_idx is not None:
            idx = np.ascontiguousarray(lut_idx, dtype=np.uint32)
        rc = simd_lib().simd_mb_pbs_batch(self._fourier.ctypes.data_as(f64p), self.n, self.k, self.N, self.base_log,
                                          self.level, self.g, _p(lwe_in), _p(out), _p(luts),
                                          idx.ctypes.data_as(u32p) if idx is not None else None, cnt, threads)
        assert rc == 0, "pbs_simd: unsupported shape"
        return out


def _fbsk_blind_rotate(self, lwe_in, luts, lut_idx=None, threads=8) -> np.ndarray:
    lwe_in = _u64(lwe_in).reshape(-1, self.n + 1)
    luts = _u64(luts)
    cnt = lwe_in.shape[0]
    out = np.zeros((cnt, (self.k + 1) * self.N), dtype=np.uint64)
    idx = None if lut_idx is None else np.ascontiguousarray(lut_idx, dtype=np.uint32)
    lib().orc_blind_rotate_batch(self.h, _p(lwe_in), _p(out), _p(luts),
                                 idx.ctypes.data_as(u32p) if idx is not None else None, cnt, threads)
    return out


FourierBsk.blind_rotate = _fbsk_blind_rotate


def keyswitch(ksk, in_dim, out_dim, base_log, level, lwe_in) -> np.ndarray:
    lwe_in = _u64(lwe_in).reshape(-1, in_dim + 1)
    out = np.zeros((lwe_in.shape[0], out_dim + 1), dtype=np.uint64)
    lib().orc_keyswitch_batch(_p(_u64(ksk)), in_dim, out_dim, base_log, level, _p(lwe_in),
                              _p(out), lwe_in.shape[0])
    return out


def gen_pksk(seed, in_sk, glwe_sk, k, N, base_log, level, std) -> np.ndarray:
    in_sk, glwe_sk = _u64(in_sk), _u64(glwe_sk)
    out = np.zeros(len(in_sk) * level * (k + 1) * N, dtype=np.uint64)
    lib().orc_gen_pksk(seed, _p(in_sk), len(in_sk), _p(glwe_sk), k, N, base_log, level, std, _p(out))
    return out


def packing_keyswitch(pksk, in_dim, k, N, base_log, level, lwe_in) -> np.ndarray:
    x = _u64(lwe_in).reshape(-1, in_dim + 1)
    out = np.zeros((len(x), (k + 1) * N), dtype=np.uint64)
    lib().orc_packing_keyswitch_batch(_p(_u64(pksk)), in_dim, k, N, base_log, level, _p(x), _p(out), len(x))
    return out


def glwe_poly_mul(k, N, glwe_in, polys, extract: bool) -> np.ndarray:
    """glwe_in [count][J][(k+1)N], polys [npoly][J][N] -> [count][npoly][(k+1)N or kN+1]."""
    g = _u64(glwe_in)
    v = _u64(polys)
    if g.ndim == 2:
        g = g.reshape(g.shape[0], 1, -1)
    if v.ndim == 2:
        v = v.reshape(v.shape[0], 1, -1)
    count, J = g.shape[0], g.shape[1]
    npoly = v.shape[0]
    assert v.shape[1] == J and v.shape[2] == N and g.shape[2] == (k + 1) * N
    out = np.zeros((count, npoly, k * N + 1 if extract else (k + 1) * N), dtype=np.uint64)
    lib().orc_glwe_poly_mul(k, N, _p(g), J, _p(v), npoly, count, int(extract), _p(out))
    return out


# ---- seeded keys (csprng_oracle.c) ----------------------------------------------------------
def aes128_encrypt(key: bytes, block: bytes) -> bytes:
    rk = (ctypes.c_uint8 * 176)()
    out = (ctypes.c_uint8 * 16)()
    lib().orc_aes128_expand(key, rk)
    lib().orc_aes128_encrypt(rk, block, out)
    return bytes(out)


def aes128_round_keys(key: bytes) -> bytes:
    rk = (ctypes.c_uint8 * 176)()
    lib().orc_aes128_expand(key, rk)
    return bytes(rk)


def _seed(seed: int):
    return seed & 0xFFFFFFFFFFFFFFFF, (seed >> 64) & 0xFFFFFFFFFFFFFFFF


def csprng_bytes(seed: int, offset: int, count: int) -> bytes:
    out = (ctypes.c_uint8 * count)()
    lib().orc_csprng_bytes(*_seed(seed), offset, count, out)
    return bytes(out)


def seeded_mask_words(seed: int, first_word: int, count: int) -> np.ndarray:
    out = np.zeros(count, dtype=np.uint64)
    lib().orc_seeded_mask_words(*_seed(seed), first_word, count, _p(out))
    return out


def decompress_seeded_bsk(seed: int, bodies, n_ggsw: int, level: int, k: int, N: int) -> np.ndarray:
    b = _u64(bodies)
    out = np.zeros(n_ggsw * level * (k + 1) * (k + 1) * N, dtype=np.uint64)
    lib().orc_decompress_seeded_bsk(*_seed(seed), _p(b), n_ggsw, level, k, N, _p(out))
    return out


def decompress_seeded_ksk(seed: int, bodies, in_dim: int, level: int, out_dim: int) -> np.ndarray:
    b = _u64(bodies)
    out = np.zeros(in_dim * level * (out_dim + 1), dtype=np.uint64)
    lib().orc_decompress_seeded_ksk(*_seed(seed), _p(b), in_dim, level, out_dim, _p(out))
    return out


class OracleEngine:
    """The oracle (CPU restatement) behind the Engine's host API, so host-side orchestration
    (shortint / integer layers) can run its exact DAG on the CPU as the parity reference."""

    def __init__(self, params, threads=8, simd=False):
        """simd: run the PBS and keyswitch through pbs_simd.c (bit-identical; the CPU baseline)."""
        import sys

        O = sys.modules[__name__]
        build()
        self.O, self.p, self.threads, self.simd = O, params, threads, simd
        self.fb = self.ksk = None

    def _pbs(self, x, luts, lut_indexes):
        f = self.fb.pbs_simd if self.simd else self.fb.pbs
        return f(x, luts, lut_indexes, threads=self.threads)

    def upload_bootstrap_key(self, bsk):
        p = self.p
        self.fb = self.O.FourierBsk(bsk, p.lwe_dimension, p.glwe_dimension, p.polynomial_size,
                                    p.pbs_base_log, p.pbs_level)

    def upload_keyswitch_key(self, ksk):
        self.ksk = np.ascontiguousarray(ksk, dtype=np.uint64)

    def keyswitch(self, x):
        from concurrent.futures import ThreadPoolExecutor

        p = self.p
        parts = [c for c in np.array_split(np.asarray(x), min(self.threads, len(x))) if len(c)]
        with ThreadPoolExecutor(len(parts)) as ex:
            ks = self.O.keyswitch_simd if self.simd else self.O.keyswitch
            outs = list(ex.map(lambda c: ks(self.ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log,
                                            p.ks_level, c), parts))
        return np.concatenate(outs)

    def keyswitch_programmable_bootstrap(self, x, luts, lut_indexes=None):
        return self._pbs(self.keyswitch(x), luts, lut_indexes)

    def programmable_bootstrap(self, x, luts, lut_indexes=None):
        return self._pbs(x, luts, lut_indexes)

    def programmable_bootstrap_keyswitch(self, x, luts, lut_indexes=None):
        return self.keyswitch(self._pbs(x, luts, lut_indexes))

    def blind_rotate(self, x, luts, lut_indexes=None):
        return self.fb.blind_rotate(x, luts, lut_indexes, threads=self.threads)

    def upload_packing_keyswitch_key(self, pksk, base_log, level):
        self.pksk, self.pks = np.ascontiguousarray(pksk, dtype=np.uint64), (base_log, level)

    def packing_keyswitch(self, x):
        p = self.p
        return packing_keyswitch(self.pksk, p.big_lwe_dimension, p.glwe_dimension, p.polynomial_size,
                                 self.pks[0], self.pks[1], x)

    def glwe_poly_mul(self, glwe_in, polys, extract=False):
        p = self.p
        return glwe_poly_mul(p.glwe_dimension, p.polynomial_size, glwe_in, polys, extract)
