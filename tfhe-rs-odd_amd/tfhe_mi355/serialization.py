"""Wire formats of the reference's shortint server keys.

A tfhe-rs 0.5 server key travels as the bincode 1.3.3 encoding of its serde derive
(`bincode::serialize(&key)`; tfhe/Cargo.toml:36,57).  Reading is done by the C ABI
(csrc/serde.cpp: tfhe_mi355_{compressed_,}server_key_{inspect,upload}); this module mirrors the
reference's types on the host:

  * `inspect_compressed_server_key` / `inspect_server_key` -> `ServerKeyInfo` (no GPU needed);
  * `serialize_compressed_server_key` / `serialize_server_key`: the writer side, byte for byte the
    Serialize derives of CompressedServerKey (shortint/server_key/compressed.rs:43-55) and
    ServerKey (server_key/mod.rs:112-143,283-297) under bincode's default options -- what a
    tfhe-rs client produces, so that keys made by this engine's client side can be shipped the
    same way (and the reader tested without a Rust toolchain).

bincode default options: little-endian fixed-width integers, usize = u64, u128 = low then high
u64, Vec / serialize_seq = u64 length + elements, enum variant = u32 index, bool = 1 byte,
newtype structs (LweSize(usize), ...) = their field.
"""
from __future__ import annotations

import ctypes
import struct
from dataclasses import dataclass

import numpy as np

from . import _lib
from .parameters import ALL, ClassicPBSParameters

KEYSWITCH_BOOTSTRAP, BOOTSTRAP_KEYSWITCH = 0, 1   # PBSOrder variants (commons/parameters.rs:234-246)


@dataclass
class ServerKeyInfo:
    """What a serialized server key implies (tfhe_mi355.h TfheMi355ServerKeyInfo)."""

    lwe_dimension: int
    glwe_dimension: int
    polynomial_size: int
    pbs_base_log: int
    pbs_level: int
    ks_base_log: int
    ks_level: int
    message_modulus: int
    carry_modulus: int
    grouping_factor: int
    pbs_order: int
    deterministic_execution: bool
    max_degree: int
    max_noise_level: int
    ksk_seed: int   # CompressionSeed (u128) of a CompressedServerKey's keys, else 0
    bsk_seed: int

    def parameters(self) -> ClassicPBSParameters:
        """The known parameter set with these values (std devs are not serialized: a key that
        matches none gets a set named 'deserialized' with zero std devs -- the server side never
        samples noise)."""
        fields = ("lwe_dimension", "glwe_dimension", "polynomial_size", "pbs_base_log", "pbs_level",
                  "ks_base_log", "ks_level", "message_modulus", "carry_modulus", "grouping_factor")
        choice = "Big" if self.pbs_order == KEYSWITCH_BOOTSTRAP else "Small"
        for p in ALL.values():
            if all(getattr(p, f) == getattr(self, f) for f in fields) and p.encryption_key_choice == choice:
                return p
        return ClassicPBSParameters(
            lwe_dimension=self.lwe_dimension, glwe_dimension=self.glwe_dimension,
            polynomial_size=self.polynomial_size, lwe_modular_std_dev=0.0, glwe_modular_std_dev=0.0,
            pbs_base_log=self.pbs_base_log, pbs_level=self.pbs_level, ks_base_log=self.ks_base_log,
            ks_level=self.ks_level, message_modulus=self.message_modulus,
            carry_modulus=self.carry_modulus, encryption_key_choice=choice,
            grouping_factor=self.grouping_factor, name="deserialized")


def _info(fn: str, data: bytes) -> ServerKeyInfo:
    buf = np.frombuffer(data, dtype=np.uint8)
    out = _lib.TfheMi355ServerKeyInfo()
    _lib.call(fn, buf.ctypes.data_as(_lib.u8p), buf.size, ctypes.byref(out))
    p = out.params
    return ServerKeyInfo(p.lwe_dimension, p.glwe_dimension, p.polynomial_size, p.pbs_base_log, p.pbs_level,
                         p.ks_base_log, p.ks_level, p.message_modulus, p.carry_modulus, p.grouping_factor,
                         out.pbs_order, bool(out.deterministic_execution), out.max_degree, out.max_noise_level,
                         out.ksk_seed_lo | (out.ksk_seed_hi << 64), out.bsk_seed_lo | (out.bsk_seed_hi << 64))


def inspect_compressed_server_key(data: bytes) -> ServerKeyInfo:
    return _info("tfhe_mi355_compressed_server_key_inspect", data)


def inspect_server_key(data: bytes) -> ServerKeyInfo:
    return _info("tfhe_mi355_server_key_inspect", data)


def engine_frequency(N: int) -> np.ndarray:
    """freq[e]: natural DFT index held by element e of a polynomial in the engine Fourier layout."""
    f = np.zeros(N // 2, dtype=np.uint32)
    _lib.call("tfhe_mi355_fourier_engine_frequency", N, f.ctypes.data_as(_lib.u32p))
    return f


# ---- writer (the Serialize derives under bincode's default options) -----------------------------

def _u32(v):
    return struct.pack("<I", v)


def _u64(v):
    return struct.pack("<Q", v)


def _u128(v):
    return struct.pack("<QQ", v & (2 ** 64 - 1), v >> 64)


def _vec_u64(a):
    a = np.ascontiguousarray(a, dtype="<u8").ravel()
    return _u64(a.size) + a.tobytes()


def _modulus():
    """CiphertextModulus<u64>::new_native(): {modulus: 0u128, scalar_bits: 64} (ciphertext_modulus.rs:41-64)"""
    return _u128(0) + _u64(64)


def _default_max_degree(p):
    return p.message_modulus * p.carry_modulus - 1


def serialize_compressed_server_key(p: ClassicPBSParameters, ksk_bodies, ksk_seed: int, bsk_bodies, bsk_seed: int,
                                    max_degree: int | None = None, deterministic_execution: bool = False) -> bytes:
    """CompressedServerKey: seeded KSK bodies [k N][ks_level] and seeded BSK bodies
    [ggsw][level][k+1][N] (multi-bit: ggsw = (n/g) 2^g) with their CompressionSeeds."""
    out = [_vec_u64(ksk_bodies), _u64(p.ks_base_log), _u64(p.ks_level), _u64(p.lwe_dimension + 1),
           _u128(ksk_seed), _modulus()]
    ggsw = [_vec_u64(bsk_bodies), _u64(p.glwe_dimension + 1), _u64(p.polynomial_size), _u64(p.pbs_base_log),
            _u64(p.pbs_level), _u128(bsk_seed), _modulus()]
    if p.grouping_factor:
        out += [_u32(1)] + ggsw + [_u64(p.grouping_factor), bytes([int(deterministic_execution)])]
    else:
        out += [_u32(0)] + ggsw
    order = KEYSWITCH_BOOTSTRAP if p.encryption_key_choice == "Big" else BOOTSTRAP_KEYSWITCH
    out += [_u64(p.message_modulus), _u64(p.carry_modulus),
            _u64(_default_max_degree(p) if max_degree is None else max_degree), _modulus(), _u32(order)]
    return b"".join(out)


def serialize_server_key(p: ClassicPBSParameters, ksk, fourier_bsk, max_degree: int | None = None,
                         max_noise_level: int = 5, deterministic_execution: bool = False) -> bytes:
    """ServerKey: standard KSK [k N][ks_level][n+1] and the Fourier BSK as complex128
    [polys][M] in natural DFT order (FourierPolynomialList, fft64/math/fft/mod.rs:588-632; each
    polynomial a seq of M (re, im) pairs -- concrete-fft's serialize_fourier_buffer, restated)."""
    fb = np.ascontiguousarray(fourier_bsk, dtype=np.complex128)
    M = p.polynomial_size // 2
    fb = fb.reshape(-1, M)
    polys = fb.shape[0]
    four = [_u64(2 + polys), _u64(p.polynomial_size), _u64(polys)]
    body = np.empty((polys, 8 + 16 * M), dtype=np.uint8)
    body[:, :8] = np.frombuffer(_u64(M), dtype=np.uint8)
    body[:, 8:] = fb.view("<f8").view(np.uint8).reshape(polys, 16 * M)
    four.append(body.tobytes())
    out = [_vec_u64(ksk), _u64(p.ks_base_log), _u64(p.ks_level), _u64(p.lwe_dimension + 1), _modulus()]
    fields = [_u64(p.lwe_dimension), _u64(p.glwe_dimension + 1), _u64(p.pbs_base_log), _u64(p.pbs_level)]
    if p.grouping_factor:
        out += [_u32(1)] + four + fields + [_u64(p.grouping_factor), bytes([int(deterministic_execution)])]
    else:
        out += [_u32(0)] + four + fields
    order = KEYSWITCH_BOOTSTRAP if p.encryption_key_choice == "Big" else BOOTSTRAP_KEYSWITCH
    out += [_u64(p.message_modulus), _u64(p.carry_modulus),
            _u64(_default_max_degree(p) if max_degree is None else max_degree), _u64(max_noise_level),
            _modulus(), _u32(order)]
    return b"".join(out)
