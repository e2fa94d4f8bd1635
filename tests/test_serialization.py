"""Serialized server keys without a GPU: the bincode layout of the reference's
CompressedServerKey / ServerKey is parsed by the C ABI (csrc/serde.cpp), validated field by field,
and the engine Fourier layout map agrees with the oracle's FFT position order.

Pinning: the reference holds no serialized keys (no fixture files), so the byte layout is pinned
by a tiny key assembled here BY HAND from the reference's type definitions (the field order of
each serde derive, cited inline) and bincode 1.3's default options -- independent of the writer
in tfhe_mi355/serialization.py, which must produce the same bytes.  concrete-fft's Fourier
buffer order (absent crate) is parity unpinned."""
import struct

import numpy as np
import pytest

from tfhe_mi355 import serialization as S
from tfhe_mi355.parameters import (PARAM_MESSAGE_2_CARRY_2_KS_PBS, PARAM_MESSAGE_4_CARRY_4_KS_PBS,
                                   PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS)

TINY = PARAM_MESSAGE_2_CARRY_2_KS_PBS.with_(lwe_dimension=2, polynomial_size=4, ks_level=2, ks_base_log=4,
                                            pbs_level=1, pbs_base_log=20, name="tiny")


def q(v):
    return struct.pack("<Q", v)


def _tiny_compressed_by_hand(ksk, kseed, bsk, bseed):
    b = b""
    # CompressedServerKey.key_switching_key: SeededLweKeyswitchKey (seeded_lwe_keyswitch_key.rs:11-21)
    b += q(len(ksk)) + b"".join(q(int(x)) for x in ksk)       # data: Vec<u64>
    b += q(4) + q(2)                                           # decomp_base_log, decomp_level_count
    b += q(3)                                                  # output_lwe_size = n + 1
    b += q(kseed & (2 ** 64 - 1)) + q(kseed >> 64)             # CompressionSeed { Seed(u128) }
    b += q(0) + q(0) + q(64)                                   # CiphertextModulus {modulus u128, scalar_bits}
    # .bootstrapping_key: ShortintCompressedBootstrappingKey::Classic (compressed.rs:10-17)
    b += struct.pack("<I", 0)
    b += q(len(bsk)) + b"".join(q(int(x)) for x in bsk)       # SeededGgswCiphertextList.data
    b += q(2) + q(4) + q(20) + q(1)                            # glwe_size, polynomial_size, base_log, level
    b += q(bseed & (2 ** 64 - 1)) + q(bseed >> 64) + q(0) + q(0) + q(64)
    b += q(4) + q(4) + q(15)                                   # message_modulus, carry_modulus, max_degree
    b += q(0) + q(0) + q(64)                                   # ciphertext_modulus
    b += struct.pack("<I", 0)                                  # PBSOrder::KeyswitchBootstrap
    return b


def test_compressed_server_key_bytes_match_hand_layout():
    rng = np.random.default_rng(0)
    ksk = rng.integers(0, 2 ** 64, 4 * 2, dtype=np.uint64)     # [k N = 4][ks_level = 2] bodies
    bsk = rng.integers(0, 2 ** 64, 2 * 1 * 2 * 4, dtype=np.uint64)  # [n][L][k+1][N] bodies
    kseed, bseed = (0xDEAD << 64) | 0xBEEF, 0x1234
    hand = _tiny_compressed_by_hand(ksk, kseed, bsk, bseed)
    assert S.serialize_compressed_server_key(TINY, ksk, kseed, bsk, bseed) == hand
    info = S.inspect_compressed_server_key(hand)
    assert (info.lwe_dimension, info.glwe_dimension, info.polynomial_size) == (2, 1, 4)
    assert (info.pbs_base_log, info.pbs_level, info.ks_base_log, info.ks_level) == (20, 1, 4, 2)
    assert (info.message_modulus, info.carry_modulus, info.max_degree) == (4, 4, 15)
    assert (info.ksk_seed, info.bsk_seed, info.pbs_order, info.grouping_factor) == (kseed, bseed, 0, 0)


def _shapes(p):
    g = p.grouping_factor
    ggsw = (p.lwe_dimension // g) << g if g else p.lwe_dimension
    return ggsw, p.big_lwe_dimension * p.ks_level, ggsw * p.pbs_level * (p.glwe_dimension + 1) * p.polynomial_size


@pytest.mark.parametrize("p", [PARAM_MESSAGE_2_CARRY_2_KS_PBS, PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS,
                               PARAM_MESSAGE_4_CARRY_4_KS_PBS.with_(lwe_dimension=4)],
                         ids=["2_2", "mb_g3", "4_4_n4"])
def test_compressed_round_trip_full_shapes(p):
    _, kw, bw = _shapes(p)
    ksk = np.arange(kw, dtype=np.uint64)
    bsk = np.arange(bw, dtype=np.uint64)[::-1].copy()
    data = S.serialize_compressed_server_key(p, ksk, 5, bsk, 6, deterministic_execution=True)
    info = S.inspect_compressed_server_key(data)
    for f in ("lwe_dimension", "glwe_dimension", "polynomial_size", "pbs_base_log", "pbs_level", "ks_base_log",
              "ks_level", "message_modulus", "carry_modulus", "grouping_factor"):
        assert getattr(info, f) == getattr(p, f), f
    assert info.deterministic_execution == bool(p.grouping_factor)
    from tfhe_mi355.parameters import ALL

    if ALL.get(p.name) == p:
        assert info.parameters() == p


def test_every_truncation_is_rejected():
    rng = np.random.default_rng(1)
    data = S.serialize_compressed_server_key(TINY, rng.integers(0, 9, 8, dtype=np.uint64), 1,
                                             rng.integers(0, 9, 16, dtype=np.uint64), 2)
    for cut in range(len(data)):
        with pytest.raises(Exception, match="truncated"):
            S.inspect_compressed_server_key(data[:cut])
    with pytest.raises(Exception, match="trailing"):
        S.inspect_compressed_server_key(data + b"\0")


def test_inconsistent_or_unsupported_keys_are_rejected():
    ksk, bsk = np.zeros(8, dtype=np.uint64), np.zeros(16, dtype=np.uint64)
    good = _tiny_compressed_by_hand(ksk, 1, bsk, 2)
    ks_mod = 8 + 64 + 8 * 3 + 16            # offset of the KSK's CiphertextModulus
    bad = bytearray(good)
    bad[ks_mod] = 1                          # modulus 1 (non-native)
    with pytest.raises(Exception, match="non-native"):
        S.inspect_compressed_server_key(bytes(bad))
    bad = bytearray(good)
    bad[ks_mod + 16] = 32                    # scalar_bits 32
    with pytest.raises(Exception, match="32-bit"):
        S.inspect_compressed_server_key(bytes(bad))
    bad = bytearray(good)
    bad[ks_mod + 24] = 2                     # ShortintCompressedBootstrappingKey variant 2
    with pytest.raises(Exception, match="variant 2"):
        S.inspect_compressed_server_key(bytes(bad))
    with pytest.raises(Exception, match="keyswitching key"):  # 3 KSK bodies per input coefficient
        S.inspect_compressed_server_key(_tiny_compressed_by_hand(np.zeros(12, dtype=np.uint64), 1, bsk, 2))
    with pytest.raises(Exception, match="whole number of GGSWs"):
        S.inspect_compressed_server_key(_tiny_compressed_by_hand(ksk, 1, np.zeros(17, dtype=np.uint64), 2))
    mb = S.serialize_compressed_server_key(TINY.with_(grouping_factor=1, lwe_dimension=2), ksk, 1,
                                           np.zeros(4 * 8, dtype=np.uint64), 2, deterministic_execution=True)
    bad = bytearray(mb)
    bad[-(8 * 3 + 24 + 4) - 1] = 7           # deterministic_execution: bool byte 7
    with pytest.raises(Exception, match="invalid bool"):
        S.inspect_compressed_server_key(bytes(bad))


def test_oversized_header_fields_fail_with_a_message():
    """Header fields that would wrap the word-count products (glwe_size = N = 2^32, L = 1 makes
    L (k+1) N = 0 mod 2^64 and the next `% per` a division by zero) are range-checked before any
    arithmetic: the call returns an error, it does not crash the process."""
    ksk, bsk = np.zeros(8, dtype=np.uint64), np.zeros(16, dtype=np.uint64)
    good = _tiny_compressed_by_hand(ksk, 1, bsk, 2)
    glwe_off = 8 + 64 + 8 * 3 + 16 + 24 + 4 + 8 + 16 * 8   # SeededGgswCiphertextList.glwe_size
    assert struct.unpack_from("<QQ", good, glwe_off) == (2, 4)
    for gs, n, lvl in [(2 ** 32, 2 ** 32, 1), (2, 2 ** 63, 1), (2, 4, 2 ** 63), (2 ** 63, 4, 1), (2, 6, 1)]:
        bad = bytearray(good)
        struct.pack_into("<QQ", bad, glwe_off, gs, n)
        struct.pack_into("<Q", bad, glwe_off + 24, lvl)
        with pytest.raises(Exception, match="out of range|power of two"):
            S.inspect_compressed_server_key(bytes(bad))
    # ServerKey: a FourierPolynomialList claiming N = 2^62 (M * 16 would wrap the bounds check)
    p = PARAM_MESSAGE_2_CARRY_2_KS_PBS.with_(lwe_dimension=3)
    ksk = np.zeros(p.big_lwe_dimension * p.ks_level * (p.lwe_dimension + 1), dtype=np.uint64)
    fb = np.zeros((3 * 4, p.polynomial_size // 2), dtype=np.complex128)
    data = bytearray(S.serialize_server_key(p, ksk, fb))
    off = 8 + ksk.size * 8 + 8 * 3 + 24 + 4
    struct.pack_into("<Q", data, off + 8, 2 ** 62)
    with pytest.raises(Exception, match="polynomial size"):
        S.inspect_server_key(bytes(data))


def test_server_key_round_trip_and_layout():
    p = PARAM_MESSAGE_2_CARRY_2_KS_PBS.with_(lwe_dimension=3)
    M = p.polynomial_size // 2
    rng = np.random.default_rng(2)
    ksk = rng.integers(0, 2 ** 64, p.big_lwe_dimension * p.ks_level * (p.lwe_dimension + 1), dtype=np.uint64)
    fb = rng.standard_normal((3 * 4, M)) + 1j * rng.standard_normal((3 * 4, M))
    data = S.serialize_server_key(p, ksk, fb, max_noise_level=9)
    info = S.inspect_server_key(data)
    assert (info.lwe_dimension, info.polynomial_size, info.max_noise_level, info.max_degree) == (3, 2048, 9, 15)
    # hand check of the FourierPolynomialList framing (fft64/math/fft/mod.rs:610-626)
    off = 8 + ksk.size * 8 + 8 * 3 + 24 + 4
    assert struct.unpack_from("<QQQQ", data, off) == (2 + 12, 2048, 12, M)
    assert struct.unpack_from("<dd", data, off + 32) == (fb[0, 0].real, fb[0, 0].imag)
    ksk4 = np.zeros(p.big_lwe_dimension * p.ks_level * 5, dtype=np.uint64)
    with pytest.raises(Exception, match="input_lwe_dimension 4 but 3 GGSWs"):
        S.inspect_server_key(S.serialize_server_key(p.with_(lwe_dimension=4), ksk4, fb))


@pytest.mark.parametrize("N", [2048, 4096, 8192, 16384, 32768])
def test_engine_frequency_matches_oracle_position_order(orc, N):
    """freq[e] = pos_freq(position of engine element e): the layout DESIGN.md 2 documents,
    against the oracle's digit-reversal map of its FFT plan."""
    e = np.arange(N // 2)
    lane, s, blk = e % 64, (e // 64) % 16, e // 1024
    pos = 1024 * blk + 64 * (lane & 15) + 16 * (lane >> 4) + s
    assert np.array_equal(S.engine_frequency(N).astype(np.int64), orc.pos_freq(N)[pos])
    with pytest.raises(Exception, match="supports"):
        S.engine_frequency(128)


@pytest.mark.parametrize("N", [256, 512, 1024])
def test_small_n_engine_frequency_matches_oracle_position_order(orc, N):
    """N <= 1024 (WaveFft<128> / <256> / <512>, fft_device.h): element e of the engine layout holds
    FFT position P(e), whose frequency is the oracle's digit reversal of the plan."""
    e = np.arange(N // 2)
    lane, s = e % 64, e // 64
    if N == 1024:    # [8, 8, 8]: lane L, slot s <-> 64 (L & 7) + 8 (L >> 3) + s
        pos = 64 * (lane & 7) + 8 * (lane >> 3) + s
    elif N == 512:   # [16, 16]: lane L, slot q <-> 16 (L & 15) + (L >> 4) + 4 q
        pos = 16 * (lane & 15) + (lane >> 4) + 4 * s
    else:            # [16, 8]: natural = Fourier layout
        pos = e
    f = S.engine_frequency(N).astype(np.int64)
    assert np.array_equal(np.sort(f), e)
    assert np.array_equal(f, orc.pos_freq(N)[pos])
