"""Seeded (compressed) keys, SURVEY.md 8f row f2: the reference's AES-CTR mask stream and the
seeded-key decompression (oracle/csprng_oracle.c), the client's seeded keygen, CPU only.

Pinning: AES-128 by the FIPS-197 known answers (appendix A.1 key expansion, C.1 cipher) and the
SP 800-38A F.5.1 CTR keystream block.  The stream layout (table index (0,1) start, contiguous
forks, LE u64 words) is restated from concrete-csprng / tfhe-rs sources with file:line in the
oracle; the reference holds no seeded-key fixtures, so beyond AES it is "parity unpinned" and
checked by decryption of decompressed keys.
"""
import numpy as np
import pytest

from conftest import OracleEngine


def test_aes128_fips197_known_answers(orc):
    key = bytes(range(16))
    assert orc.aes128_encrypt(key, bytes.fromhex("00112233445566778899aabbccddeeff")).hex() == \
        "69c4e0d86a7b0430d8cdb78070b4c55a"                                  # FIPS-197 C.1
    rk = orc.aes128_round_keys(bytes.fromhex("2b7e151628aed2a6abf7158809cf4f3c"))
    assert rk[160:].hex() == "d014f9a8c9ee2589e13f0cc8b6630ca6"             # FIPS-197 A.1 w[40..43]
    assert orc.aes128_encrypt(bytes.fromhex("2b7e151628aed2a6abf7158809cf4f3c"),
                              bytes.fromhex("f0f1f2f3f4f5f6f7f8f9fafbfcfdfeff")).hex() == \
        "ec8cdf7398607cb0f2d21675ea9ea1e4"                                  # SP 800-38A F.5.1 block 1


def test_stream_layout(orc):
    """byte g = AES_seed(LE u128 counter g // 16)[g % 16]; mask word w = LE bytes [1 + 8w, 9 + 8w)."""
    seed = 0x0123456789ABCDEF_FEDCBA9876543210
    key = seed.to_bytes(16, "little")
    b = orc.csprng_bytes(seed, 0, 64)
    for a in range(4):
        assert b[16 * a:16 * a + 16] == orc.aes128_encrypt(key, a.to_bytes(16, "little"))
    words = orc.seeded_mask_words(seed, 0, 7)
    for w in range(7):
        assert int(words[w]) == int.from_bytes(b[1 + 8 * w:9 + 8 * w], "little")
    assert np.array_equal(orc.seeded_mask_words(seed, 3, 4), words[3:7])


@pytest.mark.parametrize("seed", [0, 1, (1 << 128) - 1, 0xDEADBEEF << 70])
def test_client_stream_matches_oracle(orc, seed):
    from tfhe_mi355 import client

    for first, count in ((0, 1), (0, 33), (5, 2), (1000, 17)):
        assert np.array_equal(client.csprng_mask_words(seed, first, count), orc.seeded_mask_words(seed, first, count))


def test_seeded_bsk_and_ksk_decompress_and_bootstrap(orc):
    """Client seeded keys -> oracle decompression -> KS -> PBS through the oracle engine decrypts."""
    from tfhe_mi355 import client, fill_accumulator
    from tfhe_mi355.parameters import MANTICORE_PARAMETERS as P0

    P = P0.with_(lwe_dimension=64)
    lwe_sk = client.gen_binary_key(5, 1, P.lwe_dimension)
    glwe_sk = client.gen_binary_key(5, 2, P.big_lwe_dimension)
    cseed = 0x5EED_0000_1111_2222_3333_4444_5555_6666
    bodies = client.gen_seeded_bootstrap_key(9, cseed, lwe_sk, glwe_sk, 1, P.polynomial_size, P.pbs_base_log,
                                             P.pbs_level, P.glwe_modular_std_dev)
    assert bodies.shape == (P.lwe_dimension * P.pbs_level * 2 * P.polynomial_size,)
    bsk = orc.decompress_seeded_bsk(cseed, bodies, P.lwe_dimension, P.pbs_level, 1, P.polynomial_size)
    # the mask rows are the seed's stream, the bodies the given ones
    glwe = 2 * P.polynomial_size
    rows = bsk.reshape(-1, glwe)
    assert np.array_equal(rows[5, :P.polynomial_size], orc.seeded_mask_words(cseed, 5 * P.polynomial_size,
                                                                               P.polynomial_size))
    assert np.array_equal(rows[:, P.polynomial_size:].ravel(), bodies)
    kseed = 0xABCDEF
    kb = client.gen_seeded_keyswitch_key(11, kseed, glwe_sk, lwe_sk, P.ks_base_log, P.ks_level,
                                         P.lwe_modular_std_dev)
    ksk = orc.decompress_seeded_ksk(kseed, kb, P.big_lwe_dimension, P.ks_level, P.lwe_dimension)
    eng = OracleEngine(P)
    eng.upload_bootstrap_key(bsk)
    eng.upload_keyswitch_key(ksk)
    delta = 1 << 61
    msgs = np.arange(8, dtype=np.uint64) % 4
    cts = client.lwe_encrypt(3, glwe_sk, msgs * np.uint64(delta), P.glwe_modular_std_dev)
    out = eng.keyswitch_programmable_bootstrap(cts, fill_accumulator(P, lambda x: (x + 1) % 4))
    dec = client.decode(client.lwe_decrypt(glwe_sk, out), delta) % 4
    assert np.array_equal(dec, (msgs + 1) % 4)
