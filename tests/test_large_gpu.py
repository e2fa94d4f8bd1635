"""GPU parity tests for the N = 32768 PBS (PARAM_MESSAGE_4_CARRY_4_KS_PBS, BASELINE config 3):
the HIP engine through its C ABI against the oracle (same FFT DAG, [16,16,16,4]) on the same inputs.

Keys come from the engine's client-side keygen (exact FFT negacyclic products; the oracle's
schoolbook keygen is too slow at N = 32768) and are fed to both sides as standard u64 keys.
Bar: bit-exact u64 outputs; decryption round trips.
"""
import numpy as np
import pytest

from conftest import decode

pytestmark = pytest.mark.gpu


class LargeKeys:
    def __init__(self, orc, params, seed):
        from tfhe_mi355 import client

        p = self.params = params
        self.lwe_sk = client.gen_binary_key(seed, 1, p.lwe_dimension)
        self.glwe_sk = client.gen_binary_key(seed, 2, p.big_lwe_dimension)
        self.bsk = client.gen_bootstrap_key(seed + 1, self.lwe_sk, self.glwe_sk, 1, p.polynomial_size,
                                            p.pbs_base_log, p.pbs_level, p.glwe_modular_std_dev)
        self.fbsk = orc.FourierBsk(self.bsk, p.lwe_dimension, 1, p.polynomial_size, p.pbs_base_log, p.pbs_level)

    def encrypt(self, orc, msgs, seed):
        p = self.params
        return orc.lwe_encrypt(seed, self.lwe_sk, np.asarray(msgs, dtype=np.uint64) * np.uint64(p.delta),
                               p.lwe_modular_std_dev)


@pytest.fixture(scope="module")
def small_n_4_4(orc):
    """4_4 at N = 32768, L = 2, base 2^15 with a short LWE (n = 24): full-size FFTs and external
    products, few CMUXes, so the oracle finishes in seconds."""
    from tfhe_mi355 import Engine
    from tfhe_mi355.parameters import PARAM_MESSAGE_4_CARRY_4_KS_PBS

    keys = LargeKeys(orc, PARAM_MESSAGE_4_CARRY_4_KS_PBS.with_(lwe_dimension=24), 31)
    eng = Engine(keys.params, 0)
    eng.upload_bootstrap_key(keys.bsk)
    return keys, eng


def _device_to_host(ptr, nbytes):
    import ctypes

    import torch  # noqa: F401  (loads libamdhip64)

    hip = ctypes.CDLL("libamdhip64.so")
    out = np.empty(nbytes // 8, dtype=np.uint64)
    assert hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes), 2) == 0
    return out


def engine_position(N):
    """FFT position of each engine-layout spectrum element (fft_device.h WaveFft<1024>; at
    N = 32768 sub-block c' = 2 wave + h holds positions 1024 c' + [0, 1024))."""
    e = np.arange(N // 2)
    lane, s = e % 64, (e // 64) % 16
    blk = e // 1024
    return 1024 * blk + 64 * (lane & 15) + 16 * (lane >> 4) + s


@pytest.mark.parametrize("N", [2048, 32768])
def test_fourier_bsk_bit_exact_vs_oracle(orc, N):
    """The GPU standard->Fourier BSK conversion (forward_as_torus, fft/mod.rs:197-218) equals the
    oracle's transform element for element, in the engine's position layout."""
    from tfhe_mi355 import Engine, client
    from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS, PARAM_MESSAGE_4_CARRY_4_KS_PBS

    p = (PARAM_MESSAGE_2_CARRY_2_KS_PBS if N == 2048 else PARAM_MESSAGE_4_CARRY_4_KS_PBS).with_(lwe_dimension=2)
    lwe_sk = client.gen_binary_key(3, 1, 2)
    glwe_sk = client.gen_binary_key(3, 2, N)
    bsk = client.gen_bootstrap_key(4, lwe_sk, glwe_sk, 1, N, p.pbs_base_log, p.pbs_level, p.glwe_modular_std_dev)
    eng = Engine(p, 0)
    eng.upload_bootstrap_key(bsk)
    ptr, nbytes = eng.fourier_bootstrap_key()
    got = _device_to_host(ptr, nbytes).view(np.complex128).reshape(-1, N // 2)
    exp = orc.FourierBsk(bsk, 2, 1, N, p.pbs_base_log, p.pbs_level).fourier().reshape(-1, N // 2)
    exp = np.ascontiguousarray(exp[:, engine_position(N)])
    # the resident key carries the backward 1/M (fft_device.h fourier_key_scale): an exact
    # power-of-two scale of the reference transform
    exp = np.ldexp(exp.view(np.float64), -int(np.log2(N // 2))).view(np.complex128)
    diff = got.view(np.uint64) != exp.view(np.uint64)
    bad = np.count_nonzero(diff)
    where = np.nonzero(diff.reshape(got.shape[0], -1)[0])[0][:8] // 2
    assert bad == 0, (f"{bad} of {got.size * 2} doubles differ; max |diff| {np.max(np.abs(got - exp))}; "
                      f"first positions {engine_position(N)[where]} got {got[0, where]} exp {exp[0, where]}")


def test_large_pbs_single_cmux_bit_exact(orc):
    from tfhe_mi355 import Engine
    from tfhe_mi355.parameters import PARAM_MESSAGE_4_CARRY_4_KS_PBS

    keys = LargeKeys(orc, PARAM_MESSAGE_4_CARRY_4_KS_PBS.with_(lwe_dimension=1), 33)
    eng = Engine(keys.params, 0)
    eng.upload_bootstrap_key(keys.bsk)
    cts = keys.encrypt(orc, [3, 100], 305)
    acc = orc.fill_accumulator(32768, 1, 16, 16, lambda x: x)
    got = eng.programmable_bootstrap(cts, acc)
    exp = keys.fbsk.pbs(cts, acc, threads=2)
    bad = np.nonzero(got[0] != exp[0])[0]
    assert bad.size == 0, f"{bad.size} words differ, first at {bad[:8]}; diffs {(got[0][bad[:8]] - exp[0][bad[:8]]).view(np.int64)}"


def test_large_pbs_bit_exact_vs_oracle(orc, small_n_4_4):
    keys, eng = small_n_4_4
    p = keys.params
    N = p.polynomial_size
    fs = [lambda x: x, lambda x: (x * 7 + 3) % 256]
    luts = np.stack([orc.fill_accumulator(N, 1, 16, 16, f) for f in fs])
    msgs = np.array([0, 1, 77, 128, 200, 255])
    idx = np.array([0, 1, 1, 0, 1, 0])
    cts = keys.encrypt(orc, msgs, 301)
    exp = keys.fbsk.pbs(cts, luts, lut_idx=idx, threads=6)
    got = eng.programmable_bootstrap(cts, luts, lut_indexes=idx)
    assert got.shape == exp.shape == (6, N + 1)
    assert np.array_equal(got, exp), f"{np.count_nonzero(got != exp)} words differ"


def test_large_pbs_edge_inputs_bit_exact(orc, small_n_4_4):
    keys, eng = small_n_4_4
    n, N = keys.params.lwe_dimension, keys.params.polynomial_size
    rng = np.random.default_rng(9)
    cts = rng.integers(0, 2 ** 64, (4, n + 1), dtype=np.uint64)
    cts[0, n] = np.uint64((1 << 64) - 1)  # b~ = 2N
    cts[1, :n] = 0                        # every CMUX skipped
    cts[2, :n] = np.uint64(1 << 63)       # a~ = N
    cts[3, ::2] = np.uint64((1 << 64) - 1)
    acc = orc.fill_accumulator(N, 1, 16, 16, lambda x: 255 - x)
    assert np.array_equal(eng.programmable_bootstrap(cts, acc), keys.fbsk.pbs(cts, acc, threads=4))


@pytest.mark.timeout(900)
def test_full_4_4_pbs_and_keyswitch(orc):
    """Full PARAM_MESSAGE_4_CARRY_4_KS_PBS (n = 996): KS -> PBS decrypts to f(m) for a spread of
    8-bit messages; two ciphertexts checked bit-exactly against the oracle."""
    from tfhe_mi355 import Engine, client
    from tfhe_mi355.parameters import PARAM_MESSAGE_4_CARRY_4_KS_PBS as P

    keys = LargeKeys(orc, P, 41)
    ksk = client.gen_keyswitch_key(43, keys.glwe_sk, keys.lwe_sk, P.ks_base_log, P.ks_level, P.lwe_modular_std_dev)
    eng = Engine(P, 0)
    eng.upload_bootstrap_key(keys.bsk)
    eng.upload_keyswitch_key(ksk)
    msgs = np.array([0, 5, 99, 160, 255, 31, 64, 200])
    big = orc.lwe_encrypt(302, keys.glwe_sk, msgs.astype(np.uint64) * np.uint64(P.delta), P.glwe_modular_std_dev)
    acc = orc.fill_accumulator(P.polynomial_size, 1, 16, 16, lambda x: (x + 17) % 256)
    small = eng.keyswitch(big)
    assert np.array_equal(small[:2], orc.keyswitch(ksk, P.big_lwe_dimension, P.lwe_dimension, P.ks_base_log,
                                                   P.ks_level, big[:2]))
    out = eng.programmable_bootstrap(small, acc)
    dec = decode(orc.lwe_decrypt(keys.glwe_sk, out), P.delta) % 256
    assert np.array_equal(dec, (msgs + 17) % 256)
    assert np.array_equal(out[:2], keys.fbsk.pbs(small[:2], acc, threads=2))
    both = eng.keyswitch_programmable_bootstrap(big, acc)
    assert np.array_equal(both, out)


def test_large_pbs_two_chunks_ragged(orc, small_n_4_4):
    """200 ciphertexts: two passes of the chunked N = 32768 CMUX (128 + a ragged 72, not a multiple
    of the 8-XCD block grouping); every output decrypts, a sample from each chunk is bit-exact."""
    keys, eng = small_n_4_4
    p = keys.params
    N = p.polynomial_size
    msgs = np.random.default_rng(21).integers(0, 256, 200)
    cts = keys.encrypt(orc, msgs, 321)
    acc = orc.fill_accumulator(N, 1, 16, 16, lambda x: (x * 5 + 1) % 256)
    got = eng.programmable_bootstrap(cts, acc)
    dec = decode(orc.lwe_decrypt(keys.glwe_sk, got), p.delta) % 256
    assert np.array_equal(dec, (msgs * 5 + 1) % 256)
    # one sample per sub-block rotation of the group kernel (rotation (cl / 8) mod 4: 0, 1, 2, 3)
    sample = np.array([0, 40, 80, 127, 128, 199])
    assert np.array_equal(got[sample], keys.fbsk.pbs(cts[sample], acc, threads=6))


@pytest.mark.parametrize("mask", ["interleave", "block"])
def test_large_pbs_cu_lanes_bit_exact(orc, small_n_4_4, mask, monkeypatch):
    """The grouped N = 32768 CMUX on two CU-masked lanes (TFHE_MI355_LANES_MCUS: group kernels of one
    chunk beside the streaming kernels of another): 220 ciphertexts in lane chunks of
    24 (four full pairs, then a pair whose second chunk holds 4) -- identical to
    the one-stream context row for row, every output decrypting, a sample bit-exact vs the oracle."""
    from tfhe_mi355 import Engine

    keys, single = small_n_4_4
    p = keys.params
    N = p.polynomial_size
    monkeypatch.setenv("TFHE_MI355_LANES_MCUS", "8")
    monkeypatch.setenv("TFHE_MI355_LANES_CHUNK", "24")
    monkeypatch.setenv("TFHE_MI355_LANES_MASK", mask)
    lanes = Engine(p, 0)
    lanes.upload_bootstrap_key(keys.bsk)
    msgs = np.random.default_rng(23).integers(0, 256, 220)
    cts = keys.encrypt(orc, msgs, 323)
    fs = [lambda x: (x * 3 + 5) % 256, lambda x: 255 - x]
    luts = np.stack([orc.fill_accumulator(N, 1, 16, 16, f) for f in fs])
    idx = (np.arange(220) % 2).astype(np.uint32)
    got = lanes.programmable_bootstrap(cts, luts, lut_indexes=idx)
    assert np.array_equal(got, single.programmable_bootstrap(cts, luts, lut_indexes=idx))
    dec = decode(orc.lwe_decrypt(keys.glwe_sk, got), p.delta) % 256
    assert np.array_equal(dec, np.where(idx == 1, 255 - msgs, (msgs * 3 + 5) % 256))
    sample = np.array([0, 23, 24, 47, 200, 219])
    assert np.array_equal(got[sample], keys.fbsk.pbs(cts[sample], luts, lut_idx=idx[sample], threads=6))
    lanes.close()
