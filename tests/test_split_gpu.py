"""GPU parity tests of the split CMUX (N = 4096 ... 32768, pbs_large.hip) and of every shortint
parameter set of the reference (shortint/parameters/mod.rs:598-1201).

The split CMUX runs the oracle's [R | 16, 16, 4] FFT DAG (R = N / 2048) with the accumulator in
device scratch: top radix-R stage, 1024-point sub-block FFTs + MAC, top inverse stage.  The bar is
bit-exact u64 outputs against the oracle on the same inputs (and decryption round trips), at
reduced LWE dimension n so that the oracle finishes in seconds; the full 3_3 shape (n = 864) is
checked through KS -> PBS decryptions plus two bit-exact ciphertexts.

Keys come from the engine's client-side keygen (exact FFT negacyclic products) and are fed to both
sides as standard u64 keys.
"""
import numpy as np
import pytest

from conftest import decode

pytestmark = pytest.mark.gpu


def _keys(orc, p, seed):
    from tfhe_mi355 import client

    lwe_sk = client.gen_binary_key(seed, 1, p.lwe_dimension)
    glwe_sk = client.gen_binary_key(seed, 2, p.big_lwe_dimension)
    bsk = client.gen_bootstrap_key(seed + 1, lwe_sk, glwe_sk, p.glwe_dimension, p.polynomial_size, p.pbs_base_log,
                                   p.pbs_level, p.glwe_modular_std_dev)
    fbsk = orc.FourierBsk(bsk, p.lwe_dimension, p.glwe_dimension, p.polynomial_size, p.pbs_base_log, p.pbs_level)
    return lwe_sk, glwe_sk, bsk, fbsk


def _engine(p, bsk, ksk=None):
    from tfhe_mi355 import Engine

    e = Engine(p, 0)
    e.upload_bootstrap_key(bsk)
    if ksk is not None:
        e.upload_keyswitch_key(ksk)
    return e


def _device_to_host(ptr, nbytes):
    import ctypes

    import torch  # noqa: F401  (loads libamdhip64)

    hip = ctypes.CDLL("libamdhip64.so")
    out = np.empty(nbytes // 8, dtype=np.uint64)
    assert hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes), 2) == 0
    return out


def _cus():
    """Compute units of device 0: the CMUX form thresholds of capi.cpp scale with it."""
    import torch

    return torch.cuda.get_device_properties(0).multi_processor_count


def _ran(eng, f):
    """f()'s result and the kernel families it launched (the engine's kernel timer)."""
    eng.kernel_timing(1)
    out = f()
    ran = set(eng.kernel_times())
    eng.kernel_timing(0)
    return out, ran


def engine_position(N):
    """FFT position of each engine-layout spectrum element: sub-block q = e // 1024 holds
    positions 1024 q + the WaveFft<1024> layout."""
    e = np.arange(N // 2)
    lane, s, blk = e % 64, (e // 64) % 16, e // 1024
    return 1024 * blk + 64 * (lane & 15) + 16 * (lane >> 4) + s


SPLIT = ["PARAM_MESSAGE_1_CARRY_4_KS_PBS",   # N = 4096,  L = 2, base 2^15
         "PARAM_MESSAGE_2_CARRY_3_KS_PBS",   # N = 4096,  L = 1, base 2^22
         "PARAM_MESSAGE_3_CARRY_3_KS_PBS",   # N = 8192,  L = 2
         "PARAM_MESSAGE_6_CARRY_0_KS_PBS",   # N = 8192,  L = 1, base 2^22
         "PARAM_MESSAGE_1_CARRY_6_KS_PBS",   # N = 16384, L = 3, base 2^11 (33 decomposed bits)
         "PARAM_MESSAGE_2_CARRY_5_KS_PBS",   # N = 16384, L = 2
         "PARAM_MESSAGE_1_CARRY_7_KS_PBS"]   # N = 32768, L = 3 (the generic path, not the grouped one)


@pytest.mark.parametrize("N", [4096, 8192, 16384])
def test_split_fourier_bsk_bit_exact_vs_oracle(orc, N):
    from tfhe_mi355 import client
    from tfhe_mi355.parameters import SHORTINT_ALL

    p = next(q for q in SHORTINT_ALL.values() if q.polynomial_size == N).with_(lwe_dimension=2)
    lwe_sk = client.gen_binary_key(3, 1, 2)
    glwe_sk = client.gen_binary_key(3, 2, N)
    bsk = client.gen_bootstrap_key(4, lwe_sk, glwe_sk, 1, N, p.pbs_base_log, p.pbs_level, p.glwe_modular_std_dev)
    eng = _engine(p, bsk)
    ptr, nbytes = eng.fourier_bootstrap_key()
    got = _device_to_host(ptr, nbytes).view(np.complex128).reshape(-1, N // 2)
    exp = orc.FourierBsk(bsk, 2, 1, N, p.pbs_base_log, p.pbs_level).fourier().reshape(-1, N // 2)
    exp = np.ascontiguousarray(exp[:, engine_position(N)])
    exp = np.ldexp(exp.view(np.float64), -int(np.log2(N // 2))).view(np.complex128)  # the resident 1/M
    bad = np.count_nonzero(got.view(np.uint64) != exp.view(np.uint64))
    assert bad == 0, f"{bad} of {got.size * 2} doubles differ; max |diff| {np.max(np.abs(got - exp))}"


@pytest.mark.parametrize("name", SPLIT)
def test_split_pbs_bit_exact_vs_oracle(orc, name):
    """Per-ciphertext LUTs, 8-bit-wide message spaces, edge inputs (b~ = 2N, every a~ = 0, a~ = N,
    alternating all-ones masks): bit-exact against the oracle's PBS at n = 6."""
    from tfhe_mi355.parameters import SHORTINT_ALL

    p = SHORTINT_ALL[name].with_(lwe_dimension=6)
    N, space = p.polynomial_size, p.message_modulus * p.carry_modulus
    lwe_sk, glwe_sk, bsk, fbsk = _keys(orc, p, 51)
    eng = _engine(p, bsk)
    fs = [lambda x: x, lambda x: (3 * x + 1) % space]
    luts = np.stack([orc.fill_accumulator(N, 1, p.message_modulus, p.carry_modulus, f) for f in fs])
    msgs = np.array([0, 1, space // 2, space - 1, 5 % space, 7 % space])
    idx = np.array([0, 1, 1, 0, 1, 0])
    cts = orc.lwe_encrypt(61, lwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta), p.lwe_modular_std_dev)
    edge = np.random.default_rng(9).integers(0, 2 ** 64, (4, p.lwe_dimension + 1), dtype=np.uint64)
    edge[0, -1] = np.uint64((1 << 64) - 1)
    edge[1, :-1] = 0
    edge[2, :-1] = np.uint64(1 << 63)
    edge[3, ::2] = np.uint64((1 << 64) - 1)
    allc = np.concatenate([cts, edge])
    alli = np.concatenate([idx, [0, 1, 0, 1]]).astype(np.uint32)
    got = eng.programmable_bootstrap(allc, luts, lut_indexes=alli)
    exp = fbsk.pbs(allc, luts, lut_idx=alli, threads=8)
    bad = np.nonzero(np.any(got != exp, axis=1))[0]
    assert bad.size == 0, f"{name}: ciphertexts {bad} differ ({np.count_nonzero(got != exp)} words)"
    dec = decode(orc.lwe_decrypt(glwe_sk, got[:6]), p.delta) % space
    assert np.array_equal(dec, [fs[i](m) for i, m in zip(idx, msgs)])


def test_split_pbs_chunks_ragged(orc):
    """More ciphertexts than one pass of the split CMUX holds (TFHE_MI355_LARGE_CHUNK is not set:
    the chunk follows from the scratch given): 3 passes of 64 + a ragged 17 through the async entry
    with a deliberately small scratch; every output equals the one-pass host call."""
    import torch

    from tfhe_mi355.parameters import PARAM_MESSAGE_3_CARRY_3_KS_PBS

    p = PARAM_MESSAGE_3_CARRY_3_KS_PBS.with_(lwe_dimension=4)
    lwe_sk, glwe_sk, bsk, fbsk = _keys(orc, p, 71)
    eng = _engine(p, bsk)
    msgs = np.random.default_rng(3).integers(0, 64, 209)
    cts = orc.lwe_encrypt(72, lwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta), p.lwe_modular_std_dev)
    acc = orc.fill_accumulator(p.polynomial_size, 1, 8, 8, lambda x: (x * 5 + 3) % 64)
    ref = eng.programmable_bootstrap(cts, acc)
    dev = torch.device("cuda", 0)
    per = eng.pbs_scratch_bytes(1)
    d_in = torch.from_numpy(cts.view(np.int64)).to(dev)
    d_out = torch.zeros((209, p.big_lwe_dimension + 1), dtype=torch.int64, device=dev)
    d_lut = torch.from_numpy(acc.view(np.int64)).to(dev)
    scratch = torch.empty(per * 64, dtype=torch.uint8, device=dev)
    eng.programmable_bootstrap_async(d_in, d_out, d_lut, 1, 209, d_scratch=scratch)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(np.uint64)
    assert np.array_equal(got, ref)
    assert np.array_equal(decode(orc.lwe_decrypt(glwe_sk, got), p.delta) % 64, (msgs * 5 + 3) % 64)
    sample = np.array([0, 63, 64, 200, 208])
    assert np.array_equal(got[sample], fbsk.pbs(cts[sample], acc, threads=5))


@pytest.mark.parametrize("name", ["PARAM_MESSAGE_3_CARRY_3_KS_PBS",    # N = 8192, L = 2, base 2^15
                                  "PARAM_MESSAGE_6_CARRY_0_KS_PBS",    # N = 8192, L = 1, base 2^22
                                  "PARAM_MESSAGE_1_CARRY_4_KS_PBS",    # N = 4096, L = 2 (two ciphertexts per workgroup)
                                  "PARAM_MESSAGE_2_CARRY_3_KS_PBS"])   # N = 4096, L = 1
def test_onchip_and_split_cmux_agree(orc, name):
    """N = 8192 and 4096, L = 2 and 1: one call of C ciphertexts runs the on-chip CMUX (onchip_cmux_kernel;
    capi.cpp onchip_min: >= 96 rows at N = 8192, >= 160 at N = 4096 on 256 CUs; at N = 4096 two
    ciphertexts per workgroup, the odd count leaving a padding slot), the same ciphertexts in two calls
    below the threshold the split CMUX (digits-fed at L = 2, three launches at L = 1) or, at most
    CUs / R rows, the quad / duo CMUX; every row
    identical, a sample bit-exact against the oracle, edge masks and per-ciphertext LUTs included."""
    from tfhe_mi355.parameters import SHORTINT_ALL

    p = SHORTINT_ALL[name].with_(lwe_dimension=6)
    space = p.message_modulus * p.carry_modulus
    lwe_sk, glwe_sk, bsk, fbsk = _keys(orc, p, 77)
    eng = _engine(p, bsk)
    cus = _cus()
    on_min = cus * 3 // 8 if p.polynomial_size == 8192 else cus * 5 // 8  # capi.cpp onchip_min
    C = on_min + 35
    h = C // 2
    quad = h <= cus // (p.polynomial_size // 2048)  # capi.cpp quad_max (quad / duo, L = 1 and 2)
    msgs = np.random.default_rng(5).integers(0, space, C)
    cts = orc.lwe_encrypt(78, lwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta), p.lwe_modular_std_dev)
    cts[0, :-1] = 0                                   # every a~ = 0
    cts[1, :-1] = np.uint64(1 << 63)                  # a~ = N
    cts[2, -1] = np.uint64((1 << 64) - 1)             # b~ = 2N
    fs = [lambda x: (x * 7 + 2) % space, lambda x: (x + space // 2 + 1) % space]
    luts = np.stack([orc.fill_accumulator(p.polynomial_size, 1, p.message_modulus, p.carry_modulus, f) for f in fs])
    idx = (np.arange(C) % 3 == 1).astype(np.uint32)  # per-ciphertext LUTs
    whole, ran = _ran(eng, lambda: eng.programmable_bootstrap(cts, luts, lut_indexes=idx))
    assert "onchip_cmux_kernel" in ran, ran
    halves = []
    for a, b in ((0, h), (h, C)):
        out, ran = _ran(eng, lambda: eng.programmable_bootstrap(cts[a:b], luts, lut_indexes=idx[a:b]))
        assert "onchip_cmux_kernel" not in ran and ("quad_cmux_kernel" in ran) == quad, ran
        halves.append(out)
    halves = np.concatenate(halves)
    assert np.array_equal(whole, halves), f"{np.count_nonzero(np.any(whole != halves, axis=1))} rows differ"
    sample = np.array([0, 1, 2, h - 1, h, C - 1])
    assert np.array_equal(whole[sample], fbsk.pbs(cts[sample], luts, lut_idx=idx[sample], threads=6))
    dec = decode(orc.lwe_decrypt(glwe_sk, whole[3:]), p.delta) % space
    assert np.array_equal(dec, [fs[i](m) for i, m in zip(idx[3:], msgs[3:])])


@pytest.mark.parametrize("name", ["PARAM_MESSAGE_3_CARRY_3_KS_PBS", "PARAM_MESSAGE_2_CARRY_4_KS_PBS",
                                  "PARAM_MESSAGE_1_CARRY_4_KS_PBS", "PARAM_MESSAGE_6_CARRY_0_KS_PBS",
                                  "PARAM_MESSAGE_2_CARRY_3_KS_PBS"])
def test_quad_onchip_and_split_cmux_agree(orc, name):
    """N = 8192 and 4096, L = 2 and 1: the same ciphertexts through the three CMUX forms -- one call above
    the on-chip threshold (on-chip CMUX, one ciphertext per CU), calls of 1, 7 and CUs/R - 12 (quad /
    duo CMUX: R = N / 2048 workgroups per ciphertext exchanging their sub-blocks every CMUX; capi.cpp
    quad_max = CUs / R) and one call of the rest (split CMUX, between the quad and the on-chip ranges),
    the kernel of each call checked by the engine's kernel timer -- every row identical, a sample
    bit-exact against the oracle, edge masks and per-ciphertext LUTs included."""
    from tfhe_mi355.parameters import SHORTINT_ALL

    p = SHORTINT_ALL[name].with_(lwe_dimension=6)
    space = p.message_modulus * p.carry_modulus
    lwe_sk, glwe_sk, bsk, fbsk = _keys(orc, p, 79)
    eng = _engine(p, bsk)
    cus = _cus()
    R = p.polynomial_size // 2048
    Q, O = cus // R, cus * (5 if R == 2 else 3) // 8  # capi.cpp quad_max, onchip_min
    C = max(O + 35, Q - 4 + (Q + O) // 2)  # the last call (Q - 4 .. C) lands between Q and O
    msgs = np.random.default_rng(8).integers(0, space, C)
    cts = orc.lwe_encrypt(80, lwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta), p.lwe_modular_std_dev)
    cts[0, :-1] = 0                                   # every a~ = 0
    cts[1, :-1] = np.uint64(1 << 63)                  # a~ = N
    cts[2, -1] = np.uint64((1 << 64) - 1)             # b~ = 2N
    cts[3, ::2] = np.uint64((1 << 64) - 1)
    fs = [lambda x: (x * 5 + 1) % space, lambda x: (space - 1 - x) % space]
    luts = np.stack([orc.fill_accumulator(p.polynomial_size, 1, p.message_modulus, p.carry_modulus, f) for f in fs])
    idx = (np.arange(C) % 3 == 2).astype(np.uint32)
    whole, ran = _ran(eng, lambda: eng.programmable_bootstrap(cts, luts, lut_indexes=idx))
    assert "onchip_cmux_kernel" in ran, ran
    parts = []
    split = "large_dsub_kernel" if p.pbs_level == 2 else "large_sub_kernel"  # digits-fed at L = 2
    for a, b, kern in ((0, 1, "quad_cmux_kernel"), (1, 8, "quad_cmux_kernel"), (8, Q - 4, "quad_cmux_kernel"),
                       (Q - 4, C, split)):
        assert 0 < b - a <= Q if kern.startswith("quad") else Q < b - a < O
        out, ran = _ran(eng, lambda: eng.programmable_bootstrap(cts[a:b], luts, lut_indexes=idx[a:b]))
        assert kern in ran and "onchip_cmux_kernel" not in ran, (a, b, ran)
        parts.append(out)
    got = np.concatenate(parts)
    assert np.array_equal(whole, got), f"{np.count_nonzero(np.any(whole != got, axis=1))} rows differ"
    sample = np.array([0, 1, 2, 3, 7, 8, Q - 5, Q - 4, C - 1])
    assert np.array_equal(whole[sample], fbsk.pbs(cts[sample], luts, lut_idx=idx[sample], threads=9))
    dec = decode(orc.lwe_decrypt(glwe_sk, whole[4:]), p.delta) % space
    assert np.array_equal(dec, [fs[i](m) for i, m in zip(idx[4:], msgs[4:])])
    # the async entry with scratch for 5 ciphertexts: quad passes of 5, 5, 2 (pbs_large.hip launch_quad)
    import torch

    dev = torch.device("cuda", 0)
    n = 12
    ref = eng.programmable_bootstrap(cts[:n], luts[0])
    d_in = torch.from_numpy(cts[:n].view(np.int64)).to(dev)
    d_out = torch.zeros((n, p.big_lwe_dimension + 1), dtype=torch.int64, device=dev)
    d_lut = torch.from_numpy(luts[0].view(np.int64)).to(dev)
    scratch = torch.empty(eng.pbs_scratch_bytes(1) * 5, dtype=torch.uint8, device=dev)

    def run_async():
        eng.programmable_bootstrap_async(d_in, d_out, d_lut, 1, n, d_scratch=scratch)
        torch.cuda.synchronize()

    _, ran = _ran(eng, run_async)
    assert "quad_cmux_kernel" in ran, ran
    assert np.array_equal(d_out.cpu().numpy().view(np.uint64), ref)


@pytest.mark.timeout(900)
def test_full_3_3_keyswitch_pbs(orc):
    """Full PARAM_MESSAGE_3_CARRY_3_KS_PBS (n = 864, N = 8192, L = 2; the reference's 121 ms
    KS+PBS set, benchmarks.md:42): KS -> PBS decrypts to f(m); two ciphertexts bit-exact."""
    from tfhe_mi355 import client
    from tfhe_mi355.parameters import PARAM_MESSAGE_3_CARRY_3_KS_PBS as P

    lwe_sk, glwe_sk, bsk, fbsk = _keys(orc, P, 81)
    ksk = client.gen_keyswitch_key(83, glwe_sk, lwe_sk, P.ks_base_log, P.ks_level, P.lwe_modular_std_dev)
    eng = _engine(P, bsk, ksk)
    msgs = np.array([0, 5, 17, 33, 63, 40, 9, 50])
    big = orc.lwe_encrypt(84, glwe_sk, msgs.astype(np.uint64) * np.uint64(P.delta), P.glwe_modular_std_dev)
    acc = orc.fill_accumulator(P.polynomial_size, 1, 8, 8, lambda x: (x + 11) % 64)
    out = eng.keyswitch_programmable_bootstrap(big, acc)
    assert np.array_equal(decode(orc.lwe_decrypt(glwe_sk, out), P.delta) % 64, (msgs + 11) % 64)
    small = orc.keyswitch(ksk, P.big_lwe_dimension, P.lwe_dimension, P.ks_base_log, P.ks_level, big[:2])
    assert np.array_equal(out[:2], fbsk.pbs(small, acc, threads=2))


def _all_sets():
    from tfhe_mi355.parameters import SHORTINT_ALL

    return sorted(SHORTINT_ALL)


@pytest.mark.parametrize("name", _all_sets())
def test_every_shortint_parameter_set_bit_exact(orc, name):
    """Every shortint ClassicPBSParameters set of the reference creates a context, and its keyswitch
    and PBS (KS -> PBS for the Big-key sets, PBS -> KS for the Small-key ones) are bit-exact
    against the oracle at n = 4, outputs decrypting to f(m)."""
    from tfhe_mi355 import client
    from tfhe_mi355.parameters import SHORTINT_ALL

    p = SHORTINT_ALL[name].with_(lwe_dimension=4)
    N, k, space = p.polynomial_size, p.glwe_dimension, p.message_modulus * p.carry_modulus
    lwe_sk, glwe_sk, bsk, fbsk = _keys(orc, p, 91)
    ksk = client.gen_keyswitch_key(92, glwe_sk, lwe_sk, p.ks_base_log, p.ks_level, p.lwe_modular_std_dev)
    eng = _engine(p, bsk, ksk)
    f = lambda x: (x * 3 + 1) % space  # noqa: E731
    acc = orc.fill_accumulator(N, k, p.message_modulus, p.carry_modulus, f)
    msgs = np.arange(4) * max(1, space // 4) % space
    if p.encryption_key_choice == "Big":
        big = orc.lwe_encrypt(93, glwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta), p.glwe_modular_std_dev)
        small = orc.keyswitch(ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log, p.ks_level, big)
        assert np.array_equal(eng.keyswitch(big), small), "keyswitch differs from the oracle"
        out = eng.keyswitch_programmable_bootstrap(big, acc)
        assert np.array_equal(out, fbsk.pbs(small, acc, threads=4)), "KS -> PBS differs from the oracle"
        dec = decode(orc.lwe_decrypt(glwe_sk, out), p.delta) % space
    else:
        small = orc.lwe_encrypt(93, lwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta), p.lwe_modular_std_dev)
        big = fbsk.pbs(small, acc, threads=4)
        out = eng.programmable_bootstrap_keyswitch(small, acc)
        exp = orc.keyswitch(ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log, p.ks_level, big)
        assert np.array_equal(out, exp), "PBS -> KS differs from the oracle"
        dec = decode(orc.lwe_decrypt(lwe_sk, out), p.delta) % space
    assert np.array_equal(dec, [f(m) for m in msgs])


MB_SPLIT = ["PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_2_KS_PBS",   # N = 8192, L = 2, g = 2 (multi_bit.rs:134)
            "PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_3_KS_PBS"]   # N = 8192, L = 2, g = 3 (multi_bit.rs:192)


@pytest.mark.parametrize("name", MB_SPLIT)
def test_split_multi_bit_pbs_bit_exact_vs_oracle(orc, name):
    """Multi-bit PBS through the split CMUX (keybundle built inside large_sub_kernel from the
    2^g - 1 resident GGSWs of each group): KS -> PBS bit-exact against the oracle's
    MultiBitFourierBsk at n = 6 (both groupings divide it), per-ciphertext LUTs, edge inputs,
    outputs decrypting to f(m)."""
    from tfhe_mi355 import client
    from tfhe_mi355.parameters import MULTI_BIT_ALL

    p = MULTI_BIT_ALL[name].with_(lwe_dimension=6)
    N, g, space = p.polynomial_size, p.grouping_factor, p.message_modulus * p.carry_modulus
    lwe_sk = client.gen_binary_key(101, 1, p.lwe_dimension)
    glwe_sk = client.gen_binary_key(101, 2, p.big_lwe_dimension)
    bsk = client.gen_multi_bit_bootstrap_key(102, lwe_sk, glwe_sk, 1, N, p.pbs_base_log, p.pbs_level, g,
                                             p.glwe_modular_std_dev, threads=8)
    fb = orc.MultiBitFourierBsk(bsk, p.lwe_dimension, 1, N, p.pbs_base_log, p.pbs_level, g)
    ksk = client.gen_keyswitch_key(103, glwe_sk, lwe_sk, p.ks_base_log, p.ks_level, p.lwe_modular_std_dev)
    eng = _engine(p, bsk, ksk)
    fs = [lambda x: (x + 7) % space, lambda x: (5 * x) % space]
    luts = np.stack([orc.fill_accumulator(N, 1, p.message_modulus, p.carry_modulus, f) for f in fs])
    msgs = np.array([0, 1, 31, 63, 40, 17])
    idx = np.array([0, 1, 0, 1, 1, 0], dtype=np.uint32)
    big = orc.lwe_encrypt(104, glwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta), p.glwe_modular_std_dev)
    small = orc.keyswitch(ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log, p.ks_level, big)
    out = eng.keyswitch_programmable_bootstrap(big, luts, lut_indexes=idx)
    exp = fb.pbs(small, luts, lut_idx=idx, threads=6)
    bad = np.nonzero(np.any(out != exp, axis=1))[0]
    assert bad.size == 0, f"{name}: ciphertexts {bad} differ"
    assert np.array_equal(decode(orc.lwe_decrypt(glwe_sk, out), p.delta) % space,
                          [fs[i](m) for i, m in zip(idx, msgs)])
    edge = np.random.default_rng(11).integers(0, 2 ** 64, (3, p.lwe_dimension + 1), dtype=np.uint64)
    edge[0, :-1] = 0
    edge[1, :-1] = np.uint64(1 << 63)
    edge[2, -1] = np.uint64((1 << 64) - 1)
    assert np.array_equal(eng.programmable_bootstrap(edge, luts[0]), fb.pbs(edge, luts[0], threads=3))


@pytest.mark.parametrize("name", MB_SPLIT)
def test_onchip_and_split_multi_bit_agree(orc, name):
    """Multi-bit N = 8192: a 130-ciphertext call (one chunk of the split CMUX with a
    partial pair) and the same ciphertexts in calls of 65 (odd counts: a pair workgroup with an idle
    slot) and in 47-ciphertext passes through the async entry; every row identical, a sample bit-exact
    against the oracle.  (Round 5 also ran it against
    the measured-slower multi-bit on-chip CMUX: profiles/r05_onchip_mb_tests.log.)"""
    from tfhe_mi355 import client
    from tfhe_mi355.parameters import MULTI_BIT_ALL

    p = MULTI_BIT_ALL[name].with_(lwe_dimension=6)
    N, g = p.polynomial_size, p.grouping_factor
    lwe_sk = client.gen_binary_key(121, 1, p.lwe_dimension)
    glwe_sk = client.gen_binary_key(121, 2, p.big_lwe_dimension)
    bsk = client.gen_multi_bit_bootstrap_key(122, lwe_sk, glwe_sk, 1, N, p.pbs_base_log, p.pbs_level, g,
                                             p.glwe_modular_std_dev, threads=8)
    fb = orc.MultiBitFourierBsk(bsk, p.lwe_dimension, 1, N, p.pbs_base_log, p.pbs_level, g)
    eng = _engine(p, bsk)
    msgs = np.random.default_rng(6).integers(0, 64, 130)
    cts = orc.lwe_encrypt(123, lwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta), p.lwe_modular_std_dev)
    cts[0, :-1] = 0
    cts[1, :-1] = np.uint64(1 << 63)
    cts[2, -1] = np.uint64((1 << 64) - 1)
    acc = orc.fill_accumulator(N, 1, 8, 8, lambda x: (x * 5 + 1) % 64)
    whole = eng.programmable_bootstrap(cts, acc)
    halves = np.concatenate([eng.programmable_bootstrap(cts[:65], acc), eng.programmable_bootstrap(cts[65:], acc)])
    assert np.array_equal(whole, halves), f"{np.count_nonzero(np.any(whole != halves, axis=1))} rows differ"
    # several passes of the split CMUX: the async entry with scratch for 47 ciphertexts (chunks of
    # 47, 47, 36: odd chunks end on a half-used pair workgroup)
    import torch

    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(cts.view(np.int64)).to(dev)
    d_out = torch.zeros((130, p.big_lwe_dimension + 1), dtype=torch.int64, device=dev)
    d_lut = torch.from_numpy(acc.view(np.int64)).to(dev)
    scratch = torch.empty(eng.pbs_scratch_bytes(1) * 47, dtype=torch.uint8, device=dev)
    eng.programmable_bootstrap_async(d_in, d_out, d_lut, 1, 130, d_scratch=scratch)
    torch.cuda.synchronize()
    assert np.array_equal(d_out.cpu().numpy().view(np.uint64), whole)
    sample = np.array([0, 1, 2, 64, 129])
    assert np.array_equal(whole[sample], fb.pbs(cts[sample], acc, threads=5))
    assert np.array_equal(decode(orc.lwe_decrypt(glwe_sk, whole[3:]), p.delta) % 64, (msgs[3:] * 5 + 1) % 64)


@pytest.mark.timeout(900)
def test_full_multi_bit_3_3_group_3_decrypts(orc):
    """Full PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_3_KS_PBS (n = 972, N = 8192): KS -> PBS of 64
    ciphertexts decrypts to f(m); one ciphertext bit-exact against the oracle."""
    from tfhe_mi355 import client
    from tfhe_mi355.parameters import PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_3_KS_PBS as P

    lwe_sk = client.gen_binary_key(111, 1, P.lwe_dimension)
    glwe_sk = client.gen_binary_key(111, 2, P.big_lwe_dimension)
    bsk = client.gen_multi_bit_bootstrap_key(112, lwe_sk, glwe_sk, 1, P.polynomial_size, P.pbs_base_log,
                                             P.pbs_level, 3, P.glwe_modular_std_dev, threads=16)
    ksk = client.gen_keyswitch_key(113, glwe_sk, lwe_sk, P.ks_base_log, P.ks_level, P.lwe_modular_std_dev)
    eng = _engine(P, bsk, ksk)
    msgs = np.random.default_rng(5).integers(0, 64, 64)
    big = orc.lwe_encrypt(114, glwe_sk, msgs.astype(np.uint64) * np.uint64(P.delta), P.glwe_modular_std_dev)
    acc = orc.fill_accumulator(P.polynomial_size, 1, 8, 8, lambda x: (x * 3 + 2) % 64)
    out = eng.keyswitch_programmable_bootstrap(big, acc)
    assert np.array_equal(decode(orc.lwe_decrypt(glwe_sk, out), P.delta) % 64, (msgs * 3 + 2) % 64)
    fb = orc.MultiBitFourierBsk(bsk, P.lwe_dimension, 1, P.polynomial_size, P.pbs_base_log, P.pbs_level, 3)
    small = orc.keyswitch(ksk, P.big_lwe_dimension, P.lwe_dimension, P.ks_base_log, P.ks_level, big[:1])
    assert np.array_equal(out[:1], fb.pbs(small, acc, threads=1))
