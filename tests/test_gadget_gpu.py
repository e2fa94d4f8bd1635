"""GPU parity of the gadget layer's kernels against the oracle.

Bar: bit-exact u64 outputs for the blind rotation without sample extraction, the LWE -> GLWE
packing keyswitch (MFMA and scalar kernels), the GLWE x polynomial products, and the complete
gadget evaluations (apply_lut, BPR24 gadget, MVB, depth-2 tree bootstrapping) run once on the
engine and once on OracleEngine from the same client key.
"""
import numpy as np
import pytest

from conftest import OracleEngine

pytestmark = pytest.mark.gpu


def _rand(rng, shape):
    return rng.integers(0, 2 ** 63, size=shape, dtype=np.uint64) * np.uint64(2) + rng.integers(
        0, 2, size=shape, dtype=np.uint64)


@pytest.mark.parametrize("which", ["2_2", "manticore"])
def test_blind_rotate_bit_exact(orc, which, request):
    from tfhe_mi355 import Engine

    keys = request.getfixturevalue(f"keys_{which}")
    p = keys.params
    eng = Engine(p, 0)
    eng.upload_bootstrap_key(keys.bsk)
    N = p.polynomial_size
    rng = np.random.default_rng(17)
    cts = rng.integers(0, 2 ** 64, (40, p.lwe_dimension + 1), dtype=np.uint64)
    luts = _rand(rng, (3, (p.glwe_dimension + 1) * N))   # non-trivial (GLWE) accumulators
    idx = (np.arange(40) % 3).astype(np.uint32)
    exp = keys.fbsk.blind_rotate(cts, luts, idx, threads=8)
    got = eng.blind_rotate(cts, luts, idx)
    assert np.array_equal(got, exp), f"{np.count_nonzero(got != exp)} words differ"
    # sample extraction of the rotated accumulator = the PBS output
    pbs = eng.programmable_bootstrap(cts, luts, idx)
    ext = orc.glwe_poly_mul(p.glwe_dimension, N, got, np.eye(1, N, dtype=np.uint64), extract=True)[:, 0]
    assert np.array_equal(ext, pbs)


@pytest.mark.parametrize("mfma", [True, False])
def test_packing_keyswitch_bit_exact(orc, keys_manticore, mfma, monkeypatch):
    from tfhe_mi355 import Engine

    p = keys_manticore.params
    k, N = p.glwe_dimension, p.polynomial_size
    if not mfma:
        monkeypatch.setenv("TFHE_MI355_KS_NO_MFMA", "1")
    eng = Engine(p, 0)
    pksk = orc.gen_pksk(31, keys_manticore.glwe_sk, keys_manticore.glwe_sk, k, N, p.ks_base_log, p.ks_level,
                        p.glwe_modular_std_dev)
    eng.upload_packing_keyswitch_key(pksk, p.ks_base_log, p.ks_level)
    rng = np.random.default_rng(5)
    x = rng.integers(0, 2 ** 64, (67, k * N + 1), dtype=np.uint64)
    x[3] = 0
    x[4, :] = np.uint64(1 << 63)
    exp = orc.packing_keyswitch(pksk, k * N, k, N, p.ks_base_log, p.ks_level, x)
    got = eng.packing_keyswitch(x)
    assert np.array_equal(got, exp), f"{np.count_nonzero(got != exp)} words differ"


@pytest.mark.parametrize("which", ["2_2", "manticore"])
def test_glwe_poly_mul_bit_exact(orc, which, request):
    from tfhe_mi355 import Engine
    from tfhe_mi355.gadget import Encoding, create_vi_for_mvb, pack_window_polys

    p = request.getfixturevalue(f"params_{which}") if which == "2_2" else request.getfixturevalue(
        "keys_manticore").params
    k, N = p.glwe_dimension, p.polynomial_size
    eng = Engine(p, 0)
    rng = np.random.default_rng(9)
    # MVB shape: one GLWE per item, sparse v_i, extraction
    g = _rand(rng, (33, 1, (k + 1) * N))
    vis = np.stack([create_vi_for_mvb(N, Encoding.new_trivial(q), Encoding.new_trivial(q)) for q in (3, 5, 7, 17)])
    for extract in (True, False):
        exp = orc.glwe_poly_mul(k, N, g, vis[:, None], extract)
        got = eng.glwe_poly_mul(g, vis[:, None], extract)
        assert np.array_equal(got, exp), f"mvb extract={extract}: {np.count_nonzero(got != exp)} differ"
    # packing shape: p GLWEs per item, window polys (N nonzeros in total), no extraction
    q = 7
    g = _rand(rng, (5, q, (k + 1) * N))
    w = pack_window_polys(N, q)[None]
    assert np.array_equal(eng.glwe_poly_mul(g, w, False), orc.glwe_poly_mul(k, N, g, w, False))
    # dense random polynomials (more nonzeros than one LDS window)
    g = _rand(rng, (3, 2, (k + 1) * N))
    v = _rand(rng, (2, 2, N))
    for extract in (True, False):
        assert np.array_equal(eng.glwe_poly_mul(g, v, extract), orc.glwe_poly_mul(k, N, g, v, extract))


def test_glwe_poly_mul_large_n(orc):
    """N = 32768 (output tiles loop 32x per item)."""
    from tfhe_mi355 import Engine
    from tfhe_mi355.parameters import PARAM_MESSAGE_4_CARRY_4_KS_PBS as p

    k, N = p.glwe_dimension, p.polynomial_size
    eng = Engine(p, 0)
    rng = np.random.default_rng(4)
    g = _rand(rng, (2, 1, (k + 1) * N))
    v = np.zeros((2, 1, N), dtype=np.uint64)
    v[0, 0, [0, 17, N - 1]] = [1, 5, (1 << 64) - 3]
    v[1, 0, ::4096] = 3
    for extract in (True, False):
        assert np.array_equal(eng.glwe_poly_mul(g, v, extract), orc.glwe_poly_mul(k, N, g, v, extract))


# ---- whole gadget evaluations: engine vs oracle engine, same keys ---------------------------
@pytest.fixture(scope="module")
def gadget_pair(orc):
    from tfhe_mi355 import gadget
    from tfhe_mi355.parameters import MANTICORE_PARAMETERS as P

    ck = gadget.ClientKey(P, seed=33)
    gpu = gadget.ServerKey(ck, device=0)
    cpu = gadget.ServerKey(ck, engine=OracleEngine(P))
    return gadget, ck, gpu, cpu


def _same(a, b):
    return all(np.array_equal(x.ct, y.ct) and x.encoding == y.encoding for x, y in zip(a, b))


def test_gadget_apply_lut_and_gadget_bit_exact(gadget_pair):
    gadget, ck, gpu, cpu = gadget_pair
    enc = gadget.Encoding.new_trivial(7)
    cts = ck.encrypt_arithmetic_many([x % 7 for x in range(64)], enc)
    f = lambda x: (3 * x * x + 1) % 7  # noqa: E731
    a = gpu.apply_lut_batch(cts, enc, f)
    b = cpu.apply_lut_batch(cts, enc, f)
    assert _same(a, b)
    assert ck.decrypt_many(a) == [f(x % 7) for x in range(64)]
    g = gadget.Gadget.new_canonical([1, 2, 4], 1, 11, 11, 3, lambda bits: bits[0] ^ (bits[1] & bits[2]))
    g.test_full(ck, gpu)
    bits = [gadget.split_int_in_booleans(x, 3, False) for x in range(8)]
    ins = [[ck.encrypt_arithmetic(b, g.encodings_in[i]) for i, b in enumerate(bb)] for bb in bits]
    assert _same(g.exec_batch(ins, gpu), g.exec_batch(ins, cpu))


def test_gadget_mvb_bit_exact(gadget_pair):
    gadget, ck, gpu, cpu = gadget_pair
    enc = gadget.Encoding.new_trivial(5)
    cts = ck.encrypt_arithmetic_many([x % 5 for x in range(20)], enc)
    fis = [lambda x: (x + 1) % 5, lambda x: (2 * x) % 5, lambda x: (x * x) % 5, lambda x: 4 - x]
    a = gpu.mvb_batch(cts, [enc] * 4, fis)
    b = cpu.mvb_batch(cts, [enc] * 4, fis)
    assert all(_same(x, y) for x, y in zip(a, b))
    for x, row in enumerate(a):
        assert ck.decrypt_many(row) == [f(x % 5) for f in fis]


def test_gadget_tree_bootstrapping_bit_exact(gadget_pair):
    gadget, ck, gpu, cpu = gadget_pair
    o = 3
    enc_in = gadget.Encoding.new_canonical(o, [0, 1, 2], 7)
    enc_out = gadget.Encoding.new_trivial(o)
    t = o * o
    f = lambda x: (4 * x + 7) % t  # noqa: E731
    pairs = [(x0, x1) for x0 in range(o) for x1 in range(o)]
    inputs = [[ck.encrypt_arithmetic(x0, enc_in), ck.encrypt_arithmetic(x1, enc_in)] for x0, x1 in pairs]
    a = gpu.full_tree_bootstrapping_batch(inputs, [enc_out, enc_out], t, f)
    b = cpu.full_tree_bootstrapping_batch(inputs, [enc_out, enc_out], t, f)
    assert all(_same(x, y) for x, y in zip(a, b))
    for (x0, x1), (r1, r0) in zip(pairs, a):
        X = x1 + o * x0
        assert ck.decrypt(r0) == f(X) % o and ck.decrypt(r1) == f(X) // o
