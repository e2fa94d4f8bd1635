"""Gadget layer (fork tfhe/src/gadget): host logic and the oracle-backed DAG.

CPU tests: encodings and accumulator builders against the reference's rules (restated below with
file:line), the packing keyswitch / GLWE-product oracles, and end-to-end gadget evaluation, MVB
and tree bootstrapping at MANTICORE_PARAMETERS through OracleEngine (the oracle behind the
Engine's host API), checked by decryption.  The reference's own gadget tests are copies of the
boolean tests, so there are no gadget golden vectors: parity of these paths is
"unpinned" beyond the oracle restatement.
"""
import numpy as np
import pytest

from conftest import OracleEngine


# ---- encodings (gadget/ciphertext/mod.rs) ----------------------------------------------------
def test_encoding_constructors_and_validity():
    from tfhe_mi355.gadget import Encoding

    e = Encoding.new_canonical(3, [0, 2, 4], 7)
    assert e.is_canonical() and e.get_modulus() == 7 and e.get_origin_modulus() == 3
    assert e.inverse_encoding(4) == 2 and e.inverse_encoding(1) is None
    assert Encoding.parity_encoding() == Encoding.new_canonical_binary(1, 2)
    t = Encoding.new_trivial(5)
    assert [t.get_part_single_value_if_canonical(i) for i in range(5)] == list(range(5))
    assert t.negative_on_p_ring(2) == 3 and t.negative_on_o_ring(0) == 0
    # even p: negacyclicity (x + p/2 may only lie in part -i)
    Encoding(2, [[0], [1]], 4)                      # 0+2=2, 1+2=3: free
    with pytest.raises(ValueError):
        Encoding(2, [[0], [2]], 4)                  # opposite of 0 (=2) lies in part 1 != -0
    w = Encoding.new_all_one_wopbs(4)               # wopbs encodings skip the check
    assert w.wopbs and not Encoding.new_trivial(3).wopbs


def test_encoding_transformations():
    from tfhe_mi355.gadget import Encoding

    e = Encoding.new_canonical(3, [0, 1, 2], 5)
    assert e.add_constant(4) == Encoding.new_canonical(3, [4, 0, 1], 5)
    assert e.multiply_encoding_by_constant(3) == Encoding.new_canonical(3, [0, 3, 1], 5)
    # apply_lut_to_encoding: part j = union of parts i with f(i) = j (ciphertext/mod.rs:217-247)
    g = e.apply_lut_to_encoding(lambda x: 0 if x < 2 else 1)
    assert g.get_part(0) == {0, 1} and g.get_part(1) == {2} and g.get_part(2) == set()


def test_create_accumulator_odd_p():
    from tfhe_mi355.gadget import Encoding, create_accumulator

    enc_in = Encoding.new_trivial(5)
    enc_out = Encoding.new_canonical(5, [0, 3, 1, 4, 2], 5)
    acc = create_accumulator(enc_in, enc_out)
    # k even -> value k/2 encoded out; k odd -> negative of the value (p+1)/2 + (k-1)/2
    exp = []
    for k in range(5):
        if k % 2 == 0:
            exp.append([0, 3, 1, 4, 2][k // 2])
        else:
            exp.append((5 - [0, 3, 1, 4, 2][3 + (k - 1) // 2]) % 5)
    assert acc == exp


def test_fill_lookup_table_windows():
    from tfhe_mi355.gadget import Encoding, create_accumulator, fill_lookup_table
    from tfhe_mi355.parameters import MANTICORE_PARAMETERS as P

    N, p = P.polynomial_size, 5
    enc = Encoding.new_trivial(p)
    lut = fill_lookup_table(P, enc, enc)
    assert not lut[:N].any()                        # mask zero
    body = lut[N:]
    data = create_accumulator(enc, enc)
    unit = (1 << 64) // p
    half = N // (2 * p)
    # windows [half + (k-1)N/p, half + kN/p): N/p products computed before the division
    for k in range(1, p):
        lo, hi = half + (k - 1) * N // p, half + k * N // p
        assert (body[lo:hi] == np.uint64(unit * data[k])).all()
    assert (body[:half] == np.uint64(unit * data[0])).all()
    assert (body[N - half:] == np.uint64(unit * ((p - data[0]) % p))).all()
    gap = slice(half + (p - 1) * N // p, N - half)   # untouched by the reference: zero here
    assert not body[gap].any()


def test_fill_lookup_table_binary_and_common_factor():
    from tfhe_mi355.gadget import Encoding, fill_common_factor_lookup_table, fill_lookup_table
    from tfhe_mi355.parameters import MANTICORE_PARAMETERS as P

    N = P.polynomial_size
    # p = 2: the output must be negacyclic (false = -true); window 0 holds the image of the part
    # containing 0 (bootstrapping.rs:186-205)
    lut = fill_lookup_table(P, Encoding.parity_encoding(), Encoding.new_canonical(2, [1, 2], 3))
    body = lut[N:]
    unit = (1 << 64) // 3
    assert (body[:N // 2] == np.uint64(unit * 1)).all() and (body[N // 2:] == np.uint64(unit * 2)).all()
    lut = fill_lookup_table(P, Encoding(2, [[1], [0]], 2), Encoding.new_canonical(2, [1, 2], 3))
    assert (lut[N:N + N // 2] == np.uint64(unit * 2)).all()
    cf = fill_common_factor_lookup_table(P, Encoding.new_trivial(5))
    assert (cf[N:] == np.uint64((1 << 64) // 5)).all()
    cf = fill_common_factor_lookup_table(P, Encoding.new_canonical_binary(1, 4))
    assert (cf[N:] == np.uint64((1 << 63) // 4)).all()


def test_mvb_vi_and_pack_windows():
    from tfhe_mi355.gadget import Encoding, create_vi_for_mvb, pack_window_polys

    N, p = 1024, 5
    enc = Encoding.new_trivial(p)
    v = create_vi_for_mvb(N, enc, enc)
    nz = np.nonzero(v)[0]
    assert set(nz) <= {N // (2 * p) + i * N // p for i in range(p)}
    w = pack_window_polys(N, p)
    s = N // p
    assert (w[0, :s // 2] == 1).all() and (w[0, N - s // 2:] == np.uint64((1 << 64) - 1)).all()
    # every coefficient used by at most one element, the windows tile [0, p*s) minus a tail
    used = (w != 0).sum(axis=0)
    assert used.max() == 1 and used.sum() == (p - 1) * s + 2 * (s // 2)


# ---- oracle kernels ----------------------------------------------------------------------------
def test_packing_key_client_decrypts(orc):
    """Client (product) packing KSK: block (i, level) decrypts to in_sk[i] * 2^(64 - base_log*lvl)
    on the constant coefficient (levels stored L..1), ~0 elsewhere."""
    from tfhe_mi355 import client

    k, N, in_dim, bl, lv = 1, 256, 12, 4, 3
    in_sk = orc.binary_key(5, 1, in_dim)
    glwe_sk = orc.binary_key(5, 2, k * N)
    key = client.gen_packing_keyswitch_key(77, in_sk, glwe_sk, k, N, bl, lv, 2.0 ** -50)
    key = key.reshape(in_dim, lv, (k + 1) * N)
    for i in range(in_dim):
        for l in range(lv):
            body = _glwe_decrypt(key[i, l], glwe_sk, k, N)
            body[:1] -= np.uint64((int(in_sk[i]) << (64 - bl * (lv - l))) % (1 << 64))
            assert np.all(np.minimum(body, np.uint64(0) - body) < np.uint64(2 ** 20))


def _glwe_decrypt(glwe, glwe_sk, k, N):
    from oracle.oracle import negacyclic_mul

    body = glwe[k * N:].copy()
    for p in range(k):
        body -= negacyclic_mul(glwe[p * N:(p + 1) * N], glwe_sk[p * N:(p + 1) * N])
    return body


def test_packing_keyswitch_decrypts(orc):
    k, N, bl, lv = 1, 256, 4, 3
    big = orc.binary_key(9, 2, k * N)          # input LWE key (kN)
    glwe_sk = orc.binary_key(9, 3, k * N)
    pksk = orc.gen_pksk(11, big, glwe_sk, k, N, bl, lv, 2.0 ** -45)
    msgs = np.array([3 << 60, 7 << 59, 0, (1 << 64) - (5 << 58)], dtype=np.uint64)
    cts = orc.lwe_encrypt(12, big, msgs, 2.0 ** -45)
    out = orc.packing_keyswitch(pksk, k * N, k, N, bl, lv, cts)
    for c, m in zip(out, msgs):
        body = _glwe_decrypt(c, glwe_sk, k, N)
        err = (int(body[0]) - int(m)) % (1 << 64)
        err = err - (1 << 64) if err >= 1 << 63 else err
        # decomposition rounding: sum of ~N/2 terms < 2^51 each -> ~2^54
        assert abs(err) < 2 ** 57
        assert np.all(np.minimum(body[1:], np.uint64(0) - body[1:]) < np.uint64(2 ** 57))


def test_glwe_poly_mul_oracle_matches_schoolbook(orc):
    rng = np.random.default_rng(3)
    k, N = 2, 64
    g = rng.integers(0, 2 ** 63, size=(2, 3, (k + 1) * N), dtype=np.uint64) * np.uint64(2)
    v = np.zeros((2, 3, N), dtype=np.uint64)
    v[0, 0, 5] = 1
    v[0, 2, 63] = (1 << 64) - 1
    v[1] = rng.integers(0, 7, size=(3, N), dtype=np.uint64)
    out = orc.glwe_poly_mul(k, N, g, v, extract=False)
    for c in range(2):
        for i in range(2):
            exp = np.zeros((k + 1) * N, dtype=np.uint64)
            for j in range(3):
                for p in range(k + 1):
                    exp[p * N:(p + 1) * N] += orc.negacyclic_mul(g[c, j, p * N:(p + 1) * N], v[i, j])
            assert np.array_equal(out[c, i], exp)
    ext = orc.glwe_poly_mul(k, N, g, v, extract=True)
    full = out[1, 1]
    assert ext[1, 1][0] == full[0] and int(ext[1, 1][1]) == (-int(full[N - 1])) % (1 << 64)
    assert ext[1, 1][N] == full[N] and ext[1, 1][-1] == full[k * N]


# ---- end to end at MANTICORE through the oracle engine ---------------------------------------
@pytest.fixture(scope="module")
def gadget_cpu(orc):
    from tfhe_mi355 import gadget
    from tfhe_mi355.parameters import MANTICORE_PARAMETERS as P

    ck = gadget.ClientKey(P, seed=21)
    sk = gadget.ServerKey(ck, engine=OracleEngine(P))
    return gadget, ck, sk


def test_gadget_apply_lut_cpu(gadget_cpu):
    gadget, ck, sk = gadget_cpu
    enc = gadget.Encoding.new_trivial(5)
    cts = ck.encrypt_arithmetic_many(list(range(5)), enc)
    assert ck.decrypt_many(cts) == list(range(5))
    out_enc = gadget.Encoding.new_canonical(5, [0, 2, 4, 1, 3], 5)
    res = sk.apply_lut_batch(cts, out_enc, lambda x: (x * x) % 5)
    assert ck.decrypt_many(res) == [(x * x) % 5 for x in range(5)]


def test_gadget_boolean_and_cpu(gadget_cpu):
    """BPR24 AND gate: inputs encoded 0/1 in Z_5 (q = 1, 2), their sum decides the output."""
    gadget, ck, sk = gadget_cpu
    g = gadget.Gadget.new_canonical([1, 2], 1, 5, 5, 2, lambda b: b[0] & b[1])
    g.test_full(ck, sk)


def test_gadget_mvb_cpu(gadget_cpu):
    gadget, ck, sk = gadget_cpu
    enc = gadget.Encoding.new_trivial(5)
    cts = ck.encrypt_arithmetic_many(list(range(5)), enc)
    fis = [lambda x: (x + 1) % 5, lambda x: (2 * x) % 5, lambda x: x]
    outs = sk.mvb_batch(cts, [enc] * 3, fis)
    for x, row in enumerate(outs):
        assert ck.decrypt_many(row) == [f(x) for f in fis]


def test_gadget_tree_bootstrapping_cpu(gadget_cpu):
    gadget, ck, sk = gadget_cpu
    o = 3
    enc_in = gadget.Encoding.new_canonical(o, [0, 1, 2], 7)
    enc_out = gadget.Encoding.new_trivial(o)
    t = o * o
    f = lambda x: (5 * x + 2) % t  # noqa: E731
    pairs = [(x0, x1) for x0 in range(o) for x1 in range(o)]
    inputs = [[ck.encrypt_arithmetic(x0, enc_in), ck.encrypt_arithmetic(x1, enc_in)] for x0, x1 in pairs]
    res = sk.full_tree_bootstrapping_batch(inputs, [enc_out, enc_out], t, f)
    for (x0, x1), (r1, r0) in zip(pairs, res):
        X = x1 + o * x0
        assert ck.decrypt(r0) == f(X) % o and ck.decrypt(r1) == f(X) // o, (x0, x1)


@pytest.mark.parametrize("name", ["GADGET_ZAMA_TRIVIUM_PARAMETERS", "GADGET_SIMON_PARAMETERS_40"])
def test_gadget_apply_lut_gadget_params_cpu(orc, name):
    """k = 3, N = 512 sets through the oracle engine: Small key (PBS -> KS) and Big key (KS -> PBS)."""
    from tfhe_mi355 import gadget
    from tfhe_mi355.parameters import ALL

    P = ALL[name]
    ck = gadget.ClientKey(P, seed=4)
    sk = gadget.ServerKey(ck, engine=OracleEngine(P))
    enc = gadget.Encoding.new_trivial(3)
    cts = ck.encrypt_arithmetic_many([0, 1, 2, 2, 1], enc)
    res = sk.apply_lut_batch(cts, enc, lambda x: (x + 1) % 3)
    assert ck.decrypt_many(res) == [1, 2, 0, 0, 2]
