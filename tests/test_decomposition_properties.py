"""Property tests of the signed decomposer the keyswitch and every PBS kernel restate, ported
from the reference's own tests (core_crypto/commons/math/decomposition/tests.rs:14-115) and run
on the oracle's u64 decomposer (oracle/pbs_oracle.c orc_decompose / orc_closest_representable,
restating decomposer.rs:99-153 and iter.rs:134-141):

  * every valid decomposer (base_log * level < 64, tests.rs:14-29);
  * decompose -> recompose gives closest_representable, every term balanced in
    [-2^(base_log-1), 2^(base_log-1)] with levels in iterator order (tests.rs:31-62);
  * closest_representable is stable under +- epsilon = 2^(64 - base_log level - 1) / 2
    (tests.rs:74-100) and idempotent (tests.rs:112-128).

The reference runs 100,000 random inputs spread over the decomposers (divide_ceil(100_000, n));
here the same budget, seeded.  The GPU kernels' 32-bit and 64-bit digit extractions (pbs_common.h,
pbs_large.hip decompose64) are pinned against this decomposer by the bit-exact GPU tests.
"""
import numpy as np


def _valid_decomposers():
    out = []
    for base_log in range(1, 64):
        for level in range(1, 64):
            if base_log * level < 64:
                out.append((base_log, level))
            else:
                break
    return out


def test_decompose_recompose_every_decomposer(orc):
    decs = _valid_decomposers()
    runs = -(-100_000 // len(decs))
    rng = np.random.default_rng(2024)
    for base_log, level in decs:
        half = 1 << (base_log - 1)
        for x in rng.integers(0, 2 ** 64, runs, dtype=np.uint64):
            x = int(x)
            digits = orc.decompose(x, base_log, level)
            assert len(digits) == level
            total = 0
            for idx, d in enumerate(digits):          # term idx has level `level - idx`
                ds = d - (1 << 64) if d >= (1 << 63) else d
                assert -half <= ds <= half, (base_log, level, x, idx, ds)
                total += ds << (64 - base_log * (level - idx))
            assert total % (1 << 64) == orc.closest_representable(x, base_log, level), (base_log, level, x)


def test_closest_representable_stable_and_idempotent(orc):
    decs = _valid_decomposers()
    runs = -(-100_000 // len(decs))
    rng = np.random.default_rng(2025)
    for base_log, level in decs:
        eps = (1 << (64 - base_log * level - 1)) // 2
        for x in rng.integers(0, 2 ** 64, runs, dtype=np.uint64):
            r = orc.closest_representable(int(x), base_log, level)
            assert orc.closest_representable((r + eps) % 2 ** 64, base_log, level) == r
            assert orc.closest_representable((r - eps) % 2 ** 64, base_log, level) == r
            assert orc.closest_representable(r, base_log, level) == r
