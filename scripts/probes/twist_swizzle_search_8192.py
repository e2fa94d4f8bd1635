"""Bank-conflict cost of an LDS twist-table layout for the N = 8192 multi-bit paired sub-block
kernel (large_mb_pair2_kernel, csrc/pbs_large.hip): a monomial read of lane l fetches entry
r = t mod M of t = d (1 - 4 f) mod 2N, M = 4096, f = q + 4 (freq_lane(l) + freq_slot(s)) for
sub-block q < 4 and slot s < 16; ds_read_b64 serves 32-lane groups, bank pair = position mod 32.
Cost = mean over sampled d, q, s of the largest number of distinct entries on one bank.
Searches the two-instruction family position = r ^ ((r >> k) & m).
usage: python twist_swizzle_search_8192.py [n_d_samples]"""
import sys

import numpy as np

M, N2 = 4096, 16384
rng = np.random.default_rng(0)
nd = int(sys.argv[1]) if len(sys.argv) > 1 else 256
d = np.concatenate([np.arange(1, 65), rng.integers(0, N2 // 2 + 1, nd)])[:, None, None, None]
q = np.arange(4)[None, :, None, None]
s = np.arange(16)[None, None, :, None]
lane = np.arange(64)[None, None, None, :]
fl = (lane & 15) + 64 * (lane >> 4)
f = q + 4 * (fl + 16 * (s >> 2) + 256 * (s & 3))
t = (d * (1 - 4 * f)) % N2
r = t % M


def cost(p):
    tot, worst = 0.0, 0
    for g in range(2):
        a = r[..., 32 * g:32 * g + 32]
        pp = p[..., 32 * g:32 * g + 32]
        key = (pp % 32) * M + a
        ks = np.sort(key, axis=-1)
        uniq = np.concatenate([np.ones(ks.shape[:-1] + (1,), bool), ks[..., 1:] != ks[..., :-1]], axis=-1)
        ub = np.where(uniq, ks // M, -1)
        cnt = np.stack([(ub == b).sum(axis=-1) for b in range(32)], axis=-1)
        m = cnt.max(axis=-1)
        tot += m.mean()
        worst = max(worst, int(m.max()))
    return tot / 2, worst


print("plain", cost(r), flush=True)
best = []
for k in range(1, 12):
    for m in range(1, 1 << min(12 - k, 10)):
        if m >> (12 - k):
            continue
        c = cost(r ^ ((r >> k) & m))
        best.append((c, k, m))
best.sort()
for c, k, m in best[:10]:
    print("k", k, "m", m, c, flush=True)
