"""Batched integer radix layer on top of the GPU PBS engine.

Mirror of the reference's radix_parallel multiplication DAG, executed for K independent
operand pairs at once:

  ServerKey.mul_parallelized / mul_assign_parallelized      integer/server_key/radix_parallel/mul.rs:553-590
  ServerKey.unchecked_mul_assign_parallelized               mul.rs:300-414
  ServerKey.unchecked_sum_ciphertexts_vec_parallelized      radix_parallel/add.rs:783-960
  ServerKey.add_assign_parallelized                         add.rs:206-242
  unchecked_add_assign_parallelized_low_latency,
  propagate_single_carry_parallelized_low_latency,
  compute_carry_propagation_parallelized_low_latency,
  compute_prefix_sum_hillis_steele, generate_init_carry_array
                                                            add.rs:487-771
  full_propagate_parallelized / partial_propagate_parallelized
                                                            radix_parallel/mod.rs:88-155
  ServerKey.blockshift                                      radix/scalar_mul.rs:345-355
  shortint unchecked_apply_lookup_table_bivariate_assign    shortint/server_key/bivariate_pbs.rs:69-182

Execution model.  The reference's DAG depends only on block degrees and noise levels, never on
the encrypted values, so K operand pairs with the same input shape follow the same DAG.  A
RadixBatch therefore stores the K ciphertexts as one u64 array [K, blocks, lwe_size] with a single
(degree, noise_level) per block, and every PBS layer of the DAG -- across all terms and all K
pairs -- is handed to the engine as ONE batched keyswitch+PBS launch with per-ciphertext LUT
indexes (the "PBS-DAG scheduler" of SURVEY.md 8f row f1).  Trivial blocks take the reference's
trivial-PBS shortcut (shortint/server_key/mod.rs:763-781).  With the GPU engine the batch stays
resident in HBM between layers (torch tensors for storage; the LWE arithmetic and trivial PBS in
the engine's lwe_ops kernels); with any other engine object (the oracle, in the tests) it is a
numpy array on the host -- same DAG, same bits.

Carry propagation uses the Hillis-Steele branch; the reference selects it whenever
should_hillis_steele_propagation_be_faster (add.rs:44-76) holds, i.e. with >= 16 rayon threads
for 16 blocks.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .shortint import KEYSWITCH_BOOTSTRAP, NOISE_NOMINAL, NOISE_ZERO, LookupTable, ServerKey as ShortintServerKey

OUTPUT_CARRY_NONE, OUTPUT_CARRY_GENERATED, OUTPUT_CARRY_PROPAGATED = 0, 1, 2  # add.rs:13-21


@dataclass
class RadixBatch:
    """K radix ciphertexts with shared block metadata (integer/ciphertext/mod.rs RadixCiphertext)."""

    data: np.ndarray      # [K, blocks, lwe_size] u64
    degree: list          # per block
    noise: list           # per block

    @property
    def count(self) -> int:
        return self.data.shape[0]

    @property
    def num_blocks(self) -> int:
        return self.data.shape[1]

    def clone(self) -> "RadixBatch":
        d = self.data.copy() if isinstance(self.data, np.ndarray) else self.data.clone()
        return RadixBatch(d, list(self.degree), list(self.noise))

    def block_carries_are_empty(self, message_modulus: int) -> bool:
        return all(d < message_modulus for d in self.degree)

    def holds_boolean_value(self) -> bool:
        return self.degree[0] <= 1 and all(d == 0 for d in self.degree[1:])

    def is_trivial_block(self, j: int) -> bool:
        return self.noise[j] == NOISE_ZERO


class _PbsLayer:
    """Collects the independent LUT applications of one DAG layer and runs them in one launch."""

    def __init__(self, sk: "ServerKey"):
        self.sk = sk
        self.reqs = []  # (batch, block, lut)

    def add(self, rb: RadixBatch, j: int, lut: LookupTable):
        self.reqs.append((rb, j, lut))

    def flush(self):
        reqs, self.reqs = self.reqs, []
        if not reqs:
            return
        sk = self.sk
        todo, luts, lut_of = [], [], {}
        for rb, j, lut in reqs:
            if rb.is_trivial_block(j):
                sk._trivial_pbs(rb, j, lut)
                continue
            if id(lut) not in lut_of:
                lut_of[id(lut)] = len(luts)
                luts.append(lut)
            todo.append((rb, j, lut_of[id(lut)]))
        if todo:
            n = sk.ops.pbs_rows([(rb, j, li) for rb, j, li in todo], luts)
            sk.pbs_count += n
            sk.launches += 1
            for rb, j, _ in todo:
                rb.noise[j] = NOISE_NOMINAL
        for rb, j, lut in reqs:
            rb.degree[j] = lut.degree



def _is_gpu_engine(engine) -> bool:
    """A single-device GPU engine: radix batches stay in its HBM between layers (_DeviceOps).  A
    multi-device context (Engine(devices=[...])) takes the host path instead: every layer is ONE
    host-pointer KS+PBS call, which the context splits over its devices -- the reference's one
    process with its rayon pool (radix_parallel/mul.rs:347-407) on the one-process drop-in."""
    from .engine import Engine

    return isinstance(engine, Engine) and not engine.multi_device


class _HostOps:
    """numpy arrays on the host; PBS through the engine's host-pointer API (any engine object
    with keyswitch_programmable_bootstrap, e.g. the oracle's in the tests)."""

    def __init__(self, sk: "ServerKey"):
        self.sk = sk

    def zeros(self, k, b, s):
        return np.zeros((k, b, s), dtype=np.uint64)

    def roll(self, data, shift):
        return np.roll(data, shift, axis=1)

    def to_host(self, data):
        return data

    def from_host(self, data):
        return data

    def copy_block(self, dst, j, src, i):
        dst.data[:, j, :] = src.data[:, i, :]

    def set_trivial(self, rb, j, body):
        rb.data[:, j, :] = 0
        rb.data[:, j, -1] = np.uint64(body)

    def mul_add(self, dst, j, scalar, src, i):
        if scalar != 1:
            dst.data[:, j, :] *= np.uint64(scalar)
        if src is not None:
            dst.data[:, j, :] += src.data[:, i, :]

    def trivial_pbs(self, rb, j, lut):
        p = self.sk.p
        modulus_sup = p.message_modulus * p.carry_modulus
        box = p.polynomial_size // modulus_sup
        body = lut.acc[p.glwe_dimension * p.polynomial_size:]
        value = rb.data[:, j, -1] // np.uint64(p.delta)
        neg = value >= np.uint64(modulus_sup)
        entry = body[((value % np.uint64(modulus_sup)) * np.uint64(box)).astype(np.int64)]
        rb.data[:, j, -1] = np.where(neg, np.uint64(0) - entry, entry)

    def pbs_rows(self, todo, luts):
        K = todo[0][0].count
        x = np.concatenate([rb.data[:, j, :] for rb, j, _ in todo], axis=0)
        idx = np.repeat(np.asarray([li for _, _, li in todo], dtype=np.uint32), K)
        out = self.sk.shortint.engine_ks_pbs(x, np.stack([lut.acc for lut in luts]), idx if len(luts) > 1 else None)
        for q, (rb, j, _) in enumerate(todo):
            rb.data[:, j, :] = out[q * K:(q + 1) * K]
        return x.shape[0]


class _BoundedCache:
    """LRU map of device tables (LUT stacks, index arrays) with at most `cap` entries.  Entries
    touched while a hipGraph is being captured are pinned and never evicted: a captured graph
    keeps reading their device memory on every replay, so freeing them would let the caching
    allocator hand that memory to someone else under the graph."""

    def __init__(self, cap: int, capturing):
        from collections import OrderedDict

        self.cap, self._capturing = cap, capturing
        self._d = OrderedDict()
        self._pinned = {}

    def get(self, key):
        if key in self._pinned:
            return self._pinned[key]
        v = self._d.get(key)
        if v is not None:
            self._d.move_to_end(key)
            if self._capturing():
                self._pinned[key] = self._d.pop(key)
        return v

    def put(self, key, value):
        if self._capturing():
            self._pinned[key] = value
            return
        self._d[key] = value
        self._d.move_to_end(key)
        while len(self._d) > self.cap:
            self._d.popitem(last=False)

    def __len__(self):
        return len(self._d) + len(self._pinned)


class _DeviceOps:
    """torch int64 tensors resident on the engine's GPU between layers; the LWE arithmetic runs in
    the engine's own kernels (lwe_ops.hip), torch only allocates, slices and copies."""

    CACHE_ENTRIES = 256  # distinct layer tables kept on the device (a FheUint32 multiply uses 11)

    def __init__(self, sk: "ServerKey"):
        import torch

        self.torch = torch
        self.sk = sk
        self.eng = sk.shortint.engine
        self.device = torch.device("cuda", self.eng.device)
        capturing = torch.cuda.is_current_stream_capturing
        self._lut_dev = _BoundedCache(self.CACHE_ENTRIES, capturing)
        # LUT stacks and per-row LUT index arrays of the layers seen so far (bounded LRU)
        self._stacks = _BoundedCache(self.CACHE_ENTRIES, capturing)
        self._scratch = None

    def zeros(self, k, b, s):
        return self.torch.zeros((k, b, s), dtype=self.torch.int64, device=self.device)

    def roll(self, data, shift):
        return self.torch.roll(data, shift, dims=1) if shift else data

    def to_host(self, data):
        return data.cpu().numpy().view(np.uint64)

    def from_host(self, data):
        return self.torch.from_numpy(np.ascontiguousarray(data).view(np.int64)).to(self.device)

    def copy_block(self, dst, j, src, i):
        dst.data[:, j, :].copy_(src.data[:, i, :])

    def set_trivial(self, rb, j, body):
        rb.data[:, j, :].zero_()
        rb.data[:, j, -1] = int(np.uint64(body).view(np.int64))

    def _row_ptr(self, rb, j, word=0):
        d = rb.data
        return d.data_ptr() + 8 * (j * d.shape[2] + word), d.shape[1] * d.shape[2]

    def mul_add(self, dst, j, scalar, src, i):
        yp, ys = self._row_ptr(dst, j)
        xp, xs = self._row_ptr(src, i) if src is not None else (None, 0)
        self.eng.lwe_scalar_mul_add_async(yp, xp, scalar, dst.count, dst.data.shape[2], ys, xs)

    def lut(self, lut):
        t = self._lut_dev.get(id(lut))
        if t is None or t[0] is not lut:
            t = (lut, self.from_host(lut.acc))
            self._lut_dev.put(id(lut), t)
        return t[1]

    def trivial_pbs(self, rb, j, lut):
        bp, stride = self._row_ptr(rb, j, rb.data.shape[2] - 1)
        self.eng.trivial_pbs_async(bp, rb.count, stride, self.lut(lut))

    def _layer_tables(self, todo, luts):
        """Device LUT stack and LUT-index array of a layer, uploaded the first time its shape is
        seen: the DAG repeats the same layers for every multiply, so a steady-state multiply does
        no host-to-device copy (nothing stalls the stream between launches, and the whole DAG can
        be captured into one hipGraph)."""
        K = todo[0][0].count
        key = (K, tuple(id(lut) for lut in luts), tuple(li for _, _, li in todo) if len(luts) > 1 else ())
        hit = self._stacks.get(key)
        if hit is None or any(a is not b for a, b in zip(hit[0], luts)):
            d_luts = self.from_host(np.stack([lut.acc for lut in luts]))
            idx = None
            if len(luts) > 1:
                li = np.repeat(np.asarray([li for _, _, li in todo], dtype=np.int32), K)
                idx = self.torch.from_numpy(li).to(self.device)
            hit = (list(luts), d_luts, idx)
            self._stacks.put(key, hit)
        return hit[1], hit[2]

    def pbs_rows(self, todo, luts):
        torch = self.torch
        K = todo[0][0].count
        x = torch.cat([rb.data[:, j, :] for rb, j, _ in todo], dim=0)
        n = x.shape[0]
        d_luts, idx = self._layer_tables(todo, luts)
        out = torch.empty_like(x)
        need = self.eng.ks_pbs_scratch_bytes(n)
        if self._scratch is None or self._scratch.numel() < need:
            self._scratch = torch.empty(need, dtype=torch.uint8, device=self.device)
        self.eng.keyswitch_programmable_bootstrap_async(x, out, d_luts, len(luts), n, self._scratch,
                                                        d_lut_indexes=idx)
        for q, (rb, j, _) in enumerate(todo):
            rb.data[:, j, :].copy_(out[q * K:(q + 1) * K])
        return n


class ServerKey:
    """integer ServerKey (integer/server_key/mod.rs) over a shortint ServerKey with the GPU engine."""

    def __init__(self, shortint_key: ShortintServerKey):
        self.shortint = shortint_key
        p = shortint_key.parameters
        if shortint_key.pbs_order != KEYSWITCH_BOOTSTRAP:
            raise NotImplementedError("integer layer implemented for PBSOrder::KeyswitchBootstrap keys")
        self.p = p
        self.msg = p.message_modulus
        self.carry = p.carry_modulus
        self.lwe_size = p.big_lwe_dimension + 1
        self.pbs_count = 0
        self.launches = 0
        self.ops = _DeviceOps(self) if _is_gpu_engine(shortint_key.engine) else _HostOps(self)
        m = self.msg
        self.lut_message = self.shortint.generate_lookup_table(lambda x: x % m)
        self.lut_carry = self.shortint.generate_lookup_table(lambda x: x // m)
        self.lut_mul_lsb = self.generate_lookup_table_bivariate(lambda x, y: (x * y) % m)
        self.lut_mul_msb = self.generate_lookup_table_bivariate(lambda x, y: (x * y) // m)
        self.lut_gen_carry = self.shortint.generate_lookup_table(
            lambda x: OUTPUT_CARRY_GENERATED if x >= m else OUTPUT_CARRY_NONE)
        self.lut_gen_or_prop = self.shortint.generate_lookup_table(
            lambda x: OUTPUT_CARRY_GENERATED if x >= m else (OUTPUT_CARRY_PROPAGATED if x == m - 1
                                                             else OUTPUT_CARRY_NONE))
        self.lut_prefix = self.generate_lookup_table_bivariate(
            lambda msb, lsb: lsb if msb == OUTPUT_CARRY_PROPAGATED else msb)

    # -- lookup tables -----------------------------------------------------------------------
    def generate_lookup_table_bivariate(self, f) -> LookupTable:
        """generate_lookup_table_bivariate (bivariate_pbs.rs:69-100), left scaling = message modulus."""
        m = self.msg
        return self.shortint.generate_lookup_table(lambda x: f((x // m) % m, (x % m) % m))

    # -- block primitives (shortint) -----------------------------------------------------------
    def _trivial_pbs(self, rb: RadixBatch, j: int, lut: LookupTable):
        """trivial_pbs_assign (shortint/server_key/mod.rs:763-781) for every ciphertext of the batch."""
        self.ops.trivial_pbs(rb, j, lut)

    def _set_trivial(self, rb: RadixBatch, j: int, value: int = 0):
        """create_trivial_assign (shortint server_key create_trivial)."""
        self.ops.set_trivial(rb, j, (value % (self.msg * self.carry)) * self.p.delta)
        rb.degree[j] = value
        rb.noise[j] = NOISE_ZERO

    def _add_block(self, dst: RadixBatch, j: int, src: RadixBatch, i: int):
        """shortint unchecked_add_assign: LWE add, degree and noise level add."""
        self.ops.mul_add(dst, j, 1, src, i)
        dst.degree[j] += src.degree[i]
        dst.noise[j] += src.noise[i]

    def _scalar_mul_block(self, rb: RadixBatch, j: int, s: int):
        self.ops.mul_add(rb, j, s, None, 0)
        rb.degree[j] *= s
        rb.noise[j] *= s

    def _bivariate(self, layer: _PbsLayer, left: RadixBatch, j: int, right: RadixBatch, i: int, lut: LookupTable):
        """unchecked_apply_lookup_table_bivariate_assign (bivariate_pbs.rs:167-182):
        left = left * message_modulus + right, then the LUT (queued on `layer`)."""
        assert right.degree[i] + 1 <= self.msg
        self._scalar_mul_block(left, j, self.msg)
        self._add_block(left, j, right, i)
        layer.add(left, j, lut)

    # -- radix helpers -------------------------------------------------------------------------
    def create_trivial_zero(self, count: int, num_blocks: int) -> RadixBatch:
        return RadixBatch(self.ops.zeros(count, num_blocks, self.lwe_size), [0] * num_blocks,
                          [NOISE_ZERO] * num_blocks)

    def blockshift(self, ct: RadixBatch, shift: int) -> RadixBatch:
        """radix/scalar_mul.rs:345-355: rotate_right(shift), low blocks trivial zeros."""
        res = ct.clone()
        nb = ct.num_blocks
        s = shift % nb if nb else 0
        res.data = self.ops.roll(res.data, s)
        res.degree = res.degree[nb - s:] + res.degree[:nb - s]
        res.noise = res.noise[nb - s:] + res.noise[:nb - s]
        for j in range(min(shift, nb)):
            self._set_trivial(res, j, 0)
        return res

    def unchecked_add_assign(self, lhs: RadixBatch, rhs: RadixBatch):
        for j in range(lhs.num_blocks):
            self._add_block(lhs, j, rhs, j)

    # -- carry propagation (Hillis-Steele branch) ------------------------------------------
    def _propagate_single_carry_low_latency(self, ct: RadixBatch):
        """propagate_single_carry_parallelized_low_latency (add.rs:518-537)."""
        nb = ct.num_blocks
        layer = _PbsLayer(self)
        gp = ct.clone()
        for j in range(nb):   # generate_init_carry_array (add.rs:724-771)
            layer.add(gp, j, self.lut_gen_carry if j == 0 else self.lut_gen_or_prop)
        layer.flush()
        # compute_prefix_sum_hillis_steele (add.rs:572-603)
        num_steps = (nb - 1).bit_length() if nb > 1 else 0
        space = 1
        for _ in range(num_steps):
            step = gp.clone()
            for b in range(space, nb):
                self._bivariate(layer, step, b, gp, b - space, self.lut_prefix)
            layer.flush()
            for b in range(space, nb):
                self.ops.copy_block(gp, b, step, b)
                gp.degree[b] = step.degree[b]
                gp.noise[b] = step.noise[b]
            space *= 2
        # compute_carry_propagation_parallelized_low_latency (add.rs:544-570): the last carry is
        # swapped out for a trivial zero, then rotate_right(1)
        carries = gp
        self._set_trivial(carries, nb - 1, 0)
        carries.data = self.ops.roll(carries.data, 1)
        carries.degree = carries.degree[-1:] + carries.degree[:-1]
        carries.noise = carries.noise[-1:] + carries.noise[:-1]
        for j in range(nb):
            self._add_block(ct, j, carries, j)
            layer.add(ct, j, self.lut_message)
        layer.flush()

    def _unchecked_add_assign_low_latency(self, lhs: RadixBatch, rhs: RadixBatch):
        """unchecked_add_assign_parallelized_low_latency (add.rs:487-507)."""
        assert all(a + b < self.msg * 2 for a, b in zip(lhs.degree, rhs.degree))
        self.unchecked_add_assign(lhs, rhs)
        self._propagate_single_carry_low_latency(lhs)

    def full_propagate(self, ct: RadixBatch):
        """full_propagate_parallelized = partial_propagate_parallelized(ct, 0) (mod.rs:88-155)."""
        nb = ct.num_blocks
        carries = ct.clone()
        layer = _PbsLayer(self)
        for j in range(nb):
            layer.add(ct, j, self.lut_message)
        for j in range(nb - 1):
            layer.add(carries, j, self.lut_carry)
        layer.flush()
        self._set_trivial(carries, nb - 1, 0)
        carries.data = self.ops.roll(carries.data, 1)
        carries.degree = carries.degree[-1:] + carries.degree[:-1]
        carries.noise = carries.noise[-1:] + carries.noise[:-1]
        self._unchecked_add_assign_low_latency(ct, carries)

    def add_assign_parallelized(self, lhs: RadixBatch, rhs: RadixBatch):
        """add.rs:206-242 (Hillis-Steele branch)."""
        if not rhs.block_carries_are_empty(self.msg):
            rhs = rhs.clone()
            self.full_propagate(rhs)
        if not lhs.block_carries_are_empty(self.msg):
            self.full_propagate(lhs)
        self._unchecked_add_assign_low_latency(lhs, rhs)

    # -- sum of terms ------------------------------------------------------------------------
    def unchecked_sum_ciphertexts_vec(self, cts: list) -> RadixBatch | None:
        """unchecked_sum_ciphertexts_vec_parallelized (add.rs:783-960)."""
        if not cts:
            return None
        if len(cts) == 1:
            return cts[0]
        nb = cts[0].num_blocks
        if len(cts) == 2:
            res = cts[0].clone()
            self.add_assign_parallelized(res, cts[1])
            return res
        assert all(c.block_carries_are_empty(self.msg) for c in cts)
        total = self.msg * self.carry
        fill = (total - 1) // (self.msg - 1)
        cts = list(cts)
        while len(cts) > fill:
            nchunks = len(cts) // fill
            rem = cts[nchunks * fill:]
            layer = _PbsLayer(self)
            outs = []
            for c in range(nchunks):
                chunk = cts[c * fill:(c + 1) * fill]
                s = chunk[0].clone()
                first_where, last_where = nb - 1, 0
                for a in chunk[1:]:
                    nz = [j for j in range(nb) if a.degree[j] != 0]
                    first_add = nz[0] if nz else nb
                    last_add = nz[-1] if nz else nb - 1
                    first_where = min(first_where, first_add)
                    last_where = max(last_where, last_add)
                    for j in range(first_add, last_add + 1):
                        self._add_block(s, j, a, j)
                carry = s.clone()
                for j in range(first_where, last_where + 1):
                    layer.add(s, j, self.lut_message)
                start = first_where
                end = last_where - 1 if last_where == nb - 1 else last_where
                for j in range(start, end + 1):
                    layer.add(carry, j, self.lut_carry)
                outs.append((s, carry, start, end))
            layer.flush()
            new = []
            for s, carry, start, end in outs:
                for j in range(0, start):
                    self._set_trivial(carry, j, 0)
                for j in range(end + 1, nb):
                    self._set_trivial(carry, j, 0)
                carry.data = self.ops.roll(carry.data, 1)
                carry.degree = carry.degree[-1:] + carry.degree[:-1]
                carry.noise = carry.noise[-1:] + carry.noise[:-1]
                new += [s, carry]
            cts = new + rem
        result = cts[0].clone()
        for t in cts[1:]:
            self.unchecked_add_assign(result, t)
        carry = result.clone()
        layer = _PbsLayer(self)
        for j in range(nb):
            layer.add(result, j, self.lut_message)
        for j in range(nb - 1):
            layer.add(carry, j, self.lut_carry)
        layer.flush()
        self._set_trivial(carry, nb - 1, 0)
        carry.data = self.ops.roll(carry.data, 1)
        carry.degree = carry.degree[-1:] + carry.degree[:-1]
        carry.noise = carry.noise[-1:] + carry.noise[:-1]
        self.add_assign_parallelized(result, carry)
        assert result.block_carries_are_empty(self.msg)
        return result

    def to_device(self, rb: RadixBatch) -> RadixBatch:
        """Host RadixBatch (from ClientKey.encrypt) -> this key's residency."""
        return RadixBatch(self.ops.from_host(rb.data), list(rb.degree), list(rb.noise))

    def to_host(self, rb: RadixBatch) -> RadixBatch:
        return RadixBatch(self.ops.to_host(rb.data) if not isinstance(rb.data, np.ndarray) else rb.data,
                          list(rb.degree), list(rb.noise))

    # -- multiplication ------------------------------------------------------------------------
    def unchecked_mul(self, lhs: RadixBatch, rhs: RadixBatch) -> RadixBatch:
        """unchecked_mul_assign_parallelized (mul.rs:300-414)."""
        lhs, rhs = self._resident(lhs), self._resident(rhs)
        if rhs.holds_boolean_value() or lhs.holds_boolean_value():
            raise NotImplementedError("boolean-valued operand (zero_out_if_condition_is_false path)")
        nb = lhs.num_blocks
        layer = _PbsLayer(self)
        terms = []
        rhs_nz = [i for i in range(nb) if rhs.degree[i] != 0]
        for i in rhs_nz:                       # message part: (x * y) % modulus
            res = self.blockshift(lhs, i)
            for j in range(i, nb):
                if res.degree[j] != 0:
                    self._bivariate(layer, res, j, rhs, i, self.lut_mul_lsb)
            terms.append(res)
        if self.msg > 2:                       # carry part: (x * y) / modulus, shifted one more
            for i in rhs_nz:
                res = self.blockshift(lhs, i + 1)
                for j in range(i + 1, nb):
                    if res.degree[j] != 0:
                        self._bivariate(layer, res, j, rhs, i, self.lut_mul_msb)
                terms.append(res)
        layer.flush()                          # every bivariate PBS of the product in one launch
        out = self.unchecked_sum_ciphertexts_vec(terms)
        return out if out is not None else self.create_trivial_zero(lhs.count, nb)

    def _resident(self, rb: RadixBatch) -> RadixBatch:
        if isinstance(rb.data, np.ndarray) and isinstance(self.ops, _DeviceOps):
            return self.to_device(rb)
        return rb

    def mul_parallelized(self, lhs: RadixBatch, rhs: RadixBatch) -> RadixBatch:
        """mul.rs:553-590."""
        lhs, rhs = self._resident(lhs), self._resident(rhs)
        lhs = lhs.clone()
        if not rhs.block_carries_are_empty(self.msg):
            rhs = rhs.clone()
            self.full_propagate(rhs)
        if not lhs.block_carries_are_empty(self.msg):
            self.full_propagate(lhs)
        return self.unchecked_mul(lhs, rhs)


class ClientKey:
    """integer RadixClientKey over a shortint ClientKey (integer/client_key/radix.rs)."""

    def __init__(self, shortint_client_key, num_blocks: int):
        self.key = shortint_client_key
        self.num_blocks = num_blocks

    def encrypt(self, values) -> RadixBatch:
        """Radix decomposition, least significant block first (integer/client_key/mod.rs)."""
        p = self.key.parameters
        v = np.asarray(values, dtype=np.uint64)
        m = np.uint64(p.message_modulus)
        bits = int(np.log2(p.message_modulus))
        digits = [(v >> np.uint64(bits * j)) % m for j in range(self.num_blocks)]
        blocks = [self.key.encrypt_many(d) for d in digits]   # each: list of K shortint cts
        data = np.stack([np.stack([c.ct for c in blk]) for blk in blocks], axis=1)
        return RadixBatch(data, [p.message_modulus - 1] * self.num_blocks, [NOISE_NOMINAL] * self.num_blocks)

    def decrypt(self, rb: RadixBatch) -> np.ndarray:
        p = self.key.parameters
        from . import client

        if not isinstance(rb.data, np.ndarray):
            rb = RadixBatch(rb.data.cpu().numpy().view(np.uint64), rb.degree, rb.noise)
        bits = int(np.log2(p.message_modulus))
        out = np.zeros(rb.count, dtype=np.uint64)
        for j in range(rb.num_blocks):
            raw = client.lwe_decrypt(self.key.large_lwe_secret_key, np.ascontiguousarray(rb.data[:, j, :]))
            d = client.decode(raw, p.delta) % np.uint64(p.message_modulus)
            out += d << np.uint64(bits * j)
        return out
