"""Mirror of the reference shortint API on the PBS path (tfhe/src/shortint), backed by the engine.

  ClientKey.encrypt / decrypt_message_and_carry / decrypt   engine/client_side.rs:58-140,
                                                            client_key/mod.rs:281-330
  ServerKey.generate_lookup_table / generate_msg_lookup_table
                                                            server_key/mod.rs:383-432
  ServerKey.apply_lookup_table[_assign]                     server_key/mod.rs:457-476
  ServerKey.keyswitch_programmable_bootstrap_assign         server_key/mod.rs:783-857
  ServerKey.programmable_bootstrap_keyswitch_assign         server_key/mod.rs:859-932
  ServerKey.trivial_pbs_assign                              server_key/mod.rs:763-781
  gen_keys                                                  shortint/mod.rs (gen_keys)

Batched forms (`apply_lookup_table_batch`) hand a whole layer of independent ciphertexts to the
GPU in one launch -- the shape the integer layer produces (radix_parallel/mul.rs:347-407).
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field

import numpy as np

from . import client
from .engine import Engine, fill_accumulator
from .parameters import ClassicPBSParameters

NOISE_ZERO = 0
NOISE_NOMINAL = 1
KEYSWITCH_BOOTSTRAP = "KeyswitchBootstrap"
BOOTSTRAP_KEYSWITCH = "BootstrapKeyswitch"


@dataclass
class Ciphertext:
    """shortint Ciphertext (shortint/ciphertext/mod.rs:263-270)."""

    ct: np.ndarray
    degree: int
    noise_level: int
    message_modulus: int
    carry_modulus: int
    pbs_order: str

    def is_trivial(self) -> bool:
        return self.noise_level == NOISE_ZERO and not np.any(self.ct[:-1])

    def clone(self) -> "Ciphertext":
        return copy.deepcopy(self)


@dataclass
class LookupTable:
    """LookupTableOwned { acc: GlweCiphertext, degree } (server_key/mod.rs)."""

    acc: np.ndarray
    degree: int


@dataclass
class ClientKey:
    parameters: ClassicPBSParameters
    seed: int = 0
    small_lwe_secret_key: np.ndarray = field(init=False)
    glwe_secret_key: np.ndarray = field(init=False)
    _enc_counter: int = field(init=False, default=0)

    def __post_init__(self):
        p = self.parameters
        self.small_lwe_secret_key = client.gen_binary_key(self.seed, 1, p.lwe_dimension)
        self.glwe_secret_key = client.gen_binary_key(self.seed, 2, p.glwe_dimension * p.polynomial_size)

    @property
    def large_lwe_secret_key(self) -> np.ndarray:
        return self.glwe_secret_key  # GlweSecretKey::into_lwe_secret_key

    @property
    def pbs_order(self) -> str:
        return KEYSWITCH_BOOTSTRAP if self.parameters.encryption_key_choice == "Big" else BOOTSTRAP_KEYSWITCH

    def _enc_key(self):
        p = self.parameters
        if self.pbs_order == KEYSWITCH_BOOTSTRAP:
            return self.large_lwe_secret_key, p.glwe_modular_std_dev
        return self.small_lwe_secret_key, p.lwe_modular_std_dev

    def encrypt_many(self, messages) -> list[Ciphertext]:
        p = self.parameters
        m = np.asarray(messages, dtype=np.uint64) % np.uint64(p.message_modulus)
        key, std = self._enc_key()
        self._enc_counter += 1
        cts = client.lwe_encrypt((self.seed << 20) + self._enc_counter, key, m * np.uint64(p.delta), std)
        return [Ciphertext(cts[i].copy(), p.message_modulus - 1, NOISE_NOMINAL, p.message_modulus,
                           p.carry_modulus, self.pbs_order) for i in range(len(m))]

    def encrypt(self, message: int) -> Ciphertext:
        return self.encrypt_many([message])[0]

    def decrypt_message_and_carry_many(self, cts: list[Ciphertext]) -> np.ndarray:
        key = self.large_lwe_secret_key if cts[0].pbs_order == KEYSWITCH_BOOTSTRAP else self.small_lwe_secret_key
        raw = client.lwe_decrypt(key, np.stack([c.ct for c in cts]))
        return client.decode(raw, self.parameters.delta)

    def decrypt_message_and_carry(self, ct: Ciphertext) -> int:
        return int(self.decrypt_message_and_carry_many([ct])[0])

    def decrypt(self, ct: Ciphertext) -> int:
        return self.decrypt_message_and_carry(ct) % ct.message_modulus


class ServerKey:
    """shortint ServerKey whose bootstrapping key is the MI355X engine (the `Gpu` arm of
    ShortintBootstrappingKey, server_key/mod.rs:104-111)."""

    def __init__(self, client_key: ClientKey | None = None, device: int = 0, *, engine: Engine | None = None,
                 bsk: np.ndarray | None = None, ksk: np.ndarray | None = None,
                 parameters: ClassicPBSParameters | None = None):
        p = client_key.parameters if client_key is not None else parameters
        if p is None:
            raise ValueError("parameters required")
        self.parameters = p
        self.message_modulus = p.message_modulus
        self.carry_modulus = p.carry_modulus
        self.engine = engine or Engine(p, device)
        if client_key is not None and bsk is None:
            ck = client_key
            if p.grouping_factor:
                bsk = client.gen_multi_bit_bootstrap_key(
                    ck.seed * 7 + 3, ck.small_lwe_secret_key, ck.glwe_secret_key, p.glwe_dimension,
                    p.polynomial_size, p.pbs_base_log, p.pbs_level, p.grouping_factor, p.glwe_modular_std_dev)
            else:
                bsk = client.gen_bootstrap_key(ck.seed * 7 + 3, ck.small_lwe_secret_key, ck.glwe_secret_key,
                                               p.glwe_dimension, p.polynomial_size, p.pbs_base_log,
                                               p.pbs_level, p.glwe_modular_std_dev)
            ksk = client.gen_keyswitch_key(ck.seed * 7 + 4, ck.large_lwe_secret_key, ck.small_lwe_secret_key,
                                           p.ks_base_log, p.ks_level, p.lwe_modular_std_dev)
        if bsk is not None:
            self.engine.upload_bootstrap_key(bsk)
        if ksk is not None:
            self.engine.upload_keyswitch_key(ksk)
        self.pbs_order = KEYSWITCH_BOOTSTRAP if p.encryption_key_choice == "Big" else BOOTSTRAP_KEYSWITCH

    @classmethod
    def deserialize(cls, data: bytes, device: int = 0, parameters: ClassicPBSParameters | None = None) -> "ServerKey":
        """A bincode-serialized shortint ServerKey (server_key/mod.rs:283-297: standard KSK +
        Fourier BSK) straight onto the GPU (serialization.py, csrc/serde.cpp)."""
        from .serialization import inspect_server_key

        p = parameters or inspect_server_key(data).parameters()
        eng = Engine(p, device)
        eng.upload_server_key(data)
        return cls(None, engine=eng, parameters=p)

    # -- lookup tables ---------------------------------------------------------------------
    def generate_lookup_table(self, f) -> LookupTable:
        p = self.parameters
        acc = fill_accumulator(p, f)
        max_value = max(int(f(i)) for i in range(p.message_modulus * p.carry_modulus))
        return LookupTable(acc, max_value)

    def generate_msg_lookup_table(self, f, modulus: int) -> LookupTable:
        return self.generate_lookup_table(lambda x: f(x % modulus) % modulus)

    # -- PBS ---------------------------------------------------------------------------------
    def trivial_pbs_assign(self, ct: Ciphertext, acc: LookupTable) -> None:
        assert ct.noise_level == NOISE_ZERO
        p = self.parameters
        modulus_sup = p.message_modulus * p.carry_modulus
        delta = p.delta
        value = int(ct.ct[-1]) // delta
        box = p.polynomial_size // modulus_sup
        body = acc.acc[p.glwe_dimension * p.polynomial_size:]
        if value >= modulus_sup:
            res = (0 - int(body[(value % modulus_sup) * box])) % (1 << 64)
        else:
            res = int(body[value * box])
        ct.ct[-1] = np.uint64(res)
        ct.degree = acc.degree

    def create_trivial(self, value: int) -> Ciphertext:
        p = self.parameters
        dim = p.big_lwe_dimension if self.pbs_order == KEYSWITCH_BOOTSTRAP else p.lwe_dimension
        ct = np.zeros(dim + 1, dtype=np.uint64)
        ct[-1] = np.uint64((value % (p.message_modulus * p.carry_modulus)) * p.delta)
        return Ciphertext(ct, value, NOISE_ZERO, p.message_modulus, p.carry_modulus, self.pbs_order)

    def engine_ks_pbs(self, x: np.ndarray, luts: np.ndarray, lut_indexes=None) -> np.ndarray:
        """One batched launch of the key's PBS order over rows of x (big-key LWEs for KS->PBS)."""
        if self.pbs_order == KEYSWITCH_BOOTSTRAP:
            return self.engine.keyswitch_programmable_bootstrap(x, luts, lut_indexes)
        return self.engine.programmable_bootstrap_keyswitch(x, luts, lut_indexes)

    def apply_lookup_table_batch_assign(self, cts: list[Ciphertext], accs) -> None:
        """One GPU launch for a whole layer; accs: one LookupTable or one per ciphertext."""
        if isinstance(accs, LookupTable):
            accs = [accs] * len(cts)
        todo = [i for i, c in enumerate(cts) if not c.is_trivial()]
        for i, c in enumerate(cts):
            if c.is_trivial():
                self.trivial_pbs_assign(c, accs[i])
        if todo:
            uniq, idx = {}, []
            for i in todo:
                key = id(accs[i])
                if key not in uniq:
                    uniq[key] = (len(uniq), accs[i].acc)
                idx.append(uniq[key][0])
            luts = np.stack([a for _, a in sorted(uniq.values(), key=lambda t: t[0])])
            x = np.stack([cts[i].ct for i in todo])
            lut_idx = np.asarray(idx, dtype=np.uint32) if len(uniq) > 1 else None
            if self.pbs_order == KEYSWITCH_BOOTSTRAP:
                out = self.engine.keyswitch_programmable_bootstrap(x, luts, lut_idx)
            else:
                out = self.engine.programmable_bootstrap_keyswitch(x, luts, lut_idx)
            for j, i in enumerate(todo):
                cts[i].ct = out[j].copy()
                cts[i].noise_level = NOISE_NOMINAL
        for i, c in enumerate(cts):
            c.degree = accs[i].degree

    def apply_lookup_table_batch(self, cts: list[Ciphertext], accs) -> list[Ciphertext]:
        res = [c.clone() for c in cts]
        self.apply_lookup_table_batch_assign(res, accs)
        return res

    def apply_lookup_table_assign(self, ct: Ciphertext, acc: LookupTable) -> None:
        self.apply_lookup_table_batch_assign([ct], acc)

    def apply_lookup_table(self, ct: Ciphertext, acc: LookupTable) -> Ciphertext:
        res = ct.clone()
        self.apply_lookup_table_assign(res, acc)
        return res

    def keyswitch_programmable_bootstrap_assign(self, ct: Ciphertext, acc: LookupTable) -> None:
        if ct.is_trivial():
            self.trivial_pbs_assign(ct, acc)
            return
        ct.ct = self.engine.keyswitch_programmable_bootstrap(ct.ct, acc.acc)[0].copy()
        ct.degree = acc.degree
        ct.noise_level = NOISE_NOMINAL

    def programmable_bootstrap_keyswitch_assign(self, ct: Ciphertext, acc: LookupTable) -> None:
        if ct.is_trivial():
            self.trivial_pbs_assign(ct, acc)
            return
        ct.ct = self.engine.programmable_bootstrap_keyswitch(ct.ct, acc.acc)[0].copy()
        ct.degree = acc.degree
        ct.noise_level = NOISE_NOMINAL

    def message_extract(self, ct: Ciphertext) -> Ciphertext:
        acc = self.generate_lookup_table(lambda x: x % ct.message_modulus)
        return self.apply_lookup_table(ct, acc)

    def carry_extract(self, ct: Ciphertext) -> Ciphertext:
        acc = self.generate_lookup_table(lambda x: x // ct.message_modulus)
        return self.apply_lookup_table(ct, acc)


class CompressedServerKey:
    """shortint CompressedServerKey (server_key/compressed.rs:43-55) in its serialized (bincode)
    form: seeded keyswitching and bootstrapping keys, decompressed on the GPU."""

    def __init__(self, data: bytes):
        from .serialization import inspect_compressed_server_key

        self.data = bytes(data)
        self.info = inspect_compressed_server_key(self.data)   # validates the whole buffer

    @classmethod
    def deserialize(cls, data: bytes) -> "CompressedServerKey":
        return cls(data)

    def decompress(self, device: int = 0, parameters: ClassicPBSParameters | None = None) -> ServerKey:
        """CompressedServerKey::decompress (compressed.rs) + the Fourier conversion, on the GPU."""
        p = parameters or self.info.parameters()
        eng = Engine(p, device)
        eng.upload_compressed_server_key(self.data)
        return ServerKey(None, engine=eng, parameters=p)


def gen_keys(parameters: ClassicPBSParameters, seed: int = 0, device: int = 0):
    ck = ClientKey(parameters, seed)
    sk = ServerKey(ck, device)
    return ck, sk
