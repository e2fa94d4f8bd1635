"""Mirror of the reference core_crypto entry points on the PBS path, backed by the HIP engine.

  convert_standard_lwe_bootstrap_key_to_fourier   lwe_bootstrap_key_conversion.rs:21-151
  programmable_bootstrap_lwe_ciphertext           lwe_programmable_bootstrapping.rs:1017-1111
  multi_bit_programmable_bootstrap_lwe_ciphertext lwe_multi_bit_programmable_bootstrapping.rs:1035-1128
  keyswitch_lwe_ciphertext                        lwe_keyswitch.rs:96-170

Argument meaning and error behaviour follow the reference: output buffers are caller-owned and
overwritten; dimension mismatches raise (the reference asserts, lwe_programmable_bootstrapping.rs
:1088-1102, lwe_keyswitch.rs:106-141).  The `_batch` forms are the engine's native shape.
"""
from __future__ import annotations

import numpy as np

from .engine import Engine
from .parameters import ClassicPBSParameters


class FourierLweBootstrapKey:
    """Fourier-domain BSK resident on one GPU (FourierLweBootstrapKey, bootstrap.rs:27-173)."""

    def __init__(self, engine: Engine):
        self.engine = engine

    @property
    def input_lwe_dimension(self):
        return self.engine.params.lwe_dimension

    @property
    def output_lwe_dimension(self):
        return self.engine.big_dim

    @property
    def polynomial_size(self):
        return self.engine.params.polynomial_size

    @property
    def glwe_size(self):
        return self.engine.params.glwe_dimension + 1


class LweKeyswitchKey:
    """Keyswitching key resident on one GPU (entities/lwe_keyswitch_key.rs)."""

    def __init__(self, engine: Engine):
        self.engine = engine

    @property
    def input_key_lwe_dimension(self):
        return self.engine.big_dim

    @property
    def output_key_lwe_dimension(self):
        return self.engine.params.lwe_dimension


def convert_standard_lwe_bootstrap_key_to_fourier(standard_bsk: np.ndarray, params: ClassicPBSParameters,
                                                  device: int = 0, engine: Engine | None = None
                                                  ) -> FourierLweBootstrapKey:
    eng = engine or Engine(params, device)
    eng.upload_bootstrap_key(standard_bsk)
    return FourierLweBootstrapKey(eng)


def upload_keyswitch_key(ksk: np.ndarray, params: ClassicPBSParameters, device: int = 0,
                         engine: Engine | None = None) -> LweKeyswitchKey:
    eng = engine or Engine(params, device)
    eng.upload_keyswitch_key(ksk)
    return LweKeyswitchKey(eng)


def programmable_bootstrap_lwe_ciphertext(input_ct: np.ndarray, output_ct: np.ndarray, accumulator: np.ndarray,
                                          fourier_bsk: FourierLweBootstrapKey) -> None:
    eng = fourier_bsk.engine
    if input_ct.shape[-1] != eng.n + 1:
        raise ValueError(f"input LweDimension {input_ct.shape[-1] - 1} != bsk input {eng.n}")
    if output_ct.shape[-1] != eng.big_dim + 1:
        raise ValueError(f"output LweDimension {output_ct.shape[-1] - 1} != bsk output {eng.big_dim}")
    output_ct[...] = eng.programmable_bootstrap(input_ct, accumulator).reshape(output_ct.shape)


def programmable_bootstrap_lwe_ciphertext_batch(inputs: np.ndarray, accumulators: np.ndarray,
                                                fourier_bsk: FourierLweBootstrapKey,
                                                lut_indexes=None) -> np.ndarray:
    return fourier_bsk.engine.programmable_bootstrap(inputs, accumulators, lut_indexes)


def multi_bit_programmable_bootstrap_lwe_ciphertext(input_ct: np.ndarray, output_ct: np.ndarray,
                                                    accumulator: np.ndarray, multi_bit_bsk: FourierLweBootstrapKey,
                                                    thread_count: int = 0) -> None:
    """The multi-bit PBS (deterministic group order); `thread_count` is accepted for signature
    parity with the reference and ignored (the GPU kernel fuses the keybundle producers)."""
    if not multi_bit_bsk.engine.params.grouping_factor:
        raise ValueError("multi_bit_programmable_bootstrap_lwe_ciphertext needs a multi-bit key")
    programmable_bootstrap_lwe_ciphertext(input_ct, output_ct, accumulator, multi_bit_bsk)


def keyswitch_lwe_ciphertext(ksk: LweKeyswitchKey, input_ct: np.ndarray, output_ct: np.ndarray) -> None:
    eng = ksk.engine
    if input_ct.shape[-1] != eng.big_dim + 1:
        raise ValueError("Mismatched input LweDimension")
    if output_ct.shape[-1] != eng.n + 1:
        raise ValueError("Mismatched output LweDimension")
    output_ct[...] = eng.keyswitch(input_ct).reshape(output_ct.shape)


def keyswitch_lwe_ciphertext_batch(ksk: LweKeyswitchKey, inputs: np.ndarray) -> np.ndarray:
    return ksk.engine.keyswitch(inputs)
