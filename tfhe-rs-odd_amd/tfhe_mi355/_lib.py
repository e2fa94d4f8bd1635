"""ctypes binding of lib/libtfhe_mi355.so (the C ABI declared in include/tfhe_mi355.h).

The HIP engine is the product path: there is no CPU fallback.  If the shared library is
missing, loading fails loudly.  torch is imported first (when available) so that the engine
and torch share one HIP runtime (torch bundles libamdhip64.so with the same SONAME).
"""
from __future__ import annotations

import ctypes
import os

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("TFHE_MI355_LIB") or os.path.join(_PKG_ROOT, "lib", "libtfhe_mi355.so")

u64p = ctypes.POINTER(ctypes.c_uint64)
u32p = ctypes.POINTER(ctypes.c_uint32)
vp = ctypes.c_void_p
sz = ctypes.c_size_t


class TfheMi355Parameters(ctypes.Structure):
    _fields_ = [
        ("lwe_dimension", ctypes.c_uint32),
        ("glwe_dimension", ctypes.c_uint32),
        ("polynomial_size", ctypes.c_uint32),
        ("pbs_base_log", ctypes.c_uint32),
        ("pbs_level", ctypes.c_uint32),
        ("ks_base_log", ctypes.c_uint32),
        ("ks_level", ctypes.c_uint32),
        ("message_modulus", ctypes.c_uint32),
        ("carry_modulus", ctypes.c_uint32),
        ("grouping_factor", ctypes.c_uint32),
    ]


class TfheMi355ServerKeyInfo(ctypes.Structure):
    _fields_ = [
        ("params", TfheMi355Parameters),
        ("pbs_order", ctypes.c_uint32),
        ("deterministic_execution", ctypes.c_uint32),
        ("max_degree", ctypes.c_uint64),
        ("max_noise_level", ctypes.c_uint64),
        ("ksk_seed_lo", ctypes.c_uint64),
        ("ksk_seed_hi", ctypes.c_uint64),
        ("bsk_seed_lo", ctypes.c_uint64),
        ("bsk_seed_hi", ctypes.c_uint64),
    ]


u8p = ctypes.POINTER(ctypes.c_uint8)

# (name, restype, argtypes) -- every symbol declared in include/tfhe_mi355.h
SIGNATURES = [
    ("tfhe_mi355_last_error", ctypes.c_char_p, []),
    ("tfhe_mi355_device_count", ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    ("tfhe_mi355_host_alloc", ctypes.c_int, [sz, ctypes.POINTER(vp)]),
    ("tfhe_mi355_host_free", ctypes.c_int, [vp]),
    ("tfhe_mi355_context_create", ctypes.c_int,
     [ctypes.POINTER(TfheMi355Parameters), ctypes.c_int, ctypes.POINTER(vp)]),
    ("tfhe_mi355_context_create_devices", ctypes.c_int,
     [ctypes.POINTER(TfheMi355Parameters), ctypes.POINTER(ctypes.c_int), sz, ctypes.POINTER(vp)]),
    ("tfhe_mi355_context_devices", ctypes.c_int, [vp, ctypes.POINTER(sz)]),
    ("tfhe_mi355_context_replication", ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_char_p)]),
    ("tfhe_mi355_context_device_context", ctypes.c_int, [vp, sz, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int)]),
    ("tfhe_mi355_context_destroy", ctypes.c_int, [vp]),
    ("tfhe_mi355_bootstrap_key_upload", ctypes.c_int, [vp, u64p, sz]),
    ("tfhe_mi355_bootstrap_key_convert_async", ctypes.c_int, [vp, vp, sz, vp]),
    ("tfhe_mi355_bootstrap_key_fourier", ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.POINTER(sz)]),
    ("tfhe_mi355_bootstrap_key_fourier_set_ready", ctypes.c_int, [vp]),
    ("tfhe_mi355_keyswitch_key_upload", ctypes.c_int, [vp, u64p, sz]),
    ("tfhe_mi355_keyswitch_key_upload_async", ctypes.c_int, [vp, vp, sz, vp]),
    ("tfhe_mi355_keyswitch_key_device", ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.POINTER(sz)]),
    ("tfhe_mi355_keyswitch_key_set_ready", ctypes.c_int, [vp]),
    ("tfhe_mi355_programmable_bootstrap", ctypes.c_int, [vp, u64p, u64p, u64p, sz, u32p, sz]),
    ("tfhe_mi355_programmable_bootstrap_async", ctypes.c_int, [vp, vp, vp, vp, sz, vp, sz, vp, sz, vp]),
    ("tfhe_mi355_programmable_bootstrap_scratch", ctypes.c_int, [vp, sz, ctypes.POINTER(sz)]),
    ("tfhe_mi355_keyswitch", ctypes.c_int, [vp, u64p, u64p, sz]),
    ("tfhe_mi355_keyswitch_async", ctypes.c_int, [vp, vp, vp, sz, vp, sz, vp]),
    ("tfhe_mi355_keyswitch_scratch", ctypes.c_int, [vp, sz, ctypes.POINTER(sz)]),
    ("tfhe_mi355_keyswitch_programmable_bootstrap", ctypes.c_int, [vp, u64p, u64p, u64p, sz, u32p, sz]),
    ("tfhe_mi355_keyswitch_programmable_bootstrap_async", ctypes.c_int,
     [vp, vp, vp, vp, sz, vp, sz, vp, sz, vp]),
    ("tfhe_mi355_keyswitch_programmable_bootstrap_scratch", ctypes.c_int, [vp, sz, ctypes.POINTER(sz)]),
    ("tfhe_mi355_programmable_bootstrap_keyswitch", ctypes.c_int, [vp, u64p, u64p, u64p, sz, u32p, sz]),
    ("tfhe_mi355_programmable_bootstrap_keyswitch_async", ctypes.c_int,
     [vp, vp, vp, vp, sz, vp, sz, vp, sz, vp]),
    ("tfhe_mi355_programmable_bootstrap_keyswitch_scratch", ctypes.c_int, [vp, sz, ctypes.POINTER(sz)]),
    ("tfhe_mi355_fill_accumulator", ctypes.c_int, [ctypes.POINTER(TfheMi355Parameters), u64p, u64p]),
    ("tfhe_mi355_client_gen_binary_key", ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint64, u64p, sz]),
    ("tfhe_mi355_client_gen_bootstrap_key", ctypes.c_int,
     [ctypes.c_uint64, u64p, ctypes.c_uint32, u64p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
      ctypes.c_uint32, ctypes.c_double, u64p, ctypes.c_uint32]),
    ("tfhe_mi355_blind_rotate", ctypes.c_int, [vp, u64p, u64p, u64p, ctypes.c_size_t, u32p, ctypes.c_size_t]),
    ("tfhe_mi355_blind_rotate_async", ctypes.c_int,
     [vp, vp, vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t, vp]),
    ("tfhe_mi355_lwe_scalar_mul_add_async", ctypes.c_int,
     [vp, vp, vp, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, vp]),
    ("tfhe_mi355_trivial_pbs_async", ctypes.c_int, [vp, vp, ctypes.c_size_t, ctypes.c_size_t, vp, vp]),
    ("tfhe_mi355_client_gen_multi_bit_bootstrap_key", ctypes.c_int,
     [ctypes.c_uint64, u64p, ctypes.c_uint32, u64p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
      ctypes.c_uint32, ctypes.c_uint32, ctypes.c_double, u64p, ctypes.c_uint32]),
    ("tfhe_mi355_client_gen_keyswitch_key", ctypes.c_int,
     [ctypes.c_uint64, u64p, ctypes.c_uint32, u64p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
      ctypes.c_double, u64p]),
    ("tfhe_mi355_packing_keyswitch_key_upload", ctypes.c_int, [vp, u64p, sz, ctypes.c_uint32, ctypes.c_uint32]),
    ("tfhe_mi355_packing_keyswitch", ctypes.c_int, [vp, u64p, u64p, sz]),
    ("tfhe_mi355_packing_keyswitch_async", ctypes.c_int, [vp, vp, vp, sz, vp, sz, vp]),
    ("tfhe_mi355_packing_keyswitch_scratch", ctypes.c_int, [vp, sz, ctypes.POINTER(sz)]),
    ("tfhe_mi355_glwe_poly_mul", ctypes.c_int, [vp, u64p, sz, u64p, sz, sz, ctypes.c_int, u64p]),
    ("tfhe_mi355_glwe_poly_mul_async", ctypes.c_int, [vp, vp, sz, vp, sz, sz, ctypes.c_int, vp, vp]),
    ("tfhe_mi355_client_gen_packing_keyswitch_key", ctypes.c_int,
     [ctypes.c_uint64, u64p, ctypes.c_uint32, u64p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
      ctypes.c_uint32, ctypes.c_double, u64p, ctypes.c_uint32]),
    ("tfhe_mi355_bootstrap_key_upload_seeded", ctypes.c_int, [vp, u64p, sz, ctypes.c_uint64, ctypes.c_uint64]),
    ("tfhe_mi355_keyswitch_key_upload_seeded", ctypes.c_int, [vp, u64p, sz, ctypes.c_uint64, ctypes.c_uint64]),
    ("tfhe_mi355_csprng_mask_words", ctypes.c_int, [vp, ctypes.c_uint64, ctypes.c_uint64, u64p, sz]),
    ("tfhe_mi355_debug_torus_from_fraction", ctypes.c_int,
     [ctypes.c_int, ctypes.POINTER(ctypes.c_double), u64p, u64p, sz]),
    ("tfhe_mi355_client_gen_seeded_bootstrap_key", ctypes.c_int,
     [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u64p, ctypes.c_uint32, u64p, ctypes.c_uint32,
      ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_double, u64p, ctypes.c_uint32]),
    ("tfhe_mi355_client_gen_seeded_keyswitch_key", ctypes.c_int,
     [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u64p, ctypes.c_uint32, u64p, ctypes.c_uint32,
      ctypes.c_uint32, ctypes.c_uint32, ctypes.c_double, u64p]),
    ("tfhe_mi355_client_csprng_mask_words", ctypes.c_int,
     [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, sz, u64p]),
    ("tfhe_mi355_client_lwe_encrypt", ctypes.c_int,
     [ctypes.c_uint64, u64p, ctypes.c_uint32, u64p, sz, ctypes.c_double, u64p]),
    ("tfhe_mi355_client_lwe_decrypt", ctypes.c_int, [u64p, ctypes.c_uint32, u64p, sz, u64p]),
    ("tfhe_mi355_context_parameters", ctypes.c_int, [vp, ctypes.POINTER(TfheMi355Parameters)]),
    ("tfhe_mi355_compressed_server_key_inspect", ctypes.c_int, [u8p, sz, ctypes.POINTER(TfheMi355ServerKeyInfo)]),
    ("tfhe_mi355_compressed_server_key_upload", ctypes.c_int, [vp, u8p, sz]),
    ("tfhe_mi355_server_key_inspect", ctypes.c_int, [u8p, sz, ctypes.POINTER(TfheMi355ServerKeyInfo)]),
    ("tfhe_mi355_server_key_upload", ctypes.c_int, [vp, u8p, sz]),
    ("tfhe_mi355_fourier_engine_frequency", ctypes.c_int, [ctypes.c_uint32, u32p]),
    ("tfhe_mi355_kernel_timing_enable", ctypes.c_int, [vp, ctypes.c_int]),
    ("tfhe_mi355_kernel_timing_entry", ctypes.c_int,
     [vp, sz, ctypes.c_char_p, sz, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]),
    ("tfhe_mi355_submit", ctypes.c_int,
     [vp, ctypes.c_int, u64p, u64p, u64p, sz, u32p, sz, ctypes.POINTER(vp)]),
    ("tfhe_mi355_wait", ctypes.c_int, [vp]),
    ("tfhe_mi355_coalesce_stats", ctypes.c_int,
     [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
      ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_double)]),
]

_lib = None


class EngineError(RuntimeError):
    """Raised when a C-ABI call returns 1 (the reference panics in the same situations)."""


def load():
    global _lib
    if _lib is not None:
        return _lib
    try:  # share torch's HIP runtime if torch is present (see module docstring)
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is always present in this image
        pass
    if not os.path.exists(LIB_PATH):
        raise EngineError(
            f"HIP engine library not built: {LIB_PATH} (run __graft_entry__.build() or make -C "
            f"tfhe-rs-odd_amd); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def call(name: str, *args) -> None:
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.tfhe_mi355_last_error()
        raise EngineError(f"{name}: {msg.decode() if msg else 'failure'}")
