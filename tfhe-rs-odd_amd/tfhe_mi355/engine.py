"""Engine = one C-ABI context on one GPU (include/tfhe_mi355.h), numpy in/out or torch device
tensors in/out.  This is the object a reference `ShortintBootstrappingKey::Gpu{handle}` arm would
hold (SURVEY.md 8b seam 1).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import TfheMi355Parameters, sz, u32p, u64p, vp
from .parameters import ClassicPBSParameters


def _u64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint64)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(u64p)


def _dev_ptr(t) -> int:
    """Device pointer of a torch tensor (or a raw int)."""
    if t is None:
        return None
    if isinstance(t, int):
        return t
    if not t.is_contiguous():
        raise ValueError("device tensors must be contiguous")
    return t.data_ptr()


def _stream_ptr(stream) -> int:
    if stream is None:
        import torch

        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def c_params(p: ClassicPBSParameters) -> TfheMi355Parameters:
    return TfheMi355Parameters(p.lwe_dimension, p.glwe_dimension, p.polynomial_size, p.pbs_base_log,
                               p.pbs_level, p.ks_base_log, p.ks_level, p.message_modulus,
                               p.carry_modulus, p.grouping_factor)


def _free_host(ptr: int) -> None:
    try:
        _lib.load().tfhe_mi355_host_free(vp(ptr))
    except Exception:  # interpreter shutdown
        pass


def pinned_empty(shape, dtype=np.uint64) -> np.ndarray:
    """An uninitialised numpy array in page-locked host memory (tfhe_mi355_host_alloc), freed with
    the array.  Batches passed to the host-pointer entry points in such arrays are DMA'd directly."""
    import weakref

    n = int(np.prod(shape)) * np.dtype(dtype).itemsize
    p = vp()
    _lib.call("tfhe_mi355_host_alloc", max(n, 1), ctypes.byref(p))
    buf = (ctypes.c_uint8 * max(n, 1)).from_address(p.value)
    weakref.finalize(buf, _free_host, p.value)
    return np.frombuffer(buf, dtype=np.uint8, count=n).view(dtype).reshape(shape)


def device_count() -> int:
    n = ctypes.c_int(0)
    _lib.call("tfhe_mi355_device_count", ctypes.byref(n))
    return n.value


class Engine:
    """MI355X PBS engine context bound to `device`, or -- `devices` = a list of device ordinals
    (repeats allowed; [] = every visible GPU) -- one context over several GPUs of this process
    (tfhe_mi355_context_create_devices): keys replicated from the first device, batched calls split
    over the devices, small calls and submits spread round robin; device-tensor (async) calls run on
    the first device."""

    def __init__(self, params: ClassicPBSParameters, device: int = 0, devices=None):
        self.params = params
        self._cp = c_params(params)
        h = vp()
        if devices is None:
            self.device = device
            _lib.call("tfhe_mi355_context_create", ctypes.byref(self._cp), device, ctypes.byref(h))
        else:
            arr = (ctypes.c_int * max(len(devices), 1))(*devices)
            _lib.call("tfhe_mi355_context_create_devices", ctypes.byref(self._cp), arr, len(devices),
                      ctypes.byref(h))
        self._h = h
        self.devices = self.device_ordinals() if devices is not None else [device]
        self.device = self.devices[0]

    @property
    def multi_device(self) -> bool:
        """True for a context over several shards (tfhe_mi355_context_create_devices with > 1 entry)."""
        return len(self.devices) > 1

    def device_ordinals(self) -> list:
        """Device ordinal of each shard (one entry for a single-device context)."""
        n = sz()
        _lib.call("tfhe_mi355_context_devices", self._h, ctypes.byref(n))
        out = []
        for i in range(n.value):
            sub, dev = vp(), ctypes.c_int()
            _lib.call("tfhe_mi355_context_device_context", self._h, i, ctypes.byref(sub), ctypes.byref(dev))
            out.append(dev.value)
        return out

    REPLICATION = {0: "none", 1: "rccl", 2: "peer_copy", 3: "device_copy"}

    def replication(self):
        """How the last key replication ran ('none' | 'rccl' | 'peer_copy' | 'device_copy') and why auto
        mode did not use RCCL ('' when it did or had no need)."""
        mode, note = ctypes.c_int(), ctypes.c_char_p()
        _lib.call("tfhe_mi355_context_replication", self._h, ctypes.byref(mode), ctypes.byref(note))
        return self.REPLICATION.get(mode.value, str(mode.value)), (note.value or b"").decode()

    # -- lifetime ---------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib.call("tfhe_mi355_context_destroy", self._h)
            self._h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- sizes --------------------------------------------------------------------------
    @property
    def n(self):
        return self.params.lwe_dimension

    @property
    def big_dim(self):
        return self.params.glwe_dimension * self.params.polynomial_size

    @property
    def glwe_len(self):
        return (self.params.glwe_dimension + 1) * self.params.polynomial_size

    # -- keys ---------------------------------------------------------------------------
    def upload_bootstrap_key(self, standard_bsk: np.ndarray) -> None:
        b = _u64(standard_bsk).ravel()
        _lib.call("tfhe_mi355_bootstrap_key_upload", self._h, _ptr(b), b.size)

    def convert_bootstrap_key_device(self, d_standard_bsk, numel: int, stream=None) -> None:
        _lib.call("tfhe_mi355_bootstrap_key_convert_async", self._h, _dev_ptr(d_standard_bsk), numel,
                  _stream_ptr(stream))

    def fourier_bootstrap_key(self):
        """(device pointer, bytes) of the Fourier BSK buffer (for RCCL broadcast)."""
        p, b = vp(), ctypes.c_size_t()
        _lib.call("tfhe_mi355_bootstrap_key_fourier", self._h, ctypes.byref(p), ctypes.byref(b))
        return p.value, b.value

    def fourier_bootstrap_key_set_ready(self):
        _lib.call("tfhe_mi355_bootstrap_key_fourier_set_ready", self._h)

    def upload_keyswitch_key(self, ksk: np.ndarray) -> None:
        k = _u64(ksk).ravel()
        _lib.call("tfhe_mi355_keyswitch_key_upload", self._h, _ptr(k), k.size)

    def upload_keyswitch_key_device(self, d_ksk, numel: int, stream=None) -> None:
        _lib.call("tfhe_mi355_keyswitch_key_upload_async", self._h, _dev_ptr(d_ksk), numel, _stream_ptr(stream))

    def keyswitch_key_device(self):
        p, b = vp(), ctypes.c_size_t()
        _lib.call("tfhe_mi355_keyswitch_key_device", self._h, ctypes.byref(p), ctypes.byref(b))
        return p.value, b.value

    def keyswitch_key_set_ready(self):
        _lib.call("tfhe_mi355_keyswitch_key_set_ready", self._h)

    # -- profiling -----------------------------------------------------------------------
    def kernel_timing(self, every: int) -> None:
        """Time every `every`-th launch of each kernel family with HIP events on its stream
        (0 = off); clears the totals."""
        _lib.call("tfhe_mi355_kernel_timing_enable", self._h, int(every))

    def kernel_times(self) -> dict:
        """{kernel family: (average ms per timed launch, timed launches)}; waits for the events."""
        out = {}
        name = ctypes.create_string_buffer(128)
        tot, cnt = ctypes.c_double(), ctypes.c_uint64()
        lib = _lib.load()
        i = 0
        while lib.tfhe_mi355_kernel_timing_entry(self._h, i, name, 128, ctypes.byref(tot), ctypes.byref(cnt)) == 0:
            out[name.value.decode()] = (tot.value / max(cnt.value, 1), cnt.value)
            i += 1
        return out

    def coalesce_stats(self, reset: bool = False) -> dict:
        """Request-coalescing counters: batches, ciphertexts, most batches in flight, batch wall
        seconds (summed); `reset` clears them after reading."""
        b, r, m = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        t = ctypes.c_double()
        _lib.call("tfhe_mi355_coalesce_stats", self._h, int(bool(reset)), ctypes.byref(b), ctypes.byref(r),
                  ctypes.byref(m), ctypes.byref(t))
        return {"batches": b.value, "rows": r.value, "max_in_flight": m.value, "batch_seconds": t.value,
                "mean_batch_rows": r.value / b.value if b.value else None,
                "mean_batch_ms": 1e3 * t.value / b.value if b.value else None}

    # -- host (numpy) batched ops ---------------------------------------------------------
    def _luts(self, luts):
        luts = _u64(luts)
        if luts.ndim == 1:
            luts = luts.reshape(1, -1)
        if luts.shape[1] != self.glwe_len:
            raise ValueError(f"lookup table has {luts.shape[1]} words, expected {self.glwe_len}")
        return luts

    @staticmethod
    def _idx(lut_indexes, count, lut_count):
        if lut_indexes is None:
            return None, None
        idx = np.ascontiguousarray(lut_indexes, dtype=np.uint32)
        if idx.shape != (count,):
            raise ValueError("lut_indexes must have one entry per ciphertext")
        return idx, idx.ctypes.data_as(u32p)

    @staticmethod
    def _out(out, shape):
        if out is None:
            return np.empty(shape, dtype=np.uint64)
        if out.dtype != np.uint64 or out.shape != shape or not out.flags.c_contiguous:
            raise ValueError(f"out must be a C-contiguous uint64 array of shape {shape}")
        return out

    def programmable_bootstrap(self, lwe_in, luts, lut_indexes=None, out=None) -> np.ndarray:
        """`out` (optional): the caller's output array; in and out arrays from `pinned_empty` are
        DMA'd directly by the ABI (no staging copies)."""
        x = _u64(lwe_in).reshape(-1, self.n + 1)
        L = self._luts(luts)
        idx, idxp = self._idx(lut_indexes, x.shape[0], L.shape[0])
        out = self._out(out, (x.shape[0], self.big_dim + 1))
        _lib.call("tfhe_mi355_programmable_bootstrap", self._h, _ptr(x), _ptr(out), _ptr(L), L.shape[0],
                  idxp, x.shape[0])
        return out

    def blind_rotate(self, lwe_in, luts, lut_indexes=None) -> np.ndarray:
        """bootstrap_without_sample_extract (fork, fft64/crypto/bootstrap.rs:383-412): the rotated
        accumulators, [count][(k+1)N]."""
        x = _u64(lwe_in).reshape(-1, self.n + 1)
        L = self._luts(luts)
        idx, idxp = self._idx(lut_indexes, x.shape[0], L.shape[0])
        out = np.empty((x.shape[0], self.glwe_len), dtype=np.uint64)
        _lib.call("tfhe_mi355_blind_rotate", self._h, _ptr(x), _ptr(out), _ptr(L), L.shape[0], idxp, x.shape[0])
        return out

    def keyswitch(self, lwe_in) -> np.ndarray:
        x = _u64(lwe_in).reshape(-1, self.big_dim + 1)
        out = np.empty((x.shape[0], self.n + 1), dtype=np.uint64)
        _lib.call("tfhe_mi355_keyswitch", self._h, _ptr(x), _ptr(out), x.shape[0])
        return out

    def keyswitch_programmable_bootstrap(self, lwe_in, luts, lut_indexes=None, out=None) -> np.ndarray:
        x = _u64(lwe_in).reshape(-1, self.big_dim + 1)
        L = self._luts(luts)
        idx, idxp = self._idx(lut_indexes, x.shape[0], L.shape[0])
        out = self._out(out, (x.shape[0], self.big_dim + 1))
        _lib.call("tfhe_mi355_keyswitch_programmable_bootstrap", self._h, _ptr(x), _ptr(out), _ptr(L),
                  L.shape[0], idxp, x.shape[0])
        return out

    # -- asynchronous small calls (tfhe_mi355_submit / _wait, the coalescer's queue) ----------
    OPS = {"pbs": (0, "n", "big"), "ks_pbs": (1, "big", "big"), "pbs_ks": (2, "n", "n"), "ks": (3, "big", "n")}

    def submit(self, op: str, lwe_in, luts=None, lut_indexes=None) -> "Request":
        """Enqueue 1..1024 ciphertexts of `op` ("pbs", "ks_pbs", "pbs_ks", "ks") and return at once;
        `Request.wait()` returns the outputs (every request must be waited on)."""
        code, din, dout = self.OPS[op]
        w_in = (self.n if din == "n" else self.big_dim) + 1
        w_out = (self.n if dout == "n" else self.big_dim) + 1
        x = np.ascontiguousarray(_u64(lwe_in).reshape(-1, w_in))
        if code == 3:
            L, idx, idxp = np.zeros((1, 1), dtype=np.uint64), None, None
        else:
            L = self._luts(luts)
            idx, idxp = self._idx(lut_indexes, x.shape[0], L.shape[0])
        out = np.empty((x.shape[0], w_out), dtype=np.uint64)
        h = ctypes.c_void_p()
        _lib.call("tfhe_mi355_submit", self._h, code, _ptr(x), _ptr(out), _ptr(L), 0 if code == 3 else L.shape[0],
                  idxp, x.shape[0], ctypes.byref(h))
        return Request(h, (x, L, idx, out))

    def programmable_bootstrap_keyswitch(self, lwe_in, luts, lut_indexes=None) -> np.ndarray:
        x = _u64(lwe_in).reshape(-1, self.n + 1)
        L = self._luts(luts)
        idx, idxp = self._idx(lut_indexes, x.shape[0], L.shape[0])
        out = np.empty((x.shape[0], self.n + 1), dtype=np.uint64)
        _lib.call("tfhe_mi355_programmable_bootstrap_keyswitch", self._h, _ptr(x), _ptr(out), _ptr(L),
                  L.shape[0], idxp, x.shape[0])
        return out

    def upload_compressed_server_key(self, data: bytes) -> None:
        """Both keys of a bincode-serialized shortint CompressedServerKey (serialization.py)."""
        buf = np.frombuffer(data, dtype=np.uint8)
        _lib.call("tfhe_mi355_compressed_server_key_upload", self._h,
                  buf.ctypes.data_as(_lib.u8p), buf.size)

    def upload_server_key(self, data: bytes) -> None:
        """Both keys of a bincode-serialized shortint ServerKey (Fourier BSK, serialization.py)."""
        buf = np.frombuffer(data, dtype=np.uint8)
        _lib.call("tfhe_mi355_server_key_upload", self._h, buf.ctypes.data_as(_lib.u8p), buf.size)

    def upload_seeded_bootstrap_key(self, bodies: np.ndarray, compression_seed: int) -> None:
        """decompress_seeded_lwe_bootstrap_key on the GPU + Fourier conversion."""
        b = _u64(bodies)
        _lib.call("tfhe_mi355_bootstrap_key_upload_seeded", self._h, _ptr(b), b.size,
                  compression_seed & 0xFFFFFFFFFFFFFFFF, (compression_seed >> 64) & 0xFFFFFFFFFFFFFFFF)

    def upload_seeded_keyswitch_key(self, bodies: np.ndarray, compression_seed: int) -> None:
        """decompress_seeded_lwe_keyswitch_key on the GPU."""
        b = _u64(bodies)
        _lib.call("tfhe_mi355_keyswitch_key_upload_seeded", self._h, _ptr(b), b.size,
                  compression_seed & 0xFFFFFFFFFFFFFFFF, (compression_seed >> 64) & 0xFFFFFFFFFFFFFFFF)

    def csprng_mask_words(self, compression_seed: int, count: int) -> np.ndarray:
        out = np.empty(count, dtype=np.uint64)
        _lib.call("tfhe_mi355_csprng_mask_words", self._h, compression_seed & 0xFFFFFFFFFFFFFFFF,
                  (compression_seed >> 64) & 0xFFFFFFFFFFFFFFFF, _ptr(out), count)
        return out

    def upload_packing_keyswitch_key(self, pksk: np.ndarray, base_log: int, level: int) -> None:
        k = _u64(pksk)
        _lib.call("tfhe_mi355_packing_keyswitch_key_upload", self._h, _ptr(k), k.size, base_log, level)

    def packing_keyswitch(self, lwe_in) -> np.ndarray:
        """keyswitch_lwe_ciphertext_into_glwe_ciphertext (lwe_packing_keyswitch.rs:102-186), batched."""
        x = _u64(lwe_in).reshape(-1, self.big_dim + 1)
        out = np.empty((x.shape[0], self.glwe_len), dtype=np.uint64)
        _lib.call("tfhe_mi355_packing_keyswitch", self._h, _ptr(x), _ptr(out), x.shape[0])
        return out

    def glwe_poly_mul(self, glwe_in, polys, extract: bool = False) -> np.ndarray:
        """out[c][i] = sum_j glwe_in[c][j] * polys[i][j] (negacyclic, wrapping), optionally sample-
        extracted: glwe_in [count][J][(k+1)N], polys [npoly][J][N]."""
        N = self.params.polynomial_size
        g = _u64(glwe_in)
        if g.ndim == 2:
            g = g.reshape(g.shape[0], 1, -1)
        v = _u64(polys)
        if v.ndim == 2:
            v = v.reshape(v.shape[0], 1, -1)
        count, J = g.shape[0], g.shape[1]
        if g.shape[2] != self.glwe_len or v.shape[1] != J or v.shape[2] != N:
            raise ValueError("glwe_poly_mul: shape mismatch")
        out = np.empty((count, v.shape[0], self.big_dim + 1 if extract else self.glwe_len), dtype=np.uint64)
        _lib.call("tfhe_mi355_glwe_poly_mul", self._h, _ptr(g), J, _ptr(v), v.shape[0], count, int(extract), _ptr(out))
        return out

    # -- device (torch) async ops -------------------------------------------------------
    # Every device scratch the C ABI needs comes from the caller (include/tfhe_mi355.h): pass
    # d_scratch (>= the matching *_scratch_bytes), or let these wrappers allocate it from torch's
    # caching allocator for the call.
    def _scratch_query(self, fn: str, count: int) -> int:
        b = ctypes.c_size_t()
        _lib.call(fn, self._h, count, ctypes.byref(b))
        return b.value

    def pbs_scratch_bytes(self, count: int) -> int:
        return self._scratch_query("tfhe_mi355_programmable_bootstrap_scratch", count)

    def ks_scratch_bytes(self, count: int) -> int:
        return self._scratch_query("tfhe_mi355_keyswitch_scratch", count)

    def pks_scratch_bytes(self, count: int) -> int:
        return self._scratch_query("tfhe_mi355_packing_keyswitch_scratch", count)

    def ks_pbs_scratch_bytes(self, count: int) -> int:
        return self._scratch_query("tfhe_mi355_keyswitch_programmable_bootstrap_scratch", count)

    def pbs_ks_scratch_bytes(self, count: int) -> int:
        return self._scratch_query("tfhe_mi355_programmable_bootstrap_keyswitch_scratch", count)

    def _scratch(self, d_scratch, need: int, stream):
        """(pointer, bytes, keep-alive) of the scratch for one async call."""
        if d_scratch is not None:
            nbytes = d_scratch.numel() * d_scratch.element_size() if hasattr(d_scratch, "numel") else need
            return _dev_ptr(d_scratch), nbytes, d_scratch
        if need == 0:
            return None, 0, None
        import torch

        t = torch.empty(need, dtype=torch.uint8, device=torch.device("cuda", self.device))
        # The tensor is freed when the wrapper returns, while the kernel may still run: tell the
        # caching allocator which stream uses the block so it is not handed out before that
        # stream reaches this point (raw int handles are wrapped as an ExternalStream).
        if isinstance(stream, int):
            stream = torch.cuda.ExternalStream(stream, device=t.device)
        if stream is not None and stream != torch.cuda.current_stream(t.device):
            t.record_stream(stream)
        return t.data_ptr(), need, t

    def programmable_bootstrap_async(self, d_in, d_out, d_luts, lut_count: int, count: int,
                                     d_lut_indexes=None, stream=None, d_scratch=None) -> None:
        sp, sb, _keep = self._scratch(d_scratch, self.pbs_scratch_bytes(count), stream)
        _lib.call("tfhe_mi355_programmable_bootstrap_async", self._h, _dev_ptr(d_in), _dev_ptr(d_out),
                  _dev_ptr(d_luts), lut_count, _dev_ptr(d_lut_indexes), count, sp, sb, _stream_ptr(stream))

    def blind_rotate_async(self, d_in, d_glwe_out, d_luts, lut_count: int, count: int, d_lut_indexes=None,
                           stream=None) -> None:
        _lib.call("tfhe_mi355_blind_rotate_async", self._h, _dev_ptr(d_in), _dev_ptr(d_glwe_out), _dev_ptr(d_luts),
                  lut_count, _dev_ptr(d_lut_indexes), count, _stream_ptr(stream))

    def keyswitch_async(self, d_in, d_out, count: int, stream=None, d_scratch=None) -> None:
        sp, sb, _keep = self._scratch(d_scratch, self.ks_scratch_bytes(count), stream)
        _lib.call("tfhe_mi355_keyswitch_async", self._h, _dev_ptr(d_in), _dev_ptr(d_out), count, sp, sb,
                  _stream_ptr(stream))

    def keyswitch_programmable_bootstrap_async(self, d_in, d_out, d_luts, lut_count: int, count: int,
                                               d_scratch=None, d_lut_indexes=None, stream=None) -> None:
        sp, sb, _keep = self._scratch(d_scratch, self.ks_pbs_scratch_bytes(count), stream)
        _lib.call("tfhe_mi355_keyswitch_programmable_bootstrap_async", self._h, _dev_ptr(d_in),
                  _dev_ptr(d_out), _dev_ptr(d_luts), lut_count, _dev_ptr(d_lut_indexes), count,
                  sp, sb, _stream_ptr(stream))

    def programmable_bootstrap_keyswitch_async(self, d_in, d_out, d_luts, lut_count: int, count: int,
                                               d_scratch=None, d_lut_indexes=None, stream=None) -> None:
        sp, sb, _keep = self._scratch(d_scratch, self.pbs_ks_scratch_bytes(count), stream)
        _lib.call("tfhe_mi355_programmable_bootstrap_keyswitch_async", self._h, _dev_ptr(d_in),
                  _dev_ptr(d_out), _dev_ptr(d_luts), lut_count, _dev_ptr(d_lut_indexes), count,
                  sp, sb, _stream_ptr(stream))

    def lwe_scalar_mul_add_async(self, y_ptr: int, x_ptr, scalar: int, rows: int, words: int, y_stride: int,
                                 x_stride: int = 0, stream=None) -> None:
        """y[r] = y[r] * scalar + x[r] (u64 wrapping) on device rows (raw pointers: strided views allowed)."""
        _lib.call("tfhe_mi355_lwe_scalar_mul_add_async", self._h, y_ptr, x_ptr, scalar % (1 << 64), rows, words,
                  y_stride, x_stride, _stream_ptr(stream))

    def trivial_pbs_async(self, body_ptr: int, rows: int, stride: int, d_lut, stream=None) -> None:
        _lib.call("tfhe_mi355_trivial_pbs_async", self._h, body_ptr, rows, stride, _dev_ptr(d_lut),
                  _stream_ptr(stream))

    def packing_keyswitch_async(self, d_in, d_out, count: int, stream=None, d_scratch=None) -> None:
        sp, sb, _keep = self._scratch(d_scratch, self.pks_scratch_bytes(count), stream)
        _lib.call("tfhe_mi355_packing_keyswitch_async", self._h, _dev_ptr(d_in), _dev_ptr(d_out), count, sp, sb,
                  _stream_ptr(stream))

    def glwe_poly_mul_async(self, d_glwe, glwe_per_item: int, d_polys, npoly: int, count: int, extract: bool,
                            d_out, stream=None) -> None:
        _lib.call("tfhe_mi355_glwe_poly_mul_async", self._h, _dev_ptr(d_glwe), glwe_per_item, _dev_ptr(d_polys),
                  npoly, count, int(extract), _dev_ptr(d_out), _stream_ptr(stream))


def fill_accumulator(params: ClassicPBSParameters, f) -> np.ndarray:
    """shortint fill_accumulator (shortint/engine/mod.rs:72-128) through the C ABI."""
    p = params.message_modulus * params.carry_modulus
    fv = _u64([int(f(i)) & 0xFFFFFFFFFFFFFFFF for i in range(p)])
    acc = np.zeros((params.glwe_dimension + 1) * params.polynomial_size, dtype=np.uint64)
    cp = c_params(params)
    _lib.call("tfhe_mi355_fill_accumulator", ctypes.byref(cp), _ptr(fv), _ptr(acc))
    return acc


class Request:
    """Handle of a submitted small call (Engine.submit): keeps the host buffers alive until wait()."""

    def __init__(self, handle, buffers):
        self._h, self._bufs = handle, buffers

    def wait(self) -> np.ndarray:
        if self._h is None:
            raise RuntimeError("request already waited on")
        h, self._h = self._h, None
        _lib.call("tfhe_mi355_wait", h)
        return self._bufs[3]

    def __del__(self):
        # Dropped without wait() (e.g. an exception between a loop of submits and the waits): the
        # dispatcher may still copy from / into the numpy buffers this object keeps alive, so block
        # until the request is done (this also frees its native handle); errors are ignored here.
        h, self._h = getattr(self, "_h", None), None
        if h is not None:
            try:
                _lib.load().tfhe_mi355_wait(h)
            except Exception:  # interpreter shutdown
                pass
