"""ctypes binding of libjanusgpu (include/janus_gpu.h) — the same C ABI the C#/.NET host binds with
[DllImport("janusgpu")].  No torch types cross it: plain pointers and sizes.

There is no fallback: if the HIP library is missing or the device is not gfx950, every entry point
raises.  Arrays are numpy; the library copies them during the call (caller-owned host memory).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

_PKG = Path(__file__).resolve().parent.parent  # janus-crdt_amd/
LIB_PATH = Path(os.environ.get("JANUS_GPU_LIB", _PKG / "lib" / "libjanusgpu.so"))

JG_OK, JG_EINVAL, JG_ENOMEM, JG_EOVERFLOW, JG_ETYPE, JG_EHIP, JG_ESTATE = range(7)
NULL_ELEM = 0xFFFFFFFF
REC_DTYPE = np.dtype([("key", "<u8"), ("tag_lo", "<u8"), ("tag_hi", "<u8"), ("ord", "<u8")])  # jg_tagrec

# Every entry point include/janus_gpu.h declares (tests check the .so exports all of them).
EXPORTS = [
    "jg_abi_version", "jg_open", "jg_close", "jg_last_error", "jg_fence", "jg_stream",
    "jg_pnc_create", "jg_pnc_destroy", "jg_pnc_write_rows", "jg_pnc_read_rows", "jg_pnc_merge_rows",
    "jg_pnc_apply_ops", "jg_pnc_values",
    "jg_rows_create", "jg_rows_destroy", "jg_rows_upload", "jg_pnc_merge_batch",
    "jg_orset_create", "jg_orset_destroy", "jg_orset_load", "jg_orset_size", "jg_orset_read",
    "jg_orset_merge", "jg_orset_merge_store", "jg_orset_union", "jg_orset_contains", "jg_orset_apply_ops",
    "jg_synth_pnc_store", "jg_synth_pnc_rows", "jg_synth_orset",
    "jg_pnc_intern", "jg_pnc_columns", "jg_pnc_merge_json",
    "jg_wave_create", "jg_wave_destroy", "jg_wave_upload", "jg_pnc_merge_wave", "jg_host_alloc", "jg_host_free",
    "jg_pnc_wave_begin", "jg_pnc_wave_append", "jg_pnc_wave_commit", "jg_pnc_wave_abort",
    "jg_orset_lookup_all", "jg_pnc_encode_json", "jg_pnc_encode_json_before", "jg_pnc_apply_ops_rewind", "jg_pnc_apply_ops_encode", "jg_orset_encode_json", "jg_orset_apply_ops_ords",
    "jg_rows_route", "jg_pnc_merge_device", "jg_orset_route", "jg_orset_merge_device", "jg_orset_read_sets",
    "jg_orset_names_sync", "jg_orset_wave_begin", "jg_orset_wave_append", "jg_orset_wave_check", "jg_orset_wave_commit",
    "jg_orset_wave_abort", "jg_orset_wave_names", "jg_orset_names_since", "jg_orset_merge_json",
    "jg_update_digests", "jg_wave_update_digests", "jg_waves_update_digests", "jg_wave_sha256", "jg_sha256_batch", "jg_update_digests_of",
    "jg_node_create", "jg_node_destroy", "jg_node_register", "jg_node_set_shard", "jg_shard_of", "jg_node_last_stats",
    "jg_tracker_create", "jg_tracker_destroy", "jg_tracker_add", "jg_tracker_size", "jg_tracker_contains",
    "jg_apply_committed", "jg_apply_block", "jg_apply_stream_begin", "jg_apply_stream_append", "jg_apply_stream_end",
    "jg_comm_unique_id", "jg_comm_init", "jg_comm_destroy", "jg_pnc_exchange", "jg_orset_exchange", "jg_comm_last_stats",
    "jg_comm_init_host", "jg_exchange_plan", "jg_global_key",
]

_u8p = C.POINTER(C.c_uint8)
_vp = C.c_void_p
_u64 = C.c_uint64
_u32 = C.c_uint32
_SIGS = {
    "jg_abi_version": ([], C.c_int),
    "jg_open": ([C.c_int, C.POINTER(_vp)], C.c_int),
    "jg_close": ([_vp], C.c_int),
    "jg_last_error": ([C.c_char_p, C.c_size_t], C.c_int),
    "jg_fence": ([_vp], C.c_int),
    "jg_stream": ([_vp, C.POINTER(_vp)], C.c_int),
    "jg_pnc_create": ([_vp, _u64, _u32, _u32, C.POINTER(_vp)], C.c_int),
    "jg_pnc_destroy": ([_vp], C.c_int),
    "jg_pnc_write_rows": ([_vp, _vp, _u64, _vp, _vp], C.c_int),
    "jg_pnc_read_rows": ([_vp, _vp, _u64, _vp, _vp], C.c_int),
    "jg_pnc_merge_rows": ([_vp, _vp, _u64, _vp, _vp], C.c_int),
    "jg_pnc_apply_ops": ([_vp, _u64, _vp, _vp, _vp, _vp], C.c_int),
    "jg_pnc_values": ([_vp, _vp, _u64, _vp, _vp], C.c_int),
    "jg_rows_create": ([_vp, _u64, _u32, _u32, C.POINTER(_vp)], C.c_int),
    "jg_rows_destroy": ([_vp], C.c_int),
    "jg_rows_upload": ([_vp, _vp, _vp, _vp], C.c_int),
    "jg_pnc_merge_batch": ([_vp, _vp, C.c_int], C.c_int),
    "jg_orset_create": ([_vp, _u64, _u64, C.POINTER(_vp)], C.c_int),
    "jg_orset_destroy": ([_vp], C.c_int),
    "jg_orset_load": ([_vp, _vp, _u64, _vp, _u64], C.c_int),
    "jg_orset_size": ([_vp, C.POINTER(_u64), C.POINTER(_u64)], C.c_int),
    "jg_orset_read": ([_vp, _vp, _u64, _vp, _u64], C.c_int),
    "jg_orset_merge": ([_vp, _vp, _u64, _vp, _u64], C.c_int),
    "jg_orset_merge_store": ([_vp, _vp, C.c_int], C.c_int),
    "jg_orset_union": ([_vp, _vp, _vp, C.c_int], C.c_int),
    "jg_orset_contains": ([_vp, _vp, _vp, _u64, _vp], C.c_int),
    "jg_orset_apply_ops": ([_vp, _u64, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "jg_synth_pnc_store": ([_vp, _u64], C.c_int),
    "jg_synth_pnc_rows": ([_vp, _u64, _u64], C.c_int),
    "jg_synth_orset": ([_vp, _u64, _u64, _u32, _u32, _u32, _u32, _u32], C.c_int),
    "jg_pnc_intern": ([_vp, _u64, _vp, _vp, _vp], C.c_int),
    "jg_pnc_columns": ([_vp, _u64, _vp, _vp, _vp], C.c_int),
    "jg_pnc_merge_json": ([_vp, _u64, _vp, _vp, _vp, C.POINTER(_u64)], C.c_int),
    "jg_wave_create": ([_vp, _u64, _u64, C.POINTER(_vp)], C.c_int),
    "jg_wave_destroy": ([_vp], C.c_int),
    "jg_update_digests": ([_vp, _u64, _vp, _vp, _vp, _u64, _vp, _vp, _vp], C.c_int),
    "jg_wave_update_digests": ([_vp, _u64, _vp, _vp, _vp], C.c_int),
    "jg_waves_update_digests": ([_vp, _u64, _vp, _vp, _vp], C.c_int),
    "jg_wave_sha256": ([_vp, _vp, C.c_uint8], C.c_int),
    "jg_sha256_batch": ([_vp, _u64, _vp, _vp, _vp], C.c_int),
    "jg_update_digests_of": ([_vp, _u64, _vp, _vp, _u64, _vp, _vp], C.c_int),
    "jg_wave_upload": ([_vp, _u64, _vp, _vp, _vp], C.c_int),
    "jg_pnc_merge_wave": ([_vp, _vp, C.POINTER(_u64)], C.c_int),
    "jg_host_alloc": ([_vp, _u64, C.POINTER(_vp)], C.c_int),
    "jg_host_free": ([_vp], C.c_int),
    "jg_pnc_wave_begin": ([_vp, _u64, _u64], C.c_int),
    "jg_pnc_wave_append": ([_vp, _u64, _vp, _vp, _vp], C.c_int),
    "jg_pnc_wave_commit": ([_vp, C.POINTER(_u64)], C.c_int),
    "jg_pnc_wave_abort": ([_vp], C.c_int),
    "jg_orset_lookup_all": ([_vp, _u64, _vp, _vp, _vp, _u64], C.c_int),
    "jg_pnc_encode_json": ([_vp, _u64, _vp, _vp, _vp, _u64], C.c_int),
    "jg_pnc_encode_json_before": ([_vp, _u64, _vp, C.c_uint32, _vp, _vp, _vp, _vp, _u64, _vp], C.c_int),
    "jg_pnc_apply_ops_rewind": ([_vp, _u64, _vp, C.c_uint32, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "jg_pnc_apply_ops_encode": ([_vp, _u64, _vp, C.c_uint32, _vp, _vp, _vp, _vp, _u64, _vp], C.c_int),
    "jg_orset_encode_json": ([_vp, _u64, _vp, _vp, _vp, _vp, _vp, _u64, _vp], C.c_int),
    "jg_orset_apply_ops_ords": ([_vp, _u64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "jg_rows_route": ([_vp, _u32, _vp, _vp, _vp, _vp, _u64], C.c_int),
    "jg_pnc_merge_device": ([_vp, _u64, _vp, _vp, _vp], C.c_int),
    "jg_orset_route": ([_vp, _u32, _vp, _vp, _vp, _vp, _vp, _u64, _vp, _vp, _vp, _u64], C.c_int),
    "jg_orset_merge_device": ([_vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "jg_orset_read_sets": ([_vp, _u64, _vp, _vp, _vp, _u64, _vp, _vp, _u64], C.c_int),
    "jg_orset_names_sync": ([_vp, _u64, _vp, _vp, _vp, _u64, _vp, _vp, _vp, _vp], C.c_int),
    "jg_orset_wave_begin": ([_vp, _u64, _u64], C.c_int),
    "jg_orset_wave_append": ([_vp, _u64, _vp, _vp, _vp], C.c_int),
    "jg_orset_wave_check": ([_vp, C.POINTER(_u64)], C.c_int),
    "jg_orset_wave_commit": ([_vp, _u64], C.c_int),
    "jg_orset_wave_abort": ([_vp], C.c_int),
    "jg_orset_wave_names": ([_vp, C.POINTER(_u64), C.POINTER(_u64), _vp, _vp, _vp, _vp], C.c_int),
    "jg_orset_names_since": ([_vp, _u64, C.POINTER(_u64), C.POINTER(_u64), _vp, _vp, _vp, _vp], C.c_int),
    "jg_orset_merge_json": ([_vp, _u64, _vp, _vp, _vp, C.POINTER(_u64)], C.c_int),
    "jg_node_create": ([_vp, _vp, C.POINTER(_vp)], C.c_int),
    "jg_node_destroy": ([_vp], C.c_int),
    "jg_node_register": ([_vp, _u64, _vp, _vp, _vp], C.c_int),
    "jg_node_set_shard": ([_vp, _u32, _u32], C.c_int),
    "jg_shard_of": ([_vp, _u32, C.POINTER(_u32)], C.c_int),
    "jg_node_last_stats": ([_vp, _vp], C.c_int),
    "jg_tracker_create": ([_vp, C.POINTER(_vp)], C.c_int),
    "jg_tracker_destroy": ([_vp], C.c_int),
    "jg_tracker_add": ([_vp, _u64, _vp, _vp], C.c_int),
    "jg_tracker_size": ([_vp, C.POINTER(_u64)], C.c_int),
    "jg_tracker_contains": ([_vp, _u64, _vp, _vp], C.c_int),
    "jg_apply_committed": ([_vp, _vp, _vp, _vp, C.POINTER(_u64), C.POINTER(_u64)], C.c_int),
    "jg_apply_block": ([_vp, _vp, C.POINTER(_u64)], C.c_int),
    "jg_apply_stream_begin": ([_vp, _vp, _u64, _u64], C.c_int),
    "jg_apply_stream_append": ([_vp, _vp], C.c_int),
    "jg_apply_stream_end": ([_vp, _vp, C.POINTER(_u64), C.POINTER(_u64)], C.c_int),
    "jg_comm_unique_id": ([_vp], C.c_int),
    "jg_comm_init": ([_vp, _u32, _u32, _vp, C.POINTER(_vp)], C.c_int),
    "jg_comm_init_host": ([_vp, _u32, _u32, _vp, _vp, C.POINTER(_vp)], C.c_int),
    "jg_exchange_plan": ([_u32, _u32, _u32, _vp, C.c_uint8, _vp, _vp, _vp, _vp], C.c_int),
    "jg_global_key": ([_vp, _u32, _u32, C.POINTER(_u32)], C.c_int),
    "jg_comm_destroy": ([_vp], C.c_int),
    "jg_pnc_exchange": ([_vp, _vp, _vp, _vp, _vp], C.c_int),
    "jg_orset_exchange": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "jg_comm_last_stats": ([_vp, _vp], C.c_int),
}
GUID_DTYPE = np.dtype([("lo", "<u8"), ("hi", "<u8")])  # jg_guid


class JanusError(RuntimeError):
    def __init__(self, code: int, msg: str, bad_msg: int | None = None):
        super().__init__(f"[{code}] {msg}")
        self.code = code
        self.bad_msg = bad_msg  # jg_pnc_merge_json / merge_wave: first rejected message


_lib: C.CDLL | None = None


def load(path: str | os.PathLike | None = None) -> C.CDLL:
    """Load libjanusgpu.so (raises if it was not built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise FileNotFoundError(f"libjanusgpu not built: {p} (run __graft_entry__.build())")
    lib = C.CDLL(str(p))
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if path is None:
        _lib = lib
    return lib


def _check(rc: int, bad_msg: int | None = None) -> None:
    if rc != JG_OK:
        buf = C.create_string_buffer(1024)
        load().jg_last_error(buf, 1024)
        raise JanusError(rc, buf.value.decode(errors="replace"), bad_msg)


def pack_wave(msgs) -> tuple[np.ndarray, np.ndarray]:
    """Concatenate encoded messages (bytes) into (payload u8, offsets u64[n+1])."""
    off = np.zeros(len(msgs) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs], dtype=np.uint64) if msgs else []
    data = np.frombuffer(b"".join(msgs), np.uint8) if msgs else np.zeros(0, np.uint8)
    return np.ascontiguousarray(data), off


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(_vp)


def _arr(a, dtype) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=dtype)


class Context:
    """One device + one HIP stream (jg_open)."""

    def __init__(self, device: int = 0):
        self._h = _vp()
        _check(load().jg_open(device, C.byref(self._h)))
        self.device = device

    @property
    def handle(self):
        return self._h

    def fence(self) -> None:
        _check(load().jg_fence(self._h))

    def stream(self) -> int:
        s = _vp()
        _check(load().jg_stream(self._h, C.byref(s)))
        return s.value or 0

    def close(self) -> None:
        if self._h:
            _check(load().jg_close(self._h))
            self._h = _vp()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def _elem_dtype(eb: int):
    return np.int32 if eb == 4 else np.int64


class Rows:
    """Device-resident batch of received PN-Counter rows (jg_rows)."""

    def __init__(self, ctx: Context, n_rows: int, n_replicas: int, elem_bytes: int = 8):
        self.ctx, self.n_rows, self.R, self.eb = ctx, n_rows, n_replicas, elem_bytes
        self._h = _vp()
        _check(load().jg_rows_create(ctx.handle, n_rows, n_replicas, elem_bytes, C.byref(self._h)))

    def upload(self, P, N, key_idx=None) -> None:
        dt = _elem_dtype(self.eb)
        P, N = _arr(P, dt), _arr(N, dt)
        assert P.size == N.size == self.n_rows * self.R
        k = None if key_idx is None else _arr(key_idx, np.uint32)
        _check(load().jg_rows_upload(self._h, _ptr(k), _ptr(P), _ptr(N)))

    def synth(self, seed: int, key0: int = 0) -> None:
        _check(load().jg_synth_pnc_rows(self._h, seed, key0))

    def route(self, world: int, d_keys: int, d_P: int, d_N: int, cap_rows: int | None = None) -> np.ndarray:
        """jg_rows_route: stable partition of the batch by owner rank (key % world) into caller DEVICE
        buffers (raw addresses); returns the rows per destination."""
        counts = np.zeros(world, np.uint64)
        _check(load().jg_rows_route(self._h, world, _ptr(counts), d_keys, d_P, d_N, self.n_rows if cap_rows is None else cap_rows))
        return counts

    def close(self) -> None:
        if self._h:
            _check(load().jg_rows_destroy(self._h))
            self._h = _vp()


class PNCStore:
    """PN-Counter store [n_keys x n_replicas] (jg_pnc)."""

    ABSENT = {4: np.iinfo(np.int32).min, 8: np.iinfo(np.int64).min}

    def __init__(self, ctx: Context, n_keys: int, n_replicas: int, elem_bytes: int = 8):
        self.ctx, self.n_keys, self.R, self.eb = ctx, n_keys, n_replicas, elem_bytes
        self.dtype = _elem_dtype(elem_bytes)
        self._h = _vp()
        _check(load().jg_pnc_create(ctx.handle, n_keys, n_replicas, elem_bytes, C.byref(self._h)))

    def _rows(self, P, N):
        P, N = _arr(P, self.dtype), _arr(N, self.dtype)
        if P.shape != N.shape or P.size % self.R:
            raise ValueError("P/N must be [n_rows x R] of the store's width")
        return P, N, P.size // self.R

    def write_rows(self, P, N, key_idx=None) -> None:
        P, N, n = self._rows(P, N)
        k = None if key_idx is None else _arr(key_idx, np.uint32)
        _check(load().jg_pnc_write_rows(self._h, _ptr(k), n, _ptr(P), _ptr(N)))

    def read_rows(self, key_idx=None, n: int | None = None):
        k = None if key_idx is None else _arr(key_idx, np.uint32)
        n = (self.n_keys if n is None else n) if k is None else k.size
        P = np.empty((n, self.R), self.dtype)
        N = np.empty((n, self.R), self.dtype)
        _check(load().jg_pnc_read_rows(self._h, _ptr(k), n, _ptr(P), _ptr(N)))
        return P, N

    def merge_rows(self, P, N, key_idx=None) -> None:
        P, N, n = self._rows(P, N)
        k = None if key_idx is None else _arr(key_idx, np.uint32)
        _check(load().jg_pnc_merge_rows(self._h, _ptr(k), n, _ptr(P), _ptr(N)))

    def merge_batch(self, rows: Rows, async_: bool = False) -> None:
        _check(load().jg_pnc_merge_batch(self._h, rows._h, 1 if async_ else 0))

    def merge_device(self, n_rows: int, d_keys: int, d_P: int, d_N: int) -> None:
        """jg_pnc_merge_device: merge rows held in caller DEVICE memory (raw addresses)."""
        _check(load().jg_pnc_merge_device(self._h, n_rows, d_keys, d_P, d_N))

    def apply_ops(self, key, col, delta, is_n) -> None:
        key, col = _arr(key, np.uint32), _arr(col, np.uint32)
        delta, is_n = _arr(delta, np.int64), _arr(is_n, np.uint8)
        _check(load().jg_pnc_apply_ops(self._h, key.size, _ptr(key), _ptr(col), _ptr(delta), _ptr(is_n)))

    def values(self, key_idx=None, n: int | None = None):
        k = None if key_idx is None else _arr(key_idx, np.uint32)
        n = (self.n_keys if n is None else n) if k is None else k.size
        out = np.empty(n, np.int64)
        ovf = np.empty(n, np.uint8)
        _check(load().jg_pnc_values(self._h, _ptr(k), n, _ptr(out), _ptr(ovf)))
        return out, ovf

    def synth(self, seed: int) -> None:
        _check(load().jg_synth_pnc_store(self._h, seed))

    # ---- replica table + wire-format apply (json.hip) ----
    def intern(self, key_idx, lo, hi) -> np.ndarray:
        k = _arr(key_idx, np.uint32)
        g = np.empty(k.size, GUID_DTYPE)
        g["lo"], g["hi"] = lo, hi
        out = np.empty(k.size, np.uint32)
        _check(load().jg_pnc_intern(self._h, k.size, _ptr(k), _ptr(g), _ptr(out)))
        return out

    def columns(self, key_idx):
        """(guids [n x R] of GUID_DTYPE, ncols [n])."""
        k = _arr(key_idx, np.uint32)
        g = np.zeros((k.size, self.R), GUID_DTYPE)
        n = np.empty(k.size, np.uint32)
        _check(load().jg_pnc_columns(self._h, k.size, _ptr(k), _ptr(g), _ptr(n)))
        return g, n

    def merge_json(self, key_idx, msgs=None, data=None, off=None) -> None:
        """Apply encoded PNCounterMsg payloads (list of bytes, or packed data + off)."""
        if msgs is not None:
            data, off = pack_wave(msgs)
        k = _arr(key_idx, np.uint32)
        data, off = _arr(data, np.uint8), _arr(off, np.uint64)
        bad = _u64(0)
        rc = load().jg_pnc_merge_json(self._h, k.size, _ptr(k), _ptr(off), _ptr(data) if data.size else _ptr(np.zeros(16, np.uint8)),
                                      C.byref(bad))
        _check(rc, bad.value)

    # streamed wave: begin, append chunks (their buffers are kept alive here until commit/abort)
    def wave_begin(self, cap_msgs: int = 0, cap_bytes: int = 0) -> None:
        self._chunks = []
        _check(load().jg_pnc_wave_begin(self._h, cap_msgs, cap_bytes))

    def wave_append(self, key_idx, msgs) -> None:
        data, off = pack_wave(msgs)
        k = _arr(key_idx, np.uint32)
        data = data if data.size else np.zeros(16, np.uint8)
        self._chunks.append((k, data, off))
        _check(load().jg_pnc_wave_append(self._h, k.size, _ptr(k), _ptr(off), _ptr(data)))

    def wave_commit(self) -> None:
        bad = _u64(0)
        rc = load().jg_pnc_wave_commit(self._h, C.byref(bad))
        self._chunks = []
        _check(rc, bad.value)

    def wave_abort(self) -> None:
        _check(load().jg_pnc_wave_abort(self._h))
        self._chunks = []

    def encode_json(self, key_idx) -> list:
        """GetLastSynchronizedUpdate().Encode() of each row (jg_pnc_encode_json): list of bytes."""
        k = _arr(key_idx, np.uint32)
        off = np.zeros(k.size + 1, np.uint64)
        _check(load().jg_pnc_encode_json(self._h, k.size, _ptr(k), _ptr(off), None, 0))
        out = np.empty(max(16, int(off[-1])), np.uint8)
        _check(load().jg_pnc_encode_json(self._h, k.size, _ptr(k), _ptr(off), _ptr(out), out.size))
        b = out.tobytes()
        return [b[int(off[i]):int(off[i + 1])] for i in range(k.size)]

    def apply_ops_rewind(self, key, delta, is_n, need, col=0):
        """jg_pnc_apply_ops_rewind: apply the ops to column `col`; for each op with need[i], in op order, the amounts
        the later ops on its key added to P and N (the rewind jg_pnc_encode_json_before takes)."""
        key, delta = _arr(key, np.uint32), _arr(delta, np.int64)
        is_n, need = _arr(is_n, np.uint8), _arr(need, np.uint8)
        k = int(np.count_nonzero(need))
        dp, dn = np.zeros(max(1, k), np.int64), np.zeros(max(1, k), np.int64)
        _check(load().jg_pnc_apply_ops_rewind(self._h, key.size, _ptr(key), col, _ptr(delta), _ptr(is_n), _ptr(need), _ptr(dp), _ptr(dn)))
        return dp[:k], dn[:k]

    def apply_ops_encode(self, key, delta, is_n, col=0, cap=None):
        """jg_pnc_apply_ops_encode: op i's snapshot (the key's row right after op i) for every op, as bytes, with
        its SHA-256 (u8[n, 32]); the ops applied.  `cap` (bytes) forces a small output buffer (JG_ESTATE: nothing
        applied)."""
        key, delta, is_n = _arr(key, np.uint32), _arr(delta, np.int64), _arr(is_n, np.uint8)
        n = key.size
        off = np.zeros(n + 1, np.uint64)
        out = np.empty(max(16, n * 512 if cap is None else cap), np.uint8)
        h = np.zeros((max(1, n), 32), np.uint8)
        call = lambda: load().jg_pnc_apply_ops_encode(self._h, n, _ptr(key), col, _ptr(delta), _ptr(is_n), _ptr(off), _ptr(out),
                                                      out.size if cap is None else cap, _ptr(h))
        rc = call()
        if rc == JG_ESTATE and cap is None and int(off[-1]) > out.size:  # nothing applied: again with room for every byte
            out = np.empty(int(off[-1]), np.uint8)
            rc = call()
        _check(rc)
        b = out[:int(off[-1])].tobytes()
        return [b[int(off[i]):int(off[i + 1])] for i in range(n)], h[:n]

    def encode_json_before(self, key_idx, dp, dn, col=0, sha=False):
        """jg_pnc_encode_json_before: each row as it stood before its last dp[i] / dn[i] of increments to `col`
        (list of bytes; with sha=True also each state's SHA-256, u8[n, 32])."""
        k = _arr(key_idx, np.uint32)
        p, q = _arr(dp, np.int64), _arr(dn, np.int64)
        off = np.zeros(k.size + 1, np.uint64)
        _check(load().jg_pnc_encode_json_before(self._h, k.size, _ptr(k), col, _ptr(p), _ptr(q), _ptr(off), None, 0, None))
        out = np.empty(max(16, int(off[-1])), np.uint8)
        h = np.zeros((k.size, 32), np.uint8) if sha else None
        _check(load().jg_pnc_encode_json_before(self._h, k.size, _ptr(k), col, _ptr(p), _ptr(q), _ptr(off), _ptr(out), out.size,
                                                _ptr(h) if sha else None))
        b = out.tobytes()
        states = [b[int(off[i]):int(off[i + 1])] for i in range(k.size)]
        return (states, h) if sha else states

    def merge_wave(self, wave: "Wave") -> None:
        bad = _u64(0)
        rc = load().jg_pnc_merge_wave(self._h, wave._h, C.byref(bad))
        _check(rc, bad.value)

    def close(self) -> None:
        if self._h:
            _check(load().jg_pnc_destroy(self._h))
            self._h = _vp()


class Wave:
    """Device-resident wave of encoded state messages (jg_wave)."""

    def __init__(self, ctx: Context, cap_msgs: int, cap_bytes: int):
        self.ctx = ctx
        self._h = _vp()
        _check(load().jg_wave_create(ctx.handle, cap_msgs, cap_bytes, C.byref(self._h)))

    def upload(self, key_idx, msgs=None, data=None, off=None) -> None:
        if msgs is not None:
            data, off = pack_wave(msgs)
        k = _arr(key_idx, np.uint32)
        data, off = _arr(data, np.uint8), _arr(off, np.uint64)
        _check(load().jg_wave_upload(self._h, k.size, _ptr(k), _ptr(off), _ptr(data)))

    def update_digests(self, first, msg_digests: bool = False):
        """UpdateMessage.ComputeDigest for updates [first[u], first[u+1]) of this wave (jg_wave_update_digests):
        returns digests u8[n_updates, 32] (and the per-message SHA-256s u8[n, 32] if msg_digests)."""
        first = _arr(first, np.uint64)
        nu = first.size - 1
        dig = np.zeros((max(nu, 0), 32), np.uint8)
        md = np.zeros((int(first[-1]), 32), np.uint8) if msg_digests else None
        _check(load().jg_wave_update_digests(self._h, nu, _ptr(first), _ptr(md), _ptr(dig)))
        return (dig, md) if msg_digests else dig

    def sha256_device(self, d_out: int, async_: bool = False) -> None:
        """SHA-256 of every payload into device memory at address d_out (jg_wave_sha256)."""
        _check(load().jg_wave_sha256(self._h, _vp(d_out), 1 if async_ else 0))

    def close(self) -> None:
        if self._h:
            _check(load().jg_wave_destroy(self._h))
            self._h = _vp()


def waves_update_digests(waves, firsts):
    """UpdateMessage.ComputeDigest over several device-resident waves in one pipelined call
    (jg_waves_update_digests): wave k's UpdateMessages are firsts[k] (as in Wave.update_digests).
    Returns one u8[n_updates_k, 32] array per wave."""
    firsts = [_arr(f, np.uint64) for f in firsts]
    n = len(waves)
    if len(firsts) != n:
        raise ValueError("waves_update_digests: one first[] per wave")
    nu = np.array([f.size - 1 for f in firsts], np.uint64)
    digs = [np.zeros((int(k), 32), np.uint8) for k in nu]
    hw = (_vp * max(n, 1))(*[w._h for w in waves])
    fp = (_vp * max(n, 1))(*[_vp(f.ctypes.data) for f in firsts])
    dp = (_vp * max(n, 1))(*[_vp(d.ctypes.data) for d in digs])
    _check(load().jg_waves_update_digests(hw, n, _ptr(nu), fp, dp))
    return digs


def update_digests(ctx: Context, msgs, first, msg_digests: bool = False):
    """UpdateMessage.ComputeDigest (DAGUpdateMessage.cs:32-55) on the device (jg_update_digests).
    msgs: NetworkProtocol.message payloads (bytes, or None for a C# null); update u holds
    msgs[first[u]:first[u+1]].  Returns digests u8[n_updates, 32] (and u8[n, 32] per message)."""
    is_null = np.array([m is None for m in msgs], np.uint8)
    data, off = pack_wave([b"" if m is None else m for m in msgs])
    first = _arr(first, np.uint64)
    nu = first.size - 1
    dig = np.zeros((max(nu, 0), 32), np.uint8)
    md = np.zeros((len(msgs), 32), np.uint8) if msg_digests else None
    _check(load().jg_update_digests(ctx.handle, len(msgs), _ptr(off), _ptr(data), _ptr(is_null) if is_null.any() else None, nu,
                                    _ptr(first), _ptr(md), _ptr(dig)))
    return (dig, md) if msg_digests else dig


def sha256_batch(ctx: Context, msgs) -> np.ndarray:
    """SHA-256 of every payload (jg_sha256_batch): u8[n, 32]."""
    data, off = pack_wave(list(msgs))
    out = np.zeros((len(msgs), 32), np.uint8)
    _check(load().jg_sha256_batch(ctx.handle, len(msgs), _ptr(off), _ptr(data), _ptr(out)))
    return out


def update_digests_of(ctx: Context, msg_digests, first, is_null=None) -> np.ndarray:
    """ComputeDigest's second level from per-payload SHA-256s (jg_update_digests_of): u8[n_updates, 32]."""
    md = np.ascontiguousarray(msg_digests, np.uint8).reshape(-1, 32)
    first = _arr(first, np.uint64)
    nu = first.size - 1
    dig = np.zeros((max(nu, 0), 32), np.uint8)
    nl = None if is_null is None else np.ascontiguousarray(is_null, np.uint8)
    _check(load().jg_update_digests_of(ctx.handle, md.shape[0], _ptr(md), _ptr(nl) if nl is not None else None, nu, _ptr(first), _ptr(dig)))
    return dig


def records(key=None, tag_lo=None, tag_hi=None, n: int = 0, ord=None) -> np.ndarray:
    """jg_tagrec array; ord (arrival ordinal) defaults to the record's index."""
    r = np.zeros(n if key is None else len(key), REC_DTYPE)
    if key is not None:
        r["key"], r["tag_lo"], r["tag_hi"] = key, tag_lo, tag_hi
    r["ord"] = np.arange(r.size, dtype=np.uint64) if ord is None else ord
    return r


class ORSetStore:
    """OR-Set store: sorted add and tombstone tag-record streams (jg_orset)."""

    def __init__(self, ctx: Context, cap_add: int = 0, cap_rem: int = 0):
        self.ctx = ctx
        self._h = _vp()
        _check(load().jg_orset_create(ctx.handle, cap_add, cap_rem, C.byref(self._h)))

    def load(self, add, rem) -> None:
        add, rem = _arr(add, REC_DTYPE), _arr(rem, REC_DTYPE)
        _check(load().jg_orset_load(self._h, _ptr(add), add.size, _ptr(rem), rem.size))

    def size(self):
        a, r = _u64(), _u64()
        _check(load().jg_orset_size(self._h, C.byref(a), C.byref(r)))
        return a.value, r.value

    def read(self):
        na, nr = self.size()
        add, rem = np.empty(na, REC_DTYPE), np.empty(nr, REC_DTYPE)
        _check(load().jg_orset_read(self._h, _ptr(add), na, _ptr(rem), nr))
        return add, rem

    def merge(self, add, rem) -> None:
        add, rem = _arr(add, REC_DTYPE), _arr(rem, REC_DTYPE)
        _check(load().jg_orset_merge(self._h, _ptr(add), add.size, _ptr(rem), rem.size))

    def merge_store(self, src: "ORSetStore", async_: bool = False) -> None:
        _check(load().jg_orset_merge_store(self._h, src._h, 1 if async_ else 0))

    @staticmethod
    def union(a: "ORSetStore", b: "ORSetStore", out: "ORSetStore", async_: bool = False) -> None:
        _check(load().jg_orset_union(a._h, b._h, out._h, 1 if async_ else 0))

    ADD, REMOVE, CLEAR = 1, 2, 3

    def apply_ops(self, set_ids, elems, ops, tag_lo, tag_hi) -> np.ndarray:
        """ORSet.Add/Remove/Clear in order (jg_orset_apply_ops); returns each op's bool result."""
        s, e = _arr(set_ids, np.uint32), _arr(elems, np.uint32)
        o = _arr(ops, np.uint8)
        lo, hi = _arr(tag_lo, np.uint64), _arr(tag_hi, np.uint64)
        out = np.empty(s.size, np.uint8)
        _check(load().jg_orset_apply_ops(self._h, s.size, _ptr(s), _ptr(e), _ptr(o), _ptr(lo), _ptr(hi), _ptr(out)))
        return out

    def apply_ops_ords(self, set_ids, elems, ops, tag_lo, tag_hi):
        """jg_orset_apply_ops_ords: (results, add_lim, rem_lim) — per op the ord limits of its set's snapshot right after it."""
        s, e = _arr(set_ids, np.uint32), _arr(elems, np.uint32)
        o = _arr(ops, np.uint8)
        lo, hi = _arr(tag_lo, np.uint64), _arr(tag_hi, np.uint64)
        out = np.empty(s.size, np.uint8)
        al, rl = np.zeros(s.size, np.uint64), np.zeros(s.size, np.uint64)
        _check(load().jg_orset_apply_ops_ords(self._h, s.size, _ptr(s), _ptr(e), _ptr(o), _ptr(lo), _ptr(hi), _ptr(out), _ptr(al), _ptr(rl)))
        return out, al, rl

    def encode_json(self, set_ids, add_lim=None, rem_lim=None, sha=False):
        """ORSetMsg.Encode() of each set on the device (jg_orset_encode_json), optionally as of ord limits: list of bytes
        (with sha=True also each state's SHA-256, u8[n, 32])."""
        s = _arr(set_ids, np.uint32)
        al = None if add_lim is None else _arr(add_lim, np.uint64)
        rl = None if rem_lim is None else _arr(rem_lim, np.uint64)
        off = np.zeros(s.size + 1, np.uint64)
        args = (_ptr(al) if al is not None else None, _ptr(rl) if rl is not None else None)
        _check(load().jg_orset_encode_json(self._h, s.size, _ptr(s), *args, _ptr(off), None, 0, None))
        out = np.empty(max(16, int(off[-1])), np.uint8)
        h = np.zeros((s.size, 32), np.uint8) if sha else None
        _check(load().jg_orset_encode_json(self._h, s.size, _ptr(s), *args, _ptr(off), _ptr(out), out.size, _ptr(h) if sha else None))
        b = out.tobytes()
        states = [b[int(off[i]):int(off[i + 1])] for i in range(s.size)]
        return (states, h) if sha else states

    def contains(self, set_ids, elems) -> np.ndarray:
        s, e = _arr(set_ids, np.uint32), _arr(elems, np.uint32)
        out = np.empty(s.size, np.uint8)
        _check(load().jg_orset_contains(self._h, _ptr(s), _ptr(e), s.size, _ptr(out)))
        return out

    def read_sets(self, set_ids):
        """Records of whole sets (jg_orset_read_sets): list of (adds, tombstones) per set."""
        s = _arr(set_ids, np.uint32)
        ao, ro = np.zeros(s.size + 1, np.uint64), np.zeros(s.size + 1, np.uint64)
        _check(load().jg_orset_read_sets(self._h, s.size, _ptr(s), _ptr(ao), None, 0, _ptr(ro), None, 0))
        a, r = np.empty(max(1, int(ao[-1])), REC_DTYPE), np.empty(max(1, int(ro[-1])), REC_DTYPE)
        _check(load().jg_orset_read_sets(self._h, s.size, _ptr(s), _ptr(ao), _ptr(a), a.size, _ptr(ro), _ptr(r), r.size))
        return [(a[int(ao[i]):int(ao[i + 1])], r[int(ro[i]):int(ro[i + 1])]) for i in range(s.size)]

    # ---- wire-format apply (jg_orset_wave_*, csrc/orset_wire.hip) ----
    def names_sync(self, sets=(), next_ids=(), cleared=(), names=()) -> None:
        """jg_orset_names_sync: per-set (next id, Clear flag), then live names [(set, id, bytes)]."""
        s, nx, cl = _arr(sets, np.uint32), _arr(next_ids, np.uint32), _arr(cleared, np.uint8)
        ns = _arr([x[0] for x in names], np.uint32)
        ni = _arr([x[1] for x in names], np.uint32)
        data, off = pack_wave([x[2] for x in names])
        data = data if data.size else np.zeros(16, np.uint8)
        _check(load().jg_orset_names_sync(self._h, s.size, _ptr(s), _ptr(nx), _ptr(cl), ns.size, _ptr(ns), _ptr(ni), _ptr(off), _ptr(data)))

    def merge_json(self, set_ids, msgs) -> None:
        """Apply ORSetMsg payloads (list of bytes) of sets set_ids (jg_orset_merge_json): all or nothing."""
        data, off = pack_wave(msgs)
        s = _arr(set_ids, np.uint32)
        data = data if data.size else np.zeros(16, np.uint8)
        bad = _u64(0)
        rc = load().jg_orset_merge_json(self._h, s.size, _ptr(s), _ptr(off), _ptr(data), C.byref(bad))
        _check(rc, bad.value)

    def wave(self, chunks, limit=None):
        """Streamed wave: chunks = [(set_ids, msgs)]; check, then commit(limit or the first bad message).
        Returns (check code, bad message or None)."""
        n = sum(len(c[1]) for c in chunks)
        keep = []
        _check(load().jg_orset_wave_begin(self._h, n, sum(len(m) for c in chunks for m in c[1])))
        for set_ids, msgs in chunks:
            data, off = pack_wave(msgs)
            s = _arr(set_ids, np.uint32)
            data = data if data.size else np.zeros(16, np.uint8)
            keep.append((s, data, off))
            _check(load().jg_orset_wave_append(self._h, s.size, _ptr(s), _ptr(off), _ptr(data)))
        bad = _u64(0)
        rc = load().jg_orset_wave_check(self._h, C.byref(bad))
        first_bad = None if bad.value == 2**64 - 1 else bad.value
        if rc != JG_OK and first_bad is None:  # the check itself failed (no message to cut at): nothing applies
            buf = C.create_string_buffer(1024)
            load().jg_last_error(buf, 1024)
            load().jg_orset_wave_abort(self._h)
            raise JanusError(rc, buf.value.decode(errors="replace"))
        lim = (n if first_bad is None else first_bad) if limit is None else limit
        _check(load().jg_orset_wave_commit(self._h, lim))
        return rc, first_bad

    def wave_names(self):
        """Element ids the last commit issued: list of (set, id, bytes), sorted by (set, id)."""
        n, nb = _u64(), _u64()
        _check(load().jg_orset_wave_names(self._h, C.byref(n), C.byref(nb), None, None, None, None))
        if n.value == 0:
            return []
        s, i = np.empty(n.value, np.uint32), np.empty(n.value, np.uint32)
        off, b = np.empty(n.value + 1, np.uint64), np.empty(max(1, nb.value), np.uint8)
        _check(load().jg_orset_wave_names(self._h, C.byref(n), C.byref(nb), _ptr(s), _ptr(i), _ptr(off), _ptr(b)))
        raw = b.tobytes()
        return [(int(s[k]), int(i[k]), raw[int(off[k]):int(off[k + 1])]) for k in range(n.value)]

    def names_since(self, start=0):
        """The store's names log from `start`: (end, list of (set, id, bytes)) in the order the table took them."""
        to, nb = _u64(), _u64()
        _check(load().jg_orset_names_since(self._h, start, C.byref(to), C.byref(nb), None, None, None, None))
        n = to.value - start
        if n == 0:
            return to.value, []
        s, i = np.empty(n, np.uint32), np.empty(n, np.uint32)
        off, b = np.empty(n + 1, np.uint64), np.empty(max(1, nb.value), np.uint8)
        _check(load().jg_orset_names_since(self._h, start, C.byref(to), C.byref(nb), _ptr(s), _ptr(i), _ptr(off), _ptr(b)))
        raw = b.tobytes()
        return to.value, [(int(s[k]), int(i[k]), raw[int(off[k]):int(off[k + 1])]) for k in range(n)]

    def lookup_all(self, set_ids):
        """ORSet.LookupAll of each set (jg_orset_lookup_all): list of uint32 arrays of elem ids."""
        s = _arr(set_ids, np.uint32)
        off = np.zeros(s.size + 1, np.uint64)
        _check(load().jg_orset_lookup_all(self._h, s.size, _ptr(s), _ptr(off), None, 0))
        out = np.empty(max(1, int(off[-1])), np.uint32)
        _check(load().jg_orset_lookup_all(self._h, s.size, _ptr(s), _ptr(off), _ptr(out), out.size))
        return [out[int(off[i]):int(off[i + 1])] for i in range(s.size)]

    def route(self, world: int, d_add_key: int, d_add_tag: int, d_add_ord: int, cap_add: int, d_rem_key: int, d_rem_tag: int,
              d_rem_ord: int, cap_rem: int):
        """jg_orset_route: both streams partitioned by owner rank (set % world, set ids rewritten to
        set // world) into caller DEVICE buffers (keys, tags, uint32 ords); returns (add counts,
        tombstone counts) per rank."""
        ca, cr = np.zeros(world, np.uint64), np.zeros(world, np.uint64)
        _check(load().jg_orset_route(self._h, world, _ptr(ca), _ptr(cr), d_add_key, d_add_tag, d_add_ord, cap_add, d_rem_key, d_rem_tag,
                                     d_rem_ord, cap_rem))
        return ca, cr

    def merge_device(self, add_counts, rem_counts, d_add_key: int, d_add_tag: int, d_add_ord: int, d_rem_key: int, d_rem_tag: int,
                     d_rem_ord: int) -> None:
        """jg_orset_merge_device: merge received runs (run r = add_counts[r] / rem_counts[r] records,
        stored run after run in caller DEVICE buffers), in run order."""
        ca, cr = _arr(add_counts, np.uint64), _arr(rem_counts, np.uint64)
        assert ca.size == cr.size
        _check(load().jg_orset_merge_device(self._h, ca.size, _ptr(ca), _ptr(cr), d_add_key, d_add_tag, d_add_ord, d_rem_key, d_rem_tag,
                                            d_rem_ord))

    def synth(self, seed, n_groups, elems_per_set, add_per_group, add_u0, rem_per_group, rem_u0) -> None:
        _check(load().jg_synth_orset(self._h, seed, n_groups, elems_per_set, add_per_group, add_u0, rem_per_group, rem_u0))

    def close(self) -> None:
        if self._h:
            _check(load().jg_orset_destroy(self._h))
            self._h = _vp()


# ---- the committed-wave apply loop (csrc/node.hip) -------------------------------------------------------
class Commit(C.Structure):
    """jg_commit: a committed wave in commit order (contiguous payloads: off + bytes)."""
    _fields_ = [("n", _u64), ("uid", _vp), ("type", _vp), ("seq", _vp), ("off", _vp), ("bytes", _vp), ("ptr", _vp), ("len", _vp)]


class ApplyStats(C.Structure):
    """jg_apply_stats."""
    _fields_ = [("gather_s", C.c_double), ("device_wait_s", C.c_double), ("total_s", C.c_double), ("device_busy_s", C.c_double),
                ("msgs_uploaded", _u64), ("bytes_uploaded", _u64), ("msgs_applied", _u64), ("chunks", _u64),
                ("chunk_busy_s", C.c_double), ("tail_busy_s", C.c_double),
                ("setup_s", C.c_double), ("loop_s", C.c_double)]


def shard_of(lo: int, hi: int, world: int) -> int:
    """jg_shard_of: the owner rank of key uid (lo, hi) among `world` GPUs."""
    g = np.zeros(1, GUID_DTYPE)
    g["lo"], g["hi"] = lo, hi
    r = _u32()
    _check(load().jg_shard_of(_ptr(g), world, C.byref(r)))
    return r.value


def global_key(lo: int, hi: int, world: int, local: int) -> int:
    """jg_global_key: the global key (row / set id the exchange routes by) of key uid (lo, hi) registered with
    local index `local` by its owner jg_shard_of(uid, world)."""
    g = np.zeros(1, GUID_DTYPE)
    g["lo"], g["hi"] = lo, hi
    r = _u32()
    _check(load().jg_global_key(_ptr(g), world, local, C.byref(r)))
    return r.value


def exchange_plan(rank: int, world: int, counts, skip_own: bool = False):
    """jg_exchange_plan: counts[src, dst, j] (uint64, world x world x k) -> (send_off, send_n, recv_off, recv_n),
    each [world, k] for this rank (pure host arithmetic: no device needed)."""
    c = np.ascontiguousarray(counts, np.uint64)
    assert c.ndim == 3 and c.shape[0] == c.shape[1] == world
    k = c.shape[2]
    out = [np.zeros((world, k), np.uint64) for _ in range(4)]
    _check(load().jg_exchange_plan(rank, world, k, _ptr(c), 1 if skip_own else 0, *(_ptr(x) for x in out)))
    return tuple(out)


class Tracker:
    """SafeCRDTManager.safeUpdateTracker on the device (jg_tracker)."""

    def __init__(self, ctx: Context):
        self._h = _vp()
        _check(load().jg_tracker_create(ctx.handle, C.byref(self._h)))

    def add(self, seq, origin) -> None:
        s, o = _arr(seq, np.uint64), _arr(origin, np.uint64)
        _check(load().jg_tracker_add(self._h, s.size, _ptr(s), _ptr(o)))

    def size(self) -> int:
        n = _u64()
        _check(load().jg_tracker_size(self._h, C.byref(n)))
        return n.value

    def contains(self, seq) -> np.ndarray:
        s = _arr(seq, np.uint64)
        out = np.zeros(s.size, np.uint8)
        _check(load().jg_tracker_contains(self._h, s.size, _ptr(s), _ptr(out)))
        return out

    def close(self) -> None:
        if self._h:
            _check(load().jg_tracker_destroy(self._h))
            self._h = _vp()


class PinnedBytes:
    """Page-locked host bytes (jg_host_alloc): a wave whose payloads sit here uploads without the library's
    gather (the `direct` path of jg_apply_committed)."""

    def __init__(self, ctx: Context, data):
        src = _arr(data, np.uint8)
        self._p = _vp()
        self.size = max(16, src.size)
        _check(load().jg_host_alloc(ctx.handle, self.size, C.byref(self._p)))
        self.array = np.ctypeslib.as_array(C.cast(self._p, C.POINTER(C.c_uint8)), shape=(self.size,))
        self.array[: src.size] = src

    def close(self) -> None:
        if self._p:
            _check(load().jg_host_free(self._p))
            self._p = _vp()


class Node:
    """A node's copy of its keys (jg_node) over a PN-Counter and/or an OR-Set store."""

    def __init__(self, pnc: PNCStore | None = None, orset: ORSetStore | None = None):
        self._h = _vp()
        self._stores = (pnc, orset)  # keep them alive
        _check(load().jg_node_create(pnc._h if pnc else None, orset._h if orset else None, C.byref(self._h)))

    def register(self, lo, hi, types, idx) -> None:
        g = np.empty(np.size(lo), GUID_DTYPE)
        g["lo"], g["hi"] = lo, hi
        t, i = _arr(types, np.uint8), _arr(idx, np.uint32)
        _check(load().jg_node_register(self._h, g.size, _ptr(g), _ptr(t), _ptr(i)))

    def set_shard(self, rank: int, world: int) -> None:
        _check(load().jg_node_set_shard(self._h, rank, world))

    def _commit(self, lo, hi, types, seqs, msgs=None, data=None, off=None, pinned=None):
        if msgs is not None:
            data, off = pack_wave(msgs)
        g = np.empty(np.size(lo), GUID_DTYPE)
        g["lo"], g["hi"] = lo, hi
        t = _arr(types, np.uint8)
        s = None if seqs is None else _arr(seqs, np.uint64)
        data = _arr(data, np.uint8)
        data = data if data.size else np.zeros(16, np.uint8)
        if pinned is not None:  # payloads in page-locked memory: the library uploads them in place
            data = PinnedBytes(pinned, data)
        off = _arr(off, np.uint64)
        keep = (g, t, s, data, off)
        c = Commit(g.size, _ptr(g), _ptr(t), _ptr(s), _ptr(off), data._p if pinned is not None else _ptr(data), None, None)
        return c, keep

    def apply_committed(self, tracker: Tracker | None, lo, hi, types, seqs, msgs=None, data=None, off=None, pinned=None):
        """jg_apply_committed: returns (completed origins in commit order, stopped_at or None, code).  pinned: a
        Context whose page-locked memory carries the payloads (the library's direct upload, no gather)."""
        c, keep = self._commit(lo, hi, types, seqs, msgs, data, off, pinned)
        try:
            return self._apply(tracker, c)
        finally:
            if pinned is not None:
                keep[3].close()

    def _apply(self, tracker, c):
        done = np.zeros(max(1, c.n), np.uint64)
        nd, at = _u64(), _u64()
        rc = load().jg_apply_committed(self._h, tracker._h if tracker else None, C.byref(c), _ptr(done), C.byref(nd), C.byref(at))
        if rc != JG_OK and at.value == 2**64 - 1:
            try:
                _check(rc)
            except JanusError as e:  # the completions the call reported before its error (the OR-Set commit's flag)
                e.completed = done[: nd.value].copy()
                raise
        return done[: nd.value].copy(), (None if at.value == 2**64 - 1 else at.value), rc

    def apply_stream(self, tracker: Tracker | None, parts, pinned=None, n_max=None, bytes_max=None):
        """jg_apply_stream_begin / _append (one per part) / _end: parts = [(lo, hi, types, seqs, msgs)]; returns
        (completed origins, stopped_at or None, code) like apply_committed over the concatenated parts."""
        n_max = n_max or max(1, sum(len(p[4]) for p in parts))
        bytes_max = bytes_max if bytes_max is not None else sum(len(m) for p in parts for m in p[4])
        _check(load().jg_apply_stream_begin(self._h, tracker._h if tracker else None, n_max, bytes_max))
        keeps = []
        try:
            for lo, hi, types, seqs, msgs in parts:
                c, keep = self._commit(lo, hi, types, seqs, msgs, None, None, pinned)
                keeps.append(keep)
                _check(load().jg_apply_stream_append(self._h, C.byref(c)))
            done = np.zeros(max(1, n_max), np.uint64)
            nd, at = _u64(), _u64()
            rc = load().jg_apply_stream_end(self._h, _ptr(done), C.byref(nd), C.byref(at))
            if rc != JG_OK and at.value == 2**64 - 1:
                try:
                    _check(rc)
                except JanusError as e:
                    e.completed = done[: nd.value].copy()
                    raise
            return done[: nd.value].copy(), (None if at.value == 2**64 - 1 else at.value), rc
        finally:
            if pinned is not None:
                for keep in keeps:
                    keep[3].close()

    def apply_block(self, lo, hi, types, msgs=None, data=None, off=None):
        """jg_apply_block: returns (stopped_at or None, code)."""
        c, keep = self._commit(lo, hi, types, None, msgs, data, off)
        at = _u64()
        rc = load().jg_apply_block(self._h, C.byref(c), C.byref(at))
        if rc != JG_OK and at.value == 2**64 - 1:
            _check(rc)
        return (None if at.value == 2**64 - 1 else at.value), rc

    def stats(self) -> dict:
        st = ApplyStats()
        _check(load().jg_node_last_stats(self._h, C.byref(st)))
        return {k: getattr(st, k) for k, _ in ApplyStats._fields_}

    def close(self) -> None:
        if self._h:
            _check(load().jg_node_destroy(self._h))
            self._h = _vp()


class ExchangeStats(C.Structure):
    """jg_exchange_stats: device seconds of route / counts + runs / merge, link bytes, records merged."""
    _fields_ = [("route_s", C.c_double), ("exchange_s", C.c_double), ("merge_s", C.c_double),
                ("bytes_sent", C.c_uint64), ("bytes_received", C.c_uint64), ("records_received", C.c_uint64)]


_ALLTOALLV = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p, C.POINTER(C.c_uint64))


def comm_unique_id() -> bytes:
    """jg_comm_unique_id: a fresh 128-byte RCCL unique id (made by one rank, handed to the others)."""
    buf = (C.c_uint8 * 128)()
    _check(load().jg_comm_unique_id(C.cast(buf, _vp)))
    return bytes(buf)


class Comm:
    """The library's own RCCL communicator (jg_comm_init, csrc/comm.hip): one per process, one rank per GPU.
    exchange_pnc / exchange_orset route a received batch / state by owner, move the runs over RCCL and
    merge what this rank owns — the whole cross-shard exchange inside the library."""

    def __init__(self, ctx: Context, rank: int, world: int, uid: bytes | None = None, alltoallv=None):
        """uid: the RCCL transport (jg_comm_init).  alltoallv: the host transport (jg_comm_init_host) —
        alltoallv(send: bytes, send_bytes: list, recv_bytes: list) -> bytes of the peers' runs back to back."""
        self._h = _vp()
        self.rank, self.world = rank, world
        if alltoallv is not None:
            def cb(user, send, sb, recv, rb):
                try:
                    s_n = [sb[p] for p in range(world)]
                    r_n = [rb[p] for p in range(world)]
                    data = C.string_at(send, sum(s_n)) if sum(s_n) else b""
                    got = alltoallv(data, s_n, r_n)
                    if len(got) != sum(r_n):
                        return 2
                    if got:
                        C.memmove(recv, got, len(got))
                    return 0
                except Exception:  # noqa: BLE001 — an exception cannot cross the C boundary
                    import traceback
                    traceback.print_exc()
                    return 1
            self._cb = _ALLTOALLV(cb)  # kept alive with the communicator
            _check(load().jg_comm_init_host(ctx.handle, rank, world, C.cast(self._cb, _vp), None, C.byref(self._h)))
            return
        assert uid is not None and len(uid) == 128
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        _check(load().jg_comm_init(ctx.handle, rank, world, C.cast(buf, _vp), C.byref(self._h)))

    def exchange_pnc(self, store, rows):
        sent, got = np.zeros(self.world, np.uint64), np.zeros(self.world, np.uint64)
        _check(load().jg_pnc_exchange(self._h, store._h, rows._h if rows is not None else None, _ptr(sent), _ptr(got)))
        return {"sent": sent, "received": got}

    def exchange_orset(self, store, received):
        v = [np.zeros(self.world, np.uint64) for _ in range(4)]
        _check(load().jg_orset_exchange(self._h, store._h, received._h, *(_ptr(x) for x in v)))
        return {"sent": (v[0], v[1]), "received": (v[2], v[3])}

    def stats(self) -> ExchangeStats:
        st = ExchangeStats()
        _check(load().jg_comm_last_stats(self._h, C.cast(C.byref(st), _vp)))
        return st

    def close(self) -> None:
        if self._h:
            _check(load().jg_comm_destroy(self._h))
            self._h = _vp()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
