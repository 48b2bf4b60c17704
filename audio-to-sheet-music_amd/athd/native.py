"""ctypes binding of libathd.so (include/athd.h).  Raises on import if the library is missing or fails to load:
there is no CPU or PyTorch fallback for the hot path."""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ATHD_LIB", os.path.join(_HERE, "libathd.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(f"athd: native library not found at {LIB_PATH}; build it with `python -c 'import "
                      f"__graft_entry__ as g; g.build()'` (or make -C audio-to-sheet-music_amd/csrc)")
lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)

_c = ctypes
lib.athd_version.restype = _c.c_int
lib.athd_create.argtypes = [_c.POINTER(_c.c_void_p), _c.c_int, _c.c_int]
lib.athd_create.restype = _c.c_int
lib.athd_set_weight.argtypes = [_c.c_void_p, _c.c_char_p, _c.c_void_p, _c.POINTER(_c.c_int64), _c.c_int, _c.c_int]
lib.athd_set_weight.restype = _c.c_int
lib.athd_num_required_keys.restype = _c.c_int
lib.athd_required_key.argtypes = [_c.c_int]
lib.athd_required_key.restype = _c.c_char_p
lib.athd_finalize.argtypes = [_c.c_void_p]
lib.athd_finalize.restype = _c.c_int
lib.athd_workspace_bytes.argtypes = [_c.c_void_p, _c.c_int64, _c.c_int64, _c.c_int]
lib.athd_workspace_bytes.restype = _c.c_size_t
lib.athd_forward.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_void_p, _c.c_void_p,
                             _c.c_void_p, _c.c_size_t, _c.c_void_p]
lib.athd_forward.restype = _c.c_int
lib.athd_forward_prompts.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_void_p, _c.c_int,
                                     _c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_void_p]
lib.athd_forward_prompts.restype = _c.c_int
lib.athd_num_windows.argtypes = [_c.c_int64, _c.c_int64, _c.c_int64]
lib.athd_num_windows.restype = _c.c_int64
lib.athd_overlap_add.argtypes = [_c.c_void_p, _c.c_int64, _c.c_int64, _c.c_int64, _c.c_int, _c.c_int64, _c.c_int64,
                                 _c.c_void_p, _c.c_void_p]
lib.athd_overlap_add.restype = _c.c_int
lib.athd_overlap_add_weighted.argtypes = [_c.c_void_p, _c.c_int64, _c.c_int64, _c.c_int64, _c.c_int, _c.c_int64,
                                          _c.c_int64, _c.c_void_p, _c.c_void_p, _c.c_void_p]
lib.athd_overlap_add_weighted.restype = _c.c_int
lib.athd_ola_normalize.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_int, _c.c_int64, _c.c_void_p]
lib.athd_ola_normalize.restype = _c.c_int
lib.athd_sdr.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_void_p, _c.c_void_p, _c.c_void_p]
lib.athd_sdr.restype = _c.c_int
lib.athd_sisdr.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_void_p, _c.c_void_p, _c.c_void_p]
lib.athd_sisdr.restype = _c.c_int
lib.athd_set_decode_items.argtypes = [_c.c_void_p, _c.c_int64]
lib.athd_set_decode_items.restype = _c.c_int
lib.athd_profile_start.argtypes = [_c.c_void_p, _c.c_char_p]
lib.athd_profile_start.restype = _c.c_int
lib.athd_profile_stop.argtypes = [_c.c_void_p]
lib.athd_profile_stop.restype = _c.c_int
lib.athd_profile_count.argtypes = [_c.c_void_p]
lib.athd_profile_count.restype = _c.c_int
lib.athd_profile_get.argtypes = [_c.c_void_p, _c.c_int, _c.POINTER(_c.c_char_p), _c.POINTER(_c.c_longlong),
                                 _c.POINTER(_c.c_double), _c.POINTER(_c.c_double), _c.POINTER(_c.c_double)]
lib.athd_profile_get.restype = _c.c_int
lib.athd_last_error.argtypes = [_c.c_void_p]
lib.athd_last_error.restype = _c.c_char_p
lib.athd_destroy.argtypes = [_c.c_void_p]
lib.athd_destroy.restype = None

EXPORTED = ["athd_version", "athd_create", "athd_set_weight", "athd_num_required_keys", "athd_required_key",
            "athd_finalize", "athd_set_decode_items", "athd_workspace_bytes", "athd_forward", "athd_forward_prompts",
            "athd_num_windows", "athd_overlap_add", "athd_overlap_add_weighted", "athd_ola_normalize", "athd_sdr",
            "athd_sisdr", "athd_profile_start",
            "athd_profile_stop", "athd_profile_count", "athd_profile_get", "athd_last_error", "athd_destroy"]

F32, BF16 = 0, 1


class AthdError(RuntimeError):
    pass


def required_keys():
    return [lib.athd_required_key(i).decode() for i in range(lib.athd_num_required_keys())]


class Context:
    """Owns one athd_ctx (packed weights on one device)."""

    def __init__(self, device: int = 0, dtype: int = BF16):
        h = _c.c_void_p()
        rc = lib.athd_create(_c.byref(h), int(device), int(dtype))
        if rc != 0:
            raise AthdError(f"athd_create failed ({rc}) on device {device}")
        self.h = h
        self.device = device
        self.dtype = dtype

    def _check(self, rc, what):
        if rc != 0:
            raise AthdError(f"{what} failed ({rc}): {lib.athd_last_error(self.h).decode()}")

    def set_weight(self, key: str, arr):
        a = np.ascontiguousarray(np.asarray(arr, dtype=np.float32))
        shape = (_c.c_int64 * max(a.ndim, 1))(*a.shape)
        self._check(lib.athd_set_weight(self.h, key.encode(), a.ctypes.data_as(_c.c_void_p), shape, a.ndim, 0),
                    f"set_weight({key})")

    def finalize(self):
        self._check(lib.athd_finalize(self.h), "finalize")

    def set_decode_items(self, items: int):
        """(segment, prompt) items per decode chunk (the decoder's workspace scales with it; library default 64)."""
        self._check(lib.athd_set_decode_items(self.h, int(items)), "set_decode_items")

    def workspace_bytes(self, B: int, T: int, P: int = 1) -> int:
        return int(lib.athd_workspace_bytes(self.h, B, T, P))

    def forward(self, wav_ptr, B, T, text_ptr, out_ptr, ws_ptr, ws_bytes, stream_ptr):
        self._check(lib.athd_forward(self.h, wav_ptr, B, T, text_ptr, out_ptr, ws_ptr, ws_bytes, stream_ptr),
                    "athd_forward")

    def forward_prompts(self, wav_ptr, B, T, table_ptr, P, out_ptr, ws_ptr, ws_bytes, stream_ptr):
        self._check(lib.athd_forward_prompts(self.h, wav_ptr, B, T, table_ptr, P, out_ptr, ws_ptr, ws_bytes,
                                             stream_ptr), "athd_forward_prompts")

    def profile_start(self, kernel: str | None = None):
        """Time every launch of `kernel` (rocprof symbol short form; None = all kernels) with HIP events."""
        self._check(lib.athd_profile_start(self.h, kernel.encode() if kernel else None), "athd_profile_start")

    def profile_stop(self) -> list:
        """Synchronise the profile window; per kernel: launches, ms (summed event time), algorithmic flops/bytes."""
        self._check(lib.athd_profile_stop(self.h), "athd_profile_stop")
        out = []
        for i in range(lib.athd_profile_count(self.h)):
            name, n = _c.c_char_p(), _c.c_longlong()
            ms, fl, by = _c.c_double(), _c.c_double(), _c.c_double()
            self._check(lib.athd_profile_get(self.h, i, _c.byref(name), _c.byref(n), _c.byref(ms), _c.byref(fl),
                                             _c.byref(by)), "athd_profile_get")
            out.append({"kernel": name.value.decode(), "launches": n.value, "ms": ms.value, "flops": fl.value,
                        "bytes": by.value})
        return out

    def close(self):
        if getattr(self, "h", None):
            lib.athd_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
