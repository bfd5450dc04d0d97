"""ctypes loader for oracle/_build/liboracle.so -- TEST ORACLE (see linear_ref.c,
wgl_ref.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_build", "liboracle.so")


class OracleKeyResult(C.Structure):
    _fields_ = [("valid", C.c_int8), ("cause", C.c_uint8), ("fail_event", C.c_int32),
                ("peak", C.c_uint32), ("probes", C.c_uint64), ("n_events", C.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            raise ImportError(f"{SO} missing: run `make -C oracle`")
        L = C.CDLL(SO)
        L.oracle_check_history.restype = C.c_int64
        L.oracle_check_history.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_void_p, C.c_void_p, C.c_int64]
        L.oracle_check_history_model.restype = C.c_int64
        L.oracle_check_history_model.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_int, C.c_void_p, C.c_void_p,
                                                 C.c_int64]
        L.oracle_wgl_check_history_model.restype = C.c_int64
        L.oracle_wgl_check_history_model.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_int, C.c_int, C.c_void_p,
                                                     C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]
        _lib = L
    return _lib


MODELS = {"cas-register": 0, "register": 1, "mutex": 2}


def check_history(hist_c, budget: int = 1 << 20, threads: int = 1, model: str = "cas-register"):
    """Run the C restatement over an lc_history struct (lincheck.history.History.as_c()).

    Returns (keys, structured numpy array of per-key results)."""
    L = lib()
    m = MODELS[model]
    nk = L.oracle_check_history_model(C.byref(hist_c), m, budget, threads, None, None, 0)
    if nk < 0:
        raise RuntimeError(f"oracle_check_history failed: {nk}")
    keys = np.zeros(max(nk, 1), np.int64)
    res = (OracleKeyResult * max(nk, 1))()
    rc = L.oracle_check_history_model(C.byref(hist_c), m, budget, threads, keys.ctypes.data, C.addressof(res), nk)
    if rc < 0:
        raise RuntimeError(f"oracle_check_history failed: {rc}")
    dt = np.dtype({"names": [f[0] for f in OracleKeyResult._fields_],
                   "formats": [np.int8, np.uint8, np.int32, np.uint32, np.uint64, np.uint64],
                   "offsets": [getattr(OracleKeyResult, f[0]).offset for f in OracleKeyResult._fields_],
                   "itemsize": C.sizeof(OracleKeyResult)})
    arr = np.frombuffer(res, dtype=dt, count=nk).copy()
    return keys[:nk], arr


def _result_dtype():
    return np.dtype({"names": [f[0] for f in OracleKeyResult._fields_],
                     "formats": [np.int8, np.uint8, np.int32, np.uint32, np.uint64, np.uint64],
                     "offsets": [getattr(OracleKeyResult, f[0]).offset for f in OracleKeyResult._fields_],
                     "itemsize": C.sizeof(OracleKeyResult)})


def check_history_wgl(hist_c, budget: int = 1 << 20, threads: int = 1, model: str = "cas-register",
                      max_final: int = 10):
    """The C restatement of knossos.wgl (wgl_ref.c) over an lc_history.

    Returns (keys, per-key results, finals [K, max_final, 3] = (X lo, X hi,
    register value of the state), n_final [K]).  `peak` is the cache size,
    `n_events` the search's steps."""
    L = lib()
    m = MODELS[model]
    nk = L.oracle_wgl_check_history_model(C.byref(hist_c), m, budget, threads, max_final, None, None, None, None, 0)
    if nk < 0:
        raise RuntimeError(f"oracle_wgl_check_history failed: {nk}")
    n1 = max(nk, 1)
    keys = np.zeros(n1, np.int64)
    res = (OracleKeyResult * n1)()
    fin = np.zeros((n1, max(max_final, 1), 3), np.int64)
    nf = np.zeros(n1, np.uint32)
    rc = L.oracle_wgl_check_history_model(C.byref(hist_c), m, budget, threads, max_final, keys.ctypes.data,
                                          C.addressof(res), fin.ctypes.data, nf.ctypes.data, nk)
    if rc < 0:
        raise RuntimeError(f"oracle_wgl_check_history failed: {rc}")
    arr = np.frombuffer(res, dtype=_result_dtype(), count=nk).copy()
    return keys[:nk], arr, fin[:nk], nf[:nk]
