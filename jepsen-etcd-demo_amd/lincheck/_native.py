"""ctypes binding of liblincheck.so (include/lincheck.h).

The same C ABI a JNA binding on the Clojure side would use.
Loading fails loudly when the library is missing: there is no Python or CPU
fallback for the search.
"""

from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LINCHECK_LIB_OVERRIDE") or os.path.join(HERE, "liblincheck.so")  # override: diagnostics only

# ---- constants (mirror include/lincheck.h) ---------------------------------
LC_ABI_VERSION = 11
LC_MAX_DEVICES = 8
LC_COMM_ID_BYTES = 128
LC_OPT_COUNT_PROBES = 0x1
# lc_opts.path_flags (ABI 9): pinned search-path choices for A/B runs and tests
LC_PATH_SPLIT_ON, LC_PATH_SPLIT_OFF, LC_PATH_SPEC_OFF, LC_PATH_LAYERS_OFF = 0x01, 0x02, 0x04, 0x08
LC_PATH_NODE_SYNC, LC_PATH_NODE_STAGED, LC_PATH_CHUNKS_ON, LC_PATH_CHUNKS_OFF = 0x10, 0x20, 0x40, 0x80
LC_PATH_SPEC_COST, LC_PATH_EV32, LC_PATH_SPEC_NOPRIO, LC_PATH_WGL_SMALL = 0x100, 0x200, 0x400, 0x800
LC_PATH_WGL_EV_HBM = 0x2000  # ABI 11
LC_PATH_SPEC_NOSTAGE = 0x1000
LC_T0_PATH_NONE, LC_T0_PATH_LATTICE, LC_T0_PATH_SPEC, LC_T0_PATH_SEGMENTS = 0, 1, 2, 3
T0_PATH_NAMES = {0: "none", 1: "k_search_lattice", 2: "k_spec", 3: "k_search_segments"}
LC_DEV_RESULT, LC_DEV_ASYNC = 1, 2
LC_INVOKE, LC_OK_T, LC_FAIL, LC_INFO = 0, 1, 2, 3
LC_F_READ, LC_F_WRITE, LC_F_CAS, LC_F_OTHER, LC_F_ACQUIRE, LC_F_RELEASE, LC_F_TXN = 0, 1, 2, 3, 4, 5, 6
LC_MOP_READ, LC_MOP_WRITE = 0, 1
LC_MODEL_CAS_REGISTER, LC_MODEL_REGISTER, LC_MODEL_MUTEX, LC_MODEL_MULTI_REGISTER = 0, 1, 2, 3
LC_TABLE_NONE = 0xFFFF
LC_ALGO_LINEAR, LC_ALGO_WGL, LC_ALGO_COMPETITION = 0, 1, 2
ANALYZERS = {LC_ALGO_LINEAR: "linear", LC_ALGO_WGL: "wgl"}
LC_NIL = -(1 << 63)
LC_NO_KEY = LC_NIL
LC_NO_PROCESS = LC_NIL
LC_EV_OK_BIT = 0x80000000
LC_T_READ_ANY, LC_T_READ, LC_T_WRITE, LC_T_CAS = 0, 1, 2, 3
LC_STATE_NONE = 0x7FFF
LC_NARROW_MAX_SLOTS, LC_WIDE_MAX_SLOTS = 56, 112
LC_WIDE_MAX_STATES = 32767
LC_VALID, LC_INVALID, LC_UNKNOWN = 1, 0, -1
LC_CAUSE_ERROR = 5
CAUSES = {0: "none", 1: "nonlin", 2: "budget", 3: "window", 4: "states", 5: "error"}
ERRORS = {-1: "invalid", -2: "nomem", -3: "device", -4: "parse", -5: "unsupported", -6: "io"}

P = C.POINTER


class LcHistory(C.Structure):
    _fields_ = [("n", C.c_int64), ("type", P(C.c_uint8)), ("f", P(C.c_uint8)),
                ("process", P(C.c_int64)), ("key", P(C.c_int64)),
                ("v0", P(C.c_int64)), ("v1", P(C.c_int64)), ("index", P(C.c_int64)),
                ("mop_off", P(C.c_int64)), ("mop", P(C.c_int64))]


class LcBatch(C.Structure):
    _fields_ = [("n_keys", C.c_int64), ("ev_off", P(C.c_uint64)), ("events", P(C.c_uint32)),
                ("trans", P(C.c_uint32)), ("n_trans", C.c_int64), ("trans_off", P(C.c_uint32)),
                ("key_width", P(C.c_uint8)), ("key_states", P(C.c_uint16)),
                ("init_state", C.c_uint32), ("key_error", P(C.c_uint8)),
                ("table", P(C.c_uint16)), ("n_table", C.c_int64), ("events16", P(C.c_uint16))]


class LcPackOpts(C.Structure):
    _fields_ = [("model", C.c_int32), ("n_init", C.c_int32), ("init", P(C.c_int64)), ("flags", C.c_uint32)]


LC_PACK_GENERAL = 0x1  # lc_pack_opts.flags (ABI 11): always the bucketing path


class LcOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("algorithm", C.c_int32), ("max_configs", C.c_uint64),
                ("max_final", C.c_int32), ("lds_configs", C.c_int32), ("deep_slots", C.c_int32),
                ("flags", C.c_int32), ("debug_mode", C.c_int32),
                ("n_devices", C.c_int32), ("devices", C.c_int32 * LC_MAX_DEVICES),
                ("comm_rank", C.c_int32), ("comm_size", C.c_int32), ("comm_id", C.c_uint8 * LC_COMM_ID_BYTES),
                ("path_flags", C.c_int32), ("spec_segs", C.c_int32), ("spec_ck", C.c_int32),
                ("seg_len", C.c_int32)]


class LcResult(C.Structure):
    _fields_ = [("valid", P(C.c_int8)), ("fail_event", P(C.c_int32)), ("cause", P(C.c_uint8)),
                ("peak_configs", P(C.c_uint32)), ("final_configs", P(C.c_uint64)),
                ("n_final", P(C.c_uint32)), ("analyzer", P(C.c_uint8))]


class LcStats(C.Structure):
    _fields_ = [("kernel_ms", C.c_double), ("total_ms", C.c_double), ("probes", C.c_uint64),
                ("lds_keys", C.c_uint64), ("deep_keys", C.c_uint64), ("events", C.c_uint64),
                ("tier0_ms", C.c_double), ("tier3_ms", C.c_double),
                ("probes_t3", C.c_uint64), ("t3_bytes", C.c_uint64),
                ("t0_path", C.c_uint32), ("ev_word_bytes", C.c_uint32),
                ("wgl_ms", C.c_double), ("wgl_keys", C.c_uint64), ("wgl_spilled", C.c_uint64),
                ("wgl_steps", C.c_uint64)]


class LcSynthOpts(C.Structure):
    _fields_ = [("n_keys", C.c_int64), ("ops_per_key", C.c_int64), ("concurrency", C.c_int32),
                ("n_values", C.c_int32), ("info_rate", C.c_double), ("info_effect_p", C.c_double),
                ("anomaly_rate", C.c_double), ("mean_think", C.c_double),
                ("mean_latency", C.c_double), ("interleave", C.c_int32),
                ("nemesis_period", C.c_double), ("seed", C.c_uint64), ("key_base", C.c_int64)]


# Every exported symbol: name -> (restype, argtypes).  tests/test_abi.py checks
# this table against include/lincheck.h.
SIGNATURES = {
    "lc_abi_version": (C.c_int, []),
    "lc_trim": (None, []),
    "lc_last_error": (C.c_char_p, []),
    "lc_device_count": (C.c_int, []),
    "lc_create": (C.c_int, [P(LcOpts), P(C.c_void_p)]),
    "lc_destroy": (None, [C.c_void_p]),
    "lc_check_batch": (C.c_int, [C.c_void_p, P(LcBatch), P(LcResult), P(LcStats)]),
    "lc_upload": (C.c_int, [C.c_void_p, P(LcBatch), P(C.c_void_p)]),
    "lc_dev_batch_free": (None, [C.c_void_p]),
    "lc_check_device": (C.c_int, [C.c_void_p, C.c_void_p, P(LcResult), C.c_int, P(LcStats)]),
    "lc_wait": (C.c_int, [C.c_void_p, P(LcStats)]),
    "lc_wait_step": (C.c_int, [C.c_void_p, C.c_int]),
    "lc_comm_id": (C.c_int, [P(C.c_uint8)]),
    "lc_check_node": (C.c_int, [C.c_void_p, P(LcBatch), C.c_int64, P(C.c_uint64), P(LcStats)]),
    "lc_check_node_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, P(LcStats)]),
    "lc_check_node_async": (C.c_int, [C.c_void_p, P(LcBatch), C.c_int64, P(C.c_uint64), P(LcStats)]),
    "lc_host_alloc": (C.c_void_p, [C.c_size_t]),
    "lc_host_free": (None, [C.c_void_p]),
    "lc_node_records": (C.c_int, [C.c_void_p, P(C.c_uint64), C.c_int64]),
    "lc_pack": (C.c_int, [P(LcHistory), P(LcPackOpts), P(C.c_void_p)]),
    "lc_packed_free": (None, [C.c_void_p]),
    "lc_packed_view": (C.c_int, [C.c_void_p, P(LcBatch)]),
    "lc_packed_key": (C.c_int64, [C.c_void_p, C.c_int64]),
    "lc_packed_event_row": (C.c_int64, [C.c_void_p, C.c_int64, C.c_int64]),
    "lc_packed_path": (C.c_int, [C.c_void_p]),
    "lc_packed_event_rows": (C.c_int64, [C.c_void_p, P(C.c_int64)]),
    "lc_packed_subhistory": (C.c_int64, [C.c_void_p, C.c_int64, P(C.c_int64)]),
    "lc_packed_key_error": (C.c_char_p, [C.c_void_p, C.c_int64]),
    "lc_packed_state_value": (C.c_int, [C.c_void_p, C.c_int64, C.c_uint32, P(C.c_int64), P(C.c_int)]),
    "lc_packed_keys": (C.c_int, [C.c_void_p, P(C.c_int64)]),
    "lc_packed_state_map": (C.c_int64, [C.c_void_p, C.c_int64, C.c_uint32, P(C.c_int64), P(C.c_int64), C.c_int64]),
    "lc_report": (C.c_int64, [C.c_void_p, C.c_int64, C.c_int32, C.c_int32, P(C.c_uint64), C.c_uint32, C.c_int32,
                              P(C.c_int64), C.c_int64]),
    "lc_report_wgl": (C.c_int64, [C.c_void_p, C.c_int64, C.c_int32, C.c_int32, P(C.c_uint64), C.c_uint32, C.c_int32,
                                  P(C.c_int64), C.c_int64]),
    "lc_synth_generate": (C.c_int, [P(LcSynthOpts), P(C.c_void_p)]),
    "lc_hist_view": (C.c_int, [C.c_void_p, P(LcHistory)]),
    "lc_hist_anomalous_keys": (C.c_int64, [C.c_void_p, P(C.c_int64)]),
    "lc_hist_free": (None, [C.c_void_p]),
    "lc_edn_read": (C.c_int, [C.c_char_p, P(C.c_void_p)]),
    "lc_edn_parse": (C.c_int, [C.c_char_p, C.c_int64, P(C.c_void_p)]),
    "lc_edn_write": (C.c_int, [C.c_char_p, P(LcHistory)]),
    "lc_edn_write_named": (C.c_int, [C.c_char_p, P(LcHistory), P(C.c_char_p), C.c_int64]),
    "lc_hist_n_reg_names": (C.c_int64, [C.c_void_p]),
    "lc_hist_reg_name": (C.c_char_p, [C.c_void_p, C.c_int64]),
    "lc_fressian_read": (C.c_int, [C.c_char_p, P(C.c_void_p)]),
    "lc_fressian_parse": (C.c_int, [C.c_char_p, C.c_int64, P(C.c_void_p)]),
    "lc_fressian_write": (C.c_int, [C.c_char_p, P(LcHistory)]),
}

_lib: Optional[C.CDLL] = None


class LincheckError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


def lib() -> C.CDLL:
    """Load liblincheck.so (built in-tree by __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.lc_abi_version() != LC_ABI_VERSION:
            raise ImportError(f"liblincheck ABI {L.lc_abi_version()} != {LC_ABI_VERSION}")
        _lib = L
    return _lib


def check(rc: int) -> int:
    if rc < 0:
        raise LincheckError(rc, lib().lc_last_error().decode(errors="replace"))
    return rc


def ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(P(ctype))


def carray(p, n: int, dtype) -> np.ndarray:
    """Copy n elements from a ctypes pointer (NULL -> empty)."""
    if not p or n == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(p, shape=(n,)).astype(dtype, copy=True)
