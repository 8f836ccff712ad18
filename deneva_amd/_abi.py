"""ctypes binding of libdcc.so (include/dcc.h).

The library is built in-tree (deneva_amd/libdcc.so) by ``__graft_entry__.build()``
or ``make -C deneva_amd/csrc``.  Importing this module without the library is a
hard error: there is no CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# DENEVA_AMD_LIB: another build of the library (tools/: the DCC_EXPERIMENTS
# build with the A/B timing switches); tests, bench and smoke load the default
LIB_PATH = os.environ.get("DENEVA_AMD_LIB") or os.path.join(_HERE, "libdcc.so")

# ---- constants mirrored from include/dcc.h
DCC_OK = 0
DCC_EIO = -5
DCC_ENOMEM = -12
DCC_ENODEV = -19
DCC_EINVAL = -22
DCC_ERANGE = -34
DCC_ECOMM = -70
DCC_ENOTSUP = -95

RD, WR, XP, SCAN = 0, 1, 2, 3  # access_t, system/global.h:287
RC_RCOK, RC_ABORT, RC_WAIT = 0, 2, 3  # RC, system/global.h:236
KEY_RESERVED = 0xFFFFFFFFFFFFFFFF
GROUP_NONE = 0xFFFFFFFF
DEVICE_PTRS = 0x1
OCC_APPEND_HISTORY = 0x2
OCC_DEFER_FINISH = 0x8
KEYS_U32 = 0x10
ACCTYPE_2BIT = 0x20
TN_U32 = 0x40
SHARD_SELF = 0x80
MAAT_READ_AND_PREWRITE = 0x4
ROW_NONE = 0xFFFFFFFFFFFFFFFF
UNIQUE_ID_BYTES = 128
# int (*)(void* user, uint8_t* host_buf, uint64_t n): in-place MAX all-reduce
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint8), C.c_uint64)
OPT_RECHECK = 1
OPT_BATCH_MAX = 2
OPT_SOLVER = 5
OPT_SWEEP_LEVELS = 6
OPT_HIST_MERGE = 7
OPT_FAIL_RANK = 8
OPT_RO_SPLIT = 10
OPT_PIPELINE = 11
OPT_CALVIN_PATH = 12
OPT_COMM_SOLO = 13
OPT_PIPE_PARTITION = 14
OPT_PIPE_CHAIN = 15


class Batch(C.Structure):
    _fields_ = [
        ("n_txn", C.c_uint64),
        ("nnz", C.c_uint64),
        ("offsets", C.c_void_p),
        ("keys", C.c_void_p),
        ("acctype", C.c_void_p),
        ("start_tn", C.c_void_p),
        ("finish_tn", C.c_void_p),
        ("order", C.c_void_p),
        ("flags", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class Snapshot(C.Structure):
    """dcc_occ_snapshot: one captured critical-section view per txn."""
    _fields_ = [
        ("hist_top", C.c_void_p),
        ("active_off", C.c_void_p),
        ("active_idx", C.c_void_p),
    ]


class CalvinHeld(C.Structure):
    _fields_ = [("n", C.c_uint64), ("keys", C.c_void_p), ("acctype", C.c_void_p)]


class Stats(C.Structure):
    _fields_ = [
        ("rounds", C.c_uint32),
        ("n_shards", C.c_uint32),
        ("n_commit", C.c_uint64),
        ("n_abort", C.c_uint64),
        ("n_readonly", C.c_uint64),
        ("nnz_w", C.c_uint64),
        ("alg_bytes", C.c_uint64),
        ("device_ms", C.c_double),
        ("total_ms", C.c_double),
        ("phase_ms", C.c_double * 4),
        ("phase_bytes", C.c_uint64 * 4),
        ("peel_prefix", C.c_uint64),
        ("n_survivors", C.c_uint64),
        ("fallback", C.c_uint32),
        ("fin_where", C.c_uint32),
    ]

    def as_dict(self) -> dict:
        out = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            out[name] = list(v) if name.startswith("phase_") else v
        return out


class YcsbParams(C.Structure):
    _fields_ = [
        ("n_txn", C.c_uint64),
        ("req_per_query", C.c_uint32),
        ("part_cnt", C.c_uint32),
        ("table_size", C.c_uint64),
        ("zipf_theta", C.c_double),
        ("txn_write_perc", C.c_double),
        ("tup_write_perc", C.c_double),
        ("part_per_txn", C.c_uint32),
        ("strict_ppt", C.c_uint32),
        ("first_part_local", C.c_uint32),
        ("chunk_txns", C.c_uint32),
        ("seed", C.c_uint64),
        ("n_threads", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class TpccParams(C.Structure):
    _fields_ = [
        ("n_txn", C.c_uint64),
        ("num_wh", C.c_uint32),
        ("part_cnt", C.c_uint32),
        ("perc_payment", C.c_double),
        ("wh_update", C.c_uint32),
        ("max_items", C.c_uint32),
        ("cust_per_dist", C.c_uint32),
        ("dist_per_wh", C.c_uint32),
        ("max_items_per_txn", C.c_uint32),
        ("part_per_txn", C.c_uint32),
        ("mpr", C.c_double),
        ("first_part_local", C.c_uint32),
        ("chunk_txns", C.c_uint32),
        ("seed", C.c_uint64),
        ("n_threads", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class FileInfo(C.Structure):
    _fields_ = [
        ("version", C.c_uint32),
        ("kind", C.c_uint32),
        ("sections", C.c_uint32),
        ("reserved", C.c_uint32),
        ("n_txn", C.c_uint64),
        ("nnz", C.c_uint64),
        ("seed", C.c_uint64),
        ("epoch", C.c_uint64),
        ("tnc_before", C.c_uint64),
    ]


FILE_OCC = 1
FILE_CALVIN = 2
FILE_HAS_TN = 0x1
FILE_HAS_ORDER = 0x2
FILE_HAS_RC = 0x4
FILE_HAS_COMMIT_TN = 0x8
FILE_HAS_GROUP = 0x10
FILE_HAS_WAVE = 0x20


# (name, restype, argtypes) for every entry point in include/dcc.h
_P = C.c_void_p
_SIGS = [
    ("dcc_init", C.c_int, [C.POINTER(C.c_void_p), C.c_int]),
    ("dcc_init_multi", C.c_int, [C.POINTER(C.c_void_p), C.c_int, _P]),
    ("dcc_device_count", C.c_int, []),
    ("dcc_destroy", None, [_P]),
    ("dcc_strerror", C.c_char_p, [C.c_int]),
    ("dcc_last_error", C.c_char_p, [_P]),
    ("dcc_version", C.c_int, []),
    ("dcc_set_stream", C.c_int, [_P, _P]),
    ("dcc_set_profiling", C.c_int, [_P, C.c_int]),
    ("dcc_set_option", C.c_int, [_P, C.c_int, C.c_int64]),
    ("dcc_reserve", C.c_int, [_P, C.c_uint64, C.c_uint64]),
    ("dcc_host_alloc", C.c_int, [_P, C.c_uint64, C.POINTER(C.c_void_p)]),
    ("dcc_copy_bandwidth", C.c_int, [_P, C.c_uint64, C.c_int, C.POINTER(C.c_double)]),
    ("dcc_host_free", C.c_int, [_P, C.c_void_p]),
    ("dcc_comm_unique_id", C.c_int, [_P]),
    ("dcc_comm_init", C.c_int, [_P, C.c_int, C.c_int, _P]),
    ("dcc_comm_init_host", C.c_int, [_P, C.c_int, C.c_int, C.c_void_p, _P]),
    ("dcc_comm_rank", C.c_int, [_P]),
    ("dcc_comm_size", C.c_int, [_P]),
    ("dcc_comm_calls", C.c_uint64, [_P]),
    ("dcc_comm_destroy", C.c_int, [_P]),
    ("dcc_key_shard", C.c_uint32, [C.c_uint64, C.c_uint32]),
    ("dcc_key_shard_n", C.c_int, [_P, C.c_uint64, C.c_uint32, _P]),
    ("dcc_shard_filter", C.c_int, [C.POINTER(Batch), C.c_uint32, C.c_uint32, _P, _P, _P,
                                   C.POINTER(C.c_uint64)]),
    ("dcc_occ_validate_epoch", C.c_int, [_P, C.POINTER(Batch), _P, _P, C.POINTER(Stats)]),
    ("dcc_occ_finish_epoch", C.c_int, [_P, _P, _P, C.c_uint32]),
    ("dcc_occ_submit_epoch", C.c_int, [_P, C.POINTER(Batch), _P, _P, C.POINTER(C.c_uint64)]),
    ("dcc_occ_wait_epoch", C.c_int, [_P, C.c_uint64, C.POINTER(Stats)]),
    ("dcc_occ_validate_snapshot", C.c_int,
     [_P, C.POINTER(Batch), C.POINTER(Snapshot), _P, C.POINTER(Stats)]),
    ("dcc_occ_history_append", C.c_int, [_P, _P, _P, C.c_uint64]),
    ("dcc_occ_history_clear", C.c_int, [_P]),
    ("dcc_occ_history_size", C.c_uint64, [_P]),
    ("dcc_occ_history_trim", C.c_int, [_P, C.c_uint64]),
    ("dcc_occ_history_export", C.c_int, [_P, _P, _P, C.c_uint64, _P]),
    ("dcc_occ_set_tnc", C.c_int, [_P, C.c_uint64]),
    ("dcc_occ_get_tnc", C.c_uint64, [_P]),
    ("dcc_maat_validate_epoch", C.c_int, [_P, C.POINTER(Batch), _P, _P, C.POINTER(Stats)]),
    ("dcc_maat_rows_set", C.c_int, [_P, _P, _P, _P, C.c_uint64]),
    ("dcc_maat_rows_get", C.c_int, [_P, _P, _P, _P, C.c_uint64]),
    ("dcc_maat_rows_clear", C.c_int, [_P]),
    ("dcc_maat_rows_size", C.c_uint64, [_P]),
    ("dcc_maat_alg_bytes", C.c_uint64, [C.c_uint64, C.c_uint64]),
    ("dcc_calvin_order_epoch", C.c_int, [_P, C.POINTER(Batch), _P, _P, _P, C.POINTER(Stats)]),
    ("dcc_calvin_dispatch", C.c_int, [_P, _P, _P, C.c_uint64, C.c_uint32, _P, C.c_uint64, _P, _P]),
    ("dcc_index_insert", C.c_int, [_P, _P, _P, C.c_uint64]),
    ("dcc_index_probe", C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint32, _P]),
    ("dcc_index_clear", C.c_int, [_P]),
    ("dcc_index_size", C.c_uint64, [_P]),
    ("dcc_index_last_ms", C.c_double, [_P]),
    ("dcc_calvin_order_epoch_held", C.c_int,
     [_P, C.POINTER(Batch), C.POINTER(CalvinHeld), _P, _P, _P, C.POINTER(Stats)]),
    ("dcc_ycsb_params_default", None, [C.POINTER(YcsbParams)]),
    ("dcc_gen_ycsb", C.c_int, [C.POINTER(YcsbParams), _P, _P, _P, _P]),
    ("dcc_tpcc_params_default", None, [C.POINTER(TpccParams)]),
    ("dcc_tpcc_max_access", C.c_uint32, [C.POINTER(TpccParams)]),
    ("dcc_gen_tpcc", C.c_int, [C.POINTER(TpccParams), _P, _P, _P, _P, C.POINTER(C.c_uint64)]),
    ("dcc_alg_bytes", C.c_uint64, [C.c_uint64, C.c_uint64, C.c_uint64]),
    ("dcc_calvin_alg_bytes", C.c_uint64, [C.c_uint64, C.c_uint64, C.c_int, C.c_int]),
    ("dcc_file_write", C.c_int, [C.c_char_p, C.POINTER(FileInfo), C.POINTER(Batch), _P, _P, _P,
                                 _P]),
    ("dcc_file_read_info", C.c_int, [C.c_char_p, C.POINTER(FileInfo)]),
    ("dcc_file_read", C.c_int, [C.c_char_p, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
]
EXPORTED = [s[0] for s in _SIGS]


class DccError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{msg} (code {code})")
        self.code = code


def _load() -> C.CDLL:
    # torch ships its own HIP runtime (soname libamdhip64.so.7).  Load it first
    # so libdcc binds to the same runtime instead of a second copy from
    # /opt/rocm/lib (two HIP runtimes in one process do not share devices).
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libdcc.so not found at {LIB_PATH}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    lib = C.CDLL(LIB_PATH)
    for name, res, args in _SIGS:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def strerror(code: int) -> str:
    return lib.dcc_strerror(code).decode()
