"""deneva_amd — MI355X-native batched concurrency control for Deneva's hot path.

The engine decides commit/abort (OCC) and lock-grant order (Calvin) for a whole
epoch of transactions on gfx950 (libdcc.so, C ABI in include/dcc.h).  This
package is the thin Python view of that ABI used by tests and bench.py.
"""
from ._abi import (DEVICE_PTRS, GROUP_NONE, KEY_RESERVED, OCC_APPEND_HISTORY, OCC_DEFER_FINISH, RC_ABORT, RC_RCOK,
                   RC_WAIT, RD, SCAN, WR, XP, DccError, EXPORTED, LIB_PATH)
from .engine import (Engine, EpochBatch, alg_bytes, calvin_alg_bytes, comm_unique_id, gen_tpcc, gen_ycsb,
                     key_shard, read_batch_file, shard_filter, shard_of_keys, tpcc_params, write_batch_file,
                     ycsb_params)

__all__ = [
    "Engine", "EpochBatch", "DccError", "gen_ycsb", "gen_tpcc", "ycsb_params", "tpcc_params",
    "shard_filter", "shard_of_keys", "key_shard", "comm_unique_id", "alg_bytes", "calvin_alg_bytes", "RD", "WR", "XP", "SCAN",
    "RC_RCOK", "RC_ABORT", "RC_WAIT", "KEY_RESERVED", "GROUP_NONE", "DEVICE_PTRS",
    "OCC_APPEND_HISTORY", "OCC_DEFER_FINISH", "EXPORTED", "LIB_PATH", "read_batch_file", "write_batch_file",
]
