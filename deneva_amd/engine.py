"""Python mirror of the engine's C ABI for tests, bench and tooling.

The product is libdcc.so (HIP kernels + C ABI) and its C++ host shim
(deneva_amd/csrc/host/); this module is plumbing over ``include/dcc.h``:
numpy (host) or torch (device) arrays in, per-transaction RC codes out.

Names follow the reference's plugin surface:
``Engine.occ_validate_epoch`` is ``TxnManager::validate`` / ``OptCC::validate``
(concurrency_control/occ.cpp:42) for a whole epoch; ``Engine.calvin_order_epoch``
is the ``Sequencer::send_next_batch`` -> ``acquire_locks`` hand-off
(system/sequencer.cpp:283, benchmarks/ycsb_txn.cpp:49).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import _abi
from ._abi import DccError, lib


def _ptr(a) -> Optional[int]:
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags["C_CONTIGUOUS"], "arrays must be contiguous"
        return a.ctypes.data
    return int(a.data_ptr())  # torch tensor


def _itemsize(a) -> int:
    return int(a.itemsize) if isinstance(a, np.ndarray) else int(a.element_size())


def pack_acctype(at) -> np.ndarray:
    """access_t bytes -> 2-bit codes, four per byte (DCC_ACCTYPE_2BIT)."""
    at = np.asarray(at, np.uint8)
    pad = np.zeros((-at.size) % 4, np.uint8)
    q = np.concatenate([at, pad]).reshape(-1, 4) & 3
    return (q[:, 0] | (q[:, 1] << 2) | (q[:, 2] << 4) | (q[:, 3] << 6)).astype(np.uint8)


def _is_signed(a) -> bool:
    """A signed numpy array.  Device (torch) tensors are exempt: torch holds
    u32 row ids as int32 tensors, read bit for bit as DCC_KEYS_U32."""
    return isinstance(a, np.ndarray) and a.dtype.kind == "i"


def _is_device(a) -> bool:
    return a is not None and not isinstance(a, np.ndarray) and bool(getattr(a, "is_cuda", False))


@dataclass
class EpochBatch:
    """One epoch as a CSR of per-transaction access lists (dcc_batch)."""

    offsets: object            # u32 [n_txn+1]
    keys: object               # u64 [nnz]
    acctype: object            # u8  [nnz] access_t
    start_tn: object = None    # u64 [n_txn] or None
    finish_tn: object = None   # u64 [n_txn] or None
    order: object = None       # u64 [n_txn] (Calvin sequence key) or None
    meta: dict = field(default_factory=dict)

    @property
    def n_txn(self) -> int:
        return int(self.offsets.shape[0]) - 1

    @property
    def nnz(self) -> int:
        return int(self.keys.shape[0])

    @property
    def on_device(self) -> bool:
        return _is_device(self.offsets)

    def to_c(self, flags: int = 0) -> _abi.Batch:
        b = _abi.Batch()
        b.n_txn = self.n_txn
        b.nnz = self.nnz
        b.offsets = _ptr(self.offsets)
        b.keys = _ptr(self.keys)
        b.acctype = _ptr(self.acctype)
        b.start_tn = _ptr(self.start_tn)
        b.finish_tn = _ptr(self.finish_tn)
        b.order = _ptr(self.order)
        b.flags = flags | (_abi.DEVICE_PTRS if self.on_device else 0)
        # compact transfer forms (dcc.h): 4-byte keys / timestamps, packed types
        if _itemsize(self.keys) == 4:
            if _is_signed(self.keys):
                raise TypeError("4-byte keys must be an unsigned dtype (DCC_KEYS_U32 row ids)")
            b.flags |= _abi.KEYS_U32
        if self.meta.get("acctype_2bit"):
            b.flags |= _abi.ACCTYPE_2BIT
        if self.start_tn is not None:
            if self.finish_tn is None or _itemsize(self.start_tn) != _itemsize(self.finish_tn):
                raise TypeError("start_tn and finish_tn must both be set, with the same dtype size")
            if _itemsize(self.start_tn) == 4:
                b.flags |= _abi.TN_U32
        return b

    def to_torch(self, device="cuda"):
        import torch

        def cv(a):
            if a is None:
                return None
            return torch.from_numpy(np.ascontiguousarray(a)).to(device)

        return EpochBatch(cv(self.offsets), cv(self.keys), cv(self.acctype), cv(self.start_tn),
                          cv(self.finish_tn), cv(self.order), dict(self.meta))


def _check(code: int, ctx=None) -> None:
    if code != _abi.DCC_OK:
        detail = lib.dcc_last_error(ctx).decode() if ctx else ""
        raise DccError(code, f"{_abi.strerror(code)}{': ' + detail if detail else ''}")


class Engine:
    """One engine context per process and device (OptCC::init / occ_man).
    devices=[...]: one process drives several GPUs (dcc_init_multi): every
    epoch is key-sharded over them inside the context."""

    def __init__(self, device: int = 0, devices=None):
        h = C.c_void_p()
        if devices is not None:
            ids = (C.c_int * len(devices))(*devices)
            code = lib.dcc_init_multi(C.byref(h), len(devices), ids)
        else:
            code = lib.dcc_init(C.byref(h), device)
        if code != _abi.DCC_OK:
            detail = lib.dcc_last_error(h).decode() if h.value else ""
            raise DccError(code, f"dcc_init(device={device}, devices={devices}): "
                                 f"{_abi.strerror(code)} {detail}")
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib.dcc_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream_ptr: Optional[int]) -> None:
        _check(lib.dcc_set_stream(self._h, stream_ptr), self._h)

    def set_profiling(self, enable: bool) -> None:
        _check(lib.dcc_set_profiling(self._h, 1 if enable else 0), self._h)

    def set_option(self, option: int, value: int) -> None:
        _check(lib.dcc_set_option(self._h, option, value), self._h)

    def reserve(self, max_txn: int, max_nnz: int) -> None:
        _check(lib.dcc_reserve(self._h, max_txn, max_nnz), self._h)

    def host_empty(self, n: int, dtype) -> np.ndarray:
        """A numpy array in pinned host memory (dcc_host_alloc): host batches
        and outputs in it move at DMA speed with no staging copy.  Freed with
        the array."""
        import weakref
        dt = np.dtype(dtype)
        nbytes = max(int(n), 1) * dt.itemsize
        p = C.c_void_p()
        _check(lib.dcc_host_alloc(self._h, nbytes, C.byref(p)), self._h)
        buf = (C.c_uint8 * nbytes).from_address(p.value)
        arr = np.frombuffer(buf, dtype=dt, count=max(int(n), 1))[:int(n)]
        # freed with the buffer (no context needed: the engine may be gone)
        weakref.finalize(buf, lib.dcc_host_free, None, p.value)
        return arr

    def compact_host_batch(self, b: "EpochBatch") -> "EpochBatch":
        """The batch in pinned host memory and its compact transfer form:
        u32 keys when every key fits, 2-bit access types, u32 timestamps when
        they fit (dcc.h DCC_KEYS_U32 / DCC_ACCTYPE_2BIT / DCC_TN_U32) -- what a
        host shim builds directly (OccEpoch) to cut the PCIe bytes."""
        def pin(a, dtype):
            a = np.asarray(a)
            out = self.host_empty(a.size, dtype)
            out[...] = a
            return out
        keys = np.asarray(b.keys, np.uint64)
        k = pin(keys, np.uint32) if (keys.size == 0 or int(keys.max()) < (1 << 32)) else pin(keys, np.uint64)
        at = pin(pack_acctype(b.acctype), np.uint8)
        st = ft = None
        if b.start_tn is not None:
            big = max(int(np.max(b.start_tn, initial=0)), int(np.max(b.finish_tn, initial=0)))
            dt = np.uint32 if big < (1 << 32) else np.uint64
            st, ft = pin(b.start_tn, dt), pin(b.finish_tn, dt)
        od = None if b.order is None else pin(b.order, np.uint64)
        meta = dict(b.meta)
        meta["acctype_2bit"] = True
        meta["nnz"] = int(keys.size)
        return EpochBatch(pin(b.offsets, np.uint32), k, at, st, ft, od, meta)

    # ------------------------------------------------------------ OCC
    def occ_validate_epoch(self, batch: EpochBatch, want_tn: bool = False,
                           append_history: bool = False, out_rc=None, out_tn=None,
                           defer_finish: bool = False, shard_self: bool = False):
        """Decide every txn of the epoch; returns (rc u8[n], tn u64[n] | None, stats).
        defer_finish: 2PC participant -- rc is the local vote; commit tn and
        history wait for ``occ_finish_epoch(global_rc)``.  shard_self: a
        key-sharded rank given the WHOLE epoch keeps its own key shard
        (DCC_SHARD_SELF)."""
        n = batch.n_txn
        dev = batch.on_device
        if out_rc is None:
            if dev:
                import torch
                out_rc = torch.empty(max(n, 1), dtype=torch.uint8, device=batch.offsets.device)
            else:
                out_rc = np.empty(max(n, 1), np.uint8)
        if want_tn and out_tn is None:
            if dev:
                import torch
                out_tn = torch.empty(max(n, 1), dtype=torch.int64, device=batch.offsets.device)
            else:
                out_tn = np.empty(max(n, 1), np.uint64)
        st = _abi.Stats()
        flags = _abi.OCC_APPEND_HISTORY if append_history else 0
        if defer_finish:
            flags |= _abi.OCC_DEFER_FINISH
        if shard_self:
            flags |= _abi.SHARD_SELF
        b = batch.to_c(flags)
        _check(lib.dcc_occ_validate_epoch(self._h, C.byref(b), _ptr(out_rc), _ptr(out_tn),
                                          C.byref(st)), self._h)
        if defer_finish:
            self._fin_n = n
        return out_rc[:n], (out_tn[:n] if want_tn else None), st.as_dict()

    def occ_submit_epoch(self, batch: EpochBatch, out_rc, out_tn=None,
                         append_history: bool = False) -> int:
        """Enqueue an epoch on the pipeline (dcc_occ_submit_epoch) and return
        its ticket; the batch arrays and outputs must stay alive and unchanged
        until ``occ_wait_epoch(ticket)``.  Results equal dcc_occ_validate_epoch
        on the epochs in submit order (commit tn and the history append
        included: each epoch's central_finish runs on its lane right behind its
        decision once the epoch before it finished, DCC_OPT_PIPE_CHAIN, or the
        context runs it as the epoch completes)."""
        b = batch.to_c(_abi.OCC_APPEND_HISTORY if append_history else 0)
        t = C.c_uint64(0)
        _check(lib.dcc_occ_submit_epoch(self._h, C.byref(b), _ptr(out_rc), _ptr(out_tn),
                                        C.byref(t)), self._h)
        return int(t.value)

    def occ_wait_epoch(self, ticket: int) -> dict:
        """Complete every epoch up to `ticket` (submit order); that epoch's stats."""
        st = _abi.Stats()
        _check(lib.dcc_occ_wait_epoch(self._h, ticket, C.byref(st)), self._h)
        return st.as_dict()

    @property
    def pending_finish(self) -> Optional[int]:
        """n_txn of the epoch awaiting occ_finish_epoch, or None."""
        return getattr(self, "_fin_n", None)

    def occ_finish_epoch(self, final_rc, want_tn: bool = True, out_tn=None):
        """central_finish with the global RC of a deferred epoch
        (dcc_occ_finish_epoch; OptCC::finish after RFIN, occ.cpp:248-294):
        globally committed writers take tn = tnc+1.. and join the history.
        Returns tn u64[n] | None."""
        dev = _is_device(final_rc)
        n = int(final_rc.shape[0])
        if self.pending_finish is not None and n != self.pending_finish:
            raise ValueError(f"final_rc holds {n} txns, the pending epoch {self.pending_finish}")
        if not dev:
            final_rc = np.ascontiguousarray(final_rc, dtype=np.uint8)
        if want_tn and out_tn is None:
            if dev:
                import torch
                out_tn = torch.empty(max(n, 1), dtype=torch.int64, device=final_rc.device)
            else:
                out_tn = np.empty(max(n, 1), np.uint64)
        _check(lib.dcc_occ_finish_epoch(self._h, _ptr(final_rc), _ptr(out_tn),
                                        _abi.DEVICE_PTRS if dev else 0), self._h)
        self._fin_n = None
        return out_tn[:n] if want_tn else None

    # ----------------------------------------------------------------- MaaT
    def maat_validate_epoch(self, batch: EpochBatch, want_cts: bool = True,
                            read_and_prewrite: bool = False, out_rc=None, out_cts=None):
        """MaaT epoch (dcc_maat_validate_epoch): returns (rc u8[n],
        commit_ts u64[n] | None, stats).  read_and_prewrite: the TPC-C path."""
        n = batch.n_txn
        dev = batch.on_device
        if out_rc is None:
            if dev:
                import torch
                out_rc = torch.empty(max(n, 1), dtype=torch.uint8, device=batch.offsets.device)
            else:
                out_rc = np.empty(max(n, 1), np.uint8)
        if want_cts and out_cts is None:
            if dev:
                import torch
                out_cts = torch.empty(max(n, 1), dtype=torch.int64, device=batch.offsets.device)
            else:
                out_cts = np.empty(max(n, 1), np.uint64)
        st = _abi.Stats()
        b = batch.to_c(_abi.MAAT_READ_AND_PREWRITE if read_and_prewrite else 0)
        _check(lib.dcc_maat_validate_epoch(self._h, C.byref(b), _ptr(out_rc), _ptr(out_cts),
                                           C.byref(st)), self._h)
        return out_rc[:n], (out_cts[:n] if want_cts else None), st.as_dict()

    def maat_rows_set(self, keys, last_read, last_write) -> None:
        keys = np.ascontiguousarray(keys, np.uint64)
        lr = np.ascontiguousarray(last_read, np.uint64)
        lw = np.ascontiguousarray(last_write, np.uint64)
        _check(lib.dcc_maat_rows_set(self._h, _ptr(keys), _ptr(lr), _ptr(lw), keys.shape[0]),
               self._h)

    def maat_rows_get(self, keys):
        keys = np.ascontiguousarray(keys, np.uint64)
        lr = np.empty(keys.shape[0], np.uint64)
        lw = np.empty(keys.shape[0], np.uint64)
        _check(lib.dcc_maat_rows_get(self._h, _ptr(keys), _ptr(lr), _ptr(lw), keys.shape[0]),
               self._h)
        return lr, lw

    def maat_rows_clear(self) -> None:
        _check(lib.dcc_maat_rows_clear(self._h), self._h)

    @property
    def maat_rows_size(self) -> int:
        return int(lib.dcc_maat_rows_size(self._h))

    def occ_validate_snapshot(self, batch: EpochBatch, active_off, active_idx,
                              hist_top=None, out_rc=None):
        """Captured-snapshot validation (dcc_occ_validate_snapshot): every txn
        against its own captured history head and active list
        (occ.cpp:137-158); returns (rc u8[n], stats).  Arrays live where the
        batch lives (numpy on the host, torch on the device)."""
        n = batch.n_txn
        dev = batch.on_device
        if not dev:
            active_off = np.ascontiguousarray(active_off, np.uint32)
            active_idx = np.ascontiguousarray(active_idx, np.uint32)
            if hist_top is not None:
                hist_top = np.ascontiguousarray(hist_top, np.uint64)
        if out_rc is None:
            if dev:
                import torch
                out_rc = torch.empty(max(n, 1), dtype=torch.uint8, device=batch.offsets.device)
            else:
                out_rc = np.empty(max(n, 1), np.uint8)
        sn = _abi.Snapshot()
        sn.hist_top = _ptr(hist_top)
        sn.active_off = _ptr(active_off)
        sn.active_idx = _ptr(active_idx) if len(active_idx) else None
        st = _abi.Stats()
        b = batch.to_c(0)
        _check(lib.dcc_occ_validate_snapshot(self._h, C.byref(b), C.byref(sn), _ptr(out_rc),
                                             C.byref(st)), self._h)
        return out_rc[:n], st.as_dict()

    def history_append(self, keys: np.ndarray, tn: np.ndarray) -> None:
        keys = np.ascontiguousarray(keys, np.uint64)
        tn = np.ascontiguousarray(tn, np.uint64)
        _check(lib.dcc_occ_history_append(self._h, _ptr(keys), _ptr(tn), keys.shape[0]), self._h)

    def history_trim(self, tn_floor: int) -> None:
        """Drop history entries with tn <= tn_floor (dcc_occ_history_trim)."""
        _check(lib.dcc_occ_history_trim(self._h, tn_floor), self._h)

    def history_export(self):
        """The history's (key, tn) pairs, sorted by (key, tn)."""
        n = C.c_uint64(0)
        _check(lib.dcc_occ_history_export(self._h, None, None, 0, C.byref(n)), self._h)
        k = np.empty(n.value, np.uint64)
        t = np.empty(n.value, np.uint64)
        if n.value:
            _check(lib.dcc_occ_history_export(self._h, _ptr(k), _ptr(t), n.value, C.byref(n)),
                   self._h)
        o = np.lexsort((t, k))
        return k[o], t[o]

    def history_clear(self) -> None:
        _check(lib.dcc_occ_history_clear(self._h), self._h)

    @property
    def history_size(self) -> int:
        return int(lib.dcc_occ_history_size(self._h))

    @property
    def tnc(self) -> int:
        return int(lib.dcc_occ_get_tnc(self._h))

    @tnc.setter
    def tnc(self, v: int) -> None:
        _check(lib.dcc_occ_set_tnc(self._h, v), self._h)

    # ------------------------------------------------------------ Calvin
    def calvin_order_epoch(self, batch: EpochBatch, want_group: bool = True,
                           want_wave: bool = False, held=None, out_group=None, out_rc=None):
        """Returns (group u32[nnz] | None, rc u8[n], wave u32[n] | None, stats).
        held = (keys u64[h], acctype u8[h]): rows still locked at the epoch's
        start, per row owners first then waiters (dcc_calvin_order_epoch_held).
        out_group / out_rc: caller-owned output buffers (reused across epochs,
        the engine then replays the epoch's captured launches)."""
        n, nnz = batch.n_txn, batch.nnz
        dev = batch.on_device
        if dev:
            import torch
            d = batch.offsets.device
            rc = out_rc if out_rc is not None else torch.empty(max(n, 1), dtype=torch.uint8, device=d)
            grp = None
            if want_group:
                grp = out_group if out_group is not None else torch.empty(max(nnz, 1), dtype=torch.int32,
                                                                          device=d)
            wav = torch.empty(max(n, 1), dtype=torch.int32, device=d) if want_wave else None
        else:
            rc = out_rc if out_rc is not None else np.empty(max(n, 1), np.uint8)
            grp = None
            if want_group:
                grp = out_group if out_group is not None else np.empty(max(nnz, 1), np.uint32)
            wav = np.empty(max(n, 1), np.uint32) if want_wave else None
        if rc.shape[0] < n or (grp is not None and grp.shape[0] < nnz):
            raise ValueError("calvin_order_epoch: output buffer shorter than the epoch")
        st = _abi.Stats()
        b = batch.to_c()
        if held is None:
            _check(lib.dcc_calvin_order_epoch(self._h, C.byref(b), _ptr(grp), _ptr(rc), _ptr(wav),
                                              C.byref(st)), self._h)
        else:
            hk, ha = held
            if not dev:
                hk = np.ascontiguousarray(hk, np.uint64)
                ha = np.ascontiguousarray(ha, np.uint8)
            h = _abi.CalvinHeld(int(hk.shape[0]), _ptr(hk), _ptr(ha))
            _check(lib.dcc_calvin_order_epoch_held(self._h, C.byref(b), C.byref(h), _ptr(grp),
                                                   _ptr(rc), _ptr(wav), C.byref(st)), self._h)
        return (grp[:nnz] if want_group else None, rc[:n],
                (wav[:n] if want_wave else None), st.as_dict())

    def calvin_dispatch(self, wave, order=None):
        """Wave dispatch lists (dcc_calvin_dispatch): returns (wave_off u32[W+1],
        txn u32[n]) — txn[wave_off[w]:wave_off[w+1]] run in wave w."""
        dev = hasattr(wave, "device") and str(wave.device).startswith("cuda")
        n = int(wave.shape[0])
        nw = C.c_uint32(0)
        if dev:
            import torch
            txn = torch.empty(max(n, 1), dtype=torch.int32, device=wave.device)
            _check(lib.dcc_calvin_dispatch(self._h, _ptr(wave), _ptr(order), n, _abi.DEVICE_PTRS,
                                           None, 0, _ptr(txn), C.byref(nw)), self._h)
            off = torch.empty(nw.value + 1, dtype=torch.int32, device=wave.device)
            _check(lib.dcc_calvin_dispatch(self._h, _ptr(wave), _ptr(order), n, _abi.DEVICE_PTRS,
                                           _ptr(off), nw.value + 1, _ptr(txn), C.byref(nw)),
                   self._h)
            return off, txn[:n]
        wave = np.ascontiguousarray(wave, np.uint32)
        order = None if order is None else np.ascontiguousarray(order, np.uint64)
        txn = np.empty(max(n, 1), np.uint32)
        _check(lib.dcc_calvin_dispatch(self._h, _ptr(wave), _ptr(order), n, 0, None, 0,
                                       _ptr(txn), C.byref(nw)), self._h)
        off = np.empty(nw.value + 1, np.uint32)
        _check(lib.dcc_calvin_dispatch(self._h, _ptr(wave), _ptr(order), n, 0, _ptr(off),
                                       off.size, _ptr(txn), C.byref(nw)), self._h)
        return off, txn[:n]

    # ----------------------------------------------------------- GPU index
    def index_insert(self, keys, rows) -> None:
        keys = np.ascontiguousarray(keys, np.uint64)
        rows = np.ascontiguousarray(rows, np.uint64)
        _check(lib.dcc_index_insert(self._h, _ptr(keys), _ptr(rows), keys.shape[0]), self._h)

    def index_probe(self, keys):
        """Rows of keys (DCC_ROW_NONE when absent) and the missing count."""
        miss = C.c_uint64(0)
        if hasattr(keys, "device") and str(keys.device).startswith("cuda"):
            import torch
            out = torch.empty(keys.shape[0], dtype=torch.int64, device=keys.device)
            _check(lib.dcc_index_probe(self._h, _ptr(keys), keys.shape[0], _ptr(out),
                                       _abi.DEVICE_PTRS, C.byref(miss)), self._h)
            return out, miss.value
        keys = np.ascontiguousarray(keys, np.uint64)
        out = np.empty(keys.shape[0], np.uint64)
        _check(lib.dcc_index_probe(self._h, _ptr(keys), keys.shape[0], _ptr(out), 0, C.byref(miss)),
               self._h)
        return out, miss.value

    def index_clear(self) -> None:
        _check(lib.dcc_index_clear(self._h), self._h)

    @property
    def index_size(self) -> int:
        return int(lib.dcc_index_size(self._h))

    @property
    def index_last_ms(self) -> float:
        return float(lib.dcc_index_last_ms(self._h))

    # ------------------------------------------------------------ multi-GPU
    def comm_init(self, rank: int, nranks: int, unique_id: bytes) -> None:
        buf = C.create_string_buffer(bytes(unique_id), _abi.UNIQUE_ID_BYTES)
        _check(lib.dcc_comm_init(self._h, rank, nranks, buf), self._h)

    def comm_init_host(self, rank: int, nranks: int, allreduce_max) -> None:
        """Shard this engine with a host-side exchange: ``allreduce_max(buf)``
        must MAX-all-reduce the uint8 numpy array ``buf`` in place across the
        ranks (e.g. torch.distributed over gloo)."""
        def _cb(user, ptr, n):
            try:
                if n:
                    allreduce_max(np.ctypeslib.as_array(ptr, shape=(int(n),)))
                return 0
            except Exception:  # noqa: BLE001 - reported as DCC_ECOMM by the engine
                import traceback
                traceback.print_exc()
                return 1
        self._exchange = _abi.EXCHANGE_FN(_cb)  # keep alive as long as the engine
        _check(lib.dcc_comm_init_host(self._h, rank, nranks,
                                      C.cast(self._exchange, C.c_void_p), None), self._h)

    @property
    def comm_rank(self) -> int:
        return int(lib.dcc_comm_rank(self._h))

    @property
    def comm_size(self) -> int:
        return int(lib.dcc_comm_size(self._h))

    @property
    def comm_calls(self) -> int:
        """Collectives run by this engine's communicator (dcc_comm_calls)."""
        return int(lib.dcc_comm_calls(self._h))

    def comm_destroy(self) -> None:
        _check(lib.dcc_comm_destroy(self._h), self._h)


def comm_unique_id() -> bytes:
    buf = C.create_string_buffer(_abi.UNIQUE_ID_BYTES)
    _check(lib.dcc_comm_unique_id(buf))
    return buf.raw


def key_shard(key: int, nranks: int) -> int:
    return int(lib.dcc_key_shard(key, nranks))


def shard_of_keys(keys, nranks: int) -> np.ndarray:
    """dcc_key_shard of every key (u32 array)."""
    k = np.ascontiguousarray(keys, dtype=np.uint64)
    out = np.empty(max(k.size, 1), np.uint32)
    _check(lib.dcc_key_shard_n(_ptr(k), k.size, nranks, _ptr(out)))
    return out[: k.size]


def shard_filter(batch: EpochBatch, rank: int, nranks: int) -> EpochBatch:
    n, nnz = batch.n_txn, batch.nnz
    off = np.empty(n + 1, np.uint32)
    keys = np.empty(max(nnz, 1), np.uint64)
    at = np.empty(max(nnz, 1), np.uint8)
    out = C.c_uint64()
    b = batch.to_c()
    _check(lib.dcc_shard_filter(C.byref(b), rank, nranks, _ptr(off), _ptr(keys), _ptr(at),
                                C.byref(out)))
    w = out.value
    return EpochBatch(off, keys[:w].copy(), at[:w].copy(), batch.start_tn, batch.finish_tn,
                      batch.order, dict(batch.meta, shard=(rank, nranks)))


def alg_bytes(n_txn: int, nnz: int, nnz_w: int) -> int:
    return int(lib.dcc_alg_bytes(n_txn, nnz, nnz_w))


def calvin_alg_bytes(n_txn: int, nnz: int, with_order: bool, with_wave: bool) -> int:
    return int(lib.dcc_calvin_alg_bytes(n_txn, nnz, int(with_order), int(with_wave)))


# ---------------------------------------------------------------- producers
def ycsb_params(**kw) -> _abi.YcsbParams:
    p = _abi.YcsbParams()
    lib.dcc_ycsb_params_default(C.byref(p))
    for k, v in kw.items():
        if not hasattr(p, k):
            raise TypeError(f"unknown YCSB parameter {k!r}")
        setattr(p, k, v)
    return p


def gen_ycsb(want_home: bool = False, **kw) -> EpochBatch:
    """Deterministic YCSB batch (gen_requests_zipf, ycsb_query.cpp:303-376)."""
    p = ycsb_params(**kw)
    n, k = p.n_txn, p.req_per_query
    off = np.empty(n + 1, np.uint32)
    keys = np.empty(max(n * k, 1), np.uint64)
    at = np.empty(max(n * k, 1), np.uint8)
    home = np.empty(max(n, 1), np.uint32) if want_home else None
    _check(lib.dcc_gen_ycsb(C.byref(p), _ptr(off), _ptr(keys), _ptr(at), _ptr(home)))
    meta = {"workload": "ycsb", **{f: getattr(p, f) for f, _ in p._fields_ if f != "reserved"}}
    b = EpochBatch(off, keys[: n * k], at[: n * k], meta=meta)
    if want_home:
        b.meta["home"] = home[:n]
    return b


def tpcc_params(**kw) -> _abi.TpccParams:
    p = _abi.TpccParams()
    lib.dcc_tpcc_params_default(C.byref(p))
    for k, v in kw.items():
        if not hasattr(p, k):
            raise TypeError(f"unknown TPC-C parameter {k!r}")
        setattr(p, k, v)
    return p


def gen_tpcc(**kw) -> EpochBatch:
    """Deterministic TPC-C NewOrder/Payment batch (tpcc_query.cpp:149-263)."""
    p = tpcc_params(**kw)
    n = p.n_txn
    cap = n * lib.dcc_tpcc_max_access(C.byref(p))
    off = np.empty(n + 1, np.uint32)
    keys = np.empty(max(cap, 1), np.uint64)
    at = np.empty(max(cap, 1), np.uint8)
    tt = np.empty(max(n, 1), np.uint8)
    out = C.c_uint64()
    _check(lib.dcc_gen_tpcc(C.byref(p), _ptr(off), _ptr(keys), _ptr(at), _ptr(tt), C.byref(out)))
    w = out.value
    meta = {"workload": "tpcc", "txn_type": tt[:n].copy(),
            **{f: getattr(p, f) for f, _ in p._fields_ if f != "reserved"}}
    return EpochBatch(off, keys[:w].copy(), at[:w].copy(), meta=meta)


# ---------------------------------------------------------------- batch files
def write_batch_file(path: str, batch: EpochBatch, kind: int = _abi.FILE_OCC, rc=None,
                     commit_tn=None, group=None, wave=None, seed: int = 0, epoch: int = 0,
                     tnc_before: int = 0) -> None:
    """One epoch (and optionally its decisions) as a .dccb file (dcc_file_write)."""
    info = _abi.FileInfo(kind=kind, seed=seed, epoch=epoch, tnc_before=tnc_before)

    def c(a, dt):
        return None if a is None else np.ascontiguousarray(a, dt)
    at = np.asarray(batch.acctype)
    if batch.meta.get("acctype_2bit"):  # the compact transfer form: unpack to one byte per access
        nnz = int(np.asarray(batch.keys).shape[0])
        at = ((np.repeat(at.astype(np.uint8), 4) >> np.tile(np.array([0, 2, 4, 6], np.uint8), at.size)) & 3)[:nnz]
    host = EpochBatch(c(batch.offsets, np.uint32), c(batch.keys, np.uint64),
                      c(at, np.uint8), c(batch.start_tn, np.uint64),
                      c(batch.finish_tn, np.uint64), c(batch.order, np.uint64))
    arrs = [c(rc, np.uint8), c(commit_tn, np.uint64), c(group, np.uint32), c(wave, np.uint32)]
    b = host.to_c()
    _check(lib.dcc_file_write(path.encode(), C.byref(info), C.byref(b),
                              *[_ptr(a) for a in arrs]))


def read_batch_file(path: str):
    """Returns (EpochBatch, info dict, decisions dict) of a .dccb file."""
    info = _abi.FileInfo()
    _check(lib.dcc_file_read_info(path.encode(), C.byref(info)))
    n, nnz, sec = info.n_txn, info.nnz, info.sections
    off = np.empty(n + 1, np.uint32)
    keys = np.empty(max(nnz, 1), np.uint64)
    at = np.empty(max(nnz, 1), np.uint8)
    has = lambda bit: bool(sec & bit)  # noqa: E731
    st = np.empty(max(n, 1), np.uint64) if has(_abi.FILE_HAS_TN) else None
    ft = np.empty(max(n, 1), np.uint64) if has(_abi.FILE_HAS_TN) else None
    od = np.empty(max(n, 1), np.uint64) if has(_abi.FILE_HAS_ORDER) else None
    rc = np.empty(max(n, 1), np.uint8) if has(_abi.FILE_HAS_RC) else None
    tn = np.empty(max(n, 1), np.uint64) if has(_abi.FILE_HAS_COMMIT_TN) else None
    gr = np.empty(max(nnz, 1), np.uint32) if has(_abi.FILE_HAS_GROUP) else None
    wv = np.empty(max(n, 1), np.uint32) if has(_abi.FILE_HAS_WAVE) else None
    _check(lib.dcc_file_read(path.encode(), *[_ptr(a) for a in (off, keys, at, st, ft, od, rc,
                                                                   tn, gr, wv)]))
    cut = lambda a, k: None if a is None else a[:k]  # noqa: E731
    b = EpochBatch(off, keys[:nnz], at[:nnz], cut(st, n), cut(ft, n), cut(od, n))
    meta = {f: getattr(info, f) for f, _ in info._fields_ if f != "reserved"}
    dec = {"rc": cut(rc, n), "commit_tn": cut(tn, n), "group": cut(gr, nnz), "wave": cut(wv, n)}
    return b, meta, dec
