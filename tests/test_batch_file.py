"""The .dccb epoch file format (batch_file.cpp):
round trips of every section, and loud failures on corrupted, truncated or
foreign files.  CPU only."""
import os

import numpy as np
import pytest

import deneva_amd as d
from deneva_amd import DccError
from deneva_amd._abi import FILE_CALVIN, FILE_HAS_ORDER, FILE_HAS_RC, FILE_HAS_TN, FILE_OCC
from helpers import make_batch


def test_roundtrip_all_sections(tmp_path):
    b = d.gen_ycsb(n_txn=3000, zipf_theta=0.9, seed=5)
    n = b.n_txn
    rng = np.random.default_rng(0)
    b.start_tn = rng.integers(0, 1 << 40, size=n).astype(np.uint64)
    b.finish_tn = b.start_tn + 7
    b.order = np.arange(n, dtype=np.uint64)[::-1].copy()
    rc = rng.integers(0, 3, size=n).astype(np.uint8)
    tn = rng.integers(0, 100, size=n).astype(np.uint64)
    grp = rng.integers(0, 9, size=b.nnz).astype(np.uint32)
    wav = rng.integers(0, 9, size=n).astype(np.uint32)
    p = str(tmp_path / "e.dccb")
    d.write_batch_file(p, b, kind=FILE_CALVIN, rc=rc, commit_tn=tn, group=grp, wave=wav,
                       seed=0xD3E7A001, epoch=3, tnc_before=99)
    b2, meta, dec = d.read_batch_file(p)
    for f in ("offsets", "keys", "acctype", "start_tn", "finish_tn", "order"):
        assert np.array_equal(getattr(b, f), getattr(b2, f)), f
    assert np.array_equal(dec["rc"], rc) and np.array_equal(dec["commit_tn"], tn)
    assert np.array_equal(dec["group"], grp) and np.array_equal(dec["wave"], wav)
    assert meta["kind"] == FILE_CALVIN and meta["seed"] == 0xD3E7A001
    assert meta["epoch"] == 3 and meta["tnc_before"] == 99 and meta["n_txn"] == n


def test_minimal_and_empty(tmp_path):
    p = str(tmp_path / "m.dccb")
    b = make_batch([[(1, 0), (2, 1)], [], [(3, 3)]])
    d.write_batch_file(p, b)
    b2, meta, dec = d.read_batch_file(p)
    assert meta["sections"] == 0 and meta["kind"] == FILE_OCC
    assert b2.start_tn is None and dec["rc"] is None
    assert list(b2.offsets) == [0, 2, 2, 3] and list(b2.keys) == [1, 2, 3]
    d.write_batch_file(p, make_batch([]))
    b3, meta, _ = d.read_batch_file(p)
    assert b3.n_txn == 0 and meta["nnz"] == 0


def test_sections_flags(tmp_path):
    p = str(tmp_path / "f.dccb")
    b = make_batch([[(1, 1)], [(1, 0)]], start_tn=[1, 2], finish_tn=[3, 4])
    d.write_batch_file(p, b, rc=np.array([0, 2], np.uint8))
    _, meta, dec = d.read_batch_file(p)
    assert meta["sections"] == FILE_HAS_TN | FILE_HAS_RC
    assert not meta["sections"] & FILE_HAS_ORDER
    assert list(dec["rc"]) == [0, 2]


def test_corruption_detected(tmp_path):
    p = str(tmp_path / "c.dccb")
    d.write_batch_file(p, d.gen_ycsb(n_txn=500, seed=2))
    raw = bytearray(open(p, "rb").read())
    raw[64 + 4 * 501 + 13] ^= 0x40  # a key byte
    open(p, "wb").write(bytes(raw))
    with pytest.raises(DccError):
        d.read_batch_file(p)


def test_truncated_and_foreign(tmp_path):
    p = str(tmp_path / "t.dccb")
    d.write_batch_file(p, d.gen_ycsb(n_txn=500, seed=2))
    raw = open(p, "rb").read()
    open(p, "wb").write(raw[: len(raw) - 100])
    with pytest.raises(DccError):
        d.read_batch_file(p)
    open(p, "wb").write(b"not a dccb file" * 10)
    with pytest.raises(DccError):
        d.read_batch_file(p)
    with pytest.raises(DccError):
        d.read_batch_file(str(tmp_path / "missing.dccb"))
    bad = bytearray(raw)
    bad[4:6] = (3).to_bytes(2, "little")  # a future version
    open(p, "wb").write(bytes(bad))
    with pytest.raises(DccError):
        d.read_batch_file(p)
    # version 2 checksums the header too: a flipped seed / epoch is caught
    for pos in (32, 41, 50, 6, 9):
        bad = bytearray(raw)
        bad[pos] ^= 0x5A
        open(p, "wb").write(bytes(bad))
        with pytest.raises(DccError):
            d.read_batch_file(p)
    # trailing bytes are rejected
    open(p, "wb").write(raw + b"\0" * 8)
    with pytest.raises(DccError):
        d.read_batch_file(p)


def test_golden_fixture_file():
    """The committed C1-shape fixture decodes, and its stored decisions are the
    oracle's (tests/golden/*.dccb are written by tests/golden/make_fixtures.py)."""
    import _oracle as orc
    p = os.path.join(os.path.dirname(__file__), "golden", "c1_ycsb_theta06_seed7.dccb")
    b, meta, dec = d.read_batch_file(p)
    rc, tn, _ = orc.occ(b, literal=True)
    assert np.array_equal(rc, dec["rc"]) and np.array_equal(tn, dec["commit_tn"])


def test_compact_forms(tmp_path):
    """A batch in the compact transfer form (u32 keys, 2-bit access types,
    u32 timestamps: dcc.h DCC_KEYS_U32 / ACCTYPE_2BIT / TN_U32) is written
    full width by write_batch_file; the C writer and the host shard filter
    refuse compact flags instead of misreading the narrow arrays."""
    import ctypes as C
    from deneva_amd import _abi
    b = d.gen_ycsb(n_txn=777, zipf_theta=0.9, seed=11)
    b.start_tn = np.arange(b.n_txn, dtype=np.uint64)
    b.finish_tn = b.start_tn + 3
    cb = d.EpochBatch(np.asarray(b.offsets, np.uint32), np.asarray(b.keys, np.uint32),
                      d.engine.pack_acctype(b.acctype), b.start_tn.astype(np.uint32),
                      b.finish_tn.astype(np.uint32), meta={"acctype_2bit": True})
    p = str(tmp_path / "c.dccb")
    d.write_batch_file(p, cb)
    b2, _, _ = d.read_batch_file(p)
    for f in ("offsets", "keys", "acctype", "start_tn", "finish_tn"):
        assert np.array_equal(np.asarray(getattr(b, f)), getattr(b2, f)), f
    raw = cb.to_c()
    assert raw.flags & _abi.KEYS_U32 and raw.flags & _abi.ACCTYPE_2BIT and raw.flags & _abi.TN_U32
    info = _abi.FileInfo(kind=FILE_OCC)
    assert _abi.lib.dcc_file_write(p.encode(), C.byref(info), C.byref(raw), None, None, None,
                                   None) == _abi.DCC_EINVAL
    off = np.empty(b.n_txn + 1, np.uint32)
    keys = np.empty(b.nnz, np.uint64)
    at = np.empty(b.nnz, np.uint8)
    w = C.c_uint64()
    assert _abi.lib.dcc_shard_filter(C.byref(raw), 0, 2, off.ctypes.data, keys.ctypes.data,
                                     at.ctypes.data, C.byref(w)) == _abi.DCC_EINVAL


def test_to_c_rejects_ambiguous_dtypes():
    b = d.gen_ycsb(n_txn=50, zipf_theta=0.9, seed=12)
    with pytest.raises(TypeError):  # signed 4-byte keys are not row ids
        d.EpochBatch(b.offsets, np.asarray(b.keys, np.int32), b.acctype).to_c()
    with pytest.raises(TypeError):  # mixed timestamp widths
        d.EpochBatch(b.offsets, b.keys, b.acctype, np.zeros(50, np.uint32),
                     np.zeros(50, np.uint64)).to_c()
