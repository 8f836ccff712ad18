"""CPU: libdcc.so loads, exports every symbol include/dcc.h declares, behaves
without a GPU, and its batch producers are deterministic restatements of the
reference generators."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import deneva_amd as d
from deneva_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "dcc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(dcc_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_symbols_exported():
    names = header_functions()
    assert len(names) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (dcc_\w+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, f"declared but not exported: {missing}"
    assert set(names) == set(_abi.EXPORTED), "python binding out of sync with dcc.h"


def test_strerror_and_version():
    assert _abi.lib.dcc_version() >= 100
    for code in (0, -5, -12, -19, -22, -34, -70, -95):
        assert _abi.strerror(code)


def test_init_without_gpu_fails_cleanly():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except Exception:
        pass
    h = C.c_void_p()
    code = _abi.lib.dcc_init(C.byref(h), 0)
    assert code == d._abi.DCC_ENODEV and not h.value


def test_alg_bytes_formula():
    # 4(N+1) + 9 nnz + 16 nnz_w + 16 nnz + N
    assert d.alg_bytes(1 << 20, 16 << 20, 4 << 20) == \
        4 * ((1 << 20) + 1) + 9 * (16 << 20) + 16 * (4 << 20) + 16 * (16 << 20) + (1 << 20)


def test_ycsb_generator_properties():
    b = d.gen_ycsb(n_txn=20000, zipf_theta=0.9, req_per_query=16, table_size=1 << 24)
    assert b.n_txn == 20000 and b.nnz == 20000 * 16
    assert np.array_equal(b.offsets, np.arange(20001, dtype=np.uint32) * 16)
    k = b.keys.reshape(-1, 16)
    # unique keys per txn (ycsb_query.cpp:342-350)
    s = np.sort(k, axis=1)
    assert (np.diff(s, axis=1) != 0).all()
    # zipf draws are in [1, n]: row 0 never appears (ycsb_query.cpp:199-201)
    assert k.min() >= 1 and k.max() < (1 << 24)
    at = b.acctype.reshape(-1, 16)
    ro = (at == d.RD).all(axis=1).mean()
    assert 0.45 < ro < 0.6  # TXN_WRITE_PERC 0.5 (+ all-read draws)
    wfrac = (at[(at == d.WR).any(axis=1)] == d.WR).mean()
    assert 0.45 < wfrac < 0.55  # TUP_WRITE_PERC 0.5
    # hot key 1 is the most frequent
    vals, cnt = np.unique(k, return_counts=True)
    assert vals[np.argmax(cnt)] == 1


def test_ycsb_generator_deterministic_and_parallel():
    a = d.gen_ycsb(n_txn=70000, n_threads=1, seed=123)
    b = d.gen_ycsb(n_txn=70000, n_threads=8, seed=123)
    c = d.gen_ycsb(n_txn=70000, n_threads=8, seed=124)
    assert np.array_equal(a.keys, b.keys) and np.array_equal(a.acctype, b.acctype)
    assert not np.array_equal(a.keys, c.keys)


def test_ycsb_generator_golden_digest():
    # regression pin of the generator stream (myrand + zipf restatement)
    b = d.gen_ycsb(n_txn=1000, zipf_theta=0.9, seed=0xD3E7A001)
    import hashlib
    h = hashlib.sha256(b.keys.tobytes() + b.acctype.tobytes()).hexdigest()
    golden = open(os.path.join(ROOT, "tests", "golden", "ycsb_1000_seed_D3E7A001.sha256")).read()
    assert h == golden.strip()


def test_ycsb_partitions():
    b = d.gen_ycsb(n_txn=4096, part_cnt=16, chunk_txns=256, want_home=True,
                   table_size=1 << 20)
    k = b.keys.reshape(-1, 16)
    home = b.meta["home"]
    # first key is home-partition local (FIRST_PART_LOCAL, config.h:158)
    assert np.array_equal(k[:, 0] % 16, home)
    assert np.array_equal(home, (np.arange(4096) // 256) % 16)


def test_myrand_restatement():
    # helper.cpp:144-147: seed = (seed*1103515247 + 12345) % 2^63; (seed/65537) % RAND_MAX
    seed = 7
    out = []
    for _ in range(5):
        seed = (seed * 1103515247 + 12345) % (1 << 64) % (1 << 63)
        out.append((seed // 65537) % 2147483647)
    assert all(0 <= v < 2147483647 for v in out)


def test_shard_filter_partitions_accesses():
    b = d.gen_ycsb(n_txn=3000, zipf_theta=0.9)
    parts = [d.shard_filter(b, r, 4) for r in range(4)]
    assert sum(p.nnz for p in parts) == b.nnz
    for r, p in enumerate(parts):
        assert p.n_txn == b.n_txn
        assert all(d.key_shard(int(x), 4) == r for x in p.keys[:200])
    # per txn, the shards' access counts add up
    cnt = sum(np.diff(p.offsets.astype(np.int64)) for p in parts)
    assert np.array_equal(cnt, np.diff(b.offsets.astype(np.int64)))
    assert d.key_shard(12345, 1) == 0


def test_tpcc_generator_access_sets():
    # Payment: WH (WR, WH_UPDATE) / DIST WR / CUST WR; NewOrder: WH RD, CUST RD,
    # DIST WR, then ITEM RD + STOCK WR per order line (tpcc_txn.cpp:140-230)
    b = d.gen_tpcc(n_txn=20000, num_wh=16)
    tt = b.meta["txn_type"]
    off = b.offsets.astype(np.int64)
    L = np.diff(off)
    assert set(np.unique(tt)) == {1, 2}
    assert 0.45 < (tt == 1).mean() < 0.55                       # PERC_PAYMENT 0.5
    assert (L[tt == 1] == 3).all()
    assert L[tt == 2].min() >= 3 + 2 * 5 and L[tt == 2].max() <= 3 + 2 * 15  # ol_cnt in [5,15]
    tbl = (b.keys >> np.uint64(56)).astype(np.int64)
    low = b.keys & np.uint64((1 << 56) - 1)
    for t in np.nonzero(tt == 1)[0][:300]:
        s = off[t]
        assert list(tbl[s:s + 3]) == [0, 1, 2] and list(b.acctype[s:s + 3]) == [d.WR] * 3
        assert 1 <= low[s] <= 16
    for t in np.nonzero(tt == 2)[0][:300]:
        s, e = off[t], off[t + 1]
        assert list(tbl[s:s + 3]) == [0, 2, 1]
        assert list(b.acctype[s:s + 3]) == [d.RD, d.RD, d.WR]
        assert (tbl[s + 3:e:2] == 7).all() and (tbl[s + 4:e:2] == 8).all()
        assert (b.acctype[s + 3:e:2] == d.RD).all() and (b.acctype[s + 4:e:2] == d.WR).all()
        items = low[s + 3:e:2]
        assert len(np.unique(items)) == len(items)               # distinct ol_i_id
        assert items.min() >= 1 and items.max() <= 100000
        w = int(low[s])
        # district key = w * DIST_PER_WH + d (tpcc_helper.cpp:19-21)
        assert w * 10 + 1 <= int(low[s + 2]) <= w * 10 + 10
    b2 = d.gen_tpcc(n_txn=4096, num_wh=4, wh_update=0)
    pay = b2.meta["txn_type"] == 1
    assert (b2.acctype[b2.offsets[:-1][pay]] == d.RD).all()      # WH_UPDATE false -> RD


def test_tpcc_generator_golden_digest_and_threads():
    import hashlib
    b = d.gen_tpcc(n_txn=4096, seed=0xD3E7A003)
    h = hashlib.sha256(b.offsets.tobytes() + b.keys.tobytes() + b.acctype.tobytes()).hexdigest()
    golden = open(os.path.join(ROOT, "tests", "golden", "tpcc_4096_seed_D3E7A003.sha256")).read()
    assert h == golden.strip()
    b1 = d.gen_tpcc(n_txn=150000, chunk_txns=4096, n_threads=1)
    b8 = d.gen_tpcc(n_txn=150000, chunk_txns=4096, n_threads=8)
    assert np.array_equal(b1.keys, b8.keys) and np.array_equal(b1.offsets, b8.offsets)
