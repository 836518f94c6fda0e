"""CPU tests of the C ABI surface and the host-side logic of libkme.so (no device compute).

* the shared object loads (no undefined symbols) and exports every function include/kme.h and
  include/kme_processor.h declare;
* struct layouts seen by C (gcc on the public headers) match the ctypes mirror;
* the Jackson-compatible deserializer and the tape serializer (KP:477-521), the Kafka murmur2
  partitioner;
* creating an engine without a GPU fails loudly (no CPU fallback exists).
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from kme import workloads as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in ("kme.h", "kme_processor.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names |= set(re.findall(r"\b(kme_[a-z_]+)\s*\(", txt))
    return names


def test_library_loads_and_exports_every_declared_symbol(kme_mod):
    lib = C.CDLL(kme_mod.LIB_PATH)  # raises on undefined symbols
    declared = declared_functions()
    assert declared == set(kme_mod.EXPORTS)
    nm = subprocess.run(["nm", "-D", "--defined-only", kme_mod.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (kme_[a-z_]+)$", nm, flags=re.M))
    missing = declared - exported
    assert not missing, missing
    for name in declared:
        getattr(lib, name)


def test_struct_layouts_match_the_header(kme_mod, tmp_path):
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "kme.h"\n'
                   'int main(){printf("%zu %zu %zu %zu %zu %zu %zu\\n", sizeof(kme_config), sizeof(kme_orders),'
                   'sizeof(kme_trade), sizeof(kme_epoch_result), sizeof(kme_epoch_status), sizeof(kme_tob),'
                   'offsetof(kme_epoch_status, n_orders));return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = [C.sizeof(kme_mod.kme_config), C.sizeof(kme_mod.kme_orders), kme_mod.TRADE_DTYPE.itemsize,
            C.sizeof(kme_mod.kme_epoch_result), C.sizeof(kme_mod.kme_epoch_status), kme_mod.TOB_DTYPE.itemsize,
            kme_mod.kme_epoch_status.n_orders.offset]
    assert got == want


@pytest.mark.parametrize("text,want", [
    ('{"action":2,"oid":123,"aid":1,"sid":0,"price":50,"size":49}', (2, 123, 1, 0, 50, 49)),
    ('{"action":4,"oid":"8796093022208","aid":3,"sid":0,"price":0,"size":0}', (4, 8796093022208, 3, 0, 0, 0)),
    ('{"action":2,"oid":5,"aid":1,"sid":-2,"price":50.9,"size":-3,"next":null,"prev":null}', (2, 5, 1, -2, 50, -3)),
    ('{"aid":7}', (0, 0, 7, 0, 0, 0)),                                   # missing creator props -> 0
    (' { "size" : "12" , "action" : 3 } ', (3, 0, 0, 0, 0, 12)),
    ('{"action":2,"oid":9223372036854775807,"aid":-9223372036854775808,"sid":1,"price":2147483647,"size":-2147483648}',
     (2, 9223372036854775807, -9223372036854775808, 1, 2147483647, -2147483648)),
])
def test_json_deserializer_follows_jackson_defaults(kme_mod, text, want):
    assert kme_mod.order_from_json(text) == want


@pytest.mark.parametrize("text,status", [
    ('{"action":2,"oid":1,"bogus":1}', 1),              # FAIL_ON_UNKNOWN_PROPERTIES
    ('{"action":true}', 1),
    ('{"price":2147483648}', 1),                        # int overflow
    ('{"oid":9223372036854775808}', 1),
    ('{"action":2', 1),
    ('{"action":2,"next":17}', 3),                      # linked input orders are outside the domain
])
def test_json_deserializer_rejects(kme_mod, text, status):
    with pytest.raises(kme_mod.KmeError) as e:
        kme_mod.order_from_json(text)
    assert e.value.status == status


def test_murmur2_partitioner_matches_python_restatement(kme_mod):
    for sid in list(range(-50, 2000)) + [2**31, 2**40 + 7, -(2**62), 9223372036854775807]:
        for n in (1, 2, 3, 4, 8, 13):
            assert kme_mod.shard_of(sid, n) == W.shard_of(sid, n)


def test_tape_serializer_layout(kme_mod):
    """Hand-built result of one BUY that traded twice and rested; serialised like consumer.js."""
    orders = W.Orders.from_rows([(2, 77, 3, 5, 60, 10)])
    trades = np.zeros(2, kme_mod.TRADE_DTYPE)
    trades[0] = (11, 1, 5, 55, 4)
    trades[1] = (12, 2, 5, 58, 3)
    res = kme_mod.EpochResult(np.array([2], np.int32), np.array([3], np.int32), np.array([66], np.int64),
                              np.array([1], np.uint8), np.array([0, 2], np.uint32), trades, kme_mod.kme_epoch_status())
    want = ('IN {"action":2,"oid":77,"aid":3,"sid":5,"price":60,"size":10,"next":null,"prev":null}\n'
            'OUT {"action":6,"oid":11,"aid":1,"sid":5,"price":0,"size":4,"next":null,"prev":null}\n'
            'OUT {"action":5,"oid":77,"aid":3,"sid":5,"price":5,"size":4,"next":null,"prev":null}\n'
            'OUT {"action":6,"oid":12,"aid":2,"sid":5,"price":0,"size":3,"next":null,"prev":null}\n'
            'OUT {"action":5,"oid":77,"aid":3,"sid":5,"price":2,"size":3,"next":null,"prev":null}\n'
            'OUT {"action":2,"oid":77,"aid":3,"sid":5,"price":60,"size":3,"next":null,"prev":66}\n')
    assert res.tape_json(orders) == want


def test_tape_serializer_agrees_with_oracle_on_echo_records(kme_mod, oracle_mod):
    """Records that never trade: the serializer's IN/OUT echo equals the oracle's Jackson output."""
    rows = [(100, 0, 1, 0, 0, 0), (101, 0, 1, 0, 0, -5), (0, 0, 0, -3, 0, 0), (42, -1, -2, -3, -4, -5),
            (4, 2**62, 1, 0, 0, 0)]
    orders = W.Orders.from_rows(rows)
    o = oracle_mod.Oracle()
    o.process(orders)
    tape = o.tape()
    outs = tape[tape["key"] == 1]
    n = len(orders)
    res = kme_mod.EpochResult(outs["action"].astype(np.int32), outs["size"].astype(np.int32), np.zeros(n, np.int64),
                              np.zeros(n, np.uint8), np.zeros(n + 1, np.uint32), np.zeros(0, kme_mod.TRADE_DTYPE),
                              kme_mod.kme_epoch_status())
    assert res.tape_json(orders) == o.tape_text()


def test_status_strings(kme_mod):
    L = kme_mod.lib()
    for s in range(8):
        assert L.kme_strerror(s)
    assert b"KP:341-353" in L.kme_domain_str(5)


def test_engine_creation_fails_loudly_without_gpu(kme_mod):
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(kme_mod.KmeError) as e:
        kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, 8, 1024, 1024, max_accounts=8))
    assert e.value.status == 6                                   # KME_E_HIP: no CPU fallback


def test_invalid_config_rejected_before_touching_the_device(kme_mod):
    cfg = kme_mod.default_config(kme_mod.MODE_FUNDED, 8, 1024, 1024, max_accounts=0)
    with pytest.raises(kme_mod.KmeError) as e:
        kme_mod.Engine(cfg)
    assert e.value.status == 1


def test_funded_capacity_bound_on_the_oid_table(kme_mod):
    # FUNDED: max_resting + 64 (max_symbols + 1) + max_epoch <= 2^29 (kme.h), so that the oid table
    # stays within 2^30 entries and an entry's position fits the packed record's signed word
    cfg = kme_mod.default_config(kme_mod.MODE_FUNDED, 8, 1024, (1 << 29) - 64 * 9 - 1024 + 1, max_accounts=8)
    with pytest.raises(kme_mod.KmeError) as e:
        kme_mod.Engine(cfg)
    assert e.value.status == 1                                   # KME_E_INVALID, before any device call


def test_expand_rows_order_and_values(kme_mod):
    """kme_expand_rows (the JNI glue's row expansion, host only): IN, per trade the maker fill then the
    taker fill (executeTrade, KP:265-274), OUT with prev when set (KP:217)."""
    import numpy as np

    from kme import workloads as W

    orders = W.Orders.from_rows([(W.SELL, 11, 1, 5, 40, 10), (W.BUY, 12, 2, 5, 45, 4), (W.BUY, 13, 3, 5, 30, 7)])
    res = kme_mod.new_result(3, 4)
    res.out_action[:] = [W.SELL, W.BUY, W.BUY]
    res.out_size[:] = [10, 0, 7]
    res.out_flags[:] = [0, 0, 1]
    res.out_prev[:] = [0, 0, 99]
    res.trade_off[:] = [0, 0, 1, 1]
    res.trades[0] = (11, 1, -5, 40, 4)
    rows = kme_mod.expand_rows(orders, res)
    assert list(rows["kind"]) == [0, 2, 0, 1, 1, 2, 0, 2]
    assert list(rows["action"]) == [W.SELL, W.SELL, W.BUY, W.SOLD, W.BOUGHT, W.BUY, W.BUY, W.BUY]
    maker, taker = rows[3], rows[4]
    assert (maker["oid"], maker["aid"], maker["sid"], maker["price"], maker["size"]) == (11, 1, -5, 0, 4)
    assert (taker["oid"], taker["aid"], taker["sid"], taker["price"], taker["size"]) == (12, 2, 5, 5, 4)
    assert rows[7]["has_prev"] == 1 and rows[7]["prev"] == 99 and rows[5]["has_prev"] == 0
    # too small a buffer: nothing written, the count returned
    import ctypes as C

    L = kme_mod.lib()
    s, keep = kme_mod._soa(orders)
    r = kme_mod.kme_epoch_result(*[C.c_void_p(a.ctypes.data) for a in (res.out_action, res.out_size, res.out_prev,
                                                                        res.out_flags, res.trade_off, res.trades)], 4)
    need = C.c_size_t(0)
    small = np.zeros(3, kme_mod.ROW_DTYPE)
    assert L.kme_expand_rows(C.byref(s), 3, C.byref(r), C.c_void_p(small.ctypes.data), 3, C.byref(need)) == 2
    assert need.value == 8 and not small["oid"].any()


@pytest.mark.parametrize("threads", [0, 3, 16])
def test_expand_rows_threads_equal_one_thread(kme_mod, threads):
    """kme_expand_rows_mt: each thread's range starts where trade_off puts it; the rows are those of
    kme_expand_rows, byte for byte (ragged trade counts, an epoch not a multiple of the ranges)."""
    import numpy as np

    from kme import workloads as W

    n = 50_001
    rng = np.random.Generator(np.random.PCG64(5))
    orders = W.uniform(n, n_symbols=64, n_accounts=128, seed=5)
    counts = np.where(rng.random(n) < 0.3, rng.integers(1, 6, n), 0).astype(np.uint32)
    off = np.zeros(n + 1, np.uint32)
    off[1:] = np.cumsum(counts)
    res = kme_mod.new_result(n, int(off[-1]))
    res.out_action[:] = orders.action
    res.out_size[:] = rng.integers(0, 100, n)
    res.out_flags[:] = rng.integers(0, 2, n)
    res.out_prev[:] = rng.integers(1, 1 << 40, n)
    res.trade_off[:] = off
    t = res.trades
    t["maker_oid"] = rng.integers(1, 1 << 40, len(t))
    t["size"] = rng.integers(0, 50, len(t))
    one = kme_mod.expand_rows(orders, res)
    many = kme_mod.expand_rows(orders, res, threads=threads)
    assert len(one) == 2 * n + 2 * int(off[-1])
    assert one.tobytes() == many.tobytes()


def test_expand_rows_pool_under_concurrent_calls(kme_mod):
    """kme_expand_rows_mt's persistent workers: back-to-back calls and calls from several host threads
    at once (one uses the pool, the others start threads of their own) give kme_expand_rows's rows."""
    import threading

    import numpy as np

    from kme import workloads as W

    n = 40_000
    rng = np.random.Generator(np.random.PCG64(11))
    orders = W.uniform(n, n_symbols=64, n_accounts=128, seed=11)
    counts = np.where(rng.random(n) < 0.4, rng.integers(1, 4, n), 0).astype(np.uint32)
    off = np.zeros(n + 1, np.uint32)
    off[1:] = np.cumsum(counts)
    res = kme_mod.new_result(n, int(off[-1]))
    res.out_action[:] = orders.action
    res.out_size[:] = rng.integers(0, 100, n)
    res.trade_off[:] = off
    res.trades["maker_oid"] = rng.integers(1, 1 << 40, len(res.trades))
    want = kme_mod.expand_rows(orders, res).tobytes()
    bad = []

    def run():
        for _ in range(12):
            if kme_mod.expand_rows(orders, res, threads=8).tobytes() != want:
                bad.append(1)

    th = [threading.Thread(target=run) for _ in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not bad


@pytest.mark.parametrize("misalign", [0, 8])
def test_expand_rows_streaming_and_unaligned_buffers_agree(kme_mod, misalign):
    """The row writer streams 16-B stores into a 16-B aligned buffer and falls back to ordinary
    stores otherwise: both give kme_expand_rows's rows byte for byte."""
    import ctypes as C

    import numpy as np

    from kme import workloads as W

    n = 20_000
    rng = np.random.Generator(np.random.PCG64(31))
    orders = W.uniform(n, n_symbols=64, n_accounts=128, seed=31)
    counts = np.where(rng.random(n) < 0.4, rng.integers(1, 4, n), 0).astype(np.uint32)
    off = np.zeros(n + 1, np.uint32)
    off[1:] = np.cumsum(counts)
    res = kme_mod.new_result(n, int(off[-1]))
    res.out_action[:] = orders.action
    res.out_size[:] = rng.integers(0, 100, n)
    res.out_flags[:] = rng.integers(0, 2, n)
    res.out_prev[:] = rng.integers(1, 1 << 40, n)
    res.trade_off[:] = off
    res.trades["maker_oid"] = rng.integers(1, 1 << 40, len(res.trades))
    want = kme_mod.expand_rows(orders, res)
    L = kme_mod.lib()
    s, keep = kme_mod._soa(orders)
    r = kme_mod.kme_epoch_result(kme_mod._np_ptr(res.out_action), kme_mod._np_ptr(res.out_size),
                                 kme_mod._np_ptr(res.out_prev), kme_mod._np_ptr(res.out_flags),
                                 kme_mod._np_ptr(res.trade_off), kme_mod._np_ptr(res.trades), len(res.trades))
    raw = np.zeros(want.nbytes + 64, np.uint8)
    base = (-raw.ctypes.data) % 16 + misalign            # 16-B aligned, or 8 B past it
    need = C.c_size_t(0)
    for threads in (1, 4):
        raw[:] = 0
        buf = C.c_void_p(raw.ctypes.data + base)
        if threads == 1:
            rc = L.kme_expand_rows(C.byref(s), n, C.byref(r), buf, len(want), C.byref(need))
        else:
            rc = L.kme_expand_rows_mt(C.byref(s), n, C.byref(r), buf, len(want), C.byref(need), threads)
        assert rc == 0 and need.value == len(want)
        assert raw[base:base + want.nbytes].tobytes() == want.tobytes()
    del keep


def test_checkpoint_chunks_change_only_where_the_bytes_change(kme_mod, tmp_path):
    """kme_checkpoint_chunks (the state changelog's unit): fixed-size chunks, the
    last one shorter; a byte changed changes that chunk's hash only; a file that grows adds chunks at
    its end and changes the one it ended in."""
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 5 * 4096 + 1000, dtype=np.uint8).tobytes()
    f = tmp_path / "x.ckpt"
    f.write_bytes(data)
    h0 = kme_mod.checkpoint_chunks(f, 4096)
    assert len(h0) == 6 and len(set(h0.tolist())) == 6
    d = bytearray(data)
    d[2 * 4096 + 17] ^= 1
    f.write_bytes(bytes(d))
    h1 = kme_mod.checkpoint_chunks(f, 4096)
    assert [k for k in range(6) if h0[k] != h1[k]] == [2]
    f.write_bytes(bytes(d) + b"\x00" * 9000)
    h2 = kme_mod.checkpoint_chunks(f, 4096)
    assert len(h2) == 8 and (h2[:5] == h1[:5]).all() and h2[5] != h1[5]
    with pytest.raises(kme_mod.KmeError):
        kme_mod.checkpoint_chunks(f, 1024)                       # below the minimum chunk


def test_checkpoint_inspect_reads_both_trailer_formats(kme_mod, tmp_path):
    """kme_checkpoint_inspect reads the trailer only (the commit log checks a file against it): the
    round-6 tree digest (KMEDGST2: block digests of the file, written and verified on host threads)
    and the older stream digest (KMEDGST1) both; anything else is refused."""
    import struct

    body = bytes(range(256)) * 40
    for magic in (b"KMEDGST1", b"KMEDGST2"):
        f = tmp_path / ("t" + magic.decode()[-1] + ".ckpt")
        f.write_bytes(body + struct.pack("<QQ8s", 7, 0x1234567890ABCDEF, magic))
        info = kme_mod.checkpoint_inspect(f)
        assert info["file_bytes"] == len(body) + 24 and info["app_bytes"] == 7 and info["digest"] == 0x1234567890ABCDEF
    bad = tmp_path / "bad.ckpt"
    bad.write_bytes(body + struct.pack("<QQ8s", 7, 1, b"KMEDGSTX"))
    with pytest.raises(kme_mod.KmeError):
        kme_mod.checkpoint_inspect(bad)
