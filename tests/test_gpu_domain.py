"""GPU tests: the FUNDED engine with the drop-in's flags (exact ledger + serial fallback) takes every
record the reference takes (round-5 verdict, What's missing 1), and the restart / oid-table cases of
the round-5 fault analysis.

Reference: KP:131-146 (accounts), 167-182 (checkBalance), 184-191 (addSymbol), 200-223 (addOrder),
289-333 (removeOrder), 391-404 (the level bitmaps), 451-456 (Order's field types).
"""
import os

import numpy as np
import pytest

import domain_stream as D
from kme import workloads as W

pytestmark = pytest.mark.gpu

FLAGS3 = 3   # KME_FLAG_EXACT_LEDGER | KME_FLAG_SERIAL_FALLBACK: GpuMatchingEngine()'s


def _first_diff(a: str, b: str) -> str:
    la, lb = a.splitlines(), b.splitlines()
    for k, (x, y) in enumerate(zip(la, lb)):
        if x != y:
            return f"line {k}: got {x!r} want {y!r}"
    return f"length got {len(la)} want {len(lb)}"


def _drop_in_engine(kme, light_max=0, E=4096, G=8, A=64, sparse=0):
    return kme.Engine(kme.default_config(kme.MODE_FUNDED, max_symbols=G, max_epoch=E, max_resting=1 << 16,
                                         max_accounts=A, ledger_capacity=1 << 14, light_max=light_max,
                                         flags=FLAGS3, max_sparse_symbols=sparse))


def _run(eng, orders, epoch):
    text, serial, epochs = [], 0, 0
    for a in range(0, len(orders), epoch):
        part = orders.slice(a, min(len(orders), a + epoch))
        r = eng.process(part)
        text.append(r.tape_json(part))
        serial += int(r.status.serial_fallback)
        epochs += 1
    return "".join(text), serial, epochs


@pytest.mark.parametrize("light_max,epoch", [(0, 2048), (-1, 997), (1 << 30, 4096)])
def test_drop_in_flags_take_the_reference_domain(kme_mod, oracle_mod, light_max, epoch):
    """exchange_test.js's stream, untruncated, with a sparse symbol (10^12), an account id of 2^40,
    prices 101..125 and negative sizes spliced in (tests/domain_stream.py): the FUNDED engine with the
    drop-in's flags answers all of it as the reference does -- tape, books and exact ledger equal the
    oracle's -- the epochs holding such records (or touching a book that holds such an order) serially,
    the others in parallel."""
    orders = D.reference_domain_stream(oracle_mod)
    o = oracle_mod.Oracle()
    o.process(orders)                      # (the reference takes the whole stream: no NPE, no hang)
    eng = _drop_in_engine(kme_mod, light_max)
    got, serial, epochs = _run(eng, orders, epoch)
    want = o.tape_text()
    assert got == want, _first_diff(got, want)
    assert eng.snapshot_books() == o.dump_books()
    assert eng.snapshot_ledger() == o.dump_ledger()
    assert serial > 0, (serial, epochs)
    eng.close()


@pytest.mark.parametrize("light_max,epoch", [(0, 1024), (1 << 30, 3000)])
def test_drop_in_flags_funded_stream_with_the_domain_splices(kme_mod, oracle_mod, light_max, epoch):
    """The same splices into a funded uniform stream: most epochs are provable and run in parallel, the
    ones holding a spliced record -- or touching symbol 1 / 2 while its book holds the order at 110, at
    125 or of size -5 (C_ODD, k_segments) -- serially; in parallel epochs the makers of account 2^40
    are filled and the ledger pass hands the epoch to the serial replay (an account outside the dense
    range).  Tape, books and ledger equal the oracle's; both paths run."""
    orders = D.funded_domain_stream(oracle_mod)
    o = oracle_mod.Oracle()
    o.process(orders)
    eng = _drop_in_engine(kme_mod, light_max)
    got, serial, epochs = _run(eng, orders, epoch)
    want = o.tape_text()
    assert got == want, _first_diff(got, want)
    assert eng.snapshot_books() == o.dump_books()
    assert eng.snapshot_ledger() == o.dump_ledger()
    assert 0 < serial < epochs, (serial, epochs)
    eng.close()


def test_exact_mode_takes_sparse_symbols_and_accounts(kme_mod, oracle_mod):
    """EXACT mode (one wavefront in arrival order) on the same stream: the sparse symbol's books live
    in the sparse groups (kme_config.max_sparse_symbols, default 4,096)."""
    orders = D.reference_domain_stream(oracle_mod, n=20_000, seed=5)
    o = oracle_mod.Oracle()
    o.process(orders)
    eng = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_EXACT, max_symbols=8, max_epoch=1 << 12,
                                                max_resting=1 << 16, ledger_capacity=1 << 14))
    got, _, _ = _run(eng, orders, 1500)
    assert got == o.tape_text(), _first_diff(got, o.tape_text())
    assert eng.snapshot_books() == o.dump_books()
    assert eng.snapshot_ledger() == o.dump_ledger()
    eng.close()


def test_sparse_symbols_need_the_serial_engine(kme_mod, oracle_mod):
    """Without sparse groups (max_sparse_symbols = KME_SPARSE_NONE) an ADD_SYMBOL past max_symbols is a
    capacity fault at its own record, as before; a BUY on such a symbol is a plain reject."""
    rows = [(W.CREATE_BALANCE, 0, 1, 0, 0, 0), (W.TRANSFER, 0, 1, 0, 0, 100_000), (W.ADD_SYMBOL, 0, 0, 1, 0, 0),
            (W.BUY, 5, 1, 50, 40, 3), (W.ADD_SYMBOL, 0, 0, 50, 0, 0)]
    orders = W.Orders.from_rows(rows)
    eng = _drop_in_engine(kme_mod, sparse=kme_mod.SPARSE_NONE)
    with pytest.raises(kme_mod.KmeError) as ke:
        eng.process(orders)
    assert kme_mod.STATUS[ke.value.status] == "CAPACITY" and ke.value.index == 4
    eng.close()


@pytest.mark.parametrize("sid,detail", [(-(1 << 63), 19), (1 << 55, 19), (-(1 << 56) - 3, 19)])
def test_sid_outside_the_bucket_pointer_range_is_refused(kme_mod, oracle_mod, sid, detail):
    """ADD_SYMBOL of Long.MIN_VALUE or |sid| >= 2^55: (sid << 8) | price (KP:379-381) would alias other
    books' buckets; refused at the record (KME_E_DOMAIN, KME_D_SID_RANGE) rather than answered wrong."""
    rows = [(W.ADD_SYMBOL, 0, 0, 1, 0, 0), (W.ADD_SYMBOL, 0, 0, sid, 0, 0)]
    eng = _drop_in_engine(kme_mod)
    with pytest.raises(kme_mod.KmeError) as ke:
        eng.process(W.Orders.from_rows(rows))
    assert ke.value.status == 3 and ke.value.detail == detail and ke.value.index == 1
    eng.close()


def test_checkpoint_keeps_sparse_symbols_and_odd_books(kme_mod, oracle_mod, tmp_path):
    """A checkpoint taken while the sparse symbol exists and a book holds a level above 100 restores
    into a fresh engine that continues with the uninterrupted run's tape, books and ledger (format 4:
    the sparse groups and their ids; the odd-book count is rebuilt from the groups)."""
    orders = D.reference_domain_stream(oracle_mod, n=24_000, seed=11)
    cut = len(orders) * 3 // 16                                   # after the first splice
    first, second = orders.slice(0, cut), orders.slice(cut, len(orders))
    a = _drop_in_engine(kme_mod)
    _run(a, first, 2048)
    ck = tmp_path / "dom.ckpt"
    a.checkpoint(ck)
    a.close()
    b = _drop_in_engine(kme_mod)
    b.restore(ck)
    got, serial, _ = _run(b, second, 2048)
    o = oracle_mod.Oracle()
    o.process(first)
    o.clear_tape()
    o.process(second)
    assert got == o.tape_text(), _first_diff(got, o.tape_text())
    assert b.snapshot_books() == o.dump_books()
    assert b.snapshot_ledger() == o.dump_ledger()
    assert serial > 0
    b.close()


@pytest.mark.parametrize("light_max", [0, -1, 1 << 30])
def test_restored_engine_cancels_orders_of_the_same_epoch(kme_mod, oracle_mod, tmp_path, light_max):
    """Round-5 verdict (What's weak 2): restore into a fresh engine, then an epoch of BUY/SELLs cancelled
    later in the same epoch -- rested, filled, rejected, cancelled twice -- on light groups (one lane
    each, k_match_lanes reads the order's oid-table entry at the position k_route found) and busy ones
    (k_match), next to cancels of restored orders.  The rebuilt oid table holds only resting orders;
    every entry k_route hands k_match_lanes is this epoch's k_emap insert."""
    n_sym = 24
    setup = W.funded_setup(64, range(1, n_sym + 1))
    pre = W.uniform(6_000, n_symbols=n_sym, n_accounts=64, seed=41)
    a = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=1 << 13,
                                              max_resting=1 << 16, max_accounts=64, ledger_capacity=1 << 14,
                                              light_max=light_max, flags=FLAGS3))
    _run(a, W.Orders.concat([setup, pre]), 2048)
    ck = tmp_path / "same.ckpt"
    a.checkpoint(ck)
    a.close()
    # the epoch after the restore: orders and their cancels, resting ones of the restored book cancelled too
    B, S, C = W.BUY, W.SELL, W.CANCEL
    rows, oid = [], 7_000_000
    rest = [int(x) for x, act in zip(pre.oid[-400:], pre.action[-400:]) if act in (B, S)][:40]
    rest_aid = {int(x): int(a_) for x, a_ in zip(pre.oid, pre.aid)}
    for k in range(300):
        s = 1 + k % n_sym
        acct = k % 64
        rows.append((B if k % 2 else S, oid, acct, s, 40 + (k * 7) % 25, 5 + k % 9))
        if k % 3 == 0:
            rows.append((C, oid, acct, 0, 0, 0))
        if k % 7 == 0:
            rows.append((C, oid, acct, 0, 0, 0))                  # a second cancel: rejected
        if k % 11 == 0 and rest:
            x = rest.pop()
            rows.append((C, x, rest_aid[x], 0, 0, 0))              # an order of the restored book
        oid += 1
    ep = W.Orders.from_rows(rows)
    b = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=1 << 13,
                                              max_resting=1 << 16, max_accounts=64, ledger_capacity=1 << 14,
                                              light_max=light_max, flags=FLAGS3))
    b.restore(ck)
    got = b.process(ep).tape_json(ep)
    o = oracle_mod.Oracle()
    o.process(W.Orders.concat([setup, pre]))
    o.clear_tape()
    o.process(ep)
    assert got == o.tape_text(), _first_diff(got, o.tape_text())
    assert b.snapshot_books() == o.dump_books()
    assert b.snapshot_ledger() == o.dump_ledger()
    b.close()


@pytest.mark.parametrize("light_max", [0, 1 << 30])
def test_an_oid_again_at_the_same_index_of_a_later_epoch(kme_mod, oracle_mod, light_max):
    """An order that filled at once leaves its pending oid-table entry (fingerprint, PENDING | i); the
    same oid again at the same index i of a later epoch (legal: no order with it rests, KP:221) must own
    one entry, the first of its probe sequence -- a cancel later in that epoch finds the order that
    rested (k_match_lanes reads the entry at the position k_route's probe found)."""
    B, S, C = W.BUY, W.SELL, W.CANCEL
    setup = W.funded_setup(8, range(1, 4))
    e1 = W.Orders.from_rows([(S, 100, 1, 1, 55, 10), (B, 101, 2, 2, 30, 1), (B, 102, 2, 2, 30, 1),
                             (B, 103, 2, 2, 30, 1), (B, 104, 2, 2, 30, 1), (B, 777, 3, 1, 60, 10)])   # 777 fills
    e2 = W.Orders.from_rows([(B, 201, 4, 2, 31, 1), (B, 202, 4, 2, 31, 1), (B, 203, 4, 2, 31, 1),
                             (B, 204, 4, 2, 31, 1), (B, 205, 4, 2, 31, 1), (B, 777, 3, 1, 40, 10),     # rests
                             (C, 777, 3, 0, 0, 0)])
    eng = _drop_in_engine(kme_mod, light_max)
    o = oracle_mod.Oracle()
    got = []
    for part in (setup, e1, e2):
        got.append(eng.process(part).tape_json(part))
        o.process(part)
    got = "".join(got)
    assert got == o.tape_text(), _first_diff(got, o.tape_text())
    assert '"action":4,"oid":777' in got.splitlines()[-1]   # the cancel took effect
    assert eng.snapshot_books() == o.dump_books()
    eng.close()


def test_restore_allocation_failure_leaves_the_engine_untouched(kme_mod, oracle_mod, tmp_path, monkeypatch):
    """Round-5 advice: the restore allocates every larger ledger table before it frees any, so a failed
    allocation (KME_TEST_FAIL=restore_alloc) returns KME_E_CAPACITY with the engine as it was -- it
    keeps answering exactly."""
    setup = W.funded_setup(64, range(1, 9))
    pre = W.uniform(4_000, n_symbols=8, n_accounts=64, seed=3)
    a = _drop_in_engine(kme_mod, E=1 << 12, G=9)
    _run(a, W.Orders.concat([setup, pre]), 1024)
    ck = tmp_path / "a.ckpt"
    a.checkpoint(ck)
    b = _drop_in_engine(kme_mod, E=1 << 12, G=9)
    _run(b, setup, 1024)
    before = (b.snapshot_books(), b.snapshot_ledger())
    monkeypatch.setenv("KME_TEST_FAIL", "restore_alloc")
    with pytest.raises(kme_mod.KmeError) as ke:
        b.restore(ck)
    monkeypatch.delenv("KME_TEST_FAIL")
    assert kme_mod.STATUS[ke.value.status] == "CAPACITY"
    assert (b.snapshot_books(), b.snapshot_ledger()) == before
    got, _, _ = _run(b, pre, 1024)
    o = oracle_mod.Oracle()
    o.process(setup)
    o.clear_tape()
    o.process(pre)
    assert got == o.tape_text(), _first_diff(got, o.tape_text())
    a.close()
    b.close()


@pytest.mark.parametrize("light_max", [0, -1, 1 << 30])
def test_lanes_cancel_invariants(kme_mod, oracle_mod, light_max):
    """Round-5 advice (k_match_lanes' held-back stores and freed-but-live nodes): a cancel right after
    its order's rest in the same group (the rest's stores still held back: the cancel's gathers take
    them from flush_rest's registers), a cancel of an order filled earlier in the same epoch (its slot
    on the lane's free stack, its node still live), a cancel of a slot handed out again within the
    epoch, and cancels whose input size is not 0 -- their OUT echo keeps the input's size (removeOrder
    never changes it, KP:289-333) while k_route carried the order's entry position in that word."""
    B, S, C = W.BUY, W.SELL, W.CANCEL
    setup = W.funded_setup(16, range(1, 6))
    e1 = W.Orders.from_rows([(S, 10, 1, 1, 60, 5), (S, 11, 2, 2, 60, 5), (B, 12, 3, 3, 40, 5)])
    e2 = W.Orders.from_rows([
        (B, 20, 4, 4, 45, 9), (C, 20, 4, 0, 0, 13),                       # rest, then its cancel at once
        (B, 21, 5, 1, 61, 5), (C, 10, 1, 0, 0, 7),                        # 10 filled by 21, then cancelled
        (B, 22, 6, 1, 50, 4), (C, 22, 6, 0, 0, 0),                        # a slot 10 freed, cancelled
        (S, 23, 7, 3, 40, 2), (C, 12, 3, 0, 0, 99),                       # partly filled, then cancelled
        (B, 24, 8, 5, 30, 3), (S, 25, 9, 5, 31, 3), (C, 24, 8, 0, 0, 1), (C, 25, 9, 0, 0, -4),
        (B, 26, 10, 2, 59, 1), (C, 11, 2, 0, 0, 5), (C, 26, 10, 0, 0, 0)])
    eng = _drop_in_engine(kme_mod, light_max, G=6)
    o = oracle_mod.Oracle()
    got = []
    for part in (setup, e1, e2):
        got.append(eng.process(part).tape_json(part))
        o.process(part)
    got = "".join(got)
    assert got == o.tape_text(), _first_diff(got, o.tape_text())
    assert eng.snapshot_books() == o.dump_books()
    assert eng.snapshot_ledger() == o.dump_ledger()
    eng.close()
