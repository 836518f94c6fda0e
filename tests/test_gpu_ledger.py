"""The exact ledger in parallel (kme_ledger.hip; SURVEY.md §8 row f next-2, KP:167-182, 276-287,
325-333, 434-436): FUNDED matching with KME_FLAG_EXACT_LEDGER, Balances and Positions compared with
the oracle after every epoch, in the three regimes of the parallel pass --

* sparse keys (the C3 shape: many accounts x many symbols): chains independent, no repair;
* value-keyed writes into live chains (hazard H2: a fill's setPosition(UUID, ...) under the old
  position VALUE as key, which is also some account's real (aid, sid) key): the coupled chains are
  re-run in parallel rounds, each with its incoming value writes in arrival order, to a fixed point
  (kme_epoch_status.ledger_repaired > 0), still bit-exact;
* couplings the rounds cannot settle (KME_LEDGER_ROUNDS=1 while a second round is needed; more than
  32 value writes into one chain): the epoch goes to the serial replay (ledger_serial = 1).

Every stream also runs with KME_LEDGER_SERIAL=1 (the serial replay only): same tape, books, ledger.
"""
import numpy as np
import pytest

from kme import workloads as W

pytestmark = pytest.mark.gpu


def _run(kme_mod, oracle_mod, setup, body, n_sym, n_acc, E, flags, serial_env, monkeypatch, check_every=True, rounds=8):
    monkeypatch.setenv("KME_LEDGER_SERIAL", "1" if serial_env else "0")
    monkeypatch.setenv("KME_LEDGER_ROUNDS", str(rounds))
    eng = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=E,
                                                max_resting=1 << 21, max_trades=2 * E + (1 << 12), max_accounts=n_acc,
                                                ledger_capacity=1 << 20, flags=flags))
    o = oracle_mod.Oracle()
    stats = []
    parts = [setup] + [body.slice(a, min(len(body), a + E)) for a in range(0, len(body), E)]
    for k, part in enumerate(parts):
        r = eng.process(part)
        got = r.tape_json(part)
        o.process(part)
        want = o.tape_text()
        o.clear_tape()
        assert got == want, f"epoch {k}: tape"
        if check_every or k == len(parts) - 1:
            assert eng.snapshot_ledger() == o.dump_ledger(), f"epoch {k}: ledger"
        stats.append((int(r.status.ledger_repaired), int(r.status.ledger_serial)))
    assert eng.snapshot_books() == o.dump_books()
    ledger = eng.snapshot_ledger()
    eng.close()
    return stats, ledger


def test_sparse_chains_in_parallel(kme_mod, oracle_mod, monkeypatch):
    """The C3 shape scaled down: 8,192 symbols x 16,384 accounts, 2^17-record epochs."""
    n_sym, n_acc, E = 8192, 16384, 1 << 17
    body = W.uniform(4 * E, n_symbols=n_sym, n_accounts=n_acc, seed=2001)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    stats, led = _run(kme_mod, oracle_mod, setup, body, n_sym, n_acc, E, kme_mod.FLAG_EXACT_LEDGER, False, monkeypatch)
    assert all(s == 0 for _, s in stats[1:]), stats          # the parallel pass took every order epoch
    _, led_serial = _run(kme_mod, oracle_mod, setup, body, n_sym, n_acc, E, kme_mod.FLAG_EXACT_LEDGER, True,
                         monkeypatch, check_every=False)
    assert led == led_serial


def test_value_keyed_writes_into_live_chains_are_replayed(kme_mod, oracle_mod, monkeypatch):
    """64 accounts x 63 symbols with sizes around 50: a position's value (amount, available) ~ (50, 50)
    is also the key of account 50's position on symbol 50, which the epoch reads -- the reference
    clobbers it (KP:284, 434-436).  Short epochs keep each one's couplings to a few dozen chains, which
    the repair replays in arrival order."""
    n_sym, n_acc, E = 63, 64, 256
    body = W.uniform(60 * E, n_symbols=n_sym, n_accounts=n_acc, seed=2002)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    stats, led = _run(kme_mod, oracle_mod, setup, body, n_sym, n_acc, E, kme_mod.FLAG_EXACT_LEDGER, False, monkeypatch)
    repaired = [r for r, s in stats if s == 0 and r > 0]
    assert repaired, stats                                       # couplings replayed by the parallel pass
    _, led_serial = _run(kme_mod, oracle_mod, setup, body, n_sym, n_acc, E, kme_mod.FLAG_EXACT_LEDGER, True,
                         monkeypatch, check_every=False)
    assert led == led_serial


def test_dense_couplings(kme_mod, oracle_mod, monkeypatch):
    """The same universe in 2^15-record epochs: thousands of couplings per epoch, many value writes
    into the same few chains -- whichever pass keeps an epoch (the rounds or the serial replay), the
    ledger is the oracle's."""
    n_sym, n_acc, E = 63, 64, 1 << 15
    body = W.uniform(3 * E, n_symbols=n_sym, n_accounts=n_acc, seed=2003)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    stats, _ = _run(kme_mod, oracle_mod, setup, body, n_sym, n_acc, E, kme_mod.FLAG_EXACT_LEDGER, False, monkeypatch)
    assert all(r > 0 or s for r, s in stats[1:]), stats        # every order epoch coupled


def test_unsettled_couplings_take_the_serial_replay(kme_mod, oracle_mod, monkeypatch):
    """One repair round only: an epoch whose couplings need a second round (a re-run chain's value
    writes changed) goes to the serial replay, and the ledger is still the oracle's."""
    n_sym, n_acc, E = 63, 64, 1 << 12
    body = W.uniform(8 * E, n_symbols=n_sym, n_accounts=n_acc, seed=2006)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    stats, _ = _run(kme_mod, oracle_mod, setup, body, n_sym, n_acc, E, kme_mod.FLAG_EXACT_LEDGER, False, monkeypatch,
                    rounds=1)
    assert any(s for _, s in stats[1:]), stats


def test_c3_shape_ledger_in_parallel(kme_mod, oracle_mod, monkeypatch):
    """The bench's C3 universe (65,536 accounts x 65,536 symbols) in 2^18-record epochs: position
    values (amount, available) of small magnitude are also live (aid, sid) keys; whatever couplings
    arise, the parallel pass keeps every epoch (no serial replay) and the ledger is the oracle's."""
    n_sym, n_acc, E = 65_536, 65_536, 1 << 18
    body = W.uniform(3 * E, n_symbols=n_sym, n_accounts=n_acc, seed=2007)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    stats, _ = _run(kme_mod, oracle_mod, setup, body, n_sym, n_acc, E, kme_mod.FLAG_EXACT_LEDGER, False, monkeypatch,
                    check_every=False)
    assert all(s == 0 for _, s in stats[1:]), stats
    print("c3-shape epochs (chains repaired, serial):", stats[1:])


def test_one_record_with_hundreds_of_fills(kme_mod, oracle_mod, monkeypatch):
    """k_lgen spreads a wavefront's records' ops over its lanes: here one BUY sweeps 300 one-lot makers
    of a few accounts (601 ops of one record, ten rounds of the wavefront's lanes, the other 63
    records' single ops around it), in the middle of a wavefront and again at its last lane, with
    cancels and rejects beside it -- the ledger is the oracle's after each epoch."""
    n_sym, n_acc, E = 7, 16, 1024
    rows, oid = [], 1
    for rep in range(2):
        for k in range(300):                                       # the makers (rest; KP:200-223)
            rows.append((W.SELL, oid, 1 + k % 5, 3, 40 + k % 7, 1)); oid += 1
        rows.append((W.CANCEL, oid - 3, 1 + (297 % 5), 3, 0, 0))   # one of them removed (KP:289-333)
        rows.append((W.BUY, 10_000 + rep, 9, 3, 60, 300))          # the sweep: 1 + 2 x 299 ops
        rows.append((W.CANCEL, 555_555, 9, 3, 0, 0))              # a reject (no such order)
        while len(rows) % 64 != 63:                                  # next: a sweep at a wavefront's last lane
            rows.append((W.BUY, oid, 2, 5, 10, 1)); oid += 1
    for k in range(300):
        rows.append((W.SELL, oid, 3, 6, 45, 1)); oid += 1
    while len(rows) % 64 != 63:
        rows.append((W.SELL, oid, 4, 5, 90, 1)); oid += 1
    rows.append((W.BUY, 20_000, 8, 6, 45, 300))
    body = W.Orders.from_rows(rows)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    stats, led = _run(kme_mod, oracle_mod, setup, body, n_sym, n_acc, E, kme_mod.FLAG_EXACT_LEDGER, False, monkeypatch)
    _, led_serial = _run(kme_mod, oracle_mod, setup, body, n_sym, n_acc, E, kme_mod.FLAG_EXACT_LEDGER, True,
                         monkeypatch, check_every=False)
    assert led == led_serial


@pytest.mark.parametrize("kind", ["uniform", "cancel_replace"])
def test_parallel_ledger_with_cancels_and_fallback_epochs(kme_mod, oracle_mod, monkeypatch, kind):
    """Refunds (postRemoveAdjustments, value writes when a position blocks part of the order) and
    KME_FLAG_SERIAL_FALLBACK epochs mixed with parallel ones: accounts topped up every third epoch, so
    some epochs' proof fails and k_serial applies them (its own ledger), the others take the parallel
    pass; the ledger equals the oracle's after each."""
    n_sym, n_acc, ep = 512, 2048, 1 << 14
    rows = [(W.CREATE_BALANCE, 0, a, 0, 0, 0) for a in range(n_acc)]
    rows += [(W.ADD_SYMBOL, 0, 0, s, 0, 0) for s in range(1, n_sym + 1)]
    setup = W.Orders.from_rows(rows)
    stream = (W.uniform(9 * ep, n_symbols=n_sym, n_accounts=n_acc, seed=2004) if kind == "uniform"
              else W.cancel_replace(9 * ep, n_symbols=n_sym, n_accounts=n_acc, seed=2005))
    topup = W.Orders.from_rows([(W.TRANSFER, 0, a, 0, 0, 120_000 if kind == "uniform" else 2_000_000_000)
                                for a in range(n_acc)])
    chunks = [setup]
    for c in range(0, len(stream), 3 * ep):
        chunks.append(topup)
        chunks += [stream.slice(c + k, c + k + ep) for k in range(0, 3 * ep, ep)]
    monkeypatch.setenv("KME_LEDGER_SERIAL", "0")
    eng = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=ep,
                                                max_resting=1 << 20, max_trades=4 * ep, max_accounts=n_acc,
                                                ledger_capacity=1 << 18,
                                                flags=kme_mod.FLAG_EXACT_LEDGER | kme_mod.FLAG_SERIAL_FALLBACK))
    o = oracle_mod.Oracle()
    for ch in chunks:
        r = eng.process(ch)
        got = r.tape_json(ch)
        o.process(ch)
        assert got == o.tape_text()
        o.clear_tape()
        assert eng.snapshot_ledger() == o.dump_ledger()
    assert eng.snapshot_books() == o.dump_books()
    eng.close()


def test_ledger_tables_grow_online_at_the_c3_accounts(kme_mod, oracle_mod, monkeypatch, tmp_path):
    """Round-4 verdict: the drop-in's tables must survive a long stream.  C3's 65,536 accounts over
    1,024 symbols (so that the books trade from the first epochs; at 65,536 symbols a test-sized
    stream leaves them nearly empty) -- most fills open a new (aid, sid) position (KP:280) and H2 never
    removes the entry it reads (KP:283) -- from a tiny ledger_capacity: the engine rehashes Balances /
    Positions into larger tables between epochs (kme_ledger_stats) before the next epochs could
    overflow them, and the ledger equals the oracle's after every epoch; Positions grows at least three
    times.  A checkpoint of the grown tables restores into a fresh engine of the initial size, which
    grows to take it and goes on exactly."""
    monkeypatch.setenv("KME_LEDGER_SERIAL", "0")
    n_sym, n_acc, E = 1024, 65_536, 1 << 12
    n_ep = 80
    body = W.uniform(n_ep * E, n_symbols=n_sym, n_accounts=n_acc, seed=2008)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    cfg = kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=E, max_resting=1 << 20,
                                 max_trades=3000, max_accounts=n_acc, ledger_capacity=1024,
                                 flags=kme_mod.FLAG_EXACT_LEDGER | kme_mod.FLAG_SERIAL_FALLBACK)
    # (setup: 65,536 CREATE_BALANCE + TRANSFER + ADD_SYMBOL records in max_epoch-record host epochs)
    eng = kme_mod.Engine(cfg)
    first = eng.ledger_stats()
    o = oracle_mod.Oracle()
    r = eng.process(setup)
    o.process(setup)
    assert r.tape_json(setup) == o.tape_text()
    o.clear_tape()
    ck, ck_at, sizes = tmp_path / "grown.ckpt", 3 * n_ep // 4, []
    for k in range(n_ep):
        part = body.slice(k * E, (k + 1) * E)
        r = eng.process(part)
        o.process(part)
        assert r.tape_json(part) == o.tape_text(), f"epoch {k}: tape"
        o.clear_tape()
        assert eng.snapshot_ledger() == o.dump_ledger(), f"epoch {k}: ledger"
        st = eng.ledger_stats()
        sizes.append((st["pos_slots"], st["pos_used"], st["grows"]))
        assert 2 * st["pos_used"] <= st["pos_slots"] and 2 * st["bal_used"] <= st["bal_slots"]
        if k == ck_at:
            eng.checkpoint(ck)
            at_ck = eng.ledger_stats()
    last = eng.ledger_stats()
    assert last["pos_slots"] >= 8 * first["pos_slots"], (first, sizes)      # three growths of Positions or more
    assert len({p for p, _, _ in sizes}) >= 3 and last["grows"] >= 3
    assert eng.snapshot_books() == o.dump_books()
    want_books, want_ledger = eng.snapshot_books(), eng.snapshot_ledger()
    eng.close()
    # restore the grown state into an engine of the initial size, replay the epochs after it
    b = kme_mod.Engine(cfg)
    assert b.ledger_stats()["pos_slots"] == first["pos_slots"] < at_ck["pos_used"] * 2
    b.restore(ck)
    assert b.ledger_stats()["pos_used"] <= at_ck["pos_used"]   # live entries only (tombstones dropped)
    for k in range(ck_at + 1, n_ep):
        b.process(body.slice(k * E, (k + 1) * E))
    assert b.snapshot_ledger() == want_ledger
    assert b.snapshot_books() == want_books
    b.close()


def test_drop_in_shape_accounts_far_outnumber_ops(kme_mod, oracle_mod, monkeypatch):
    """The drop-in's shape: 2^20 accounts, 65,536-record epochs.  The stream's 2,048 accounts are
    spread 300 ids apart (every gap between two accounts with ops is longer than k_lseg's 256, so
    each goes to the gap list k_lseg_gaps fills, and so does the ~400K-id tail after the last one),
    and with fewer ops than accounts the sort key takes 7 sid-hash bits for three radix passes
    instead of four.  Tape, books and ledger against the oracle after every epoch."""
    n_sym, n_used, E, stride = 1024, 2048, 1 << 16, 300
    body = W.uniform(4 * E, n_symbols=n_sym, n_accounts=n_used, seed=2401)
    setup = W.funded_setup(n_used, range(1, n_sym + 1))
    body.aid[:] = body.aid * stride
    setup.aid[:] = setup.aid * stride
    stats, _ = _run(kme_mod, oracle_mod, setup, body, n_sym, 1 << 20, E, kme_mod.FLAG_EXACT_LEDGER, False, monkeypatch)
    assert all(s == 0 for _, s in stats[1:]), stats
