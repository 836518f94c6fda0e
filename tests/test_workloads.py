"""Properties of the synthetic streams that the parity and bench runs rely on."""
import numpy as np

from kme import workloads as W


def test_exchange_test_shape():
    o = W.exchange_test(20_000, seed=2)
    a = o.action
    # setup: 10 x (CREATE_BALANCE, TRANSFER), then ADD_SYMBOL 0, 1, 2 (exchange_test.js:23-32)
    assert list(a[:20:2]) == [W.CREATE_BALANCE] * 10 and list(a[1:20:2]) == [W.TRANSFER] * 10
    assert list(a[20:23]) == [W.ADD_SYMBOL] * 3 and list(o.sid[20:23]) == [0, 1, 2]
    ev = a[23:]
    frac = {k: float(np.mean(ev == k)) for k in (W.BUY, W.SELL, W.CANCEL)}
    assert abs(frac[W.BUY] - 0.332) < 0.02 and abs(frac[W.SELL] - 0.332) < 0.02
    assert abs(frac[W.CANCEL] - 0.334) < 0.02
    # cancels name an earlier order with its owner's aid, as a JSON string
    first = {}
    for i in range(23, len(o)):
        if a[i] in (W.BUY, W.SELL):
            first.setdefault(int(o.oid[i]), (i, int(o.aid[i])))
        elif a[i] == W.CANCEL and o.oid[i] != 0:
            j, aid = first[int(o.oid[i])]
            assert j < i and aid == o.aid[i] and o.oid_is_string[i]


def test_uniform_stream_properties():
    o = W.uniform(200_000, n_symbols=64, n_accounts=256, seed=4)
    bs = (o.action == W.BUY) | (o.action == W.SELL)
    assert len(np.unique(o.oid[bs])) == bs.sum()                  # unique live oids
    assert o.price[bs].min() >= 30 and o.price[bs].max() <= 75      # H5-safe band
    assert o.size[bs].min() >= 1 and o.size[bs].max() <= 100
    assert o.sid[bs].min() == 1 and o.sid[bs].max() == 64
    pos = {int(x): i for i, x in enumerate(o.oid) if bs[i]}
    can = np.nonzero(o.action == W.CANCEL)[0]
    for i in can[:5000]:
        if o.oid[i] == 0:
            continue
        j = pos[int(o.oid[i])]
        assert j < i and o.aid[j] == o.aid[i]


def test_cancel_replace_pairs_and_sweeps():
    o = W.cancel_replace(50_000, n_symbols=32, n_accounts=64, seed=3)
    c = np.nonzero(o.action == W.CANCEL)[0]
    assert abs(len(c) / len(o) - 0.45) < 0.01
    assert np.all(o.aid[c + 1] == o.aid[c]) and np.all(np.isin(o.action[c + 1], (W.BUY, W.SELL)))
    quote = np.zeros(len(o), bool)
    quote[c + 1] = True
    sweep = np.isin(o.action, (W.BUY, W.SELL)) & ~quote
    assert abs(sweep.mean() - 0.10) < 0.01
    assert np.all(np.where(o.action[sweep] == W.BUY, o.price[sweep] == 75, o.price[sweep] == 30))
    assert o.size[sweep].min() >= 1 and o.size[sweep].max() <= 50_000
    assert o.size[quote].min() >= 1 and o.size[quote].max() <= 100
    assert o.price[quote].min() >= 30 and o.price[quote].max() <= 75


def test_cancel_replace_cancels_hit_live_orders_at_steady_state(oracle_mod):
    """C5's cancels take quotes that still rest (the verdict of round 2: only 9% succeeded when they
    targeted a random earlier oid), and the book stays the same size epoch over epoch."""
    n, n_sym, n_acc, E = 1 << 20, 1024, 4096, 1 << 18
    o = W.cancel_replace(n, n_symbols=n_sym, n_accounts=n_acc, seed=1000)
    orc = oracle_mod.Oracle()
    orc.process(W.funded_setup(n_acc, range(1, n_sym + 1), transfers_per_account=W.funded_transfers_needed(n, n_acc, big=True)))
    orc.clear_tape()
    ok, books = [], []
    for k in range(0, n, E):
        part = o.slice(k, k + E)
        orc.process(part)
        t = orc.tape()
        orc.clear_tape()
        outs = t[t["key"] == 1]
        ok.append(np.count_nonzero(outs["action"] == W.CANCEL) / np.count_nonzero(part.action == W.CANCEL))
        books.append(sum(1 for l in orc.dump_books().splitlines() if l.startswith("O ")))
    assert min(ok[1:]) >= 0.5, ok
    assert max(books[1:]) < 1.1 * min(books[1:]), books


def test_live_cancels_target_resting_orders(oracle_mod):
    """uniform(cancels="live"): each cancel takes its account's most recent resting order."""
    n, n_sym, n_acc = 200_000, 64, 256
    a = W.uniform(n, n_symbols=n_sym, n_accounts=n_acc, seed=5)
    b = W.uniform(n, n_symbols=n_sym, n_accounts=n_acc, seed=5, cancels="live")
    assert np.array_equal(a.action, b.action) and np.array_equal(a.price, b.price)
    rates = []
    for o in (a, b):
        orc = oracle_mod.Oracle()
        orc.process(W.funded_setup(n_acc, range(1, n_sym + 1)))
        orc.clear_tape()
        orc.process(o)
        t = orc.tape()
        outs = t[t["key"] == 1]
        rates.append(np.count_nonzero(outs["action"] == W.CANCEL) / np.count_nonzero(o.action == W.CANCEL))
    assert rates[1] > 0.6 and rates[1] > 3 * rates[0], rates


def test_zipf_is_skewed():
    o = W.zipf(100_000, n_symbols=4096, n_accounts=1024, seed=1)
    s = o.sid[o.action != W.CANCEL]
    counts = np.bincount(s)
    top = np.sort(counts)[::-1]
    assert top[0] > 50 * np.median(counts[counts > 0])


def test_funded_setup_covers_worst_case_reservations():
    n, acc = 1_000_000, 64
    k = W.funded_transfers_needed(n, acc, big=True)
    assert k * W.INT_MAX >= 2 * (n // acc) * 50_000 * 70


def test_binary_tape_helper_matches_oracle(oracle_mod):
    """tests/tapes.engine_tape rebuilds the oracle's tape from per-input results (the GPU scale
    tests compare binary tapes this way): derive the results from an oracle tape and rebuild it."""
    import kme
    import tapes

    setup = W.funded_setup(64, range(1, 33))
    body = W.cancel_replace(4000, n_symbols=32, n_accounts=64, seed=5)
    orders = W.Orders.concat([setup, body])
    o = oracle_mod.Oracle()
    o.process(orders)
    tape = o.tape()
    starts = np.flatnonzero(tape["key"] == 0)
    assert len(starts) == len(orders)
    ends = np.r_[starts[1:], len(tape)] - 1
    ntr = (ends - starts - 1) // 2
    T = np.r_[0, np.cumsum(ntr)].astype(np.uint32)
    fill_rows = np.concatenate([np.arange(s + 1, e, 2) for s, e in zip(starts, ends)]) if ntr.sum() else np.zeros(0, int)
    trades = np.zeros(len(fill_rows), kme.TRADE_DTYPE)
    trades["maker_oid"], trades["maker_aid"], trades["maker_sid"] = tape["oid"][fill_rows], tape["aid"][fill_rows], tape["sid"][fill_rows]
    trades["size"] = tape["size"][fill_rows]
    taker_price = orders.price[np.repeat(np.arange(len(orders)), ntr)]
    trades["maker_price"] = taker_price - tape["price"][fill_rows + 1]
    res = kme.EpochResult(tape["action"][ends].astype(np.int32), tape["size"][ends].astype(np.int32),
                          tape["prev"][ends].astype(np.int64), tape["has_prev"][ends].astype(np.uint8), T, trades, None)
    assert ntr.sum() > 100
    got = tapes.engine_tape(orders, res, oracle_mod.REC_DTYPE)
    assert tapes.first_difference(got, tape) is None


def test_exchange_test_reproduces_the_reference_script():
    """C1's input stream is the reference's own: tools/gen_exchange_test_fixture.py ran
    /root/reference/exchange_test.js under node v12 (kafkajs stubbed by a recording producer,
    Math.random from the seeded stream kme.workloads._JsRandom draws) and committed the MatchIn values
    it sent; the restatement reproduces them record for record (cancel oids as JSON strings, the
    random draw createCancel makes even with no order to cancel, exchange_test.js:97-99)."""
    import gzip
    import os

    path = os.path.join(os.path.dirname(__file__), "golden", "exchange_test_js_n20000_s1.jsonl.gz")
    with gzip.open(path, "rt") as f:
        ref = f.read().split("\n")[:-1]
    got = W.exchange_test(20_000, seed=1).to_json_lines()
    assert len(got) == len(ref) == 20_023
    bad = [i for i, (a, b) in enumerate(zip(got, ref)) if a != b]
    assert not bad, f"record {bad[0]}: {got[bad[0]]} != {ref[bad[0]]}"


def test_exchange_test_reproduces_the_reference_script_live(tmp_path):
    """The same against the script itself, run here when node and the reference are present: all of
    first 40,000 events (of exchange_test.js:33-36's 100,000; the whole run matched too when the fixture
    was made) for another seed."""
    import os
    import shutil
    import subprocess
    import sys

    import pytest

    if not (shutil.which("node") and os.path.exists("/root/reference/exchange_test.js")):
        pytest.skip("node or the reference script absent (the committed fixture pins the stream)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "ex.jsonl.gz"
    subprocess.run([sys.executable, os.path.join(root, "tools", "gen_exchange_test_fixture.py"), "40000", "3", str(out)],
                   check=True, capture_output=True, timeout=600)
    import gzip
    with gzip.open(out, "rt") as f:
        ref = f.read().split("\n")[:-1]
    got = W.exchange_test(40_000, seed=3).to_json_lines()
    assert got == ref
