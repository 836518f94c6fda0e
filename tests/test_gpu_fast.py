"""k_match's fast segments (GroupWave::fast_segment: an aggregate pass over a batch's records, then
one lane per touched price level replaying its records) against the oracle, on the streams that
stress them: a few symbols with deep books (every record of a batch on one or two levels), takes that
end exactly on a maker boundary (H3's zero-size trades, KP:237), cancels of makers at the head of
the level a later record takes from, several cancels of one level in one batch, duplicate cancels,
cancels of orders of the same batch (the serial path), and takes that empty their level (the serial
path).  Every test runs with the fast path on and off (KME_FAST=0) and requires both to be the
oracle's tape and books byte for byte; "two" runs the fast path in k_match's two-wavefront mode
(KME_TWO_MAX: the aggregate pass on one wavefront, the level steps one segment behind on another).""" 
import os

import numpy as np
import pytest

from kme import workloads as W

pytestmark = pytest.mark.gpu


MODES = [True, False, "two"]


def _run(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, fast, epoch=1 << 14, light_max=-1):
    env = {"KME_FAST": "1" if fast else "0", "KME_TWO_MAX": "4096" if fast == "two" else "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        eng = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=epoch,
                                                    max_resting=1 << 20, max_trades=4 * epoch, max_accounts=n_acc,
                                                    light_max=light_max))
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    o = oracle_mod.Oracle()
    for part in [setup] + [stream.slice(a, min(len(stream), a + epoch)) for a in range(0, len(stream), epoch)]:
        got = eng.process(part).tape_json(part)
        o.process(part)
        want = o.tape_text()
        o.clear_tape()
        if got != want:
            la, lb = got.splitlines(), want.splitlines()
            k = next((k for k, (x, y) in enumerate(zip(la, lb)) if x != y), min(len(la), len(lb)))
            pytest.fail(f"fast={fast}: line {k}: got {la[k] if k < len(la) else None!r} want {lb[k] if k < len(lb) else None!r}")
    assert eng.snapshot_books() == o.dump_books()
    eng.close()


@pytest.mark.parametrize("fast", MODES)
@pytest.mark.parametrize("n_sym,seed", [(1, 1), (3, 2), (16, 3)])
def test_deep_books_few_symbols(kme_mod, oracle_mod, fast, n_sym, seed):
    """Uniform flow on 1-16 symbols: thousands of records per group and epoch, most batches one
    long fast segment; cancels hit live orders (the account's most recent resting one)."""
    n_acc = 64
    setup = W.funded_setup(n_acc, range(1, n_sym + 1), transfers_per_account=4)
    stream = W.uniform(120_000, n_symbols=n_sym, n_accounts=n_acc, seed=seed, cancels="live")
    _run(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, fast)


@pytest.mark.parametrize("fast", MODES)
def test_narrow_band_exact_boundaries(kme_mod, oracle_mod, fast):
    """Prices in a 3-tick band and sizes from {1, 2, 3}: takes end exactly on maker boundaries all
    the time (zero-size trades against the next maker of the level, SELL always, BUY when the level
    is its price), and levels empty often (those takes go to the serial path)."""
    n_sym, n_acc, n = 2, 32, 80_000
    rng = np.random.Generator(np.random.PCG64(9))
    o = W.uniform(n, n_symbols=n_sym, n_accounts=n_acc, seed=9, price_lo=49, price_hi=51, cancels="live")
    bs = np.isin(o.action, (W.BUY, W.SELL))
    o.size = np.where(bs, rng.integers(1, 4, n), o.size).astype(np.int32)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    _run(kme_mod, oracle_mod, setup, o, n_sym, n_acc, fast)


@pytest.mark.parametrize("fast", MODES)
def test_cancel_replace_churn_and_sweeps(kme_mod, oracle_mod, fast):
    """C5's shape on 8 symbols: quotes cancelled and replaced at the touch, sweeps across levels (the
    serial path) between fast segments."""
    n_sym, n_acc, n = 8, 256, 200_000
    stream = W.cancel_replace(n, n_symbols=n_sym, n_accounts=n_acc, seed=4)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1), transfers_per_account=W.funded_transfers_needed(n, n_acc, big=True))
    _run(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, fast)


@pytest.mark.parametrize("fast", MODES)
def test_constructed_batch_interactions(kme_mod, oracle_mod, fast):
    """One symbol, hand-made: a deep bid level, then in one batch cancels of its head maker and of a
    maker right behind the head, a SELL taking across the head region, rests appended behind, a
    duplicate cancel, a cancel of an order rested earlier in the same batch, a SELL ending exactly on
    a maker boundary, a BUY at the ask level ending exactly on one."""
    rows = [(W.CREATE_BALANCE, 0, a, 0, 0, 0) for a in range(4)] + \
           [(W.TRANSFER, 0, a, 0, 0, 2_000_000_000) for a in range(4)] + [(W.ADD_SYMBOL, 0, 0, 1, 0, 0)]
    setup = W.Orders.from_rows(rows)
    body = []
    oid = 100
    for k in range(20):                       # bids at 50: sizes 5, 7, 5, 7, ...
        body.append((W.BUY, oid, k % 4, 1, 50, 5 if k % 2 == 0 else 7)); oid += 1
    for k in range(10):                       # asks at 52
        body.append((W.SELL, oid, k % 4, 1, 52, 3)); oid += 1
    # one batch of mixed records
    body += [(W.CANCEL, 100, 0, 0, 0, 0),     # head of the bid level
             (W.CANCEL, 102, 2, 0, 0, 0),     # two behind it
             (W.SELL, 500, 1, 1, 50, 7 + 7),  # takes 101 (7), 103 (7): ends on a boundary -> zero trade with 104
             (W.BUY, 501, 3, 1, 50, 4),       # rests behind
             (W.CANCEL, 102, 2, 0, 0, 0),     # duplicate: rejected
             (W.CANCEL, 501, 3, 0, 0, 0),     # an order of this batch: the serial path
             (W.SELL, 502, 0, 1, 49, 5),      # takes 104 (5) exactly: zero trade with 105
             (W.BUY, 503, 1, 1, 52, 3),       # takes 120 (3) at its own price: zero trade with 121
             (W.BUY, 504, 2, 1, 53, 3),       # takes 121 exactly, next maker at 52 < 53: no zero trade
             (W.CANCEL, 119, 3, 0, 0, 0),     # the tail of the bid level
             (W.BUY, 505, 0, 1, 50, 2)]       # rests at the new tail
    stream = W.Orders.from_rows(body)
    _run(kme_mod, oracle_mod, setup, stream, 1, 4, fast, epoch=1 << 10)


@pytest.mark.parametrize("fast", MODES)
def test_constructed_sweeps_and_same_batch_cancels(kme_mod, oracle_mod, fast):
    """One symbol, hand-made, one batch: sweeps that take whole levels and end exactly on a level's
    end (the zero-size trade is against the NEXT level's head when it still crosses with size 0,
    KP:237 / H3), a sweep over more levels than a segment takes (the serial path), cancels of
    orders rested earlier in the same batch (fast), one of them twice, one of another account, one
    of an order that traded away, and one of an order whose level was taken from since."""
    rows = [(W.CREATE_BALANCE, 0, a, 0, 0, 0) for a in range(4)] + \
           [(W.TRANSFER, 0, a, 0, 0, 2_000_000_000) for a in range(4)] + [(W.ADD_SYMBOL, 0, 0, 1, 0, 0)]
    setup = W.Orders.from_rows(rows)
    body, oid = [], 100
    for p, sizes in ((52, (3,)), (53, (2, 2)), (55, (1, 4)), (56, (2,)), (57, (3,)), (58, (1,)), (60, (5,))):
        for s in sizes:
            body.append((W.SELL, oid, oid % 4, 1, p, s)); oid += 1
    for p, sizes in ((50, (5,)), (49, (2, 6)), (47, (1,)), (46, (2,)), (45, (2,)), (44, (1,)), (43, (9,))):
        for s in sizes:
            body.append((W.BUY, oid, oid % 4, 1, p, s)); oid += 1
    body += [(W.BUY, 900, 0, 1, 53, 3),        # takes 52 whole, ends on its end: zero trade with 53's head
             (W.SELL, 901, 1, 1, 49, 5),       # takes 50 whole: zero trade with 49's head (49 >= 49)
             (W.SELL, 902, 2, 1, 51, 4),       # rests at 51 (ask side)
             (W.BUY, 903, 3, 1, 48, 2),        # rests at 48
             (W.CANCEL, 902, 2, 0, 0, 0),      # an order of this batch: removed
             (W.CANCEL, 902, 2, 0, 0, 0),      # again: rejected
             (W.CANCEL, 903, 1, 0, 0, 0),      # another account's: rejected
             (W.CANCEL, 900, 0, 0, 0, 0),      # traded away: rejected
             (W.BUY, 904, 1, 1, 56, 5),        # 53 (2+2 left) then 55 (1 of 1+4): two levels
             (W.SELL, 905, 0, 1, 47, 8),       # 49 (2 + 6) whole, ends exactly: 47 >= 47 -> zero trade
             (W.SELL, 906, 3, 1, 46, 3),       # 47 (1) whole, 46 (2) whole, exactly: next 45 < 46, none
             (W.BUY, 907, 2, 1, 48, 1),        # rests at 48 behind 903
             (W.SELL, 908, 1, 1, 48, 2),       # takes 903 (2)
             (W.CANCEL, 907, 2, 0, 0, 0),      # its level was taken from since it rested: serial
             (W.BUY, 909, 0, 1, 70, 40),       # sweeps the whole ask side: more levels than a segment
             (W.SELL, 910, 3, 1, 43, 1)]       # after the serial record
    stream = W.Orders.from_rows(body)
    _run(kme_mod, oracle_mod, setup, stream, 1, 4, fast, epoch=1 << 10)


@pytest.mark.parametrize("fast", MODES)
@pytest.mark.parametrize("seed", [5, 6])
def test_sweeps_over_thin_levels(kme_mod, oracle_mod, fast, seed):
    """Thin levels (sizes 1-3) in a 10-tick band on 2 symbols, takers 1-12: most takes sweep several
    levels, many end on a level's end (zero trades against the next level), cancels of live orders
    of the same and earlier batches."""
    n_sym, n_acc, n = 2, 32, 60_000
    rng = np.random.Generator(np.random.PCG64(seed))
    o = W.uniform(n, n_symbols=n_sym, n_accounts=n_acc, seed=seed, price_lo=45, price_hi=55, cancels="live")
    bs = np.isin(o.action, (W.BUY, W.SELL))
    big = rng.random(n) < 0.3
    o.size = np.where(bs, np.where(big, rng.integers(4, 13, n), rng.integers(1, 4, n)), o.size).astype(np.int32)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    _run(kme_mod, oracle_mod, setup, o, n_sym, n_acc, fast)


@pytest.mark.parametrize("list_mode", ["1", "0"])
def test_busy_groups_after_an_all_light_epoch(kme_mod, oracle_mod, list_mode):
    """List mode (k_segments lists the busy groups, k_match_list takes them over a small grid): with
    8,192 symbols an all-light epoch (a few records per group) makes the next one run in list mode;
    that epoch has four hot symbols (~3,000 records each), the one after runs k_match's full grid
    again.  Alternating epochs, tape and books against the oracle (KME_MATCH_LIST=0: the full grid
    throughout)."""
    n_sym, n_acc, E = 8192, 512, 1 << 15
    everyone = np.arange(1, n_sym + 1)
    hot = np.concatenate([everyone, np.repeat(np.array([5, 77, 900, 4000]), 1200)])
    parts = []
    for k in range(5):
        parts.append(W.uniform(E, n_symbols=n_sym, n_accounts=n_acc, seed=40 + k, oid_base=1 + k * E,
                               symbols=hot if k % 2 else everyone))
    stream = W.Orders.concat(parts)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1), transfers_per_account=4)
    old = os.environ.get("KME_MATCH_LIST")
    os.environ["KME_MATCH_LIST"] = list_mode
    try:
        _run(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, True, epoch=E)
    finally:
        if old is None:
            os.environ.pop("KME_MATCH_LIST")
        else:
            os.environ["KME_MATCH_LIST"] = old
