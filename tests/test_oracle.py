"""CPU tests of the oracle (oracle/kme_oracle.c): the bit-scan restatement, hand-derived known
answers read off KProcessor.java, and the committed golden vectors.

The reference has no tests or fixtures of its own, so the known answers below are
derived by hand from the Java source, line by line, and the golden vectors pin the restatement
against regressions (parity unpinned against a JVM; see DESIGN.md "Oracle").
"""
import json
import os
import sys

import pytest

from kme import workloads as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "tools"))


def J(action, oid, aid, sid, price, size, nxt=None, prev=None):
    n = "null" if nxt is None else str(nxt)
    p = "null" if prev is None else str(prev)
    return ('{"action":%d,"oid":%d,"aid":%d,"sid":%d,"price":%d,"size":%d,"next":%s,"prev":%s}'
            % (action, oid, aid, sid, price, size, n, p))


def run(oracle_mod, rows):
    o = oracle_mod.Oracle()
    o.process(W.Orders.from_rows(rows))
    return o


def setup_rows(accounts=(1, 2, 3), sids=(1,), fund=10**9):
    rows = []
    for a in accounts:
        rows += [(100, 0, a, 0, 0, 0), (101, 0, a, 0, 0, fund)]
    rows += [(0, 0, 0, s, 0, 0) for s in sids]
    return rows


def tail_lines(o, n_setup_records):
    return o.tape_text().splitlines()[2 * n_setup_records:]


# ------------------------------------------------------------------ H5: the log10 bit scans
def test_first_set_bit_is_ctz_and_nan_path(oracle_mod):
    for k in range(63):
        assert oracle_mod.first_set_bit_pos(1 << k) == k
        assert oracle_mod.first_set_bit_pos((1 << k) | (1 << 62)) == k
    assert oracle_mod.first_set_bit_pos(-(1 << 63)) == 0          # log10(negative) = NaN -> 0


def test_last_set_bit_thresholds_match_correctly_rounded_log10(oracle_mod):
    import gen_log10_table as T

    D = T.thresholds(T.quotient_cr)
    assert sorted(D) == list(range(47, 63))
    for h in range(63):
        assert oracle_mod.last_set_bit_pos(1 << h) == h
        top = (1 << (h + 1)) - 1
        if h in D:
            t = (1 << (h + 1)) - D[h]
            assert oracle_mod.last_set_bit_pos(t - 1) == h
            assert oracle_mod.last_set_bit_pos(t) == h + 1
            assert oracle_mod.last_set_bit_pos(top) == h + 1
        else:
            assert oracle_mod.last_set_bit_pos(top) == h
    assert oracle_mod.last_set_bit_pos(-1) == 0                   # negative -> NaN -> 0
    # spot checks of the restatement against the Python model of the Java expression
    import random

    rng = random.Random(5)
    for _ in range(2000):
        h = rng.randrange(0, 63)
        n = (1 << h) | rng.getrandbits(h) if h else 1
        assert oracle_mod.last_set_bit_pos(n) == T.quotient_cr(n)


# ------------------------------------------------------------------ hand-derived known answers
def test_known_answer_zero_size_trade_after_exact_fill(oracle_mod):
    """KP:237 parses as (size>0 && isBuy) ? maker.price<=P : maker.price>=P.  A BUY that exactly
    exhausts maker 11 sees size 0, switches to maker.price >= 50, which maker 12 (also at 50)
    satisfies: a size-0 trade pair is forwarded, maker 12 is not consumed (size != 0 -> break)."""
    S = setup_rows()
    o = run(oracle_mod, S + [(3, 11, 1, 1, 50, 10), (3, 12, 2, 1, 50, 5), (2, 13, 3, 1, 50, 10)])
    lines = tail_lines(o, len(S))
    want = [
        "IN " + J(3, 11, 1, 1, 50, 10), "OUT " + J(3, 11, 1, 1, 50, 10),
        "IN " + J(3, 12, 2, 1, 50, 5), "OUT " + J(3, 12, 2, 1, 50, 5, prev=11),
        "IN " + J(2, 13, 3, 1, 50, 10),
        "OUT " + J(6, 11, 1, 1, 0, 10), "OUT " + J(5, 13, 3, 1, 0, 10),      # maker fill, taker fill
        "OUT " + J(6, 12, 2, 1, 0, 0), "OUT " + J(5, 13, 3, 1, 0, 0),        # the size-0 trade
        "OUT " + J(2, 13, 3, 1, 50, 0),
    ]
    assert lines == want
    books = o.dump_books().splitlines()
    assert "O 12 3 2 1 50 5 null null" in books                          # new head, prev cleared
    assert "K %d 12 12" % ((-1 << 8) | 50) in books


def test_known_answer_sell_always_tests_price_ge(oracle_mod):
    """For a SELL taker the loop condition is maker.price >= P regardless of size (H3): after an
    exact fill at 60 the next bid level 55 >= 50 yields a size-0 trade."""
    S = setup_rows()
    o = run(oracle_mod, S + [(2, 21, 1, 1, 60, 7), (2, 22, 2, 1, 55, 9), (3, 23, 3, 1, 50, 7)])
    lines = tail_lines(o, len(S))
    assert lines[4:] == [
        "IN " + J(3, 23, 3, 1, 50, 7),
        "OUT " + J(5, 21, 1, 1, 0, 7), "OUT " + J(6, 23, 3, 1, -10, 7),    # taker price - maker price
        "OUT " + J(5, 22, 2, 1, 0, 0), "OUT " + J(6, 23, 3, 1, -5, 0),
        "OUT " + J(3, 23, 3, 1, 50, 0),
    ]


def test_known_answer_sid0_single_book(oracle_mod):
    """addSymbol(0) puts books[0] twice (-0 == 0): BUY and SELL share one book, and a BUY taker
    matches the minimum price present, even a resting BUY (maker fill labelled SOLD)."""
    S = setup_rows(sids=(0,))
    o = run(oracle_mod, S + [(2, 51, 1, 0, 40, 5), (2, 53, 2, 0, 45, 3)])
    lines = tail_lines(o, len(S))
    assert lines[2:] == [
        "IN " + J(2, 53, 2, 0, 45, 3),
        "OUT " + J(6, 51, 1, 0, 0, 3), "OUT " + J(5, 53, 2, 0, 5, 3),
        "OUT " + J(2, 53, 2, 0, 45, 0),
    ]
    assert [l for l in o.dump_books().splitlines() if l.startswith("B ")] == ["B 0 0 %d" % (1 << 40)]


def test_known_answer_balance_gate_and_refunds(oracle_mod):
    """checkBalance (KP:167-182): BUY risk = size*price; reject when balance < risk; a cancel
    refunds (size+adj)*price (KP:325-333); the taker's price improvement is refunded (KP:286)."""
    S = [(100, 0, 1, 0, 0, 0), (101, 0, 1, 0, 0, 1000), (100, 0, 2, 0, 0, 0), (101, 0, 2, 0, 0, 1000),
         (0, 0, 0, 1, 0, 0)]
    o = run(oracle_mod, S + [(2, 1, 1, 1, 50, 10), (2, 2, 1, 1, 50, 11), (4, 1, 1, 0, 0, 0),
                             (2, 3, 1, 1, 50, 11), (3, 4, 2, 1, 40, 11)])
    outs = [l for l in tail_lines(o, len(S)) if l.startswith("OUT")]
    assert outs[0] == "OUT " + J(2, 1, 1, 1, 50, 10)
    assert outs[1] == "OUT " + J(7, 2, 1, 1, 50, 11)          # 500 left < 550
    assert outs[2] == "OUT " + J(4, 1, 1, 0, 0, 0)            # cancel accepted: +500
    assert outs[3] == "OUT " + J(2, 3, 1, 1, 50, 11)          # 1000 >= 550
    ledger = o.dump_ledger().splitlines()
    # account 1: 1000 - 500 + 500 - 550 = 450; the SELL taker of account 2 fills at 50:
    # risk (-11)*(40-100) = 660 -> 340; refund -11 * (40-50) = +110 -> 450
    assert "A 1 450" in ledger and "A 2 450" in ledger
    assert "P 1 1 11 11" in ledger and "P 2 1 -11 -11" in ledger


def test_known_answer_positions_written_under_value_key(oracle_mod):
    """fillOrder's second fill writes positions[oldValue] (KP:284, 434-436), not the real key."""
    S = setup_rows(accounts=(7, 8))
    o = run(oracle_mod, S + [(3, 1, 8, 1, 50, 2), (2, 2, 7, 1, 50, 2), (3, 3, 8, 1, 50, 3), (2, 4, 7, 1, 50, 3)])
    ledger = o.dump_ledger().splitlines()
    assert "P 7 1 2 2" in ledger                 # real key frozen at the first fill
    assert "P 2 2 5 5" in ledger                 # second fill landed under key (2, 2)
    assert "P -2 -2 -5 -5" in ledger


def test_known_answer_remove_symbol_and_unknown_action(oracle_mod):
    S = setup_rows()
    o = run(oracle_mod, S + [(1, 0, 0, 9, 0, 0), (1, 0, 0, 1, 0, 0), (42, 5, 1, 1, 1, 1)])
    outs = [l for l in tail_lines(o, len(S)) if l.startswith("OUT")]
    assert outs == ["OUT " + J(1, 0, 0, 9, 0, 0), "OUT " + J(7, 0, 0, 1, 0, 0), "OUT " + J(7, 5, 1, 1, 1, 1)]


def test_domain_error_on_log10_overshoot(oracle_mod):
    rows = setup_rows() + [(2, 1000 + p, 1, 1, p, 1) for p in range(48)] + [(3, 2000, 2, 1, 0, 1)]
    with pytest.raises(oracle_mod.OracleError) as e:
        run(oracle_mod, rows)
    assert e.value.code == 2 and e.value.index == len(rows) - 1
    # 47 contiguous levels (0..46): no overshoot, the SELL sweeps normally
    ok = setup_rows() + [(2, 1000 + p, 1, 1, p, 1) for p in range(47)] + [(3, 2000, 2, 1, 0, 100)]
    run(oracle_mod, ok)


# ------------------------------------------------------------------ golden vectors
import golden_io  # noqa: E402


@pytest.mark.parametrize("case", golden_io.cases())
def test_oracle_reproduces_golden(oracle_mod, case):
    orders, meta = golden_io.load_inputs(case)
    o = oracle_mod.Oracle()
    if meta["error"]:
        with pytest.raises(oracle_mod.OracleError) as e:
            o.process(orders)
        assert (e.value.code, e.value.index) == (meta["error"]["code"], meta["error"]["index"])
    else:
        o.process(orders)
    assert o.tape_text() == golden_io.load_text(case, "tape")
    assert o.dump_books() == golden_io.load_text(case, "books")
    if meta.get("ledger", False):
        assert o.dump_ledger() == golden_io.load_text(case, "ledger")


def test_golden_fixtures_present():
    cases = golden_io.cases()
    assert {"exchange_test_s1", "funded_c2_small", "funded_c5_small", "hazard_zero_trade_same_level",
            "domain_log10_overshoot"} <= set(cases)
    assert len(cases) >= 20


def test_golden_inputs_are_the_wire_format():
    """The C1 fixture carries cancel oids as JSON strings, as exchange_test.js:98-101 sends them."""
    lines = golden_io.load_json_lines("exchange_test_s1")
    cancels = [json.loads(l) for l in lines if json.loads(l)["action"] == 4]
    assert any(isinstance(c["oid"], str) for c in cancels)
