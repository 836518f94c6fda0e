"""exchange_test.js's stream with the records the reference takes but the FUNDED parallel path cannot,
spliced in (round-5 verdict, What's missing 1).

The reference accepts any int price and size and any long aid / sid (KP:451-456): prices 0..126 rest
as real levels (KP:391-404), a negative size is processed wherever the account holds a position
(checkBalance / postRemoveAdjustments only NPE without one, KP:179-180, 332), an account or symbol id
is any long (KP:131-146, 184-191).  The drop-in's defaults (FUNDED + exact ledger + serial fallback,
GpuMatchingEngine()) must answer all of it as the reference does.  Spliced in, at fixed fractions of
the stream:

  * a sparse symbol (sid 10^12, above max_symbols) added, traded on both books and an order cancelled;
  * an account id of 2^40 created, funded, resting and matching on a dense symbol, an order cancelled;
  * BUY/SELL at prices 101..125: a SELL at 110 that rests above every bid (its symbol's book then
    holds a level the parallel matchers do not stage) and is cancelled later, a BUY at 115 that
    crosses the asks, a BUY at 125 that sweeps and rests;
  * negative sizes where the account holds a position on the symbol (the oracle's prefix ledger
    names them): a SELL of size -5 above the bids that rests with a negative size and is cancelled
    later, a BUY of size -3 that trades a negative size.

The oracle (the C restatement of KP:96-445) must take the whole stream without an error: the caller
asserts that before comparing the engine with it.
"""
from __future__ import annotations

import numpy as np

from kme import workloads as W

BIG_SID = 10 ** 12
BIG_AID = 1 << 40
_OID0 = 9 * 10 ** 15          # above the JS harness's oids' usual range, below 2^53: unique


def _positions(oracle_mod, prefix):
    """(aid, sid) keys of the Positions store after `prefix` (KP:426-436), from the oracle."""
    o = oracle_mod.Oracle(keep_tape=False)
    o.process(prefix)
    keys = set()
    for line in o.dump_ledger().splitlines():
        f = line.split()
        if f and f[0] == "P":
            keys.add((int(f[1]), int(f[2])))
    o.close()
    return keys


def reference_domain_stream(oracle_mod, n: int = 40_000, seed: int = 17) -> W.Orders:
    """The splices into exchange_test.js's own stream (10 accounts, symbols 0..2: nearly every epoch
    of it is unprovable anyway -- accounts run out of cash, KP:177)."""
    return splice(oracle_mod, W.exchange_test(n, seed=seed))


def funded_domain_stream(oracle_mod, n: int = 30_000, seed: int = 23) -> W.Orders:
    """The same splices into a funded uniform stream (64 accounts, symbols 1..7): its epochs are
    provable, so the parallel path runs between the ones the splices make serial."""
    base = W.Orders.concat([W.funded_setup(64, range(1, 8)), W.uniform(n, n_symbols=7, n_accounts=64, seed=seed)])
    return splice(oracle_mod, base)


def splice(oracle_mod, base: W.Orders) -> W.Orders:
    N = len(base)
    oid = iter(range(_OID0, _OID0 + 1000))
    o = {k: next(oid) for k in ("s_big", "b_big", "b_acct", "s_acct", "s110", "b115", "b125", "sneg", "bneg", "x1")}
    B, S, C_, A = W.BUY, W.SELL, W.CANCEL, W.ADD_SYMBOL
    cuts = {}
    cuts[N // 8] = [
        (A, 0, 0, BIG_SID, 0, 0),                                   # addSymbol(10^12), KP:184-191
        (W.CREATE_BALANCE, 0, BIG_AID, 0, 0, 0),                    # createBalance(2^40), KP:131-138
        (W.TRANSFER, 0, BIG_AID, 0, 0, 10_000_000),                 # transfer, KP:140-146
        (S, o["s_big"], BIG_AID, BIG_SID, 55, 40),                  # rests on book -10^12
        (B, o["b_big"], 3, BIG_SID, 60, 25),                        # crosses it (account 3)
        (B, o["b_acct"], BIG_AID, 1, 45, 30),                       # the big account on a dense symbol
        (S, o["s_acct"], BIG_AID, -1, 47, 12),                      # (sid -1: the other book of symbol 1, H4)
        (S, o["s110"], 2, 1, 110, 20),                              # rests at 110 (msb bit 47)
    ]
    cuts[N // 4] = [
        (B, o["b115"], 4, 2, 115, 10),                              # crosses the asks of symbol 2
        (B, o["b125"], 5, 2, 125, 300),                             # sweeps, rests at 125 (msb bit 62)
        (C_, o["s_big"], BIG_AID, 0, 0, 0),                         # removeOrder on the sparse symbol
        (B, next(oid), 6, BIG_SID, 54, 5),
    ]
    cuts[(3 * N) // 8] = [
        (C_, o["s110"], 2, 0, 0, 0),                                # the level above 100 goes
        (C_, o["b_acct"], BIG_AID, 0, 0, 0),
        (S, next(oid), 7, 2, 50, 40),                               # into the bid at 125
    ]
    # negative sizes where a position exists (else the reference NPEs, KP:179-180)
    at = N // 2
    pos = _positions(oracle_mod, base.slice(0, at))
    pairs = sorted((a, s) for a, s in pos if 0 <= a < 10 and s in (1, 2))
    assert len(pairs) >= 2, pairs
    (a1, s1), (a2, s2) = pairs[0], pairs[-1]
    cuts[at] = [
        (S, o["sneg"], a1, s1, 99, -5),                             # rests with size -5 above the bids
        (B, o["bneg"], a2, s2, 40, -3),                             # trades a negative size
    ]
    cuts[(5 * N) // 8] = [
        (C_, o["sneg"], a1, 0, 0, 0),                               # postRemoveAdjustments of size -5
        (B, next(oid), BIG_AID, BIG_SID, 70, 10),
        (W.REMOVE_SYMBOL, 0, 0, BIG_SID + 1, 0, 0),                 # an absent sparse symbol: true
    ]
    parts, prev = [], 0
    for k in sorted(cuts):
        parts.append(base.slice(prev, k))
        parts.append(W.Orders.from_rows(cuts[k]))
        prev = k
    parts.append(base.slice(prev, N))
    return W.Orders.concat(parts)
