"""Symbol sharding of one MatchIn stream over N engines.

The reference runs one processor over the MatchIn topic (KP:51-52).  Books of different symbols
never interact, so in FUNDED mode (every order provably passes the balance gate, KP:167-182) the
stream splits by symbol group |sid| without changing any output:

* BUY/SELL/ADD_SYMBOL/REMOVE_SYMBOL/PAYOUT go to ``shard_of(|sid|, n)`` -- Kafka's default keyed
  partitioner (murmur2 of the decimal key), as a producer keyed by symbol would place them;
* CANCEL carries no symbol (exchange_test.js:101) and is broadcast: the shard holding the oid
  answers it, the others reject it without side effects (removeOrder, KP:289-292);
* CREATE_BALANCE/TRANSFER are broadcast: every shard keeps the account; each engine proves its own
  orders against 1/n of the credit (``kme_config.credit_shards``);
* any other action is rejected with no side effect (KP:99-123) and goes to shard 0.

``merge_tapes`` rebuilds the single-engine MatchOut stream from the shards' streams: per input
record, the chunk ``IN ..., fills..., OUT ...`` of the shard that owned it.  The ledger-coupled
EXACT mode does not shard (replicas only).
"""
from __future__ import annotations

import json

import numpy as np

from .workloads import (ADD_SYMBOL, BUY, CANCEL, CREATE_BALANCE, PAYOUT, REMOVE_SYMBOL, SELL,
                        TRANSFER, Orders, shard_of)

BROADCAST = -1


class ShardConflict(RuntimeError):
    """Shards disagree on a broadcast record (e.g. the same oid live on two shards: outside the
    parity domain, KP:221)."""


def route(orders: Orders, n: int) -> np.ndarray:
    """Shard of every record (BROADCAST for cancels and account records)."""
    a = orders.action
    sym = np.isin(a, (BUY, SELL, ADD_SYMBOL, REMOVE_SYMBOL, PAYOUT))
    out = np.zeros(len(orders), np.int64)
    if n > 1 and sym.any():
        s = np.abs(orders.sid[sym])
        uniq, inv = np.unique(s, return_inverse=True)
        out[sym] = np.array([shard_of(int(x), n) for x in uniq], np.int64)[inv]
    out[np.isin(a, (CANCEL, CREATE_BALANCE, TRANSFER))] = BROADCAST
    return out


def split(orders: Orders, n: int):
    """(routes, [indices of shard k], [Orders of shard k]) -- each shard keeps arrival order."""
    r = route(orders, n)
    idx = [np.flatnonzero((r == k) | (r == BROADCAST)) for k in range(n)]
    parts = [Orders(orders.action[i], orders.oid[i], orders.aid[i], orders.sid[i], orders.price[i],
                    orders.size[i], None if orders.oid_is_string is None else orders.oid_is_string[i])
             for i in idx]
    return r, idx, parts


def _chunks(tape: str):
    """Split a MatchOut text into per-input chunks (each starts with its "IN " line)."""
    out, cur = [], []
    for line in tape.splitlines(keepends=True):
        if line.startswith("IN ") and cur:
            out.append("".join(cur))
            cur = []
        cur.append(line)
    if cur:
        out.append("".join(cur))
    return out


def _out_action(chunk: str) -> int:
    last = chunk.rstrip("\n").rsplit("\n", 1)[-1]
    assert last.startswith("OUT "), last
    return int(json.loads(last[4:])["action"])


def merge_tapes(routes: np.ndarray, shard_tapes) -> str:
    """Single-engine MatchOut text from the per-shard texts (shard k processed ``split``'s part k)."""
    chunks = [_chunks(t) for t in shard_tapes]
    ptr = [0] * len(chunks)
    out = []
    for i, s in enumerate(routes.tolist()):
        if s != BROADCAST:
            out.append(chunks[s][ptr[s]])
            ptr[s] += 1
            continue
        mine = [c[p] for c, p in zip(chunks, ptr)]
        for k in range(len(ptr)):
            ptr[k] += 1
        first = _out_action(mine[0])
        if json.loads(mine[0].split("\n", 1)[0][3:])["action"] == CANCEL:
            won = [c for c in mine if _out_action(c) == CANCEL]
            if len(won) > 1:
                raise ShardConflict(f"record {i}: cancel accepted by {len(won)} shards")
            out.append(won[0] if won else mine[0])
        else:
            if any(c != mine[0] for c in mine[1:]):
                raise ShardConflict(f"record {i}: account record answered differently (action {first})")
            out.append(mine[0])
    if any(p != len(c) for p, c in zip(ptr, chunks)):
        raise ShardConflict("shard tapes longer than their routed inputs")
    return "".join(out)


def merge_books(shard_dumps) -> str:
    """Union of the shards' sorted store snapshots, in the single engine's order."""
    lines = [l for d in shard_dumps for l in d.splitlines()]
    return "".join(l + "\n" for l in _sort_dump(lines))


def _sort_dump(lines):
    order = {"B": 0, "K": 1, "O": 2}

    def key(l):
        p = l.split()
        return (order.get(p[0], 3), int(p[1]) if len(p) > 1 and p[1].lstrip("-").isdigit() else 0, l)
    return sorted(lines, key=key)


# ----------------------------------------------------------------------------- partitioned topics
class PartitionRouter:
    """MatchIn / MatchOut partitioned by symbol group (SURVEY.md §8 row f "next-4").

    The reference produces every record to partition 0 of MatchIn (exchange_test.js:14-16,
    topic.js:17-18).  Here each input record is answered by exactly ONE engine, so engine k's output
    is MatchOut partition k as it stands -- no host merge of the N streams:

    * BUY/SELL/ADD_SYMBOL/REMOVE_SYMBOL/PAYOUT -> ``shard_of(|sid|, n)`` (Kafka's keyed partitioner);
    * CANCEL -> the partition that received the last BUY/SELL carrying that oid (a host
      oid -> partition directory); an oid never seen goes to partition 0, which rejects
      it exactly as the reference does (``orders.get(oid) == null``, KP:290);
    * CREATE_BALANCE/TRANSFER -> every partition (each engine proves its orders against 1/n of the
      credit, ``kme_config.credit_shards``), echoed by partition 0 only;
    * any other action -> partition 0.

    Within a partition records keep arrival order; across partitions only per-symbol order is
    defined, as with any keyed Kafka topic.  FUNDED mode only (the EXACT ledger couples symbols).
    """

    def __init__(self, n: int):
        self.n = n
        self.directory: dict[int, int] = {}
        self.seq = 0

    def route(self, orders: Orders):
        """-> (parts, echo, seqs): per partition the Orders it processes, a bool mask of the records
        whose MatchOut chunk belongs in that partition, and their input sequence numbers."""
        sym_route = route(orders, self.n)
        dest = np.zeros(len(orders), np.int64)
        a = orders.action
        for i in range(len(orders)):
            ai = int(a[i])
            if ai in (BUY, SELL):
                dest[i] = sym_route[i]
                self.directory[int(orders.oid[i])] = int(dest[i])
            elif ai == CANCEL:
                dest[i] = self.directory.get(int(orders.oid[i]), 0)
            elif ai in (CREATE_BALANCE, TRANSFER):
                dest[i] = BROADCAST
            elif ai in (ADD_SYMBOL, REMOVE_SYMBOL, PAYOUT):
                dest[i] = sym_route[i]
            else:
                dest[i] = 0
        seq = np.arange(len(orders), dtype=np.int64) + self.seq
        self.seq += len(orders)
        parts, echo, seqs = [], [], []
        for k in range(self.n):
            idx = np.flatnonzero((dest == k) | (dest == BROADCAST))
            parts.append(Orders(orders.action[idx], orders.oid[idx], orders.aid[idx], orders.sid[idx],
                                orders.price[idx], orders.size[idx],
                                None if orders.oid_is_string is None else orders.oid_is_string[idx]))
            echo.append((dest[idx] == k) | ((dest[idx] == BROADCAST) & (k == 0)))
            seqs.append(seq[idx])
        return parts, echo, seqs


def partition_tape(tape: str, echo: np.ndarray) -> str:
    """MatchOut partition text: the engine's tape without the chunks of records it processed only
    for their side effects (account records echoed by partition 0)."""
    chunks = _chunks(tape)
    assert len(chunks) == len(echo), (len(chunks), len(echo))
    return "".join(c for c, e in zip(chunks, echo.tolist()) if e)
