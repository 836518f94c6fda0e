"""Seeded synthetic order streams (BASELINE.json configs).

All streams are SoA numpy arrays in the reference's `Order` shape (KP:451-456):
action i32, oid i64, aid i64, sid i64, price i32, size i32.

* ``exchange_test`` (C1) restates the load generator of /root/reference/exchange_test.js:18-36 and
  genEvent (exchange_test.js:106-117) with a seeded PRNG (JS Math.random is unseeded).  It is NOT
  funded: balances run dry and acceptance depends on the exact ledger (engine mode EXACT).
* ``uniform`` (C2/C3), ``zipf`` (C4) and ``cancel_replace`` (C5) are funded streams: every account
  receives enough cash that no BUY/SELL can fail the balance check (engine mode FUNDED).
"""
from __future__ import annotations

import functools
import json
import math
from dataclasses import dataclass, field

import numpy as np

ADD_SYMBOL, REMOVE_SYMBOL, BUY, SELL, CANCEL = 0, 1, 2, 3, 4
BOUGHT, SOLD, REJECT = 5, 6, 7
CREATE_BALANCE, TRANSFER, PAYOUT = 100, 101, 200
MAX_SAFE_INTEGER = 2**53 - 1
INT_MAX = 2**31 - 1


@dataclass
class Orders:
    action: np.ndarray
    oid: np.ndarray
    aid: np.ndarray
    sid: np.ndarray
    price: np.ndarray
    size: np.ndarray
    # exchange_test.js sends cancel oids as JSON strings (exchange_test.js:98-101); purely a
    # wire-format detail of the input JSON, the engine sees a long.
    oid_is_string: np.ndarray | None = field(default=None)

    def __len__(self) -> int:
        return int(self.action.shape[0])

    @staticmethod
    def empty(n: int = 0) -> "Orders":
        return Orders(np.zeros(n, np.int32), np.zeros(n, np.int64), np.zeros(n, np.int64),
                      np.zeros(n, np.int64), np.zeros(n, np.int32), np.zeros(n, np.int32),
                      np.zeros(n, bool))

    @staticmethod
    def from_rows(rows) -> "Orders":
        n = len(rows)
        o = Orders.empty(n)
        for i, r in enumerate(rows):
            a, oid, aid, sid, price, size = r[:6]
            o.action[i], o.oid[i], o.aid[i], o.sid[i], o.price[i], o.size[i] = a, oid, aid, sid, price, size
            if len(r) > 6:
                o.oid_is_string[i] = bool(r[6])
        return o

    def slice(self, a: int, b: int) -> "Orders":
        s = None if self.oid_is_string is None else self.oid_is_string[a:b]
        return Orders(self.action[a:b], self.oid[a:b], self.aid[a:b], self.sid[a:b],
                      self.price[a:b], self.size[a:b], s)

    def take(self, idx) -> "Orders":
        s = None if self.oid_is_string is None else self.oid_is_string[idx]
        return Orders(self.action[idx], self.oid[idx], self.aid[idx], self.sid[idx],
                      self.price[idx], self.size[idx], s)

    @staticmethod
    def concat(parts) -> "Orders":
        parts = list(parts)
        cat = lambda k: np.concatenate([getattr(p, k) for p in parts])
        strs = [p.oid_is_string if p.oid_is_string is not None else np.zeros(len(p), bool) for p in parts]
        return Orders(cat("action").astype(np.int32), cat("oid").astype(np.int64),
                      cat("aid").astype(np.int64), cat("sid").astype(np.int64),
                      cat("price").astype(np.int32), cat("size").astype(np.int32),
                      np.concatenate(strs))

    def n_orders(self) -> int:
        """Input order records (BUY/SELL/CANCEL): the unit of the headline metric."""
        a = self.action
        return int(np.count_nonzero((a == BUY) | (a == SELL) | (a == CANCEL)))

    def to_json_lines(self) -> list[str]:
        """JSON.stringify of createOrder (exchange_test.js:63-66): no next/prev fields."""
        out = []
        strs = self.oid_is_string
        for i in range(len(self)):
            oid = int(self.oid[i])
            oid_j = json.dumps(str(oid)) if (strs is not None and strs[i]) else str(oid)
            out.append('{"action":%d,"oid":%s,"aid":%d,"sid":%d,"price":%d,"size":%d}' % (
                int(self.action[i]), oid_j, int(self.aid[i]), int(self.sid[i]),
                int(self.price[i]), int(self.size[i])))
        return out


# ----------------------------------------------------------------------------- C1 (exchange_test.js)
class _JsRandom:
    """Math.random stand-in: seeded doubles in [0, 1)."""

    def __init__(self, seed: int):
        self._g = np.random.Generator(np.random.PCG64(seed))
        self._buf = self._g.random(1 << 16)
        self._i = 0

    def random(self) -> float:
        if self._i == len(self._buf):
            self._buf = self._g.random(1 << 16)
            self._i = 0
        v = float(self._buf[self._i])
        self._i += 1
        return v


def exchange_test(n_events: int = 100_000, seed: int = 1, num_accounts: int = 10,
                  num_symbols: int = 3, rake: int = 3) -> Orders:
    """exchange_test.js:18-36 + genEvent (106-117), argument evaluation order preserved."""
    R = _JsRandom(seed)

    def random_normal():  # exchange_test.js:48-53
        u = 0.0
        v = 0.0
        while u == 0:
            u = R.random()
        while v == 0:
            v = R.random()
        return math.sqrt(-2.0 * math.log(u)) * math.cos(2.0 * math.pi * v)

    def random_uniform(rng):  # :55-57
        return math.floor(R.random() * rng)

    def random_normal_param(mean, std):  # :59-61
        return math.floor(random_normal() * std + mean)

    rows = []
    orders: dict[int, int] = {}  # JS `orders` object: oid -> aid
    live: list[int] = []  # Object.keys(orders) in insertion order (oids >= 2^32 are not array indices)

    def create_order(action, oid, aid, sid, price, size, oid_str=False):
        rows.append((action, oid, aid, sid, price, size, oid_str))

    def create_buy_sell(action):
        aid = random_uniform(num_accounts)
        sid = random_uniform(num_symbols)
        price = random_normal_param(50, 10)
        size = random_normal_param(50, 10)
        oid = math.floor(R.random() * MAX_SAFE_INTEGER)
        if oid not in orders:
            live.append(oid)
        orders[oid] = aid
        create_order(action, oid, aid, sid, price, size)

    for i in range(num_accounts):  # :23-28
        create_order(CREATE_BALANCE, 0, i, 0, 0, 0)
        create_order(TRANSFER, 0, i, 0, 0, random_normal_param(500 * 100, 250 * 100))
    i = 0
    while i < num_symbols / 2 + 1:  # :29-32
        create_order(ADD_SYMBOL, 0, 0, i, 0, 0)
        i += 1
    for _ in range(n_events):  # :33-36 / genEvent :106-117
        e = random_uniform(1000)
        if e == 0:
            create_order(ADD_SYMBOL, 0, 0, random_uniform(num_symbols), 0, 0)
        elif e == 1:
            sid = random_uniform(num_symbols)
            success = random_uniform(2) == 0
            if rake <= 100:  # createPayout (:76-79) sends action 4 (CANCEL), oid 0
                create_order(CANCEL, 0, 0, sid * (1 if success else -1), 0, 100 - rake)
        elif e in (2, 3):
            aid = random_uniform(num_accounts)
            create_order(TRANSFER, 0, aid, 0, 0, random_normal_param(0, 125 * 100))
        elif 3 < e <= 335:
            create_buy_sell(BUY)
        elif 335 < e <= 667:
            create_buy_sell(SELL)
        else:  # createCancel (:97-104): Math.random() is drawn even when there is no order (:99)
            r = R.random()
            if not live:
                create_order(CANCEL, 0, 0, 0, 0, 0)
            else:
                j = math.floor(r * len(live))
                key = live[j]
                create_order(CANCEL, key, orders[key], 0, 0, 0, True)
                del orders[key]
                del live[j]
    return Orders.from_rows(rows)


# ----------------------------------------------------------------------------- funded streams
def _unique_oids(n: int, base: int) -> np.ndarray:
    """n distinct pseudo-random positive oids < 2^53 (odd multiplier: a bijection mod 2^53)."""
    ctr = (np.arange(n, dtype=np.uint64) + np.uint64(base)) & np.uint64(MAX_SAFE_INTEGER)
    x = (ctr * np.uint64(0x5DEECE66D) + np.uint64(0xB)) & np.uint64(MAX_SAFE_INTEGER)
    x = np.where(x == 0, np.uint64(MAX_SAFE_INTEGER), x)
    return x.astype(np.int64)


def funded_setup(n_accounts: int, sids, aid_base: int = 0, transfers_per_account: int = 1) -> Orders:
    """CREATE_BALANCE + TRANSFER(INT_MAX) per account, then ADD_SYMBOL per symbol."""
    A = np.arange(n_accounts, dtype=np.int64) + aid_base
    sids = np.asarray(sids, dtype=np.int64)
    k = transfers_per_account
    n = n_accounts * (1 + k) + len(sids)
    o = Orders.empty(n)
    per = 1 + k
    idx = np.arange(n_accounts) * per
    o.action[idx] = CREATE_BALANCE
    o.aid[idx] = A
    for j in range(k):
        o.action[idx + 1 + j] = TRANSFER
        o.aid[idx + 1 + j] = A
        o.size[idx + 1 + j] = INT_MAX
    s0 = n_accounts * per
    o.action[s0:] = ADD_SYMBOL
    o.sid[s0:] = sids
    return o


def _cancel_targets(action, aid, oid, rng) -> np.ndarray:
    """For each CANCEL row: a uniformly chosen earlier BUY/SELL oid of the same account (0 if none)."""
    n = len(action)
    is_ord = (action == BUY) | (action == SELL)
    is_can = action == CANCEL
    order_by_acct = np.lexsort((np.arange(n), aid))  # stable by index within account
    a_sorted = aid[order_by_acct]
    ord_sorted = is_ord[order_by_acct].astype(np.int64)
    cum = np.cumsum(ord_sorted)
    grp_start = np.searchsorted(a_sorted, a_sorted, side="left")
    cum_before_grp = np.where(grp_start > 0, cum[np.maximum(grp_start - 1, 0)], 0)
    before = cum - ord_sorted - cum_before_grp  # BUY/SELL rows of this account before this row
    ord_rows = order_by_acct[is_ord[order_by_acct]]  # BUY/SELL rows grouped by account, in order
    ord_accts = aid[ord_rows]
    out = np.zeros(n, np.int64)
    can_pos = np.nonzero(is_can[order_by_acct])[0]
    rows = order_by_acct[can_pos]
    cnt = before[can_pos]
    ok = cnt > 0
    k = np.floor(rng.random(len(rows)) * cnt).astype(np.int64)
    base = np.searchsorted(ord_accts, aid[rows], side="left")
    tgt = np.where(ok, ord_rows[np.minimum(base + k, len(ord_rows) - 1)], 0)
    out[rows] = np.where(ok, oid[tgt], 0)
    return out


@functools.lru_cache(maxsize=16)
def _shard_assignment(n_symbols: int, n_shards: int, sid_base: int) -> bytes:
    return np.array([shard_of(s, n_shards) for s in range(sid_base, sid_base + n_symbols)], np.int64).tobytes()


def shard_assignment(n_symbols: int, n_shards: int, sid_base: int = 1) -> np.ndarray:
    """Partition of each sid sid_base .. sid_base + n_symbols - 1 under Kafka's keyed partitioner
    (murmur2 of the decimal |sid|, ``shard_of``)."""
    if n_shards <= 1:
        return np.zeros(n_symbols, np.int64)
    return np.frombuffer(_shard_assignment(n_symbols, n_shards, sid_base), np.int64).copy()


def shard_symbols(n_symbols: int, n_shards: int, shard: int, sid_base: int = 1) -> np.ndarray:
    """The sids of partition ``shard`` of ``n_shards`` (``shard_assignment``), ascending."""
    sids = np.arange(sid_base, sid_base + n_symbols, dtype=np.int64)
    return sids[shard_assignment(n_symbols, n_shards, sid_base) == shard]


def uniform(n_orders: int, n_symbols: int = 1024, n_accounts: int = 4096, seed: int = 1,
            sid_base: int = 1, aid_base: int = 0, oid_base: int = 1, price_lo: int = 30,
            price_hi: int = 75, mix=(0.34, 0.33, 0.33), symbols: np.ndarray | None = None,
            cancels: str = "uniform") -> Orders:
    """C2/C3: 34/33/33 BUY/SELL/CANCEL, sid uniform, price uniform [30,75] (the
    H5-safe band), size floor(N(50,10)) clamped to [1,100], cancels of an earlier oid of the same
    account.  ``symbols``: draw sids uniformly from this set instead of sid_base + [0, n_symbols)
    (a murmur2 shard of a larger universe, ``shard_symbols``); the same draws otherwise.
    ``cancels="live"``: each cancel instead takes its account's most recent order that still rests
    (``live_cancels``), so cancels hit the book the way a trader's do."""
    rng = np.random.Generator(np.random.PCG64(seed))
    u = rng.random(n_orders)
    action = np.where(u < mix[0], BUY, np.where(u < mix[0] + mix[1], SELL, CANCEL)).astype(np.int32)
    aid = rng.integers(0, n_accounts, n_orders).astype(np.int64) + aid_base
    if symbols is None:
        sid = rng.integers(0, n_symbols, n_orders).astype(np.int64) + sid_base
    else:
        symbols = np.asarray(symbols, np.int64)
        sid = symbols[rng.integers(0, len(symbols), n_orders)]
    price = rng.integers(price_lo, price_hi + 1, n_orders).astype(np.int32)
    size = np.clip(np.floor(rng.normal(50, 10, n_orders)), 1, 100).astype(np.int32)
    oid = _unique_oids(n_orders, oid_base)
    is_can = action == CANCEL
    oid = np.where(is_can, _cancel_targets(action, aid, oid, rng), oid)
    sid = np.where(is_can, 0, sid)
    price = np.where(is_can, 0, price).astype(np.int32)
    size = np.where(is_can, 0, size).astype(np.int32)
    o = Orders(action, oid, aid, sid, price, size, np.zeros(n_orders, bool))
    if cancels == "live":
        live_cancels(o, aid_base + n_accounts)
    elif cancels != "uniform":
        raise ValueError(cancels)
    return o


def zipf(n_orders: int, n_symbols: int = 65536, n_accounts: int = 65536, s: float = 1.1,
         seed: int = 1, sid_base: int = 1, aid_base: int = 0, oid_base: int = 1,
         price_lo: int = 40, price_hi: int = 60, shard: tuple[int, int] = (0, 1)) -> Orders:
    """C4: Zipf(s) symbol popularity; a narrow price band keeps hot books deep (~1e4 resting
    orders over <= 21 levels) -- the reference's book has at most 127 levels.
    ``shard`` = (k, n): only the symbols of murmur2 partition k of n, with their popularity in
    the whole universe (the records of partition k of one Zipf stream over ``n_symbols``)."""
    o = uniform(n_orders, n_symbols, n_accounts, seed, sid_base, aid_base, oid_base, price_lo, price_hi,
                mix=(0.36, 0.36, 0.28))
    rng = np.random.Generator(np.random.PCG64(seed + 7919))
    ranks = np.arange(1, n_symbols + 1, dtype=np.float64)
    p = ranks ** (-s)
    p /= p.sum()
    perm = rng.permutation(n_symbols)  # hot symbols spread over the id space
    if shard[1] > 1:
        keep = np.isin(perm + sid_base, shard_symbols(n_symbols, shard[1], shard[0], sid_base))
        p = np.where(keep, p, 0.0)
        p /= p.sum()
    draw = rng.choice(n_symbols, size=n_orders, p=p)
    sid = perm[draw].astype(np.int64) + sid_base
    o.sid = np.where(o.action == CANCEL, 0, sid)
    return o


_GEN = None


def _gen():
    """libkme_workload.so (csrc/kme_workload.c, built with libkme): the book replay that picks cancel
    targets that still rest.  Workload generation only."""
    global _GEN
    if _GEN is None:
        import ctypes as C
        import os

        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libkme_workload.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} not built (make -C kafka-matching-engine_amd/csrc)")
        L = C.CDLL(path)
        P = C.c_void_p
        L.kme_gen_live_cancels.argtypes = [C.c_uint32, P, P, P, P, P, P, C.c_uint32, C.c_uint32]
        L.kme_gen_live_cancels.restype = C.c_int
        L.kme_gen_cancel_replace.argtypes = [C.c_uint32] + [P] * 8 + [C.c_uint32] * 3 + [C.c_double] + [P] * 6
        L.kme_gen_cancel_replace.restype = C.c_int64
        _GEN = L
    return _GEN


def live_cancels(o: Orders, n_accounts: int) -> Orders:
    """Every CANCEL row of `o` re-targeted at its account's most recent order that still rests when
    the cancel arrives (0 when the account has none), by replaying the stream through a plain
    price-time book (kme_workload.c).  In place; returns `o`."""
    import ctypes as C

    L = _gen()
    a = np.ascontiguousarray(o.action, np.int32)
    ai = np.ascontiguousarray(o.aid, np.int64)
    si = np.ascontiguousarray(o.sid, np.int64)
    pr = np.ascontiguousarray(o.price, np.int32)
    sz = np.ascontiguousarray(o.size, np.int32)
    oid = np.array(o.oid, np.int64, copy=True)
    max_sid = int(np.abs(si).max()) if len(si) else 0
    ptr = lambda x: C.c_void_p(x.ctypes.data)
    rc = L.kme_gen_live_cancels(len(o), ptr(a), ptr(ai), ptr(si), ptr(pr), ptr(sz), ptr(oid), n_accounts, max_sid)
    if rc:
        raise RuntimeError("kme_gen_live_cancels failed")
    o.oid = oid
    return o


def cancel_replace(n_orders: int, n_symbols: int = 1024, n_accounts: int = 4096, seed: int = 1,
                   sid_base: int = 1, aid_base: int = 0, oid_base: int = 1, quotes: int = 4,
                   sweep_frac: float = 0.4) -> Orders:
    """C5: 45% (CANCEL, new order of the same account) pairs = 90% of records, and 10%
    large marketable orders (BUY at 75 / SELL at 30) that sweep many levels.

    Cancel/replace as a quoting account does it: every account keeps ``quotes`` quotes and replaces
    them in turn -- the CANCEL takes the quote being replaced (a live order unless a sweep filled
    it), and the new quote goes in at a passive price near the touch (BUY up to 10 ticks under
    min(best ask - 1, mid), SELL likewise over max(best bid + 1, mid); clamped to [30, 75]; size
    floor(N(50, 10)) in [1, 100]), so the books hold ~quotes x accounts / symbols orders.  A
    sweep's size is drawn from 5,000-50,000 and capped at ``sweep_frac`` of the opposite side's
    quantity within its limit, so it clears the best levels without resting a remainder that would
    pin the book.  Flow balance bounds the sweeps: 45% of the records add a quote and 10% sweep, so a
    sweep takes ~(1 - cancel success) x 4.5 quotes on average; the defaults give ~55-60% successful
    cancels (SURVEY §8d C5's churn) and a steady book.  The book replay that places them is
    kme_workload.c (workload generation only)."""
    import ctypes as C

    rng = np.random.Generator(np.random.PCG64(seed))
    n_pairs = int(n_orders * 0.45)
    n_big = max(0, n_orders - 2 * n_pairs)
    n_units = n_pairs + n_big
    kind = rng.permutation(np.r_[np.zeros(n_pairs, np.uint8), np.ones(n_big, np.uint8)])
    acct = rng.integers(0, n_accounts, n_units).astype(np.int64) + aid_base
    sym = rng.integers(0, n_symbols, n_units).astype(np.int64) + sid_base
    is_sell = (rng.random(n_units) >= 0.5).astype(np.uint8)
    u_price = rng.random(n_units)
    qsize = np.clip(np.floor(rng.normal(50, 10, n_units)), 1, 100).astype(np.int32)
    bsize = rng.integers(5000, 50001, n_units).astype(np.int32)
    n = 2 * n_pairs + n_big
    new_oid = _unique_oids(n_units, oid_base)
    cols = Orders.empty(n)
    L = _gen()
    ptr = lambda x: C.c_void_p(x.ctypes.data)
    rows = L.kme_gen_cancel_replace(n_units, ptr(kind), ptr(acct), ptr(sym), ptr(is_sell), ptr(u_price), ptr(qsize),
                                    ptr(bsize), ptr(new_oid), aid_base + n_accounts, sid_base + n_symbols, quotes, sweep_frac,
                                    ptr(cols.action), ptr(cols.aid), ptr(cols.sid), ptr(cols.price), ptr(cols.size),
                                    ptr(cols.oid))
    if rows != n:
        raise RuntimeError(f"kme_gen_cancel_replace: {rows} rows, expected {n}")
    return cols


def funded_transfers_needed(n_orders: int, n_accounts: int, big: bool = False) -> int:
    """TRANSFER(INT_MAX) count per account so that the conservative per-account reservation bound
    (sum of max risks, refunds ignored) never exceeds the funding."""
    per_acct = max(1, n_orders // max(1, n_accounts))
    worst = per_acct * (50_000 * 70 if big else 100 * 100)
    return max(1, int(math.ceil(2 * worst / INT_MAX)))


def murmur2(data: bytes) -> int:
    """Kafka's org.apache.kafka.common.utils.Utils.murmur2 (the default keyed partitioner)."""
    length = len(data)
    seed = 0x9747B28C
    m = 0x5BD1E995
    r = 24
    h = (seed ^ length) & 0xFFFFFFFF
    length4 = length // 4
    for i in range(length4):
        i4 = i * 4
        k = (data[i4] & 0xFF) + ((data[i4 + 1] & 0xFF) << 8) + ((data[i4 + 2] & 0xFF) << 16) + ((data[i4 + 3] & 0xFF) << 24)
        k = (k * m) & 0xFFFFFFFF
        k ^= k >> r
        k = (k * m) & 0xFFFFFFFF
        h = (h * m) & 0xFFFFFFFF
        h ^= k
    rem = length % 4
    if rem == 3:
        h ^= (data[(length & ~3) + 2] & 0xFF) << 16
    if rem >= 2:
        h ^= (data[(length & ~3) + 1] & 0xFF) << 8
    if rem >= 1:
        h ^= data[length & ~3] & 0xFF
        h = (h * m) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * m) & 0xFFFFFFFF
    h ^= h >> 15
    return h


def shard_of(sid: int, n_shards: int) -> int:
    """toPositive(murmur2(utf8(decimal(|sid|)))) % n -- keyed like Kafka's default partitioner."""
    return (murmur2(str(abs(int(sid))).encode()) & 0x7FFFFFFF) % n_shards
