"""Binary MatchOut tapes for parity checks at bench scale.

At 2^22-record epochs the MatchOut text is ~1.3 GB per epoch; the parity tests at that size compare
the same records in binary instead: the engine's per-input results (kme_epoch_result) expanded into
the oracle's tape record format (oracle.REC_DTYPE, one row per forwarded record: "IN" echo, maker
fill and taker fill per trade, "OUT" echo -- KP:97, 272-273, 124), vectorised with numpy.
"""
import numpy as np

BUY, SELL, BOUGHT, SOLD = 2, 3, 5, 6


def engine_tape(orders, res, rec_dtype, n_inputs=None):
    """The oracle-format tape of the first `n_inputs` records of an epoch processed by the engine."""
    n = len(orders) if n_inputs is None else int(n_inputs)
    T = res.trade_off[: n + 1].astype(np.int64)
    ntr = np.diff(T)
    per = 2 + 2 * ntr
    base = np.zeros(n, np.int64)
    if n > 1:
        np.cumsum(per[:-1], out=base[1:])
    total = int(per.sum())
    out = np.zeros(total, rec_dtype)
    act, oid, aid, sid = orders.action[:n], orders.oid[:n], orders.aid[:n], orders.sid[:n]
    price, size = orders.price[:n], orders.size[:n]
    # IN echo: the deserialised input (KP:97)
    out["key"][base] = 0
    out["action"][base], out["oid"][base], out["aid"][base], out["sid"][base] = act, oid, aid, sid
    out["price"][base], out["size"][base] = price, size
    # OUT echo: the mutated order (KP:123-124)
    po = base + 1 + 2 * ntr
    out["key"][po] = 1
    out["action"][po], out["oid"][po], out["aid"][po], out["sid"][po] = res.out_action[:n], oid, aid, sid
    out["price"][po], out["size"][po] = price, res.out_size[:n]
    hp = (res.out_flags[:n] & 1).astype(np.int32)
    out["has_prev"][po] = hp
    out["prev"][po] = np.where(hp != 0, res.out_prev[:n], 0)
    # fills (executeTrade KP:265-274): maker {SOLD|BOUGHT, maker oid/aid/sid, 0, size}, then taker
    # {BOUGHT|SOLD, taker oid/aid/sid, taker.price - maker.price, size}
    nt = int(T[n] - T[0])
    if nt:
        tr = res.trades[T[0]:T[n]]
        inp = np.repeat(np.arange(n, dtype=np.int64), ntr)
        j = np.arange(nt, dtype=np.int64) - (T[inp] - T[0])
        pm = base[inp] + 1 + 2 * j
        buy = act[inp] == BUY
        out["key"][pm] = 1
        out["action"][pm] = np.where(buy, SOLD, BOUGHT)
        out["oid"][pm], out["aid"][pm], out["sid"][pm] = tr["maker_oid"], tr["maker_aid"], tr["maker_sid"]
        out["price"][pm], out["size"][pm] = 0, tr["size"]
        pt = pm + 1
        out["key"][pt] = 1
        out["action"][pt] = np.where(buy, BOUGHT, SOLD)
        out["oid"][pt], out["aid"][pt], out["sid"][pt] = oid[inp], aid[inp], sid[inp]
        out["price"][pt] = (price[inp].astype(np.int64) - tr["maker_price"].astype(np.int64)).astype(np.int32)
        out["size"][pt] = tr["size"]
    return out


def first_difference(got, want):
    """Index of the first differing tape row, or None."""
    m = min(len(got), len(want))
    d = np.flatnonzero(got[:m] != want[:m])
    if len(d):
        return int(d[0])
    return None if len(got) == len(want) else m
