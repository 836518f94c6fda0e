#!/usr/bin/env python3
"""How often the FUNDED proof fails when an account's credit is split over N symbol shards
(kme_config.credit_shards, kme_kernels.hip k_ledger_funded).

One global stream (C3: uniform over 65,536 symbols; C4: Zipf(1.1)) is keyed over N shards by
murmur2 (Kafka's partitioner, ``kme.workloads.shard_assignment``).  Every account holds a credit of
``f`` times the single-engine need of the whole stream (the sum over its BUY/SELL of the max risk
``size * price`` / ``size * (100 - price)``, KP:172-176 -- what one engine's proof books), and each
shard proves its records against ``floor(credit / N)``.  The bound only falls (refunds are not
credited back inside the funded proof), so shard s of account a fails from the first epoch in which
its cumulative need passes its share; an epoch with any failing (account, shard) pair of the epoch
falls back to the serial engine (KME_FLAG_SERIAL_FALLBACK) or is refused (KME_E_UNFUNDED).

Pure numpy on the workload generator (no GPU): prints one JSON line per (workload, N, f).

    python tools/credit_split_probe.py [--records 16777216] [--epoch 4194304]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kafka-matching-engine_amd"))

from kme import workloads as W  # noqa: E402

BUY, SELL = 2, 3


def max_risk(action: np.ndarray, price: np.ndarray, size: np.ndarray) -> np.ndarray:
    """checkBalance's largest possible reservation per BUY/SELL (0 for other records)."""
    r = np.where(action == BUY, size.astype(np.int64) * price,
                 np.where(action == SELL, size.astype(np.int64) * (100 - price.astype(np.int64)), 0))
    return r.astype(np.int64)


def fallback_stats(aid: np.ndarray, shard: np.ndarray, risk: np.ndarray, pos: np.ndarray, n_records: int,
                   n_accounts: int, n_shards: int, factor: float, epoch_records: int) -> dict:
    """Epochs (of ``epoch_records`` global records) in which some (account, shard) pair of the epoch
    is past its share of the credit, and the first such epoch (``pos``: each BUY/SELL's index in the
    global stream of ``n_records``)."""
    n = len(aid)
    total = np.bincount(aid, weights=risk, minlength=n_accounts).astype(np.int64)
    credit = np.floor(total * factor).astype(np.int64)
    share = credit // n_shards
    key = aid.astype(np.int64) * n_shards + shard
    order = np.argsort(key, kind="stable")
    k_sorted = key[order]
    cum = np.cumsum(risk[order])
    start = np.searchsorted(k_sorted, k_sorted, side="left")
    before = np.where(start > 0, cum[np.maximum(start - 1, 0)], 0)
    cum_pair = np.empty(n, np.int64)
    cum_pair[order] = cum - before          # cumulative need of (account, shard) through record i
    failing = (risk > 0) & (cum_pair > share[aid])
    n_ep = (n_records + epoch_records - 1) // epoch_records
    ep_fail = np.zeros(n_ep, bool)
    ep_fail[np.unique(pos[failing] // epoch_records)] = True
    first = int(np.argmax(ep_fail)) if ep_fail.any() else -1
    pairs = np.unique(key[failing]).size
    return {"epochs": int(n_ep), "fallback_epochs": int(ep_fail.sum()), "fallback_frac": float(ep_fail.mean()),
            "first_fallback_epoch": first, "failing_pairs": int(pairs),
            "failing_accounts": int(np.unique(aid[failing]).size)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 24, help="global stream length")
    ap.add_argument("--epoch", type=int, default=1 << 22, help="records per GPU per epoch (bench E)")
    ap.add_argument("--factors", default="1.0,1.1,1.25,1.5,2.0")
    ap.add_argument("--shards", default="1,2,4,8")
    ap.add_argument("--workloads", default="c3,c4")
    args = ap.parse_args()
    for wl in args.workloads.split(","):
        if wl == "c3":
            o = W.uniform(args.records, n_symbols=65536, n_accounts=65536, seed=1000)
        else:
            o = W.zipf(args.records, n_symbols=65536, n_accounts=65536, seed=1000)
        risk = max_risk(o.action, o.price, o.size)
        pos = np.nonzero(risk > 0)[0]
        aid, sid, risk = o.aid[pos], o.sid[pos], risk[pos]
        for ns in (int(x) for x in args.shards.split(",")):
            sh = W.shard_assignment(65536, ns)[np.abs(sid) - 1] if ns > 1 else np.zeros(len(sid), np.int64)
            for f in (float(x) for x in args.factors.split(",")):
                st = fallback_stats(aid, sh, risk, pos, args.records, 65536, ns, f, args.epoch * ns)
                print(json.dumps({"workload": wl, "n_shards": ns, "credit_factor": f, "records": args.records, **st}),
                      flush=True)


if __name__ == "__main__":
    main()
