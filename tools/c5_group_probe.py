"""Diagnostic (GPU box): one symbol group's records of the bench's C5 stream (its BUY/SELL and the
CANCELs that target its orders), cut at the same global epoch boundaries, through a FUNDED engine
with the given light_max; each epoch's tape compared with the oracle."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kafka-matching-engine_amd"), os.path.join(ROOT, "oracle"), ROOT]

import numpy as np  # noqa: E402
import kme  # noqa: E402
import oracle  # noqa: E402
import bench  # noqa: E402


def group_stream(stream, n, g):
    act, oid, sid = stream.action[:n], stream.oid[:n], stream.sid[:n]
    is_ord = (act == 2) | (act == 3)
    mine = is_ord & (np.abs(sid) == g)
    my_oids = set(oid[mine].tolist())
    can = (act == 4) & np.isin(oid, np.fromiter(my_oids, np.int64))
    return np.nonzero(mine | can)[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--group", type=int, default=979)
    ap.add_argument("--records", type=int, default=1572864)
    ap.add_argument("--epoch", type=int, default=262144)
    ap.add_argument("--light-max", type=int, default=-1)
    args = ap.parse_args()
    setup, stream, nsym, nacc, _ = bench.make_workload("c5", 5 << 22, 0, 1)
    idx = group_stream(stream, args.records, args.group)
    eng = kme.Engine(kme.default_config(kme.MODE_FUNDED, max_symbols=nsym + 1, max_epoch=max(len(setup), 1 << 16),
                                        max_resting=1 << 20, max_trades=1 << 20, max_accounts=nacc,
                                        light_max=args.light_max))
    o = oracle.Oracle()
    cuts = np.searchsorted(idx, np.arange(0, args.records + args.epoch, args.epoch))
    parts = [setup] + [stream.take(idx[a:b]) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
    for k, part in enumerate(parts):
        got = eng.process(part).tape_json(part)
        o.process(part)
        want = o.tape_text()
        o.clear_tape()
        if got != want:
            la, lb = got.splitlines(), want.splitlines()
            for j, (x, y) in enumerate(zip(la, lb)):
                if x != y:
                    print("DIFF epoch", k, "line", j, "got", x, "want", y, flush=True)
                    break
            sys.exit(1)
        print("epoch", k, "ok", len(part), flush=True)
    print("books equal:", eng.snapshot_books() == o.dump_books())


if __name__ == "__main__":
    main()
