#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ with the CPU restatement (oracle/).

The reference has no fixtures of its own and cannot run in this image (no JDK / kafka-streams),
so these vectors pin the restatement (and through it the HIP engine) against regressions:
parity is UNPINNED against a JVM (DESIGN.md "Oracle").  Re-run after any intended change of the
restatement:  python3 tools/gen_golden.py
"""
import gzip
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kafka-matching-engine_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]

import hazards  # noqa: E402
import oracle  # noqa: E402
from kme import workloads as W  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def write_case(name, orders, meta, keep_ledger=True):
    os.makedirs(OUT, exist_ok=True)
    o = oracle.Oracle()
    try:
        o.process(orders)
        meta["error"] = None
    except oracle.OracleError as e:
        meta["error"] = {"code": e.code, "index": e.index}
    with gzip.open(os.path.join(OUT, f"{name}.in.jsonl.gz"), "wt", compresslevel=9) as f:
        f.write("\n".join(orders.to_json_lines()) + "\n")
    with gzip.open(os.path.join(OUT, f"{name}.tape.txt.gz"), "wt", compresslevel=9) as f:
        f.write(o.tape_text())
    with open(os.path.join(OUT, f"{name}.books.txt"), "w") as f:
        f.write(o.dump_books())
    meta["ledger"] = keep_ledger
    if keep_ledger:
        with open(os.path.join(OUT, f"{name}.ledger.txt"), "w") as f:
            f.write(o.dump_ledger())
    meta["records"] = len(orders)
    meta["tape_records"] = int(o.records_forwarded())
    with open(os.path.join(OUT, f"{name}.meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(name, len(orders), "records ->", meta["tape_records"], "tape records", meta["error"] or "")


def main():
    write_case("exchange_test_s1", W.exchange_test(5000, seed=1),
               {"mode": "exact", "generator": "kme.workloads.exchange_test(5000, seed=1)",
                "source": "exchange_test.js:18-36,106-117 restated with a seeded PRNG"})
    setup = W.funded_setup(128, range(1, 17))
    stream = W.uniform(20_000, n_symbols=16, n_accounts=128, seed=3)
    write_case("funded_c2_small", W.Orders.concat([setup, stream]),
               {"mode": "funded", "generator": "funded_setup(128, 1..16) + uniform(20000, 16 sym, 128 acct, seed=3)"})
    stream = W.cancel_replace(8000, n_symbols=8, n_accounts=64, seed=4)
    setup = W.funded_setup(64, range(1, 9), transfers_per_account=W.funded_transfers_needed(8000, 64, big=True))
    write_case("funded_c5_small", W.Orders.concat([setup, stream]),
               {"mode": "funded", "generator": "cancel_replace(8000, 8 sym, 64 acct, seed=4)"})
    for name, rows in sorted(hazards.streams().items()):
        write_case(f"hazard_{name}", hazards.as_orders(rows),
                   {"mode": "funded" if name in hazards.FUNDED_OK else "exact", "generator": f"tests/hazards.py:{name}"})
    for name, (rows, detail) in sorted(hazards.domain_streams().items()):
        write_case(f"domain_{name}", hazards.as_orders(rows),
                   {"mode": "exact", "generator": f"tests/hazards.py:domain {name}", "detail": detail})


if __name__ == "__main__":
    main()
