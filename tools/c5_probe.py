"""Diagnostic (GPU box): the bench's C5 stream (1,024 symbols, 4,096 accounts, the bench's funding)
through the host path in epochs of --epoch records, each epoch's tape compared with the oracle;
stops at the first difference and prints it.  Usage: python tools/c5_probe.py --epoch 262144 --records N"""
import argparse
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kafka-matching-engine_amd"), os.path.join(ROOT, "oracle"), ROOT]

import kme  # noqa: E402
import oracle  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epoch", type=int, default=1 << 18)
    ap.add_argument("--records", type=int, default=1 << 22)
    ap.add_argument("--total", type=int, default=5 << 22, help="stream length the generator is asked for")
    ap.add_argument("--workload", default="c5")
    ap.add_argument("--light-max", type=int, default=0)
    args = ap.parse_args()
    setup, stream, nsym, nacc, desc = bench.make_workload(args.workload, args.total, 0, 1)
    E = args.epoch
    eng = kme.Engine(kme.default_config(kme.MODE_FUNDED, max_symbols=nsym + 1, max_epoch=max(E, len(setup)),
                                        max_resting=min(args.total, 1 << 28), max_trades=2 * E + (1 << 16),
                                        max_accounts=nacc, light_max=args.light_max))
    o = oracle.Oracle()
    for part in [setup] + [stream.slice(a, min(args.records, a + E)) for a in range(0, args.records, E)]:
        t = time.time()
        r = eng.process(part)
        got = r.tape_json(part)
        o.process(part)
        want = o.tape_text()
        o.clear_tape()
        if got != want:
            la, lb = got.splitlines(), want.splitlines()
            for k, (x, y) in enumerate(zip(la, lb)):
                if x != y:
                    print("DIFF line", k, "got", x, "want", y, flush=True)
                    oid = re.search(r'"oid":(-?[0-9]+)', x).group(1)
                    gb, ob = eng.snapshot_books(), o.dump_books()
                    print("engine books:", [l for l in gb.splitlines() if oid in l][:4], flush=True)
                    print("oracle books:", [l for l in ob.splitlines() if oid in l][:4], flush=True)
                    if os.environ.get("KME_WATCH"):
                        d = eng.debug_counters()[0]
                        print("watch:", [int(v) for v in d], flush=True)
                    break
            else:
                print("DIFF length", len(la), len(lb), flush=True)
            sys.exit(1)
        print("epoch ok", len(part), "trades", int(r.status.n_trades), f"{time.time() - t:.1f}s", flush=True)
    print("books equal:", eng.snapshot_books() == o.dump_books(), flush=True)


if __name__ == "__main__":
    main()
