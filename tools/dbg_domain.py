"""Diagnostic (GPU): the funded domain stream through a drop-in-flags engine, epoch by epoch; on a
fault prints the epoch, the faulting record and its neighbours, and the serial / parallel path of the
epochs before it."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("kafka-matching-engine_amd", "tests", "oracle", ""):
    sys.path.insert(0, os.path.join(ROOT, p))
import oracle  # noqa: E402
import domain_stream as D  # noqa: E402
import kme  # noqa: E402

epoch = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
light = int(sys.argv[2]) if len(sys.argv) > 2 else 0
orders = D.funded_domain_stream(oracle)
eng = kme.Engine(kme.default_config(kme.MODE_FUNDED, max_symbols=8, max_epoch=4096, max_resting=1 << 16, max_accounts=64,
                                    ledger_capacity=1 << 14, light_max=light, flags=3))
o = oracle.Oracle()
for k, a in enumerate(range(0, len(orders), epoch)):
    part = orders.slice(a, min(len(orders), a + epoch))
    try:
        r = eng.process(part)
    except kme.KmeError as e:
        i = e.index
        print("epoch", k, "start", a, "fault", e, "index", i)
        for j in range(max(0, i - 6), min(len(part), i + 3)):
            print("  ", j, a + j, int(part.action[j]), int(part.oid[j]), int(part.aid[j]), int(part.sid[j]), int(part.price[j]), int(part.size[j]))
        st = e.args[2] if len(e.args) > 2 else None
        res = getattr(e, "result", None)
        print("n_effective", getattr(e, "n_effective", None), "status", {k: getattr(res.status, k) for k, _ in res.status._fields_} if res is not None else None)
        if res is not None:
            tr = res.trades
            print("trades", len(tr), "maker aids outside [0,64):", [(int(t["maker_oid"]), int(t["maker_aid"]), int(t["maker_sid"])) for t in tr if not (0 <= t["maker_aid"] < 64)][:10])
            bad = [q for q in range(len(res.trade_off) - 1) if res.trade_off[q + 1] > res.trade_off[q]]
            print("records with trades", len(bad))
        o2 = oracle.Oracle()
        o2.process(orders.slice(0, a))
        o2.clear_tape()
        o2.process(part.slice(0, i + 1))
        t = o2.tape()
        print("oracle: last records' fills", [tuple(int(x) for x in r)[:6] for r in t[-12:]])
        break
    o.process(part)
    got = r.tape_json(part)
    want = o.tape_text()
    o.clear_tape()
    bk = eng.snapshot_books() == o.dump_books()
    lg = eng.snapshot_ledger() == o.dump_ledger()
    print("epoch", k, "serial", int(r.status.serial_fallback), "ledger_serial", int(r.status.ledger_serial),
          "ok" if got == want else "TAPE DIFF", "books", bk, "ledger", lg)
    if not lg:
        A, B = set(eng.snapshot_ledger().splitlines()), set(o.dump_ledger().splitlines())
        print(" engine only:", sorted(A - B)[:12])
        print(" oracle only:", sorted(B - A)[:12])
    if not bk:
        A, B = set(eng.snapshot_books().splitlines()), set(o.dump_books().splitlines())
        print(" engine only:", sorted(A - B)[:12])
        print(" oracle only:", sorted(B - A)[:12])
    if got != want or not bk or not lg:
        break
