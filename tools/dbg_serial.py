"""Diagnostic (GPU): a funded uniform stream whose epoch 3 is made serial by one unprovable order (a BUY
whose risk exceeds any funded bound: checkBalance rejects it, KP:177), through a drop-in-flags engine;
books and ledger compared with the oracle after every epoch.  argv: kme package dir (a built tree),
epoch, light_max."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pkg = sys.argv[1]
for p in ("tests", "oracle", ""):
    sys.path.insert(0, os.path.join(ROOT, p))
sys.path.insert(0, pkg)
import oracle  # noqa: E402
import kme  # noqa: E402
from kme import workloads as W  # noqa: E402

epoch = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
light = int(sys.argv[3]) if len(sys.argv) > 3 else 0
extra = {"max_sparse_symbols": int(sys.argv[4])} if len(sys.argv) > 4 else {}
print("kme from", kme.__file__)
base = W.Orders.concat([W.funded_setup(64, range(1, 8)), W.uniform(30_000, n_symbols=7, n_accounts=64, seed=23)])
N = len(base)
bad = W.Orders.from_rows([(W.BUY, 8_888_888_888, 5, 1, 100, 2_000_000_000)])
orders = W.Orders.concat([base.slice(0, N // 8), bad, base.slice(N // 8, N)])
eng = kme.Engine(kme.default_config(kme.MODE_FUNDED, max_symbols=8, max_epoch=4096, max_resting=1 << 16, max_accounts=64,
                                    ledger_capacity=1 << 14, light_max=light, flags=3, **extra))
o = oracle.Oracle()
for k, a in enumerate(range(0, min(len(orders), 8 * epoch), epoch)):
    part = orders.slice(a, min(len(orders), a + epoch))
    try:
        r = eng.process(part)
    except kme.KmeError as e:
        print("epoch", k, "fault", e)
        break
    o.process(part)
    got, want = r.tape_json(part), o.tape_text()
    o.clear_tape()
    bk = eng.snapshot_books() == o.dump_books()
    lg = eng.snapshot_ledger() == o.dump_ledger()
    print("epoch", k, "serial", int(r.status.serial_fallback), "ok" if got == want else "TAPE DIFF", "books", bk, "ledger", lg)
    if got != want or not bk or not lg:
        break
