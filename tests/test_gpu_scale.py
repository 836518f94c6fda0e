"""GPU parity at bench-like scale: hundreds to tens of thousands of symbol groups matched in one
launch, epochs of 2^18 records, every epoch's MatchOut tape byte-identical to the oracle's and the
final book stores equal.

The small parity tests (test_gpu_parity.py) touch a few hundred node slots; at this scale the
slots run into the tens of thousands, free-list blocks get recycled across batches, and
cancels hit orders that were swept earlier in the same epoch -- the combination that exposed a
stale-node acceptance in k_match's batch cancel prefetch (a freed slot hosting a free-list block
has a slot id in word 12, whose bit 11 was packed over the prefetch's `ok` bit).
"""
import numpy as np
import pytest

from kme import workloads as W

pytestmark = pytest.mark.gpu

E = 1 << 18


def _check(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, light_max, epoch=E):
    eng = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1,
                                                max_epoch=max(epoch, len(setup)), max_resting=1 << 22,
                                                max_trades=2 * epoch + (1 << 16), max_accounts=n_acc,
                                                light_max=light_max))
    o = oracle_mod.Oracle()
    parts = [setup] + [stream.slice(a, min(len(stream), a + epoch)) for a in range(0, len(stream), epoch)]
    for k, part in enumerate(parts):
        got = eng.process(part).tape_json(part)
        o.process(part)
        want = o.tape_text()
        o.clear_tape()
        if got != want:
            la, lb = got.splitlines(), want.splitlines()
            j = next((j for j, (x, y) in enumerate(zip(la, lb)) if x != y), min(len(la), len(lb)))
            pytest.fail(f"epoch {k}: line {j}: got {la[j] if j < len(la) else None!r} "
                        f"want {lb[j] if j < len(lb) else None!r}")
    assert eng.snapshot_books() == o.dump_books()
    eng.close()


@pytest.mark.parametrize("light_max", [-1, 0, 1 << 30])
def test_c5_cancel_replace_at_scale(kme_mod, oracle_mod, light_max):
    """C5 (1,024 symbols, 4,096 accounts): cancels of orders swept earlier in the epoch; with
    light_max = 2^30 every group (~1,500 records per epoch) runs in k_match_lanes, so the lanes
    kernel's cancel path sees the churn at scale."""
    n_sym, n_acc, n = 1024, 4096, 6 * E
    stream = W.cancel_replace(n, n_symbols=n_sym, n_accounts=n_acc, seed=1000)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1),
                           transfers_per_account=W.funded_transfers_needed(n, n_acc, big=True))
    _check(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, light_max)


def test_c3_uniform_at_scale(kme_mod, oracle_mod):
    """C3's shape (65,536 symbols and accounts): light groups in lanes, busy ones in wavefronts."""
    n_sym, n_acc, n = 65536, 65536, 4 * E
    stream = W.uniform(n, n_symbols=n_sym, n_accounts=n_acc, seed=1000)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    _check(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, 0)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("flags", [0, 3])
def test_c3_bench_stream_at_bench_shape(kme_mod, oracle_mod, flags):
    """The bench's own C3 stream (bench.make_workload: seed 1000, 65,536 symbols and accounts) in
    its own epoch size, 2^22 records, for six epochs: ~64 records per group per epoch, free-list
    blocks recycled across epochs, and an oid-table rebuild (kme_wait: (used + max_epoch) * 2 >
    capacity) between epochs 5 and 6.  Every epoch's tape is compared in binary (tests/tapes.py)
    with the oracle's, the books at the end line by line.  flags = 3: the drop-in's configuration
    (KME_FLAG_EXACT_LEDGER | KME_FLAG_SERIAL_FALLBACK, bench.py --flags exact_ledger,serial_fallback),
    Balances / Positions compared with the oracle's after every epoch, from the default initial
    ledger size (the tables grow between epochs)."""
    import bench
    import tapes

    E22, n_ep, max_resting = 1 << 22, 6, 4_000_000
    setup, stream, sids, nacc, _, _ = bench.make_workload("c3", n_ep * E22, 0, 1)
    eng = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=int(sids.max()) + 1, max_epoch=E22,
                                                max_resting=max_resting, max_trades=2 * E22 + (1 << 16),
                                                max_accounts=nacc, flags=flags))
    # the oid table's capacity (kme_create) and the epoch after which kme_wait rebuilds it
    pool = max_resting + (int(sids.max()) + 2) * 64
    cap = 1 << (2 * (pool + E22) - 1).bit_length()
    bs_per_epoch = [int(np.count_nonzero(np.isin(stream.action[k * E22:(k + 1) * E22], (W.BUY, W.SELL)))) for k in range(n_ep)]
    assert (sum(bs_per_epoch[:5]) + E22) * 2 > cap > (sum(bs_per_epoch[:4]) + E22) * 2
    o = oracle_mod.Oracle()
    o.process(setup)
    eng.process(setup)
    o.clear_tape()
    for k in range(n_ep):
        part = stream.slice(k * E22, (k + 1) * E22)
        r = eng.process(part)
        o.process(part)
        want = o.tape()
        o.clear_tape()
        got = tapes.engine_tape(part, r, oracle_mod.REC_DTYPE)
        d = tapes.first_difference(got, want)
        assert d is None, f"epoch {k}: tape row {d}: got {got[d] if d < len(got) else None} want {want[d] if d < len(want) else None}"
        assert r.status.n_trades > 1_000_000
        if flags:
            assert r.status.serial_fallback == 0 and r.status.ledger_serial == 0   # the parallel ledger pass kept it
            assert eng.snapshot_ledger() == o.dump_ledger(), f"epoch {k}: ledger"
    assert eng.snapshot_books() == o.dump_books()
    eng.close()


def test_c4_zipf_65536_symbols(kme_mod, oracle_mod):
    """C4 at its own universe, 65,536 symbols (Zipf 1.1: the hottest symbol takes ~12% of the
    records, thousands of orders deep, in k_match; the tail in k_match_lanes)."""
    n_sym, n_acc, n = 65536, 65536, 2 * E
    stream = W.zipf(n, n_symbols=n_sym, n_accounts=n_acc, seed=1002)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    _check(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, 0)


@pytest.mark.parametrize("rank", [0, 5])
def test_c4_zipf_n8_shard(kme_mod, oracle_mod, rank):
    """The records rank r of an 8-GPU C4 run matches (``W.zipf(shard=(r, 8))``: its murmur2 share of
    the 65,536 symbols, with their popularity in the whole universe) -- the shard whose hot books
    bound C4's weak scaling (bench.py --workload c4 --shard r/8)."""
    n_sym, n_acc, n = 65536, 65536, 2 * E
    stream = W.zipf(n, n_symbols=n_sym, n_accounts=n_acc, seed=1000 + rank, shard=(rank, 8))
    sids = W.shard_symbols(n_sym, 8, rank)
    setup = W.funded_setup(n_acc, sids)
    _check(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, 0)


def test_c2_uniform_at_scale(kme_mod, oracle_mod):
    """C2's shape (1,024 symbols): every group busy, one wavefront each."""
    n_sym, n_acc, n = 1024, 4096, 4 * E
    stream = W.uniform(n, n_symbols=n_sym, n_accounts=n_acc, seed=1001)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    _check(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, 0)


def test_c4_zipf_at_scale(kme_mod, oracle_mod):
    """C4's shape (Zipf(1.1) over 8,192 symbols): hot books thousands of orders deep."""
    n_sym, n_acc, n = 8192, 16384, 2 * E
    stream = W.zipf(n, n_symbols=n_sym, n_accounts=n_acc, seed=1002)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    _check(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, 0)



def test_n8_shard_shape_at_scale(kme_mod, oracle_mod):
    """The per-GPU shard of C3 at N = 8 (8,192 symbols), 2^21-record epochs: 256 records per group
    per epoch, every group busy (one wavefront each), several record batches per group."""
    n_sym, n_acc, n = 8192, 65536, 1 << 22
    stream = W.uniform(n, n_symbols=n_sym, n_accounts=n_acc, seed=1003)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    _check(kme_mod, oracle_mod, setup, stream, n_sym, n_acc, 0, epoch=1 << 21)


def test_exact_exchange_test_at_scale(kme_mod, oracle_mod):
    """C1 (exchange_test.js stream) through the EXACT engine, 300k events in 2^16-record epochs;
    tape, books and the ledger stores (Balances, Positions) against the oracle."""
    orders = W.exchange_test(300_000, seed=11)
    # N(50, 10) prices leave the parity domain eventually (a BUY/SELL priced outside 0..126 may
    # rest, where the engine refuses with KME_D_PRICE): stop before the first such order
    out = np.nonzero(((orders.action == W.BUY) | (orders.action == W.SELL)) & ((orders.price < 0) | (orders.price > 126)))[0]
    if len(out):
        orders = orders.slice(0, int(out[0]))
    assert len(orders) > 100_000
    eng = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_EXACT, max_symbols=16, max_epoch=1 << 16,
                                                max_resting=1 << 18, ledger_capacity=1 << 16))
    o = oracle_mod.Oracle()
    for a in range(0, len(orders), 1 << 16):
        part = orders.slice(a, min(len(orders), a + (1 << 16)))
        got = eng.process(part).tape_json(part)
        o.process(part)
        want = o.tape_text()
        o.clear_tape()
        assert got == want, f"epoch at {a}"
    assert eng.snapshot_books() == o.dump_books()
    assert eng.snapshot_ledger() == o.dump_ledger()


@pytest.mark.parametrize("kind", ["uniform", "cancel_replace"])
def test_exact_ledger_replay_at_scale(kme_mod, oracle_mod, kind):
    """FUNDED matching with KME_FLAG_EXACT_LEDGER at 512 symbols x 2,048 accounts, 2^18-record
    epochs: the replayed Balances / Positions equal the oracle's after every epoch."""
    n_sym, n_acc, n = 512, 2048, 3 * E
    body = (W.uniform(n, n_symbols=n_sym, n_accounts=n_acc, seed=1004) if kind == "uniform"
            else W.cancel_replace(n, n_symbols=n_sym, n_accounts=n_acc, seed=1005))
    k = W.funded_transfers_needed(n, n_acc, big=kind == "cancel_replace")
    setup = W.funded_setup(n_acc, range(1, n_sym + 1), transfers_per_account=k)
    eng = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=E,
                                                max_resting=1 << 21, max_trades=2 * E + (1 << 16), max_accounts=n_acc,
                                                ledger_capacity=1 << 20, flags=kme_mod.FLAG_EXACT_LEDGER))
    o = oracle_mod.Oracle()
    for part in [setup] + [body.slice(a, min(n, a + E)) for a in range(0, n, E)]:
        got = eng.process(part).tape_json(part)
        o.process(part)
        want = o.tape_text()
        o.clear_tape()
        assert got == want
        assert eng.snapshot_ledger() == o.dump_ledger()
    assert eng.snapshot_books() == o.dump_books()


def test_serial_fallback_at_scale(kme_mod, oracle_mod):
    """Validate-and-replay at 256 symbols x 1,024 accounts: accounts topped up before every third
    2^16-record epoch, so proven epochs run in parallel and the ones that run short of cash fall
    back to the serial exact engine; tape, books and ledger stay exact across the mix."""
    n_sym, n_acc, ep = 256, 1024, 1 << 16
    rows = [(W.CREATE_BALANCE, 0, a, 0, 0, 0) for a in range(n_acc)]
    rows += [(W.ADD_SYMBOL, 0, 0, s, 0, 0) for s in range(1, n_sym + 1)]
    setup = W.Orders.from_rows(rows)
    stream = W.uniform(9 * ep, n_symbols=n_sym, n_accounts=n_acc, seed=1006)
    topup = W.Orders.from_rows([(W.TRANSFER, 0, a, 0, 0, 300_000) for a in range(n_acc)])
    chunks = [setup]
    for c in range(0, len(stream), 3 * ep):
        chunks.append(topup)
        chunks += [stream.slice(c + k, c + k + ep) for k in range(0, 3 * ep, ep)]
    eng = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=ep,
                                                max_resting=1 << 20, max_trades=4 * ep, max_accounts=n_acc,
                                                ledger_capacity=1 << 18,
                                                flags=kme_mod.FLAG_EXACT_LEDGER | kme_mod.FLAG_SERIAL_FALLBACK))
    o = oracle_mod.Oracle()
    serial = []
    for ch in chunks:
        r = eng.process(ch)
        got = r.tape_json(ch)
        o.process(ch)
        want = o.tape_text()
        o.clear_tape()
        assert got == want
        if ch is not topup and ch is not setup:
            serial.append(int(r.status.serial_fallback))
    assert eng.snapshot_books() == o.dump_books()
    assert eng.snapshot_ledger() == o.dump_ledger()
    assert 0 < sum(serial) < len(serial), serial
