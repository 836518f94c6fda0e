"""GPU parity tests: the HIP engine (through the C ABI) against the CPU restatement (oracle/).

Bar: bit-exact MatchOut tape (byte-identical consumer.js text), bit-exact book stores, and in
EXACT mode bit-exact ledger stores.  Sizes are ones the oracle finishes in well under a second.
"""
import numpy as np
import pytest

import hazards
from kme import workloads as W

pytestmark = pytest.mark.gpu


def _funded_engine(kme, G, accounts=4096, E=1 << 16, P=1 << 18, light_max=0):
    return kme.Engine(kme.default_config(kme.MODE_FUNDED, max_symbols=G, max_epoch=E, max_resting=P,
                                         max_accounts=accounts, light_max=light_max))


def _exact_engine(kme, G=16, E=1 << 16, P=1 << 16):
    return kme.Engine(kme.default_config(kme.MODE_EXACT, max_symbols=G, max_epoch=E, max_resting=P,
                                         ledger_capacity=1 << 16))


def _run_epochs(eng, orders, epoch):
    text = []
    for a in range(0, len(orders), epoch):
        part = orders.slice(a, min(len(orders), a + epoch))
        r = eng.process(part)
        text.append(r.tape_json(part))
    return "".join(text)


def _first_diff(a: str, b: str) -> str:
    la, lb = a.splitlines(), b.splitlines()
    for k, (x, y) in enumerate(zip(la, lb)):
        if x != y:
            return f"line {k}: got {x!r} want {y!r}"
    return f"length got {len(la)} want {len(lb)}"


@pytest.mark.parametrize("seed,n_sym,epoch", [(1, 16, 4096), (2, 64, 1 << 14), (3, 1024, 1 << 16), (4, 3, 777)])
def test_funded_uniform_tape_and_books(kme_mod, oracle_mod, seed, n_sym, epoch):
    setup = W.funded_setup(512, range(1, n_sym + 1))
    stream = W.uniform(60_000, n_symbols=n_sym, n_accounts=512, seed=seed)
    allin = W.Orders.concat([setup, stream])
    eng = _funded_engine(kme_mod, n_sym + 1, accounts=512)
    got = _run_epochs(eng, allin, epoch)
    o = oracle_mod.Oracle()
    o.process(allin)
    want = o.tape_text()
    assert got == want, _first_diff(got, want)
    assert eng.snapshot_books() == o.dump_books()


def test_funded_cancel_replace_sweeps(kme_mod, oracle_mod):
    n_sym, n_acc = 32, 256
    stream = W.cancel_replace(20_000, n_symbols=n_sym, n_accounts=n_acc, seed=5)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1),
                           transfers_per_account=W.funded_transfers_needed(len(stream), n_acc, big=True))
    allin = W.Orders.concat([setup, stream])
    eng = _funded_engine(kme_mod, n_sym + 1, accounts=n_acc)
    got = _run_epochs(eng, allin, 5000)
    o = oracle_mod.Oracle()
    o.process(allin)
    assert got == o.tape_text(), _first_diff(got, o.tape_text())
    assert eng.snapshot_books() == o.dump_books()


def test_funded_zipf_hot_books(kme_mod, oracle_mod):
    n_sym, n_acc = 512, 1024
    stream = W.zipf(40_000, n_symbols=n_sym, n_accounts=n_acc, seed=9)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    allin = W.Orders.concat([setup, stream])
    eng = _funded_engine(kme_mod, n_sym + 1, accounts=n_acc)
    got = _run_epochs(eng, allin, 10_000)
    o = oracle_mod.Oracle()
    o.process(allin)
    assert got == o.tape_text(), _first_diff(got, o.tape_text())
    assert eng.snapshot_books() == o.dump_books()


@pytest.mark.parametrize("name", sorted(hazards.FUNDED_OK))
def test_funded_hazards(kme_mod, oracle_mod, name):
    orders = hazards.as_orders(hazards.streams()[name])
    eng = _funded_engine(kme_mod, 8, accounts=16, E=1024, P=4096)
    got = _run_epochs(eng, orders, 1024)
    o = oracle_mod.Oracle()
    o.process(orders)
    assert got == o.tape_text(), _first_diff(got, o.tape_text())
    assert eng.snapshot_books() == o.dump_books()


@pytest.mark.parametrize("name", sorted(hazards.streams()))
@pytest.mark.parametrize("epoch", [3, 1024])
def test_exact_hazards(kme_mod, oracle_mod, name, epoch):
    orders = hazards.as_orders(hazards.streams()[name])
    eng = _exact_engine(kme_mod, E=1024, P=4096)
    got = _run_epochs(eng, orders, epoch)
    o = oracle_mod.Oracle()
    o.process(orders)
    assert got == o.tape_text(), _first_diff(got, o.tape_text())
    assert eng.snapshot_books() == o.dump_books()
    assert eng.snapshot_ledger() == o.dump_ledger()


@pytest.mark.parametrize("name,mode", [(n, m) for n in sorted(hazards.domain_streams()) for m in ("exact", "funded")
                                       if not (m == "funded" and n == "price_126")])
def test_domain_errors_match_reference_faults(kme_mod, oracle_mod, name, mode):
    rows, detail = hazards.domain_streams()[name]
    orders = hazards.as_orders(rows)
    o = oracle_mod.Oracle()
    with pytest.raises(oracle_mod.OracleError) as oe:
        o.process(orders)
    eng = _exact_engine(kme_mod, E=1024, P=4096) if mode == "exact" else _funded_engine(kme_mod, 8, 16, 1024, 4096)
    with pytest.raises(kme_mod.KmeError) as ke:
        _run_epochs(eng, orders, 1024)
    assert ke.value.status == 3 and ke.value.detail == detail
    assert ke.value.index == oe.value.index


@pytest.mark.parametrize("seed,epoch", [(1, 100_000), (2, 4096), (3, 997)])
def test_exact_exchange_test_stream(kme_mod, oracle_mod, seed, epoch):
    orders = W.exchange_test(30_000, seed=seed)
    eng = _exact_engine(kme_mod, E=1 << 17, P=1 << 16)
    got = _run_epochs(eng, orders, epoch)
    o = oracle_mod.Oracle()
    o.process(orders)
    assert got == o.tape_text(), _first_diff(got, o.tape_text())
    assert eng.snapshot_books() == o.dump_books()
    assert eng.snapshot_ledger() == o.dump_ledger()


def test_processor_json_roundtrip(kme_mod, oracle_mod):
    """The Processor<String, Order> mirror fed the exchange_test.js wire format (string cancel
    oids included) forwards exactly the reference's MatchOut records."""
    orders = W.exchange_test(5_000, seed=11)
    cfg = kme_mod.default_config(kme_mod.MODE_EXACT, max_symbols=8, max_epoch=2048, max_resting=1 << 14)
    p = kme_mod.Processor(cfg, epoch_records=1000)
    for line in orders.to_json_lines():
        assert p.process_json(line) == 0
    assert p.close() == 0
    o = oracle_mod.Oracle()
    o.process(orders)
    assert p.tape_text() == o.tape_text()
    assert p.commits == (len(orders) + 999) // 1000


def test_funded_unfunded_is_refused(kme_mod):
    """Acceptance that depends on the ledger must not be decided in parallel."""
    rows = hazards._setup(fund=100) + [(W.BUY, 1, 1, 1, 50, 10)]
    eng = _funded_engine(kme_mod, 8, 16, 1024, 4096)
    with pytest.raises(kme_mod.KmeError) as ke:
        eng.process(hazards.as_orders(rows))
    assert ke.value.status == 4


def test_top_of_book(kme_mod, oracle_mod):
    import torch

    setup = W.funded_setup(64, range(1, 9))
    stream = W.uniform(5000, n_symbols=8, n_accounts=64, seed=2)
    eng = _funded_engine(kme_mod, 9, accounts=64)
    eng.process(W.Orders.concat([setup, stream]))
    tob = torch.zeros((9, 4), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()                          # (torch's fill before the engine's stream writes)
    eng.top_of_book(tob.data_ptr())
    torch.cuda.synchronize()
    eng.wait()
    tob = tob.cpu().numpy()
    # from the oracle's book dump: highest bid level of +g, lowest ask level of -g
    o = oracle_mod.Oracle()
    o.process(W.Orders.concat([setup, stream]))
    books = {int(l.split()[1]): (int(l.split()[2]), int(l.split()[3])) for l in o.dump_books().splitlines()
             if l.startswith("B ")}
    for g in range(1, 9):
        msb, lsb = books[g]
        bits = [p for p in range(127) if ((lsb >> p) & 1 if p < 63 else (msb >> (p - 63)) & 1)]
        assert tob[g, 0] == (max(bits) if bits else -1)
        msb, lsb = books[-g]
        bits = [p for p in range(127) if ((lsb >> p) & 1 if p < 63 else (msb >> (p - 63)) & 1)]
        assert tob[g, 1] == (min(bits) if bits else -1)


def _device_cols(orders):
    import torch

    cols = {k: torch.from_numpy(np.ascontiguousarray(getattr(orders, k))).cuda()
            for k in ("action", "oid", "aid", "sid", "price", "size")}
    return cols, {k: t.data_ptr() for k, t in cols.items()}


@pytest.mark.parametrize("mode", ["funded", "exact"])
def test_device_serializer_matches_oracle_tape(kme_mod, oracle_mod, mode):
    """kme_tape_json_device (SURVEY §8 f next-1): the GPU prints each epoch's MatchOut records
    byte-identically to the reference's Jackson + consumer.js format."""
    if mode == "funded":
        n_sym = 48
        setup = W.funded_setup(256, range(1, n_sym + 1))
        stream = W.uniform(30_000, n_symbols=n_sym, n_accounts=256, seed=21)
        eng = _funded_engine(kme_mod, n_sym + 1, accounts=256)
    else:
        orders = W.exchange_test(12_000, seed=5)
        setup, stream = orders.slice(0, 40), orders.slice(40, len(orders))
        eng = _exact_engine(kme_mod, E=1 << 14, P=1 << 16)
    o = oracle_mod.Oracle()
    o.process(setup)
    eng.process(setup)
    o.clear_tape()
    epoch = 7_001
    for a in range(0, len(stream), epoch):
        part = stream.slice(a, min(len(stream), a + epoch))
        cols, ptrs = _device_cols(part)
        eng.submit_device(ptrs, len(part))
        eng.wait()
        got = eng.tape_json_device(ptrs, len(part)).decode()
        o.process(part)
        want = o.tape_text()
        o.clear_tape()
        assert got == want, _first_diff(got, want)


@pytest.mark.parametrize("mode", ["funded", "exact"])
def test_checkpoint_restore_resumes_exactly(kme_mod, oracle_mod, mode, tmp_path):
    """Row f next-3: a checkpoint taken after an epoch, restored into a fresh engine, continues the
    stream with the tape, books (and EXACT ledger) of an uninterrupted run."""
    if mode == "funded":
        n_sym = 40
        setup = W.funded_setup(300, range(1, n_sym + 1))
        stream = W.uniform(24_000, n_symbols=n_sym, n_accounts=300, seed=31)
        allin = W.Orders.concat([setup, stream])
        make = lambda: _funded_engine(kme_mod, n_sym + 1, accounts=300)
    else:
        allin = W.exchange_test(16_000, seed=9)
        make = lambda: _exact_engine(kme_mod, E=1 << 14, P=1 << 16)
    cut = len(allin) // 2
    first, second = allin.slice(0, cut), allin.slice(cut, len(allin))
    a = make()
    _run_epochs(a, first, 4096)
    ck = tmp_path / "engine.ckpt"
    a.checkpoint(ck)
    want_rest = _run_epochs(a, second, 4096)
    b = make()
    b.restore(ck)
    got_rest = _run_epochs(b, second, 4096)
    assert got_rest == want_rest, _first_diff(got_rest, want_rest)
    o = oracle_mod.Oracle()
    o.process(first)
    o.clear_tape()
    o.process(second)
    assert got_rest == o.tape_text(), _first_diff(got_rest, o.tape_text())
    assert b.snapshot_books() == o.dump_books()
    if mode == "exact":
        assert b.snapshot_ledger() == o.dump_ledger()


@pytest.mark.parametrize("kind", ["uniform", "cancel_replace", "hazards"])
def test_funded_exact_ledger_replay(kme_mod, oracle_mod, kind):
    """Row f next-2: FUNDED matching in parallel + the serial ledger replay gives the reference's
    final Balances / Positions stores, value-keyed position writes (KP:434-436) included."""
    if kind == "hazards":
        names = [n for n in sorted(hazards.FUNDED_OK)]
        streams = [hazards.as_orders(hazards.streams()[n]) for n in names]
        G, A = 8, 16
    else:
        n_sym, n_acc = 24, 48
        body = (W.uniform(20_000, n_symbols=n_sym, n_accounts=n_acc, seed=41) if kind == "uniform"
                else W.cancel_replace(12_000, n_symbols=n_sym, n_accounts=n_acc, seed=42))
        k = W.funded_transfers_needed(len(body), n_acc, big=kind == "cancel_replace")
        streams = [W.Orders.concat([W.funded_setup(n_acc, range(1, n_sym + 1), transfers_per_account=k), body])]
        G, A = n_sym + 1, n_acc
    for orders in streams:
        eng = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=G, max_epoch=4096,
                                                    max_resting=1 << 16, max_accounts=A,
                                                    flags=kme_mod.FLAG_EXACT_LEDGER))
        got = _run_epochs(eng, orders, 4096)
        o = oracle_mod.Oracle()
        o.process(orders)
        assert got == o.tape_text(), _first_diff(got, o.tape_text())
        assert eng.snapshot_books() == o.dump_books()
        assert eng.snapshot_ledger() == o.dump_ledger()
        eng.close()


def test_funded_max_resting_is_a_guarantee(kme_mod, oracle_mod):
    """max_resting resting orders fit however they spread over symbols: the pool adds the slots
    each group can hold back in its allocation chunk (POOL_CHUNK per group)."""
    n_sym, P = 256, 1000
    setup = W.funded_setup(64, range(1, n_sym + 1))
    stream = W.uniform(P, n_symbols=n_sym, n_accounts=64, seed=11, mix=(1.0, 0.0, 0.0))  # every BUY rests
    allin = W.Orders.concat([setup, stream])
    eng = _funded_engine(kme_mod, n_sym + 1, accounts=64, E=1 << 12, P=P)
    got = _run_epochs(eng, allin, 1 << 12)
    o = oracle_mod.Oracle()
    o.process(allin)
    assert got == o.tape_text()
    assert eng.snapshot_books() == o.dump_books()


# light_max: -1 = one wavefront per group only (k_match), 1 << 30 = one lane per group only
# (k_match_lanes), 40 = both kernels in the same epoch (concurrently, on disjoint groups)
LIGHT = [-1, 1 << 30, 40]


@pytest.mark.parametrize("light_max", LIGHT)
@pytest.mark.parametrize("kind", ["uniform", "zipf", "cancel_replace"])
def test_funded_matching_paths_agree(kme_mod, oracle_mod, kind, light_max):
    """Both matching kernels, alone and together, give the reference's tape and books."""
    n_sym, n_acc = 256, 512
    if kind == "uniform":
        stream = W.uniform(30_000, n_symbols=n_sym, n_accounts=n_acc, seed=21)
    elif kind == "zipf":
        stream = W.zipf(30_000, n_symbols=n_sym, n_accounts=n_acc, seed=22)
    else:
        stream = W.cancel_replace(12_000, n_symbols=n_sym, n_accounts=n_acc, seed=23)
    setup = W.funded_setup(n_acc, range(1, n_sym + 1),
                           transfers_per_account=W.funded_transfers_needed(len(stream), n_acc, big=kind == "cancel_replace"))
    allin = W.Orders.concat([setup, stream])
    eng = _funded_engine(kme_mod, n_sym + 1, accounts=n_acc, light_max=light_max)
    got = _run_epochs(eng, allin, 8192)
    o = oracle_mod.Oracle()
    o.process(allin)
    assert got == o.tape_text(), _first_diff(got, o.tape_text())
    assert eng.snapshot_books() == o.dump_books()


@pytest.mark.parametrize("light_max", LIGHT)
@pytest.mark.parametrize("name", sorted(hazards.FUNDED_OK))
def test_funded_hazards_both_paths(kme_mod, oracle_mod, name, light_max):
    orders = hazards.as_orders(hazards.streams()[name])
    eng = _funded_engine(kme_mod, 8, accounts=16, E=1024, P=4096, light_max=light_max)
    got = _run_epochs(eng, orders, 1024)
    o = oracle_mod.Oracle()
    o.process(orders)
    assert got == o.tape_text(), _first_diff(got, o.tape_text())
    assert eng.snapshot_books() == o.dump_books()


@pytest.mark.parametrize("light_max", [-1, 1 << 30])
@pytest.mark.parametrize("name", sorted(n for n in hazards.domain_streams() if n != "price_126"))
def test_funded_domain_errors_both_paths(kme_mod, oracle_mod, name, light_max):
    rows, detail = hazards.domain_streams()[name]
    orders = hazards.as_orders(rows)
    o = oracle_mod.Oracle()
    with pytest.raises(oracle_mod.OracleError) as oe:
        o.process(orders)
    eng = _funded_engine(kme_mod, 8, 16, 1024, 4096, light_max=light_max)
    with pytest.raises(kme_mod.KmeError) as ke:
        _run_epochs(eng, orders, 1024)
    assert ke.value.status == 3 and ke.value.detail == detail
    assert ke.value.index == oe.value.index


@pytest.mark.parametrize("light_max", [0, -1])
def test_funded_serial_fallback_is_exact(kme_mod, oracle_mod, light_max):
    """Row f next-2, validate-and-replay: epochs whose funded proof fails (accounts running out of
    cash, checkBalance rejects) are matched serially on the exact ledger; the others in parallel.
    Tape, books and ledger stay bit-exact, and both paths are taken."""
    n_sym, n_acc = 32, 64
    rows = [(W.CREATE_BALANCE, 0, a, 0, 0, 0) for a in range(n_acc)]
    rows += [(W.ADD_SYMBOL, 0, 0, s, 0, 0) for s in range(1, n_sym + 1)]
    setup = W.Orders.from_rows(rows)
    stream = W.uniform(18_000, n_symbols=n_sym, n_accounts=n_acc, seed=31)
    topup = W.Orders.from_rows([(W.TRANSFER, 0, a, 0, 0, 160_000) for a in range(n_acc)])
    chunks = [setup]
    for c in range(0, len(stream), 6000):   # top up, then three epochs of 2,000 orders
        chunks.append(topup)
        chunks += [stream.slice(c + k, min(len(stream), c + k + 2000)) for k in range(0, 6000, 2000)]
    cfg = kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=1 << 12, max_resting=1 << 16,
                                 max_accounts=n_acc, ledger_capacity=1 << 14, light_max=light_max,
                                 flags=kme_mod.FLAG_EXACT_LEDGER | kme_mod.FLAG_SERIAL_FALLBACK)
    eng = kme_mod.Engine(cfg)
    got, serial = [], []
    for ch in chunks:
        r = eng.process(ch)
        got.append(r.tape_json(ch))
        if ch is not topup and ch is not setup:
            serial.append(int(r.status.serial_fallback))
    o = oracle_mod.Oracle()
    o.process(W.Orders.concat(chunks))
    got = "".join(got)
    assert got == o.tape_text(), _first_diff(got, o.tape_text())
    assert eng.snapshot_books() == o.dump_books()
    assert eng.snapshot_ledger() == o.dump_ledger()
    assert 0 < sum(serial) < len(serial), serial
    assert '"action":7' in got   # balance rejects happened (serial epochs)


def test_serial_fallback_needs_exact_ledger(kme_mod):
    cfg = kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=4, max_epoch=64, max_resting=256, max_accounts=8,
                                 flags=kme_mod.FLAG_SERIAL_FALLBACK)
    with pytest.raises(kme_mod.KmeError):
        kme_mod.Engine(cfg)


@pytest.mark.parametrize("light_max", LIGHT)
def test_funded_cancels_of_orders_of_the_same_epoch(kme_mod, oracle_mod, light_max):
    """Cancels of orders submitted earlier in the same epoch, whose oid-table entry the matching
    kernel finalises (rest slot or DEAD) before the cancel reads it: an order that rested, one
    cancelled twice, one filled at once, one rejected for its book, one rejected for its account,
    one filled later in the epoch, next to cancels of orders of earlier epochs (KP:289-323)."""
    B, S, C = W.BUY, W.SELL, W.CANCEL
    setup = W.funded_setup(8, range(1, 5))
    e1 = W.Orders.from_rows([
        (B, 10, 1, 1, 50, 40), (S, 11, 2, 2, 60, 10), (B, 12, 3, 3, 30, 7)])
    e2 = W.Orders.from_rows([
        (B, 20, 1, 1, 40, 10), (C, 20, 1, 0, 0, 0), (C, 20, 1, 0, 0, 0),      # rested, cancelled twice
        (S, 21, 2, 1, 50, 30), (C, 21, 2, 0, 0, 0),                          # filled against 10
        (B, 22, 3, 9, 40, 5), (C, 22, 3, 0, 0, 0),                           # no book for sid 9
        (B, 23, 200, 3, 40, 5), (C, 23, 200, 0, 0, 0),                       # no balance (account beyond the table)
        (C, 10, 1, 0, 0, 0),                                                 # earlier epoch, partly filled
        (B, 24, 4, 2, 45, 5), (S, 25, 5, 2, 45, 5), (C, 24, 4, 0, 0, 0), (C, 25, 5, 0, 0, 0),
        (B, 26, 6, 4, 55, 8), (S, 27, 7, 4, 50, 3), (C, 26, 6, 0, 0, 0),     # partly filled, then cancelled
        (C, 11, 1, 0, 0, 0), (C, 11, 2, 0, 0, 0),                            # wrong account, then the owner
        (B, 28, 3, 3, 31, 4), (S, 29, 4, 3, 30, 11), (C, 28, 3, 0, 0, 0), (C, 12, 3, 0, 0, 0)])
    e3 = W.Orders.from_rows([
        (C, 24, 4, 0, 0, 0), (C, 26, 6, 0, 0, 0), (C, 29, 4, 0, 0, 0), (B, 30, 1, 1, 41, 2), (C, 30, 1, 0, 0, 0)])
    eng = _funded_engine(kme_mod, 10, accounts=128, light_max=light_max)
    o = oracle_mod.Oracle()
    got, want = [], []
    for part in (setup, e1, e2, e3):
        got.append(eng.process(part).tape_json(part))
        o.process(part)
    want = o.tape_text()
    assert "".join(got) == want, _first_diff("".join(got), want)
    assert eng.snapshot_books() == o.dump_books()
