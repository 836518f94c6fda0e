"""Faults and refusals, through the C ABI on the GPU:

* a domain fault mid-epoch: the reference forwards and commits every record before the one that
  throws (KP:97, 124-125), so the processor forwards exactly the oracle's tape of those records,
  in both modes, for faults found before matching (k_emap / k_route) and during it (H5 NPE in
  k_match or k_match_lanes while other symbol groups run past the fault in parallel);
* KME_E_UNFUNDED is not fatal: nothing of a refused order epoch takes effect, the engine accepts
  the next epoch and the refused records can be resubmitted after a top-up;
* capacity and persistence edges from the round-1 advisor: trade scratch with one trade per light
  group, restore of a mismatched / truncated checkpoint, checkpoint of a failed or in-flight epoch.
"""
import numpy as np
import pytest

import hazards
from kme import workloads as W

pytestmark = pytest.mark.gpu


def _funded_cfg(kme, G, accounts=64, E=1 << 16, P=1 << 18, light_max=0, max_trades=None):
    return kme.default_config(kme.MODE_FUNDED, max_symbols=G, max_epoch=E, max_resting=P, max_accounts=accounts,
                              light_max=light_max, max_trades=max_trades)


def _exact_cfg(kme, G=65, E=1 << 16, P=1 << 18):
    return kme.default_config(kme.MODE_EXACT, max_symbols=G, max_epoch=E, max_resting=P, ledger_capacity=1 << 16)


def _prefix_tape(oracle_mod, orders, k):
    o = oracle_mod.Oracle()
    o.process(orders.slice(0, k))
    return o.tape_text()


def _with_overshoot(n_body=6000, seed=3):
    """A funded body over symbols 3..40 with the H5 overshoot of symbol 1 in the middle: 48 bids on
    levels 0..47, then a SELL at 0 whose sweep NPEs (KP:234-235, 252-253) -- other symbols' records
    after it are matched in parallel on the device but must not be answered."""
    rows, _ = hazards.domain_streams()["log10_overshoot"]
    setup = [r for r in rows if r[0] in (W.CREATE_BALANCE, W.TRANSFER, W.ADD_SYMBOL)]
    setup += [(W.ADD_SYMBOL, 0, 0, s, 0, 0) for s in range(3, 41)]
    hot = [r for r in rows if r[0] in (W.BUY, W.SELL)]
    body = W.uniform(n_body, n_symbols=38, n_accounts=4, seed=seed, sid_base=3, aid_base=1, oid_base=10_000)
    half = n_body // 2
    return W.Orders.concat([W.Orders.from_rows(setup), body.slice(0, half), W.Orders.from_rows(hot),
                            body.slice(half, n_body)])


def _inject(orders, i, row):
    o = W.Orders.concat([orders.slice(0, i), W.Orders.from_rows([row]), orders.slice(i + 1, len(orders))])
    return o


def _fault_cases():
    setup = W.funded_setup(64, range(1, 65))
    body = W.uniform(20_000, n_symbols=64, n_accounts=64, seed=17)
    base = W.Orders.concat([setup, body])
    i = len(setup) + 12_345
    dup_oid = int(body.oid[100]) if body.action[100] in (W.BUY, W.SELL) else int(body.oid[101])
    return {
        # k_emap: a BUY/SELL reusing the oid of a live order (KP:221 would corrupt the lists)
        "dup_oid": (lambda: _inject(base, i, (W.BUY, dup_oid, 5, 7, 50, 3)), ("funded", "exact"), 8),
        # k_emap: FUNDED price outside 0..100
        "funded_range": (lambda: _inject(base, i, (W.BUY, 99_999_999, 5, 7, 101, 3)), ("funded",), 9),
        # k_match / k_match_lanes: the H5 NPE while other groups run on
        "overshoot_parallel": (_with_overshoot, ("funded", "exact"), 2),
    }


@pytest.mark.parametrize("case,mode,light_max", [(c, m, lm) for c, (_, modes, _) in sorted(_fault_cases().items())
                                                 for m in modes for lm in ((0, -1, 1 << 30) if m == "funded" else (0,))])
def test_processor_forwards_the_records_before_a_fault(kme_mod, oracle_mod, case, mode, light_max):
    make, _, detail = _fault_cases()[case]
    orders = make()
    cfg = _funded_cfg(kme_mod, 65, light_max=light_max) if mode == "funded" else _exact_cfg(kme_mod)
    p = kme_mod.Processor(cfg, epoch_records=1 << 16)
    for line in orders.to_json_lines():
        assert p.process_json(line) == 0
    rc = p.punctuate()
    assert kme_mod.STATUS[rc] == "DOMAIN"
    st = p.last_status()
    assert p.close() == 0   # a dead processor has nothing left to flush
    assert st.detail == detail
    k = int(st.error_index)
    assert k > len(orders) // 3 and st.n_effective == k
    if case == "overshoot_parallel":
        o = oracle_mod.Oracle()
        with pytest.raises(oracle_mod.OracleError) as oe:
            o.process(orders)
        assert oe.value.index == k
    want = _prefix_tape(oracle_mod, orders, k)
    got = p.tape_text()
    assert got == want
    assert p.commits == 1


@pytest.mark.parametrize("light_max", [0, 1 << 30])
def test_engine_results_before_a_fault(kme_mod, oracle_mod, light_max):
    """The host-buffer ABI: kme_submit_epoch fills out_* / trade_off / trades for the records
    [0, n_effective) of a faulting submission (here spanning an account sub-epoch and an order one)."""
    orders = _with_overshoot(n_body=20_000, seed=5)
    eng = kme_mod.Engine(_funded_cfg(kme_mod, 65, light_max=light_max))
    with pytest.raises(kme_mod.KmeError) as ke:
        eng.process(orders)
    assert ke.value.detail == 2
    k = ke.value.index
    assert ke.value.n_effective == k > 0
    part = orders.slice(0, k)
    assert ke.value.result.tape_json(part) == _prefix_tape(oracle_mod, orders, k)
    # a failed engine accepts nothing further
    with pytest.raises(kme_mod.KmeError) as again:
        eng.process(orders.slice(0, 10))
    assert kme_mod.STATUS[again.value.status] == "FAILED"


@pytest.mark.parametrize("light_max", [0, 1 << 30])
def test_unfunded_epoch_is_refused_without_effect(kme_mod, oracle_mod, light_max):
    n_sym, n_acc = 16, 8
    setup = W.Orders.from_rows([r for a in range(n_acc) for r in ((W.CREATE_BALANCE, 0, a, 0, 0, 0),
                                                                  (W.TRANSFER, 0, a, 0, 0, 200_000))]
                               + [(W.ADD_SYMBOL, 0, 0, s, 0, 0) for s in range(1, n_sym + 1)])
    first = W.uniform(200, n_symbols=n_sym, n_accounts=n_acc, seed=1, oid_base=1)
    big = W.uniform(3000, n_symbols=n_sym, n_accounts=n_acc, seed=2, oid_base=10_000)   # ~375 orders/account: unprovable
    topup = W.Orders.from_rows([(W.TRANSFER, 0, a, 0, 0, 2_000_000_000) for a in range(n_acc)])
    eng = kme_mod.Engine(_funded_cfg(kme_mod, n_sym + 1, accounts=n_acc, light_max=light_max))
    got = eng.process(setup).tape_json(setup) + eng.process(first).tape_json(first)
    books = eng.snapshot_books()
    with pytest.raises(kme_mod.KmeError) as ke:
        eng.process(big)
    assert kme_mod.STATUS[ke.value.status] == "UNFUNDED"
    assert eng.snapshot_books() == books                      # nothing of it took effect
    got += eng.process(topup).tape_json(topup)                 # the engine is alive
    got += eng.process(big).tape_json(big)                     # and takes the records now
    o = oracle_mod.Oracle()
    for part in (setup, first, topup, big):
        o.process(part)
    assert got == o.tape_text()
    assert eng.snapshot_books() == o.dump_books()


def test_unfunded_debit_keeps_the_records_before_it(kme_mod, oracle_mod):
    """A TRANSFER debit that cannot be proven (KP:142) stops an account epoch at its index: the
    records before it took effect, the engine goes on."""
    n_acc = 4
    setup = W.Orders.from_rows([r for a in range(n_acc) for r in ((W.CREATE_BALANCE, 0, a, 0, 0, 0),
                                                                  (W.TRANSFER, 0, a, 0, 0, 1000))]
                               + [(W.ADD_SYMBOL, 0, 0, 1, 0, 0)])
    acct = W.Orders.from_rows([(W.TRANSFER, 0, 0, 0, 0, 50), (W.CREATE_BALANCE, 0, 7, 0, 0, 0),
                               (W.TRANSFER, 0, 1, 0, 0, -5000), (W.TRANSFER, 0, 2, 0, 0, 70)])
    eng = kme_mod.Engine(_funded_cfg(kme_mod, 2, accounts=8))
    eng.process(setup)
    with pytest.raises(kme_mod.KmeError) as ke:
        eng.process(acct)
    assert kme_mod.STATUS[ke.value.status] == "UNFUNDED" and ke.value.index == 2
    after = W.Orders.from_rows([(W.BUY, 5, 0, 1, 50, 20), (W.SELL, 6, 7, 1, 40, 0), (W.BUY, 8, 2, 1, 10, 1)])
    got = eng.process(after).tape_json(after)
    o = oracle_mod.Oracle()
    o.process(setup)
    o.process(acct.slice(0, 2))
    o.clear_tape()
    o.process(after)
    assert got == o.tape_text()


def test_trade_scratch_one_trade_per_light_group(kme_mod, oracle_mod):
    """Advisor (round 1): k_match_lanes reserves trade scratch 8 slots per lane; an epoch of
    16,384 one-trade light groups with max_trades = max_epoch must still fit."""
    G, E = 16384, 16384
    setup = W.funded_setup(8, range(1, G + 1))
    rest = W.Orders.from_rows([(W.SELL, 1_000_000 + s, s % 8, s, 50, 3) for s in range(1, G + 1)])
    take = W.Orders.from_rows([(W.BUY, 2_000_000 + s, (s + 1) % 8, s, 50, 2) for s in range(1, G + 1)])
    eng = kme_mod.Engine(_funded_cfg(kme_mod, G + 1, accounts=8, E=E, P=1 << 16, max_trades=E))
    o = oracle_mod.Oracle()
    got = ""
    for part in (setup, rest, take):
        r = eng.process(part)
        got += r.tape_json(part)
        o.process(part)
    assert int(r.status.n_trades) == G
    assert got == o.tape_text()


def test_restore_refuses_mismatched_or_truncated_checkpoints(kme_mod, oracle_mod, tmp_path):
    """Advisor (round 1): a checkpoint of another geometry (max_epoch sizes the oid table) or a
    truncated file is refused before anything reaches the device; the engine stays usable."""
    setup = W.funded_setup(32, range(1, 17))
    a_part = W.uniform(4000, n_symbols=16, n_accounts=32, seed=8, oid_base=1)
    b_part = W.uniform(4000, n_symbols=16, n_accounts=32, seed=9, oid_base=100_000)
    src = kme_mod.Engine(_funded_cfg(kme_mod, 17, accounts=32, E=1 << 14))
    src.process(setup)
    src.process(a_part)
    ck = tmp_path / "a.ckpt"
    src.checkpoint(ck)
    raw = ck.read_bytes()
    (tmp_path / "short.ckpt").write_bytes(raw[: len(raw) - 100])
    for path, E in ((ck, 1 << 18), (tmp_path / "short.ckpt", 1 << 14)):
        dst = kme_mod.Engine(_funded_cfg(kme_mod, 17, accounts=32, E=E))
        dst.process(setup)
        before = dst.snapshot_books()
        with pytest.raises(kme_mod.KmeError) as ke:
            dst.restore(path)
        assert kme_mod.STATUS[ke.value.status] == "INVALID"
        assert dst.snapshot_books() == before
        got = dst.process(b_part).tape_json(b_part)          # untouched and alive
        o = oracle_mod.Oracle()
        o.process(setup)
        o.clear_tape()
        o.process(b_part)
        assert got == o.tape_text()
        dst.close()


def test_checkpoint_refuses_failed_or_pending_epochs(kme_mod, tmp_path):
    import torch

    rows, _ = hazards.domain_streams()["remove_nonempty"]
    orders = hazards.as_orders(rows)
    eng = kme_mod.Engine(_funded_cfg(kme_mod, 8, accounts=8))
    with pytest.raises(kme_mod.KmeError):
        eng.process(orders)
    with pytest.raises(kme_mod.KmeError) as ke:
        eng.checkpoint(tmp_path / "f.ckpt")
    assert kme_mod.STATUS[ke.value.status] == "FAILED"
    # an epoch in flight (submitted, not yet waited for)
    eng = kme_mod.Engine(_funded_cfg(kme_mod, 8, accounts=8))
    setup = W.funded_setup(8, range(1, 8))
    eng.process(setup)
    part = W.uniform(1000, n_symbols=7, n_accounts=8, seed=4)
    cols = {k: torch.from_numpy(np.ascontiguousarray(getattr(part, k))).cuda() for k in ("action", "oid", "aid", "sid", "price", "size")}
    eng.submit_device({k: t.data_ptr() for k, t in cols.items()}, len(part))
    with pytest.raises(kme_mod.KmeError) as ke:
        eng.checkpoint(tmp_path / "p.ckpt")
    assert kme_mod.STATUS[ke.value.status] == "INVALID"
    eng.wait()
    eng.checkpoint(tmp_path / "ok.ckpt")


def _device_cols(orders):
    import torch

    cols = {k: torch.from_numpy(np.ascontiguousarray(getattr(orders, k))).cuda()
            for k in ("action", "oid", "aid", "sid", "price", "size")}
    return cols, {k: t.data_ptr() for k, t in cols.items()}


def _unprovable(n_sym=16, n_acc=8):
    """Setup funded with 200,000 per account, then an order stream of ~375 orders per account that
    the per-account proof cannot hold, and the top-up that makes it provable."""
    setup = W.Orders.from_rows([r for a in range(n_acc) for r in ((W.CREATE_BALANCE, 0, a, 0, 0, 0),
                                                                  (W.TRANSFER, 0, a, 0, 0, 200_000))]
                               + [(W.ADD_SYMBOL, 0, 0, s, 0, 0) for s in range(1, n_sym + 1)])
    big = W.uniform(3000, n_symbols=n_sym, n_accounts=n_acc, seed=2, oid_base=10_000)
    topup = W.Orders.from_rows([(W.TRANSFER, 0, a, 0, 0, 2_000_000_000) for a in range(n_acc)])
    return setup, big, topup


@pytest.mark.parametrize("light_max", [0, 1 << 30])
def test_unproven_epoch_outranks_an_indexed_fault(kme_mod, oracle_mod, light_max):
    """Advisor (round 2): an epoch whose funded proof fails AND that holds an indexed fault further
    on (here FUNDED_RANGE) is refused as a whole -- no record of it is matched on an unproven
    ledger.  After the top-up the same records run up to the fault, as the reference would."""
    n_sym, n_acc = 16, 8
    setup, big, topup = _unprovable(n_sym, n_acc)
    i = 1700
    bad = _inject(big, i, (W.BUY, 99_999_999, 3, 5, 101, 3))
    eng = kme_mod.Engine(_funded_cfg(kme_mod, n_sym + 1, accounts=n_acc, light_max=light_max))
    got = eng.process(setup).tape_json(setup)
    books = eng.snapshot_books()
    with pytest.raises(kme_mod.KmeError) as ke:
        eng.process(bad)
    assert kme_mod.STATUS[ke.value.status] == "UNFUNDED" and ke.value.detail == 18   # KME_D_UNPROVEN
    assert ke.value.index == -1 and ke.value.n_effective == 0
    assert eng.snapshot_books() == books
    got += eng.process(topup).tape_json(topup)
    with pytest.raises(kme_mod.KmeError) as ke2:
        eng.process(bad)
    assert kme_mod.STATUS[ke2.value.status] == "DOMAIN" and ke2.value.detail == 9 and ke2.value.index == i
    got += ke2.value.result.tape_json(bad.slice(0, i))
    o = oracle_mod.Oracle()
    for part in (setup, topup, bad.slice(0, i)):
        o.process(part)
    assert got == o.tape_text()


def test_refused_mixed_device_epoch_leaves_no_account(kme_mod, oracle_mod):
    """Advisor (round 2): a device epoch mixing account records with orders (not split like host
    epochs) that the proof refuses must not leave its CREATE_BALANCE behind: after the documented
    top-up the resubmitted epoch creates the account, as the reference does."""
    import torch

    n_sym = 16
    setup, big, topup = _unprovable(n_sym, 7)                 # accounts 0..6; account 7 absent
    new_acct = W.Orders.from_rows([(W.CREATE_BALANCE, 0, 7, 0, 0, 0), (W.TRANSFER, 0, 7, 0, 0, 5000)])
    mixed = W.Orders.concat([new_acct, big])
    topup = W.Orders.concat([topup, W.Orders.from_rows([(W.TRANSFER, 0, 7, 0, 0, 1000)])])
    eng = kme_mod.Engine(_funded_cfg(kme_mod, n_sym + 1, accounts=8))
    got = eng.process(setup).tape_json(setup)
    cols, ptrs = _device_cols(mixed)
    eng.submit_device(ptrs, len(mixed))
    with pytest.raises(kme_mod.KmeError) as ke:
        eng.wait()
    assert kme_mod.STATUS[ke.value.status] == "UNFUNDED" and ke.value.n_effective == 0
    got += eng.process(topup).tape_json(topup)     # account 7 does not exist: its TRANSFER is rejected
    eng.submit_device(ptrs, len(mixed))
    eng.wait()
    got += eng.tape_json_device(ptrs, len(mixed)).decode()
    torch.cuda.synchronize()
    o = oracle_mod.Oracle()
    for part in (setup, topup, mixed):
        o.process(part)
    assert got == o.tape_text()
    assert eng.snapshot_books() == o.dump_books()


def test_checkpoint_after_an_unfunded_refusal(kme_mod, oracle_mod, tmp_path):
    """Advisor (round 2): KME_E_UNFUNDED is not fatal, so the engine can be checkpointed right after
    the refusal; a restored engine takes the top-up and the refused records like the original."""
    n_sym, n_acc = 16, 8
    setup, big, topup = _unprovable(n_sym, n_acc)
    eng = kme_mod.Engine(_funded_cfg(kme_mod, n_sym + 1, accounts=n_acc))
    got = eng.process(setup).tape_json(setup)
    with pytest.raises(kme_mod.KmeError):
        eng.process(big)
    ck = tmp_path / "after_refusal.ckpt"
    eng.checkpoint(ck)
    b = kme_mod.Engine(_funded_cfg(kme_mod, n_sym + 1, accounts=n_acc))
    b.restore(ck)
    got += b.process(topup).tape_json(topup) + b.process(big).tape_json(big)
    o = oracle_mod.Oracle()
    for part in (setup, topup, big):
        o.process(part)
    assert got == o.tape_text()
    assert b.snapshot_books() == o.dump_books()


def test_fault_at_record_zero_of_an_unproven_epoch(kme_mod, oracle_mod):
    """Advisor (round 3): at index 0 the error word orders by detail, and KME_D_UNPROVEN is the largest,
    so a fault of record 0 itself is reported instead of the refusal.  That is the reference's outcome
    (it throws at record 0 whatever the ledger holds): status DOMAIN at index 0, nothing takes
    effect, and the engine is failed as after any domain fault."""
    n_sym, n_acc = 16, 8
    setup, big, topup = _unprovable(n_sym, n_acc)
    bad = _inject(big, 0, (W.BUY, 99_999_999, 3, 5, 101, 3))            # record 0: FUNDED_RANGE
    eng = kme_mod.Engine(_funded_cfg(kme_mod, n_sym + 1, accounts=n_acc))
    eng.process(setup)
    books = eng.snapshot_books()
    with pytest.raises(kme_mod.KmeError) as ke:
        eng.process(bad)
    assert kme_mod.STATUS[ke.value.status] == "DOMAIN" and ke.value.detail == 9
    assert ke.value.index == 0 and ke.value.n_effective == 0
    assert eng.snapshot_books() == books
    with pytest.raises(kme_mod.KmeError) as ke2:
        eng.process(topup)
    assert kme_mod.STATUS[ke2.value.status] == "FAILED"


def test_host_epoch_refuses_a_short_trades_buffer_and_overlapping_registrations(kme_mod):
    """Advisor (round 3): a host epoch whose trades buffer holds fewer than max_trades records is
    refused at submit (the device may commit more trades than it could take), the engine stays
    usable; registering a range that shares a page with another registered range is refused, the
    same range twice is counted, and only the registering engine undoes a registration."""
    n_sym = 8
    E = 1 << 12
    cfg = _funded_cfg(kme_mod, n_sym + 1, accounts=16, E=E, P=1 << 14, max_trades=2 * E)
    eng = kme_mod.Engine(cfg)
    eng.process(W.funded_setup(16, range(1, n_sym + 1)))
    stream = W.uniform(E, n_symbols=n_sym, n_accounts=16, seed=4)
    cols = {k: np.ascontiguousarray(getattr(stream, k)) for k in ("action", "oid", "aid", "sid", "price", "size")}
    short = kme_mod.new_result(E, 2 * E - 1)
    with pytest.raises(kme_mod.KmeError) as ke:
        eng.submit_host(cols, E, short)
    assert kme_mod.STATUS[ke.value.status] == "INVALID"
    full = kme_mod.new_result(E, 2 * E)
    eng.submit_host(cols, E, full)
    st = eng.wait()
    assert st.status == 0 and full.trade_off[E] == st.n_trades
    # registrations: page-granular ownership
    raw = np.zeros(3 * 4096, np.uint8)
    base = (-raw.ctypes.data) % 4096
    a = raw[base:base + 100]
    b = raw[base + 200:base + 300]                       # the same page as a
    eng.host_register(a)
    eng.host_register(a)                                 # counted
    with pytest.raises(kme_mod.KmeError):
        eng.host_register(b)
    eng.host_unregister(a)
    eng.host_unregister(a)
    with pytest.raises(kme_mod.KmeError):
        eng.host_unregister(a)                           # no longer registered by this engine
    eng.host_register(b)                                 # the page is free again
    eng.host_unregister(b)
    eng.close()
