"""The host path at rate (include/kme.h "Host epochs at device rate"): kme_submit_epoch_host over
registered host memory, two epochs in flight, kme_poll / kme_wait, and kme_expand_rows -- the calls
the Java processor's JNI glue makes -- against the oracle's tape (KP:96-126), plus the C harness that
bench.py times (integration/host_harness.c)."""
import ctypes as C
import os
import time

import numpy as np
import pytest

from kme import workloads as W

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cols(epoch):
    out = {}
    for name, dt in (("action", np.int32), ("oid", np.int64), ("aid", np.int64), ("sid", np.int64),
                     ("price", np.int32), ("size", np.int32)):
        raw = np.zeros(epoch * np.dtype(dt).itemsize + 4096, np.uint8)
        off = (-raw.ctypes.data) % 4096
        out[name] = raw[off:off + epoch * np.dtype(dt).itemsize].view(dt)
    return out


@pytest.mark.parametrize("register", [True, False])
def test_host_epochs_two_in_flight_equal_oracle(kme_mod, oracle_mod, register):
    """Epoch k + 1 is queued before epoch k is waited for; each epoch's results land in its own
    registered host arrays (unregistered ones take the synchronous copies) and its MatchOut rows
    equal the oracle's tape."""
    n_sym, n_acc, epoch = 48, 512, 1 << 13
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    stream = W.uniform(60_000, n_symbols=n_sym, n_accounts=n_acc, seed=41)
    eng = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=epoch,
                                                max_resting=1 << 18, max_accounts=n_acc, max_trades=4 * epoch))
    eng.process(setup)
    slots = [(_cols(epoch), kme_mod.new_result(epoch, 4 * epoch)) for _ in range(2)]
    if register:
        for cols, res in slots:
            for a in list(cols.values()) + [res.out_action, res.out_size, res.out_prev, res.out_flags, res.trade_off,
                                             res.trades]:
                eng.host_register(a)
    assert eng.poll()                                  # nothing in flight
    parts = [stream.slice(a, min(len(stream), a + epoch)) for a in range(0, len(stream), epoch)]
    pending, got = [], []

    def complete():
        k, part = pending.pop(0)
        t0 = time.time()
        while not eng.poll():
            assert time.time() - t0 < 60
        st = eng.wait()
        assert st.status == 0 and st.n_inputs == len(part)
        cols, res = slots[k % 2]
        got.append(kme_mod.expand_rows(part, res))
        r = kme_mod.EpochResult(res.out_action[:len(part)], res.out_size[:len(part)], res.out_prev[:len(part)],
                                res.out_flags[:len(part)], res.trade_off[:len(part) + 1], res.trades, st)
        return r.tape_json(part)

    text = []
    for k, part in enumerate(parts):
        if len(pending) == 2:
            text.append(complete())
        cols, _ = slots[k % 2]
        for name, v in cols.items():
            v[:len(part)] = getattr(part, name)
        eng.submit_host(cols, len(part), slots[k % 2][1])
        pending.append((k, part))
    while pending:
        text.append(complete())
    o = oracle_mod.Oracle()
    o.process(setup)
    o.clear_tape()
    o.process(stream)
    assert "".join(text) == o.tape_text()
    rows = np.concatenate(got)
    want = o.tape()
    assert len(rows) == len(want)
    assert (rows["oid"] == want["oid"]).all() and (rows["size"] == want["size"]).all()
    assert ((rows["kind"] != 0).astype(np.int32) == want["key"]).all()
    if register:
        for cols, res in slots:
            for a in list(cols.values()) + [res.out_action, res.out_size, res.out_prev, res.out_flags, res.trade_off,
                                             res.trades]:
                eng.host_unregister(a)


def test_host_harness_runs_the_processor_schedule(kme_mod):
    """integration/libkme_host_harness.so (bench.py host_path): every epoch forwarded, 2 rows per
    record plus 2 per trade."""
    import bench

    n_sym, n_acc, epoch, n_ep = 256, 1024, 1 << 15, 4
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    stream = W.uniform(n_ep * epoch, n_symbols=n_sym, n_accounts=n_acc, seed=43)
    eng = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=epoch,
                                                max_resting=1 << 20, max_accounts=n_acc, max_trades=2 * epoch + 1024))
    eng.process(setup)
    hp = bench.measure_host_path(eng, stream, 0, n_ep, epoch, 2 * epoch + 1024)
    assert hp["value"] > 0 and hp["epochs"] == n_ep
    ref = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=epoch,
                                                max_resting=1 << 20, max_accounts=n_acc, max_trades=2 * epoch + 1024))
    ref.process(setup)
    trades = sum(int(ref.process(stream.slice(k * epoch, (k + 1) * epoch)).status.n_trades) for k in range(n_ep))
    assert hp["trades"] == trades and hp["rows"] == 2 * n_ep * epoch + 2 * trades
