"""Two device epochs in flight (kme.h: kme_submit_epoch_device may be called again before kme_wait;
kme_wait takes the older epoch), with caller-owned result buffers per epoch -- the bench's timed loop
and host path.  The tapes of every epoch, the books afterwards, and the refusals (a third submit,
checkpoint or host submit while epochs are in flight) are checked; FUNDED, both matchers."""
import numpy as np
import pytest

import kme
from kme import workloads as W

pytestmark = pytest.mark.gpu


def _dev_out(torch, dev, E, cap):
    return {"out_action": torch.empty(E, dtype=torch.int32, device=dev),
            "out_size": torch.empty(E, dtype=torch.int32, device=dev),
            "out_prev": torch.empty(E, dtype=torch.int64, device=dev),
            "out_flags": torch.empty(E, dtype=torch.uint8, device=dev),
            "trade_off": torch.empty(E + 1, dtype=torch.int32, device=dev),
            "trades": torch.empty(4 * cap, dtype=torch.int64, device=dev)}


def _result(out, n, st):
    nt = int(st.n_trades)
    trades = np.frombuffer(out["trades"][:4 * nt].cpu().numpy().tobytes(), dtype=kme.TRADE_DTYPE)
    return kme.EpochResult(out["out_action"][:n].cpu().numpy(), out["out_size"][:n].cpu().numpy(),
                           out["out_prev"][:n].cpu().numpy(), out["out_flags"][:n].cpu().numpy(),
                           out["trade_off"][:n + 1].cpu().numpy().astype(np.uint32), trades, st)


@pytest.mark.parametrize("light_max", [0, -1])
def test_two_epochs_in_flight(oracle_mod, tmp_path, light_max):
    import torch

    dev = torch.device("cuda", 0)
    n_sym, n_acc, E, epochs = 512, 256, 1 << 14, 6
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    stream = W.uniform(E * epochs, n_symbols=n_sym, n_accounts=n_acc, seed=21)
    cfg = kme.default_config(kme.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=E, max_resting=1 << 17,
                             max_accounts=n_acc, light_max=light_max, max_trades=4 * E)
    eng = kme.Engine(cfg)
    eng.process(setup)
    cols = {c: torch.from_numpy(np.ascontiguousarray(getattr(stream, c))).to(dev)
            for c in ("action", "oid", "aid", "sid", "price", "size")}

    def ptrs(k):
        return {c: t.data_ptr() + k * E * t.element_size() for c, t in cols.items()}

    outs = [_dev_out(torch, dev, E, 4 * E) for _ in range(2)]

    def out_ptrs(b):
        p = {k: t.data_ptr() for k, t in outs[b].items()}
        p["trades_cap"] = 4 * E
        return p

    o = oracle_mod.Oracle()
    o.process(setup)
    o.clear_tape()
    eng.submit_device(ptrs(0), E, out=out_ptrs(0))
    for k in range(epochs):
        if k + 1 < epochs:
            eng.submit_device(ptrs(k + 1), E, out=out_ptrs((k + 1) % 2))
            if k == 0:
                with pytest.raises(kme.KmeError):                       # a third epoch in flight
                    eng.submit_device(ptrs(k + 1), E)
                with pytest.raises(kme.KmeError):                       # checkpoint between epochs only
                    eng.checkpoint(tmp_path / "x.ckpt")
        st = eng.wait()
        assert st.status == 0 and st.n_inputs == E
        part = stream.slice(k * E, (k + 1) * E)
        got = _result(outs[k % 2], E, st).tape_json(part)
        o.process(part)
        assert got == o.tape_text(), f"epoch {k}"
        o.clear_tape()
    assert eng.snapshot_books() == o.dump_books()


@pytest.mark.parametrize("light_max", [0, -1])
def test_device_epoch_with_account_records(oracle_mod, light_max):
    """A device epoch is not split at account records (kme_submit_epoch splits host epochs): orders
    of an account created earlier in the same epoch pass the balance gate (KP:170), orders before
    its CREATE_BALANCE do not -- k_emap routes the orders against the accounts as they stood, k_route
    redoes acct_ok after k_ledger_funded.  Zero-risk orders (BUY at 0, SELL at 100, size 0) keep the
    epoch inside the funded proof."""
    import torch

    dev = torch.device("cuda", 0)
    B, S, C = W.BUY, W.SELL, W.CANCEL
    setup = W.funded_setup(8, range(1, 5))
    rows = [(B, 100, 50, 2, 0, 5),           # account 50 not created yet: REJECT
            (100, 0, 50, 0, 0, 0),           # CREATE_BALANCE 50
            (B, 101, 50, 2, 0, 5),           # risk 0: accepted, rests at 0
            (S, 102, 50, 3, 100, 7),         # risk 0: accepted, rests at 100
            (B, 103, 1, 2, 40, 3),           # a funded account's order
            (C, 101, 50, 0, 0, 0),           # cancel of the order of the new account
            (100, 0, 51, 0, 0, 0), (S, 104, 51, 3, 100, 0), (B, 105, 51, 3, 0, 2)]
    part = W.Orders.from_rows(rows)
    E = 64
    cfg = kme.default_config(kme.MODE_FUNDED, max_symbols=8, max_epoch=E, max_resting=1 << 12,
                             max_accounts=64, light_max=light_max, max_trades=4 * E)
    eng = kme.Engine(cfg)
    eng.process(setup)
    cols = {c: torch.from_numpy(np.ascontiguousarray(getattr(part, c))).to(dev)
            for c in ("action", "oid", "aid", "sid", "price", "size")}
    out = _dev_out(torch, dev, E, 4 * E)
    ptrs = {c: t.data_ptr() for c, t in cols.items()}
    optrs = {k: t.data_ptr() for k, t in out.items()}
    optrs["trades_cap"] = 4 * E
    eng.submit_device(ptrs, len(part), out=optrs)
    st = eng.wait()
    assert st.status == 0
    o = oracle_mod.Oracle()
    o.process(setup)
    o.clear_tape()
    o.process(part)
    assert _result(out, len(part), st).tape_json(part) == o.tape_text()
    assert eng.snapshot_books() == o.dump_books()
