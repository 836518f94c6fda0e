"""Multi-GPU product path, on the one GPU of a test box: the RCCL communicator of
the library ABI (kme_comm_*), the per-epoch market-data all-gather through it, and credit
re-splitting between symbol shards (kme_credit_state / kme_credit_adjust / kme_credit_rebalance).

RCCL refuses two ranks on one device, so the collective runs here as a one-rank communicator (the
full call path: unique id, init, in-place all-gather on the engine stream); the credit re-split is
checked with four shard engines on the same GPU whose (bound, demand) blocks are gathered by a device
copy -- the data kme_credit_rebalance all-gathers over RCCL on a node.
"""
import numpy as np
import pytest

from kme import sharding
from kme import workloads as W

pytestmark = pytest.mark.gpu


def _max_risk(o):
    return np.where(o.action == W.BUY, o.size.astype(np.int64) * o.price,
                    np.where(o.action == W.SELL, o.size.astype(np.int64) * (100 - o.price.astype(np.int64)), 0))


def test_one_rank_communicator_market_data_and_rebalance(kme_mod):
    import torch

    # the RCCL copy bench.py hands the library (torch's own), so one RCCL serves both: chosen explicitly
    # (round-4 verdict: a first-call latch of an env var made the choice depend on test order)
    trccl = kme_mod.torch_rccl_path()
    if trccl:
        kme_mod.rccl_load(trccl)
        kme_mod.rccl_load(trccl)                      # (the same copy again: fine)
        if kme_mod.lib().kme_rccl_load(b"/nonexistent/librccl.so") != 1:   # another copy: KME_E_INVALID
            raise AssertionError("a second RCCL copy must be refused")

    n_sym, n_acc = 64, 128
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    stream = W.uniform(20_000, n_symbols=n_sym, n_accounts=n_acc, seed=5)
    cfg = kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=1 << 15, max_resting=1 << 16,
                                 max_accounts=n_acc)
    eng = kme_mod.Engine(cfg)
    eng.process(setup)
    eng.process(stream)
    comm = eng.comm_init(1, 0, kme_mod.comm_unique_id())
    groups = torch.arange(1, n_sym + 1, dtype=torch.int32, device="cuda")
    rows = n_sym + 7                                  # padded rows: -1 / 0
    allv = torch.zeros((rows, 4), dtype=torch.int32, device="cuda")
    own = torch.zeros((n_sym, 4), dtype=torch.int32, device="cuda")
    # torch fills its tensors on its own stream, the engine writes them on the engine stream: nothing
    # orders the two, so the fills must be done before the engine's kernels are queued
    torch.cuda.synchronize()
    comm.market_data_allgather(groups.data_ptr(), n_sym, rows, allv.data_ptr())
    eng.top_of_book_groups(groups.data_ptr(), n_sym, own.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(allv[:n_sym], own) and (own[:, 0] >= 0).any()
    assert (allv[n_sym:, :2] == -1).all() and (allv[n_sym:, 2:] == 0).all()
    before = torch.zeros(2 * n_acc, dtype=torch.int64, device="cuda")
    after = torch.zeros(2 * n_acc, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()                          # (the fills before the engine writes, as above)
    eng.credit_state(before.data_ptr())
    comm.credit_rebalance()                           # one shard: its own bound back
    eng.credit_state(after.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(before, after) and (before[:n_acc] > 0).all()
    comm.close()


@pytest.mark.parametrize("rebalance", [False, True])
def test_credit_resplit_keeps_every_epoch_parallel(kme_mod, oracle_mod, rebalance):
    """Four symbol shards, every account funded with 1.25x its single-engine need over the whole
    stream (booked as a quarter on each shard).  With the static split some shard's share runs dry
    in the last epochs (KME_E_UNFUNDED); re-splitting the pooled bounds between epochs keeps every
    epoch provable, and the partitions' MatchOut equals the single-engine tape."""
    import torch

    NS, n_sym, n_acc, E, n_ep = 4, 4096, 4096, 1 << 16, 8
    body = W.uniform(NS * E * n_ep, n_symbols=n_sym, n_accounts=n_acc, seed=77)
    need = np.bincount(body.aid, weights=_max_risk(body), minlength=n_acc).astype(np.int64)
    credit = np.floor(need * 1.25).astype(np.int64)
    assert credit.max() < 2**31 - 1
    rows = [(W.CREATE_BALANCE, 0, a, 0, 0, 0) for a in range(n_acc)]
    rows += [(W.TRANSFER, 0, a, 0, 0, int(credit[a])) for a in range(n_acc)]
    rows += [(W.ADD_SYMBOL, 0, 0, s, 0, 0) for s in range(1, n_sym + 1)]
    setup = W.Orders.from_rows(rows)
    router = sharding.PartitionRouter(NS)
    engines = []
    for _ in range(NS):
        cfg = kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=max(2 * E, len(setup)),
                                     max_resting=1 << 21, max_trades=4 * E, max_accounts=n_acc)
        cfg.credit_shards = NS
        engines.append(kme_mod.Engine(cfg))
    state = torch.zeros((NS, 2, n_acc), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()                          # (torch's fill before the engines write)
    chunks, refused = {}, None
    allin = W.Orders.concat([setup, body])
    bounds = [len(setup)] + [len(setup) + (k + 1) * NS * E for k in range(n_ep)]
    starts = [0] + bounds[:-1]
    for ep, (a, b) in enumerate(zip(starts, bounds)):
        parts, echo, seqs = router.route(allin.slice(a, b))
        for k, eng in enumerate(engines):
            try:
                r = eng.process(parts[k])
            except kme_mod.KmeError as e:
                assert kme_mod.STATUS[e.status] == "UNFUNDED"
                refused = ep
                break
            text = sharding.partition_tape(r.tape_json(parts[k]), echo[k])
            chunks.update(zip(seqs[k][echo[k]].tolist(), sharding._chunks(text)))   # (global indices)
        if refused is not None:
            break
        if rebalance and ep > 0:
            for k, eng in enumerate(engines):
                eng.credit_state(state[k].data_ptr())
            torch.cuda.synchronize()
            for k, eng in enumerate(engines):
                eng.credit_adjust(state.data_ptr(), NS, k)
            torch.cuda.synchronize()
            # the re-split keeps the pooled bound of every account
            after = torch.zeros_like(state)
            torch.cuda.synchronize()
            for k, eng in enumerate(engines):
                eng.credit_state(after[k].data_ptr())
            torch.cuda.synchronize()
            assert torch.equal(after[:, 0].sum(0), state[:, 0].sum(0))
    if not rebalance:
        assert refused is not None and refused >= 3, refused    # the static split runs dry late
        return
    assert refused is None
    o = oracle_mod.Oracle()
    o.process(allin)
    assert "".join(chunks[i] for i in range(len(allin))) == o.tape_text()


def test_rebalance_of_a_failed_engine_still_takes_part(kme_mod):
    """Advisor (round 3): kme_credit_rebalance is a collective; a rank whose engine failed must still
    join the all-gather (else its peers wait forever) and every rank must skip the adjust.  One rank
    here: the call returns KME_E_FAILED instead of returning before the collective, and the
    communicator still works afterwards (a market-data all-gather completes)."""
    import torch

    trccl = kme_mod.torch_rccl_path()
    if trccl:
        kme_mod.rccl_load(trccl)
    n_sym, n_acc = 8, 16
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    body = W.uniform(2000, n_symbols=n_sym, n_accounts=n_acc, seed=3)
    cfg = kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=n_sym + 1, max_epoch=1 << 13, max_resting=1 << 14,
                                 max_accounts=n_acc)
    eng = kme_mod.Engine(cfg)
    eng.process(setup)
    eng.process(body)
    comm = eng.comm_init(1, 0, kme_mod.comm_unique_id())
    comm.credit_rebalance()                                       # healthy: OK
    with pytest.raises(kme_mod.KmeError):                        # REMOVE_SYMBOL of a non-empty book: fatal
        eng.process(W.Orders.from_rows([(W.REMOVE_SYMBOL, 0, 0, 3, 0, 0)]))
    with pytest.raises(kme_mod.KmeError) as ke:
        comm.credit_rebalance()
    assert kme_mod.STATUS[ke.value.status] == "FAILED"
    groups = torch.arange(1, n_sym + 1, dtype=torch.int32, device="cuda")
    allv = torch.zeros((n_sym, 4), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    comm.market_data_allgather(groups.data_ptr(), n_sym, n_sym, allv.data_ptr())
    torch.cuda.synchronize()
    comm.close()


def test_credit_state_marks_absent_accounts(kme_mod):
    """Advisor (round 3): an account a shard does not hold reports demand -1, and the re-split gives
    it nothing there: the pooled bound goes to the shards that hold it, none of it is lost."""
    import torch

    n_acc = 8
    cfgs = []
    engines = []
    for k in range(2):
        cfg = kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=5, max_epoch=1 << 10, max_resting=1 << 12,
                                     max_accounts=n_acc)
        cfg.credit_shards = 2
        cfgs.append(cfg)
        engines.append(kme_mod.Engine(cfg))
    # account 3 exists on shard 0 only (its CREATE_BALANCE reached one shard), with 1000 of credit
    rows = [(W.CREATE_BALANCE, 0, a, 0, 0, 0) for a in range(n_acc) if a != 3]
    rows += [(W.TRANSFER, 0, a, 0, 0, 1000) for a in range(n_acc) if a != 3]
    both = W.Orders.from_rows(rows)
    engines[0].process(W.Orders.concat([both, W.Orders.from_rows([(W.CREATE_BALANCE, 0, 3, 0, 0, 0),
                                                                  (W.TRANSFER, 0, 3, 0, 0, 1000)])]))
    engines[1].process(both)
    state = torch.zeros((2, 2, n_acc), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    for k, e in enumerate(engines):
        e.credit_state(state[k].data_ptr())
    torch.cuda.synchronize()
    assert int(state[1, 1, 3]) == -1 and int(state[1, 0, 3]) == 0
    assert int(state[0, 1, 3]) == 0 and int(state[0, 0, 3]) == 500            # floor(1000 / 2) booked
    pooled = state[:, 0].sum(0).clone()
    for k, e in enumerate(engines):
        e.credit_adjust(state.data_ptr(), 2, k)
    after = torch.zeros_like(state)
    torch.cuda.synchronize()
    for k, e in enumerate(engines):
        e.credit_state(after[k].data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(after[:, 0].sum(0), pooled)                          # nothing leaves the pool
    assert int(after[0, 0, 3]) == 500 and int(after[1, 0, 3]) == 0
    for e in engines:
        e.close()
