"""Symbol sharding: N engines, each on the records `kme.sharding.split` routes to it,
merged back by input sequence, must print the single engine's MatchOut stream and hold, together,
its book stores.

CPU: the shards are oracle instances -- in-process, and as a world_size-2 `gloo` job exchanging
their tapes with all_gather_object.  GPU: two HIP engines with `credit_shards=2`.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import hazards
from kme import sharding
from kme import workloads as W


def _funded_stream(n_sym=24, n_acc=64, n=6000, seed=11, kind="uniform"):
    if kind == "uniform":
        body = W.uniform(n, n_symbols=n_sym, n_accounts=n_acc, seed=seed)
        k = 1
    else:
        body = W.cancel_replace(n, n_symbols=n_sym, n_accounts=n_acc, seed=seed)
        k = W.funded_transfers_needed(len(body), n_acc, big=True)
    # credit split over up to 3 shards: fund 3x what one engine needs
    return W.Orders.concat([W.funded_setup(n_acc, range(1, n_sym + 1), transfers_per_account=3 * k), body])


def _single(oracle_mod, orders):
    o = oracle_mod.Oracle()
    o.process(orders)
    return o.tape_text(), o.dump_books()


def _sharded(oracle_mod, orders, n):
    routes, _, parts = sharding.split(orders, n)
    tapes, books = [], []
    for p in parts:
        o = oracle_mod.Oracle()
        o.process(p)
        tapes.append(o.tape_text())
        books.append(o.dump_books())
    return sharding.merge_tapes(routes, tapes), sharding.merge_books(books)


def test_route_follows_kafka_keyed_partitioner():
    o = W.uniform(2000, n_symbols=50, seed=3)
    r = sharding.route(o, 4)
    buy = np.flatnonzero(np.isin(o.action, (W.BUY, W.SELL)))
    for i in buy[:200]:
        assert r[i] == W.shard_of(abs(int(o.sid[i])), 4)
    assert (r[o.action == W.CANCEL] == sharding.BROADCAST).all()
    assert (sharding.route(o, 1)[np.isin(o.action, (W.BUY, W.SELL))] == 0).all()


@pytest.mark.parametrize("n", [2, 3, 5])
@pytest.mark.parametrize("kind", ["uniform", "cancel_replace"])
def test_sharded_oracle_equals_single(oracle_mod, n, kind):
    orders = _funded_stream(kind=kind)
    want_tape, want_books = _single(oracle_mod, orders)
    got_tape, got_books = _sharded(oracle_mod, orders, n)
    assert got_tape == want_tape
    assert got_books == want_books


def test_sharded_funded_hazards(oracle_mod):
    """sid 0 (one shared book, H4), negative sids (books +g/-g live on one shard), zero-size
    trades (H3): all stay within one shard."""
    for name, rows in hazards.streams().items():
        if name not in hazards.FUNDED_OK:
            continue
        orders = hazards.as_orders(rows)
        assert _sharded(oracle_mod, orders, 2) == _single(oracle_mod, orders), name


def test_merge_detects_duplicate_live_oid_across_shards(oracle_mod):
    # the same oid resting on two symbols of different shards is outside the parity domain
    # (KP:221): a broadcast cancel is then accepted twice
    n = 2
    a, b = 1, 2
    while W.shard_of(b, n) == W.shard_of(a, n):
        b += 1
    rows = [(W.CREATE_BALANCE, 0, 7, 0, 0, 0), (W.TRANSFER, 0, 7, 0, 0, 10**6),
            (W.ADD_SYMBOL, 0, 0, a, 0, 0), (W.ADD_SYMBOL, 0, 0, b, 0, 0),
            (W.BUY, 99, 7, a, 10, 1), (W.BUY, 99, 7, b, 10, 1), (W.CANCEL, 99, 7, 0, 0, 0)]
    orders = W.Orders.from_rows(rows)
    routes, _, parts = sharding.split(orders, n)
    tapes = []
    for p in parts:
        o = oracle_mod.Oracle()
        o.process(p)
        tapes.append(o.tape_text())
    with pytest.raises(sharding.ShardConflict):
        sharding.merge_tapes(routes, tapes)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_rank(rank, world, port, kind, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle

        orders = _funded_stream(kind=kind)
        routes, _, parts = sharding.split(orders, world)
        o = oracle.Oracle()
        o.process(parts[rank])
        mine = (o.tape_text(), o.dump_books())
        allv = [None] * world
        dist.all_gather_object(allv, mine)
        if rank == 0:
            tape = sharding.merge_tapes(routes, [t for t, _ in allv])
            books = sharding.merge_books([b for _, b in allv])
            ref = oracle.Oracle()
            ref.process(orders)
            q.put((tape == ref.tape_text(), books == ref.dump_books(), len(tape)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["uniform", "cancel_replace"])
def test_gloo_world2_shards_merge_to_single_engine(oracle_mod, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_rank, args=(r, 2, port, kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    tape_ok, books_ok, n = q.get(timeout=5)
    assert n > 0 and tape_ok and books_ok


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["uniform", "cancel_replace"])
def test_gpu_two_engines_credit_split(kme_mod, oracle_mod, kind):
    orders = _funded_stream(kind=kind, n=20_000)
    routes, _, parts = sharding.split(orders, 2)
    tapes, books = [], []
    for p in parts:
        cfg = kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=32, max_epoch=1 << 12,
                                     max_resting=1 << 16, max_accounts=64)
        cfg.credit_shards = 2
        eng = kme_mod.Engine(cfg)
        t = []
        for a in range(0, len(p), 1 << 12):
            part = p.slice(a, min(len(p), a + (1 << 12)))
            t.append(eng.process(part).tape_json(part))
        tapes.append("".join(t))
        books.append(eng.snapshot_books())
        eng.close()
    want_tape, want_books = _single(oracle_mod, orders)
    assert sharding.merge_tapes(routes, tapes) == want_tape
    assert sharding.merge_books(books) == want_books


@pytest.mark.gpu
def test_gpu_credit_split_is_enforced(kme_mod):
    """Credit 1000 over 2 shards: a BUY of risk 600 cannot be proven on one shard (500 each)."""
    rows = [(W.CREATE_BALANCE, 0, 3, 0, 0, 0), (W.TRANSFER, 0, 3, 0, 0, 1000), (W.ADD_SYMBOL, 0, 0, 1, 0, 0)]
    buy = [(W.BUY, 77, 3, 1, 10, 60)]
    for shards, ok in ((1, True), (2, False)):
        cfg = kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=4, max_epoch=64, max_resting=256,
                                     max_accounts=8)
        cfg.credit_shards = shards
        eng = kme_mod.Engine(cfg)
        eng.process(W.Orders.from_rows(rows))
        if ok:
            eng.process(W.Orders.from_rows(buy))
        else:
            with pytest.raises(kme_mod.KmeError) as ei:
                eng.process(W.Orders.from_rows(buy))
            assert kme_mod.STATUS[ei.value.status] == "UNFUNDED"
        eng.close()


# ----------------------------------------------------------------------------- partitioned topics
def _partitioned(oracle_mod, orders, n, epochs=3):
    """Row f next-4: each record answered by one partition; the partitions' chunks, put back in
    input order, are the single engine's MatchOut stream."""
    router = sharding.PartitionRouter(n)
    engines = [oracle_mod.Oracle() for _ in range(n)]
    chunks = {}
    books = None
    step = (len(orders) + epochs - 1) // epochs
    for a in range(0, len(orders), step):
        parts, echo, seqs = router.route(orders.slice(a, min(len(orders), a + step)))
        for k in range(n):
            engines[k].process(parts[k])
            text = sharding.partition_tape(engines[k].tape_text(), echo[k])
            engines[k].clear_tape()
            mine = sharding._chunks(text)
            s = seqs[k][echo[k]]
            assert len(mine) == len(s)
            for q, c in zip(s.tolist(), mine):
                assert q not in chunks, f"record {q} answered twice"
                chunks[q] = c
    books = sharding.merge_books([e.dump_books() for e in engines])
    return "".join(chunks[q] for q in range(len(orders))), books


@pytest.mark.parametrize("n", [2, 4])
@pytest.mark.parametrize("kind", ["uniform", "cancel_replace"])
def test_partitioned_topics_need_no_merge(oracle_mod, n, kind):
    orders = _funded_stream(kind=kind, n=5000)
    want_tape, want_books = _single(oracle_mod, orders)
    got_tape, got_books = _partitioned(oracle_mod, orders, n)
    assert got_tape == want_tape
    assert got_books == want_books


def test_partition_router_sends_cancels_to_the_oid_owner():
    orders = W.uniform(3000, n_symbols=40, n_accounts=32, seed=5)
    router = sharding.PartitionRouter(3)
    parts, echo, seqs = router.route(orders)
    owner = {}
    for k in range(3):
        for i, q in enumerate(seqs[k].tolist()):
            if parts[k].action[i] in (W.BUY, W.SELL):
                owner[int(parts[k].oid[i])] = k
    for k in range(3):
        for i in range(len(parts[k])):
            if parts[k].action[i] == W.CANCEL and int(parts[k].oid[i]) in owner:
                assert owner[int(parts[k].oid[i])] == k
    # every record is echoed by exactly one partition
    counts = np.zeros(len(orders), int)
    for k in range(3):
        counts[seqs[k][echo[k]]] += 1
    assert (counts == 1).all()


def _gloo_partition_rank(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle

        orders = _funded_stream(kind="cancel_replace", n=4000)
        router = sharding.PartitionRouter(world)   # every rank routes the same stream identically
        parts, echo, seqs = router.route(orders)
        o = oracle.Oracle()
        o.process(parts[rank])
        text = sharding.partition_tape(o.tape_text(), echo[rank])   # this rank's MatchOut partition
        mine = (seqs[rank][echo[rank]].tolist(), sharding._chunks(text), o.dump_books())
        allv = [None] * world
        dist.all_gather_object(allv, mine)   # only to check: the partitions need no merge
        if rank == 0:
            chunks = {}
            for s, c, _ in allv:
                chunks.update(zip(s, c))
            ref = oracle.Oracle()
            ref.process(orders)
            tape = "".join(chunks[i] for i in range(len(orders)))
            books = sharding.merge_books([b for _, _, b in allv])
            q.put((tape == ref.tape_text(), books == ref.dump_books(), len(chunks) == len(orders)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gloo_world2_partitioned_topics():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_partition_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert all(q.get(timeout=5))


@pytest.mark.gpu
def test_gpu_partitioned_engines(kme_mod, oracle_mod):
    orders = _funded_stream(kind="cancel_replace", n=20_000)
    router = sharding.PartitionRouter(2)
    engines = []
    for _ in range(2):
        cfg = kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=32, max_epoch=1 << 12,
                                     max_resting=1 << 16, max_accounts=64)
        cfg.credit_shards = 2
        engines.append(kme_mod.Engine(cfg))
    chunks = {}
    for a in range(0, len(orders), 1 << 12):
        parts, echo, seqs = router.route(orders.slice(a, min(len(orders), a + (1 << 12))))
        for k, eng in enumerate(engines):
            text = sharding.partition_tape(eng.process(parts[k]).tape_json(parts[k]), echo[k])
            chunks.update(zip(seqs[k][echo[k]].tolist(), sharding._chunks(text)))
    want_tape, want_books = _single(oracle_mod, orders)
    assert "".join(chunks[i] for i in range(len(orders))) == want_tape
    assert sharding.merge_books([e.snapshot_books() for e in engines]) == want_books
