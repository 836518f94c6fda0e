"""The multi-GPU glue of bench.py on CPU (gloo, world size 2): the murmur2 symbol partition of the
65,536-symbol C3 universe, disjoint oids and credit shards per rank, the per-epoch market-data
all-gather and its check, the MAX / SUM / MIN reductions of the bench line, and the self-launch
of N ranks by ``bench.py --gpus N`` (the reference is one partition,
topic.js:17-18, exchange_test.js:14-16).  The GPU ranks run the same functions over RCCL.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from kme import workloads as W


def test_partition_of_the_c3_universe():
    for world in (1, 2, 8):
        parts = [bench.rank_symbols("c3", world, r) for r in range(world)]
        allsid = np.sort(np.concatenate(parts))
        assert (allsid == np.arange(1, 65537)).all()          # a partition of the universe
        for r, p in enumerate(parts[:2]):
            for s in p[:50].tolist():
                assert W.shard_of(s, world) == r               # Kafka's keyed partitioner
    rows, per_rank = bench.market_data_layout(8, "c3")
    assert rows == max(len(p) for p in per_rank) and 7000 < rows < 9000


def test_rank_workload_stays_in_its_partition():
    world = 4
    seen = []
    for r in range(world):
        setup, stream, sids, nacc, shards, _ = bench.make_workload("c3", 20_000, r, world)
        assert shards == world and nacc == 65536
        bs = np.isin(stream.action, (W.BUY, W.SELL))
        assert np.isin(stream.sid[bs], sids).all()
        added = setup.sid[setup.action == W.ADD_SYMBOL]
        assert (np.sort(added) == sids).all()
        # each account's credit is split over the shards: N x the single-engine transfers
        assert np.count_nonzero(setup.action == W.TRANSFER) == nacc * W.funded_transfers_needed(20_000, nacc) * world
        seen.append(stream.oid[bs])
    allo = np.concatenate(seen)
    assert len(np.unique(allo)) == len(allo)                   # oids unique across the ranks


def test_n1_stream_is_the_round1_c3_stream():
    _, stream, sids, _, shards, _ = bench.make_workload("c3", 50_000, 0, 1)
    ref = W.uniform(50_000, n_symbols=65536, n_accounts=65536, seed=1000)
    assert shards == 1 and len(sids) == 65536
    for k in ("action", "oid", "aid", "sid", "price", "size"):
        assert (getattr(stream, k) == getattr(ref, k)).all(), k


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows, per_rank = bench.market_data_layout(world, "c3")
        sids = per_rank[rank]
        tob = torch.full((rows, 4), -1, dtype=torch.int32)
        tob[:len(sids), 0] = torch.from_numpy((sids % 100).astype(np.int32))
        tob[:len(sids), 1] = rank
        tob_all = torch.zeros((world * rows, 4), dtype=torch.int32)
        bench.exchange_market_data(dist, tob, tob_all)
        ok = bench.verify_market_data(tob_all, tob, rank, rows)
        # rank 0 sees every rank's block: the union snapshot of all 65,536 symbols
        union = {}
        for r in range(world):
            blk = tob_all[r * rows:(r + 1) * rows]
            for j, s in enumerate(per_rank[r].tolist()):
                union[s] = (int(blk[j, 0]), int(blk[j, 1]))
        union_ok = len(union) == 65536 and all(v == (s % 100, bench_rank) for s, v in union.items()
                                               for bench_rank in [W.shard_of(s, world)])
        el, no, nt, md = bench.reduce_stats(dist, torch, 1.0 + rank, 10 * (rank + 1), 3 * (rank + 1), ok, "cpu")
        # a rank whose check fails makes the whole job's flag fail
        _, _, _, md_bad = bench.reduce_stats(dist, torch, 0.0, 0, 0, rank == 0, "cpu")
        q.put((rank, ok, union_ok, el, no, nt, md, md_bad))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gloo_world2_market_data_and_reductions():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = sorted(q.get(timeout=5) for _ in range(2))
    for rank, ok, union_ok, el, no, nt, md, md_bad in res:
        assert ok and union_ok
        assert el == 2.0 and no == 30.0 and nt == 9.0 and md is True and md_bad is False


def test_self_launch_starts_n_ranks(monkeypatch):
    calls = []
    monkeypatch.setattr(subprocess, "call", lambda cmd, env=None: calls.append((cmd, env)) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    with pytest.raises(SystemExit) as ei:
        bench.main()
    assert ei.value.code == 0
    cmd, env = calls[0]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "2"] and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_launcher_world_must_match_gpus(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(SystemExit) as ei:
        bench.main()
    assert "--gpus 2" in str(ei.value.code)


def test_c4_shard_workload_is_its_partition():
    """bench.py --workload c4 --shard R/N: rank R's records of the N-GPU C4 run (its murmur2 share of the
    65,536 symbols, Zipf popularity of the whole universe), funded for N credit shards."""
    world = 8
    for r in (0, 5):
        setup, stream, sids, nacc, shards, _ = bench.make_workload("c4", 20_000, r, world)
        assert shards == world and len(sids) == len(W.shard_symbols(65536, world, r))
        bs = np.isin(stream.action, (W.BUY, W.SELL))
        assert np.isin(stream.sid[bs], sids).all()


def test_router_rate_is_timed_by_the_c_harness():
    """bench.py's `router` field: kme_router_rate_run (integration/host_harness.c) routes and splits
    epochs of the bench stream in C and reports the best epoch of each (host CPU only)."""
    st = W.uniform(4 * (1 << 14), n_symbols=65536, n_accounts=65536, seed=1)
    r = bench.measure_router(st, 1 << 14)
    assert r["route_records_per_s"] > 1e5 and r["split_records_per_s"] > 1e5
    assert r["partitions"] == 8 and 0 < r["directory"] <= 4 * (1 << 14)
