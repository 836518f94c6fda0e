#!/usr/bin/env python3
"""Benchmark of the matching hot path (BASELINE.json metric) on 1..N MI355X GPUs.

One step = one epoch of E input records through the whole device pipeline (oid map, funded-ledger
proof, cancel routing, radix partition by symbol group, per-group matching, trade compaction,
oid-table upkeep, top-of-book snapshot; + the RCCL all-gather of the snapshots when N > 1).
Inputs are resident in HBM before the timed region; outputs stay in HBM.

Default workload: the metric's own configuration, C3 (BASELINE.json configs[2]):
one universe of 65,536 symbols keyed over the N ranks by Kafka's partitioner (murmur2 of the
decimal sid, ``kme_shard_of``), so rank r matches the records of its own ~65,536 / N
symbols -- N = 8 is exactly C3.  65,536 accounts, each funded on every rank with 1/N of its credit
(``credit_shards``).  Every rank processes E = 2^22 records per step (per-GPU work per step is
fixed: "weak" scaling in records).  No collective in the data path; the ranks' top-of-book
snapshots (16 B per symbol, their own symbols only) are all-gathered over RCCL every epoch and
checked against each rank's own snapshot after the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--epoch E] [--workload c3|c2|c4|c5]

``--gpus N`` > 1 outside a torch.distributed launcher starts the N ranks itself (torchrun as a
child process; this parent never touches the GPU) and exits with their status.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kafka-matching-engine_amd"))

from kme import workloads as W  # noqa: E402  (numpy only: no HIP runtime is loaded here)

METRIC = "matched orders/sec (node) at 65,536 symbols; p99 epoch latency; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
C3_SYMBOLS, C3_ACCOUNTS = 65536, 65536  # BASELINE configs[2] / SURVEY §8d C3


def algorithmic_bytes(st) -> int:
    """SURVEY.md §8d byte model per epoch: 52 B per input record (36 B of Order information + 16 B
    of result), 36 B per trade, 32 B per resting-order write, 32 B per maker node visited, 48 B per
    successful cancel."""
    return (52 * st.n_inputs + 36 * st.n_trades + 32 * st.n_rests + 32 * st.n_maker_visits
            + 48 * st.n_cancel_ok)


def rank_symbols(name: str, world: int, rank: int, symbols: int = 0) -> np.ndarray:
    """The symbol ids rank `rank` owns: for the 65,536-symbol configurations (c3, c4) its murmur2
    partition of the universe; c2 / c5 (and the --symbols diagnostic) are per-GPU configurations
    of their own symbols 1..n."""
    if name in ("c3", "c4") and not symbols:
        return W.shard_symbols(C3_SYMBOLS, world, rank)
    n = symbols or 1024
    return np.arange(1, n + 1, dtype=np.int64)


def make_workload(name: str, n_orders: int, rank: int, world: int, symbols: int = 0, mix=None):
    """(setup, stream, sids, accounts, description) of rank `rank`: its records of the configuration."""
    seed = 1000 + rank
    mix = tuple(mix) if mix else (0.34, 0.33, 0.33)
    sids = rank_symbols(name, world, rank, symbols)
    oid_base = 1 + rank * n_orders   # disjoint oid ranges: every oid is unique across the ranks
    keyed = name in ("c3", "c4") and not symbols
    shards = world if keyed else 1
    if name == "c2":
        nacc = 4096
        stream = W.uniform(n_orders, n_accounts=nacc, seed=seed, mix=mix, symbols=sids, oid_base=oid_base)
        desc = "C2: 1,024 symbols x 16M uniform limit/cancel orders per GPU (BASELINE configs[1])"
    elif name == "c3":
        nacc = C3_ACCOUNTS
        stream = W.uniform(n_orders, n_accounts=nacc, seed=seed, mix=mix, symbols=sids, oid_base=oid_base)
        desc = (f"C3: 65,536 symbols keyed (murmur2) over {world} GPU(s), {len(sids):,} symbols on rank {rank}, "
                f"uniform limit/cancel orders (BASELINE configs[2])" if keyed else
                f"C3 diagnostic: {len(sids):,} symbols per GPU, uniform limit/cancel orders")
    elif name == "c4":
        nacc = C3_ACCOUNTS
        stream = W.zipf(n_orders, n_symbols=C3_SYMBOLS, n_accounts=nacc, seed=seed, oid_base=oid_base,
                        shard=(rank, world))
        desc = f"C4: Zipf(1.1) symbol popularity over 65,536 symbols keyed over {world} GPU(s), 21-level band"
    elif name == "c5":
        nacc = 4096
        stream = W.cancel_replace(n_orders, n_symbols=len(sids), n_accounts=nacc, seed=seed, oid_base=oid_base)
        desc = "C5: 90% cancel/replace + 10% sweeping orders of 5k-50k, 1,024 symbols per GPU"
    else:
        raise SystemExit(f"unknown workload {name}")
    need = W.funded_transfers_needed(n_orders, nacc, big=name == "c5")
    setup = W.funded_setup(nacc, sids, transfers_per_account=need * shards)
    return setup, stream, sids, nacc, shards, desc


def parse_flags(text: str) -> int:
    """--flags exact_ledger,serial_fallback -> kme_config.flags (include/kme.h KME_FLAG_*)."""
    names = {"exact_ledger": 1, "serial_fallback": 2}
    flags = 0
    for f in filter(None, (x.strip() for x in text.split(","))):
        if f not in names:
            raise SystemExit(f"bench.py: unknown flag {f!r} (known: {', '.join(names)})")
        flags |= names[f]
    if flags & 2:
        flags |= 1   # the serial fallback runs on the exact ledger
    return flags


def pmc_for_build(path: str, build_id: str):
    """(traffic, derived) of the committed PMC summary, only when it was collected on the library
    this process loaded (its `build_id` = kme_build_id()); (None, None) otherwise, so the line never
    carries counters of code that is not the code measured."""
    if not os.path.exists(path):
        return None, None, "no PMC summary committed for this configuration"
    with open(path) as f:
        pj = json.load(f)
    if pj.get("build_id") != build_id:
        return None, None, f"PMC summary of build {pj.get('build_id')}, not of the loaded build {build_id}"
    return pj.get("hbm_bytes_per_launch"), pj.get("per_kernel_derived"), pj.get("source")


def cpu_baseline(setup, stream, max_orders: int):
    """The oracle (CPU restatement of KProcessor.MatchingEngine, single thread) on a bounded
    prefix of the same stream.  The reference itself (Java/Kafka Streams) cannot run here."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    o = oracle.Oracle(keep_tape=False)
    o.process(setup)
    m = min(len(stream), max_orders)
    part = stream.slice(0, m)
    t0 = time.perf_counter()
    o.process(part)
    dt = time.perf_counter() - t0
    n = part.n_orders()
    return {"value": n / dt, "unit": "orders/s", "cores": 1, "kind": "port",
            "sample": f"first {m:,} records ({n:,} BUY/SELL/CANCEL) of the same stream after setup, "
                      f"C restatement of KProcessor.MatchingEngine with hash-map stores, {dt:.1f} s"}


def _free_port() -> int:
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def self_launch(gpus: int) -> int:
    """--gpus N > 1 without a launcher: the N ranks as a torchrun child process.  Called before
    anything initialises HIP (no torch.cuda call, libkme not loaded), so nothing here is replaced
    by exec; the parent only waits and returns the ranks' exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # RCCL over dmabuf IPC on this host driver
    return subprocess.call(cmd, env=env)


def market_data_layout(world: int, name: str, symbols: int = 0):
    """(rows per rank in the all-gathered snapshot, symbols of each rank): every rank pads its
    snapshot to the largest partition so the all-gather is one equal-sized block per rank."""
    per_rank = [rank_symbols(name, world, r, symbols) for r in range(world)]
    return max(len(p) for p in per_rank), per_rank


def exchange_market_data(dist, tob_local, tob_all):
    """The per-epoch market-data collective: every rank's top-of-book rows -> every rank (RCCL
    over xGMI on the GPU ranks; gloo in the CPU tests of this glue and in the one-GPU rehearsal,
    where device tensors go through host copies)."""
    if tob_local.is_cuda and dist.get_backend() == "gloo":
        host = tob_all.cpu()
        dist.all_gather_into_tensor(host, tob_local.cpu())
        tob_all.copy_(host)
        return
    dist.all_gather_into_tensor(tob_all, tob_local)


def library_comm(dist, torch, kme, eng, world: int, rank: int, dev):
    """The library's own RCCL communicator over the ranks' engines (kme_comm_init; the unique id
    made on rank 0 and broadcast over torch.distributed), for kme_market_data_allgather.  None when it
    cannot be made (RCCL not loadable by the library): the bench then all-gathers through torch's
    RCCL and says so in its line."""
    # one RCCL for both: the library dlopens the copy torch's own collectives already use
    trccl = kme.torch_rccl_path()
    try:
        kme.rccl_load(trccl)
    except kme.KmeError as ex:   # noqa: BLE001 (reported; the all-gather falls back to torch's)
        print(f"rank {rank}: {ex}", file=sys.stderr, flush=True)
    uid = torch.zeros(128, dtype=torch.uint8, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    if rank == 0:
        try:
            uid.copy_(torch.frombuffer(bytearray(kme.comm_unique_id()), dtype=torch.uint8))
        except Exception as ex:   # noqa: BLE001 (the fallback is reported)
            print(f"kme_comm_unique_id: {ex}", file=sys.stderr, flush=True)
            err.fill_(1)
    dist.broadcast(err, 0)
    if int(err.item()):
        return None
    dist.broadcast(uid, 0)
    try:
        return eng.comm_init(world, rank, bytes(uid.cpu().numpy().tobytes()))
    except Exception as ex:   # noqa: BLE001
        print(f"rank {rank}: kme_comm_init: {ex}", file=sys.stderr, flush=True)
        return None


def verify_market_data(tob_all, tob_local, rank: int, rows: int) -> bool:
    """After the all-gather, block `rank` of every rank's copy is this rank's own snapshot."""
    return bool((tob_all[rank * rows:(rank + 1) * rows] == tob_local).all().item())


def reduce_stats(dist, torch, elapsed: float, n_orders: int, n_trades: int, ok: bool, device):
    """Whole-job figures: the slowest rank's time (MAX) and the records / trades of all ranks (SUM),
    the market-data check of every rank (MIN)."""
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    sums = torch.tensor([float(n_orders), float(n_trades)], dtype=torch.float64, device=device)
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        if dist.get_backend() == "gloo":
            t, sums, flag = t.cpu(), sums.cpu(), flag.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return float(t.item()), float(sums[0].item()), float(sums[1].item()), bool(flag.item())


def measure_router(stream, E, n_epochs=4, parts=8):
    """The partition router that splits one MatchIn stream over N GPUs (kme_router.cpp, the front of
    kme_multi), timed by the committed C harness (integration/host_harness.c kme_router_rate_run):
    epochs of this stream into 8 partitions, alternately route and split, best epoch of each.
    Host-only work on this box's CPU threads (KME_ROUTER_THREADS, default min(16, cores))."""
    import ctypes as C

    import kme

    lib = C.CDLL(os.path.join(ROOT, "integration", "libkme_host_harness.so"))
    lib.kme_router_rate_run.argtypes = [C.POINTER(kme.kme_orders), C.c_uint32, C.c_uint32, C.c_uint32,
                                        C.POINTER(C.c_double)]
    lib.kme_router_rate_run.restype = C.c_int
    n_epochs = min(n_epochs, len(stream) // E)
    if n_epochs < 2:
        return None
    n_rec = n_epochs * E
    cols = {c: np.ascontiguousarray(getattr(stream, c)[:n_rec]) for c in ("action", "oid", "aid", "sid", "price", "size")}
    ko = kme.kme_orders(*[C.c_void_p(cols[c].ctypes.data) for c in ("action", "oid", "aid", "sid", "price", "size")])
    stats = (C.c_double * 3)()
    rc = lib.kme_router_rate_run(C.byref(ko), E, n_epochs, parts, stats)
    if rc:
        raise kme.KmeError(rc, "kme_router_rate_run")
    return {"route_records_per_s": stats[0], "split_records_per_s": stats[1], "partitions": parts,
            "epoch_records": E, "directory": int(stats[2]),
            "threads": int(os.environ.get("KME_ROUTER_THREADS", 0)) or min(16, os.cpu_count() or 1),
            "path": "integration/host_harness.c kme_router_rate_run: kme_router_route / kme_router_split, C-timed"}


def measure_host_path(eng, stream, first, n_epochs, E, max_trades):
    """The Java processor's path at rate, timed by the committed C harness
    (integration/host_harness.c): GpuMatchingEngine.java's schedule -- records written into two
    slots of registered host columns, kme_submit_epoch_host (H2D, kernels, D2H queued), kme_wait +
    kme_expand_rows into the slot's row buffer and a pass over the rows -- over exactly the C ABI
    calls kme_jni.c makes.  PCIe- and host-inclusive: a secondary field, never the headline value."""
    import ctypes as C

    import kme

    lib = C.CDLL(os.path.join(ROOT, "integration", "libkme_host_harness.so"))
    lib.kme_host_path_run.argtypes = [C.c_void_p, C.POINTER(kme.kme_orders), C.c_uint32, C.c_uint32, C.c_uint32,
                                      C.POINTER(C.c_double)]
    lib.kme_host_path_run.restype = C.c_int
    a0, n_rec = first * E, n_epochs * E
    cols = {c: np.ascontiguousarray(getattr(stream, c)[a0:a0 + n_rec]) for c in ("action", "oid", "aid", "sid", "price", "size")}
    ko = kme.kme_orders(*[C.c_void_p(cols[c].ctypes.data) for c in ("action", "oid", "aid", "sid", "price", "size")])
    stats = (C.c_double * 8)()
    rc = lib.kme_host_path_run(eng.handle, C.byref(ko), E, n_epochs, max_trades, stats)
    if rc:
        raise kme.KmeError(rc, "kme_host_path_run")
    dt = stats[0]
    h2d_b = 36 * E
    d2h_b = 21 * E + 4 + 32 * (stats[5] / n_epochs)
    return {"value": n_rec / dt, "unit": "records/s", "epochs": n_epochs, "epoch_records": E,
            "rows": int(stats[1]), "trades": int(stats[5]), "rows_per_s": stats[1] / dt, "h2d_bytes_per_epoch": h2d_b, "d2h_bytes_per_epoch": int(d2h_b),
            "pcie_GBps_each_way": round(max(h2d_b, d2h_b) * n_epochs / dt / 1e9, 2),
            "host_s": {"fill": round(stats[2], 4), "wait": round(stats[3], 4), "rows": round(stats[4], 4),
                       "rows_expand": round(stats[7], 4), "rows_read": round(stats[4] - stats[7], 4), "total": round(dt, 4)},
            "path": "integration/host_harness.c: GpuMatchingEngine.java's schedule over kme_jni.c's C ABI calls "
                    "(registered host columns -> kme_submit_epoch_host -> kme_wait + kme_expand_rows -> rows read), "
                    "two epochs in flight; PCIe- and host-inclusive, not the headline value"}


def measure_checkpoint(kme, eng, cfg, directory, next_epoch=None):
    """The commit point's cost at this shape: kme_checkpoint_app of the engine's
    state (format 4: the live stores, a tree digest trailer; fsync'd and renamed), the state changelog's
    chunk hashes, and its restore into a fresh engine of the same configuration; both books must then
    agree.  With next_epoch: one more epoch, a second commit, and how many of its 512-KiB chunks
    changed -- what the state changelog carries for a commit one epoch after the last."""
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, "bench.ckpt")
    t0 = time.perf_counter()
    eng.checkpoint_app(path, b"offset")
    t1 = time.perf_counter()
    info = kme.checkpoint_inspect(path)
    # the state changelog's unit: the file's 512-KiB chunks hashed (the processor puts the changed ones
    # into its changelogged commit store)
    tc0 = time.perf_counter()
    chunks = kme.checkpoint_chunks(path, 512 << 10)
    tc1 = time.perf_counter()
    other = kme.Engine(cfg)
    t2 = time.perf_counter()
    assert other.restore_app(path) == b"offset"
    t3 = time.perf_counter()
    same = other.snapshot_books() == eng.snapshot_books()
    if cfg.flags & 1:
        same = same and other.snapshot_ledger() == eng.snapshot_ledger()
    other.close()
    os.remove(path)
    delta = None
    if next_epoch is not None:
        before = set(enumerate(chunks.tolist()))
        next_epoch()
        path2 = os.path.join(directory, "bench2.ckpt")
        t4 = time.perf_counter()
        eng.checkpoint_app(path2, b"offset")
        t5 = time.perf_counter()
        chunks2 = kme.checkpoint_chunks(path2, 512 << 10)
        changed = sum(1 for kc in enumerate(chunks2.tolist()) if kc not in before)
        delta = {"write_ms": (t5 - t4) * 1e3, "chunks": len(chunks2), "chunks_changed": changed,
                 "changed_bytes": changed * (512 << 10)}
        os.remove(path2)
    return {"file_bytes": info["file_bytes"], "write_ms": (t1 - t0) * 1e3, "restore_ms": (t3 - t2) * 1e3,
            "chunks": len(chunks), "chunk_hash_ms": (tc1 - tc0) * 1e3, "after_one_more_epoch": delta,
            "restored_state_equal": same,
            "path": "kme_checkpoint_app (device compaction, D2H, digest, fsync, rename) / kme_restore_app into a new engine"}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--epoch", type=int, default=1 << 22)
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--symbols", type=int, default=0, help="diagnostic: symbols per GPU for c3 (default: the murmur2 partition of 65,536)")
    ap.add_argument("--shard", default="", help="diagnostic: R/N, the records of rank R of an N-GPU run (c3, c4) on this one GPU")
    ap.add_argument("--mix", default="", help="diagnostic: BUY,SELL,CANCEL fractions of the c2/c3 stream")
    ap.add_argument("--orders", type=int, default=16_000_000, help="stream length per GPU (>= (W+K)*E)")
    ap.add_argument("--max-resting", type=int, default=0,
                    help="diagnostic: resting-order capacity (default: the whole stream, every order could rest)")
    ap.add_argument("--light-max", type=int, default=0,
                    help="diagnostic: kme_config.light_max (0 = default 128 records per group and epoch)")
    ap.add_argument("--cpu-sample", type=int, default=10_000_000)
    ap.add_argument("--pipeline", action="store_true",
                    help="queue epoch k+1 before waiting for epoch k (+1.3% orders/s measured, p99 epoch "
                         "latency 1.9 -> 3.7 ms: an epoch then waits behind the previous one)")
    ap.add_argument("--host-path-epochs", type=int, default=-1,
                    help="N = 1: epochs of the host-buffer path (pinned H2D + kernels + D2H, pipelined) "
                         "measured after the device-resident ones (0 = skip; default: 3, or 2^24 records' "
                         "worth of smaller epochs)")
    ap.add_argument("--java-defaults", action="store_true",
                    help="the engine configuration of GpuMatchingEngine() (integration/jni): 65,536-record epochs, "
                         "max_trades 2^18, 65,537 symbols, 2^20 accounts, 2^26 resting orders, exact ledger + serial "
                         "fallback, initial ledger capacity 2^20")
    ap.add_argument("--checkpoint", default="",
                    help="directory: after the timed epochs, time a commit point's checkpoint (kme_checkpoint_app) "
                         "of the engine and its restore into a fresh engine; the line gets bytes and ms")
    ap.add_argument("--flags", default="",
                    help="kme_config.flags, comma-separated: exact_ledger, serial_fallback (the drop-in's own "
                         "configuration, GpuMatchingEngine.java: exact_ledger,serial_fallback; N = 1 only)")
    ap.add_argument("--ledger-capacity", type=int, default=0,
                    help="with --flags exact_ledger: Balances / Positions capacity (0 = sized for the stream)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stamps", action="store_true", help="diagnostic: print k_match cycle shares and exit")
    ap.add_argument("--lane-stamps", action="store_true", help="diagnostic: print k_match_lanes step-segment shares and exit")
    ap.add_argument("--serialize", action="store_true",
                    help="also print each epoch's MatchOut tape on the GPU (kme_tape_json_device) inside the step")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if args.stamps:  # diagnostic build with in-kernel s_memtime stamps (never the bench line)
        os.environ["KME_LIB"] = os.path.join(ROOT, "kafka-matching-engine_amd", "kme", "libkme_stamps.so")
    if args.lane_stamps:
        os.environ.setdefault("KME_LIB", os.path.join(ROOT, "kafka-matching-engine_amd", "kme", "libkme_lstamps.so"))

    import torch
    import torch.distributed as dist

    import kme

    # KME_BENCH_REHEARSAL=1 (diagnostic, never a bench line): every rank on GPU 0 with gloo
    # collectives, to rehearse the N-rank path on a one-GPU box
    rehearsal = os.environ.get("KME_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local_rank = 0
    if world > 1:
        torch.cuda.set_device(local_rank)
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        assert dist.get_world_size() == args.gpus
    dev = torch.device("cuda", local_rank)

    if args.java_defaults:
        # GpuMatchingEngine()'s configuration and schedule: two epochs in flight (its two slots)
        args.epoch, args.flags, args.pipeline = 1 << 16, "exact_ledger,serial_fallback", True
    E = args.epoch
    if args.host_path_epochs < 0:
        args.host_path_epochs = max(3, (1 << 24) // E)
    host_epochs = args.host_path_epochs if world == 1 else 0
    if os.environ.get("KME_LIB") and host_epochs:
        # integration/libkme_host_harness.so is linked against the tree's libkme.so: with another build
        # loaded as the engine (KME_LIB, A/B runs) it would drive that engine through a library of
        # another kme_engine layout -- a device fault, not a measurement.  No host path then.
        print("bench.py: KME_LIB set: no host-path / router measurement (the harness links the tree's libkme.so)",
              file=sys.stderr, flush=True)
        host_epochs = 0
    # + 1: the phase-breakdown epoch; then the host-path epochs
    # (+ 1 with --checkpoint: the epoch between its two commits)
    total = max(args.orders, (args.warmup + args.steps + 1 + host_epochs + (1 if args.checkpoint else 0)) * E)
    # --shard R/N (one GPU): the records rank R of an N-GPU run would match, e.g. C4's hot shard
    w_rank, w_world = (rank, world) if not args.shard else tuple(int(x) for x in args.shard.split("/"))
    if args.shard and world > 1:
        raise SystemExit("bench.py: --shard is a one-GPU diagnostic")
    setup, stream, sids, nacc, shards, desc = make_workload(
        args.workload, total, w_rank, w_world, args.symbols, [float(x) for x in args.mix.split(",")] if args.mix else None)
    if args.shard:
        desc += f" -- shard {w_rank} of {w_world} on one GPU"
    max_sid = int(sids.max())
    flags = parse_flags(args.flags)
    if flags and world > 1:
        raise SystemExit("bench.py: --flags exact_ledger needs one engine (the exact ledger couples every symbol)")

    cfg = kme.default_config(kme.MODE_FUNDED, max_symbols=max_sid + 1, max_epoch=E,
                             max_resting=args.max_resting or min(total, (1 << 29) - 64 * (max_sid + 2) - E), max_trades=2 * E + (1 << 16),
                             max_accounts=nacc, device=local_rank, light_max=args.light_max)
    cfg.credit_shards = shards
    cfg.flags = flags
    if flags:   # the tables' initial size (they grow between epochs: kme_ledger_stats)
        cfg.ledger_capacity = args.ledger_capacity or (1 << 20)
    if args.java_defaults:   # GpuMatchingEngine() (integration/jni/GpuMatchingEngine.java)
        cfg.max_trades, cfg.max_symbols, cfg.max_accounts, cfg.max_resting = 1 << 18, 65537, 1 << 20, 1 << 26
        cfg.ledger_capacity = 1 << 20
        if max_sid + 1 > cfg.max_symbols or nacc > cfg.max_accounts:
            raise SystemExit("bench.py --java-defaults: the workload exceeds GpuMatchingEngine()'s configuration")
    eng = kme.Engine(cfg)
    # one explicit stream for the engine and every torch / collective op of this rank, so they are
    # ordered (the default stream's handle is 0, which would leave the engine on its own
    # non-blocking stream, unordered with the all-gather's reads of the snapshot)
    work = torch.cuda.Stream(dev)
    torch.cuda.set_stream(work)
    assert work.cuda_stream != 0
    eng.set_stream(work.cuda_stream)
    eng.enable_timing("match")   # timed epochs: events around the matching kernels only
    eng.process(setup)  # CREATE_BALANCE / TRANSFER / ADD_SYMBOL records (host path)

    # inputs resident in HBM before timing
    cols = {
        "action": torch.from_numpy(stream.action).to(dev), "oid": torch.from_numpy(stream.oid).to(dev),
        "aid": torch.from_numpy(stream.aid).to(dev), "sid": torch.from_numpy(stream.sid).to(dev),
        "price": torch.from_numpy(stream.price).to(dev), "size": torch.from_numpy(stream.size).to(dev),
    }
    orders_per_epoch = [int(stream.slice(k * E, (k + 1) * E).n_orders()) for k in range(args.warmup + args.steps + 1)]
    cancels_timed = int(np.count_nonzero(stream.action[args.warmup * E:(args.warmup + args.steps) * E] == W.CANCEL))
    # market data: this rank's symbols' top of book, all-gathered (16 B per symbol)
    rows, per_rank = market_data_layout(world, args.workload, args.symbols)
    groups = torch.from_numpy(sids.astype(np.int32)).to(dev)
    tobs = [torch.full((rows, 4), -1, dtype=torch.int32, device=dev) for _ in range(2)]
    tob = tobs[0]
    tob_all = torch.zeros((world * rows, 4), dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)   # torch's fills before the engine's (non-blocking) stream writes them
    # N > 1 on GPU ranks: the market data goes through the library's ABI entry (its own RCCL
    # communicator, kme_market_data_allgather on the engine stream); torch's RCCL all-gather only if
    # that communicator cannot be made, and in the gloo rehearsal
    comm = library_comm(dist, torch, kme, eng, world, rank, dev) if world > 1 and not rehearsal else None
    if world > 1 and not rehearsal:
        ok = torch.tensor([1 if comm is not None else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if not int(ok.item()) and comm is not None:
            comm.close()
            comm = None

    def epoch_ptrs(k):
        return {name: t.data_ptr() + k * E * t.element_size() for name, t in cols.items()}

    tape_buf = torch.empty(args.serialize * (512 * E + (1 << 20)), dtype=torch.uint8, device=dev)
    tape_bytes = []

    def submit_epoch(k):
        """Queue epoch k and its market-data snapshot (double-buffered: the next epoch may be queued
        before this one is waited for)."""
        nonlocal tob, comm
        tob = tobs[k % 2]
        eng.submit_device(epoch_ptrs(k), E)
        if comm is not None:   # own rows into this rank's block, all-gathered in place over xGMI
            try:
                comm.market_data_allgather(groups.data_ptr(), len(sids), rows, tob_all.data_ptr())
                tob = tob_all[rank * rows:(rank + 1) * rows]
                return
            except kme.KmeError as ex:   # (reported in the line: the collective falls back to torch's)
                print(f"rank {rank}: kme_market_data_allgather: {ex}; torch.distributed from here on",
                      file=sys.stderr, flush=True)
                comm = None
        eng.top_of_book_groups(groups.data_ptr(), len(sids), tob.data_ptr())
        if world > 1:
            exchange_market_data(dist, tob, tob_all)   # market-data snapshot over RCCL / xGMI

    def run_epoch(k):
        submit_epoch(k)
        st = eng.wait()
        if args.serialize:  # MatchOut text of the epoch, printed on the GPU, left in HBM
            tape_bytes.append(eng.tape_json_device_into(epoch_ptrs(k), E, tape_buf.data_ptr(), tape_buf.numel()))
        return st

    for k in range(args.warmup):
        run_epoch(k)

    lat, match_ms, bytes_alg, n_orders, n_trades = [], [], [], 0, 0
    mix = {"inputs": 0, "trades": 0, "rests": 0, "maker_visits": 0, "cancels_ok": 0}
    ledger = {"epochs_parallel": 0, "epochs_serial_replay": 0, "chains_repaired": 0, "epochs_serial_fallback": 0}
    # --pipeline: two epochs in flight (kme.h), epoch k + 1 queued before epoch k is waited for, so
    # the GPU never idles on the host's turnaround between epochs (--serialize reads the
    # engine-owned results of each epoch, so it runs them one at a time)
    pipelined = args.pipeline and not args.serialize
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    t_sub = {}
    sub_cpu = []   # the host's time inside each submit call (launches), beside the epoch's wall time
    wait_cpu = []  # ... and blocked in each wait (~0: the host, not the device, paces the epochs)
    for j in range(args.steps):
        k = args.warmup + j
        if pipelined:
            if j == 0:
                t_sub[k] = time.perf_counter()
                submit_epoch(k)
                sub_cpu.append(time.perf_counter() - t_sub[k])
            if j + 1 < args.steps:
                t_sub[k + 1] = time.perf_counter()
                submit_epoch(k + 1)
                sub_cpu.append(time.perf_counter() - t_sub[k + 1])
            t_w = time.perf_counter()
            st = eng.wait()
            wait_cpu.append(time.perf_counter() - t_w)
        else:
            t_sub[k] = time.perf_counter()
            submit_epoch(k)
            sub_cpu.append(time.perf_counter() - t_sub[k])
            t_w = time.perf_counter()
            st = eng.wait()
            wait_cpu.append(time.perf_counter() - t_w)
            if args.serialize:  # MatchOut text of the epoch, printed on the GPU, left in HBM
                tape_bytes.append(eng.tape_json_device_into(epoch_ptrs(k), E, tape_buf.data_ptr(), tape_buf.numel()))
        lat.append((time.perf_counter() - t_sub[k]) * 1e3)   # submit -> results ready
        ph = eng.phase_times()
        match_ms.append(ph["match"])
        bytes_alg.append(algorithmic_bytes(st))
        n_orders += int(st.n_orders)
        n_trades += int(st.n_trades)
        for name, v in (("inputs", st.n_inputs), ("trades", st.n_trades), ("rests", st.n_rests),
                     ("maker_visits", st.n_maker_visits), ("cancels_ok", st.n_cancel_ok)):
            mix[name] += int(v)
        if flags & 1:   # the exact ledger: which pass kept each epoch's Balances / Positions
            ledger["epochs_serial_fallback"] += int(st.serial_fallback != 0)
            ledger["epochs_serial_replay"] += int(st.ledger_serial != 0)
            ledger["epochs_parallel"] += int(st.serial_fallback == 0 and st.ledger_serial == 0)
            ledger["chains_repaired"] += int(st.ledger_repaired)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    assert n_orders == sum(orders_per_epoch[args.warmup:args.warmup + args.steps]), "device order count mismatch"
    # the phase breakdown, from one more epoch with every phase's events (outside the timed region:
    # the events serialise the stream)
    eng.enable_timing("all")
    run_epoch(args.warmup + args.steps)
    phases_all = eng.phase_times()
    eng.enable_timing(False)

    # market data check (outside the timed region): this rank's rows of the full-range snapshot,
    # its own compact snapshot, and its block of the all-gathered one agree
    full = torch.zeros((max_sid + 1, 4), dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    eng.top_of_book(full.data_ptr())
    torch.cuda.synchronize(dev)
    md_local = bool((full[groups.long()] == tob[:len(sids)]).all().item()) and bool((tob[:len(sids), 0] >= 0).any().item())
    md_gather = verify_market_data(tob_all, tob, rank, rows) if world > 1 else True
    if comm is not None:   # the library's all-gather against torch's, on the last snapshot
        ref = torch.zeros_like(tob_all)
        exchange_market_data(dist, tob_all[rank * rows:(rank + 1) * rows].contiguous(), ref)
        torch.cuda.synchronize(dev)
        md_gather = md_gather and bool(torch.equal(ref, tob_all))
    md_ok = md_local and md_gather
    if not md_ok:
        print(f"rank {rank}: market data check failed (own snapshot vs full-range: {md_local}, "
              f"all-gathered block: {md_gather})", file=sys.stderr, flush=True)
    # the host-buffer path (after the market-data check: its epochs move the books on)
    host_path = measure_host_path(eng, stream, args.warmup + args.steps + 1, host_epochs, E, cfg.max_trades) \
        if host_epochs else None
    router = measure_router(stream, E) if world == 1 and host_epochs else None   # (host CPU only)
    ckpt = measure_checkpoint(kme, eng, cfg, args.checkpoint,
                              lambda: eng.submit_device(epoch_ptrs(args.warmup + args.steps + 1 + host_epochs), E) or eng.wait()) \
        if args.checkpoint and world == 1 else None
    ledger_tables = eng.ledger_stats() if flags & 1 else None

    if args.lane_stamps:  # -DKME_LANE_STAMPS build: k_match_lanes wavefront steps (kme_kernels.hip LST)
        d = eng.debug_counters().astype(np.float64).reshape(-1)[:12]
        names = ["drain", "gather1", "gather2", "record", "out", "record.try_match", "record.rest"]
        tot = d[:5].sum()
        print(json.dumps({"lane_stamps": {"share": {n: d[q] / tot for q, n in enumerate(names)},
                                          "cycles_per_step": {n: d[q] / max(1, d[7]) for q, n in enumerate(names)},
                                          "sweep": {"steps_with_extra_maker_load": d[8] / max(1, d[7]),
                                                    "extra_loads_per_lane_step": d[9] / max(1, d[7]) / 32,
                                                    "max_extra_loads_per_step": d[10] / max(1, d[7])},
                                          "steps": d[7], "ms_per_epoch_match": float(np.mean(match_ms))}}), flush=True)
        return
    if args.stamps:  # -DKME_STAMPS build: cycle shares of k_match (kme_kernels.hip enum Stamp)
        rows_ = eng.debug_counters().astype(np.float64).reshape(-1, 48)
        hot = int(np.argmax(rows_[:, 7]))   # the group with the most k_match cycles (C4: the hot symbol)
        d = rows_[hot] if os.environ.get("KME_STAMPS_HOT") else rows_.sum(axis=0)
        names = ["group_in", "batch", "trade_rec", "rest_rec", "cancel_rec", "other_rec", "group_out", "kernel",
                 "n_trade_rec", "n_rest_rec", "n_cancel_rec", "maker_wait", "n_maker", "victim_wait", "n_victim",
                 "flush", "rest_alloc", "rest_level", "rest_node", "rec_pick", "rec_out", "tm_pre_norest", "rest_pre",
                 "fast", "n_fast_rec", "n_fast_seg", "fast_pass", "fast_drain", "fast_level", "fast_epi",
                 "pass_rest", "n_pass_rest", "pass_sweep", "n_pass_sweep", "pass_cancel", "n_pass_cancel",
                 "pass_reject", "n_pass_reject", "pass_absorb", "n_pass_absorb"]
        v = dict(zip(names, d))
        per = {"share_of_kernel": {n: v[n] / v["kernel"] for n in ("group_in", "batch", "trade_rec", "rest_rec",
                                                                     "cancel_rec", "other_rec", "group_out", "flush")},
               "cycles_per_trade_rec": v["trade_rec"] / max(1, v["n_trade_rec"]),
               "cycles_per_rest_rec": v["rest_rec"] / max(1, v["n_rest_rec"]),
               "cycles_per_cancel_rec": v["cancel_rec"] / max(1, v["n_cancel_rec"]),
               "maker_wait_per_load": v["maker_wait"] / max(1, v["n_maker"]),
               "makers_per_trade_rec": v["n_maker"] / max(1, v["n_trade_rec"]),
               "victim_wait_per_load": v["victim_wait"] / max(1, v["n_victim"]),
               "victim_loads_per_cancel": v["n_victim"] / max(1, v["n_cancel_rec"]),
               "rest_parts_per_rest": {n: v[n] / max(1, v["n_rest_rec"]) for n in ("rest_alloc", "rest_level", "rest_node", "tm_pre_norest")},
               "rec_pick_per_rec": v["rec_pick"] / max(1, v["n_trade_rec"] + v["n_rest_rec"] + v["n_cancel_rec"]),
               "rec_total_per_rec": v["rec_out"] / max(1, v["n_trade_rec"] + v["n_rest_rec"] + v["n_cancel_rec"]),
               "counts": {n: v[n] for n in ("n_trade_rec", "n_rest_rec", "n_cancel_rec", "n_maker", "n_victim")},
               "fast": {"records": v["n_fast_rec"], "segments": v["n_fast_seg"],
                        "share_of_kernel": v["fast"] / v["kernel"],
                        "cycles_per_fast_rec": v["fast"] / max(1, v["n_fast_rec"]),
                        "pass_cycles_per_fast_rec": v["fast_pass"] / max(1, v["n_fast_rec"]),
                        "drain_cycles_per_fast_rec": v["fast_drain"] / max(1, v["n_fast_rec"]),
                        "level_cycles_per_fast_rec": v["fast_level"] / max(1, v["n_fast_rec"]),
                        "epilogue_cycles_per_fast_rec": v["fast_epi"] / max(1, v["n_fast_rec"]),
                        "records_per_segment": v["n_fast_rec"] / max(1, v["n_fast_seg"]),
                        "pass_by_kind": {k: {"records": v["n_pass_" + k], "cycles_per_rec": v["pass_" + k] / max(1, v["n_pass_" + k])}
                                         for k in ("rest", "absorb", "sweep", "cancel", "reject")}}}
        per["group"] = hot if os.environ.get("KME_STAMPS_HOT") else "all"
        print(json.dumps({"stamps": per}), flush=True)
        return
    elapsed, n_orders_all, n_trades_all, md_all = reduce_stats(dist if world > 1 else None, torch, elapsed,
                                                              n_orders, n_trades, md_ok, dev)

    if rank == 0:
        avg_match_s = float(np.mean(match_ms)) / 1e3
        achieved = float(np.mean(bytes_alg)) / avg_match_s / 1e9 if avg_match_s > 0 else 0.0
        build_id = kme.lib().kme_build_id().decode()
        traffic, pmc_derived, pmc_src = None, None, "PMC passes cover the default single-GPU configurations only"
        pmc = os.path.join(ROOT, "profiles", f"pmc_k_match_{args.workload}.json")
        # the committed PMC pass is of the default single-GPU configuration only (tools/gpu_round4.sh),
        # and counts only when it profiled this very build
        if world == 1 and not args.symbols and not args.mix and not args.shard and E == (1 << 22) and not flags:
            traffic, pmc_derived, pmc_src = pmc_for_build(pmc, build_id)
        out = {
            "metric": METRIC,
            "value": n_orders_all / elapsed,
            "unit": "orders/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            "config": {"workload": desc, "symbols_per_gpu_rank0": int(len(sids)), "accounts": nacc, "epoch_records": E,
                       "stream_records_per_gpu": total,
                       "mode": "FUNDED (symbol groups in parallel)" + (" + exact ledger" if flags & 1 else "")
                               + (" + serial fallback" if flags & 2 else ""),
                       "parallelism": f"symbol-keyed x{world} (murmur2, Kafka's keyed partitioner)",
                       "credit_shards": shards, "flags": args.flags or "none",
                       "engine": "GpuMatchingEngine() defaults" if args.java_defaults else "bench",
                       "epochs_in_flight": 2 if pipelined else 1},
            "build_id": build_id,
            "p99_epoch_ms": float(np.percentile(lat, 99)),
            "p50_epoch_ms": float(np.percentile(lat, 50)),
            "host_submit_ms": float(np.mean(sub_cpu) * 1e3),   # the host's time in each submit (kernel launches)
            "host_wait_ms": float(np.mean(wait_cpu) * 1e3),    # ... and blocked in each wait
            "fills_per_s": 2 * n_trades_all / elapsed,
            "trades_per_s": n_trades_all / elapsed,
            "market_data": {"symbols": int(sum(len(p) for p in per_rank)), "bytes_per_epoch": int(world * rows * 16),
                            "collective": ("gloo all_gather (one-GPU rehearsal)" if rehearsal else
                                           "kme_market_data_allgather (libkme's RCCL communicator) per epoch" if comm is not None
                                           else "torch.distributed RCCL all_gather_into_tensor per epoch (libkme communicator unavailable)")
                            if world > 1 else "none (N = 1)",
                            "verified": md_all},
            "phase_ms_last_epoch": {k: round(v, 4) for k, v in phases_all.items()},   # (the epoch after the timed ones)
            "host_path": host_path,
            "router": router,
            "exact_ledger": dict(ledger, tables=ledger_tables) if flags & 1 else None,
            "checkpoint": ckpt,
            "match_ms_per_step": [round(v, 3) for v in match_ms],
            "events_per_epoch_rank0": {k: v / args.steps for k, v in mix.items()},
            # cancels that removed a resting order (KP:289-323) / cancels in the timed epochs
            "cancel_success_rank0": mix["cancels_ok"] / max(1, cancels_timed),
            "roofline": {"kernel": "k_match_lanes+k_match (match phase: light groups one lane each, heavy groups "
                                   "one wavefront each, concurrent)", "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "bytes_model": "SURVEY §8d: 52/in + 36/trade + 32/rest + 32/maker visit + 48/cancel",
                         "avg_launch_ms": avg_match_s * 1e3, "alg_bytes_per_launch": float(np.mean(bytes_alg)),
                         "traffic_source": pmc_src},
            # occupancy and LDS bank conflicts of the match-phase kernels, from the committed rocprofv3
            # PMC passes of this configuration (tools/pmc_kmatch.sh, tools/pmc_summary.py)
            "pmc_match_phase": pmc_derived,
        }
        if args.serialize:
            out["serialize"] = {"tape_bytes_per_epoch": float(np.mean(tape_bytes[-args.steps:])),
                                "note": "step includes kme_tape_json_device (MatchOut text in HBM)"}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(setup, stream, args.cpu_sample)
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    eng.close()
    if world > 1:
        dist.destroy_process_group()
    if not md_all:
        raise SystemExit("bench.py: the all-gathered market data does not match the ranks' own snapshots")


if __name__ == "__main__":
    main()
