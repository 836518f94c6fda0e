#!/usr/bin/env python3
"""Benchmark of the matching hot path (BASELINE.json metric) on 1..N MI355X GPUs.

One step = one epoch of E input records through the whole device pipeline (oid map, funded-ledger
proof, cancel routing, radix partition by symbol group, per-group matching, trade compaction,
oid-table upkeep, top-of-book snapshot; + an RCCL all-gather of top-of-book when N > 1).
Inputs are resident in HBM before the timed region; outputs stay in HBM.

Default workload: the metric's own configuration, C3 (BASELINE.json configs[2]):
65,536 symbols symbol-sharded over the N ranks (65,536 / N symbols per GPU, so every N measures the
same 65,536-symbol universe and N = 8 is exactly C3), 65,536 accounts, uniform limit / cancel
orders; every rank processes its own stream, E = 2^22 records per epoch and step (per-GPU work per
step is fixed: "weak" in records).  No collective in the data path; the top-of-book snapshot is
all-gathered over RCCL per epoch.  --workload c2 runs configs[1] (1,024 symbols per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--epoch E] [--workload c3|c2|c4|c5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kafka-matching-engine_amd"))

if "--stamps" in sys.argv:  # diagnostic build with in-kernel s_memtime stamps (never the bench line)
    os.environ["KME_LIB"] = os.path.join(ROOT, "kafka-matching-engine_amd", "kme", "libkme_stamps.so")

import torch  # noqa: E402  (first: one HIP runtime per process, see kme.lib)
import torch.distributed as dist  # noqa: E402

import kme  # noqa: E402
from kme import workloads as W  # noqa: E402

METRIC = "matched orders/sec (node) at 65,536 symbols; p99 epoch latency; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
C3_SYMBOLS, C3_ACCOUNTS = 65536, 65536  # BASELINE configs[2] / SURVEY §8d C3


def algorithmic_bytes(st) -> int:
    """SURVEY.md §8d byte model per epoch: 52 B per input record (36 B of Order information + 16 B
    of result), 36 B per trade, 32 B per resting-order write, 32 B per maker node visited, 48 B per
    successful cancel."""
    return (52 * st.n_inputs + 36 * st.n_trades + 32 * st.n_rests + 32 * st.n_maker_visits
            + 48 * st.n_cancel_ok)


def make_workload(name: str, n_orders: int, rank: int, world: int, symbols: int = 0, mix=None):
    seed = 1000 + rank
    mix = tuple(mix) if mix else (0.34, 0.33, 0.33)
    if name == "c2":
        nsym, nacc = 1024, 4096
        stream = W.uniform(n_orders, n_symbols=nsym, n_accounts=nacc, seed=seed, mix=mix)
        desc = "C2: 1,024 symbols x 16M uniform limit/cancel orders per GPU (BASELINE configs[1])"
    elif name == "c3":
        nsym, nacc = (symbols or C3_SYMBOLS // world), C3_ACCOUNTS
        stream = W.uniform(n_orders, n_symbols=nsym, n_accounts=nacc, seed=seed, mix=mix)
        desc = (f"C3: 65,536 symbols symbol-sharded over {world} GPU(s) = {nsym:,} symbols per GPU, "
                f"uniform limit/cancel orders (BASELINE configs[2])")
    elif name == "c4":
        nsym, nacc = C3_SYMBOLS // world, C3_ACCOUNTS
        stream = W.zipf(n_orders, n_symbols=nsym, n_accounts=nacc, seed=seed)
        desc = f"C4: Zipf(1.1) symbol popularity, 65,536 symbols over {world} GPU(s), 21-level band"
    elif name == "c5":
        nsym, nacc = 1024, 4096
        stream = W.cancel_replace(n_orders, n_symbols=nsym, n_accounts=nacc, seed=seed)
        desc = "C5: 90% cancel/replace + 10% sweeping orders of 5k-50k, 1,024 symbols per GPU"
    else:
        raise SystemExit(f"unknown workload {name}")
    setup = W.funded_setup(nacc, range(1, nsym + 1),
                           transfers_per_account=W.funded_transfers_needed(n_orders, nacc, big=name == "c5"))
    return setup, stream, nsym, nacc, desc


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--epoch", type=int, default=1 << 22)
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--symbols", type=int, default=0, help="diagnostic: symbols per GPU for c3 (default 65,536 / N)")
    ap.add_argument("--mix", default="", help="diagnostic: BUY,SELL,CANCEL fractions of the c2/c3 stream")
    ap.add_argument("--orders", type=int, default=16_000_000, help="stream length per GPU (>= (W+K)*E)")
    ap.add_argument("--max-resting", type=int, default=0,
                    help="diagnostic: resting-order capacity (default: the whole stream, every order could rest)")
    ap.add_argument("--light-max", type=int, default=0,
                    help="diagnostic: kme_config.light_max (0 = default 128 records per group and epoch)")
    ap.add_argument("--cpu-sample", type=int, default=10_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stamps", action="store_true", help="diagnostic: print k_match cycle shares and exit")
    ap.add_argument("--serialize", action="store_true",
                    help="also print each epoch's MatchOut tape on the GPU (kme_tape_json_device) inside the step")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)

    E = args.epoch
    total = max(args.orders, (args.warmup + args.steps) * E)
    setup, stream, nsym, nacc, desc = make_workload(args.workload, total, rank, world, args.symbols,
                                                   [float(x) for x in args.mix.split(",")] if args.mix else None)

    cfg = kme.default_config(kme.MODE_FUNDED, max_symbols=nsym + 1, max_epoch=E,
                             max_resting=args.max_resting or min(total, 1 << 30), max_trades=2 * E + (1 << 16),
                             max_accounts=nacc, device=local_rank, light_max=args.light_max)
    eng = kme.Engine(cfg)
    stream_handle = torch.cuda.current_stream(dev).cuda_stream
    eng.set_stream(stream_handle)
    eng.enable_timing(True)
    eng.process(setup)  # CREATE_BALANCE / TRANSFER / ADD_SYMBOL records (host path)

    # inputs resident in HBM before timing
    cols = {
        "action": torch.from_numpy(stream.action).to(dev), "oid": torch.from_numpy(stream.oid).to(dev),
        "aid": torch.from_numpy(stream.aid).to(dev), "sid": torch.from_numpy(stream.sid).to(dev),
        "price": torch.from_numpy(stream.price).to(dev), "size": torch.from_numpy(stream.size).to(dev),
    }
    orders_per_epoch = [int(stream.slice(k * E, (k + 1) * E).n_orders()) for k in range(args.warmup + args.steps)]
    tob = torch.zeros((nsym + 1, 4), dtype=torch.int32, device=dev)
    tob_all = torch.zeros((world * (nsym + 1), 4), dtype=torch.int32, device=dev) if world > 1 else None

    def epoch_ptrs(k):
        return {name: t.data_ptr() + k * E * t.element_size() for name, t in cols.items()}

    tape_buf = torch.empty(args.serialize * (512 * E + (1 << 20)), dtype=torch.uint8, device=dev)
    tape_bytes = []

    def run_epoch(k):
        eng.submit_device(epoch_ptrs(k), E)
        eng.top_of_book(tob.data_ptr())
        if world > 1:
            dist.all_gather_into_tensor(tob_all, tob)  # market-data snapshot over RCCL / xGMI
        st = eng.wait()
        if args.serialize:  # MatchOut text of the epoch, printed on the GPU, left in HBM
            tape_bytes.append(eng.tape_json_device_into(epoch_ptrs(k), E, tape_buf.data_ptr(), tape_buf.numel()))
        return st

    for k in range(args.warmup):
        run_epoch(k)

    lat, match_ms, bytes_alg, n_orders, n_trades = [], [], [], 0, 0
    mix = {"inputs": 0, "trades": 0, "rests": 0, "maker_visits": 0, "cancels_ok": 0}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for j in range(args.steps):
        k = args.warmup + j
        e0 = time.perf_counter()
        st = run_epoch(k)
        lat.append((time.perf_counter() - e0) * 1e3)
        ph = eng.phase_times()
        match_ms.append(ph["match"])
        bytes_alg.append(algorithmic_bytes(st))
        n_orders += int(st.n_orders)
        n_trades += int(st.n_trades)
        for name, v in (("inputs", st.n_inputs), ("trades", st.n_trades), ("rests", st.n_rests),
                     ("maker_visits", st.n_maker_visits), ("cancels_ok", st.n_cancel_ok)):
            mix[name] += int(v)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    assert n_orders == sum(orders_per_epoch[args.warmup:]), "device order count mismatch"

    if args.stamps:  # -DKME_STAMPS build: cycle shares of k_match (kme_kernels.hip enum Stamp)
        rows = eng.debug_counters().astype(np.float64).reshape(-1, 32)
        hot = int(np.argmax(rows[:, 7]))   # the group with the most k_match cycles (C4: the hot symbol)
        d = rows[hot] if os.environ.get("KME_STAMPS_HOT") else rows.sum(axis=0)
        names = ["group_in", "batch", "trade_rec", "rest_rec", "cancel_rec", "other_rec", "group_out", "kernel",
                 "n_trade_rec", "n_rest_rec", "n_cancel_rec", "maker_wait", "n_maker", "victim_wait", "n_victim",
                 "flush", "rest_alloc", "rest_level", "rest_node", "rec_pick", "rec_out", "tm_pre_norest", "rest_pre"]
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
               "counts": {n: v[n] for n in ("n_trade_rec", "n_rest_rec", "n_cancel_rec", "n_maker", "n_victim")}}
        per["group"] = hot if os.environ.get("KME_STAMPS_HOT") else "all"
        print(json.dumps({"stamps": per}), flush=True)
        return
    stats = torch.tensor([elapsed, float(n_orders), float(n_trades)], dtype=torch.float64, device=dev)
    if world > 1:
        t_max = stats[0:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        sums = stats[1:].clone()
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
        elapsed, n_orders_all, n_trades_all = float(t_max.item()), float(sums[0].item()), float(sums[1].item())
    else:
        n_orders_all, n_trades_all = float(n_orders), float(n_trades)

    if rank == 0:
        avg_match_s = float(np.mean(match_ms)) / 1e3
        achieved = float(np.mean(bytes_alg)) / avg_match_s / 1e9 if avg_match_s > 0 else 0.0
        traffic, pmc_derived = None, None
        pmc = os.path.join(ROOT, "profiles", f"pmc_k_match_{args.workload}.json")
        # the committed PMC pass is of the default single-GPU configuration only (tools/gpu_round.sh)
        if os.path.exists(pmc) and world == 1 and not args.symbols and not args.mix and E == (1 << 22):
            with open(pmc) as f:
                pj = json.load(f)
            traffic = pj.get("hbm_bytes_per_launch")
            pmc_derived = pj.get("per_kernel_derived")
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
            "config": {"workload": desc, "symbols_per_gpu": nsym, "accounts": nacc, "epoch_records": E,
                       "stream_records_per_gpu": total, "mode": "FUNDED (symbol groups in parallel)",
                       "parallelism": f"symbol-sharded x{world}"},
            "p99_epoch_ms": float(np.percentile(lat, 99)),
            "p50_epoch_ms": float(np.percentile(lat, 50)),
            "fills_per_s": 2 * n_trades_all / elapsed,
            "trades_per_s": n_trades_all / elapsed,
            "phase_ms_last_epoch": {k: round(v, 4) for k, v in eng.phase_times().items()},
            "events_per_epoch_rank0": {k: v / args.steps for k, v in mix.items()},
            "roofline": {"kernel": "k_match_lanes+k_match (match phase: light groups one lane each, heavy groups "
                                   "one wavefront each, concurrent)", "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "bytes_model": "SURVEY §8d: 52/in + 36/trade + 32/rest + 32/maker visit + 48/cancel",
                         "avg_launch_ms": avg_match_s * 1e3, "alg_bytes_per_launch": float(np.mean(bytes_alg))},
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
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
