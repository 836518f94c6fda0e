"""Measurement tooling (CPU): the PMC summary's derived occupancy / LDS figures and the bench's
algorithmic byte model."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import pmc_summary  # noqa: E402


def _res(per_kernel):
    out = {}
    for k, counters in per_kernel.items():
        for c, v in counters.items():
            out.setdefault(c, {"mean_per_dispatch": 0.0, "per_kernel": {}})
            out[c]["per_kernel"][k] = v
            out[c]["mean_per_dispatch"] += v
    return out


def test_occupancy_formula():
    # 2,048 waves resident for the whole kernel: 8 per CU; SQ_WAVE_CYCLES in quad-cycles summed over
    # waves, SQ_BUSY_CYCLES in cycles summed over the 32 shader engines
    cycles = 1_000_000
    res = _res({"k": {"SQ_WAVES": 2048, "SQ_WAVE_CYCLES": 2048 * cycles / 4, "SQ_BUSY_CYCLES": 32 * cycles,
                      "SQ_LDS_BANK_CONFLICT": 10.0, "SQ_INSTS_LDS": 1000.0}})
    d = pmc_summary.derived(res)["k"]
    assert abs(d["mean_resident_waves_per_cu"] - 8.0) < 1e-9
    assert abs(d["occupancy_frac"] - 8.0 / 32) < 1e-9
    assert d["lds_bank_conflict_cycles"] == 10.0 and d["lds_insts"] == 1000.0


def test_committed_pmc_summaries_carry_derived_fields():
    for name in ("pmc_k_match_c3.json", "pmc_k_match_c3_s8192.json"):
        with open(os.path.join(ROOT, "profiles", name)) as f:
            d = json.load(f)
        assert d["hbm_bytes_per_launch"] > 0
        for k, v in d["per_kernel_derived"].items():
            assert 0.0 <= v["occupancy_frac"] <= 1.0, (name, k)


def test_bench_byte_model():
    import types
    sys.path.insert(0, ROOT)
    src = open(os.path.join(ROOT, "bench.py")).read()
    ns = {}
    start = src.index("def algorithmic_bytes")
    end = src.index("\n\n\n", start)
    exec(src[start:end], ns)
    st = types.SimpleNamespace(n_inputs=10, n_trades=3, n_rests=4, n_maker_visits=3, n_cancel_ok=2)
    assert ns["algorithmic_bytes"](st) == 52 * 10 + 36 * 3 + 32 * 4 + 32 * 3 + 48 * 2


def test_credit_split_probe_counts_the_first_failing_epoch():
    import numpy as np
    import credit_split_probe as probe

    # one account, two shards, four BUY/SELL of risk 10 at records 0, 1, 5, 6 (epochs of 4 records):
    # shard 0 gets three of them (30 > 40 // 2 = 20 from the third on, record 6 -> epoch 1)
    aid = np.zeros(4, np.int64)
    shard = np.array([0, 0, 1, 0], np.int64)
    risk = np.full(4, 10, np.int64)
    pos = np.array([0, 1, 5, 6], np.int64)
    st = probe.fallback_stats(aid, shard, risk, pos, 8, 1, 2, 1.0, 4)
    assert st["epochs"] == 2 and st["fallback_epochs"] == 1 and st["first_fallback_epoch"] == 1
    assert st["failing_pairs"] == 1 and st["failing_accounts"] == 1
    # one shard: the whole credit, nothing fails; twice the credit on two shards: nothing fails
    assert probe.fallback_stats(aid, np.zeros(4, np.int64), risk, pos, 8, 1, 1, 1.0, 4)["fallback_epochs"] == 0
    assert probe.fallback_stats(aid, shard, risk, pos, 8, 1, 2, 2.0, 4)["fallback_epochs"] == 0
    # the max risk of checkBalance (KP:172-176): BUY size * price, SELL size * (100 - price)
    r = probe.max_risk(np.array([2, 3, 4]), np.array([30, 30, 0]), np.array([10, 10, 0]))
    assert r.tolist() == [300, 700, 0]


def test_bench_reports_traffic_only_for_the_profiled_build(tmp_path):
    """roofline.traffic comes from the committed PMC summary only when that summary profiled the very
    library the bench loaded (its kme_build_id()); otherwise the line says why it has none."""
    sys.path.insert(0, ROOT)
    import bench

    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"build_id": "abc", "hbm_bytes_per_launch": 123.0, "per_kernel_derived": {"k": {}},
                             "source": "passes of build abc"}))
    traffic, derived, src = bench.pmc_for_build(str(p), "abc")
    assert traffic == 123.0 and derived == {"k": {}} and "abc" in src
    traffic, derived, src = bench.pmc_for_build(str(p), "def")
    assert traffic is None and derived is None and "abc" in src and "def" in src
    assert bench.pmc_for_build(str(tmp_path / "missing.json"), "abc")[0] is None


def test_pmc_summary_records_the_profiled_build(tmp_path):
    """tools/pmc_summary.py takes the build id from the bench lines its passes printed."""
    d = tmp_path / "pmc"
    d.mkdir()
    (d / "p1.log").write_text("some rocprof noise\n" + json.dumps({"metric": "m", "build_id": "0123456789abcdef"}) + "\n")
    assert pmc_summary.build_id_of(str(d)) == "0123456789abcdef"
