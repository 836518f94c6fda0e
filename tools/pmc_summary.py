"""Per-launch HBM traffic of one kernel from rocprofv3 --pmc passes (tools/pmc_round.sh output).

FETCH_SIZE and WRITE_SIZE (KiB per dispatch) come from separate passes (FETCH_SIZE uses 3 of the 4
TCC slots, WRITE_SIZE 2).  Following MI355X_MICROARCH.md §HBM: FETCH_SIZE on gfx950 tallies 128-B
memory requests at 64 B, so read bytes = 2 x FETCH_SIZE; WRITE_SIZE is taken as reported.  Both
count Infinity-Cache (MALL) hits too, so this is L2-miss traffic, an upper bound on HBM bytes.

usage: python tools/pmc_summary.py <pmc dir> <kernel regex> <out.json> [skip_first_n]
"""
import csv
import glob
import json
import os
import re
import sys


def counters(d, kernel_re):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if not re.search(kernel_re, row.get("Kernel_Name", "")):
                    continue
                name = row["Counter_Name"]
                kern = row.get("Kernel_Name", "").split("(")[0]
                disp = int(row.get("Dispatch_Id", 0))
                vals.setdefault(name, {}).setdefault(kern, {}).setdefault(disp, 0.0)
                vals[name][kern][disp] += float(row["Counter_Value"])
    return vals


N_SE, N_CU, WAVES_PER_CU = 32, 256, 32   # MI355X: 8 XCDs x 4 shader engines, 256 CUs, 32 waves/CU cap


def derived(res):
    """Per kernel: occupancy and LDS bank conflicts.  SQ_WAVE_CYCLES counts quad-cycles summed over
    the waves; SQ_BUSY_CYCLES counts cycles summed over the 32 shader engines, so the kernel's own
    duration in cycles is SQ_BUSY_CYCLES / 32 and the mean resident waves per CU is
    4 * SQ_WAVE_CYCLES / (SQ_BUSY_CYCLES / 32) / 256.  SQ_LDS_BANK_CONFLICT = extra LDS cycles."""
    get = lambda c, k: res.get(c, {}).get("per_kernel", {}).get(k)
    out = {}
    for k in res.get("SQ_WAVES", {}).get("per_kernel", {}):
        wc, bc = get("SQ_WAVE_CYCLES", k), get("SQ_BUSY_CYCLES", k)
        d = {"waves": get("SQ_WAVES", k)}
        if wc and bc:
            w = 4 * wc / (bc / N_SE) / N_CU
            d["mean_resident_waves_per_cu"] = w
            d["occupancy_frac"] = w / WAVES_PER_CU
        if get("SQ_LDS_BANK_CONFLICT", k) is not None:
            d["lds_bank_conflict_cycles"] = get("SQ_LDS_BANK_CONFLICT", k)
            d["lds_insts"] = get("SQ_INSTS_LDS", k)
        out[k] = d
    return out


def build_id_of(d):
    """kme_build_id() of the library the profiled bench runs loaded: bench.py prints it in its line
    (one per pass log, <d>/p*.log); None when the passes disagree or none printed one."""
    ids = set()
    for f in glob.glob(os.path.join(d, "p*.log")) + glob.glob(os.path.join(d, "*.p*.log")):
        with open(f) as fh:
            for line in fh:
                if line.startswith("{") and '"build_id"' in line:
                    try:
                        ids.add(json.loads(line)["build_id"])
                    except (ValueError, KeyError):
                        pass
    return ids.pop() if len(ids) == 1 else None


def main():
    d, kre, out = sys.argv[1], sys.argv[2], sys.argv[3]
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    allv = {}
    for sub in sorted(glob.glob(os.path.join(d, "p*"))):
        if os.path.isdir(sub):
            for k, v in counters(sub, kre).items():
                allv[k] = v
    res = {"kernel_regex": kre, "source": os.path.relpath(d), "build_id": build_id_of(d)}
    # several kernels may match (k_match and k_match_lanes both run once per epoch): the figure per
    # epoch ("per launch" of the match phase) is the sum of each kernel's mean per dispatch
    for k, kerns in sorted(allv.items()):
        tot, per_kernel = 0.0, {}
        for kern, per in sorted(kerns.items()):
            xs = [per[i] for i in sorted(per)][skip:]
            if xs:
                per_kernel[kern] = sum(xs) / len(xs)
                tot += per_kernel[kern]
        if per_kernel:
            res[k] = {"mean_per_dispatch": tot, "per_kernel": per_kernel}
    f = res.get("FETCH_SIZE", {}).get("mean_per_dispatch")
    w = res.get("WRITE_SIZE", {}).get("mean_per_dispatch")
    if f is not None and w is not None:
        res["read_bytes_per_launch"] = 2 * f * 1024
        res["write_bytes_per_launch"] = w * 1024
        res["hbm_bytes_per_launch"] = 2 * f * 1024 + w * 1024
        res["note"] = "FETCH_SIZE doubled per the gfx950 calibration; MALL hits included (upper bound)"
    res["per_kernel_derived"] = derived(res)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
