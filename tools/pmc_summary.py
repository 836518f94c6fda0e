"""Per-launch HBM traffic of one kernel from rocprofv3 --pmc passes (tools/pmc_round.sh output).

FETCH_SIZE and WRITE_SIZE (KiB per dispatch) come from separate passes (FETCH_SIZE uses 3 of the 4
TCC slots, WRITE_SIZE 2).  MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports half the bytes of a
WIDE COALESCED STREAMING read (128-B requests tallied at 64 B).  The matching kernels' reads are random
gathers instead, and for those FETCH_SIZE is the bytes the line fills move, as reported: calibrated with
tools/pmc_randcal.sh (profiles/r05_randcal.json: random 16 / 32 / 64-B gathers over a 2 GiB table give
FETCH_SIZE = 4.0 / 2.0 / 1.05 x the bytes named = one 64-B fill per gather, TCC_EA0_RDREQ = 1.00 / 1.00
/ 1.05 per gather).  So read bytes = FETCH_SIZE (x2 only with --streaming); WRITE_SIZE as reported.
Both count Infinity-Cache (MALL) hits too, so this is L2-miss traffic, an upper bound on HBM bytes.

usage: python tools/pmc_summary.py <pmc dir> <kernel regex> <out.json> [skip_first_n] [--streaming]
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
    args = [a for a in sys.argv[1:] if a != "--streaming"]
    streaming = "--streaming" in sys.argv[1:]
    d, kre, out = args[0], args[1], args[2]
    skip = int(args[3]) if len(args) > 3 else 0
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
        k = 2 if streaming else 1
        res["read_bytes_per_launch"] = k * f * 1024
        res["write_bytes_per_launch"] = w * 1024
        res["hbm_bytes_per_launch"] = k * f * 1024 + w * 1024
        res["note"] = ("FETCH_SIZE doubled (wide coalesced streaming reads)" if streaming else
                       "FETCH_SIZE as reported (random gathers: one 64-B fill each, tools/pmc_randcal.sh)") + \
                      "; MALL hits included (upper bound)"
    res["per_kernel_derived"] = derived(res)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
