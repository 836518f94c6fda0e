"""Per-kernel duration summary of a rocprofv3 --kernel-trace run of bench.py.

Only the last `timed` dispatches of each epoch kernel are averaged: they are the timed epochs of
`bench.py --steps <timed>` (setup and warmup epochs come first).

usage: python tools/trace_summary.py <run_kernel_trace.csv> <timed> <out.json> [note]
"""
import csv
import json
import sys


def main():
    path, timed, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    note = sys.argv[4] if len(sys.argv) > 4 else ""
    per = {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            name = row["Kernel_Name"].split("(")[0]
            dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
            per.setdefault(name, []).append((int(row["Dispatch_Id"]), dur))
    res = {"_note": note, "_source": path}
    for name, xs in sorted(per.items()):
        xs.sort()
        last = [d for _, d in xs[-timed:]]
        res[name] = {"dispatches": len(xs), "avg_ns_timed": sum(last) / len(last), "min_ns_timed": min(last),
                     "max_ns_timed": max(last)}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    for name in sorted(res):
        if not name.startswith("_"):
            print(f"{res[name]['avg_ns_timed'] / 1e3:10.1f} us  {name}")


if __name__ == "__main__":
    main()
