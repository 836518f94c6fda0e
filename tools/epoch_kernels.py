"""Per-kernel time inside one epoch of a rocprofv3 kernel trace (the span between the last two k_emap
launches, i.e. the last complete epoch): python3 tools/epoch_kernels.py <kernel_trace.csv> [n] [--seq]
(--seq: also every launch of that epoch in order, with its start offset and duration)"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
args = [a for a in sys.argv[2:] if a != "--seq"]
top = int(args[0]) if args else 40
by = collections.defaultdict(list)
for r in rows:
    by[r["Kernel_Name"].split("(")[0]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
em = sorted(by["kme::k_emap"])
t0, t1 = em[-2][0], em[-1][0]
tot = collections.Counter()
for k, v in by.items():
    for s, d in v:
        if t0 <= s < t1:
            tot[k] += d
for k, d in tot.most_common(top):
    print(f"{d / 1e3:9.1f} us  {k}")
print(f"kernels {sum(tot.values()) / 1e3:.1f} us, epoch span {(t1 - t0) / 1e3:.1f} us")
if "--seq" in sys.argv:
    seq = sorted((s, d, k) for k, v in by.items() for s, d in v if t0 <= s < t1)
    for s, d, k in seq:
        print(f"  +{(s - t0) / 1e3:8.1f} us {d / 1e3:8.1f} us  {k}")
