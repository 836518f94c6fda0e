"""The host path's timeline from a rocprofv3 run with --kernel-trace --memory-copy-trace: the last
`n` ms of copies and kernels in start order, with gaps -- which of them serialise.
Usage: python3 tools/host_path_timeline.py <dir with *_kernel_trace.csv and *_memory_copy_trace.csv> [ms]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
span_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
ev = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"].split("(")[0][-28:],
                   r.get("Queue_Id", r.get("Stream_Id", ""))))
for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        kind = r.get("Direction", r.get("Operation", "copy"))
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C " + kind + " " + r.get("Size", r.get("Bytes", "")),
                   r.get("Queue_Id", r.get("Stream_Id", ""))))
ev.sort()
t_end = max(e[1] for e in ev)
t0 = t_end - int(span_ms * 1e6)
last = None
for s, e, name, q in ev:
    if s < t0:
        continue
    print(f"{(s - t0) / 1e3:9.1f} us  +{(e - s) / 1e3:7.1f}  q{q:>3}  {name}")
