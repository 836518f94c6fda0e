#!/bin/bash
# FETCH_SIZE / TCC_EA0_RDREQ calibration for random gathers: tools/randbench2's
# k_load<16|32|64> over a 2 GiB table issue 4 x iters independent random loads per lane of a known
# width, so the bytes they name are known exactly; one PMC pass per counter group, each its own run.
# Usage (through gpurun): bash tools/pmc_randcal.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-randcal}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for PMC in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_REQ_sum TCC_READ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-include-regex "k_load" --output-format csv -d $OUT/p$i -o run -- ./tools/randbench2 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 - $OUT <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
# randbench2: blocks = 1024, 256 threads, iters = 32, 4 loads per iteration -> 33,554,432 loads per dispatch;
# tables 0.5 / 64 / 256 / 2048 MiB in order, each case launched twice (warm-up, timed)
loads = 1024 * 256 * 32 * 4
rows = collections.defaultdict(dict)
for f in sorted(glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        key = (r["Kernel_Name"].split("(")[0], int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))))
        rows[key][r["Counter_Name"]] = rows[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
res = collections.defaultdict(list)
for (k, d), v in sorted(rows.items(), key=lambda x: x[0][1]):
    res[k].append(v)
summary = {}
for k, lst in res.items():
    width = int(k.split("<")[1].rstrip(">")) if "<" in k else 0
    # the last dispatch of each kernel is the 2 GiB table's timed run
    last = lst[-1]
    alg = loads * width
    summary[k] = {"bytes_named": alg, **{c: v for c, v in last.items()},
                  "fetch_size_bytes_over_named": last.get("FETCH_SIZE", 0) * 1024 / alg,
                  "rdreq_per_load": last.get("TCC_EA0_RDREQ_sum", 0) / loads,
                  "rdreq32_per_load": last.get("TCC_EA0_RDREQ_32B_sum", 0) / loads}
json.dump(summary, open(out + "/randcal.json", "w"), indent=1)
print(json.dumps(summary, indent=1))
PY
