#!/bin/bash
# L2 / memory-side counters of one kernel for several builds of libkme.so (diagnostic A/B).
# Usage (through gpurun): bash tools/pmc_tcc.sh <tag> <kernel regex> lib1.so lib2.so ...
set -o pipefail
TAG=${1:-pmctcc}
KRE=${2:-k_match_lanes}
shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for L in "$@"; do
  n=$(basename $L .so)
  i=0
  for PMC in "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_64B_sum TCC_REQ_sum TCC_WRITE_sum"; do
    i=$((i+1))
    KME_LIB=$L timeout -s KILL 150 rocprofv3 --pmc $PMC --kernel-include-regex "$KRE" --output-format csv -d $OUT/$n/p$i -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$n.p$i.log 2>&1
    rc=$?; echo "$n pass $i rc=$rc"
    [ $rc -eq 0 ] || { tail -5 $OUT/$n.p$i.log; exit $rc; }
  done
  python3 tools/pmc_summary.py $OUT/$n "$KRE" $OUT/$n.json 1 > /dev/null
  python3 - $OUT/$n.json "$KRE" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
row = {}
for k, v in d.items():
    if isinstance(v, dict) and "per_kernel" in v:
        for kern, x in v["per_kernel"].items():
            if sys.argv[2] in kern:
                row[k] = x
print(sys.argv[1], json.dumps({k: round(v / 1e6, 3) for k, v in sorted(row.items())}))
PY
done
