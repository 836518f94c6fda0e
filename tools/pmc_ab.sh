#!/bin/bash
# Instruction / wait counters of one kernel for several builds of libkme.so (diagnostic A/B).
# Usage (through gpurun): bash tools/pmc_ab.sh <tag> <kernel regex> lib1.so lib2.so ...
set -o pipefail
TAG=${1:-pmcab}
KRE=${2:-k_match_lanes}
shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for L in "$@"; do
  n=$(basename $L .so)
  i=0
  for PMC in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES" \
             "SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_IFETCH SQ_INST_LEVEL_VMEM SQ_INSTS_LDS"; do
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
            if kern.endswith(sys.argv[2]) or sys.argv[2] in kern:
                row[k] = x
print(sys.argv[1], json.dumps({k: round(v / 1e6, 2) for k, v in sorted(row.items())}))
PY
done
