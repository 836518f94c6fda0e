#!/bin/bash
# HBM / L2 counters of the streaming epoch kernels (one rocprofv3 pass per counter group).
# Usage (through gpurun): bash tools/pmc_mem.sh <tag> <kernel regex> [bench args...]
set -o pipefail
TAG=${1:-pmcmem}
KRE=${2:-k_emap}
shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for PMC in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_ATOMIC_sum TCC_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $PMC --kernel-include-regex "$KRE" --output-format csv -d $OUT/p$i -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --host-path-epochs 0 "$@" > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 tools/pmc_summary.py $OUT "$KRE" $OUT/pmc_summary.json 1 > /dev/null && echo "summary: $OUT/pmc_summary.json"
