#!/bin/bash
# PMC passes over a short bench run, one counter group per rocprofv3 run, dispatches of one kernel.
# Usage (through gpurun): bash tools/pmc_kmatch.sh <tag> <kernel regex> [bench args...]
set -o pipefail
TAG=${1:-pmc}
KRE=${2:-k_match}
shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline $@"
i=0
for PMC in "SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES" \
           "SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_IFETCH GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $PMC --kernel-include-regex "$KRE" --output-format csv -d $OUT/p$i -o run -- python3 -u bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 tools/pmc_summary.py $OUT "$KRE" $OUT/pmc_summary.json 1 > /dev/null && echo "summary: $OUT/pmc_summary.json"
