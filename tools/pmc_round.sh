#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 run), k_match dispatches only.
set -o pipefail
TAG=${1:-pmc}
shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 4 --warmup 1 --orders 5242880 --no-cpu-baseline $@"
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for PMC in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $PMC --kernel-include-regex "k_match|k_table|k_emap" --output-format csv -d $OUT/p$i -o run -- python3 -u bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($PMC) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
