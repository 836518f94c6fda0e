#!/bin/bash
# Latency breakdown of k_match: instruction counts, in-flight levels (level / count = mean latency).
set -o pipefail
TAG=${1:-pmclat}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 4 --warmup 1 --orders 5242880 --no-cpu-baseline"
i=0
for PMC in "SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_IFETCH"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $PMC --kernel-include-regex "k_match" --output-format csv -d $OUT/p$i -o run -- python3 -u bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
