#!/bin/bash
# Kernel trace of one bench configuration, and the per-kernel time of its last complete epoch.
# Usage (through gpurun): bash tools/gpu_prof_epoch.sh <tag> "<bench args>"
set -o pipefail
OUT=gpurun_out/${1:-epochprof}
ARGS=$2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 -u bench.py --no-cpu-baseline --host-path-epochs 0 $ARGS > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "prof_rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 tools/epoch_kernels.py $f 40 --seq | tee $OUT/epoch_kernels.txt
