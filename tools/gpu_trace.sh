#!/bin/bash
# A rocprofv3 kernel trace of one bench.py command and its per-kernel summary (timed epochs only).
# Usage (through gpurun): bash tools/gpu_trace.sh <tag> <timed steps> [bench args...]
set -o pipefail
TAG=${1:-trace}
STEPS=${2:-5}
shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 -u bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --host-path-epochs 0 "$@" > $OUT/prof.log 2>&1
rc=$?; echo "prof_rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/prof.log; exit $rc; }
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py $f $STEPS $OUT/trace_summary.json "bench.py --steps $STEPS $*"
