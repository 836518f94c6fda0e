#!/bin/bash
# Kernel trace of the drop-in's configuration (bench.py --java-defaults): which ledger-pass kernels
# take the epoch.  Usage (through gpurun): bash tools/gpu_prof_java.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-javaprof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 -u bench.py --java-defaults --steps 10 --warmup 3 --orders 2000000 --host-path-epochs 0 --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?; echo "prof_rc=$rc"
[ $rc -eq 0 ] || exit $rc
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py $f 10 $OUT/trace_summary.json "java defaults, E = 65,536, 10 timed epochs" | sort -t: -k2 -n | tail -30
