#!/bin/bash
# k_match cycle shares from the -DKME_STAMPS build (diagnostic; never a bench line).
# Usage (through gpurun): bash tools/gpu_stamps.sh <tag> "<bench args 1>" ...
# Each args string may start with HOT=1 to read the hottest group's row instead of the sum.
set -o pipefail
OUT=gpurun_out/${1:-stamps}
shift || true
mkdir -p $OUT
export TMPDIR=/tmp
for args in "$@"; do
  hot=""
  case "$args" in HOT=1*) hot=1; args="${args#HOT=1 }";; esac
  KME_STAMPS_HOT=$hot timeout -k 10 300 python3 -u bench.py --stamps --no-cpu-baseline --host-path-epochs 0 $args >> $OUT/stamps.jsonl 2>> $OUT/stamps.err
  rc=$?; echo "stamps [$args] hot=$hot rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/stamps.err; exit $rc; }
done
cat $OUT/stamps.jsonl
