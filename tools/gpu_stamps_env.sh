#!/bin/bash
# k_match cycle shares (-DKME_STAMPS build) under an environment setting (diagnostic).
# Usage (through gpurun): bash tools/gpu_stamps_env.sh <tag> "<ENV=v ...>" "<bench args>" ...
set -o pipefail
OUT=gpurun_out/${1:-stampsenv}
ENVSET=$2
shift 2 || true
mkdir -p $OUT
for args in "$@"; do
  hot=""
  case "$args" in HOT=1*) hot=1; args="${args#HOT=1 }";; esac
  env $ENVSET KME_STAMPS_HOT=$hot timeout -k 10 300 python3 -u bench.py --stamps --no-cpu-baseline --host-path-epochs 0 $args >> $OUT/stamps.jsonl 2>> $OUT/stamps.err
  rc=$?; echo "stamps [$ENVSET] [$args] rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/stamps.err; exit $rc; }
done
cat $OUT/stamps.jsonl
