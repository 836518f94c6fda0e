#!/bin/bash
# Epoch size / light_max exploration (diagnostic, no tests): one bench line per argument set.
# Usage (through gpurun): bash tools/epoch_sweep.sh "<bench args 1>" "<bench args 2>" ...
set -o pipefail
OUT=gpurun_out/sweep
mkdir -p $OUT
for args in "$@"; do
  timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --steps 6 --warmup 2 $args > $OUT/one.json 2> $OUT/err.log
  rc=$?
  [ $rc -eq 0 ] || { echo "[$args] rc=$rc"; tail -3 $OUT/err.log; exit $rc; }
  cat $OUT/one.json >> $OUT/all.jsonl
  python3 -c "import json;d=json.load(open('$OUT/one.json'));print('[$args]', round(d['value']/1e6,1), 'M/s p99', round(d['p99_epoch_ms'],2), d['phase_ms_last_epoch'])"
done
