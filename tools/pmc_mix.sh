#!/bin/bash
# Instruction mix of k_match per record type: one PMC pass per stream mix (BUY,SELL,CANCEL).
# Usage (through gpurun): bash tools/pmc_mix.sh <tag> "<mix1>" "<mix2>" ...   e.g. "1,0,0" "0.5,0,0.5"
set -o pipefail
TAG=${1:-pmcmix}
shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for MIX in "$@"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --kernel-include-regex k_match --output-format csv -d $OUT/m$i/p1 -o run -- \
    python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --mix $MIX > $OUT/m$i.log 2>&1
  rc=$?; echo "mix $MIX rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/m$i.log; exit $rc; }
  python3 tools/pmc_summary.py $OUT/m$i k_match $OUT/m$i.json 1 > /dev/null
done
python3 - $OUT "$@" <<'PY'
import json, sys, glob
out = sys.argv[1]
for i, mix in enumerate(sys.argv[2:], 1):
    d = json.load(open(f"{out}/m{i}.json"))
    b = [json.loads(l) for l in open(f"{out}/m{i}.log") if l.startswith("{")][-1]
    ev = b["events_per_epoch_rank0"]
    n = ev["inputs"]
    print(mix, {k: round(v, 1) for k, v in ev.items()},
          {k.replace("SQ_INSTS_", ""): round(d[k]["mean_per_dispatch"] / n, 1) for k in d if isinstance(d[k], dict)})
PY
