#!/bin/bash
# Rehearsal of the N-rank bench on a one-GPU box (diagnostic): N ranks on GPU 0, gloo collectives.
# Usage (through gpurun): bash tools/gpu_rehearse.sh <tag> <N> [bench args...]
set -o pipefail
OUT=gpurun_out/${1:-rehearse}
N=${2:-2}
shift 2 || true
mkdir -p $OUT
export TMPDIR=/tmp
KME_BENCH_REHEARSAL=1 timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node=$N \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $N "$@" > $OUT/rehearse_n$N.json 2> $OUT/rehearse_n$N.err
rc=$?; echo "rehearse N=$N rc=$rc"; cat $OUT/rehearse_n$N.json; tail -3 $OUT/rehearse_n$N.err
exit $rc
