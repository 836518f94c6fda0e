#!/bin/bash
# pass variant: A/B against the previous build (diagnostic)
set -o pipefail
bash tools/ab_lib.sh kafka-matching-engine_amd/kme/libkme_var.so "--workload c2 --steps 5 --warmup 2 --host-path-epochs 0" "--workload c4 --steps 3 --warmup 1 --host-path-epochs 0" "--workload c3 --symbols 8192 --steps 5 --warmup 2 --host-path-epochs 0" "--workload c5 --steps 5 --warmup 2 --host-path-epochs 0"
