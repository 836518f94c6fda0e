set -o pipefail
bash tools/gpu_stamps_env.sh st3a 'KME_TWO_MAX=0' 'HOT=1 --workload c4 --steps 2 --warmup 1' '--workload c2 --steps 3 --warmup 1' > /dev/null && bash tools/gpu_stamps_env.sh st3b 'KME_TWO_MAX=4096' 'HOT=1 --workload c4 --steps 2 --warmup 1' '--workload c2 --steps 3 --warmup 1' > /dev/null
rc=$?
for t in st3a st3b; do echo $t; cat gpurun_out/$t/stamps.jsonl; done
exit $rc
