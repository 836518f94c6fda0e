#!/bin/bash
# Resource usage of k_match and the loops LLVM's uniformity analysis considers to have divergent
# exits.  Only the free-list spill loop (a per-lane loop) may be listed: any other entry means the
# wave-uniform matching state was demoted to exec-masked VGPR code.
set -o pipefail
cd "$(dirname "$0")/../kafka-matching-engine_amd/csrc"
F=${1:-kme_kernels.hip}
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -I../../include -I. --offload-device-only"
/opt/rocm/bin/hipcc $FLAGS -c $F -o /tmp/kme_chk.o -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep -A11 "Name: _ZN3kme7k_match" | grep -E "SGPRs:|VGPRs:|Occupancy|Spill|LDS Size" | sed 's/.*remark: *//'
/opt/rocm/bin/hipcc $FLAGS -emit-llvm -S $F -o /tmp/kme_chk.ll 2>/dev/null
/opt/rocm/lib/llvm/bin/opt -passes='print<uniformity>' -disable-output /tmp/kme_chk.ll 2>&1 \
  | awk '/UniformityInfo for function .*_ZN3kme7k_matchE/{f=1;next} /UniformityInfo for function/{f=0} f' \
  | awk '/CYCLES WITH DIVERGENT EXIT/{f=1;print;next} /^$/{f=0} f' | cut -c1-100
