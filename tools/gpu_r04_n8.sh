#!/bin/bash
# Round 4, VERDICT item 4: one-device rehearsals of the driver's N=8 bench
# launch for the two 8-GPU configs (configs[3] vlan6_tcp, configs[4]
# jumbo_tcp4): 8 ranks share device 0, each classifying its own 2^24-packet
# shard, rank 0 ANDs bit_exact over the ranks and times the CPU baseline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for p in vlan6_tcp jumbo_tcp4; do
    echo "== n8 $p"
    tools/gpu_rehearse.sh 8 "$p" || exit 1
done
