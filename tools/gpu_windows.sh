#!/bin/bash
# Worker forms at F-Stack's 32-packet bursts and at 1024: mbuf pointers (0),
# (data, data_len) pairs (1), windows the dispatcher copies (2).
# tools/gpu_windows.sh TAG -> gpurun_out/TAG_windows.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/${1:-w}_windows.log
: > "$out"
for frames in 0 1 2; do
  for cfg in "32 128" "32 64" "1024 32"; do
    set -- $cfg
    YRSS_CBENCH_MODES=4 YRSS_CBENCH_WORKER_DEPTH=$((4 * $2)) YRSS_CBENCH_WORKER_BLOCKS=$2 \
    YRSS_CBENCH_WORKER_SLOTOUT=1 YRSS_CBENCH_WORKER_FRAMES=$frames \
      timeout -k 10 120 tools/yrss_cbench 0 $((1 << 20)) $1 1 >> "$out" 2>&1 || exit 1
  done
done
echo done >> "$out"
