#!/bin/bash
# round-6 call: the next set's zeroing moved out of wave 0 (ahead of waves
# 1-7's loads).  Layout and fuzz tests, then a 12-round same-process A/B
# against HEAD's library (ablib/libyrss_head7.so) on 2-list and one-list traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${TAG:-c21}
timeout -k 10 400 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/r06_${T}_tests.log 2>&1 || { tail -30 gpurun_out/r06_${T}_tests.log; exit 1; }
tail -1 gpurun_out/r06_${T}_tests.log
for prof in tcp4 imix udp4; do
    timeout -k 10 500 python -u tools/ab_inproc.py --nb-procs 3 --libs cur,ablib/libyrss_head7.so \
        --rounds 12 --profile $prof > gpurun_out/r06_ab_${T}_$prof.log 2>&1 || { tail -20 gpurun_out/r06_ab_${T}_$prof.log; exit 1; }
    grep -E '^q[0-9]' gpurun_out/r06_ab_${T}_$prof.log
done
