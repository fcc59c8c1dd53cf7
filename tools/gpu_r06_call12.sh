#!/bin/bash
# round-6 call: 12-round same-process A/B of the parse kernel's scalar counts
# (tree), the power-of-two divisor alone (ablib/libyrss_pow2.so) and HEAD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${TAG:-c16}
for prof in tcp4 imix udp4; do
    timeout -k 10 500 python -u tools/ab_inproc.py --nb-procs 3 \
        --libs cur,ablib/libyrss_pow2.so,ablib/libyrss_r6head.so \
        --rounds 12 --profile $prof > gpurun_out/r06_ab_${T}_$prof.log 2>&1 || { tail -20 gpurun_out/r06_ab_${T}_$prof.log; exit 1; }
    grep -E '^q[0-9]' gpurun_out/r06_ab_${T}_$prof.log
done
