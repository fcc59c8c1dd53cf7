#!/bin/bash
# round-6 call: scalar bucket counts in the parse kernel up to 4 buckets
# (kCount 3) and the power-of-two divisor as a mask.  The whole GPU suite,
# then same-process A/Bs against HEAD's library (ablib/libyrss_r6head.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${TAG:-c15}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r06_${T}_pytest.log 2>&1 || { tail -30 gpurun_out/r06_${T}_pytest.log; exit 1; }
tail -2 gpurun_out/r06_${T}_pytest.log
for prof in tcp4 imix udp4 jumbo_tcp4; do
    nbp=3; [ $prof = tcp4 ] && nbp=3,8
    timeout -k 10 400 python -u tools/ab_inproc.py --nb-procs $nbp --libs cur,ablib/libyrss_r6head.so \
        --rounds 6 --profile $prof > gpurun_out/r06_ab_${T}_$prof.log 2>&1 || { tail -20 gpurun_out/r06_ab_${T}_$prof.log; exit 1; }
    grep -E '^q[0-9]' gpurun_out/r06_ab_${T}_$prof.log
done
