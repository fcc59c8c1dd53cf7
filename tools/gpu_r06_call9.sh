#!/bin/bash
# round-6 call: the first span's streams issued at scatter entry (in-scatter
# prefixes), the next set's zeroing in waves 1-7 before their loads.
# Layout tests, same-process A/B against HEAD's library (ablib/libyrss_r6head.so)
# on 2-list and one-list traffic, and the phase clock's prologue milestones.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${TAG:-c14}
timeout -k 10 400 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/r06_${T}_tests.log 2>&1 || { tail -30 gpurun_out/r06_${T}_tests.log; exit 1; }
tail -2 gpurun_out/r06_${T}_tests.log
for prof in tcp4 imix udp4; do
    nbp=3,8; [ $prof = tcp4 ] || nbp=3
    timeout -k 10 400 python -u tools/ab_inproc.py --nb-procs $nbp --libs cur,ablib/libyrss_r6head.so \
        --rounds 6 --profile $prof > gpurun_out/r06_ab_${T}_$prof.log 2>&1 || { tail -20 gpurun_out/r06_ab_${T}_$prof.log; exit 1; }
    grep -E '^q[0-9]' gpurun_out/r06_ab_${T}_$prof.log
done
tools/build_ab_lib.sh prof -DYRSS_PROF_LINES=1 > gpurun_out/build_prof.log 2>&1 || exit 1
timeout -k 10 200 python tools/line_prof.py --lib ab/lib/libyrss_prof.so --nb-procs 3,8 > gpurun_out/r06_lineprof_${T}.log 2>&1 || exit 1
grep -E "prologue|span total|end after" gpurun_out/r06_lineprof_${T}.log
