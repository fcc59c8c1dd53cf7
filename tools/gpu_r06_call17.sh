#!/bin/bash
# (the ablib/ libraries: python tools/build_measure_libs.py)
# round-6 call: the line scatter at one workgroup a CU (ablib/libyrss_grid1.so,
# eight spans a workgroup at 2^24 packets) against the tree's two a CU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${TAG:-c20}
for prof in tcp4 imix; do
    timeout -k 10 500 python -u tools/ab_inproc.py --nb-procs 3,8,64 --libs cur,ablib/libyrss_grid1.so \
        --rounds 6 --profile $prof > gpurun_out/r06_ab_${T}_$prof.log 2>&1 || { tail -20 gpurun_out/r06_ab_${T}_$prof.log; exit 1; }
    grep -E '^q[0-9]' gpurun_out/r06_ab_${T}_$prof.log
done
