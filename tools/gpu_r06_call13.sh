#!/bin/bash
# (the ablib/ libraries: python tools/build_measure_libs.py)
# round-6 call: the parse kernel with counts but no ranks (ablib/libyrss_pD.so,
# kCount 1's work in the kCount 2 kernel; lists wrong) and with no counting at
# all (ablib/libyrss_pA.so), against the tree, 12 rounds, hashed traffic
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for prof in tcp4 imix; do
    timeout -k 10 500 python -u tools/ab_inproc.py --nb-procs 3 \
        --libs cur,ablib/libyrss_pD.so,ablib/libyrss_pA.so \
        --rounds 12 --profile $prof --ignore-faults > gpurun_out/r06_parse_abl2_$prof.log 2>&1 \
        || { tail -20 gpurun_out/r06_parse_abl2_$prof.log; exit 1; }
    grep -E '^q[0-9]' gpurun_out/r06_parse_abl2_$prof.log
done
