#!/bin/bash
# (the ablib/ libraries: python tools/build_measure_libs.py)
# round-6 call: where the hashed parse kernel's extra time goes (measurement
# builds, lists wrong by design where they drop work):
#   ablib/libyrss_pA.so  no counting and no ranks in the parse kernel
#   ablib/libyrss_pB.so  no Toeplitz table lookups (a multiply mix of the tuple)
#   ablib/libyrss_pC.so  hash % d as h & (d - 1): exact at nb_procs 3 (d = 2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for prof in tcp4 imix; do
    timeout -k 10 400 python -u tools/ab_inproc.py --nb-procs 3 \
        --libs cur,ablib/libyrss_pA.so,ablib/libyrss_pB.so,ablib/libyrss_pC.so \
        --rounds 6 --profile $prof --ignore-faults > gpurun_out/r06_parse_abl_$prof.log 2>&1 \
        || { tail -20 gpurun_out/r06_parse_abl_$prof.log; exit 1; }
    grep -E '^q[0-9]' gpurun_out/r06_parse_abl_$prof.log
done
