#!/bin/bash
# (the ablib/ libraries: python tools/build_measure_libs.py)
# Round-6 measurements: upper bounds, from measurement-only builds of the tree
# (lists wrong by design, their end-of-range check taken out):
#   ablib/libyrss_noload.so  span g+1's rank-stream loads replaced by span g's
#                            registers: what a smaller per-packet stream (bucket
#                            codes) could save, at most (<= 16 buckets)
#   ablib/libyrss_noconf.so  the placement's table reads and stage writes at
#                            conflict-free LDS addresses: what any swizzle of the
#                            stage or the table could save, at most
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() {   # tag profile nb-procs libs
    timeout -k 10 400 python -u tools/ab_inproc.py --nb-procs "$3" --libs "$4" --rounds 6 \
        --profile "$2" --ignore-faults > "gpurun_out/r06_ub_$1.log" 2>&1 \
        || { tail -20 "gpurun_out/r06_ub_$1.log"; exit 1; }
    grep -E '^q[0-9]' "gpurun_out/r06_ub_$1.log"
}
run tcp4_few tcp4 3,8 cur,ablib/libyrss_noload.so,ablib/libyrss_noconf.so
run imix_few imix 3 cur,ablib/libyrss_noload.so,ablib/libyrss_noconf.so
run tcp4_many tcp4 64,255 cur,ablib/libyrss_noconf.so
