#!/bin/bash
# (the ablib/ libraries: python tools/build_measure_libs.py)
# round-6 call: the parse kernel with two tiles of loads ahead (three register
# sets, ablib/libyrss_pf2.so): parity through that library, then a 12-round
# same-process A/B against the tree on hashed and UDP traffic
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${TAG:-c17}
YRSS_LIB=$PWD/ablib/libyrss_pf2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_${T}_tests.log 2>&1 \
    || { tail -30 gpurun_out/r06_${T}_tests.log; exit 1; }
tail -2 gpurun_out/r06_${T}_tests.log
for prof in tcp4 imix udp4; do
    timeout -k 10 500 python -u tools/ab_inproc.py --nb-procs 3 --libs cur,ablib/libyrss_pf2.so \
        --rounds 12 --profile $prof > gpurun_out/r06_ab_${T}_$prof.log 2>&1 || { tail -20 gpurun_out/r06_ab_${T}_$prof.log; exit 1; }
    grep -E '^q[0-9]' gpurun_out/r06_ab_${T}_$prof.log
done
