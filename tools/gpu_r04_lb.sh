#!/bin/bash
# Round 4: GPU suite; same-process A/B of the tree against round 3's library
# (abl/libyrss_r03.so); the line scatter's phase clock with kernel-entry
# stamps (tools/line_prof.py, -DYRSS_PROF_LINES build); the host dispatcher's
# NUMA placement and CPU-quota sensitivity (tools/numa_probe.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
out=gpurun_out/lb.log
: > "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_lb.log 2>&1 || { echo "pytest rc=$?"; tail -n 30 gpurun_out/pytest_lb.log; exit 1; }
tail -n 1 gpurun_out/pytest_lb.log >> "$out"
timeout -k 10 900 python tools/ab_inproc.py --nb-procs 3,64 --rounds 2 --steps 20 \
    --libs cur,abl/libyrss_r03.so >> "$out" 2>&1 || { echo "ab failed"; tail "$out"; exit 1; }
tools/build_ab_lib.sh prof -DYRSS_PROF_LINES=1 >> "$out" 2>&1 || { echo build failed; tail "$out"; exit 1; }
timeout -k 10 300 python tools/line_prof.py --lib ab/lib/libyrss_prof.so --nb-procs 3,8,64,255 >> "$out" 2>&1 &&
timeout -k 10 300 python tools/numa_probe.py --load 15 >> "$out" 2>&1
rc=$?
grep -v "^round\|amdgpu.ids\|^built\|warning\|^ *[0-9]* |\|\^" "$out"
exit $rc
