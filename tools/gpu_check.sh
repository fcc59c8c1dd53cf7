#!/bin/bash
# One GPU-box session: smoke → gpu parity tests → bench → rocprof kernel stats.
# Every GPU step runs under its own time limit; the script stops at the first
# crash/timeout (exit status > 1) and never retries a step.
#   usage: tools/gpu_check.sh [steps...]   (default: smoke pytest bench prof pmc cbench)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-r01}

step() {   # name timeout cmd...
    local name=$1 t=$2
    shift 2
    echo "== $name: $*"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 12 "gpurun_out/$name.log"
    return $rc
}

want() { [ $# -eq 0 ] && return 0; for s in $STEPS; do [ "$s" = "$1" ] && return 0; done; return 1; }
STEPS=${*:-smoke pytest bench prof pmc cbench}

if want smoke; then step smoke 600 python __graft_entry__.py smoke || exit 1; fi
if want pytest; then
    step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread
    rc=$?; [ $rc -le 1 ] || exit $rc
fi
if want bench; then
    step bench 600 python bench.py || exit 1
fi
if want prof; then
    # the bench command itself under the profiler: the JSON line it prints
    # (prof.log) and the kernel stats come from one process
    step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run \
        --output-format csv -- python bench.py || exit 1
    find gpurun_out/prof -name '*stats*' | head
fi
if want pmc; then
    BENCH="python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --check 0 --pcie 0"
    step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run \
        --output-format csv -- $BENCH || exit 1
    step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run \
        --output-format csv -- $BENCH || exit 1
    python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write \
        --out gpurun_out/pmc_parse_hash.json > gpurun_out/pmc_summary.log 2>&1
    tail -n 20 gpurun_out/pmc_summary.log
fi
if want cbench; then
    step cbench 600 tools/yrss_cbench 1 1048576 0 2 || exit 1
    step host_async 600 bash tools/gpu_cbprof.sh || exit 1
fi
echo "== done"
