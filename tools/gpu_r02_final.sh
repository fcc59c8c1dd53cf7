#!/bin/bash
# Round-2 measurement set: smoke, every GPU test, the bench (and the same
# command under rocprofv3), PMC FETCH/WRITE passes for udp4 and tcp4, the
# per-config table, and the worker / burst soaks.  Each GPU step has its own
# time limit; a crash or timeout (status > 1) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() {   # name timeout cmd...
    local name=$1 t=$2
    shift 2
    echo "== $name: $*"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 3 "gpurun_out/$name.log" | cut -c1-400
    return $rc
}
step smoke 600 python __graft_entry__.py smoke || exit 1
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread
rc=$?; [ $rc -le 1 ] || exit $rc
step bench 600 python bench.py || exit 1
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py || exit 1
python tools/trace_gaps.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/trace_gaps.log 2>&1
cp profiles/pmc_parse_hash.json gpurun_out/pmc_parse_hash.json
for p in udp4 tcp4; do
    B="python bench.py --profile $p --steps 10 --warmup 3 --cpu-seconds 0 --check 0 --pcie 0"
    step pmc_fetch_$p 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$p -o run --output-format csv -- $B || exit 1
    step pmc_write_$p 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$p -o run --output-format csv -- $B || exit 1
    python tools/pmc_summary.py gpurun_out/pmc_fetch_$p gpurun_out/pmc_write_$p --profile $p \
        --out gpurun_out/pmc_parse_hash.json > gpurun_out/pmc_summary_$p.log 2>&1
    grep -E '"traffic_over_algorithmic"|"step_traffic_over_algorithmic"' gpurun_out/pmc_summary_$p.log
done
step configs 900 python tools/configs_table.py --steps 50 --cpu-seconds 5 || exit 1
step worker_soak 300 python tools/worker_soak.py --seconds 30 || exit 1
step burst_soak 300 python tools/burst_soak.py --seconds 30 || exit 1
step fanout_soak 300 python tools/fanout_soak.py --seconds 30 || exit 1
echo "== done"
