#!/bin/bash
# Round-5 measurement set, in three gpurun calls (PART=a, b, c):
#   a  smoke; every GPU test; the bench (headline + configs[3]/[4] + CPU baseline +
#      host-resident rows) and the same command under rocprofv3 --kernel-trace
#      --stats; PMC FETCH/WRITE passes for udp4 and tcp4 (profiles/pmc_parse_hash.json)
#   b  the all-TCP q-rows (3/8/64/255 procs: bench line + rocprof kernel stats),
#      per-kernel PMC at the same rows, the line scatter's phase clock
#   c  the driver's N>1 launch rehearsed on one device: N=8 on udp4 (its
#      configs_extra rows are configs[3] and configs[4] at 8 ranks), N=2; every
#      BASELINE config (tools/configs_table.py)
# Each GPU step has its own time limit; a crash or timeout ends the script.
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
    tail -n 2 "gpurun_out/$name.log" | cut -c1-300
    return $rc
}
case "${PART:-a}" in
a)
    step smoke 300 python __graft_entry__.py smoke || exit 1
    step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
    step bench 600 python bench.py || exit 1
    step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --pcie 0 --cpu-seconds 0 --extra-configs= || exit 1
    cp profiles/pmc_parse_hash.json gpurun_out/pmc_parse_hash.json
    for p in udp4 tcp4; do
        B="python bench.py --profile $p --steps 10 --warmup 3 --cpu-seconds 0 --check 0 --pcie 0 --extra-configs="
        step pmc_fetch_$p 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$p -o run --output-format csv -- $B || exit 1
        step pmc_write_$p 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$p -o run --output-format csv -- $B || exit 1
        python tools/pmc_summary.py gpurun_out/pmc_fetch_$p gpurun_out/pmc_write_$p --profile $p \
            --out gpurun_out/pmc_parse_hash.json > gpurun_out/pmc_summary_$p.log 2>&1
    done
    ;;
b)
    tools/build_ab_lib.sh prof -DYRSS_PROF_LINES=1 > /dev/null 2>&1 || exit 1
    bash tools/gpu_r03_qrows.sh r05 || exit 1
    step lineprof 200 python tools/line_prof.py --lib ab/lib/libyrss_prof.so --nb-procs 3,8,64,255 || exit 1
    bash tools/gpu_pmc.sh r05 "3 8 64 255" || exit 1
    ;;
c)
    step rehearse_n8 900 bash tools/gpu_rehearse.sh 8 udp4 || exit 1
    step rehearse_n2 600 bash tools/gpu_rehearse.sh 2 udp4 || exit 1
    step configs 900 python tools/configs_table.py || exit 1
    ;;
esac
echo "== done (part ${PART:-a})"
