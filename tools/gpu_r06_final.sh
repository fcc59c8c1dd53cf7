#!/bin/bash
# Round-6 measurement set, in gpurun calls (PART=a, b, c):
#   a  smoke; every GPU test; the bench (headline + configs[3]/[4] + CPU baseline +
#      host-resident rows + fan-out + TCP-share crossover) and the same command
#      under rocprofv3 --kernel-trace --stats; PMC FETCH/WRITE passes for udp4 and
#      tcp4 (profiles/pmc_parse_hash.json)
#   b  every BASELINE config and the all-TCP queue rows (tools/configs_table.py);
#      rocprof kernel stats of the IMIX and jumbo configs; per-kernel PMC at
#      4 and 256 buckets; the line scatter's phase clock (TCP and IMIX)
#   c  the driver's N>1 launch rehearsed on one device: N=8 (the whole default
#      command, fan-out leg included) and N=2
# Each GPU step has its own time limit; a crash or timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() {   # name timeout cmd...
    local name=$1 t=$2
    shift 2
    echo "== $name: $*"
    timeout -k 10 "$t" "$@" > "gpurun_out/r06f_$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 2 "gpurun_out/r06f_$name.log" | cut -c1-300
    return $rc
}
case "${PART:-a}" in
a)
    step smoke 300 python __graft_entry__.py smoke || exit 1
    step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
    step bench 600 python bench.py || exit 1
    step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r06f_prof -o run --output-format csv -- python bench.py --pcie 0 --cpu-seconds 0 --extra-configs= || exit 1
    cp profiles/pmc_parse_hash.json gpurun_out/pmc_parse_hash.json
    for p in udp4 tcp4; do
        B="python bench.py --profile $p --steps 10 --warmup 3 --cpu-seconds 0 --check 0 --pcie 0 --extra-configs="
        step pmc_fetch_$p 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r06f_pmc_fetch_$p -o run --output-format csv -- $B || exit 1
        step pmc_write_$p 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r06f_pmc_write_$p -o run --output-format csv -- $B || exit 1
        python tools/pmc_summary.py gpurun_out/r06f_pmc_fetch_$p gpurun_out/r06f_pmc_write_$p --profile $p \
            --out gpurun_out/pmc_parse_hash.json > gpurun_out/r06f_pmc_summary_$p.log 2>&1
    done
    ;;
b)
    step configs 1200 python tools/configs_table.py || exit 1
    for p in imix jumbo_tcp4; do
        step prof_$p 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06f_prof_$p -o run --output-format csv -- python bench.py --profile $p --pcie 0 --cpu-seconds 0 --extra-configs= || exit 1
    done
    bash tools/gpu_pmc.sh r06f "3 255" > /dev/null || exit 1
    tools/build_ab_lib.sh prof -DYRSS_PROF_LINES=1 > /dev/null 2>&1 || exit 1
    step lineprof_tcp4 200 python tools/line_prof.py --lib ab/lib/libyrss_prof.so --nb-procs 3,8,64,255 || exit 1
    step lineprof_imix 200 python tools/line_prof.py --lib ab/lib/libyrss_prof.so --nb-procs 3,64,255 --profile imix || exit 1
    ;;
c)
    PART=n8 bash tools/gpu_r06.sh || exit 1
    step rehearse_n2 600 bash tools/gpu_rehearse.sh 2 udp4 || exit 1
    ;;
esac
echo "== done (part ${PART:-a})"
