#!/bin/bash
# Round-4 measurement set: smoke; every GPU test; the bench (headline, with the PCIe rows and
# the CPU baseline) and the same command under rocprofv3; PMC FETCH/WRITE
# passes for udp4 and tcp4 (profiles/pmc_parse_hash.json, read by the bench);
# the all-TCP q-rows (3/8/64/255 procs: bench line + rocprof kernel stats);
# per-kernel PMC passes at the same rows.  Each GPU step has its own time
# limit; a crash or timeout (status > 1) ends the script.
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
if [ "${PART:-all}" != b ]; then
step smoke 300 python __graft_entry__.py smoke || exit 1
step pytest 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step bench 600 python bench.py || exit 1
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --pcie 0 --cpu-seconds 0 || exit 1
cp profiles/pmc_parse_hash.json gpurun_out/pmc_parse_hash.json
for p in udp4 tcp4; do
    B="python bench.py --profile $p --steps 10 --warmup 3 --cpu-seconds 0 --check 0 --pcie 0"
    step pmc_fetch_$p 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$p -o run --output-format csv -- $B || exit 1
    step pmc_write_$p 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$p -o run --output-format csv -- $B || exit 1
    python tools/pmc_summary.py gpurun_out/pmc_fetch_$p gpurun_out/pmc_write_$p --profile $p \
        --out gpurun_out/pmc_parse_hash.json > gpurun_out/pmc_summary_$p.log 2>&1
done
fi
# PART=a stops here (the set in three gpurun calls: PART=a, b, c)
[ "${PART:-all}" = a ] && { echo "== done (part a)"; exit 0; }
if [ "${PART:-all}" = c ]; then
    # the 8-GPU configs, rehearsed on one device (8 ranks share it)
    step rehearse_n8_vlan6 620 bash tools/gpu_rehearse.sh 8 vlan6_tcp || exit 1
    step rehearse_n8_jumbo 620 bash tools/gpu_rehearse.sh 8 jumbo_tcp4 || exit 1
    step configs 900 python tools/configs_table.py || exit 1
    # last (a host SIGSEGV ends the call): can the host write device memory?
    # (bar_probe is no part of build(): built here, where it runs)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 tools/bar_probe.hip -o tools/bar_probe || exit 1
    for m in 0 1 2; do
        step bar_probe_$m 60 tools/bar_probe $m || exit 1
    done
    echo "== done (part c)"
    exit 0
fi
tools/build_ab_lib.sh prof -DYRSS_PROF_LINES=1 > /dev/null 2>&1 || exit 1
bash tools/gpu_r03_qrows.sh r04 || exit 1
if [ -f ab/lib/libyrss_prof.so ]; then   # the line scatter's phase clock (a YRSS_PROF_LINES build)
    step lineprof 200 python tools/line_prof.py --lib ab/lib/libyrss_prof.so --nb-procs 3,8,64,255 || exit 1
fi
bash tools/gpu_pmc.sh r04 "3 8 64 255" || exit 1
echo "== done"
