#!/bin/bash
# Round-3 measurement set: smoke; every GPU test; the bench (headline, with the PCIe rows and
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
# PART=a stops here (the set in two gpurun calls: PART=a, then PART=b)
[ "${PART:-all}" = a ] && { echo "== done (part a)"; exit 0; }
bash tools/gpu_r03_qrows.sh r03 || exit 1
if [ -f ab/lib/libyrss_prof7.so ]; then   # the line scatter's phase clock (a YRSS_PROF_LINES build)
    step lineprof 200 python tools/line_prof.py --lib ab/lib/libyrss_prof7.so --nb-procs 3,8,64,255 || exit 1
fi
bash tools/gpu_pmc.sh r03 "3 8 64 255" || exit 1
echo "== done"
