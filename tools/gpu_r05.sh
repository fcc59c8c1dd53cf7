#!/bin/bash
# Round-5 GPU steps, chosen by PART (each a separate gpurun call):
#   check  smoke, the GPU suite, the default bench line (headline + configs[3]/[4]
#          + CPU baseline + host-resident rows), the list-write pattern sweep
#   ab     same-process A/B of the tree against ablib/*.so (AB_LIBS, AB_Q)
# Each GPU step has its own time limit; a failure ends the script.
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
    tail -n 2 "gpurun_out/$name.log" | cut -c1-400
    return $rc
}
case "${PART:-check}" in
check)
    step smoke 300 python __graft_entry__.py smoke || exit 1
    step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
    step bench 600 python bench.py || exit 1
    : > gpurun_out/listbw.log
    for nb in 4 64 256; do
        for span in 8192 16384; do
            for wpc in 1 2; do
                for aux in 2 18; do
                    timeout -k 5 60 tools/list_write_bw 16777216 $nb $span $wpc $aux 20 \
                        >> gpurun_out/listbw.log 2>&1 || { echo "listbw rc=$?"; exit 1; }
                done
            done
        done
    done
    cat gpurun_out/listbw.log
    ;;
wide1)
    step tests_wide 400 python -u -m pytest tests/test_gpu_layout.py -x -q --timeout 120 \
        --timeout-method thread -k "wide or forced_line or capacity or bucket_counts" || exit 1
    step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
    step ab 900 python tools/ab_inproc.py --nb-procs "${AB_Q:-3,64,129,255}" \
        --libs "cur,ablib/libyrss_r05base.so" --rounds "${AB_ROUNDS:-6}" || exit 1
    step winab 600 python tools/win_ab.py || exit 1
    cat gpurun_out/ab.log gpurun_out/winab.log
    ;;
ab)
    step ab 900 python tools/ab_inproc.py --nb-procs "${AB_Q:-3,64,255}" --libs "${AB_LIBS}" \
        --rounds "${AB_ROUNDS:-6}" || exit 1
    cat gpurun_out/ab.log
    ;;
esac
echo "== done"
