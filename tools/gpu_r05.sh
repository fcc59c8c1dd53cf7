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
        --timeout-method thread -k "many_bucket or forced_line or capacity or bucket_counts" || exit 1
    step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
    step ab 900 python tools/ab_inproc.py --nb-procs "${AB_Q:-3,64,129,255}" \
        --libs "cur,${AB_BASE:-ablib/libyrss_r05base.so}" --rounds "${AB_ROUNDS:-6}" || exit 1
    step winab 600 python tools/win_ab.py || exit 1
    # write bytes: the bare list-write pattern, then the scatter at 255 queues
    for nb in 64 256; do
        timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_lw$nb -o run \
            --output-format csv -- tools/list_write_bw 16777216 $nb 8192 2 2 5 \
            > gpurun_out/pmc_lw$nb.log 2>&1 || { echo "pmc lw rc=$?"; exit 1; }
        python tools/pmc_kernels.py gpurun_out/pmc_lw$nb > gpurun_out/pmc_lw$nb.sum 2>&1
    done
    B="--profile tcp4 --nb-procs 255 --steps 5 --warmup 2 --cpu-seconds 0 --pcie 0 --check 0 --extra-configs="
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w255 -o run --output-format csv \
        -- python bench.py $B > gpurun_out/pmc_w255.log 2>&1 || { echo "pmc w255 rc=$?"; exit 1; }
    python tools/pmc_kernels.py gpurun_out/pmc_w255 > gpurun_out/pmc_w255.sum 2>&1
    cat gpurun_out/ab.log gpurun_out/winab.log gpurun_out/pmc_lw*.sum gpurun_out/pmc_w255.sum
    ;;
skel)
    : > gpurun_out/skel.log
    for cfg in "4 16384 1" "64 8192 2" "256 16384 1" "256 8192 2"; do
        set -- $cfg
        for rd in 0 1 2; do
            timeout -k 5 60 tools/list_write_bw 16777216 $1 $2 $3 2 20 $rd >> gpurun_out/skel.log 2>&1 \
                || { echo "skel rc=$?"; exit 1; }
        done
    done
    cat gpurun_out/skel.log
    step ab 900 python tools/ab_inproc.py --nb-procs "${AB_Q:-8,64,255}" \
        --libs "test,test@dbg_merge=1" --rounds "${AB_ROUNDS:-4}" || exit 1
    cat gpurun_out/ab.log
    for m in 0 1; do
        for q in 64 255; do
            B="--profile tcp4 --nb-procs $q --steps 5 --warmup 2 --cpu-seconds 0 --pcie 0 --check 0 --extra-configs= --test-hooks merge=$m"
            timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_m${m}_$q -o run --output-format csv \
                -- python bench.py $B > gpurun_out/pmc_m${m}_$q.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
            echo "== merge $m q$q"; python tools/pmc_kernels.py gpurun_out/pmc_m${m}_$q | grep -A2 scatter
        done
    done
    ;;
merge)
    step tests 400 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_worker.py -x -q \
        --timeout 120 --timeout-method thread -k "many_bucket or forced_line or capacity or merge or guard" || exit 1
    step ab 1200 python tools/ab_inproc.py --nb-procs "${AB_Q:-8,64,255}" \
        --libs "test,test@dbg_merge=1" --rounds "${AB_ROUNDS:-8}" || exit 1
    step winab 600 python tools/win_ab.py --pools 1048576,16384 || exit 1
    cat gpurun_out/ab.log gpurun_out/winab.log
    ;;
abl)
    # (round 5's ablation builds, YRSS_ABL_NOSTORE / _NOLOAD: their paths left
    # yrss.hip in round 6; the results are profiles/r05_lineprof_ablation.log)
    echo "PART=abl retired in round 6"; exit 2
    ;;
carry)
    step tests 600 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_small_burst.py -x -q \
        --timeout 120 --timeout-method thread || exit 1
    step ab 1200 python tools/ab_inproc.py --nb-procs "${AB_Q:-8,64,255}" \
        --libs "cur,${AB_BASE:-ablib/libyrss_r05base.so}" --rounds "${AB_ROUNDS:-6}" || exit 1
    cat gpurun_out/ab.log
    ;;
prof)
    # the line scatter's phase clock (a tools build with the test hooks)
    tools/build_ab_lib.sh prof -DYRSS_PROF_LINES=1 -DYRSS_TEST_HOOKS=1 > gpurun_out/build_prof.log 2>&1 || exit 1
    : > gpurun_out/lineprof.log
    for g in ${PROF_GROUPS:-0 4}; do
        timeout -k 10 200 python tools/line_prof.py --lib ab/lib/libyrss_prof.so \
            --nb-procs "${PROF_Q:-64,128,255}" --groups $g >> gpurun_out/lineprof.log 2>&1 || exit 1
    done
    cat gpurun_out/lineprof.log
    ;;
ab)
    step ab 900 python tools/ab_inproc.py --nb-procs "${AB_Q:-3,64,255}" --libs "${AB_LIBS}" \
        --rounds "${AB_ROUNDS:-6}" || exit 1
    cat gpurun_out/ab.log
    ;;
esac
echo "== done"
