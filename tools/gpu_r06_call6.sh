# round-6 call: parity subset, then a same-process A/B of the tree against a
# saved library (AB_BASE), and the phase clock at 4 buckets
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_layout.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_pytest_quick.log 2>&1 || { tail -30 gpurun_out/r06_pytest_quick.log; exit 1; }
tail -1 gpurun_out/r06_pytest_quick.log
for prof in ${PROFS:-imix tcp4}; do
  timeout -k 10 500 python -u tools/ab_inproc.py --nb-procs "${NBS:-3,8,64}" --libs "cur,${AB_BASE}" --rounds ${ROUNDS:-6} --profile $prof > gpurun_out/r06_ab_${TAG}_$prof.log 2>&1 || { tail -20 gpurun_out/r06_ab_${TAG}_$prof.log; exit 1; }
  grep "^q" gpurun_out/r06_ab_${TAG}_$prof.log
done
tools/build_ab_lib.sh prof -DYRSS_PROF_LINES=1 > gpurun_out/build_prof.log 2>&1 || exit 1
timeout -k 10 200 python tools/line_prof.py --lib ab/lib/libyrss_prof.so --nb-procs 3,64 > gpurun_out/r06_lineprof_${TAG}.log 2>&1 || exit 1
grep -E "^q|entry|span total|prologue|   b |   c |wait|   d " gpurun_out/r06_lineprof_${TAG}.log
