# round-6 call: quick parity + A/B of in-scatter prefixes against the scan kernel
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_layout.py -x -q --timeout 120 --timeout-method thread -k "in_scatter or bucket_counts or forced" > gpurun_out/r06_pytest_quick.log 2>&1 || { tail -30 gpurun_out/r06_pytest_quick.log; exit 1; }
tail -1 gpurun_out/r06_pytest_quick.log
PART=ab AB_TAG=${TAG:-c4} AB_PROFILES="${PROFS:-udp4 imix}" AB_NB=${NBS:-3} bash tools/gpu_r06.sh || exit 1
tools/build_ab_lib.sh prof -DYRSS_PROF_LINES=1 > gpurun_out/build_prof.log 2>&1 || exit 1
for sk in 0 1; do
  timeout -k 10 200 python tools/line_prof.py --lib ab/lib/libyrss_prof.so --nb-procs 3 --scan-kernel $sk > gpurun_out/r06_lineprof_${TAG:-c4}_sk$sk.log 2>&1 || exit 1
  grep -E "^q|entry|span total|prologue|   b |   c |wait" gpurun_out/r06_lineprof_${TAG:-c4}_sk$sk.log
done
