# round-6 call: GPU tests of the paths the in-scatter prefixes touch, A/B
# against the scan kernel, the phase clock at q3/q8, the N=8 rehearsal
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_worker.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_pytest_part.log 2>&1 || { tail -30 gpurun_out/r06_pytest_part.log; exit 1; }
tail -2 gpurun_out/r06_pytest_part.log
PART=ab AB_TAG=bins AB_PROFILES="imix udp4" AB_NB=3,8 bash tools/gpu_r06.sh || exit 1
tools/build_ab_lib.sh prof -DYRSS_PROF_LINES=1 > gpurun_out/build_prof.log 2>&1 || exit 1
timeout -k 10 200 python tools/line_prof.py --lib ab/lib/libyrss_prof.so --nb-procs 3,8 > gpurun_out/r06_lineprof_bins.log 2>&1 || exit 1
grep -E "^q|entry|span total|   b |   c |wait" gpurun_out/r06_lineprof_bins.log
PART=n8 bash tools/gpu_r06.sh || exit 1
grep -c "device fault" gpurun_out/r06_n8_one_device_full.log || true
