# Device-wide worker yield: the worker GPU tests, then the batch latency with
# and without it (tools/yield_check.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py -k preempt -x -q --timeout 120 --timeout-method thread > gpurun_out/yield_pytest.log 2>&1 || { tail -40 gpurun_out/yield_pytest.log; exit 1; }
tail -2 gpurun_out/yield_pytest.log
for f in "" --filter; do
  timeout -k 10 120 python tools/yield_check.py $f > gpurun_out/yield_on.log 2>&1 || { tail gpurun_out/yield_on.log; exit 1; }
  YRSS_NO_YIELD=1 timeout -k 10 120 python tools/yield_check.py $f > gpurun_out/yield_off.log 2>&1 || { tail gpurun_out/yield_off.log; exit 1; }
  tail -1 gpurun_out/yield_on.log; tail -1 gpurun_out/yield_off.log
done
