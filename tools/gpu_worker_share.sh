# A device batch beside another context's / process's resident worker: the
# worker GPU tests for it, then the latencies (tools/yield_check.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py -k beside -x -q --timeout 120 --timeout-method thread > gpurun_out/share_pytest.log 2>&1 || { tail -40 gpurun_out/share_pytest.log; exit 1; }
tail -2 gpurun_out/share_pytest.log
for f in "" --filter; do
  timeout -k 10 120 python tools/yield_check.py $f > gpurun_out/share.log 2>&1 || { tail gpurun_out/share.log; exit 1; }
  tail -1 gpurun_out/share.log
done
