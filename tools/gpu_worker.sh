# Persistent worker: parity tests, then cbench worker mode at bursts 32 / 1024
# with several ring depths.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py -m gpu -v -x --timeout 120 --timeout-method thread > gpurun_out/pt_worker.log 2>&1
rc=$?; tail -8 gpurun_out/pt_worker.log; [ $rc -eq 0 ] || exit $rc
for d in 4 16 64; do
  for b in 1 4; do
    YRSS_CBENCH_MODES=4 YRSS_CBENCH_WORKER_DEPTH=$d YRSS_CBENCH_WORKER_BLOCKS=$b timeout -k 10 120 tools/yrss_cbench 1 262144 0 1 > gpurun_out/cbw.log 2>&1 || { cat gpurun_out/cbw.log; exit 1; }
    python3 tools/cb_summary.py gpurun_out/cbw.log | sed "s/\$/  blocks $b/"
  done
done
