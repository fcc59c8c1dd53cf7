# Host gather into pinned staging with non-temporal stores (YRSS_GATHER_NT=1,
# default) vs plain memcpy (0): yrss_dispatch_burst in tools/yrss_cbench (mode
# 0), one and two bursts in flight; the host-burst GPU tests and a short burst
# soak first (SKIP_TESTS=1 skips them).  Measured and not kept:
# YRSS_GATHER_NT is no longer in the source.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_small_burst.py tests/test_gpu_parity.py tests/test_gpu_register.py > gpurun_out/gnt_pytest.log 2>&1 || { tail -40 gpurun_out/gnt_pytest.log; exit 1; }
tail -1 gpurun_out/gnt_pytest.log
timeout -k 10 120 python tools/burst_soak.py --seconds 20 > gpurun_out/gnt_soak.log 2>&1 || { tail gpurun_out/gnt_soak.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gnt_soak.log | tail -1
fi
for rep in 1 2; do
  for inf in 1 2; do
    for nt in 0 1; do
      YRSS_GATHER_NT=$nt YRSS_CBENCH_MODES=0 YRSS_CBENCH_INFLIGHT=$inf timeout -k 10 120 tools/yrss_cbench 1 1048576 0 1.5 > gpurun_out/gnt.log 2>&1 || { tail gpurun_out/gnt.log; exit 1; }
      echo "r$rep nt=$nt: $(python3 tools/cb_summary.py gpurun_out/gnt.log | tr '\n' ';')"
    done
  done
done
