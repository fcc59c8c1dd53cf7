# One-launch bursts (<= 4096 packets) and the worker: per-queue lists built in
# LDS and copied out contiguously (default, YRSS_SMALL_IMG=1) vs per-lane
# stores into the lists (build/si0: -DYRSS_SMALL_IMG=0); the small-burst and
# worker GPU tests on the default build first.  Measured and not kept:
# YRSS_SMALL_IMG is no longer in the source.
#   mkdir -p build/si0; hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DYRSS_SMALL_IMG=0 \
#     -I include yastack_amd/csrc/yrss.hip yastack_amd/csrc/yrss_pcap.cpp yastack_amd/csrc/yrss_shard.cpp \
#     yastack_amd/csrc/yrss_fanout.cpp -o build/si0/libyrss.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_small_burst.py tests/test_gpu_worker.py tests/test_gpu_register.py tests/test_gpu_fanout.py > gpurun_out/si_pytest.log 2>&1 || { tail -40 gpurun_out/si_pytest.log; exit 1; }
tail -1 gpurun_out/si_pytest.log
for rep in 1 2; do
  for B in 32 1024 4096; do
    for v in new old; do
      lp=""; [ $v = old ] && lp="$PWD/build/si0"
      LD_LIBRARY_PATH=$lp YRSS_CBENCH_MODES=03 YRSS_CBENCH_INFLIGHT=2 timeout -k 10 120 tools/yrss_cbench 1 1048576 $B 1 > gpurun_out/si.log 2>&1 || { tail gpurun_out/si.log; exit 1; }
      echo "r$rep $v burst $B: $(python3 tools/cb_summary.py gpurun_out/si.log | tr '\n' ';')"
    done
  done
  for B in 32 1024; do
    for v in new old; do
      lp=""; [ $v = old ] && lp="$PWD/build/si0"
      LD_LIBRARY_PATH=$lp YRSS_CBENCH_MODES=4 YRSS_CBENCH_WORKER_FRAMES=1 YRSS_CBENCH_WORKER_BLOCKS=$([ $B = 32 ] && echo 128 || echo 32) timeout -k 10 120 tools/yrss_cbench 1 1048576 $B 1 > gpurun_out/si.log 2>&1 || { tail gpurun_out/si.log; exit 1; }
      echo "r$rep $v worker frames burst $B: $(python3 tools/cb_summary.py gpurun_out/si.log | tr '\n' ';')"
    done
  done
done
