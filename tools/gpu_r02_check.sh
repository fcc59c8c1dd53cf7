# Round-2 check: fan-out and beside-a-worker GPU tests, the default bench, and
# the N=2 launch rehearsed on one device (bench.py --gpus 2 spawns its ranks).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fanout.py tests/test_gpu_worker.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest.log 2>&1 || { tail -40 gpurun_out/r02_pytest.log; exit 1; }
tail -2 gpurun_out/r02_pytest.log
timeout -k 10 600 python bench.py > gpurun_out/r02_bench.log 2>&1 || { tail -20 gpurun_out/r02_bench.log; exit 1; }
tail -1 gpurun_out/r02_bench.log | cut -c1-600
YRSS_BENCH_ONE_DEVICE=1 timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/r02_bench_n2.log 2>&1 || { tail -20 gpurun_out/r02_bench_n2.log; exit 1; }
grep '^{"metric"' gpurun_out/r02_bench_n2.log | cut -c1-400
grep -o '"pcie_fanout".*' gpurun_out/r02_bench.log gpurun_out/r02_bench_n2.log | cut -c1-700
