# A/B of the few-bucket scatter's LDS list image (default) against per-lane
# plain stores (YRSS_NO_IMG=1), after the GPU parity suite on the new build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/img_pytest.log 2>&1 || { tail -30 gpurun_out/img_pytest.log; exit 1; }
tail -2 gpurun_out/img_pytest.log
for p in tcp4 imix udp4; do
  AB_VARIANTS="YRSS_NO_IMG=1;YRSS_NO_IMG=0" AB_ROUNDS=${AB_ROUNDS:-3} BENCH_ARGS="--profile $p" bash tools/gpu_ab.sh > gpurun_out/ab_img_$p.log 2>&1 || { cat gpurun_out/ab_img_$p.log; exit 1; }
  echo "== $p"; cat gpurun_out/ab_img_$p.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/img_prof -o run --output-format csv -- python bench.py --profile tcp4 --cpu-seconds 0 --pcie 0 > gpurun_out/img_prof.log 2>&1 || { tail gpurun_out/img_prof.log; exit 1; }
cut -d, -f1-4 gpurun_out/img_prof/run_kernel_stats.csv
