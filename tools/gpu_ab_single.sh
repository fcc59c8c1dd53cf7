# A/B of the scatter's one-list path (grid-stride identity stores when a
# batch's totals show a single non-empty list; default) against the group
# path (YRSS_NO_SINGLE=1), after the GPU parity suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/single_pytest.log 2>&1 || { tail -30 gpurun_out/single_pytest.log; exit 1; }
tail -2 gpurun_out/single_pytest.log
AB_VARIANTS="YRSS_NO_SINGLE=1;YRSS_NO_SINGLE=0" AB_ROUNDS=${AB_ROUNDS:-5} BENCH_ARGS="--profile udp4" bash tools/gpu_ab.sh > gpurun_out/ab_single.log 2>&1 || { cat gpurun_out/ab_single.log; exit 1; }
cat gpurun_out/ab_single.log
for v in 1 0; do
  YRSS_NO_SINGLE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/single_prof$v -o run --output-format csv -- python bench.py --cpu-seconds 0 --pcie 0 > gpurun_out/single_prof$v.log 2>&1 || { tail gpurun_out/single_prof$v.log; exit 1; }
  echo "== YRSS_NO_SINGLE=$v"; grep -E "scatter|seg_scan|parse_hash" gpurun_out/single_prof$v/run_kernel_stats.csv | cut -d, -f1-4
done
