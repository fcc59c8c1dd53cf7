# A/B of the single-list short path (bucket-seen mask; commit "Single-list short path (WIP"; removed after) against the
# full scan + scatter (YRSS_NO_MASK=1), after the GPU parity suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mask_pytest.log 2>&1 || { tail -30 gpurun_out/mask_pytest.log; exit 1; }
tail -2 gpurun_out/mask_pytest.log
for p in udp4 tcp4; do
  AB_VARIANTS="YRSS_NO_MASK=1;YRSS_NO_MASK=0" AB_ROUNDS=${AB_ROUNDS:-4} BENCH_ARGS="--profile $p" bash tools/gpu_ab.sh > gpurun_out/ab_mask_$p.log 2>&1 || { cat gpurun_out/ab_mask_$p.log; exit 1; }
  echo "== $p"; cat gpurun_out/ab_mask_$p.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mask_prof -o run --output-format csv -- python bench.py --cpu-seconds 0 --pcie 0 > gpurun_out/mask_prof.log 2>&1 || { tail gpurun_out/mask_prof.log; exit 1; }
cut -d, -f1-4 gpurun_out/mask_prof/run_kernel_stats.csv
