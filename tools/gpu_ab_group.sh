# A/B of the scatter group size (YRSS_GROUP_TILES: 64 = 4096-packet groups,
# 18 KB LDS image per wave, 2 workgroups per CU; 32 and 16 halve it) on the
# few-bucket LDS-image path, after the scatter/layout GPU tests on each size.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
for g in 32 16; do
  YRSS_GROUP_TILES=$g timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py -x -q --timeout 120 --timeout-method thread > gpurun_out/group_pytest_$g.log 2>&1 || { tail -30 gpurun_out/group_pytest_$g.log; exit 1; }
  tail -1 gpurun_out/group_pytest_$g.log
done
for p in tcp4 imix; do
  AB_VARIANTS="YRSS_GROUP_TILES=64;YRSS_GROUP_TILES=32;YRSS_GROUP_TILES=16" AB_ROUNDS=3 BENCH_ARGS="--profile $p" bash tools/gpu_ab.sh > gpurun_out/ab_group_$p.log 2>&1 || { cat gpurun_out/ab_group_$p.log; exit 1; }
  echo "== $p"; cat gpurun_out/ab_group_$p.log
done
for g in 64 32 16; do
  YRSS_GROUP_TILES=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/group_prof$g -o run --output-format csv -- python bench.py --profile tcp4 --cpu-seconds 0 --pcie 0 > gpurun_out/group_prof$g.log 2>&1 || { tail gpurun_out/group_prof$g.log; exit 1; }
  echo "== rocprof tcp4 GROUP_TILES=$g"; grep -E "scatter|seg_scan" gpurun_out/group_prof$g/run_kernel_stats.csv | cut -d, -f1-4
done
