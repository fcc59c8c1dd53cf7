# The new default scatter group (32 tiles when nb <= 8, image slack by nb)
# against 64 tiles: GPU tests on the default, then udp4 / tcp4 / imix A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/group2_pytest.log 2>&1 || { tail -30 gpurun_out/group2_pytest.log; exit 1; }
tail -1 gpurun_out/group2_pytest.log
for p in udp4 tcp4 imix; do
  AB_VARIANTS="YRSS_GROUP_TILES=64;YRSS_GROUP_TILES=0" AB_ROUNDS=3 BENCH_ARGS="--profile $p" bash tools/gpu_ab.sh > gpurun_out/ab_group2_$p.log 2>&1 || { cat gpurun_out/ab_group2_$p.log; exit 1; }
  echo "== $p"; cat gpurun_out/ab_group2_$p.log
done
