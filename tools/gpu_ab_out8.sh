# Parse output burst of 8 tiles (YRSS_PARSE_OUT_TILES=8 build, needs 8-tile chunks)
# Requires the YRSS_PARSE_OUT_TILES build from commit 7115730 (removed from the source afterwards).
# against the default 4, with 8-tile chunks on the default build as the control.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_default.log 2>&1 || { tail -20 gpurun_out/pytest_default.log; exit 1; }
tail -1 gpurun_out/pytest_default.log
YRSS_LIB=build/out8/libyrss.so YRSS_CHUNK_TILES=8 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_out8.log 2>&1 || { tail -20 gpurun_out/pytest_out8.log; exit 1; }
tail -1 gpurun_out/pytest_out8.log
V="YRSS_NT=1;YRSS_CHUNK_TILES=8;YRSS_LIB=build/out8/libyrss.so YRSS_CHUNK_TILES=8"
AB_VARIANTS="$V" AB_ROUNDS=4 BENCH_ARGS="--profile udp4" bash tools/gpu_ab.sh > gpurun_out/ab_out8_udp.log 2>&1 || { cat gpurun_out/ab_out8_udp.log; exit 1; }
AB_VARIANTS="$V" AB_ROUNDS=2 BENCH_ARGS="--profile tcp4" bash tools/gpu_ab.sh > gpurun_out/ab_out8_tcp.log 2>&1 || { cat gpurun_out/ab_out8_tcp.log; exit 1; }
cat gpurun_out/ab_out8_udp.log gpurun_out/ab_out8_tcp.log
