# Occupancy A/B of the parse kernel: 8 resident waves per CU (default) against 12
# and 16, with the LDS cap taken for the filter-off kernel (YRSS_LDS_BLOCKS).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V="YRSS_WAVES_PER_CU=8;YRSS_LDS_BLOCKS=2 YRSS_WAVES_PER_CU=16;YRSS_LDS_BLOCKS=3 YRSS_WAVES_PER_CU=12 YRSS_BLOCK=256"
AB_VARIANTS="$V" AB_ROUNDS=3 BENCH_ARGS="--profile tcp4" bash tools/gpu_ab.sh > gpurun_out/ab_occ_tcp.log 2>&1 || { cat gpurun_out/ab_occ_tcp.log; exit 1; }
AB_VARIANTS="$V" AB_ROUNDS=3 BENCH_ARGS="--profile udp4" bash tools/gpu_ab.sh > gpurun_out/ab_occ_udp.log 2>&1 || { cat gpurun_out/ab_occ_udp.log; exit 1; }
cat gpurun_out/ab_occ_tcp.log gpurun_out/ab_occ_udp.log
