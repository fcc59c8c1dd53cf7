# A/B of two VALU trims on the hashed path: power-of-two modulo as a mask
# (YRSS_MOD_POW2) and SDWA byte-address forms (YRSS_SDWA=1, =2 base-free LDS).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V="${AB_V:?set AB_V to YRSS_LIB=... variants built from commit caf6010}"
AB_VARIANTS="$V" AB_ROUNDS=${AB_TCP_ROUNDS:-3} BENCH_ARGS="--profile tcp4" bash tools/gpu_ab.sh > gpurun_out/ab_ops_tcp.log 2>&1 || { cat gpurun_out/ab_ops_tcp.log; exit 1; }
AB_VARIANTS="$V" AB_ROUNDS=${AB_UDP_ROUNDS:-2} BENCH_ARGS="--profile udp4" bash tools/gpu_ab.sh > gpurun_out/ab_ops_udp.log 2>&1 || { cat gpurun_out/ab_ops_udp.log; exit 1; }
cat gpurun_out/ab_ops_tcp.log gpurun_out/ab_ops_udp.log
