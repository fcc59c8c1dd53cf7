# A/B of the hash split between LDS byte tables and VALU bit-serial words.
# Build the variants first, on the CPU side:
#   for v in 0 1 2 3; do mkdir -p build/vw$v; hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC \
#     -shared -DYRSS_VALU_WORDS=$v -I include yastack_amd/csrc/yrss.hip yastack_amd/csrc/yrss_pcap.cpp \
#     yastack_amd/csrc/yrss_shard.cpp -o build/vw$v/libyrss.so; done
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V="YRSS_LIB=build/vw0/libyrss.so;YRSS_LIB=build/vw1/libyrss.so;YRSS_LIB=build/vw2/libyrss.so;YRSS_LIB=build/vw3/libyrss.so"
AB_VARIANTS="$V" AB_ROUNDS=3 BENCH_ARGS="--profile tcp4" bash tools/gpu_ab.sh > gpurun_out/ab_tcp.log 2>&1 || { cat gpurun_out/ab_tcp.log; exit 1; }
AB_VARIANTS="$V" AB_ROUNDS=2 BENCH_ARGS="--profile udp4" bash tools/gpu_ab.sh > gpurun_out/ab_udp.log 2>&1 || { cat gpurun_out/ab_udp.log; exit 1; }
cat gpurun_out/ab_tcp.log gpurun_out/ab_udp.log
