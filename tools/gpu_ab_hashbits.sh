# A/B of the Toeplitz table field width: byte tables (12 lookups, bank
# conflicts) vs nibble tables (24 conflict-free lookups).  Build first:
#   for v in 8 4; do mkdir -p build/hb$v; hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC \
#     -shared -DYRSS_HASH_BITS=$v -I include yastack_amd/csrc/yrss.hip yastack_amd/csrc/yrss_pcap.cpp \
#     yastack_amd/csrc/yrss_shard.cpp -o build/hb$v/libyrss.so; done
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
YRSS_LIB=build/hb4/libyrss.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/hb4_pytest.log 2>&1 || { tail -30 gpurun_out/hb4_pytest.log; exit 1; }
tail -2 gpurun_out/hb4_pytest.log
V="YRSS_LIB=build/hb8/libyrss.so;YRSS_LIB=build/hb4/libyrss.so"
for p in tcp4 udp4 imix; do
  AB_VARIANTS="$V" AB_ROUNDS=${AB_ROUNDS:-3} BENCH_ARGS="--profile $p" bash tools/gpu_ab.sh > gpurun_out/ab_hb_$p.log 2>&1 || { cat gpurun_out/ab_hb_$p.log; exit 1; }
  echo "== $p"; cat gpurun_out/ab_hb_$p.log
done
for v in 8 4; do
  YRSS_LIB=build/hb$v/libyrss.so bash tools/gpu_lds_pmc.sh > gpurun_out/lds_hb$v.log 2>&1 || { tail -20 gpurun_out/lds_hb$v.log; exit 1; }
  echo "== LDS counters hb$v"; cat gpurun_out/lds_hb$v.log
done
