# Where the hashed (TCP) path's time goes.  Diagnosis builds (-DYRSS_DIAG=bits,
# outputs wrong, so --check 0): 1 no table lookups, 2 no fastmod, 8 hash words
# written as 0, 4 one bucket (q = 2; the compiler then drops the whole hashed
# block), 32 one bucket with the hashed block kept, 16 UDP packets spread over
# two buckets (no hashed block); 128 few-bucket scatter with non-temporal
# per-lane stores.  The switches live in commit 4d8d485 (removed after).
# Build from that commit: for v in ...; do mkdir -p build/dg$v;
# hipcc <build() flags> -DYRSS_DIAG=$v ... -o build/dg$v/libyrss.so; done
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
V="YRSS_LIB=build/dg0/libyrss.so;YRSS_LIB=build/dg11/libyrss.so;YRSS_LIB=build/dg43/libyrss.so;YRSS_LIB=build/dg7/libyrss.so"
AB_VARIANTS="$V" AB_ROUNDS=3 BENCH_ARGS="--profile tcp4 --check 0" bash tools/gpu_ab.sh > gpurun_out/diag_tcp4.log 2>&1 || { cat gpurun_out/diag_tcp4.log; exit 1; }
V="YRSS_LIB=build/dg0/libyrss.so;YRSS_LIB=build/dg16/libyrss.so"
AB_VARIANTS="$V" AB_ROUNDS=3 BENCH_ARGS="--profile udp4 --check 0" bash tools/gpu_ab.sh > gpurun_out/diag_udp4.log 2>&1 || { cat gpurun_out/diag_udp4.log; exit 1; }
echo "== tcp4"; cat gpurun_out/diag_tcp4.log; echo "== udp4"; cat gpurun_out/diag_udp4.log
