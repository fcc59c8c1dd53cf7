# Host-resident burst latency: cbench at bursts 32 / 1024 (+ pool-size and THP
# variants of the zero-copy mbuf path), then a kernel/API trace of burst_zc.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for b in 32 1024; do
  YRSS_CBENCH_MODES=013 timeout -k 10 120 tools/yrss_cbench 1 65536 $b 1 > gpurun_out/cb$b.log 2>&1 || { cat gpurun_out/cb$b.log; exit 1; }
  cat gpurun_out/cb$b.log | cut -c1-190
done
for pool in 2048 1048576; do
  YRSS_CBENCH_MODES=1 timeout -k 10 120 tools/yrss_cbench 1 $pool 1024 1 | cut -c1-170
done
YRSS_CBENCH_THP=0 YRSS_CBENCH_MODES=1 timeout -k 10 120 tools/yrss_cbench 1 65536 1024 1 | cut -c1-170
YRSS_NO_SMALL=1 YRSS_CBENCH_MODES=013 timeout -k 10 120 tools/yrss_cbench 1 65536 1024 1 | cut -c1-170
YRSS_CBENCH_MODES=1 timeout -k 10 200 rocprofv3 --kernel-trace --runtime-trace -d gpurun_out/cbprof -o run --output-format csv -- tools/yrss_cbench 1 65536 1024 1 > gpurun_out/cbprof.log 2>&1 || { tail gpurun_out/cbprof.log; exit 1; }
