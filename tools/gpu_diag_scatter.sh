# Does the few-bucket scatter's plain-store output (64 MB of qidx left dirty in
# the caches) get written back during the NEXT parse kernel?  dg128 = the same
# build with non-temporal scatter stores (YRSS_DIAG, commit 4d8d485).  Parse µs (kernel_avg_us) and step
# time per variant, plus rocprof per-kernel stats of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
V="YRSS_LIB=build/dg0/libyrss.so;YRSS_LIB=build/dg128/libyrss.so"
AB_VARIANTS="$V" AB_ROUNDS=3 BENCH_ARGS="--profile tcp4" bash tools/gpu_ab.sh > gpurun_out/dscat_tcp4.log 2>&1 || { cat gpurun_out/dscat_tcp4.log; exit 1; }
cat gpurun_out/dscat_tcp4.log
for v in 0 128; do
  YRSS_LIB=build/dg$v/libyrss.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dscat_prof$v -o run --output-format csv -- python bench.py --profile tcp4 --cpu-seconds 0 --pcie 0 > gpurun_out/dscat_prof$v.log 2>&1 || { tail gpurun_out/dscat_prof$v.log; exit 1; }
  echo "== dg$v"; cut -d, -f1-4 gpurun_out/dscat_prof$v/run_kernel_stats.csv | head -6
done
