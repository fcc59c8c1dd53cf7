# Persistent worker throughput vs workgroups (ring depth = 4 x workgroups).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for b in 2 4 8 16 32; do
  d=$((b * 4))
  YRSS_CBENCH_MODES=4 YRSS_CBENCH_WORKER_DEPTH=$d YRSS_CBENCH_WORKER_BLOCKS=$b timeout -k 10 120 tools/yrss_cbench 1 1048576 0 1 > gpurun_out/cbw.log 2>&1 || { cat gpurun_out/cbw.log; exit 1; }
  python3 tools/cb_summary.py gpurun_out/cbw.log | sed "s/\$/  blocks $b/"
done
for p in 5 2; do
  YRSS_CBENCH_MODES=4 YRSS_CBENCH_WORKER_DEPTH=64 YRSS_CBENCH_WORKER_BLOCKS=16 timeout -k 10 120 tools/yrss_cbench $p 1048576 0 1 > gpurun_out/cbw.log 2>&1 || { cat gpurun_out/cbw.log; exit 1; }
  python3 tools/cb_summary.py gpurun_out/cbw.log | sed "s/\$/  blocks 16 profile $p/"
done
