# Persistent worker throughput vs workgroups (ring depth = 4 x workgroups), mbuf
# and frames submission.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for fr in 0 1; do
  for b in 4 16 32 64 128; do
    d=$((b * 4))
    YRSS_CBENCH_WORKER_FRAMES=$fr YRSS_CBENCH_MODES=4 YRSS_CBENCH_WORKER_DEPTH=$d YRSS_CBENCH_WORKER_BLOCKS=$b timeout -k 10 120 tools/yrss_cbench 1 1048576 0 1 > gpurun_out/cbw.log 2>&1 || { cat gpurun_out/cbw.log; exit 1; }
    python3 tools/cb_summary.py gpurun_out/cbw.log | sed "s/\$/  blocks $b/"
  done
done
