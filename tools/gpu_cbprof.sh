# Host-resident burst rates (tools/yrss_cbench): bursts 32 / 1024 / 32K with 1, 2
# and 4 bursts in flight (YRSS_F_ASYNC over that many contexts).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for b in 32 1024 32768; do
  for k in 1 2 4; do
    YRSS_CBENCH_INFLIGHT=$k YRSS_CBENCH_MODES=013 timeout -k 10 120 tools/yrss_cbench 1 262144 $b 1 > gpurun_out/cb_${b}_$k.log 2>&1 || { cat gpurun_out/cb_${b}_$k.log; exit 1; }
    python3 tools/cb_summary.py gpurun_out/cb_${b}_$k.log
  done
done
