# Persistent worker at 32-packet bursts: outputs per ring slot (F-Stack's
# pattern, output addresses cached by the workgroups) vs outputs following the
# packets (addresses change every burst), mbufs and frames.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for fr in 1 0; do
  for b in 16 64 128; do
    for so in 0 1; do
      d=$((b * 4))
      YRSS_CBENCH_WORKER_SLOTOUT=$so YRSS_CBENCH_WORKER_FRAMES=$fr YRSS_CBENCH_MODES=4 YRSS_CBENCH_WORKER_DEPTH=$d YRSS_CBENCH_WORKER_BLOCKS=$b timeout -k 10 120 tools/yrss_cbench 1 1048576 32 1 > gpurun_out/cbw.log 2>&1 || { cat gpurun_out/cbw.log; exit 1; }
      python3 tools/cb_summary.py gpurun_out/cbw.log | sed "s/\$/  blocks $b slotout $so/"
    done
  done
done
