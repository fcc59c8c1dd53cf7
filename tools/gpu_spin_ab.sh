# Host-burst completion A/B: YRSS_SPIN_WAIT=1 (spin on the small kernel's
# completion word) vs 0 (hipStreamSynchronize), interleaved, on the three
# host APIs (cbench modes 0 1 3) at bursts 32 and 1024, one and two in flight.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for sw in 0 1; do
    for bk in "32 1" "32 2" "1024 1" "1024 2"; do
      set -- $bk
      YRSS_SPIN_WAIT=$sw YRSS_CBENCH_INFLIGHT=$2 YRSS_CBENCH_MODES=013 timeout -k 10 120 tools/yrss_cbench 1 262144 $1 1 > gpurun_out/ab.log 2>&1 || { cat gpurun_out/ab.log; exit 1; }
      python3 tools/cb_summary.py gpurun_out/ab.log | sed "s/\$/  spin $sw/"
    done
  done
done
