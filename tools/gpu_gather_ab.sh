# Host-gather A/B: yrss_dispatch_burst (mode 0) with the library under
# build/old (LD_LIBRARY_PATH overrides cbench's RUNPATH) against the in-tree
# one, interleaved, bursts 1024 / 32K / 1M.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for lib in old new; do
    for bk in "1024 1" "1024 2" "32768 1" "32768 2" "1048576 1"; do
      set -- $bk
      if [ $lib = old ]; then lp="$PWD/build/old"; else lp="$PWD/yastack_amd/_lib"; fi
      LD_LIBRARY_PATH="$lp" YRSS_CBENCH_INFLIGHT=$2 YRSS_CBENCH_MODES=${MODES:-0} timeout -k 10 120 tools/yrss_cbench 1 1048576 $1 1 > gpurun_out/ab.log 2>&1 || { cat gpurun_out/ab.log; exit 1; }
      python3 tools/cb_summary.py gpurun_out/ab.log | sed "s/\$/  $lib/"
    done
  done
done
