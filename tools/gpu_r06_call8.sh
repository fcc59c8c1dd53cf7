# round-6 call: phase clock of the line scatter on IMIX (one bucket holds every
# UDP packet) against all-TCP, 65 and 256 buckets
set -o pipefail
tools/build_ab_lib.sh prof -DYRSS_PROF_LINES=1 > gpurun_out/build_prof.log 2>&1 || exit 1
for pr in imix tcp4; do
  timeout -k 10 200 python tools/line_prof.py --lib ab/lib/libyrss_prof.so --nb-procs ${NBS:-64,255} --profile $pr > gpurun_out/r06_lineprof_skew_$pr.log 2>&1 || exit 1
  grep -E "^q|   b|   c |wait|   d |span total|p50" gpurun_out/r06_lineprof_skew_$pr.log
done
