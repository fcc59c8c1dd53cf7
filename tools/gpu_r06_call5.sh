# round-6 call: the line scatter's prologue milestones, in-scatter prefixes
# against the scan kernel, 4 buckets
set -o pipefail
tools/build_ab_lib.sh prof -DYRSS_PROF_LINES=1 > gpurun_out/build_prof.log 2>&1 || exit 1
for sk in 0 1; do
  timeout -k 10 200 python tools/line_prof.py --lib ab/lib/libyrss_prof.so --nb-procs 3 --scan-kernel $sk > gpurun_out/r06_lineprof_pro$sk.log 2>&1 || exit 1
  grep -E "^q|entry|span total|prologue" gpurun_out/r06_lineprof_pro$sk.log
done
