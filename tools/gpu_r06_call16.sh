#!/bin/bash
# round-6 call: what the in-scatter prefixes cost the parse kernel (its tail:
# per-workgroup bucket sums and device-scope atomics into the totals and the
# range bins), 12 rounds, scan_kernel 0 (in-scatter) against 1 (scan kernel)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${TAG:-c19}
for prof in tcp4 imix udp4; do
    timeout -k 10 500 python -u tools/ab_inproc.py --nb-procs 3 --libs cur@scan_kernel=0,cur@scan_kernel=1 \
        --rounds 12 --profile $prof > gpurun_out/r06_ab_${T}_$prof.log 2>&1 || { tail -20 gpurun_out/r06_ab_${T}_$prof.log; exit 1; }
    grep -E '^q[0-9]' gpurun_out/r06_ab_${T}_$prof.log
done
