#!/bin/bash
# Round-6: the default bench line (configs_extra now holds configs[2] IMIX too), timed
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
t0=$(date +%s%N)
timeout -k 10 600 python bench.py > gpurun_out/r06i_bench.log 2>&1 || { tail -20 gpurun_out/r06i_bench.log; exit 1; }
t1=$(date +%s%N)
echo "wall_s $(( (t1 - t0) / 1000000 ))e-3" | tee -a gpurun_out/r06i_bench.log
grep configs_extra gpurun_out/r06i_bench.log | cut -c1-400
