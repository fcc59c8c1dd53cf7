#!/bin/bash
# Round-6: configs_extra measured like the headline (four rotated batches,
# 50 steps) against the same config as the headline (configs table's form)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --pcie 0 --cpu-seconds 0 --extra-configs=imix,jumbo_tcp4 > gpurun_out/r06j_bench_extra.log 2>&1 || { tail -20 gpurun_out/r06j_bench_extra.log; exit 1; }
grep configs_extra gpurun_out/r06j_bench_extra.log | cut -c1-330
for p in imix jumbo_tcp4; do
    timeout -k 10 300 python bench.py --profile $p --pcie 0 --cpu-seconds 0 --extra-configs= > gpurun_out/r06j_bench_$p.log 2>&1 || { tail -20 gpurun_out/r06j_bench_$p.log; exit 1; }
    tail -1 gpurun_out/r06j_bench_$p.log | grep -o '"value": [0-9.]*, "unit": "Mpkt/s", "n_gpus": 1, "steps": 50, "warmup": 50, "ms_per_step": [0-9.]*'
done
