#!/bin/bash
# Round-6 robustness at the final HEAD, every result checked against the
# oracle: 400 random small configurations and 40 random large batches (many
# spans and scatter ranges; prefix form, XCD mapping and parse grid drawn),
# then the host-burst, worker and fan-out soaks, 30 s each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
YRSS_FUZZ_CASES=400 YRSS_FUZZ_LARGE_CASES=40 YRSS_FUZZ_SEED=2026 timeout -k 10 900 \
    python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r06_fuzz_soak.log 2>&1 || { tail -30 gpurun_out/r06_fuzz_soak.log; exit 1; }
tail -2 gpurun_out/r06_fuzz_soak.log
for s in burst worker fanout; do
    timeout -k 10 300 python -u tools/${s}_soak.py --seconds 30 > gpurun_out/r06_${s}_soak.log 2>&1 \
        || { tail -20 gpurun_out/r06_${s}_soak.log; exit 1; }
    tail -1 gpurun_out/r06_${s}_soak.log | cut -c1-300
done
