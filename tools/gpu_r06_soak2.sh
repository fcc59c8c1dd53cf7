#!/bin/bash
# Round-6 extra robustness at the final HEAD: 200 random large batches
# (2^17-2^21 packets; prefix form, XCD mapping and parse grid drawn), another seed
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
YRSS_FUZZ_CASES=0 YRSS_FUZZ_LARGE_CASES=200 YRSS_FUZZ_SEED=7 timeout -k 10 1000 \
    python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k large > gpurun_out/r06_fuzz_large200.log 2>&1 || { tail -30 gpurun_out/r06_fuzz_large200.log; exit 1; }
tail -1 gpurun_out/r06_fuzz_large200.log
