#!/bin/bash
# Round-6: full-size (2^24) parity for every BASELINE stream, configs[3] and [4]
# with their own flow counts, then the whole GPU suite once more
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r06k_pytest.log 2>&1 || { tail -30 gpurun_out/r06k_pytest.log; exit 1; }
tail -1 gpurun_out/r06k_pytest.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k full_size --durations=0 \
    > gpurun_out/r06k_full_size.log 2>&1 || { tail -30 gpurun_out/r06k_full_size.log; exit 1; }
grep -E "passed|s call" gpurun_out/r06k_full_size.log | head -8
