#!/bin/bash
# Round-6 last check at the final HEAD: smoke, the whole GPU suite (455 tests,
# the large-batch fuzz included), the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r06h_smoke.log 2>&1 || { tail -20 gpurun_out/r06h_smoke.log; exit 1; }
tail -1 gpurun_out/r06h_smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r06h_pytest.log 2>&1 || { tail -30 gpurun_out/r06h_pytest.log; exit 1; }
tail -1 gpurun_out/r06h_pytest.log
timeout -k 10 600 python bench.py > gpurun_out/r06h_bench.log 2>&1 || { tail -20 gpurun_out/r06h_bench.log; exit 1; }
tail -1 gpurun_out/r06h_bench.log | cut -c1-400
