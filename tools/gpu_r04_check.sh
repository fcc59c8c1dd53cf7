#!/bin/bash
# Round 4: GPU suite, then same-process A/B of the tree's library against
# prebuilt variants in abl/ (tools/ab_inproc.py), then optional extra steps.
#   tools/gpu_r04_check.sh TAG "AB_ARGS;AB_ARGS..." [tests 0|1]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1
runs=${2:-}
tests=${3:-1}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
out=gpurun_out/chk_$tag.log
: > "$out"
if [ "$tests" = 1 ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > gpurun_out/pytest_$tag.log 2>&1 || { echo "pytest rc=$?"; tail -n 30 gpurun_out/pytest_$tag.log; exit 1; }
    tail -n 3 gpurun_out/pytest_$tag.log >> "$out"
fi
IFS=';' read -ra RUNS <<< "$runs"
for r in "${RUNS[@]}"; do
    [ -z "$r" ] && continue
    echo "== ab $r" >> "$out"
    timeout -k 10 900 python tools/ab_inproc.py $r >> "$out" 2>&1 || { echo "ab rc=$?"; tail -n 20 "$out"; exit 1; }
done
echo "== done" >> "$out"
grep -v "^round\|amdgpu.ids" "$out"
