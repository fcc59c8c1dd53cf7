#!/bin/bash
# Round 4: build library variants on the box (tools/build_ab_lib.sh), check
# each for parity (tools/quick_parity.py), then same-process A/B rounds
# (tools/ab_inproc.py).  Usage:
#   tools/gpu_r04_ab.sh TAG "name:-DMACRO=V ..." "AB_ARGS;AB_ARGS..." [parity 0|1]
# Each AB_ARGS is one ab_inproc.py argument string (';'-separated runs); the
# libs named NAME in it are ab/lib/libyrss_NAME.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1
variants=$2
runs=$3
parity=${4:-1}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
out=gpurun_out/ab_$tag.log
: > "$out"
for v in $variants; do
    name=${v%%:*}
    flags=${v#*:}
    tools/build_ab_lib.sh "$name" ${flags//,/ } >> "$out" 2>&1 || { echo "build $name failed"; exit 1; }
done
if [ "$parity" = 1 ]; then
    for v in $variants; do
        name=${v%%:*}
        echo "== parity $name" >> "$out"
        timeout -k 10 300 python tools/quick_parity.py --lib ab/lib/libyrss_$name.so > gpurun_out/parity_${tag}_$name.log 2>&1 \
            || { echo "parity $name rc=$?"; tail -n 5 gpurun_out/parity_${tag}_$name.log; exit 1; }
        tail -n 1 gpurun_out/parity_${tag}_$name.log >> "$out"
    done
fi
IFS=';' read -ra RUNS <<< "$runs"
for r in "${RUNS[@]}"; do
    echo "== ab $r" >> "$out"
    timeout -k 10 900 python tools/ab_inproc.py $r >> "$out" 2>&1 || { echo "ab rc=$?"; exit 1; }
done
echo "== done" >> "$out"
cat "$out" | grep -v "^round"
