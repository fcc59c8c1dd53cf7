#!/bin/bash
# Round 3: the all-TCP step at 3/8/64/255 queues, each
# row once as a plain bench line and once under rocprofv3 --kernel-trace
# --stats (per-kernel averages).  Usage: tools/gpu_r03_qrows.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-base}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
out=gpurun_out/qrows_$tag.log
: > "$out"
for np in 3 8 64 255; do
    B="--profile tcp4 --nb-procs $np --steps 30 --warmup 10 --cpu-seconds 0 --pcie 0 --check 1048576 --extra-configs="
    echo "== q$np bench" | tee -a "$out"
    timeout -k 10 240 python bench.py $B >> "$out" 2>&1 || { echo "bench q$np rc=$?"; exit 1; }
    echo "== q$np rocprof" | tee -a "$out"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_q$np -o run \
        --output-format csv -- python bench.py $B --check 0 > gpurun_out/prof_${tag}_q$np.log 2>&1 \
        || { echo "rocprof q$np rc=$?"; exit 1; }
    f=$(ls gpurun_out/prof_${tag}_q$np/*/run_kernel_stats.csv gpurun_out/prof_${tag}_q$np/run_kernel_stats.csv 2>/dev/null | head -n 1)
    [ -n "$f" ] && cut -d, -f1-8 "$f" | head -n 8 >> "$out"
done
echo "== done" | tee -a "$out"
