#!/bin/bash
# Same-box A/B of library builds of the current tree (YRSS_LIB selects the
# .so bench.py loads; "cur" is yastack_amd/_lib/libyrss.so): the all-TCP
# bench rows at the given nb_procs, every variant in turn, two rounds.
#   tools/gpu_ab_libs.sh TAG "8 64" "cur ab/lib/libyrss_st1.so ..." [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1
qs=$2
libs=$3
extra=${4:-}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
out=gpurun_out/abl_$tag.log
: > "$out"
for round in 1 2; do
    for np in $qs; do
        for lib in $libs; do
            B="--profile tcp4 --nb-procs $np --steps 30 --warmup 10 --cpu-seconds 0 --pcie 0 --check 0 $extra"
            echo "== r$round q$np $(basename $lib)" >> "$out"
            if [ "$lib" = cur ]; then
                timeout -k 10 240 python bench.py $B >> "$out" 2>&1 || { echo "$lib q$np rc=$?"; exit 1; }
            else
                YRSS_LIB=$lib timeout -k 10 240 python bench.py $B >> "$out" 2>&1 || { echo "$lib q$np rc=$?"; exit 1; }
            fi
        done
    done
    echo "round $round done"
done
python - "$out" <<'EOF'
import json, sys
name = None
for ln in open(sys.argv[1]):
    if ln.startswith("== "):
        name = ln[3:].strip()
    elif ln.startswith("{"):
        d = json.loads(ln); r = d["roofline"]; s = r["step"]
        print(f"{name:28s} step {d['ms_per_step']:.4f}  parse {r['kernel_avg_us']:6.1f}  probe "
              f"{r['probe']['us']:6.1f} ({r['probe']['parse_frac_of_probe']:.3f})  scan "
              f"{s.get('scan_us')}  scatter {s.get('scatter_us')}")
EOF
