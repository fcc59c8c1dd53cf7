#!/bin/bash
# Same-box A/B of the current tree against ab/base (a copy of an earlier
# commit's bench + package, built in this container): the all-TCP bench rows
# at the given nb_procs, alternating A and B, two rounds.
#   tools/gpu_ab_tree.sh TAG "3 8 64 255" [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1
qs=${2:-"3 8 64 255"}
extra=${3:-}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
out=gpurun_out/ab_$tag.log
: > "$out"
for round in 1 2; do
    for np in $qs; do
        for side in base new; do
            B="--profile tcp4 --nb-procs $np --steps 30 --warmup 10 --cpu-seconds 0 --pcie 0 --check 0 $extra"
            if [ $side = base ]; then exe=ab/base/bench.py; else exe=bench.py; fi
            echo "== r$round q$np $side" >> "$out"
            timeout -k 10 240 python $exe $B >> "$out" 2>&1 || { echo "$side q$np rc=$?"; exit 1; }
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
        print(f"{name:16s} step {d['ms_per_step']:.4f}  parse {r['kernel_avg_us']:6.1f}  probe "
              f"{r['probe']['us']:6.1f} ({r['probe']['parse_frac_of_probe']:.3f})  scan "
              f"{s.get('scan_us')}  scatter {s.get('scatter_us')}")
EOF
