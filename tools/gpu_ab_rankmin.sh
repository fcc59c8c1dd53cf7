# Ranked group stage below 9 buckets (YRSS_RANK_MINNB=2) against the
# few-bucket path (default), all-TCP and IMIX at 3 and 5 procs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
row() { grep '^{"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; s=r["step"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], s["scan_us"], s["scatter_us"], r["probe"]["us"], d["check"]["bit_exact"])'; }
for rep in 1 2; do
for cfg in "tcp4 3" "imix 3" "tcp4 5" "tcp4 7"; do
  set -- $cfg
  for rm in 8 2; do
    f=gpurun_out/rm.log
    YRSS_RANK_MINNB=$rm timeout -k 10 120 python bench.py --profile $1 --nb-procs $2 --cpu-seconds 0 --pcie 0 > $f 2>&1 || { tail $f; exit 1; }
    echo "r$rep $1 np$2 rank_min=$rm: $(row $f)"
  done
done
done
