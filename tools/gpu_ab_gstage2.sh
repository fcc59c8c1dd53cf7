# Group stage (YRSS_RANK_GSTAGE=1) at 26..65 buckets against the LDS image
# (default there) and at 17..25 against count mode; group size 16 tiles (one
# chunk) vs the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
row() { grep '^{"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; s=r["step"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], s["scan_us"], s["scatter_us"], r["probe"]["us"], d["check"]["bit_exact"])'; }
for rep in 1 2; do
for np in 20 25 32 40 48 64; do
  for v in base g0 g16 g32; do
    f=gpurun_out/gs2.log
    case $v in
      base) envs="" ;;
      g0) envs="YRSS_RANK_GSTAGE=1 YRSS_RANK_IMG=0 YRSS_NO_COUNT=1" ;;
      g16) envs="YRSS_RANK_GSTAGE=1 YRSS_RANK_IMG=0 YRSS_NO_COUNT=1 YRSS_GROUP_TILES=16" ;;
      g32) envs="YRSS_RANK_GSTAGE=1 YRSS_RANK_IMG=0 YRSS_NO_COUNT=1 YRSS_GROUP_TILES=32" ;;
    esac
    env $envs timeout -k 10 120 python bench.py --profile tcp4 --nb-procs $np --cpu-seconds 0 --pcie 0 > $f 2>&1 || { tail $f; exit 1; }
    echo "r$rep tcp4 np$np $v: $(row $f)"
  done
done
done
