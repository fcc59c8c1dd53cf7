# New defaults (group stage for ranked batches past 17 buckets, count mode up
# to 17) on every GPU test, then all-TCP by nb_procs: the ranked group stage
# below 18 buckets (YRSS_RANK_MINNB=8, count mode off) against the default
# paths there, and the default rows for the configs table.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gs3_pytest.log 2>&1 || { tail -40 gpurun_out/gs3_pytest.log; exit 1; }
tail -1 gpurun_out/gs3_pytest.log
row() { grep '^{"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; s=r["step"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], s["scan_us"], s["scatter_us"], r["probe"]["us"], d["check"]["bit_exact"])'; }
for rep in 1 2; do
for np in 8 12 16; do
  for v in base rk; do
    f=gpurun_out/gs3.log
    case $v in
      base) envs="" ;;
      rk) envs="YRSS_RANK_MINNB=8 YRSS_NO_COUNT=1" ;;
    esac
    env $envs timeout -k 10 120 python bench.py --profile tcp4 --nb-procs $np --cpu-seconds 0 --pcie 0 > $f 2>&1 || { tail $f; exit 1; }
    echo "r$rep tcp4 np$np $v: $(row $f)"
  done
done
done
for np in 3 20 32 64 128 255; do
  f=gpurun_out/gs3.log
  timeout -k 10 120 python bench.py --profile tcp4 --nb-procs $np --cpu-seconds 0 --pcie 0 > $f 2>&1 || { tail $f; exit 1; }
  echo "default tcp4 np$np: $(row $f)"
done
