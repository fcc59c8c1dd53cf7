# A/B of engine knobs on one box: bench.py alternately under each environment
# setting (AB_VARIANTS, ';'-separated "VAR=val VAR2=val" lists), AB_ROUNDS times.
#   AB_VARIANTS="YRSS_AHEAD=1;YRSS_AHEAD=2" AB_ROUNDS=3 BENCH_ARGS="--profile tcp4" bash tools/gpu_ab.sh
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
IFS=';' read -r -a VARS <<< "${AB_VARIANTS:-YRSS_AHEAD=1;YRSS_AHEAD=2}"
for r in $(seq 1 "${AB_ROUNDS:-3}"); do
  for v in "${VARS[@]}"; do
    env $v timeout -k 10 300 python bench.py --cpu-seconds 0 --pcie 0 ${BENCH_ARGS:-} > gpurun_out/ab.log 2>&1 || { tail gpurun_out/ab.log; exit 1; }
    echo "[$v] $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], r["probe"] and r["probe"]["us"], d["check"] and d["check"]["bit_exact"])')"
  done
done
