# Step, parse and scatter time by bucket count on all-TCP (nb_procs 3 / 8 / 16 /
# 32 / 64), many-bucket LDS image on and off (YRSS_NO_GIMG=1), after the GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep_pytest.log 2>&1 || { tail -30 gpurun_out/sweep_pytest.log; exit 1; }
tail -2 gpurun_out/sweep_pytest.log
row() { grep '^{"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; s=r["step"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], s["scan_us"], s["scatter_us"], r["probe"]["us"], d["check"]["bit_exact"])'; }
for prof in ${PROFILES:-tcp4}; do
for np in ${NPS:-3 8 16 32 64}; do
  for g in 0 1; do
    YRSS_NO_GIMG=$g timeout -k 10 300 python bench.py --profile $prof --nb-procs $np --cpu-seconds 0 --pcie 0 > gpurun_out/nbq_${prof}_${np}_$g.log 2>&1 || { tail gpurun_out/nbq_${prof}_${np}_$g.log; exit 1; }
    echo "$prof nb_procs $np no_gimg $g: $(row gpurun_out/nbq_${prof}_${np}_$g.log)"
  done
done
done
