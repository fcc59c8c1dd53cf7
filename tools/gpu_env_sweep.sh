# A/B sweep: each line of $1 is "label|env assignments|bench.py args"; every
# case runs bench.py once and prints value, ms/step, parse, scan, scatter,
# probe (us) and the bit-exact check.  Set TESTS=1 to run the GPU tests first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sweep; export TMPDIR=/tmp PYTHONUNBUFFERED=1
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep/pytest.log 2>&1 || { tail -30 gpurun_out/sweep/pytest.log; exit 1; }
  tail -1 gpurun_out/sweep/pytest.log
fi
row() { grep '^{"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; s=r["step"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], s["scan_us"], s["scatter_us"], r["probe"]["us"], (d.get("check") or {}).get("bit_exact"))'; }
i=0
while IFS='|' read -r label envs args; do
  [ -z "$label" ] && continue
  i=$((i+1)); f=gpurun_out/sweep/case$i.log
  env $envs timeout -k 10 300 python bench.py --cpu-seconds 0 --pcie 0 $args > $f 2>&1 || { echo "$label FAILED"; tail $f; exit 1; }
  echo "$label: $(row $f)"
done < "$1"
