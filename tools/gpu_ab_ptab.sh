# Ranked group stage: the group's prefixes loaded as one (bucket, column)
# table with consecutive lanes on consecutive columns (default) vs one word
# per lane per bucket row (build/pt0, the previous commit's library), by
# bucket count; the ranked parity tests first.  Measured and not kept.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_layout.py tests/test_gpu_count.py > gpurun_out/pt_pytest.log 2>&1 || { tail -40 gpurun_out/pt_pytest.log; exit 1; }
tail -1 gpurun_out/pt_pytest.log
row() { grep '^{"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; s=r["step"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], s["scan_us"], s["scatter_us"], r["probe"]["us"], d["check"]["bit_exact"])'; }
for rep in 1 2; do
for np in 8 16 64 128 255; do
  for lib in yastack_amd/_lib/libyrss.so build/pt0/libyrss.so; do
    f=gpurun_out/pt.log
    YRSS_LIB=$lib timeout -k 10 120 python bench.py --profile tcp4 --nb-procs $np --cpu-seconds 0 --pcie 0 > $f 2>&1 || { tail $f; exit 1; }
    echo "r$rep tcp4 np$np $lib: $(row $f)"
  done
done
done
