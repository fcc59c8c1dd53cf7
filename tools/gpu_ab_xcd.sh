# Scatter groups XCD-contiguous (YRSS_SCATTER_XCD=1) vs round-robin (0), all-TCP
# by nb_procs and the headline UDP stream, alternating on one box; the count
# and layout GPU tests under the new mapping first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
YRSS_SCATTER_XCD=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_count.py tests/test_gpu_layout.py tests/test_gpu_parity.py > gpurun_out/xcd_pytest.log 2>&1 || { tail -30 gpurun_out/xcd_pytest.log; exit 1; }
tail -1 gpurun_out/xcd_pytest.log
row() { grep '^{"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; s=r["step"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], s["scan_us"], s["scatter_us"], r["probe"]["us"], d["check"]["bit_exact"])'; }
for rep in 1 2; do
for cfg in "udp4 3" "tcp4 3" "tcp4 8" "tcp4 16" "tcp4 32" "tcp4 64" "tcp4 128" "tcp4 255" "imix 64"; do
  set -- $cfg
  for x in 0 1; do
    f=gpurun_out/xcd_${1}_${2}_$x.log
    YRSS_SCATTER_XCD=$x timeout -k 10 120 python bench.py --profile $1 --nb-procs $2 --cpu-seconds 0 --pcie 0 > $f 2>&1 || { tail $f; exit 1; }
    echo "r$rep $1 np$2 xcd=$x: $(row $f)"
  done
done
done
