# Byte ranks for chunks of <= 256 packets on the group stage (default,
# YRSS_RANK8=1) vs 2-byte ranks (0): all-TCP at 8-17 buckets (4-tile chunks)
# and 33 (1024-packet chunks: unchanged); ranked parity tests first.  Measured
# and not kept: YRSS_RANK8 is no longer in the source.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_layout.py tests/test_gpu_count.py tests/test_gpu_fuzz.py > gpurun_out/r8_pytest.log 2>&1 || { tail -40 gpurun_out/r8_pytest.log; exit 1; }
tail -1 gpurun_out/r8_pytest.log
row() { grep '^{"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; s=r["step"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], s["scan_us"], s["scatter_us"], r["probe"]["us"], d["check"]["bit_exact"])'; }
for rep in 1 2; do
for cfg in "tcp4 7" "tcp4 8" "tcp4 12" "tcp4 16" "imix 16" "tcp4 32"; do
  set -- $cfg
  for r8 in 1 0; do
    f=gpurun_out/r8.log
    YRSS_RANK8=$r8 timeout -k 10 120 python bench.py --profile $1 --nb-procs $2 --cpu-seconds 0 --pcie 0 > $f 2>&1 || { tail $f; exit 1; }
    echo "r$rep $1 np$2 rank8=$r8: $(row $f)"
  done
done
done
