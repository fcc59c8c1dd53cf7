# Ranked scatter walked in bucket slices (YRSS_BPASS buckets per pass) x group
# size (YRSS_GROUP_TILES) vs the per-chunk stage (YRSS_BPASS=0), all-TCP past
# 65 buckets; the bucket-pass parity tests first.  Measured and not kept
# (DESIGN §9): YRSS_BPASS is no longer in the source.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_layout.py -k "bucket_passes or bucket_count or xcd" > gpurun_out/bp_pytest.log 2>&1 || { tail -40 gpurun_out/bp_pytest.log; exit 1; }
tail -1 gpurun_out/bp_pytest.log
row() { grep '^{"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; s=r["step"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], s["scan_us"], s["scatter_us"], r["probe"]["us"], d["check"]["bit_exact"])'; }
for rep in 1 2; do
for np in 128 255; do
  for v in "0 32" "32 32" "64 32" "32 64" "64 64" "32 128" "64 128"; do
    set -- $v
    f=gpurun_out/bp.log
    YRSS_BPASS=$1 YRSS_GROUP_TILES=$2 timeout -k 10 120 python bench.py --profile tcp4 --nb-procs $np --cpu-seconds 0 --pcie 0 > $f 2>&1 || { tail $f; exit 1; }
    echo "r$rep tcp4 np$np bpass=$1 group_tiles=$2: $(row $f)"
  done
done
done
