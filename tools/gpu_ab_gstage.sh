# Ranked scatter with one packed stage per group (YRSS_RANK_GSTAGE=1) vs the
# per-chunk stage (0) x group size, all-TCP; at 65 buckets also the LDS image
# (default there).  The group-stage parity tests first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_layout.py -k "group_stage or bucket_count or xcd" > gpurun_out/gs_pytest.log 2>&1 || { tail -40 gpurun_out/gs_pytest.log; exit 1; }
tail -1 gpurun_out/gs_pytest.log
row() { grep '^{"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; s=r["step"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], s["scan_us"], s["scatter_us"], r["probe"]["us"], d["check"]["bit_exact"])'; }
for rep in 1 2; do
for np in 64 128 255; do
  for v in "0 1 0" "0 0 0" "0 0 1" "64 0 1" "16 0 1"; do
    set -- $v
    f=gpurun_out/gs.log
    gt=""; [ "$1" != 0 ] && gt="YRSS_GROUP_TILES=$1"
    env $gt YRSS_RANK_IMG=$2 YRSS_RANK_GSTAGE=$3 timeout -k 10 120 python bench.py --profile tcp4 --nb-procs $np --cpu-seconds 0 --pcie 0 > $f 2>&1 || { tail $f; exit 1; }
    echo "r$rep tcp4 np$np group_tiles=$1 rank_img=$2 gstage=$3: $(row $f)"
  done
done
done
