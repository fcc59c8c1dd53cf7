# With XCD-contiguous scatter groups (default from 10 buckets): the ranked
# scatter's LDS image (YRSS_RANK_IMG=1) vs its per-chunk stage (0) past 33
# buckets, all-TCP; every GPU test first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/ri_pytest.log 2>&1 || { tail -30 gpurun_out/ri_pytest.log; exit 1; }
tail -1 gpurun_out/ri_pytest.log
row() { grep '^{"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; s=r["step"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], s["scan_us"], s["scatter_us"], r["probe"]["us"], d["check"]["bit_exact"])'; }
for rep in 1 2; do
for np in 48 64 128 255; do
  for ri in 0 1; do
    f=gpurun_out/ri_${np}_$ri.log
    YRSS_RANK_IMG=$ri timeout -k 10 120 python bench.py --profile tcp4 --nb-procs $np --cpu-seconds 0 --pcie 0 > $f 2>&1 || { tail $f; exit 1; }
    echo "r$rep tcp4 np$np rank_img=$ri: $(row $f)"
  done
done
done
