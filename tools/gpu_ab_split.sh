# Split scatter (YRSS_SPLIT=1: coarse pass over 16-bucket regions + fine pass,
# no parse-side ranks) vs the ranked scatter (0), all-TCP by nb_procs; the
# layout GPU tests (split on, off, fine item sizes) first.  Measured and not
# kept: the YRSS_SPLIT / YRSS_SPLIT_FSHIFT knobs and the
# yrss_split_coarse / yrss_split_fine kernels are no longer in the source.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_layout.py -k "split or ballot or bucket_count" > gpurun_out/split_pytest.log 2>&1 || { tail -40 gpurun_out/split_pytest.log; exit 1; }
tail -1 gpurun_out/split_pytest.log
row() { grep '^{"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; s=r["step"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], s["scan_us"], s["scatter_us"], r["probe"]["us"], d["check"]["bit_exact"])'; }
for rep in 1 2; do
for np in 32 64 128 255; do
  for sp in 0 1; do
    f=gpurun_out/split.log
    YRSS_SPLIT=$sp timeout -k 10 120 python bench.py --profile tcp4 --nb-procs $np --cpu-seconds 0 --pcie 0 > $f 2>&1 || { tail $f; exit 1; }
    echo "r$rep tcp4 np$np split=$sp: $(row $f)"
  done
done
done
for fs in 0 1 3; do
  f=gpurun_out/split.log
  YRSS_SPLIT_FSHIFT=$fs timeout -k 10 120 python bench.py --profile tcp4 --nb-procs 255 --cpu-seconds 0 --pcie 0 > $f 2>&1 || { tail $f; exit 1; }
  echo "tcp4 np255 split fshift=$fs: $(row $f)"
done
