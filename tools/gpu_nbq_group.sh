# Step / parse / scatter on all-TCP by nb_procs x scatter group size (tiles) x
# many-bucket LDS image on/off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
row() { grep '^{"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; s=r["step"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], s["scan_us"], s["scatter_us"], r["probe"]["us"], d["check"]["bit_exact"])'; }
for np in ${NPS:-8 16 32 64}; do
  for gt in ${GTS:-16 32 64 128}; do
    for g in 0 1; do
      f=gpurun_out/nbg_${np}_${gt}_$g.log
      YRSS_GROUP_TILES=$gt YRSS_NO_GIMG=$g timeout -k 10 300 python bench.py --profile ${PROFILE:-tcp4} --nb-procs $np --cpu-seconds 0 --pcie 0 > $f 2>&1 || { tail $f; exit 1; }
      echo "nb_procs $np group $gt no_gimg $g: $(row $f)"
    done
  done
done
