set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
: > gpurun_out/ct_sweep.log
for rep in 1 2 3; do
  for q in 64 32; do
    for ct in 8 16 32; do
      echo "== rep $rep q $q ct $ct" >> gpurun_out/ct_sweep.log
      timeout -k 10 120 python bench.py --profile tcp4 --nb-procs $q --steps 30 --warmup 10 --cpu-seconds 0 --pcie 0 --extra-configs= --check 0 --tune chunk_tiles=$ct 2>/dev/null | grep '"metric"' >> gpurun_out/ct_sweep.log || exit 1
    done
  done
done
echo done
