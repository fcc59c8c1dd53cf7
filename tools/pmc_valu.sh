set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
B="--profile tcp4 --nb-procs 255 --steps 5 --warmup 2 --cpu-seconds 0 --pcie 0 --check 0 --extra-configs="
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1
grep -o "SQ_[A-Z_0-9]*" gpurun_out/avail.txt | sort -u > gpurun_out/avail_sq.txt
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES" "SQ_INST_CYCLES_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
  n=$(echo $pass | cut -c1-12 | tr -d ' ')
  timeout -s KILL 120 rocprofv3 --pmc $pass -d gpurun_out/pmcv_$n -o run --output-format csv -- python bench.py $B > gpurun_out/pmcv_$n.log 2>&1 || { echo "pass rc=$?"; tail -5 gpurun_out/pmcv_$n.log; }
done
python tools/pmc_kernels.py gpurun_out/pmcv_* > gpurun_out/pmcv.sum 2>&1
cat gpurun_out/pmcv.sum
