#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each, counters within gfx950's per-block
# limits) over the all-TCP bench at the given nb_procs; summarized per kernel
# (tools/pmc_kernels.py).  Usage: tools/gpu_pmc.sh TAG "3 8 64 255" [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1
qs=$2
extra=${3:-}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"
P2="FETCH_SIZE"
P3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
P4="SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
out=gpurun_out/pmc_$tag.log
: > "$out"
for np in $qs; do
    B="--profile tcp4 --nb-procs $np --steps 5 --warmup 2 --cpu-seconds 0 --pcie 0 --check 0 --extra-configs= $extra"
    i=0
    for pass in "$P1" "$P2" "$P3" "$P4"; do
        i=$((i + 1))
        d=gpurun_out/pmc_${tag}_q${np}_p$i
        timeout -s KILL 120 rocprofv3 --pmc $pass -d $d -o run --output-format csv \
            -- python bench.py $B > $d.log 2>&1 || { echo "pmc q$np pass $i rc=$?"; exit 1; }
    done
    echo "== q$np" >> "$out"
    python tools/pmc_kernels.py gpurun_out/pmc_${tag}_q${np}_p* >> "$out" || exit 1
done
cat "$out"
