#!/bin/bash
# Round-6 GPU work.  PART selects:
#   n8     the driver's default N-GPU bench command, rehearsed in full on one
#          device (YRSS_BENCH_ONE_DEVICE=1, --pcie 1: the fan-out leg included,
#          its workers capped so 8 contexts stay co-resident), with its wall
#          time against the driver's 600 s limit
#   suite  the GPU test suite and smoke
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
part=${PART:-suite}
case $part in
n8)
    n=${N:-8}
    log=gpurun_out/r06_n${n}_one_device_full.log
    t0=$(date +%s%N)
    YRSS_BENCH_ONE_DEVICE=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port 29517 bench.py \
        --gpus "$n" > "$log" 2>&1
    rc=$?
    t1=$(date +%s%N)
    echo "{\"rehearsal\": \"bench.py --gpus $n (defaults) under torch.distributed.run, one device\", \"rc\": $rc, \"wall_s\": $(( (t1 - t0) / 1000000 ))e-3}" | tee -a "$log"
    exit $rc
    ;;
ab)
    # same-process A/B of tunings (AB_LIBS, ab_inproc.py --libs form) on
    # each AB_PROFILES stream at AB_NB bucket counts
    for prof in ${AB_PROFILES:-imix tcp4 udp4}; do
        timeout -k 10 400 python -u tools/ab_inproc.py --nb-procs "${AB_NB:-3,8}" \
            --libs "${AB_LIBS:-cur@scan_kernel=1,cur@scan_kernel=0}" --rounds "${AB_ROUNDS:-6}" \
            --profile "$prof" > "gpurun_out/r06_ab_${AB_TAG:-x}_$prof.log" 2>&1 \
            || { tail -20 "gpurun_out/r06_ab_${AB_TAG:-x}_$prof.log"; exit 1; }
        tail -8 "gpurun_out/r06_ab_${AB_TAG:-x}_$prof.log"
    done
    ;;
suitefirst)
    # the GPU suite, then PART=ab
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 \
        --timeout-method thread > gpurun_out/r06_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r06_pytest_gpu.log; exit 1; }
    tail -3 gpurun_out/r06_pytest_gpu.log
    PART=ab bash "$0"
    ;;
suite)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 \
        --timeout-method thread > gpurun_out/r06_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r06_pytest_gpu.log; exit 1; }
    tail -3 gpurun_out/r06_pytest_gpu.log
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1
    ;;
*)
    echo "unknown PART $part"; exit 2 ;;
esac
