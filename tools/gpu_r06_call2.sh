# round-6 call: the fan-out leg on one device with 8 contexts, direct, then
# the N=8 one-device rehearsal of the whole bench command
set -o pipefail
for q in 4 20; do
  GPU_MAX_HW_QUEUES=$q YRSS_CBENCH_MODES=5 YRSS_CBENCH_REPEAT=1 YRSS_CBENCH_FANOUT_DEVICES=0,0,0,0,0,0,0,0 \
    YRSS_CBENCH_WORKER_DEPTH=96 YRSS_CBENCH_WORKER_BLOCKS=24 YRSS_CBENCH_WORKER_FRAMES=1 \
    timeout -k 10 120 tools/yrss_cbench 1 1048576 32 1 > gpurun_out/r06_fanout8_q$q.log 2>&1
  echo "hwq $q rc=$?"; tail -c 600 gpurun_out/r06_fanout8_q$q.log; echo
done
PART=n8 bash tools/gpu_r06.sh || exit 1
grep -c "device fault" gpurun_out/r06_n8_one_device_full.log || true
