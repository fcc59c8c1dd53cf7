# Rehearsal of the driver's N>1 bench launch on a one-GPU box: two ranks
# (torchrun, gloo control plane) share device 0 (YRSS_BENCH_ONE_DEVICE=1).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
YRSS_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 \
    > gpurun_out/bench_n2.log 2>&1 || { tail -20 gpurun_out/bench_n2.log; exit 1; }
grep '^{"metric"' gpurun_out/bench_n2.log | cut -c1-400
