#!/bin/bash
# Rehearsal of the driver's N>1 bench launch on a one-GPU box: N ranks
# (torch.distributed.run, gloo control plane) share device 0
# (YRSS_BENCH_ONE_DEVICE=1), each classifying its own 2^24-packet shard.
#   tools/gpu_rehearse.sh N PROFILE [extra bench args]
# The host-resident fan-out (--pcie) is left out: N workers on one device
# would not all be resident; on a real N-GPU node each has its own GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
n=$1
prof=$2
shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
log=gpurun_out/bench_n${n}_$prof.log
YRSS_BENCH_ONE_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus "$n" \
    --profile "$prof" --steps 20 --warmup 5 --pcie 0 "$@" > "$log" 2>&1 \
    || { tail -20 "$log"; exit 1; }
grep '^{"metric"' "$log" | python -c '
import json, sys
d = json.loads(sys.stdin.read())
c = d["check"]
print(json.dumps({"n_gpus": d["n_gpus"], "profile": d["config"]["workload"], "value": d["value"],
                  "ms_per_step": d["ms_per_step"], "ranks_checked": c["ranks_checked"],
                  "bit_exact": c["bit_exact"], "cpu_baseline": d["cpu_baseline"] is not None}))
for x in d.get("configs_extra") or []:
    print(json.dumps({k: x[k] for k in ("config", "profile", "n_gpus", "value", "ms_per_step",
                                        "parse_us", "roofline_frac", "ranks_checked",
                                        "bit_exact")}))'
