# Quick GPU iteration: [pytest -m gpu] + bench + kernel trace with gaps.
#   usage: QUICK_TESTS=1 BENCH_ARGS="--profile tcp4" bash tools/gpu_quick.sh
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
if [ "${QUICK_TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
B="python bench.py --cpu-seconds 0 --pcie 0 ${BENCH_ARGS:-}"
timeout -k 10 300 $B > gpurun_out/bench_q.log 2>&1 || { tail gpurun_out/bench_q.log; exit 1; }
tail -1 gpurun_out/bench_q.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("value", d["value"], "ms", d["ms_per_step"], "parse_us", r["kernel_avg_us"], "probe_us", r["probe"] and r["probe"]["us"], "frac", r["frac"], d["check"])'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --check 0 --pcie 0 ${BENCH_ARGS:-} > gpurun_out/prof_q.log 2>&1 || { tail gpurun_out/prof_q.log; exit 1; }
python tools/trace_gaps.py gpurun_out/prof_q/run_kernel_trace.csv
