# round-6 call: the whole GPU suite, smoke, the default bench line, the
# phase clock with phase b split (tags/carried vs placement)
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r06_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r06_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 || { tail gpurun_out/r06_smoke.log; exit 1; }
tail -1 gpurun_out/r06_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r06_bench.log 2> gpurun_out/r06_bench.err || { tail -20 gpurun_out/r06_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r06_bench.log").read().strip().splitlines()[-1])
print({k: d[k] for k in ("value", "ms_per_step")}, d["roofline"]["frac"], d["roofline"]["step"])
print(d["check"]["bit_exact"], [(x["config"], x["value"], x["ms_per_step"], x["bit_exact"]) for x in d["configs_extra"]])
PY
tools/build_ab_lib.sh prof -DYRSS_PROF_LINES=1 > gpurun_out/build_prof.log 2>&1 || exit 1
timeout -k 10 200 python tools/line_prof.py --lib ab/lib/libyrss_prof.so --nb-procs 3,8,64 > gpurun_out/r06_lineprof_split.log 2>&1 || exit 1
grep -E "^q|span total|   b|   c |wait|   d " gpurun_out/r06_lineprof_split.log
