set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
YRSS_AHEAD=2 YRSS_OUT16=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pt_knobs.log 2>&1; rc=$?; tail -3 gpurun_out/pt_knobs.log; [ $rc -eq 0 ] || exit $rc
YRSS_OUT16=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k "profiles_configs or ragged or full_size" > gpurun_out/pt_knobs1.log 2>&1; rc=$?; tail -2 gpurun_out/pt_knobs1.log; [ $rc -eq 0 ] || exit $rc
AB_ROUNDS=2 AB_VARIANTS="YRSS_AHEAD=1;YRSS_AHEAD=2;YRSS_OUT16=1;YRSS_OUT16=2;YRSS_AHEAD=2 YRSS_OUT16=2" bash tools/gpu_ab.sh
AB_ROUNDS=1 AB_VARIANTS="YRSS_AHEAD=1;YRSS_AHEAD=2;YRSS_OUT16=2;YRSS_AHEAD=2 YRSS_OUT16=2" BENCH_ARGS="--profile tcp4" bash tools/gpu_ab.sh
