# Parse kernel count slots flushed by the workgroup (8 columns per bucket row
# per store, default YRSS_CNT_WG=1) vs by each wave (one word per row per
# lane; build/cwg0: -DYRSS_CNT_WG=0), by bucket count; the parity suites on
# the default build first.
#   mkdir -p build/cwg0; hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DYRSS_CNT_WG=0 \
#     -I include yastack_amd/csrc/yrss.hip yastack_amd/csrc/yrss_pcap.cpp yastack_amd/csrc/yrss_shard.cpp \
#     yastack_amd/csrc/yrss_fanout.cpp -o build/cwg0/libyrss.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_layout.py tests/test_gpu_count.py tests/test_gpu_parity.py > gpurun_out/cwg_pytest.log 2>&1 || { tail -40 gpurun_out/cwg_pytest.log; exit 1; }
tail -1 gpurun_out/cwg_pytest.log
row() { grep '^{"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; s=r["step"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], s["scan_us"], s["scatter_us"], r["probe"]["us"], d["check"]["bit_exact"])'; }
for rep in 1 2; do
for cfg in "udp4 3" "tcp4 3" "tcp4 16" "tcp4 64" "tcp4 255"; do
  set -- $cfg
  for lib in yastack_amd/_lib/libyrss.so build/cwg0/libyrss.so; do
    f=gpurun_out/cwg.log
    YRSS_LIB=$lib timeout -k 10 120 python bench.py --profile $1 --nb-procs $2 --cpu-seconds 0 --pcie 0 > $f 2>&1 || { tail $f; exit 1; }
    echo "r$rep $1 np$2 $lib: $(row $f)"
  done
done
done
