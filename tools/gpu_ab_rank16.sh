# Ranks as 16-byte stores (default build, YRSS_RANK16=1) vs per-lane 2-byte
# stores (build/r16_0: -DYRSS_RANK16=0), ranked paths on all-TCP; the ranked
# GPU tests on the default build first.  The YRSS_RANK16 branch (flush_out's
# kRank part writing a whole tile batch as one raw_buffer_store_b128 per lane,
# exactly as its q part does) was measured and not kept, so this script no
# longer has two variants to compare.
#   mkdir -p build/r16_0; hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DYRSS_RANK16=0 \
#     -I include yastack_amd/csrc/yrss.hip yastack_amd/csrc/yrss_pcap.cpp yastack_amd/csrc/yrss_shard.cpp \
#     yastack_amd/csrc/yrss_fanout.cpp -o build/r16_0/libyrss.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_layout.py tests/test_gpu_count.py tests/test_gpu_parity.py > gpurun_out/r16_pytest.log 2>&1 || { tail -30 gpurun_out/r16_pytest.log; exit 1; }
tail -1 gpurun_out/r16_pytest.log
row() { grep '^{"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; s=r["step"]; print(d["value"], d["ms_per_step"], r["kernel_avg_us"], s["scan_us"], s["scatter_us"], r["probe"]["us"], d["check"]["bit_exact"])'; }
for rep in 1 2; do
for np in 32 64 128 255; do
  for lib in yastack_amd/_lib/libyrss.so build/r16_0/libyrss.so; do
    f=gpurun_out/r16.log
    YRSS_LIB=$lib timeout -k 10 120 python bench.py --profile tcp4 --nb-procs $np --cpu-seconds 0 --pcie 0 > $f 2>&1 || { tail $f; exit 1; }
    echo "r$rep tcp4 np$np $lib: $(row $f)"
  done
done
done
