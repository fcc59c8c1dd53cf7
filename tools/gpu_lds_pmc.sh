# LDS / VALU activity of the parse kernel, all-TCP (hashed) vs UDP: one
# rocprofv3 --pmc pass per profile (8 SQ counters), then a per-kernel summary.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
for p in tcp4 udp4; do
  timeout -s KILL 150 rocprofv3 --pmc $C -d gpurun_out/lds_$p -o run --output-format csv -- python bench.py --profile $p --steps 10 --warmup 3 --cpu-seconds 0 --check 0 --pcie 0 > gpurun_out/lds_$p.log 2>&1 || { tail -20 gpurun_out/lds_$p.log; exit 1; }
  python3 - "$p" <<'PY'
import csv, glob, sys, collections
p = sys.argv[1]
f = glob.glob(f"gpurun_out/lds_{p}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f)):
    if "yrss_parse_hash" not in r["Kernel_Name"]:
        continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print(p, {k: round(v / max(n[k], 1) / 1e6, 2) for k, v in sorted(acc.items())}, "(millions per dispatch)")
PY
done
