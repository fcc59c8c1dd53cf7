# SQ counters of the scatter kernel per case: each line of $1 is
# "label|env assignments|bench.py args"; two rocprofv3 --pmc passes per case
# (8 SQ counters each), summarised per dispatch.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/spmc; export TMPDIR=/tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
B="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM"
i=0
while IFS='|' read -r label envs args; do
  [ -z "$label" ] && continue
  i=$((i+1))
  for set in A B; do
    d=gpurun_out/spmc/c${i}_$set
    env $envs timeout -s KILL 150 rocprofv3 --pmc ${!set} -d $d -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --check 0 --pcie 0 $args > $d.log 2>&1 || { echo "$label $set FAILED"; tail -20 $d.log; exit 1; }
  done
  python3 - "$label" gpurun_out/spmc/c${i}_A gpurun_out/spmc/c${i}_B <<'PY'
import csv, glob, sys, collections
label = sys.argv[1]
acc = collections.defaultdict(float); n = collections.Counter()
for d in sys.argv[2:]:
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if "scatter" not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print(label, {k: round(v / max(n[k], 1) / 1e6, 3) for k, v in sorted(acc.items())}, "(millions per dispatch)", flush=True)
PY
done < "$1"
