# Round-end measurement: tools/gpu_check.sh (all steps) then the per-config table.
# usage: gpurun -- bash tools/gpu_full.sh
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/gpu_check.sh > gpurun_out/check.log 2>&1; rc=$?
tail -60 gpurun_out/check.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/configs_table.py --steps 50 --cpu-seconds 5 > gpurun_out/configs.log 2>&1 || { tail -20 gpurun_out/configs.log; exit 1; }
tail -9 gpurun_out/configs.log
