# A/B of KB_BIN_BIG_DIV (flat lists for large multi-table bins) on C2 and the N=2/4/8 emulation
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread -k "heavy or split or partition or full_scale" tests > gpurun_out/t_bd.log 2>&1 || exit 1
for bd in 0 1 2 4; do
  for w in "1000000 5000000 1 5" "2000000 10000000 2 2" "4000000 20000000 4 1" "8000000 40000000 8 1"; do
    set -- $bd $w
    KB_BIN_BIG_DIV=$1 timeout -k 10 300 python bench.py --reads $2 --genome $3 --parts $4 --steps $5 --warmup 1 --cpu-sample 0 > gpurun_out/bd.log 2>&1 || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/bd.log').read().strip().splitlines()[-1]); print('bd=$1 P=$4', round(d['value']/1e9,2), d['ms_per_step'], 'per pass', round(d['phases_ms']['total_ms']/$4, 3), d['phases_ms'])" >> gpurun_out/bdab.txt
  done
done
echo rc=$?
