# automatic flat threshold: parity, C2 and the N=2/4/8 emulation
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/t_all.log 2>&1 || exit 1
for w in "1000000 5000000 1 10" "2000000 10000000 2 2" "4000000 20000000 4 1" "8000000 40000000 8 1"; do
  set -- $w
  timeout -k 10 300 python bench.py --reads $1 --genome $2 --parts $3 --steps $4 --warmup 1 --cpu-sample 0 > gpurun_out/au.log 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/au.log').read().strip().splitlines()[-1]); print('P=$3', round(d['value']/1e9,2), d['ms_per_step'], 'per pass', round(d['phases_ms']['total_ms']/$3, 3), d['phases_ms'])" >> gpurun_out/auto.txt
done
echo rc=$?
