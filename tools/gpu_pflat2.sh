set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread -k "heavy or split or partition or full_scale or two_word" tests > gpurun_out/t_pf.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pfk -o kt -- python3 bench.py --reads 8000000 --genome 40000000 --parts 8 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/pfk.log 2>&1 || exit 1
for cfg in "3 0" "2 0" "3 2" "2 2" "1 2"; do
  set -- $cfg
  for w in "1000000 5000000 1 5" "8000000 40000000 8 1"; do
    set -- $cfg $w
    KB_BIN_FLAT_L=$1 KB_BIN_SPLIT_DIV=$2 timeout -k 10 300 python bench.py --reads $3 --genome $4 --parts $5 --steps $6 --warmup 1 --cpu-sample 0 > gpurun_out/pf.log 2>&1 || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/pf.log').read().strip().splitlines()[-1]); print('fl=$1 sd=$2 P=$5', round(d['value']/1e9,2), d['ms_per_step'], d['phases_ms'])" >> gpurun_out/pfab.txt
  done
done
echo rc=$?
