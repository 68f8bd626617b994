# split bins (re-expansion per partition) vs flat lists on the N=4/8 receiver emulation
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "1 0" "3 2" "3 8" "4 8" "4 32"; do
  for w in "4000000 20000000 4 1" "8000000 40000000 8 1"; do
    set -- $cfg $w
    KB_BIN_FLAT_L=$1 KB_BIN_SPLIT_DIV=$2 timeout -k 10 300 python bench.py --reads $3 --genome $4 --parts $5 --steps $6 --warmup 1 --cpu-sample 0 > gpurun_out/sa.log 2>&1 || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/sa.log').read().strip().splitlines()[-1]); p=d['phases_ms']; print('fl=$1 sd=$2 P=$5', 'per pass', round(p['total_ms']/$5, 3), 'bins', round(p['runs_ms']/$5,3))" >> gpurun_out/sa.txt
  done
done
echo rc=$?
