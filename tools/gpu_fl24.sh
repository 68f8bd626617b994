# flat threshold at the N=2/4 receiver emulation
set -o pipefail
cd $GRAFT_REPO_ROOT
for fl in 1 2 3; do
  for w in "2000000 10000000 2 2" "4000000 20000000 4 1"; do
    set -- $fl $w
    KB_BIN_FLAT_L=$1 timeout -k 10 300 python bench.py --reads $2 --genome $3 --parts $4 --steps $5 --warmup 1 --cpu-sample 0 > gpurun_out/fl.log 2>&1 || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/fl.log').read().strip().splitlines()[-1]); p=d['phases_ms']; print('fl=$1 P=$4', 'per pass', round(p['total_ms']/$4, 3), 'bins', round(p['runs_ms']/$4,3), 'bins/pass', d['result']['bins'])" >> gpurun_out/fl24.txt
  done
done
echo rc=$?
