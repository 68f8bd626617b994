# split bins: parity (split, heavy, partition tests), then A/B of KB_BIN_SPLIT_DIV on C2 and the N-rank emulation
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread -k "split or heavy or partition or full_scale or random_vs or two_word" tests > gpurun_out/t_split.log 2>&1 || exit 1
for sd in 0 2 4; do
  for w in "--reads 1000000 --parts 1" "--reads 2000000 --parts 2" "--reads 8000000 --parts 8"; do
    KB_BIN_SPLIT_DIV=$sd timeout -k 10 200 python bench.py $w --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/ab.log 2>&1 || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('sd=$sd', '$w', round(d['value']/1e9,2), d['ms_per_step'], d['phases_ms'])" >> gpurun_out/splitab.txt
  done
done
echo rc=$?
