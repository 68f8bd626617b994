# A/B of the flat-list threshold on the N-rank receiver emulation and C2
set -o pipefail
cd $GRAFT_REPO_ROOT
for fl in 1 2 3; do
  for w in "--reads 1000000 --parts 1" "--reads 2000000 --parts 2" "--reads 8000000 --parts 8"; do
    KB_BIN_FLAT_L=$fl timeout -k 10 200 python bench.py $w --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/ab.log 2>&1 || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('fl=$fl', '$w', round(d['value']/1e9,2), d['ms_per_step'], d['phases_ms'])" >> gpurun_out/flatab.txt
  done
done
echo rc=$?
