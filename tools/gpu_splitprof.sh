# kernel split of the bin phase (phase 0 / phase 1) on the N-rank emulation, split off/on
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for sd in 0 2; do
  for w in "2000000 2" "8000000 8"; do
    set -- $w
    KB_BIN_SPLIT_DIV=$sd timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp_${sd}_$2 -o kt -- python3 bench.py --reads $1 --parts $2 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/sp.log 2>&1 || exit 1
  done
done
echo rc=$?
