# r06 A/B: local bucket count (KB_BIN_NB) for C3's received-record
# conversion (fewer buckets: longer runs per bucket and block trip) --
# C3 at 1024 (default), 512, 256 buckets, digest-checked, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_nb; mkdir -p $O
for i in 1 2; do
  for nb in 1024 512 256; do
    KB_BIN_NB=$nb timeout -k 10 400 python -u bench.py --workload c3 --steps 3 --warmup 1 --cpu-sample 0 --digest > $O/c3_nb${nb}_$i.json 2>> $O/err.txt || exit 1
  done
done
echo done
