# r05 g37: C3's long-list sub-bin size on the final tree (KB_BIN_SUB_FILL_PCT:
# 40 default in the rank regime) -- 30 / 40 / 55, two runs each, digest asserted
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g37; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
for i in 1 2; do
  for f in 40 30 55; do
    KB_BIN_SUB_FILL_PCT=$f timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3_f${f}_$i.json 2> $O/c3_f${f}_$i.err || exit 1
  done
done
echo done
