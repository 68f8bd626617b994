# r05 g7: ablation -- the price of the prune's returning device-scope
# allocation atomic (KB_DIAG_ALLOC=1: a second returning atomic in series; results
# unchanged) on the diagnostic build, alternating with ablate 0
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g7; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
for i in 1 2; do
  for a in 0 1; do
    KB_LIB_PATH=genome-assembly_amd/lib/abl/libkbin.so KB_DIAG_ALLOC=$a timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/abl${a}_$i.json 2> $O/abl${a}_$i.err || exit 1
  done
done
echo done
