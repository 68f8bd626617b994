# r05 g27: bin_kernel ablation on the current build (diagnostic build,
# KB_BIN_ABLATE: 0 everything, 4 no window sorts, 3 no prune / windows,
# 2 probes + counts only, 5 no sweep 1 at all = the per-bin overheads, 1
# expansion only), 30 steps each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g27; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 30 --warmup 5"
timeout -k 10 200 python -u bench.py $NOX > $O/prod.json 2> $O/prod.err || exit 1
for m in 0 4 3 2 1 5; do
  KB_LIB_PATH=genome-assembly_amd/lib/abl/libkbin.so KB_BIN_ABLATE=$m timeout -k 10 200 python -u bench.py $NOX > $O/abl$m.json 2> $O/abl$m.err || exit 1
done
echo done
