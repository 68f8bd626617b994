# A/B: bank-spread probe (product lib) vs the previous probe (lib/ab_old),
# alternating; then bin-kernel ablation timings (lib/abl, no profiler)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3s; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 30 --warmup 5"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $NOX > $O/new$i.json 2> $O/new$i.err || exit 1
  KB_LIB_PATH=genome-assembly_amd/lib/ab_old/libkbin.so timeout -k 10 200 python -u bench.py $NOX > $O/old$i.json 2> $O/old$i.err || exit 1
done
for m in 0 7 1 2 3 5; do
  KB_LIB_PATH=genome-assembly_amd/lib/abl/libkbin.so KB_BIN_ABLATE=$m timeout -k 10 200 python -u bench.py $NOX > $O/abl$m.json 2> $O/abl$m.err || exit 1
done
echo rc=$?
