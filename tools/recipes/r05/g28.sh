# r05 g28: the per-bin fixed overhead (KB_BIN_ABLATE=5: no sweep 1) and the
# full kernel, phase counters of a prof + ablation build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g28; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 5 --warmup 2"
for m in 0 5; do
  KB_LIB_PATH=genome-assembly_amd/lib/profabl/libkbin.so KB_BIN_ABLATE=$m timeout -k 10 200 python -u bench.py $NOX > $O/pa$m.json 2> $O/pa$m.err || exit 1
done
echo done
