# r05 g12: C3 stage/ranking accounting (prof build counters: stage entries
# read by window and bitmap passes, ranked records, windows)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g12; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 400 python -u bench.py $NOX --workload c3 --steps 1 --warmup 2 > $O/c3_prof.json 2> $O/c3_prof.err || exit 1
echo done
