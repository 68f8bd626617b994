# r05 g16: the bin-claim phase split (prof build): the bin's tail, the
# loop-top barrier, tid 0's claim wait -- C2 and C3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g16; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 300 python -u bench.py $NOX --steps 5 --warmup 2 > $O/c2_prof.json 2> $O/c2_prof.err || exit 1
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 400 python -u bench.py $NOX --workload c3 --steps 1 --warmup 2 > $O/c3_prof.json 2> $O/c3_prof.err || exit 1
echo done
