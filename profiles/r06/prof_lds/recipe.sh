# r06: bin_kernel phase counters on C2 with the accumulators in LDS (lib/prof)
# against the scratch-resident accumulators of the round-5 prof build (lib/prof_old)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof2; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
L=genome-assembly_amd/lib
timeout -k 10 300 python -u bench.py $NOX --steps 20 --warmup 3 > $O/base.json 2>> $O/err.txt || exit 1
KB_LIB_PATH=$L/prof/libkbin.so timeout -k 10 300 python -u bench.py $NOX --steps 5 --warmup 2 > $O/prof_lds.json 2> $O/prof_lds.err || exit 1
KB_LIB_PATH=$L/prof_old/libkbin.so timeout -k 10 300 python -u bench.py $NOX --steps 5 --warmup 2 > $O/prof_scratch.json 2> $O/prof_scratch.err || exit 1
echo done
