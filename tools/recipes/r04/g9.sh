# r04 g9: bin_kernel phase cycles (prof build): C3 ranked vs unranked, C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g9; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
export KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so
KB_BIN_RANK=0 timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 1 --warmup 1 > $O/c3_r0.json 2> $O/c3_r0.err && \
KB_BIN_RANK=2 timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 1 --warmup 1 > $O/c3_r2.json 2> $O/c3_r2.err && \
timeout -k 10 300 python -u bench.py $NOX --steps 3 --warmup 2 > $O/c2.json 2> $O/c2.err
echo rc=$?
