# r04 g15: ranking phase cycles (prof build), C3 ranked
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g15; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so KB_BIN_RANK=2 timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 1 --warmup 1 > $O/c3_r2.json 2> $O/c3_r2.err
echo rc=$?
