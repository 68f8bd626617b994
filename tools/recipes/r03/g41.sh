# round 3b: C4-share record pass bisect (round-3a build, the record-pass
# commit 35c61e3, current), KB_DEBUG host timings
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3c4; mkdir -p $O
ARGS="--cpu-sample 0 --workload c4 --steps 1 --warmup 1 --no-capacity --no-host-input"
KB_DEBUG=1 KB_LIB_PATH=genome-assembly_amd/lib/r3a/libkbin.so timeout -k 10 300 python -u bench.py $ARGS > $O/c4_r3a.json 2> $O/c4_r3a.err || exit 1
KB_DEBUG=1 KB_LIB_PATH=genome-assembly_amd/lib/c35/libkbin.so timeout -k 10 300 python -u bench.py $ARGS > $O/c4_c35.json 2> $O/c4_c35.err || exit 1
KB_DEBUG=1 timeout -k 10 300 python -u bench.py $ARGS > $O/c4_new.json 2> $O/c4_new.err || exit 1
echo rc=$?
