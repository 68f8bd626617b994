# r04 g28: bitmap emission A/B -- one word per lane (product) vs 64 ranks per
# ballot step with coalesced stores (-DKB_EMIT_BALLOT, lib/ab): ranked parity
# on the A/B build, C3 alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g28; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
KB_LIB_PATH=genome-assembly_amd/lib/ab/libkbin.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "ranked or large_lists or clustered_long" > $O/tests_ab.txt 2>&1 && \
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 --digest > $O/c3_word.json 2> $O/c3_word.err && \
KB_LIB_PATH=genome-assembly_amd/lib/ab/libkbin.so timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 --digest > $O/c3_ballot.json 2> $O/c3_ballot.err && \
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 > $O/c3_word2.json 2> $O/c3_word2.err && \
KB_LIB_PATH=genome-assembly_amd/lib/ab/libkbin.so timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 > $O/c3_ballot2.json 2> $O/c3_ballot2.err
echo rc=$?
