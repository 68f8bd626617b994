set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3k; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "dropin or host_cli" > $O/t.log 2>&1 || exit 1
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 300 python -u bench.py $NOX --steps 10 --warmup 3 --dropin > $O/c2_dropin.json 2> $O/c2_dropin.err || exit 1
KBH_THREADS=8 timeout -k 10 300 python -u bench.py $NOX --steps 10 --warmup 3 --dropin > $O/c2_dropin8.json 2> $O/c2_dropin8.err || exit 1
nproc > $O/nproc.txt
echo rc=$?
