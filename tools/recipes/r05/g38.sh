# r05 g38: K < 2M on the binned engine (the record pass walks the
# reference's incremental branch): the whole GPU suite (the new K < 2M cases
# included), then the default C2 line (unchanged kernel instantiation)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g38; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 1000 python -u -m pytest -x -q -m gpu --timeout 600 --timeout-method thread tests > $O/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2.json 2> $O/c2.err || exit 1
echo done
