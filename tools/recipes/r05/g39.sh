# r05 g39: K < 2M (records hash-routed: their mmer codes are not canonical,
# no bucket map) -- the K < 2M parity cases alone, then the whole GPU suite,
# then the default C2 line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g39; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "k_below_2m" > $O/k2m.txt 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest -x -q -m gpu --timeout 600 --timeout-method thread tests > $O/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2.json 2> $O/c2.err || exit 1
echo done
