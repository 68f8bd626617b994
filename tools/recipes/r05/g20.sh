# r05 g20: C3 record re-expansion by bin kind (prof build counters) and the
# pass's bin table (KB_DIAG_BINS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g20; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
KB_DIAG_BINS=$O/c3_bins.txt KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 400 python -u bench.py $NOX --workload c3 --steps 1 --warmup 2 > $O/c3_prof.json 2> $O/c3_prof.err || exit 1
echo done
