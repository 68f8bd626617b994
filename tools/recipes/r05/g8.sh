# r05 g8: per-phase block-cycles of bin_kernel at C2 (the prof build,
# lib/prof: clock64 marks on tid 0 between barriers)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g8; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 300 python -u bench.py $NOX --steps 5 --warmup 2 > $O/prof.json 2> $O/prof.err || exit 1
echo done
