# r06 g8: the prof build's phase counters at C2 (record pass and bin kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6g8; mkdir -p $O
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 10 --warmup 2 > $O/prof.json 2> $O/prof.err || exit 1
echo done
