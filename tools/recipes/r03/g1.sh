set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3a
O=gpurun_out/r3a
timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 20 --warmup 5 > $O/c2.json 2> $O/c2.err && \
timeout -k 10 300 python -u bench.py --cpu-sample 0 --reads 8000000 --genome 40000000 --parts 8 --steps 4 --warmup 2 > $O/zs8.json 2> $O/zs8.err && \
timeout -k 10 300 python -u bench.py --cpu-sample 0 --reads 2000000 --genome 10000000 --parts 2 --steps 4 --warmup 2 > $O/zs2.json 2> $O/zs2.err && \
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 3 --warmup 2 > $O/c2_prof.json 2> $O/c2_prof.err && \
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 300 python -u bench.py --cpu-sample 0 --reads 8000000 --genome 40000000 --parts 8 --steps 1 --warmup 1 > $O/zs8_prof.json 2> $O/zs8_prof.err
echo rc=$?
