# C3 (100 M reads, digest) and C5 per-GPU share bench lines for profiles/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --workload c3 --steps 2 --warmup 1 --digest --cpu-sample 0 > gpurun_out/v9_c3.json 2> gpurun_out/v9_c3.err && \
timeout -k 10 500 python bench.py --workload c5 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/v9_c5.json 2> gpurun_out/v9_c5.err
echo rc=$?
