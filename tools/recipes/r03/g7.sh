set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3f; mkdir -p $O
KB_DEBUG=1 timeout -k 10 120 python -u tools/cold.py --workload c2 --steps 3 > $O/cold_c2.txt 2>&1 && \
KB_DEBUG=1 timeout -k 10 200 python -u tools/cold.py --workload c3 --steps 2 > $O/cold_c3.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 20 --warmup 5 > $O/c2.json 2> $O/c2.err
echo rc=$?
