set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3g; mkdir -p $O
KB_DEBUG=1 timeout -k 10 120 python -u tools/cold.py --workload c2 --steps 3 > $O/cold_c2.txt 2>&1 && \
bash tools/gpu.sh ktrace c3 --workload c3 --no-capacity --no-host-input --steps 2 --warmup 2
echo rc=$?
