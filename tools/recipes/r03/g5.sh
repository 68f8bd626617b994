set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3d; mkdir -p $O
KB_DEBUG=1 timeout -k 10 120 python -u tools/cold.py --workload c2 --steps 4 > $O/cold_c2.txt 2>&1 && \
KB_DEBUG=1 timeout -k 10 200 python -u bench.py --cpu-sample 0 --no-capacity --no-host-input --reads 8000000 --genome 40000000 --parts 8 --steps 2 --warmup 2 > $O/zs8.json 2> $O/zs8.err && \
bash tools/gpu.sh ktrace c2 --no-capacity --no-host-input --steps 10 --warmup 3 && \
bash tools/gpu.sh ktrace zs8 --no-capacity --no-host-input --reads 8000000 --genome 40000000 --parts 8 --steps 2 --warmup 2
echo rc=$?
