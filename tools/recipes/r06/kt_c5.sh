# r06: kernel trace + stats of the C5 share (1 timed step): where the bin
# phase's 100 ms per pass go
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/kt_c5; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --cpu-sample 0 --workload c5 --steps 1 --warmup 1 > $O/kt.log 2>&1 || exit 1
echo done
