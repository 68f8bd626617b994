# r05 g33: bucket_kernel's dense bin index from wave ballots (no serial walk
# over the slots), bins_plan_kernel's descriptor gathers a round ahead: the
# whole GPU suite, C2 alternating against lib/ab_prev, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g33; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 1000 python -u -m pytest -x -q -m gpu --timeout 600 --timeout-method thread tests > $O/gpu_suite.txt 2>&1 || exit 1
for i in 1 2; do
  KB_LIB_PATH=genome-assembly_amd/lib/ab_prev/libkbin.so timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2_prev_$i.json 2> $O/c2_prev_$i.err || exit 1
  timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2_new_$i.json 2> $O/c2_new_$i.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py $NOX --steps 20 --warmup 3 > $O/kt.log 2>&1 || exit 1
echo done
