# r04 g1: price the read-id ordering on the shipped build.
#  (a) bin_kernel ablation incl. mode 4 (id windows without their sorts), no profiler
#  (b) C3 per-kernel trace (lists_* vs the rest)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g1; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 30 --warmup 5"
timeout -k 10 200 python -u bench.py $NOX > $O/prod.json 2> $O/prod.err || exit 1
for m in 0 4 3 2; do
  KB_LIB_PATH=genome-assembly_amd/lib/abl/libkbin.so KB_BIN_ABLATE=$m timeout -k 10 200 python -u bench.py $NOX > $O/abl$m.json 2> $O/abl$m.err || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3 -o kt \
  -- python3 bench.py --cpu-sample 0 --no-capacity --no-host-input --workload c3 --steps 2 --warmup 1 > $O/kt_c3.log 2>&1 || exit 1
echo rc=$?
