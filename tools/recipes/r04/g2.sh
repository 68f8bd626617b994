# r04 g2: g1 (ablation incl. mode 4, C3 trace) + the drop-in with the
# strong expand_read_id_list: byte-identity tests and the C2-shape wall time
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g2; mkdir -p $O
NCCL_DEBUG=WARN timeout -k 10 400 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dist.py \
  -k "dropin or host_cli or invariant or knobs_off or group" -m gpu > $O/dropin_tests.txt 2>&1 || exit 1
timeout -k 10 600 python -u tools/unitig_time.py --reads 100000 1000000 --full-max 1000000 --timeout 280 > $O/unitig_c2.jsonl 2> $O/unitig_c2.err || exit 1
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 30 --warmup 5"
timeout -k 10 200 python -u bench.py $NOX > $O/prod.json 2> $O/prod.err || exit 1
for m in 0 4 3 2; do
  KB_LIB_PATH=genome-assembly_amd/lib/abl/libkbin.so KB_BIN_ABLATE=$m timeout -k 10 200 python -u bench.py $NOX > $O/abl$m.json 2> $O/abl$m.err || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3 -o kt \
  -- python3 bench.py --cpu-sample 0 --no-capacity --no-host-input --workload c3 --steps 2 --warmup 1 > $O/kt_c3.log 2>&1 || exit 1
echo rc=$?
