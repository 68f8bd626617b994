# round 3b: sweep 2's global path with (ordinal, slot, position) in 32-bit
# registers (lib/sw2) vs the committed build: tracking / heavy / long-list
# parity, then C5 share and C3 capacity (the global-path users)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3c9; mkdir -p $O
KB_LIB_PATH=genome-assembly_amd/lib/sw2/libkbin.so timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_capacity.py tests/test_gpu_scale.py -k "heavy or prefilter or large or clustered or dropin or host_cli or track or capacity or c3 or c5 or offset or split" > $O/test_sw2.txt 2>&1 || exit 1
for i in 1 2; do
  KB_LIB_PATH=genome-assembly_amd/lib/sw2/libkbin.so timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 1 --digest > $O/c5_sw2_$i.json 2> $O/c5_sw2_$i.err || exit 1
  timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 1 --digest > $O/c5_cur_$i.json 2> $O/c5_cur_$i.err || exit 1
done
KB_LIB_PATH=genome-assembly_amd/lib/sw2/libkbin.so timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c3 --steps 2 --warmup 1 --digest > $O/c3_sw2.json 2> $O/c3_sw2.err || exit 1
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c3 --steps 2 --warmup 1 --digest > $O/c3_cur.json 2> $O/c3_cur.err || exit 1
echo rc=$?
