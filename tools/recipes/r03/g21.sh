# bank-spread probe: parity, C2 bench + SQ, and the per-phase LDS attribution
# (ablation build: KB_BIN_ABLATE switches bin-kernel phases off)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3r; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py::test_c2_full_vs_oracle > $O/t.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py $NOX --steps 20 --warmup 5 > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/sq -o sq -- python3 bench.py $NOX --steps 5 --warmup 2 > $O/sq.log 2>&1 || exit 1
for m in 0 7 1 2 3 5; do
  KB_LIB_PATH=genome-assembly_amd/lib/abl/libkbin.so KB_BIN_ABLATE=$m timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/abl$m -o sq -- python3 bench.py $NOX --steps 5 --warmup 2 > $O/abl$m.log 2>&1 || exit 1
done
echo rc=$?
