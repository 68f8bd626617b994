# Round profile set for profiles/: PMC calibration, kernel trace stats, HBM
# traffic (FETCH_SIZE and WRITE_SIZE in separate --pmc passes), default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/cal_f -o cal -- tools/pmc_calib > gpurun_out/cal_f.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/cal_w -o cal -- tools/pmc_calib > gpurun_out/cal_w.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/prof_kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o pmc -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/pmc_f.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o pmc -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/pmc_w.log 2>&1 && \
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo rc=$?
