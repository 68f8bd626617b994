#!/usr/bin/env bash
# tools/gpu.sh -- the GPU-box recipes, run under gpurun from the repo root:
#   gpurun --timeout 1200 -- 'bash tools/gpu.sh test && bash tools/gpu.sh bench c2'
#
#   test [pytest args]          the -m gpu suite (one process, per-test timeout)
#   bench TAG [bench.py args]   one bench line -> gpurun_out/bench_TAG.json
#   ktrace TAG [bench.py args]  rocprofv3 kernel trace + stats -> gpurun_out/kt_TAG/
#   pmc TAG [bench.py args]     FETCH_SIZE and WRITE_SIZE in two separate --pmc
#                               passes -> gpurun_out/pmc_TAG_{fetch,write}/
#   sq TAG [bench.py args]      one --pmc pass of 8 SQ counters (or $SQ_SET) -> gpurun_out/sq_TAG/
#
# Every GPU step runs under its own `timeout -k 10`; a failing step ends the
# script with its exit status (callers chain modes with &&).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
mode=${1:?mode}; shift
case $mode in
  test)
    timeout -k 10 1500 python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread \
      tests "$@" > gpurun_out/tests.log 2>&1
    rc=$?; tail -3 gpurun_out/tests.log; exit $rc ;;
  bench)
    tag=${1:?tag}; shift
    timeout -k 10 900 python -u bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
    rc=$?; cat gpurun_out/bench_$tag.json; exit $rc ;;
  ktrace)
    tag=${1:?tag}; shift
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$tag -o kt \
      -- python3 bench.py --cpu-sample 0 "$@" > gpurun_out/kt_$tag.log 2>&1 ;;
  pmc)
    tag=${1:?tag}; shift
    timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${tag}_fetch -o pmc \
      -- python3 bench.py --cpu-sample 0 "$@" > gpurun_out/pmc_${tag}_fetch.log 2>&1 && \
    timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${tag}_write -o pmc \
      -- python3 bench.py --cpu-sample 0 "$@" > gpurun_out/pmc_${tag}_write.log 2>&1 ;;
  sq)
    tag=${1:?tag}; shift
    # SQ_SET: another 8 counters for the same pass (one block, at most 8 SQ_)
    timeout -k 10 600 rocprofv3 --pmc ${SQ_SET:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE} --output-format csv \
      -d gpurun_out/sq_$tag -o sq -- python3 bench.py --cpu-sample 0 "$@" > gpurun_out/sq_$tag.log 2>&1 ;;
  *) echo "unknown mode $mode" >&2; exit 2 ;;
esac
