# N-rank receiver emulation with per-rank genomes (genome grows with N, 30x coverage), kernel traces
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for w in "2000000 10000000 2" "8000000 40000000 8"; do
  set -- $w
  timeout -k 10 300 python bench.py --reads $1 --genome $2 --parts $3 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/g_$3.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gk_$3 -o kt -- python3 bench.py --reads $1 --genome $2 --parts $3 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/gk_$3.log 2>&1 || exit 1
done
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 200 python bench.py --reads 8000000 --genome 40000000 --parts 8 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/gbp8.log 2>&1
echo rc=$?
