# r06: the conversion's time against its fan-out: C3 kernel stats with 1024
# (default), 256 and 64 local buckets (KB_BIN_NB) -- what a grouped
# conversion (each batch scattering into 64 buckets) could reach
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/kt_c3_nb; mkdir -p $O
for nb in 1024 256 64; do
  KB_BIN_NB=$nb timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/nb$nb -o kt -- python3 bench.py --cpu-sample 0 --workload c3 --steps 1 --warmup 1 > $O/nb$nb.log 2>&1 || exit 1
done
echo done
