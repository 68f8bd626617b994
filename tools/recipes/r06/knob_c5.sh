# r06: C5 share knob sweep (digest-checked): table load for partition sizing
# (KB_BIN_FILL_PCT 60 default), the heavy windows (KB_BIN_WIN_HEAVY2), the
# flat depth (KB_BIN_FLAT_L)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/knob_c5; mkdir -p $O
run() {
  local nm=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 1 --digest > $O/$nm.json 2>> $O/err.txt || exit 1
}
run base KB_BIN_FILL_PCT=60
run fill70 KB_BIN_FILL_PCT=70
run fill80 KB_BIN_FILL_PCT=80
run wh2off KB_BIN_WIN_HEAVY2=0
run flatl4 KB_BIN_FLAT_L=4
run base2 KB_BIN_FILL_PCT=60
echo done
