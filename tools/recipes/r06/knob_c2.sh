# r06: C2 knob sweep (20 steps each, alternating with the default)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/knob_c2; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 3"
run() { local nm=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $NOX > $O/$nm.json 2>> $O/err.txt || exit 1; }
run base1 KB_X=0
run fl40 KB_BIN_FILL_LIGHT_PCT=40
run fl60 KB_BIN_FILL_LIGHT_PCT=60
run base2 KB_X=0
run f50 KB_BIN_FILL_PCT=50
run f70 KB_BIN_FILL_PCT=70
run base3 KB_X=0
run op3 KB_BIN_OPART=3
run sub96 KB_BIN_SUB_EXTRA=96
run base4 KB_X=0
run fsl0 KB_BIN_FSL=0
run bal0 KB_BIN_BIG_DIV=4
echo done
