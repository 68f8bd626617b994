# r06: the routed C4 leg's receive slot after the fix -- self records by
# device copy (default), by RCCL in 256-MB pieces (KB_GROUP_SELF_RCCL=1), and
# by RCCL in one message (KB_GROUP_CHUNK=0: the failing round-6 exchange), at
# 1/4 of a rank's reads; then the default at full size
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/legs5; mkdir -p $O
run() {  # name, scale, env...
  local nm=$1 sc=$2; shift 2
  env "$@" KB_DEBUG=1 KB_CAPACITY_SCALE=$sc timeout -k 10 400 python -u bench.py --routed --multi-legs --steps 1 --warmup 0 --cpu-sample 0 --no-host-input > $O/$nm.json 2> $O/$nm.err
  local rc=$?; echo "$nm rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
run s4_copy 4 KB_GROUP_CHUNK=33554432
run s4_rccl_chunk 4 KB_GROUP_SELF_RCCL=1
run s4_rccl_whole 4 KB_GROUP_SELF_RCCL=1 KB_GROUP_CHUNK=0
run s1_copy 1 KB_GROUP_CHUNK=33554432
run s1_rccl_chunk 1 KB_GROUP_SELF_RCCL=1
echo done
