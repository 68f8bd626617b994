set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu.sh ktrace zs8 --reads 8000000 --genome 40000000 --parts 8 --steps 3 --warmup 1 && \
bash tools/gpu.sh ktrace zs2 --reads 2000000 --genome 10000000 --parts 2 --steps 3 --warmup 1
echo rc=$?
