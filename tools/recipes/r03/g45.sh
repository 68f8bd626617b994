# round 3b: g43 (serpentine vs LPT prior maps: cold C2 steps, prior parity
# cases) then g44 (a C4-share run's large allocations after another job)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/recipes/r03/g43.sh && bash tools/recipes/r03/g44.sh
