# round-4 closing measurement: stage-1 profile (bench line, pass timeline, serial stats)
# and the PMC passes at the bench's c4 config (profiles/pmc_stage1.json must match it).
# usage: bash profiles/gpu_r4_final2.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r04f}
cd $R
bash profiles/gpu_r3_prof.sh $TAG || exit 1
bash profiles/gpu_pmc.sh $TAG 5000 2500 || exit 1
