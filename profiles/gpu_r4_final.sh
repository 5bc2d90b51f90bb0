# round-4 final measurement of the working tree: every -m gpu test, smoke(), the default
# bench line, the stage-1 rocprofv3 profile (overlapped timeline + serial stats) and the
# PMC passes.  usage: bash profiles/gpu_r4_final.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r04c}
cd $R
bash profiles/gpu_round_check.sh $TAG || exit 1
bash profiles/gpu_r3_prof.sh $TAG || exit 1
bash profiles/gpu_pmc.sh $TAG || exit 1
