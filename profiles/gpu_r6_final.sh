# round-6 measurement of the working tree: every -m gpu test, smoke(), the default bench
# line, the stage-1 rocprofv3 profile (overlapped timeline + serial stats) and the c4 PMC
# passes (profiles/pmc_stage1.json is refreshed from them).
# usage: bash profiles/gpu_r6_final.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06f}
cd $R
bash profiles/gpu_r6_check.sh $TAG || exit 1
bash profiles/gpu_r3_prof.sh $TAG || exit 1
bash profiles/gpu_pmc.sh $TAG 5000 2500 || exit 1
head -12 $R/gpurun_out/pmc_$TAG/table.txt
