# round 3: GPU tests of the working tree, then A/B of the pass (a = HEAD, b = tree, + VARIANTS)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash profiles/gpu_tests.sh ${TESTS:-} || exit 1
VARIANTS="${VARIANTS:-a b}" bash profiles/gpu_ab.sh
