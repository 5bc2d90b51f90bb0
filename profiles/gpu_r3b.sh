# round 3: GPU tests, stage-3 rank A/B (a = HEAD, b = working tree), then the group-kernel
# ablations (serial launches: per-kernel stats)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash profiles/gpu_tests.sh || exit 1
VARIANTS="a b" bash profiles/gpu_s3_ab.sh || exit 1
MFF_PDF_OVERLAP=0 MFF_HL_STREAM=0 VARIANTS="${VARIANTS:-a c d e f}" bash profiles/gpu_ab.sh
