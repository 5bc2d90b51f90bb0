# round 3: stage-3 rank ablations (a HEAD, b no in-bucket scan, c no rank_of) and
# group-kernel ablations (d no LVL moments, e no PDF thresholds, f no val stores)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
VARIANTS="a b c" bash profiles/gpu_s3_ab.sh || exit 1
MFF_PDF_OVERLAP=0 MFF_HL_STREAM=0 VARIANTS="a d e f" bash profiles/gpu_ab.sh
