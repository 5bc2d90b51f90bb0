# round 4: parity of the working tree (selected GPU test files, then everything), then an
# A/B bench of HEAD (libmff_a) vs the working tree (libmff_b).
# usage: bash profiles/gpu_r4_check_ab.sh TAG "test files"
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r04}
FIRST=${2:-tests/test_gpu_parity.py}
OUT=$R/gpurun_out/tests_$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest $FIRST -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/first.log 2>&1 || { echo FIRST_FAILED; tail -60 $OUT/first.log; exit 1; }
tail -2 $OUT/first.log
bash profiles/gpu_ab.sh || exit 1
if [ "$3" = "all" ]; then
  cd $R
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/all.log 2>&1 || { echo ALL_FAILED; tail -60 $OUT/all.log; exit 1; }
  tail -2 $OUT/all.log
fi
