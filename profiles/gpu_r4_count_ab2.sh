# doc_pdf count variants: pdf / golden / null / full-size GPU tests on the default build,
# then every stage-1 launch alone for VARIANTS (profiles/gpu_r4_alone_ab.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "pdf or golden or null or fullsize" > gpurun_out/pdf_tests.log 2>&1 || { tail -30 gpurun_out/pdf_tests.log; exit 1; }
tail -2 gpurun_out/pdf_tests.log
VARIANTS="${VARIANTS:-a b c}" bash profiles/gpu_r4_alone_ab.sh
