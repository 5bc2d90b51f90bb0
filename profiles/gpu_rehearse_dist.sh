# 2-rank torchrun rehearsal of bench.py on ONE GPU (both ranks share cuda:0; gloo host
# collectives instead of RCCL): exercises the launcher env, shard bounds, the doc_pdf /
# stage-3 exchange path, barriers and the max-over-ranks timing end to end.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/dist
cd $R
MFF_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --days ${DAYS:-250} \
  --no-cpu-baseline > gpurun_out/dist/bench2.log 2>&1 || { echo DIST_FAILED; tail -40 gpurun_out/dist/bench2.log; exit 1; }
grep '^{' gpurun_out/dist/bench2.log
# the same launcher with an asserted result: sharded engine == unsharded pass (rank 0)
MFF_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 profiles/dist_check.py > gpurun_out/dist/check2.log 2>&1 \
  || { echo DIST_CHECK_FAILED; tail -40 gpurun_out/dist/check2.log; exit 1; }
grep -E "mismatches|NaN pattern|doc_pdf rows|DIST_CHECK" gpurun_out/dist/check2.log
