# Launch-order / stream-priority sweep of one build: bench.py (pass throughput) under each
# environment given as an argument ("-" = defaults), interleaved, REPS rounds.
# usage: bash profiles/gpu_r4_env_sweep.sh - "MFF_HL_PRIO=0" "MFF_PDF_PRIO=-1" ...
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/envsweep
mkdir -p $OUT
cd $R
for rep in $(seq 1 ${REPS:-2}); do
  i=0
  for E in "$@"; do
    [ "$E" = "-" ] && E=""
    env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --steps ${STEPS:-10} --warmup 2 > $OUT/v$i.$rep.log 2>&1 || { echo "RUN [$E] FAILED"; tail -20 $OUT/v$i.$rep.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/v$i.$rep.log') if l.startswith('{')][0]); print('v$i.$rep', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', '[$E]')"
    i=$((i+1))
  done
done
