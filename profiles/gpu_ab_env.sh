# A/B of one build under two environments: bench.py alternately with ENV_A and ENV_B
# (e.g. ENV_A="MFF_PDF_OVERLAP=0" ENV_B="MFF_PDF_OVERLAP=1"), two runs each.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/abenv
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for v in A B; do
    eval "E=\$ENV_$v"
    env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --steps 5 --warmup 2 ${BENCH_ARGS:-} > $OUT/$v$rep.log 2>&1 || { echo "RUN $v$rep FAILED"; tail -20 $OUT/$v$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/$v$rep.log') if l.startswith('{')][0]); print('$v$rep', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms/step', 'stage1', d['roofline']['avg_kernel_ms'])"
  done
done
