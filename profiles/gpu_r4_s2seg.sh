# stage-2 day segments: parity tests, then the bench's stage-2 extra (z, N = 20, all 58
# rows at c4) under MFF_S2_SEGS = 1 / 4 / 8, interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "stage2" > gpurun_out/s2seg_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/s2seg_tests.log; exit 1; }
tail -1 gpurun_out/s2seg_tests.log
for rep in 1 2; do
  for n in 1 4 8; do
    MFF_S2_SEGS=$n timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/s2seg_$n.$rep.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/s2seg_$n.$rep.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/s2seg_$n.$rep.log') if l.startswith('{')][0]); e=d['extras']; print('segs $n rep $rep', e['stage2_z20_all58_ms'], 'ms', e['stage2_z20_GBps'], 'GB/s')"
  done
done
