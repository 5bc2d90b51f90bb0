#!/usr/bin/env bash
# Profiling recipe (run on the GPU box via gpurun from the repo root):
#   1. kernel trace + stats of the default bench (c4: 5000 x 2500, all 58 factors)
#   2. PMC passes on the same workload, one counter group per run (gfx950 slot limits),
#      restricted to the stage-1 pass launches (k_stage1s_pair, k_stage1s<OLS|MOMH>,
#      k_stage1g<ORD|LVL|PDF>, k_stage1 exact list, k_pdf_sort / k_pdf_count).
# Outputs land in gpurun_out/prof_<tag>/; the summaries worth keeping are copied into
# profiles/<round>/ and profiles/pmc_stage1.json by profiles/summarize.py.
set -euo pipefail
TAG=${1:-r01}
STEPS=${STEPS:-3}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BENCH=("$R/bench.py" --no-cpu-baseline --no-extras)

timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv \
  -- python3 "${BENCH[@]}" --steps "$STEPS" --warmup 1 > "$OUT/trace_bench.log" 2>&1

for pmc in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  name=$(echo "$pmc" | awk '{print $1}')_$(echo "$pmc" | wc -w)
  timeout -s KILL 240 rocprofv3 --pmc $pmc --kernel-include-regex "k_stage1|k_pdf" -d "$OUT/pmc_$name" -o pmc \
    --output-format csv -- python3 "${BENCH[@]}" --steps 1 --warmup 0 > "$OUT/pmc_$name.log" 2>&1
done
python3 "$R/profiles/pass_span.py" "$OUT/trace" "$OUT/pass_spans.csv" > "$OUT/pass_spans.log" 2>&1 || true
find "$OUT" -name "*kernel_trace.csv" -delete
echo "profiles done: $OUT"
