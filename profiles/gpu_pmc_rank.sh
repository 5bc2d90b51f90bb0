# PMC passes over the stage-3 rank of all 58 rows at c4 (profiles/stage3_probe.py --all-only)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_rank
mkdir -p $OUT
export TMPDIR=/tmp; cd /tmp
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --kernel-include-regex "xs_rank" -d $OUT/p$i -o pmc --output-format csv -- python3 $R/profiles/stage3_probe.py --all-only --days 500 > $OUT/p$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 $R/profiles/pmc_table.py $OUT > $OUT/table.txt && cat $OUT/table.txt
