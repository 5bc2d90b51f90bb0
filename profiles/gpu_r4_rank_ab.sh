# stage-3 rank A/B: all 58 rows at c4 with each in-tree mff/libmff_<v>.so (VARIANTS), twice
# each, then PMC passes over the default library's rank kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT
PKG=replication-of-minute-frequency-factor_amd
O=$R/gpurun_out/r4rank_ab
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in ${VARIANTS:-a b}; do
    echo -n "$v$rep "
    MFF_LIBRARY=$R/$PKG/mff/libmff_$v.so timeout -k 10 200 python3 profiles/stage3_probe.py --all-only 2>&1 | grep "all rows" || exit 1
  done
done
export TMPDIR=/tmp
cd /tmp
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  MFF_LIBRARY=$R/$PKG/mff/libmff_${PMC_VARIANT:-a}.so timeout -s KILL 90 rocprofv3 --pmc $pmc --kernel-include-regex "xs_rank" -d $O/p$i -o pmc --output-format csv -- python3 $R/profiles/stage3_probe.py --all-only --days 500 > $O/p$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 $R/profiles/pmc_table.py $O > $O/table.txt && cat $O/table.txt
