# A/B of stage-2 builds: profiles/stage2_probe.py quick with each in-tree
# mff/libmff_<v>.so (VARIANTS="a b ..."), twice each.
set -o pipefail
R=$GRAFT_REPO_ROOT
PKG=replication-of-minute-frequency-factor_amd
for rep in 1 2; do
  for v in ${VARIANTS:-a b}; do
    echo -n "$v$rep "
    MFF_LIBRARY=$R/$PKG/mff/libmff_$v.so timeout -k 10 200 python3 $R/profiles/stage2_probe.py quick 2>&1 | grep "^{" || exit 1
  done
done
