# Build commit $1 (default HEAD) as mff/libmff_<$2, default a>.so in-tree (git archive into /tmp:
# the working tree is never touched), for profiles/gpu_ab.sh.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
PKG=replication-of-minute-frequency-factor_amd
REF=${1:-HEAD}
V=${2:-a}
T=/tmp/mff_ab_ref_$V
rm -rf $T && mkdir -p $T
git -C "$R" archive "$REF" "$PKG/csrc" "$PKG/Makefile" include | tar -x -C $T
make -s -C $T/$PKG -j8 BUILD=$T/build LIB="$R/$PKG/mff/libmff_$V.so"
ls -la "$R/$PKG/mff/libmff_$V.so"
