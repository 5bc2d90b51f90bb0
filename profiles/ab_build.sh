# Build the committed HEAD as mff/libmff_a.so and the working tree as mff/libmff_b.so
# (both in-tree, git-ignored) for profiles/gpu_ab.sh.  HEAD is exported with
# `git archive` into /tmp, so the working tree is never touched.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
PKG=replication-of-minute-frequency-factor_amd
rm -rf /tmp/mff_ab_head && mkdir -p /tmp/mff_ab_head
git -C "$R" archive HEAD "$PKG/csrc" "$PKG/Makefile" include | tar -x -C /tmp/mff_ab_head
make -s -C /tmp/mff_ab_head/$PKG -j8 BUILD=/tmp/mff_ab_head/build LIB="$R/$PKG/mff/libmff_a.so"
make -s -C "$R/$PKG" -j8 BUILD=build_b LIB=mff/libmff_b.so
ls -la "$R/$PKG/mff/"libmff_[ab].so
