"""Build a variant of the working tree's csrc as mff/libmff_<v>.so for profiles/gpu_ab.sh.

usage: python profiles/ab_variant.py <letter> <file> <old> <new> [<file> <old> <new> ...]
The sources are copied to /tmp/mff_ab_<letter> and patched there (exact string
replacement, each `old` must occur once), so the working tree is never touched.  Used
for ablations (time a kernel with one section removed) and quick alternatives.
"""
import os
import shutil
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "replication-of-minute-frequency-factor_amd"


def main():
    v = sys.argv[1]
    edits = sys.argv[2:]
    tmp = f"/tmp/mff_ab_{v}"
    shutil.rmtree(tmp, ignore_errors=True)
    os.makedirs(f"{tmp}/{PKG}")
    shutil.copytree(f"{R}/{PKG}/csrc", f"{tmp}/{PKG}/csrc")
    shutil.copy(f"{R}/{PKG}/Makefile", f"{tmp}/{PKG}/Makefile")
    shutil.copytree(f"{R}/include", f"{tmp}/include")
    for i in range(0, len(edits), 3):
        f, old, new = edits[i:i + 3]
        p = f"{tmp}/{PKG}/csrc/{f}"
        s = open(p).read()
        assert s.count(old) == 1, f"{f}: pattern found {s.count(old)} times: {old[:60]!r}"
        open(p, "w").write(s.replace(old, new))
    subprocess.check_call(["make", "-s", "-C", f"{tmp}/{PKG}", "-j8", f"BUILD={tmp}/build",
                           f"LIB={R}/{PKG}/mff/libmff_{v}.so"])
    print(f"built {PKG}/mff/libmff_{v}.so")


if __name__ == "__main__":
    main()
