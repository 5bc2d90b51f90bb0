"""Per-kernel table of rocprofv3 --pmc counter values (summed over dispatches) from the
pass directories written by profiles/gpu_pmc.sh.   python profiles/pmc_table.py DIR"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    tab = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for path in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if not (name.startswith("mff") or name.startswith("void mff")):
                    continue
                short = name.split("(")[0].replace("void ", "")
                tab[short][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[short].add(row["Dispatch_Id"])
    for k, cs in sorted(tab.items()):
        print(f"== {k}  dispatches={len(disp[k])}")
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {v:18.6g}")


if __name__ == "__main__":
    main()
