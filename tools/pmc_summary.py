"""Summarise rocprofv3 ``--pmc`` CSVs: per kernel (name prefix), the mean of every counter over its
dispatches.  Usage: python tools/pmc_summary.py <counter_collection.csv>... [--match fa_]"""
import csv
import sys
from collections import defaultdict


def main(argv):
    match = ""
    if "--match" in argv:
        i = argv.index("--match")
        match = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    acc = defaultdict(lambda: defaultdict(list))
    for path in argv:
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"].split("(")[0].replace("void ", "")
                if match and match not in name:
                    continue
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for name, ctrs in sorted(acc.items()):
        print(name)
        for c, vals in sorted(ctrs.items()):
            print(f"  {c:32s} {sum(vals) / len(vals):16.1f}  (n={len(vals)})")


if __name__ == "__main__":
    main(sys.argv[1:])
