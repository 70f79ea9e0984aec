"""Summarise rocprofv3 ``--pmc`` output: per kernel (name prefix), the mean of every counter over its
dispatches.  Reads CSVs (``--output-format csv``) or the default rocpd SQLite ``*.db`` (view
``counters_collection``); ``--split-ms X`` keys dispatches of one kernel by duration (< / >= X ms) so
two shapes with the same kernel and grid are reported apart.
Usage: python tools/pmc_summary.py <counter_collection.csv | results.db>... [--match fa_] [--split-ms 1]"""
import csv
import sqlite3
import sys
from collections import defaultdict


def _rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        q = ("select kernel_name, grid_size, counter_name, sum(value), max(duration) from counters_collection "
             "group by dispatch_id, counter_name")
        for name, grid, ctr, val, dur in c.execute(q):
            yield {"Kernel_Name": name, "Grid_Size": grid, "Counter_Name": ctr, "Counter_Value": val, "dur_ns": dur}
        return
    with open(path) as f:
        yield from csv.DictReader(f)


def main(argv):
    match = ""
    if "--match" in argv:
        i = argv.index("--match")
        match = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    split = None
    if "--split-ms" in argv:
        i = argv.index("--split-ms")
        split = float(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    acc = defaultdict(lambda: defaultdict(list))
    for path in argv:
        for row in _rows(path):
            name = row["Kernel_Name"].split("(")[0].replace("void ", "")
            if match and match not in name:
                continue
            if split is not None and row.get("dur_ns") is not None:
                name += f"  [grid {row.get('Grid_Size')}, {'>=' if row['dur_ns'] >= split * 1e6 else '<'}{split} ms]"
            acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for name, ctrs in sorted(acc.items()):
        print(name)
        for c, vals in sorted(ctrs.items()):
            print(f"  {c:32s} {sum(vals) / len(vals):16.1f}  (n={len(vals)})")


if __name__ == "__main__":
    main(sys.argv[1:])
