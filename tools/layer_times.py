"""Per-kernel durations of one decoder layer (fwd + bwd) from a rocprofv3 kernel trace (last step)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[2 * len(rows) // 3:]
def dur(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
fw = [i for i, r in enumerate(last) if "fa_fwd" in r["Kernel_Name"]]
bw = [i for i, r in enumerate(last) if "dkdv" in r["Kernel_Name"]]
for title, idx, lo, hi in (("forward", fw, -6, 5), ("backward", bw, -12, 7)):
    if len(idx) < 4:
        continue
    i = idx[3]
    print("==", title)
    for r in last[i + lo:i + hi]:
        print(f"{dur(r):8.1f}us  {r['Kernel_Name'][:100]}")
