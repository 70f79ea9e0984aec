"""Per-step kernel breakdown of a serving run from a rocprofv3 ``*_kernel_trace.csv``.

Steps are delimited by ``sample_kernel`` dispatches; a step containing ``paged_decode_kernel`` is a
decode step.  Prints, for the decode steps (optionally only the last N), the mean wall time per
step (first kernel start -> sampler end) and the mean time per step of each kernel family."""
import collections
import csv
import sys


def family(name: str) -> str:
    n = name.split("(")[0].replace("void ", "")
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"):
        return "gemm:" + n.split("_MT")[1].split("_")[0] if "_MT" in n else "gemm"
    return n.split("<")[0]


rows = list(csv.DictReader(open(sys.argv[1])))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 0
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
steps, cur = [], []
for r in rows:
    cur.append(r)
    if r["Kernel_Name"].startswith("sample_kernel"):
        steps.append(cur)
        cur = []
dec = [s for s in steps if any("paged_decode_kernel" in r["Kernel_Name"] for r in s)]
if last:
    dec = dec[-last:]
agg = collections.defaultdict(float)
wall = 0.0
for s in dec:
    ks = [r for r in s if int(r["End_Timestamp"]) > 0]
    first = next(i for i, r in enumerate(ks) if "rocclr" not in r["Kernel_Name"])
    ks = ks[first:]
    wall += (int(ks[-1]["End_Timestamp"]) - int(ks[0]["Start_Timestamp"])) / 1e3
    for r in ks:
        agg[family(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
n = max(1, len(dec))
busy = sum(agg.values()) / n
print(f"decode steps: {len(dec)}  wall/step {wall/n:.1f} us  kernel-busy/step {busy:.1f} us")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
    print(f"  {v/n:10.1f} us  {100*v/n/busy:5.1f}%  {k}")
