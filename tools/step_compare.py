"""Per-kernel time of the last full step (between the last two optimizer launches) of two
rocprofv3 kernel traces: python tools/step_compare.py DIR_A DIR_B"""
import collections
import csv
import glob
import sys


def last_step(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "rmsprop" in r["Kernel_Name"]]
    seg = rows[marks[-2] + 1:marks[-1] + 1]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in seg:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[n][0] += 1
        agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
    return agg, span


a, sa = last_step(sys.argv[1])
b, sb = last_step(sys.argv[2])
print(f"step span A {sa:.0f} us  B {sb:.0f} us")
for k in sorted(set(a) | set(b), key=lambda k: -max(a.get(k, [0, 0])[1], b.get(k, [0, 0])[1])):
    ca, ta = a.get(k, [0, 0.0])
    cb, tb = b.get(k, [0, 0.0])
    if max(ta, tb) > 5:
        print(f"{ca:4d} {ta:9.1f}  {cb:4d} {tb:9.1f}  {tb - ta:+8.1f}  {k[:70]}")
