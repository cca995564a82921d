"""Per-step kernel time vs wall time from a rocprofv3 kernel trace: the
decode steps of a single-stream run (one step = the dispatches between two
sample_kernel launches).  Usage: python tools/trace_gaps.py run_kernel_trace.csv"""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(.*", "", n)
    return n.replace("void ", "").replace("lsd::", "")[:60]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
steps, cur = [], []
for r in rows:
    cur.append(r)
    if "sample_kernel" in r["Kernel_Name"]:
        steps.append(cur)
        cur = []
steps = steps[-20:]  # steady-state decode steps
busy = gaps = span = 0
per = collections.defaultdict(lambda: [0, 0.0])
gap_after = collections.defaultdict(lambda: [0, 0.0])
for s in steps[1:]:
    t0, t1 = int(s[0]["Start_Timestamp"]), int(s[-1]["End_Timestamp"])
    span += t1 - t0
    prev_end = None
    for r in s:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += b - a
        k = short(r["Kernel_Name"])
        per[k][0] += 1
        per[k][1] += b - a
        if prev_end is not None:
            gaps += max(0, a - prev_end)
            gap_after[k][0] += 1
            gap_after[k][1] += max(0, a - prev_end)
        prev_end = b
n = len(steps) - 1
print(f"steps {n}: span {span / n / 1e3:.1f} us, kernel busy {busy / n / 1e3:.1f} us, gaps {gaps / n / 1e3:.1f} us, "
      f"{sum(v[0] for v in per.values()) / n:.0f} dispatches per step")
for k, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
    g = gap_after[k]
    print(f"  {k:60s} {c / n:6.1f}/step {t / c / 1e3:7.2f} us avg  gap-before {g[1] / max(1, g[0]) / 1e3:5.2f} us")
