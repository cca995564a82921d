"""Idle gaps of a multi-lane kernel trace: the union of all kernels' busy
intervals over the last `window_ms`, and the idle gaps >= `min_us` grouped by
the kernel that ended before the gap and the one that started after it.
Usage: python tools/gap_union.py run_kernel_trace.csv [window_ms] [min_us]"""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(.*", "", n)
    return n.replace("void ", "").replace("lsd::", "")[:48]


rows = list(csv.DictReader(open(sys.argv[1])))
window = float(sys.argv[2]) if len(sys.argv) > 2 else 200.0
min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 3.0
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
            for r in rows)
t_end = max(e for _, e, _ in ev)
ev = [x for x in ev if x[0] >= t_end - window * 1e6]
busy = 0
gaps = collections.defaultdict(lambda: [0, 0.0])
cur_s, cur_e, cur_n = ev[0]
for s, e, n in ev[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        g = (s - cur_e) / 1e3
        if g >= min_us:
            k = gaps[(cur_n, n)]
            k[0] += 1
            k[1] += g
        cur_s, cur_e, cur_n = s, e, n
    elif e > cur_e:
        cur_e, cur_n = e, n
busy += cur_e - cur_s
span = cur_e - ev[0][0]
print(f"window {span / 1e3:.1f} us  busy {busy / 1e3:.1f} us  idle {(span - busy) / 1e3:.1f} us "
      f"({100 * (span - busy) / span:.1f} %)  kernels {len(ev)}")
tot = sum(v[1] for v in gaps.values())
print(f"gaps >= {min_us} us: {tot:.1f} us")
for (a, b), (c, t) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"{t:9.1f} us  n={c:4d}  avg {t / c:7.1f}  {a}  ->  {b}")
