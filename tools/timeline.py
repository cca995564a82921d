"""Kernel-timeline summary of a rocprofv3 --kernel-trace CSV: per-window
concurrency (sum of kernel durations / wall span), idle gaps and a listing of
the first kernels of the window with their queue.

usage: python tools/timeline.py [trace.csv] [window_start_frac] [window_ms] [n_list]
"""
import csv
import re
import sys


def short(n):
    m = re.search(r"lsd::(\w+)(<[^>]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:40]


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
    frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.6
    win_ms = float(sys.argv[3]) if len(sys.argv) > 3 else 8.0
    n_list = int(sys.argv[4]) if len(sys.argv) > 4 else 40
    ks = []
    for r in csv.DictReader(open(path)):
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                   short(r["Kernel_Name"])))
    ks.sort()
    t0, t1 = ks[0][0], max(k[1] for k in ks)
    mid = t0 + (t1 - t0) * frac
    win = [k for k in ks if mid <= k[0] < mid + win_ms * 1e6]
    iv = sorted((a, b) for a, b, _, _ in win)
    busy, cur = 0, None
    for a, b in iv:
        if cur is None or a > cur[1]:
            if cur:
                busy += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    busy += cur[1] - cur[0]
    span = win[-1][1] - win[0][0]
    tot = sum(b - a for a, b, _, _ in win)
    print(f"kernels {len(win)}  span {span / 1e3:.1f} us  busy(union) {busy / 1e3:.1f} us  "
          f"sum {tot / 1e3:.1f} us  concurrency {tot / max(busy, 1):.2f}")
    per = {}
    for a, b, q, n in win:
        per.setdefault(n, [0, 0.0])
        per[n][0] += 1
        per[n][1] += (b - a) / 1e3
    for n, (c, d) in sorted(per.items(), key=lambda x: -x[1][1]):
        print(f"  {d:9.1f} us  n={c:5d}  avg {d / c:7.2f}  {n}")
    for k in win[:n_list]:
        print(f"{(k[0] - win[0][0]) / 1e3:9.2f} +{(k[1] - k[0]) / 1e3:7.2f} q{k[2]} {k[3]}")


if __name__ == "__main__":
    main()
