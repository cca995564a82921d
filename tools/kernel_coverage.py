"""GPU occupancy from a rocprofv3 kernel trace (the whole-session variant of
gap_union.py, which attributes the gaps of a short window): the union of all kernel
intervals (any stream) against the wall span, over the whole trace and over
the longest stretch of decode-step kernels.  Gaps = the device running
nothing (host issue, synchronisation, transfers outside kernels).

  python tools/kernel_coverage.py gpurun_out/cov/*kernel_trace.csv
"""
import csv
import sys


def union(iv):
    iv.sort()
    tot, cs, ce, gaps = 0, None, None, []
    for s, e in iv:
        if cs is None:
            cs, ce = s, e
        elif s > ce:
            tot += ce - cs
            gaps.append((s - ce, ce))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot, gaps


def main(path):
    rows = list(csv.DictReader(open(path)))
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    iv.sort()
    # the timed region: from the last prefill attention launch of the trace's final session on
    pf = [s for s, e, n in iv if "attn_prefill" in n]
    t0 = pf[len(pf) // 2] if pf else iv[0][0]  # skip warm-up sessions roughly: second half of the trace
    t0 = max(s for s in pf if s <= iv[-1][0]) if pf else iv[0][0]
    sub = [(s, e) for s, e, n in iv if s >= t0]
    span = max(e for _, e in sub) - min(s for s, _ in sub)
    busy, gaps = union(sub)
    gaps.sort(reverse=True)
    print(f"last session from the final prefill attention: span {span / 1e6:.2f} ms, kernels busy "
          f"{busy / 1e6:.2f} ms = {100 * busy / span:.1f} %, {len(gaps)} gaps, total {sum(g for g, _ in gaps) / 1e6:.2f} ms")
    hist = {}
    for g, _ in gaps:
        k = "<2us" if g < 2000 else "2-10us" if g < 10000 else "10-100us" if g < 100000 else ">=100us"
        hist[k] = hist.get(k, 0) + g
    print("gap time by size (ms):", {k: round(v / 1e6, 2) for k, v in hist.items()})
    print("largest gaps (us):", [round(g / 1e3, 1) for g, _ in gaps[:10]])


if __name__ == "__main__":
    main(sys.argv[1])
