#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs: per kernel (name prefix), the mean of each
counter over its dispatches, plus derived ratios when the counters are present.
Usage: python tools/pmc_summary.py DIR [DIR ...]   (each DIR holds */run_counter_collection.csv)"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    out = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[key[0]] = r["Kernel_Name"]
        for (disp, cn), v in per.items():
            out[names[disp][:80]][cn].append(v)
    return out


def main():
    agg = defaultdict(dict)
    for d in sys.argv[1:]:
        for k, cs in load(d).items():
            for cn, vs in cs.items():
                agg[k][cn] = sum(vs) / len(vs)
    for k, cs in agg.items():
        print(f"== {k}")
        for cn in sorted(cs):
            print(f"   {cn:40s} {cs[cn]:.4g}")
        g = cs.get
        if g("SQ_VALU_MFMA_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE"):
            # MFMA busy per SIMD over the kernel's active cycles (GRBM_GUI_ACTIVE sums 8 XCDs)
            simds = 256 * 4
            print(f"   -> MFMA busy / SIMD-cycles           {g('SQ_VALU_MFMA_BUSY_CYCLES') / (g('GRBM_GUI_ACTIVE') / 8 * simds):.3f}")
        if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None:
            h, m = g("TCC_HIT_sum"), g("TCC_MISS_sum")
            print(f"   -> L2 hit rate                       {h / max(h + m, 1):.3f}")
        if g("SQ_WAIT_ANY") and g("SQ_WAVE_CYCLES"):
            print(f"   -> wait_any / wave_cycles            {g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
        if g("SQ_LDS_BANK_CONFLICT") and g("SQ_LDS_IDX_ACTIVE"):
            print(f"   -> LDS bank conflict / active        {g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):.3f}")
        if g("TCP_TCC_READ_REQ_LATENCY_sum") and g("TCP_TCC_READ_REQ_sum"):
            print(f"   -> L2 read latency (cycles)          {g('TCP_TCC_READ_REQ_LATENCY_sum') / g('TCP_TCC_READ_REQ_sum'):.1f}")


if __name__ == "__main__":
    main()
