#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes: every *counter_collection.csv under the
given directories, mean per dispatch for each (kernel, counter), lsd:: GEMM
kernels only (the PMC programs also run torch init kernels).  Derived:
MFMA busy share, wait share, L2 hit rate, mean L2 read latency (cycles),
VMEM instructions in flight per wave.
usage: pmc_table.py DIR [DIR ...]   (DIR names become the row labels' prefix)"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "")
                if "lsd::" not in k:
                    continue
                k = k.split("(")[0].replace("void ", "")
                acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    return {k: {c: v / max(1, len(disp[k])) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    label_rows = defaultdict(dict)
    for d in sys.argv[1:]:
        case = os.path.basename(d.rstrip("/")).rsplit("-", 1)[0]
        for k, cs in load(d).items():
            label_rows[(case, k)].update(cs)
    for (case, k), cs in sorted(label_rows.items()):
        print(f"== {case}: {k}")
        for c in sorted(cs):
            print(f"   {c:40s} {cs[c]:.4g}")
        g = cs.get
        if g("SQ_WAVE_CYCLES"):
            print(f"   -> wait_any / wave_cycles          {g('SQ_WAIT_ANY', 0) / g('SQ_WAVE_CYCLES'):.3f}")
            print(f"   -> wait_inst_any / wave_cycles     {g('SQ_WAIT_INST_ANY', 0) / g('SQ_WAVE_CYCLES'):.3f}")
        if g("SQ_INSTS_VMEM_RD") and g("SQ_INST_LEVEL_VMEM"):
            print(f"   -> VMEM level / VMEM insts         {g('SQ_INST_LEVEL_VMEM') / g('SQ_INSTS_VMEM_RD'):.1f}")
        if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum"):
            print(f"   -> L2 hit rate                     {g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.3f}")
        if g("TCP_TCC_READ_REQ_sum"):
            print(f"   -> L2 read latency (cycles)        {g('TCP_TCC_READ_REQ_LATENCY_sum', 0) / g('TCP_TCC_READ_REQ_sum'):.1f}")


if __name__ == "__main__":
    main()
