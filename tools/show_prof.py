import csv, sys
rows = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof/run_kernel_stats.csv')))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 18]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['Percentage']):6.2f}% calls={r['Calls']:>6} avg={float(r['AverageNs'])/1e3:8.2f}us  {r['Name'][:90]}")
print('total kernel ms', round(tot / 1e6, 2))
