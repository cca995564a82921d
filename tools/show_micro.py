import json, sys
for l in open(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/micro.log'):
    l = l.strip()
    if not l.startswith('{'):
        print(l); continue
    d = json.loads(l)
    if d['case'].startswith('stamps'):
        print(d['case'], 'entry', d['entry_us'][1:3], 'load', d['load_us'], 'comp', d['compute_us'], 'pub', d['publish_us'], 'red', d['reduce_us'], 'span', d['span_us'])
    else:
        print(f"{d['case']:52s} {d['us']:8.2f}us {d['TB/s']:6.2f}TB/s  {d.get('hipblaslt_us','')} {d.get('TFLOP/s','')}")
