import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
steps=float(sys.argv[2]) if len(sys.argv)>2 else 1
for r in rows[:14]:
    n=r['Name']; n=n.replace('void ','').replace('rsvd::(anonymous namespace)::','').split('(')[0][:50]
    print(f"{n:50s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:9.2f} per_step_us={float(r['TotalDurationNs'])/1e3/steps:9.1f} pct={float(r['Percentage']):5.1f}")
