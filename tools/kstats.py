import csv, sys
f = sys.argv[1]; steps = float(sys.argv[2]) if len(sys.argv) > 2 else 7
rows = list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs'])/steps/1e6:7.3f}ms/step {float(r['Percentage']):6.2f}% n={int(r['Calls'])/steps:>5.1f} avg={float(r['AverageNs'])/1e3:8.1f}us {r['Name'][:105]}")
print('total ms/step', tot / steps / 1e6)
