import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:int(sys.argv[2]) if len(sys.argv)>2 else 20]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):7d} calls {float(r['AverageNs'])/1e3:9.2f} us {float(r['Percentage']):6.2f}%  {r['Name'][:80]}")
print("total ms", tot/1e6)
