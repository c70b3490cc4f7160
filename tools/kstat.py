import csv, sys, glob
for f in sys.argv[1:]:
    print("==", f)
    rows = list(csv.DictReader(open(f)))
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
        print(f"{float(r['AverageNs'])/1e3:9.1f} us x{int(r['Calls']):4d}  {r['Name'][:110]}")
