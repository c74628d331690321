import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 14]:
    print("%6.2f%% %8.2f ms/step %5d calls avg %8.1f us  %s" % (100 * float(r['TotalDurationNs']) / tot, float(r['TotalDurationNs']) / 1e6 / steps, int(r['Calls']), float(r['AverageNs']) / 1e3, r['Name'][:90]))
print("total ms/step %.2f" % (tot / 1e6 / steps))
