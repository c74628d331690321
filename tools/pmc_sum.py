import csv, glob, sys, collections
d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "conv"
vals = collections.defaultdict(list)
for f in sorted(glob.glob(d + "/p*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in vals.items():
    print("%-28s n=%3d  mean %.4g" % (k, len(v), sum(v) / len(v)))
