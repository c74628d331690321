"""profiles/pmc_<case>.json from a tools/pmc_conv.sh run: HBM bytes per launch of the kernel.
FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch (rocprofv3 derived counters); on gfx950
FETCH_SIZE counts half the bytes of 16-B/lane streaming reads (MI355X_MICROARCH.md, HBM), so it is
doubled.  Usage: python tools/pmc_json.py gpurun_out/pmc_tcn_fwd_c64 conv_tile profiles/pmc_tcn_fwd_c64.json"""
import collections
import csv
import glob
import json
import sys

d, kern, out = sys.argv[1], sys.argv[2], sys.argv[3]
vals = collections.defaultdict(list)
for f in sorted(glob.glob(d + "/p*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
mean = {k: sum(v) / len(v) for k, v in vals.items()}
fetch = mean.get("FETCH_SIZE")
write = mean.get("WRITE_SIZE")
res = {"kernel": kern, "source": d, "counters_mean_per_dispatch": mean}
if fetch is not None and write is not None:
    res["fetch_bytes_corrected"] = 2 * fetch * 1024
    res["write_bytes"] = write * 1024
    res["hbm_bytes_per_launch"] = res["fetch_bytes_corrected"] + res["write_bytes"]
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "counters_mean_per_dispatch"}, indent=1))
