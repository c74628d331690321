import csv
import sys

key = sys.argv[1] if len(sys.argv) > 1 else "wgrad3"
for tg in sys.argv[2:] or ("512", "1024", "2048"):
    rows = list(csv.DictReader(open(f"gpurun_out/pf{tg}/p_kernel_trace.csv")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if key in r["Kernel_Name"]]
    print(tg, " ".join(f"{x:.0f}" for x in ks[-9:]), round(sum(ks[-9:]), 1))
