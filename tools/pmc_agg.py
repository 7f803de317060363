"""Dev tool: aggregate rocprofv3 --pmc counter CSVs (one dir per pass) per kernel."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
meta = {}
for f in sorted(glob.glob(sys.argv[1] + "/pmc*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void cbh::", "").replace("cbh::", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[k] = (r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Workgroup_Size"])
for k, v in agg.items():
    print(k, "vgpr/sgpr/lds/wg", meta[k])
    for a in sorted(v):
        print(f"    {a:28s} {v[a]:.4e}")
