"""Mean counter values per kernel name from rocprofv3 --pmc CSV passes under a directory
(tools/pmc_kernel.sh output): python tools/pmc_csv_summary.py gpurun_out/<dir> [name-filter]"""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        if flt not in name:
            continue
        acc[name[:90]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for name, cs in acc.items():
    print(name)
    for c, v in sorted(cs.items()):
        print(f"  {c:28s} {sum(v) / len(v):14.0f}  (n={len(v)})")
