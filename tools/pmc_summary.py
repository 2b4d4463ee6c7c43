"""Per-kernel mean of each counter in rocprofv3 counter_collection.csv files: python tools/pmc_summary.py DIR..."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    for path in glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True):
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in acc.items():
            if "gemm" not in k and "wres" not in k:
                continue
            print(d.split("/")[-1], k)
            print("   " + "  ".join(f"{c}={sum(v) / len(v):.3g}" for c, v in sorted(cs.items())))
