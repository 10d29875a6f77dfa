"""Per-kernel sums of rocprofv3 --pmc csv files: python scripts/pmcsum.py CSV... [--match s]"""
import collections
import csv
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
agg = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(float)
for f in args:
    if f == match:
        continue
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("lfm::", "")[:44]
        if match and match not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
cols = sorted({c for d in agg.values() for c in d})
print("%-44s " % "kernel" + " ".join("%13s" % c[-13:] for c in cols))
for k, d in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", kv[1].get("SQ_LDS_IDX_ACTIVE", 0))):
    print("%-44s " % k + " ".join("%13.4g" % d.get(c, 0) for c in cols))
