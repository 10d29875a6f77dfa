"""Summarise a rocprofv3 kernel_stats.csv: per-kernel total ms / calls / avg us."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
div = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0  # e.g. number of encodes
for x in rows[: int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print("%-70s %5s %9.2f ms %9.1f us" % (x["Name"][:70], x["Calls"], float(x["TotalDurationNs"]) / 1e6 / div,
                                         float(x["AverageNs"]) / 1e3))
