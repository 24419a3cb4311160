#!/usr/bin/env python3
"""Per-wave SQ counters of the C4 search kernel from a rocprofv3 --pmc counter_collection.csv."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float)
for r in rows:
    if "c4_search_kernel" in r["Kernel_Name"]:
        agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
per = collections.defaultdict(dict)
for (d, c), v in agg.items():
    per[d][c] = v
for d, c in sorted(per.items()):
    w = c.get("SQ_WAVES", 1) or 1
    print(d, {k: round(v / w) for k, v in c.items()})
