#!/usr/bin/env python3
"""Sum PMC counters per kernel over tools/pmc_pass.sh output: pmc_sum.py DIR NBLOCKS"""
import collections
import csv
import glob
import sys

d, nb = sys.argv[1], int(sys.argv[2])
agg = collections.defaultdict(float)
for f in sorted(glob.glob(d + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "lz4" not in k or "synth" in k:
            continue
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
for (k, c), v in sorted(agg.items()):
    print("%-40s %-28s %14.4g  per-block %12.4g" % (k, c, v, v / nb))
