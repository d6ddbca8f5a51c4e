"""Sum rocprofv3 --pmc CSV counters per kernel over a directory tree (pmc_nt.sh output)."""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
match = sys.argv[2] if len(sys.argv) > 2 else ""
tot = collections.defaultdict(float)
cnt = collections.defaultdict(int)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if match and match not in r.get("Kernel_Name", ""):
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[r["Counter_Name"]] += 1
print(json.dumps({k: round(v / max(1, cnt[k]), 1) for k, v in sorted(tot.items())}, indent=0))
