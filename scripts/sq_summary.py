"""Sum SQ counters per kernel over a scripts/pmc_sq.sh run; prints JSON."""
import csv, glob, json, os, sys
from collections import defaultdict

src = sys.argv[1]
tot = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for p in glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(p) as fh:
        for r in csv.DictReader(fh):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add(r.get("Dispatch_Id", ""))
out = {k: dict(v) for k, v in tot.items()}
with open(os.path.join(src, "sq_summary.json"), "w") as fh:
    json.dump(out, fh, indent=1)
for k, v in out.items():
    if "gram" in k or len(out) < 6:
        print(k, json.dumps({c: round(x) for c, x in sorted(v.items())}))
