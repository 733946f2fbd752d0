"""Write bench.py's PMC references from a legs profile summary
(profiles/<tag>_legs/summary.json, scripts/legs_summary.py): the SW_SYM sweep's
and the energy kernel's HBM-side bytes per launch (FETCH_SIZE x2 + WRITE_SIZE,
separate rocprofv3 passes; Infinity-Cache hits included: an upper bound on DRAM
bytes).  bench.py uses a reference only when its kernel instantiation and shape
match the run.
    python scripts/bench_pmc_refs.py <tag> [rows] [dim]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
d = int(sys.argv[3]) if len(sys.argv) > 3 else 768
summ = json.load(open(os.path.join(ROOT, "profiles", f"{tag}_legs", "summary.json")))
ks = summ["kernels"]
src = f"profiles/{tag}_legs/summary.json (scripts/profile_legs.sh {tag}: kernel trace + separate " \
      f"FETCH_SIZE / WRITE_SIZE --pmc passes, FETCH x2)"


def pick(prefix):
    c = [k for k in ks if k.split("::")[-1].startswith(prefix)]
    return max(c, key=lambda k: ks[k]["total_ms"]) if c else None


for fname, prefix, extra in (("bench_pmc_gram.json", "k_gram_sweep2<0, 2, true", {"rows_per_gpu": n}),
                             ("bench_pmc_energy.json", "k_energy_rows", {"rows": n})):
    k = pick(prefix)
    if not k or "fetch_bytes" not in ks[k] or "write_bytes" not in ks[k]:
        print("no PMC data for", prefix)
        continue
    v = ks[k]
    out = {"tag": tag, "dim": d, "kernel": k.split("::")[-1], "kernel_full": k,
           "avg_ms": v["avg_ms"], "fetch_bytes_per_launch": v["fetch_bytes"],
           "write_bytes_per_launch": v["write_bytes"],
           "hbm_bytes_per_launch": v["fetch_bytes"] + v["write_bytes"], "source": src, **extra}
    json.dump(out, open(os.path.join(ROOT, fname), "w"), indent=1)
    print(fname, json.dumps({kk: out[kk] for kk in ("kernel", "avg_ms", "hbm_bytes_per_launch")}))
