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


# the energy pass is one kernel since round 4 (k_energy_rows3: the tau select
# inline, X streamed once); a list of prefixes is summed per call
for fname, prefixes, extra in (("bench_pmc_gram.json", ("k_gram_sweep3<0, 2, 2, 1, 0>",), {"rows_per_gpu": n}),
                               ("bench_pmc_energy.json", ("k_energy_rows3",), {"rows": n})):
    kk = [pick(p) for p in prefixes]
    if not all(kk) or any("fetch_bytes" not in ks[k] or "write_bytes" not in ks[k] for k in kk):
        print("no PMC data for", prefixes)
        continue
    fb = sum(ks[k]["fetch_bytes"] for k in kk)
    wb = sum(ks[k]["write_bytes"] for k in kk)
    out = {"tag": tag, "dim": d, "kernel": " + ".join(k.split("::")[-1] for k in kk),
           "kernel_full": " + ".join(kk), "avg_ms": sum(ks[k]["avg_ms"] for k in kk),
           "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
           "hbm_bytes_per_launch": fb + wb, "source": src, **extra}
    k0 = ks[kk[0]]
    if k0.get("mfma_busy") is not None and len(kk) == 1:
        out["mfma_busy"] = k0["mfma_busy"]
        if k0.get("SQ_INSTS_MFMA"):
            out["salu_per_mfma"] = round(k0["SQ_INSTS_SALU"] / k0["SQ_INSTS_MFMA"], 3)
    json.dump(out, open(os.path.join(ROOT, fname), "w"), indent=1)
    print(fname, json.dumps({kk: out[kk] for kk in ("kernel", "avg_ms", "hbm_bytes_per_launch")}))
