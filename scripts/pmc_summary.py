"""Summarise a scripts/profile_gram.sh run into profiles/ (committed evidence).

HBM bytes per launch follow MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7:
FETCH_SIZE and WRITE_SIZE are collected in SEPARATE --pmc passes (TCC slots);
both are in KiB; on gfx950 FETCH_SIZE reports 1/2 of the bytes of a wide
(16 B/lane) coalesced streaming read, so it is doubled.  Infinity-Cache hits are
counted (memory-side request counters), so this is L2-miss traffic, an upper
bound on true HBM bytes.
Usage: python scripts/pmc_summary.py gpurun_out/prof_<tag> <tag> [rows dim]
"""
import csv
import json
import os
import shutil
import sys


def rows(path):
    with open(path) as fh:
        return list(csv.DictReader(fh))


def main():
    src, tag = sys.argv[1], sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000
    d = int(sys.argv[4]) if len(sys.argv) > 4 else 768
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
    os.makedirs(dst, exist_ok=True)
    ks = os.path.join(src, "kt", "run_kernel_stats.csv")
    shutil.copy(ks, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    stats = {r["Name"]: r for r in rows(ks)}
    # the dominant kernel (largest total time) is the one the roofline is about
    dom = max(stats, key=lambda k: float(stats[k]["TotalDurationNs"]))
    dshort = dom.split("(")[0].replace("void ", "")
    out = {"tag": tag, "rows_per_gpu": n, "dim": d, "kernel": dshort.split("::")[-1],
           "kernel_full": dshort, "kernels": {},
           "source": f"profiles/{tag}_summary.json (rocprofv3 passes of run '{tag}': "
                     f"kernel trace + separate FETCH_SIZE / WRITE_SIZE --pmc passes)"}
    for name, r in stats.items():
        short = name.split("(")[0].replace("void ", "")
        out["kernels"][short] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                 "pct": float(r["Percentage"])}
    pm = {}
    for pas, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        p = os.path.join(src, pas, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        shutil.copy(p, os.path.join(dst, f"{tag}_pmc_{pas}.csv"))
        for r in rows(p):
            if r["Kernel_Name"].split("(")[0].replace("void ", "") == dshort \
                    and r["Counter_Name"] == ctr:
                pm[ctr] = pm.get(ctr, 0.0) + float(r["Counter_Value"])
                pm[ctr + "_n"] = pm.get(ctr + "_n", 0) + 1
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):  # per launch
        if ctr in pm:
            pm[ctr] /= pm[ctr + "_n"]
    if "FETCH_SIZE" in pm and "WRITE_SIZE" in pm:
        fetch_b = pm["FETCH_SIZE"] * 1024 * 2  # gfx950: FETCH_SIZE = 1/2 of wide reads
        write_b = pm["WRITE_SIZE"] * 1024
        out["dominant_pmc"] = {"FETCH_SIZE_KiB": pm["FETCH_SIZE"], "WRITE_SIZE_KiB": pm["WRITE_SIZE"],
                           "fetch_bytes_corrected": fetch_b, "write_bytes": write_b}
        out["hbm_bytes_per_launch"] = fetch_b + write_b
        # operands read once: bf16 query and corpus copies (the sweep) or the
        # f32 rows (older generators)
        out["algorithmic_bytes_per_launch"] = (2 * n * d * 2 if "sweep" in dshort else 2 * n * d * 4)
    with open(os.path.join(dst, f"{tag}_summary.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    with open(os.path.join(os.path.dirname(dst), "bench_pmc_gram.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
