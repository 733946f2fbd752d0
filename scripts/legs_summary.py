"""Per-kernel summary of a scripts/profile_legs.sh run -> profiles/<tag>_legs.json.

For every kernel: launches, average duration (kernel trace), HBM-side bytes per
launch from the separate FETCH_SIZE / WRITE_SIZE passes (KiB; FETCH doubled for
gfx950's wide-read under-count, MI355X_MICROARCH.md §HBM; Infinity-Cache hits
included, so an upper bound on DRAM bytes) and the SQ instruction mix / wait
fractions.  `algorithmic` bytes are filled in for the kernels whose per-launch
work DESIGN.md §4 states, so `frac_hbm` = algorithmic / avg / 8 TB/s.
Usage: python scripts/legs_summary.py gpurun_out/legs_<tag> <tag> [json of algorithmic bytes]
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

HBM = 8.0e12


def short(name):
    return name.split("(")[0].replace("void ", "")


def rows(path):
    with open(path) as fh:
        return list(csv.DictReader(fh))


def main():
    src, tag = sys.argv[1], sys.argv[2]
    alg = json.loads(sys.argv[3]) if len(sys.argv) > 3 else {}
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
    ks = glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True)[0]
    os.makedirs(os.path.join(dst, f"{tag}_legs"), exist_ok=True)
    shutil.copy(ks, os.path.join(dst, f"{tag}_legs", "kernel_stats.csv"))
    out = {}
    for r in rows(ks):
        out[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                 "total_ms": float(r["TotalDurationNs"]) / 1e6}
    ctr = defaultdict(lambda: defaultdict(float))
    n = defaultdict(lambda: defaultdict(int))
    for p in glob.glob(os.path.join(src, "*", "**", "*counter_collection.csv"), recursive=True):
        for r in rows(p):
            k = short(r["Kernel_Name"])
            ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k][r["Counter_Name"]] += 1
    for k, v in out.items():
        c = ctr.get(k, {})
        if "FETCH_SIZE" in c:
            v["fetch_bytes"] = c["FETCH_SIZE"] / n[k]["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in c:
            v["write_bytes"] = c["WRITE_SIZE"] / n[k]["WRITE_SIZE"] * 1024
        if "fetch_bytes" in v and "write_bytes" in v and v["avg_ms"] > 0:
            v["pmc_GBps"] = (v["fetch_bytes"] + v["write_bytes"]) / (v["avg_ms"] * 1e-3) / 1e9
        if k in alg and v["avg_ms"] > 0:
            v["algorithmic_bytes"] = alg[k]
            v["alg_GBps"] = alg[k] / (v["avg_ms"] * 1e-3) / 1e9
            v["frac_hbm"] = v["alg_GBps"] * 1e9 / HBM
        W = c.get("SQ_WAVE_CYCLES", 0.0)
        if W > 0:
            v["wait_any"] = c.get("SQ_WAIT_ANY", 0) / W
            v["wait_inst"] = c.get("SQ_WAIT_INST_ANY", 0) / W
            v["active"] = c.get("SQ_ACTIVE_INST_ANY", 0) / W
        for key in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM",
                    "SQ_INSTS_MFMA", "SQ_LDS_BANK_CONFLICT", "SQ_VALU_MFMA_BUSY_CYCLES",
                    "GRBM_GUI_ACTIVE"):
            if key in c:
                v[key] = c[key] / max(1, n[k][key])
        if c.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            g = c["GRBM_GUI_ACTIVE"] / n[k]["GRBM_GUI_ACTIVE"]
            v["mfma_busy"] = (c["SQ_VALU_MFMA_BUSY_CYCLES"] / n[k]["SQ_VALU_MFMA_BUSY_CYCLES"]) / (
                g / 8 * 256 * 4)
    res = {"tag": tag, "source": f"rocprofv3 passes of bench.py (scripts/profile_legs.sh {tag})",
           "kernels": dict(sorted(out.items(), key=lambda kv: -kv[1]["total_ms"]))}
    with open(os.path.join(dst, f"{tag}_legs", "summary.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    for k, v in res["kernels"].items():
        if v["total_ms"] >= 0.5:
            print(f"{k[:60]:60s} {v['calls']:4d} {v['avg_ms']:9.3f} ms "
                  f"pmc {v.get('pmc_GBps', 0):8.1f} GB/s valu {v.get('SQ_INSTS_VALU', 0):.3g}")


if __name__ == "__main__":
    main()
