"""Headline benchmark: k-NN graph build vector-pairs/sec (BASELINE.json configs[1] /
configs[3]) on MI355X through the HIP C ABI.

  python bench.py [--gpus N --steps K --warmup W]
  N>1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
           --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

One step = one exact kNN graph build (k=32, squared L2, self excluded) over all
rows: at N=1 the C2 workload (1M x 768 f32), at N GPUs N x 1M rows row-sharded
(C4 at N=8) through the library's C entry mn_knn_sharded_f32 on an RCCL
communicator it creates (mn_rccl_comm_init; the 128-byte id broadcast over the
torch process group): every rank keeps its 1M-row corpus shard resident,
receives all query rows (ncclAllGather over xGMI), computes the exact
per-shard top-k of every query, and the per-shard lists are exchanged
(grouped ncclSend/ncclRecv) and merged on each query's owner rank.  Inputs
are generated on device before timing.
value = N_total^2 vector pairs / max-over-ranks step time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "matternet-rs_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md chip-level table (dense f32 MFMA)
HBM_PEAK_GBS = 8000.0
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md), no sparsity
# scripts/probes/probe_mfma_peak.hip on the box (profiles/r02_mfma_peak.txt):
# the sustained 32x32x16 bf16 rate on random operands under load (DVFS)
MEASURED_BF16_32X32_TFLOPS = 1887.0
MEASURED_BF16_16X16X32_TFLOPS = 2113.0  # same probe, v_mfma_f32_16x16x32_bf16 (the sweep's shape)
FP64_VALU_PEAK_TFLOPS = 78.6


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rows-per-gpu", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="target CPU time of the sampled cpu_baseline leg (0 = skip)")
    ap.add_argument("--no-c5", dest="c5", action="store_false",
                    help="skip the configs[4] leg (1M x 3072 bf16 cosine item graph + SF-GRASS)")
    ap.add_argument("--no-c4-sim", dest="c4_sim", action="store_false",
                    help="skip the configs[3] leg at N=1 (8M x 768 as 8 simulated ranks)")
    ap.add_argument("--c5-rows", type=int, default=1_048_576)
    ap.add_argument("--c5-dim", type=int, default=3072)
    ap.add_argument("--c5-parity-rows", type=int, default=3,
                    help="rows of the C5 graph checked bit-exact against the oracle (0 = off)")
    ap.add_argument("--no-c3", dest="c3", action="store_false",
                    help="skip the C3 legs (Laplacian assembly, energy pass, sorted index)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "bench_pmc_gram.json"),
                    help="PMC-derived HBM bytes per launch of the Gram kernel (optional)")
    ap.add_argument("--time-budget-s", type=float, default=420.0,
                    help="N>1: cap warmup+steps so the whole run fits this budget (the cap is "
                         "reported in the line)")
    ap.add_argument("--query-chunk", type=int, default=2_097_152,
                    help="N>1: queries per per-shard kNN call (bounds candidate buffers)")
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    import surfface_hip as S
    from surfface_hip import _lib
    L = _lib.lib()

    n_loc, d, k = a.rows_per_gpu, a.dim, a.k
    n_tot = n_loc * world
    X = torch.empty((n_loc, d), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    _lib.check(L.mn_fill_uniform_f32(X.data_ptr(), n_loc, d, a.seed, rank * n_loc,
                                     stream.cuda_stream))
    comm = None
    if world > 1:
        from surfface_hip.dist import RcclComm, knn_sharded_capi
        uid = [RcclComm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = RcclComm(uid[0], world, rank)
    torch.cuda.synchronize()

    gram_ms = []

    last = {}

    def step():
        if world == 1:
            r = S.knn_l2sq(X, k, timing=True)
            # the dominant kernel: the bf16x1 sweep (phase 2), else the Gram
            gram_ms.append(r.stats.get("ms_sweep") or r.stats["ms_gram"])
            last["stats"] = r.stats
            return r.idx, r.dist, r.stats
        # the C entry (csrc/shard.hip): all-gather of the shards, then the
        # symmetric form (this rank's share of the node-wide SW_SYM tile table,
        # partial re-rank, exchange, merge + certify; ms_sweep = the share), or
        # the per-shard form (query chunks; the last chunk's stats x chunks)
        idx, dd = knn_sharded_capi(X, k, comm, query_chunk=a.query_chunk, timing=True,
                                   stream=stream)
        st = S.knn.last_stats()
        if st.get("sweep_slices") == -1:
            gram_ms.append(st.get("ms_sweep") or st["ms_gram"])
        else:
            chunks = (n_tot + a.query_chunk - 1) // a.query_chunk
            gram_ms.append((st.get("ms_sweep") or st["ms_gram"]) * chunks)
        last["stats"] = st
        return idx, dd, st

    steps_req, warm_req = a.steps, a.warmup
    t_w = time.perf_counter()
    for i in range(a.warmup):
        step()
        if world > 1 and i == 0:
            # time budget (N>1: every rank does N x the C2 work per step): the
            # first warmup step measured, the timed steps capped to fit (the
            # warmup runs exactly as requested)
            torch.cuda.synchronize()
            tw = torch.tensor([time.perf_counter() - t_w], dtype=torch.float64, device=dev)
            dist.all_reduce(tw, op=dist.ReduceOp.MAX)
            per = float(tw.item())
            left = max(a.time_budget_s - per * a.warmup, 0.0)
            a.steps = max(1, min(a.steps, int(left / max(per, 1e-3))))
    if world > 1 and warm_req == 0:
        # no warmup step to measure: budget on the estimate of N x ~2 s per step
        a.steps = max(1, min(a.steps, int(a.time_budget_s / (2.0 * world))))
    gram_ms.clear()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = None
    for _ in range(a.steps):
        out = step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ms_step = el * 1e3 / a.steps
    pairs = float(n_tot) * float(n_tot)
    value = pairs * a.steps / el

    # roofline of the dominant kernel: algorithmic flops per launch =
    # 2 * nq * nc * d over the rows that launch sweeps; its
    # duration from HIP events recorded on the launch stream inside the library
    st0 = out[2]
    nq = n_tot
    gms = float(np.mean(gram_ms)) if gram_ms else float("nan")
    algo = st0.get("algo")
    if algo == 3:
        # two-phase single-bf16 generator: phase 2 (k_gram_sweep2) decides the
        # rows outside the phase-1 sample (query-major sweep), or, for the self
        # kNN (sweep_slices == -1: SW_SYM), EVERY pair (i, j) of the n x n
        # Gram while executing each unordered pair once (upper-triangle tiles)
        m0 = int(st0.get("sample_rows") or 0)
        sym = st0.get("sweep_slices") == -1
        nc_sw = n_loc if sym else n_loc - m0
        kname = "k_gram_sweep2"
        # the exact instantiation (rocprofv3 name) the PMC reference must match
        kfull = "k_gram_sweep2<0, 0, true>"
        if sym:  # fp16 operands (x 2^e): the release library's only SW_SYM form
            kname = "k_gram_sweep3<SW_SYM>"
            # (round 6: gram_sweep3.hpp, DMA two k-steps ahead)
            kfull = "k_gram_sweep3<0, 2, 2, 1, 0>"
        flops_launch = 2.0 * nq * nc_sw * d
        # executed: the upper-triangle 256 x 256 tiles of the n_tot rows, a
        # rank's 1/world share of them (the sharded symmetric form)
        nbk = (n_tot + 255) // 256
        flops_exec = 2.0 * 256 * 256 * d * nbk * (nbk + 1) / 2 / world if sym else flops_launch
        achieved = flops_launch / (gms * 1e-3) / 1e12
        ms_all = float(st0["ms_gram"])
        roof = {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 3),
                "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / BF16_MFMA_PEAK_TFLOPS, 4),
                "traffic": None, "ms_per_launch": round(gms, 3), "flop_per_launch": flops_launch,
                "flop_basis": ("SURVEY 8(d): 2 nq nc d over the pairs the launch decides"
                               + ("; SW_SYM decides all n^2 pairs and executes the upper-"
                                  "triangle 256 x 256 tiles (each unordered pair once)"
                                  if sym else "")),
                # top-level scalars (round 6): the executed-flop fraction (each
                # unordered pair's tile once) and the PMC MFMA-busy fraction of
                # the same kernel instantiation (filled from the legs profile)
                "frac_executed": round(flops_exec / (gms * 1e-3) / 1e12 / BF16_MFMA_PEAK_TFLOPS, 4),
                "mfma_busy": None,
                "executed": {"flop_per_launch": flops_exec,
                             "tflops": round(flops_exec / (gms * 1e-3) / 1e12, 3),
                             "frac": round(flops_exec / (gms * 1e-3) / 1e12
                                           / BF16_MFMA_PEAK_TFLOPS, 4)},
                "peak_basis": ("dense fp16/bf16 MFMA 2500 TFLOP/s (one v_mfma_f32_16x16x32_f16 "
                               "product per f32 product: x 2^e ~ fp16, certified by the residual-"
                               "norm bound)" if sym else
                               "dense bf16 MFMA 2500 TFLOP/s (one v_mfma_f32_16x16x32_bf16 product "
                               "per f32 product: x ~ bf16(x), certified by the residual-norm bound)"),
                "measured_mfma_ceiling": {"tflops": MEASURED_BF16_16X16X32_TFLOPS,
                                          "frac": round(achieved / MEASURED_BF16_16X16X32_TFLOPS, 4),
                                          "basis": "scripts/probes/probe_mfma_peak.hip "
                                                   "(profiles/r02_mfma_peak.txt): back-to-back "
                                                   "v_mfma_f32_16x16x32_bf16 on random register "
                                                   "operands, every CU (DVFS-limited clock)"},
                "whole_gram": {"ms": round(ms_all, 3), "sample_ms": round(st0["ms_sample"], 3),
                               "sample_rows": m0,
                               "effective_tflops": round(2.0 * nq * n_loc * d / (ms_all * 1e-3) / 1e12, 1),
                               "vs_f32_mfma_peak": round(2.0 * nq * n_loc * d / (ms_all * 1e-3) / 1e12
                                                         / FP32_MFMA_PEAK_TFLOPS, 3)}}
    elif algo == 2:
        kname = kfull = "k_gram_bf16<GM_L2>"
        flops_launch = 2.0 * nq * n_loc * d
        achieved = flops_launch / (gms * 1e-3) / 1e12
        peak = BF16_MFMA_PEAK_TFLOPS / 3.0
        roof = {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 3),
                "peak": round(peak, 1), "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                "traffic": None, "ms_per_launch": round(gms, 3), "flop_per_launch": flops_launch,
                "peak_basis": ("dense bf16 MFMA 2500 TFLOP/s / 3 bf16 products per f32 product "
                               "(x = hi + lo; hi.hi + hi.lo + lo.hi)")}
    else:
        kname = kfull = "k_gram_topk"
        flops_launch = 2.0 * nq * n_loc * d
        achieved = flops_launch / (gms * 1e-3) / 1e12
        roof = {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 3),
                "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": None,
                "ms_per_launch": round(gms, 3), "flop_per_launch": flops_launch}
    if os.path.exists(a.pmc_json) and world == 1:
        # HBM bytes per launch from separate FETCH_SIZE / WRITE_SIZE rocprofv3
        # passes of an earlier run (FETCH x2 per the gfx950 note); labelled
        # with the run it came from
        try:
            pm = json.load(open(a.pmc_json))
            if (pm.get("rows_per_gpu") == n_loc and pm.get("dim") == d
                    and pm.get("kernel", "") == kfull):
                roof["traffic"] = pm.get("hbm_bytes_per_launch")
                roof["traffic_source"] = pm.get("source", os.path.relpath(a.pmc_json, ROOT))
                if "mfma_busy" in roof and pm.get("mfma_busy") is not None:
                    roof["mfma_busy"] = round(pm["mfma_busy"], 4)
                    roof["salu_per_mfma"] = pm.get("salu_per_mfma")
        except (OSError, ValueError):
            pass

    # C3 legs (configs[2]): Laplacian assembly + energymaps/taumode pass + index,
    # on this rank's rows (timed individually after the headline step)
    # (N > 1: the rank's rows carry global neighbour ids of the N x 1M graph,
    # which the single-graph C3 legs do not take — they run at N = 1 only)
    c3 = None
    if a.c3 and world == 1:
        c3 = c3_legs(S, X, out[0], out[1], k)

    c5 = None
    if a.c5 and world == 1:
        c5 = c5_leg(S, _lib, L, a, dev, stream)

    c4 = None
    if a.c4_sim and world == 1:
        c4 = c4_sim_leg(S, _lib, L, a, dev, stream)

    cpu = None
    parity = None
    energy_cpu = None
    if rank == 0 and world == 1 and a.cpu_seconds > 0:
        cpu, parity = cpu_baseline(X, out[0], out[1], k, a.cpu_seconds)
        if c3 is not None:
            energy_cpu = energy_cpu_baseline(X, c3.pop("_Lf"), a.cpu_seconds)
    elif c3 is not None:
        c3.pop("_Lf", None)

    if rank == 0:
        st = out[2]
        gen = {3: "bf16x1 two-phase MFMA (sample thresholds + fixed-threshold sweep)",
               2: "bf16x3 split MFMA", 1: "f32 MFMA"}.get(st.get("algo"), "f32 MFMA")
        energy = None
        if c3 is not None:
            er = c3["energy_rows"]
            energy = {"rows_per_sec": c3["energy_rows_per_sec"],
                      "workload": "C3: 1M items x 768 features vs the 768 x 768 feature "
                                  "Laplacian (taumode, Median tau)",
                      "roofline": er["roofline"], "cpu_baseline": energy_cpu}
        line = {
            "metric": "vector-pairs/sec for k-NN graph build (N=1M, d=768) + Laplacian energy rows/sec",
            "value": value, "unit": "pairs/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "candidate_generator": gen,
            "data": "synthetic U[-1,1) f32 (splitmix64 counter stream, seed 42), generated on device",
            "config": {"workload": ("C2: 1M x 768 f32 exact kNN k=32" if world == 1 else
                                    f"C4-style: {n_tot} x {d} f32 exact kNN k={k}, row-sharded"),
                       "n_rows": n_tot, "dim": d, "k": k, "rows_per_gpu": n_loc,
                       "metric_space": "squared L2 (reference sequential f32 fold)",
                       "parallelism": ("single GPU (no collective)" if world == 1 else
                                       f"row-shard x{world} (mn_knn_sharded_f32): RCCL "
                                       "all-gather of the shards and thresholds, each rank's "
                                       "share of the node-wide symmetric tile table, grouped "
                                       "send/recv of the partial lists, merge + certify")},
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity_sample": parity,
            "energy_rows_per_sec": (c3 or {}).get("energy_rows_per_sec"),
            "energy": energy,
            "c3_legs": c3,
            "c5_leg": c5,
            "c4_sim_leg": c4,
            "knn_stats": {kk: (round(v, 3) if isinstance(v, float) else v)
                          for kk, v in st.items()},
        }
        if world > 1:
            line["time_budget"] = {"budget_s": a.time_budget_s, "steps_requested": steps_req,
                                   "warmup_requested": warm_req, "steps_timed": a.steps,
                                   "warmup_run": a.warmup,
                                   "query_chunk": a.query_chunk}
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def _timed(fn, reps=3):
    """median wall ms of fn() (device-synchronised), after one warm call."""
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts)), r


def c3_legs(S, X, idx, dist, k):
    """BASELINE.json configs[2]: on the C2 kNN graph of X (N x F):
    item-graph Laplacian (legacy UNION, rational weights), the F x F feature
    graph (rectified-cosine kNN of the columns, topk=4, eps=1, sigma=1, p=2;
    energymaps.rs:463-471 bootstrap), its Laplacian, the taumode energy pass of
    all N items against it (Median tau), normalise_lambdas and the sorted index.
    Algorithmic bytes -> GB/s per leg."""
    n, f = X.shape
    out = {}
    ms, (Lit, _) = _timed(lambda: S.build_laplacian_from_knn(
        idx, dist, weight_kernel="rational", symmetrise="union", eps=float("inf"), sigma=1.0,
        p=2.0))
    byt = n * k * 8 + Lit.nnz * 12 + (n + 1) * 8
    lst = S.laplacian.last_stats()
    out["item_laplacian"] = {"ms": round(ms, 3), "nnz": Lit.nnz, "GB_per_s": round(byt / ms / 1e6, 1),
                             "rows_block_sorted": lst["big_rows"], "hub_rows": lst["hub_rows"]}
    # the Stage C form of the same assembly (surfface-core/src/laplacian.rs:312-394
    # build_laplacian_flat: MAX symmetrisation, f32 values, normalised), timed
    # separately as SURVEY §8(d) asks; bytes as above with f32 values
    ms, (Lmx, _) = _timed(lambda: S.build_laplacian_from_knn(
        idx, dist, weight_kernel="rational", symmetrise="max", normalize=True, eps=float("inf"),
        sigma=1.0, p=2.0))
    byt = n * k * 8 + Lmx.nnz * 8 + (n + 1) * 8
    out["item_laplacian_max_sym"] = {"ms": round(ms, 3), "nnz": Lmx.nnz,
                                     "GB_per_s": round(byt / ms / 1e6, 1)}
    del Lmx
    ms, (fi, fd, fw, fst) = _timed(lambda: S.knn_cos_columns(X, 4, eps=1.0, sigma=1.0, p=2.0), 1)
    out["feature_knn_cos"] = {"ms": round(ms, 3), "uncertified": fst["n_uncertified"],
                              "gram_tflops": round(2.0 * f * f * n / 2 / (fst["ms_gram"] * 1e9), 2)
                              if fst["ms_gram"] else None}
    ms, (Lf, _) = _timed(lambda: S.build_laplacian_from_knn(fi, fw, weight_kernel="given",
                                                           symmetrise="union"))
    out["feature_laplacian"] = {"ms": round(ms, 3), "nnz": Lf.nnz}
    ms, (E, G, lam) = _timed(lambda: S.energy_rows(X, Lf, timing=True))
    ebytes = n * f * 4 + Lf.nnz * 12 + (f + 1) * 8 + n * 3 * 8
    est = S.energy.last_stats()
    ent = est["entries"]
    # the roofline takes the rows kernel's own duration (HIP events around
    # k_energy_rows3 on its launch stream inside the library, last call); the
    # call's wall time (host list build + copies + the symmetry check) beside it
    kms = float(est["ms_rows"]) if est.get("ms_rows") else ms
    gbs = ebytes / kms / 1e6
    # bound: HBM (X streamed once, L resident); the f64 work per
    # row is reported beside it (k_energy_rows3, one pass over X: the tau
    # select inline, the list-A identity at 5 f64 ops per entry and row)
    f64_ops = 5.0 * ent * n
    out["energy_rows"] = {"ms": round(ms, 3), "GB_per_s": round(ebytes / ms / 1e6, 1),
                          "entries_per_row": ent, "ms_kernel": round(kms, 3),
                          "roofline": {"bound": "hbm", "kernel": "k_energy_rows3",
                                       "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                                       "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                                       "traffic": None, "bytes_per_launch": ebytes,
                                       "ms_per_launch": round(kms, 3),
                                       "ms_call": round(ms, 3),
                                       "f64_tflops": round(f64_ops / (kms * 1e-3) / 1e12, 2),
                                       "f64_frac_of_78.6": round(f64_ops / (kms * 1e-3) / 1e12
                                                                 / FP64_VALU_PEAK_TFLOPS, 4)}}
    # HBM bytes per launch of the energy kernel from the latest legs profile
    # (bench_pmc_energy.json: separate FETCH_SIZE / WRITE_SIZE passes, FETCH x2),
    # used when the kernel and shape match
    try:
        pe = json.load(open(os.path.join(ROOT, "bench_pmc_energy.json")))
        if pe.get("rows") == n and pe.get("dim") == f and "k_energy_rows3" in pe.get("kernel", ""):
            out["energy_rows"]["roofline"]["traffic"] = pe.get("hbm_bytes_per_launch")
            out["energy_rows"]["roofline"]["traffic_kernel"] = pe.get("kernel")
            out["energy_rows"]["roofline"]["traffic_source"] = pe.get("source")
    except (OSError, ValueError):
        pass
    out["energy_rows_per_sec"] = n / (ms * 1e-3)
    # the energymaps.rs pass BASELINE configs[2] names (node_energy_and_dispersion,
    # src_legacy/energymaps.rs:923-1045: E = x.Lx / x.x, G over the upper
    # entries, lambda = E) on the same rows and Laplacian, same bytes
    from surfface_hip import _lib as _L
    ms_em, _ = _timed(lambda: S.energy_rows(X, Lf, g_mode=_L.MN_G_ENERGYMAPS))
    out["energymaps_pass"] = {"ms": round(ms_em, 3), "GB_per_s": round(ebytes / ms_em / 1e6, 1),
                              "rows_per_s": round(n / (ms_em * 1e-3), 1),
                              "frac_of_hbm": round(ebytes / ms_em / 1e6 / HBM_PEAK_GBS, 4)}
    out["_Lf"] = Lf
    # energymaps diffusion pre-pass (eta 0.1, 4 steps; energymaps.rs:518-546) on
    # the same rows: f32 in, f64 out; bytes = N F (4 + 8)
    Xd = torch.empty((n, f), dtype=torch.float64, device=X.device)
    ms, _ = _timed(lambda: S.diffuse_rows(X, Lf, 0.1, 4, out=Xd))
    out["diffusion_4_steps"] = {"ms": round(ms, 3), "GB_per_s": round(n * f * 12 / ms / 1e6, 1)}
    del Xd
    # item-graph orientation: the F feature signals against
    # the n x n item Laplacian; bytes = one x_j row gather per stored entry
    ms, _ = _timed(lambda: S.signal_energy_and_dispersion(X, Lit))
    # algorithmic bytes: X streamed once plus the Laplacian's CSR (col i32 + f64
    # value per entry, row pointers); the kernel gathers one x_j row per upper
    # entry instead (random 3 KB rows: bound by the gather, not the stream),
    # reported beside it
    alg = n * f * 4 + Lit.nnz * 12 + (n + 1) * 8
    gat = (Lit.nnz // 2 + n) * f * 4
    out["item_graph_signals"] = {"ms": round(ms, 3), "GB_per_s": round(alg / ms / 1e6, 1),
                                 "bytes_basis": "X once + CSR (algorithmic)",
                                 "frac_of_hbm": round(alg / ms / 1e6 / HBM_PEAK_GBS, 4),
                                 "gathered_GB_per_s": round(gat / ms / 1e6, 1),
                                 "gathered_basis": "one 4F-byte x_j row per upper entry + x_i"}
    # Stage C Bhattacharyya feature kNN (§8(f) rank 3) on 2048 centroid rows of X
    cm = X[:2048].contiguous()
    cv = (X[2048:4096].abs() * 0.3 + 0.05).contiguous()
    ms, _ = _timed(lambda: S.compute_bhattacharyya_weights(cm, cv, S.LaplacianConfig(k_neighbors=15)))
    out["stage_c_bc_knn"] = {"ms": round(ms, 3), "centroids": 2048, "features": f,
                             "pair_terms_per_s": round(f * (f + 1) / 2 * 2048 / (ms * 1e-3), 1)}
    lam_n = lam.clone()
    ms, _ = _timed(lambda: S.normalise_lambdas(lam_n.copy_(lam)))
    out["normalise_ms"] = round(ms, 3)
    ms, sl = _timed(lambda: S.SortedLambdas().build_from(lam_n))
    out["sorted_index"] = {"ms": round(ms, 3), "std_dev": sl.std_dev,
                           "GB_per_s": round(n * 16 / ms / 1e6, 1)}
    # lambda-aware query path (§8(f) rank 2, core.rs:1156-1193): 64 queries
    # (rows of X) against all N items with the normalised lambdas, k=32,
    # alpha=0.7; work = 2 f64 flops per (query, item, feature) for the dots
    # plus the item norm chains; bytes = X read once per 32-query group
    nq = 64
    qrows = torch.arange(0, n, max(n // nq, 1), device=X.device)[:nq]
    Qs = X[qrows].double().contiguous()
    lq = lam_n[qrows].clone().clamp_min(1e-6)
    ms, _ = _timed(lambda: S.search_lambda_aware(X, lam_n, Qs, lq, 32, 0.7))
    out["lambda_aware_search"] = {
        "ms": round(ms, 3), "queries": nq, "k": 32, "queries_per_s": round(nq / (ms * 1e-3), 1),
        "f64_gflops": round(2.0 * (nq + 4) * n * f / (ms * 1e6), 1),
        # roofline: the reference's folds forbid FMA, so the ceiling is one f64
        # mul or add per lane per cycle = FP64 vector peak 78.6 TFLOP/s / 2
        "f64_valu_frac": round(2.0 * (nq + 4) * n * f / (ms * 1e-3) / 39.3e12, 3),
        "GB_per_s": round(n * f * 4 * ((nq + 31) // 32) / ms / 1e6, 1)}
    ms, _ = _timed(lambda: S.search_lambda_aware_hybrid(X, lam_n, Qs, lq, 32, 0.7))
    out["lambda_aware_search"]["hybrid_ms"] = round(ms, 3)
    return out


def c4_sim_leg(S, _lib, L, a, dev, stream, R=8):
    """BASELINE.json configs[3] on ONE GPU: 8M x 768 (8 ranks x the per-GPU
    rows) through mn_knn_sharded_sim_f32 — mn_knn_sharded_f32's driver over
    the loopback transport: every rank's stages of the symmetric sharded
    build run in turn on this device, the collectives as device copies, so a
    rank's share of the real 8-GPU build = its stage A + B + C time here,
    plus the RCCL all-gathers (X: 7/8 of 24.6 GB a rank over xGMI; tau0 /
    norms 64 MB) and the list exchange (2 GB), which are not in the shares.
    One row per shard checked bit-exact against the oracle over all rows."""
    from oracle import oracle as O
    from surfface_hip.dist import knn_sharded_sim
    n_loc, d, k = a.rows_per_gpu, a.dim, a.k
    n_tot = R * n_loc
    Xall = torch.empty((n_tot, d), dtype=torch.float32, device=dev)
    for r0 in range(0, n_tot, n_loc):  # each rank's shard: the same counter stream
        _lib.check(L.mn_fill_uniform_f32(Xall[r0:r0 + n_loc].data_ptr(), n_loc, d, a.seed, r0,
                                         stream.cuda_stream))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    idx, dist, ms, st = knn_sharded_sim(Xall, k, R, timing=True, stream=stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    share = ms.sum(axis=1)
    mx = float(share.max()) / 1e3
    out = {"workload": f"C4: {n_tot} x {d} f32 exact kNN k={k}, {R} ranks simulated on one GPU "
                       "(mn_knn_sharded_sim_f32)",
           "rank_share_s": [round(float(x) / 1e3, 3) for x in share],
           "max_share_s": round(mx, 3),
           "stage_ms_max": {"A_thresholds": round(float(ms[:, 0].max()), 1),
                            "B_sweep_share": round(float(ms[:, 1].max()), 1),
                            "C_merge_certify": round(float(ms[:, 2].max()), 1)},
           "pairs_per_s_at_max_share": n_tot * float(n_tot) / mx,
           "excluded": "RCCL all-gathers (X 21.5 GB received a rank, thresholds) and the "
                       "partial-list exchange (2 GB): device copies of the loopback transport "
                       "here, outside the stage shares",
           "n_uncertified": st["n_uncertified"], "n_candidates": st["n_candidates"],
           "sim_wall_s": round(wall, 2)}
    if a.c5_parity_rows > 0:
        rng = np.random.default_rng(11)
        q = np.array([r * n_loc + int(rng.integers(n_loc)) for r in range(R)], np.int64)
        Ch = Xall.cpu().numpy()
        ri, rd = O.knn_l2sq_qc(Ch[q], q, Ch, 0, k, nthreads=cpu_threads())
        gi = idx[torch.from_numpy(q).to(dev)].cpu().numpy()
        gd = dist[torch.from_numpy(q).to(dev)].cpu().numpy()
        out["parity_sample"] = {"rows": q.tolist(), "bit_exact": bool(
            np.array_equal(gi, ri) and np.array_equal(gd.view(np.uint32), rd.view(np.uint32)))}
        del Ch
    del Xall, idx, dist
    torch.cuda.empty_cache()
    return out


def c5_leg(S, _lib, L, a, dev, stream):
    """BASELINE.json configs[4]: 1M x 3072 bf16 rectified-cosine item graph
    (topk=32, eps=1, sigma=1, p=2; legacy _build_adjacency semantics) on the
    bf16 MFMA path, then SF-GRASS (sparsification.rs, ratio 0.5) on its rows.
    One timed run (the Gram alone is ~10 s), parity rows vs the oracle."""
    n, d, k = a.c5_rows, a.c5_dim, a.k
    Xb = torch.empty((n, d), dtype=torch.bfloat16, device=dev)
    ch = 1 << 17
    tmp = torch.empty((min(ch, n), d), dtype=torch.float32, device=dev)
    for r0 in range(0, n, ch):
        m = min(ch, n - r0)
        _lib.check(L.mn_fill_uniform_f32(tmp.data_ptr(), m, d, a.seed + 5, r0, stream.cuda_stream))
        Xb[r0:r0 + m].copy_(tmp[:m])  # round-to-nearest-even
    del tmp
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    idx, dist, w, st = S.knn_cos_bf16(Xb, k, eps=1.0, sigma=1.0, p=2.0, timing=True)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    ms_sp, (sidx, sw, applied) = _timed(lambda: S.sparsify_rows(idx, w, 0.5))
    kept = int((sidx >= 0).sum().item())
    m0 = st.get("sample_rows", 0)
    exec_fl = None
    if m0 > 0 and st.get("sweep_slices") == -1:
        # SW_COS_SYM: the sweep decides all n^2 pairs, executing the upper-
        # triangle 256 x 256 tiles (each unordered pair once)
        kname, kms = "k_gram_sweep3<SW_COS_SYM, tile-major>", st["ms_sweep"]
        flops = 2.0 * n * n * d
        nbk = (n + 255) // 256
        exec_fl = 2.0 * 256 * 256 * ((d + 31) // 32 * 32) * nbk * (nbk + 1) / 2
    elif m0 > 0:  # two-phase: the dominant kernel is the sweep over rows [m0, n)
        kname, kms = "k_gram_sweep2<SW_COS, tile-major>", st["ms_sweep"]
        flops = 2.0 * n * (n - m0) * d
    else:
        kname, kms = "k_gram_bf16<GM_COS>", st["ms_gram"]
        flops = 2.0 * n * n * d
    ach = flops / (kms * 1e-3) / 1e12
    out = {"workload": f"C5: {n} x {d} bf16 rectified-cosine item graph k={k} + SF-GRASS 0.5",
           "ms_total": round(ms, 1), "pairs_per_s": n * n / (ms * 1e-3),
           "roofline": {"bound": "mfma", "kernel": kname, "achieved": round(ach, 1),
                        "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(ach / BF16_MFMA_PEAK_TFLOPS, 4), "flop_per_launch": flops,
                        "ms_per_launch": round(kms, 1),
                        # (the decided-pairs basis counts each executed pair
                        # twice for SW_COS_SYM: against the measured MFMA
                        # ceiling only the executed flops are a utilisation)
                        "executed_frac_of_measured_ceiling": round(
                            (exec_fl if exec_fl else flops) / (kms * 1e-3) / 1e12
                            / MEASURED_BF16_16X16X32_TFLOPS, 4),
                        **({"frac_executed": round(exec_fl / (kms * 1e-3) / 1e12
                                                   / BF16_MFMA_PEAK_TFLOPS, 4)} if exec_fl else {}),
                        **({"executed": {"flop_per_launch": exec_fl,
                                         "tflops": round(exec_fl / (kms * 1e-3) / 1e12, 1),
                                         "frac": round(exec_fl / (kms * 1e-3) / 1e12
                                                       / BF16_MFMA_PEAK_TFLOPS, 4)}}
                           if exec_fl else {})},
           "gram_all_phases": {"ms": round(st["ms_gram"], 1),
                               "tflops_equiv": round(2.0 * n * n * d / (st["ms_gram"] * 1e-3) / 1e12, 1),
                               "ms_sample": round(st.get("ms_sample", 0.0), 1),
                               "sample_rows": m0},
           "knn_stats": {kk: (round(v, 3) if isinstance(v, float) else v) for kk, v in st.items()},
           "sfgrass": {"ms": round(ms_sp, 3), "applied": applied, "edges_kept": kept,
                       "edges_in": int((idx >= 0).sum().item())}}
    if a.c5_parity_rows > 0:
        import oracle.oracle as O
        rows = np.unique(np.linspace(0, n - 1, a.c5_parity_rows).astype(np.int64))
        bits = Xb.view(torch.int16).cpu().numpy().view(np.uint16)
        t1 = time.perf_counter()
        ri, rd, rw = O.knn_cos_bf16_rows(bits, k, rows, nthreads=16)
        oms = (time.perf_counter() - t1) * 1e3
        gi = idx[torch.from_numpy(rows).to(dev)].cpu().numpy()
        gd = dist[torch.from_numpy(rows).to(dev)].cpu().numpy()
        gw = w[torch.from_numpy(rows).to(dev)].cpu().numpy()
        same = (np.array_equal(gi, ri) and np.array_equal(gd.view(np.uint64), rd.view(np.uint64))
                and np.array_equal(gw.view(np.uint64), rw.view(np.uint64)))
        out["parity_sample"] = {"rows": rows.tolist(), "bit_exact": bool(same),
                                "oracle_ms": round(oms, 1), "oracle_threads": 16}
        del bits
    del Xb, idx, dist, w, sidx, sw
    torch.cuda.empty_cache()
    return out


def host_info():
    """Core count and model of the host the CPU baselines run on."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        import subprocess
        lines = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for ln in lines.splitlines():
            if ln.startswith("Model name:"):
                info["cpu_model"] = ln.split(":", 1)[1].strip()
            if ln.startswith("Socket(s):") or ln.startswith("Core(s) per socket:") \
                    or ln.startswith("Thread(s) per core:"):
                info[ln.split(":")[0].strip().lower().replace("(s)", "s").replace(" ", "_")] = \
                    ln.split(":", 1)[1].strip()
    except Exception:  # noqa: BLE001 — informational only
        pass
    return info


def cpu_threads():
    """All cores this run may use: OMP_NUM_THREADS when the environment sets
    it (the GPU box sets the job's CPU share), else the affinity mask."""
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if env > 0:
        return env
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_baseline(X, idx, dd, k, target_s):
    """The oracle (C restatement, OpenMP on all allowed host cores) timed on
    bounded samples of query rows against the full corpus:
    efficient = bounded-heap top-k (the restated-efficient form), faithful =
    collect all n-1 distances and sort them (mst.rs:330-360 as written).  The
    sampled rows double as a bit-exact parity check of the GPU result."""
    from oracle import oracle as O
    threads = cpu_threads()
    Xh = X.cpu().numpy()
    n = Xh.shape[0]
    rng = np.random.default_rng(1)
    cal = np.sort(rng.choice(n, threads, replace=False))  # warms pages + threads
    i0, d0 = O.knn_l2sq_rows(Xh, k, cal, nthreads=threads)
    perm = rng.permutation(n)
    batch = threads * 4  # schedule(dynamic, 1): every thread busy
    done, el = 0, 0.0
    ri_l = []
    while el < target_s and done + batch <= min(n, 65536):
        rows_b = np.sort(perm[done:done + batch])
        t0 = time.perf_counter()
        a_i, a_d = O.knn_l2sq_rows(Xh, k, rows_b, nthreads=threads)
        el += time.perf_counter() - t0
        ri_l.append((rows_b, a_i, a_d))
        done += batch
    rows = np.concatenate([r for r, _, _ in ri_l])
    ri = np.concatenate([x for _, x, _ in ri_l])
    rd = np.concatenate([x for _, _, x in ri_l])
    m = len(rows)
    gi = idx.cpu().numpy()[rows]
    gd = dd.cpu().numpy()[rows]
    ok = int(np.sum(np.all(gi == ri, axis=1) & np.all(gd.view(np.uint32) == rd.view(np.uint32),
                                                       axis=1)))
    # faithful: the first rows (full sort per row), a smaller bounded sample
    fr = max(threads, int(m * 0.5) // threads * threads)
    t0 = time.perf_counter()
    f_i, f_d = O.knn_l2sq(Xh, k, q_begin=0, q_end=fr, mode=0, nthreads=threads)
    fel = time.perf_counter() - t0
    f_ok = bool(np.array_equal(f_i, idx[:fr].cpu().numpy()))
    cpu = {"value": m * (n - 1) / el, "unit": "pairs/s", "cores": threads, "kind": "port",
           "sample": f"{m} random query rows x {n} corpus rows, d={Xh.shape[1]}, k={k} "
                     f"(oracle/or_knn_l2sq_rows_f32, bounded heap, OpenMP {threads} threads), "
                     f"{el:.1f}s",
           "form": "restated-efficient",
           "faithful": {"value": fr * (n - 1) / fel, "unit": "pairs/s", "cores": threads,
                        "sample": f"rows 0..{fr - 1} x {n} (mode 0: all n-1 distances collected "
                                  f"and sorted per row), {fel:.1f}s",
                        "rows_bit_exact": f_ok},
           "host": host_info(),
           "cores_note": ("the box allots this job OMP_NUM_THREADS=16 of the host's hardware "
                          "threads (one GPU's share; the affinity mask lists the whole machine, "
                          "which the other GPUs' jobs share), so the baseline runs 16 threads; "
                          "full_host_upper_bound scales it linearly to the affinity count "
                          "(an extrapolation, not a measurement)")}
    aff = cpu["host"].get("affinity_cpus")
    if aff and aff > threads:
        cpu["full_host_upper_bound"] = {"value": cpu["value"] * aff / threads, "cores": aff,
                                        "basis": "linear scaling of the measured value"}
    parity = {"rows_checked": m, "rows_bit_exact": ok, "plus_calibration_rows": threads,
              "calibration_bit_exact": bool(np.array_equal(i0, idx.cpu().numpy()[cal]))}
    return cpu, parity


def energy_cpu_baseline(X, Lf, target_s):
    """K3 CPU baseline: the taumode energy rows of the first
    65,536 items against the same feature Laplacian, restated-efficient (CSR
    iteration) and faithful (compute_item_dispersion's F^2 CsMat::get pairs,
    taumode.rs:366-408) on all allowed host cores; rows/s."""
    from oracle import oracle as O
    threads = cpu_threads()
    ip, ix, iv = (Lf.indptr.cpu().numpy(), Lf.indices.cpu().numpy(), Lf.values.cpu().numpy())
    Xh = X[:65536].cpu().numpy()
    t0 = time.perf_counter()
    O.energy_rows(Xh, ip, ix, iv, O.G_TAUMODE, O.TAU_MEDIAN, nthreads=threads)
    el = time.perf_counter() - t0
    # faithful: F^2 binary-search lookups per row, a bounded sample
    nf = threads * 8
    t0 = time.perf_counter()
    O.energy_rows_faithful(Xh[:nf], ip, ix, iv, O.TAU_MEDIAN, nthreads=threads)
    fel = time.perf_counter() - t0
    while fel < target_s * 0.5 and nf < 65536:
        nf = min(65536, nf * 4)
        t0 = time.perf_counter()
        O.energy_rows_faithful(Xh[:nf], ip, ix, iv, O.TAU_MEDIAN, nthreads=threads)
        fel = time.perf_counter() - t0
    return {"value": 65536 / el, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": f"first 65536 items x {X.shape[1]} features vs the feature Laplacian "
                      f"(nnz {Lf.nnz}), oracle/or_energy_rows TAUMODE Median, {el:.2f}s",
            "form": "restated-efficient",
            "faithful": {"value": nf / fel, "unit": "rows/s", "cores": threads,
                         "sample": f"first {nf} items, F^2 CsMat::get dispersion, {fel:.1f}s"}}


if __name__ == "__main__":
    main()
