"""Headline benchmark: k-NN graph build vector-pairs/sec (BASELINE.json configs[1] /
configs[3]) on MI355X through the HIP C ABI.

  python bench.py [--gpus N --steps K --warmup W]
  N>1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
           --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

One step = one exact kNN graph build (k=32, squared L2, self excluded) over all
rows: at N=1 the C2 workload (1M x 768 f32), at N GPUs N x 1M rows row-sharded
(C4 at N=8): every rank keeps its 1M-row corpus shard resident, receives all
query rows (all-gather over RCCL/xGMI), computes the exact per-shard top-k of
every query, and the per-shard lists are exchanged (all-to-all) and merged on
each query's owner rank.  Inputs are generated on device before timing.
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
    ap.add_argument("--c5-rows", type=int, default=1_048_576)
    ap.add_argument("--c5-dim", type=int, default=3072)
    ap.add_argument("--c5-parity-rows", type=int, default=3,
                    help="rows of the C5 graph checked bit-exact against the oracle (0 = off)")
    ap.add_argument("--no-c3", dest="c3", action="store_false",
                    help="skip the C3 legs (Laplacian assembly, energy pass, sorted index)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_gram_latest.json"),
                    help="PMC-derived HBM bytes per launch of the Gram kernel (optional)")
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
    if world > 1:
        from surfface_hip.dist import sharded_knn
    torch.cuda.synchronize()

    gram_ms = []

    last = {}

    def knn_fn(Q, C, kk, c_off):
        r = S.knn_l2sq_qc(Q, C, kk, q_offset=0, c_offset=c_off, timing=True)
        gram_ms.append(r.stats["ms_gram"])
        last["stats"] = r.stats
        return r.idx, r.dist

    def step():
        if world == 1:
            r = S.knn_l2sq(X, k, timing=True)
            gram_ms.append(r.stats["ms_gram"])
            return r.idx, r.dist, r.stats
        # all-gather queries, exact per-shard top-k vs the resident shard,
        # all-to-all of the lists, merge on the owner (surfface_hip/dist.py)
        idx, dd = sharded_knn(X, k, knn_fn=knn_fn, merge_fn=S.merge_parts)
        return idx, dd, last["stats"]

    for _ in range(a.warmup):
        step()
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

    # roofline of the dominant kernel: algorithmic flops per launch
    # = 2 * nq * nc_shard * d (full Gram); duration from HIP
    # events recorded on the launch stream inside the library.
    nq = n_tot
    flops_launch = 2.0 * nq * n_loc * d
    gms = float(np.mean(gram_ms)) if gram_ms else float("nan")
    achieved = flops_launch / (gms * 1e-3) / 1e12
    st0 = out[2]
    split = st0.get("algo") == 2
    kname = "k_gram_bf16<GM_L2>" if split else "k_gram_topk"
    traffic = None
    if os.path.exists(a.pmc_json):
        try:
            pm = json.load(open(a.pmc_json))
            if (pm.get("rows_per_gpu") == n_loc and pm.get("dim") == d and world == 1
                    and pm.get("kernel", "").startswith(kname.split("<")[0])):
                traffic = pm.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    if split:
        # bf16-split candidates: every f32 product is hi*hi + hi*lo + lo*hi, three
        # bf16 MFMA products, so the ceiling for this algorithm's Gram flops is the
        # dense bf16 MFMA peak / 3
        peak = BF16_MFMA_PEAK_TFLOPS / 3.0
        roof = {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 3),
                "peak": round(peak, 1), "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                "traffic": traffic, "ms_per_launch": round(gms, 3),
                "flop_per_launch": flops_launch,
                "peak_basis": ("dense bf16 MFMA 2500 TFLOP/s / 3 bf16 products per f32 product "
                               "(x = hi + lo; hi.hi + hi.lo + lo.hi)"),
                "mfma_issued_tflops": round(3.0 * achieved, 1),
                "vs_f32_mfma_peak": round(achieved / FP32_MFMA_PEAK_TFLOPS, 3)}
    else:
        roof = {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 3),
                "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
                "ms_per_launch": round(gms, 3), "flop_per_launch": flops_launch}

    # C3 legs (configs[2]): Laplacian assembly + energymaps/taumode pass + index,
    # on this rank's rows (timed individually after the headline step)
    c3 = None
    if a.c3:
        c3 = c3_legs(S, X, out[0], out[1], k)

    c5 = None
    if a.c5 and world == 1:
        c5 = c5_leg(S, _lib, L, a, dev, stream)

    cpu = None
    parity = None
    if rank == 0 and world == 1 and a.cpu_seconds > 0:
        cpu, parity = cpu_baseline(X, out[0], out[1], k, a.cpu_seconds)

    if rank == 0:
        st = out[2]
        line = {
            "metric": "vector-pairs/sec for k-NN graph build (N=1M, d=768) + Laplacian energy rows/sec",
            "value": value, "unit": "pairs/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "candidate_generator": "bf16x3 split MFMA" if split else "f32 MFMA",
            "data": "synthetic U[-1,1) f32 (splitmix64 counter stream, seed 42), generated on device",
            "config": {"workload": ("C2: 1M x 768 f32 exact kNN k=32" if world == 1 else
                                    f"C4-style: {n_tot} x {d} f32 exact kNN k={k}, row-sharded"),
                       "n_rows": n_tot, "dim": d, "k": k, "rows_per_gpu": n_loc,
                       "metric_space": "squared L2 (reference sequential f32 fold)",
                       "parallelism": (f"corpus row-shard x{world}: RCCL all-gather of queries, "
                                       "exact per-shard top-k, all-to-all + merge")},
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity_sample": parity,
            "energy_rows_per_sec": (c3 or {}).get("energy_rows_per_sec"),
            "c3_legs": c3,
            "c5_leg": c5,
            "knn_stats": {"uncertified_rows": st["n_uncertified"], "slices": st["slices"],
                          "list_len": st["list_len"], "ms_norms": st["ms_norms"],
                          "ms_gram": st["ms_gram"], "ms_rerank": st["ms_rerank"],
                          "ms_fallback": st["ms_fallback"], "algo": st.get("algo")},
        }
        print(json.dumps(line), flush=True)
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
    ms, (fi, fd, fw, fst) = _timed(lambda: S.knn_cos_columns(X, 4, eps=1.0, sigma=1.0, p=2.0), 1)
    out["feature_knn_cos"] = {"ms": round(ms, 3), "uncertified": fst["n_uncertified"],
                              "gram_tflops": round(2.0 * f * f * n / 2 / (fst["ms_gram"] * 1e9), 2)
                              if fst["ms_gram"] else None}
    ms, (Lf, _) = _timed(lambda: S.build_laplacian_from_knn(fi, fw, weight_kernel="given",
                                                           symmetrise="union"))
    out["feature_laplacian"] = {"ms": round(ms, 3), "nnz": Lf.nnz}
    ms, (E, G, lam) = _timed(lambda: S.energy_rows(X, Lf))
    ebytes = n * f * 4 + Lf.nnz * 12 + (f + 1) * 8 + n * 3 * 8
    out["energy_rows"] = {"ms": round(ms, 3), "GB_per_s": round(ebytes / ms / 1e6, 1),
                          "entries_per_row": S.energy.last_stats()["entries"]}
    out["energy_rows_per_sec"] = n / (ms * 1e-3)
    # energymaps diffusion pre-pass (eta 0.1, 4 steps; energymaps.rs:518-546) on
    # the same rows: f32 in, f64 out; bytes = N F (4 + 8)
    Xd = torch.empty((n, f), dtype=torch.float64, device=X.device)
    ms, _ = _timed(lambda: S.diffuse_rows(X, Lf, 0.1, 4, out=Xd))
    out["diffusion_4_steps"] = {"ms": round(ms, 3), "GB_per_s": round(n * f * 12 / ms / 1e6, 1)}
    del Xd
    # item-graph orientation: the F feature signals against
    # the n x n item Laplacian; bytes = one x_j row gather per stored entry
    ms, _ = _timed(lambda: S.signal_energy_and_dispersion(X, Lit))
    out["item_graph_signals"] = {"ms": round(ms, 3),
                                 "GB_per_s": round((Lit.nnz // 2 + n) * f * 4 / ms / 1e6, 1)}
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
    flops = 2.0 * n * n * d
    ach = flops / (st["ms_gram"] * 1e-3) / 1e12
    out = {"workload": f"C5: {n} x {d} bf16 rectified-cosine item graph k={k} + SF-GRASS 0.5",
           "ms_total": round(ms, 1), "pairs_per_s": n * n / (ms * 1e-3),
           "roofline": {"bound": "mfma", "kernel": "k_gram_bf16", "achieved": round(ach, 1),
                        "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(ach / BF16_MFMA_PEAK_TFLOPS, 4), "flop_per_launch": flops,
                        "ms_per_launch": round(st["ms_gram"], 1)},
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


def cpu_baseline(X, idx, dd, k, target_s):
    """Oracle (C restatement, OpenMP) timed on the host on a bounded sample of
    query rows against the full corpus; also a free bit-exact parity check of
    those rows against the GPU result."""
    from oracle import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    Xh = X.cpu().numpy()
    n = Xh.shape[0]
    rng = np.random.default_rng(1)
    cal = np.sort(rng.choice(n, threads, replace=False))  # warms pages + threads
    i0, d0 = O.knn_l2sq_rows(Xh, k, cal, nthreads=threads)
    perm = rng.permutation(n)
    batch = threads * 4
    done, el = 0, 0.0
    ri_l, rd_l = [], []
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
    cpu = {"value": m * (n - 1) / el, "unit": "pairs/s", "cores": threads, "kind": "port",
           "sample": f"{m} random query rows x {n} corpus rows, d={Xh.shape[1]}, k={k} "
                     f"(oracle/or_knn_l2sq_rows_f32, OpenMP), {el:.1f}s"}
    parity = {"rows_checked": m, "rows_bit_exact": ok, "plus_calibration_rows": threads,
              "calibration_bit_exact": bool(np.array_equal(i0, idx.cpu().numpy()[cal]))}
    return cpu, parity


if __name__ == "__main__":
    main()
