"""K3 parity on the GPU: HIP energy rows (C ABI) vs the CPU oracle.

Contract: E, G, lambda within 1e-9 relative (abs 1e-12 near
0) — the reference sums in rayon par_bridge order; normalise_lambdas uses the
same min/max so its outputs inherit that tolerance.
"""
import numpy as np
import pytest
import torch

import datagen
from oracle import oracle as O

pytestmark = pytest.mark.gpu

GS = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden",
                                        "golden_small.npz"))
RTOL, ATOL = 1e-9, 1e-12


def csr_dev(ip, ix, iv):
    import surfface_hip as S
    n = len(ip) - 1
    return S.CsrMatrix(torch.from_numpy(ip.astype(np.int64)).cuda(),
                       torch.from_numpy(ix.astype(np.int32)).cuda(),
                       torch.from_numpy(iv.astype(np.float64)).cuda(), (n, n))


def feature_laplacian(f=768, profile=1500, topk=4, seed=9):
    """F x F union Laplacian from the rectified-cosine kNN of the feature
    columns (graph.rs:214 builds the Laplacian on the transposed centroids)."""
    P = datagen.uniform(profile, f, seed=seed)
    idx, dist, w = O.knn_cos(np.ascontiguousarray(P.T), topk, eps=1.0, sigma=1.0, p=2.0)
    return O.laplacian_union(idx, w)


def run(X, ip, ix, iv, g_mode, tau):
    import surfface_hip as S
    E, G, lam = S.energy_rows(torch.from_numpy(X).cuda(), csr_dev(ip, ix, iv), g_mode, tau)
    return E.cpu().numpy(), G.cpu().numpy(), lam.cpu().numpy()


def test_golden_taumode_rows():
    import surfface_hip as S
    E, G, lam = run(GS["energy_X"], GS["lapu_indptr"], GS["lapu_indices"], GS["lapu_values"],
                    0, S.TauMode.Median)
    np.testing.assert_allclose(E, GS["energy_E"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(G, GS["energy_G"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(lam, GS["energy_lambda"], rtol=RTOL, atol=ATOL)
    assert lam[3] == 0.0


@pytest.mark.parametrize("tau", ["median", "mean", "pct", "fixed"])
def test_taumode_768_features(tau):
    import surfface_hip as S
    ip, ix, iv = feature_laplacian()
    X = datagen.uniform(20000, 768, seed=21)
    X[5] = 0.0
    X[6] = 3.0  # constant row: G = 0
    X[7, ::2] = 0.25  # many ties for the order statistics
    tm = {"median": (S.TauMode.Median, O.TAU_MEDIAN, 0.0),
          "mean": (S.TauMode.Mean, O.TAU_MEAN, 0.0),
          "pct": (S.TauMode.Percentile(0.3), O.TAU_PERCENTILE, 0.3),
          "fixed": (S.TauMode.Fixed(0.2), O.TAU_FIXED, 0.2)}[tau]
    E, G, lam = run(X, ip, ix, iv, 0, tm[0])
    rE, rG, rl = O.energy_rows(X, ip, ix, iv, O.G_TAUMODE, tm[1], tm[2])
    np.testing.assert_allclose(E, rE, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(G, rG, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(lam, rl, rtol=RTOL, atol=ATOL)
    assert lam[5] == 0.0 and G[6] == 0.0


def test_odd_feature_count_and_energymaps_mode():
    import surfface_hip as S
    ip, ix, iv = feature_laplacian(f=301, profile=800, topk=5, seed=4)
    X = datagen.clustered(5000, 301, seed=3, blobs=4)
    for gm, og in ((0, O.G_TAUMODE), (1, O.G_ENERGYMAPS)):
        E, G, lam = run(X, ip, ix, iv, gm, S.TauMode.Median)
        rE, rG, rl = O.energy_rows(X, ip, ix, iv, og, O.TAU_MEDIAN)
        np.testing.assert_allclose(E, rE, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(G, rG, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(lam, rl, rtol=RTOL, atol=ATOL)


def test_nonsymmetric_laplacian_path():
    import surfface_hip as S
    ip, ix, iv = feature_laplacian(f=200, profile=600, topk=3, seed=2)
    iv = iv.copy()
    iv[5] *= 1.5  # break exact symmetry: the kernel must stream all entries
    X = datagen.uniform(3000, 200, seed=8)
    E, G, lam = run(X, ip, ix, iv, 0, S.TauMode.Median)
    assert S.energy.last_stats()["symmetric"] == 0
    rE, rG, rl = O.energy_rows(X, ip, ix, iv, O.G_TAUMODE, O.TAU_MEDIAN)
    np.testing.assert_allclose(lam, rl, rtol=RTOL, atol=ATOL)


def test_known_answer_chain_and_constant_rows():
    import surfface_hip as S
    # surfface-core tests/test_spectral.rs:187-251 chain graph 0-1-2
    ip = np.array([0, 2, 5, 7]); ix = np.array([0, 1, 0, 1, 2, 1, 2])
    iv = np.array([1.0, -1.0, -1.0, 2.0, -1.0, -1.0, 1.0])
    X = np.array([[1, 1, 1], [1, 0, -1]], np.float32)
    E, G, lam = run(X, ip, ix, iv, 0, S.TauMode.Median)
    assert abs(E[0]) < 1e-12 and G[0] == 0.0 and lam[1] > lam[0]


def test_normalise_lambdas_vs_oracle():
    import surfface_hip as S
    lam = np.random.default_rng(0).normal(size=100_001)
    t = torch.from_numpy(lam.copy()).cuda()
    _, mn, mx, rg = S.normalise_lambdas(t)
    r, rmn, rmx, rrg = O.normalise_lambdas(lam)
    assert (mn, mx, rg) == (rmn, rmx, rrg)
    np.testing.assert_array_equal(t.cpu().numpy(), r)
    # all-negative input: max fold starts at 0.0 (core.rs:1343)
    t = torch.tensor([-1.0, -3.0, -2.0], dtype=torch.float64).cuda()
    S.normalise_lambdas(t)
    np.testing.assert_allclose(t.cpu().numpy(), [2 / 3, 0.0, 1 / 3], atol=1e-15)


def test_odd_rows_and_positive_offdiagonals():
    """n odd (the last two-row pass holds one row) and positive off-diagonal
    entries (they feed the Rayleigh numerator, never the dispersion), both
    dispersion modes."""
    import scipy.sparse as sp
    import surfface_hip as S
    ip, ix, iv = feature_laplacian(f=301, profile=800, topk=5, seed=4)
    M = sp.csr_matrix((iv, ix, ip), shape=(301, 301)).tolil()
    rng = np.random.default_rng(3)
    rows, cols = sp.triu(M.tocsr(), k=1).nonzero()
    for t in rng.choice(len(rows), 40, replace=False):
        M[rows[t], cols[t]] = M[cols[t], rows[t]] = 0.3
    M = M.tocsr()
    M.sort_indices()
    ip2, ix2, iv2 = M.indptr.astype(np.int64), M.indices.astype(np.int32), M.data
    X = datagen.clustered(1001, 301, seed=5, blobs=3)
    for gm, og in ((0, O.G_TAUMODE), (1, O.G_ENERGYMAPS)):
        E, G, lam = run(X, ip2, ix2, iv2, gm, S.TauMode.Median)
        assert S.energy.last_stats()["symmetric"] == 1
        rE, rG, rl = O.energy_rows(X, ip2, ix2, iv2, og, O.TAU_MEDIAN)
        np.testing.assert_allclose(E, rE, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(G, rG, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(lam, rl, rtol=RTOL, atol=ATOL)


def test_entry_list_beyond_lds_and_wide_rows():
    """f = 2048 with topk 24: the entry list (~50k entries) exceeds the LDS
    budget and is read from L2; rows of 2048 values (NR = 32 registers)."""
    import surfface_hip as S
    ip, ix, iv = feature_laplacian(f=2048, profile=300, topk=24, seed=6)
    X = datagen.uniform(333, 2048, seed=12)
    E, G, lam = run(X, ip, ix, iv, 0, S.TauMode.Median)
    rE, rG, rl = O.energy_rows(X, ip, ix, iv, O.G_TAUMODE, O.TAU_MEDIAN)
    np.testing.assert_allclose(E, rE, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(G, rG, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(lam, rl, rtol=RTOL, atol=ATOL)
    assert S.energy.last_stats()["entries"] * 12 > 96 * 1024


def test_stage_d_spectral_lambdas_vs_oracle():
    """compute_tau_mode_gpu (spectral/bridge.rs:27-69) on a Stage C Laplacian
    (MAX, L_sym, f32 values) and on a legacy f64 Laplacian.  The reference
    computes in f32 through Burn matmuls; this path in f64: tolerance 1e-4."""
    import surfface_hip as S
    P = datagen.uniform(400, 300, seed=31).T.copy()  # 300 feature nodes, profile 400
    idx, dist = O.knn_l2sq(P, 10)
    w = (1.0 / (1.0 + dist)).astype(np.float32)
    out = S.laplacian_stage_from_edges(torch.from_numpy(idx).cuda(), torch.from_numpy(w).cuda(),
                                       S.LaplacianConfig(k_neighbors=10))
    ip, ix, iv = out.matrix.to_numpy()
    X = datagen.uniform(5001, 300, seed=32)
    X[7] = 0.0  # zero row: R = 0 / (0 + 1e-9) = 0
    lam = S.compute_tau_mode_gpu(out, torch.from_numpy(X).cuda()).cpu().numpy()
    ref = O.spectral_lambdas(X, ip, ix, iv.astype(np.float32))
    np.testing.assert_allclose(lam, ref, rtol=1e-4, atol=1e-7)
    lam2, R, D = S.compute_lambdas_gpu(out.matrix, torch.from_numpy(X).cuda())
    D = D.cpu().numpy()
    assert (D >= 0).all() and (D <= 1).all() and abs(D.sum() - 1.0) < 1e-9
    # legacy f64 feature Laplacian (unnormalised D - W)
    lip, lix, liv = feature_laplacian(f=300, profile=500, topk=5, seed=33)
    lam3, _, _ = S.compute_lambdas_gpu(csr_dev(lip, lix, liv), torch.from_numpy(X).cuda())
    ref3 = O.spectral_lambdas(X, lip, lix, liv.astype(np.float32))
    np.testing.assert_allclose(lam3.cpu().numpy(), ref3, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("x64", [False, True])
def test_diffusion_and_matvec_bit_exact(x64):
    """EnergyMaps diffusion (energymaps.rs:518-546, eta 0.1 x 4 steps) and
    GraphLaplacian::multiply_vector (graph.rs:464-501): f64 CSR row folds in
    stored order — bit-exact vs the oracle, f32 or f64 rows, odd sizes."""
    import surfface_hip as S
    ip, ix, iv = feature_laplacian(f=301, profile=700, topk=6, seed=41)
    X = datagen.clustered(1003, 301, seed=42, blobs=5)
    Xd = torch.from_numpy(X).cuda()
    if x64:
        Xd = Xd.double()
    L = csr_dev(ip, ix, iv)
    out = S.diffuse_rows(Xd, L, 0.1, 4).cpu().numpy()
    ref = O.diffuse_rows(X.astype(np.float64), ip, ix, iv, 0.1, 4)
    np.testing.assert_array_equal(out.view(np.uint64), ref.view(np.uint64))
    Y = S.laplacian_matvec_rows(Xd, L).cpu().numpy()
    refY = O.diffuse_rows(X.astype(np.float64), ip, ix, iv, matvec=True)
    np.testing.assert_array_equal(Y.view(np.uint64), refY.view(np.uint64))
    # the reference's row sums: L 1 = 0 for the unnormalised union Laplacian
    ones = S.laplacian_matvec_rows(torch.ones((2, 301), dtype=torch.float64, device="cuda"), L)
    assert float(ones.abs().max()) < 1e-12
    # in place (f64 input aliasing the output)
    if x64:
        S.diffuse_rows(Xd, L, 0.1, 4, out=Xd)
        np.testing.assert_array_equal(Xd.cpu().numpy().view(np.uint64), ref.view(np.uint64))


@pytest.mark.parametrize("gm", [0, 1])
def test_item_graph_signal_orientation(gm):
    """node_energy_and_dispersion(X^T, L_items): the 96
    feature signals of length n = 6000 against the item kNN Laplacian (UNION,
    rational weights); tolerance 1e-9 relative; a non-symmetric L too."""
    import surfface_hip as S
    X = datagen.clustered(6000, 96, seed=51, blobs=6)
    idx, dist = O.knn_l2sq(X, 10)
    L, _ = S.build_laplacian_from_knn(torch.from_numpy(idx).cuda(), torch.from_numpy(dist).cuda(),
                                      eps=1e30, sigma=4.0)
    ip, ix, iv = L.to_numpy()
    og = O.G_TAUMODE if gm == 0 else O.G_ENERGYMAPS
    E, G = S.signal_energy_and_dispersion(torch.from_numpy(X).cuda(), L, gm)
    rE, rG, _ = O.energy_rows(np.ascontiguousarray(X.T), ip, ix, iv, og, O.TAU_MEDIAN)
    np.testing.assert_allclose(E.cpu().numpy(), rE, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(G.cpu().numpy(), rG, rtol=RTOL, atol=ATOL)
    iv2 = iv.copy()
    iv2[3] *= 1.25  # break symmetry: every stored entry is streamed
    E2, G2 = S.signal_energy_and_dispersion(torch.from_numpy(X).cuda(), csr_dev(ip, ix, iv2), gm)
    rE2, rG2, _ = O.energy_rows(np.ascontiguousarray(X.T), ip, ix, iv2, og, O.TAU_MEDIAN)
    np.testing.assert_allclose(E2.cpu().numpy(), rE2, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(G2.cpu().numpy(), rG2, rtol=RTOL, atol=ATOL)
    # symmetric, but rows stored in shuffled column order (k_check_sym bit 4):
    # the j < i prefix skip must not be taken
    rng = np.random.default_rng(3)
    ix3, iv3 = ix.copy(), iv.copy()
    for r in range(len(ip) - 1):
        a, b = int(ip[r]), int(ip[r + 1])
        pr = rng.permutation(b - a)
        ix3[a:b], iv3[a:b] = ix[a:b][pr], iv[a:b][pr]
    E3, G3 = S.signal_energy_and_dispersion(torch.from_numpy(X).cuda(), csr_dev(ip, ix3, iv3), gm)
    np.testing.assert_allclose(E3.cpu().numpy(), rE, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(G3.cpu().numpy(), rG, rtol=RTOL, atol=ATOL)


def test_item_graph_signals_768():
    """The C3 shape's 768 signals (three per thread) on a smaller item graph:
    the per-entry coefficient form (num / S / Q) within 1e-9 of the oracle."""
    import surfface_hip as S
    X = datagen.uniform(3000, 768, seed=52)
    idx, dist = O.knn_l2sq(X, 8)
    L, _ = S.build_laplacian_from_knn(torch.from_numpy(idx).cuda(), torch.from_numpy(dist).cuda(),
                                      eps=1e30, sigma=8.0)
    ip, ix, iv = L.to_numpy()
    for gm, og in ((0, O.G_TAUMODE), (1, O.G_ENERGYMAPS)):
        E, G = S.signal_energy_and_dispersion(torch.from_numpy(X).cuda(), L, gm)
        rE, rG, _ = O.energy_rows(np.ascontiguousarray(X.T), ip, ix, iv, og, O.TAU_MEDIAN)
        np.testing.assert_allclose(E.cpu().numpy(), rE, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(G.cpu().numpy(), rG, rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("tau", ["median", "pct"])
def test_tau_order_statistic_adversarial_rows(tau):
    """tau = the row's median / percentile (taumode.rs:29-70) through the
    value-linear bucket select (energy.hip wave_select_lin) and its radix
    fallback: rows whose values pile into one bucket (> 64 members: exponential
    tails, a 1e30 outlier), half-tied rows, two-valued rows, negative rows,
    huge / tiny ranges, subnormals — lambdas within the K3 tolerance."""
    import surfface_hip as S
    ip, ix, iv = feature_laplacian()
    rng = np.random.default_rng(5)
    n, f = 4096, 768
    X = datagen.uniform(n, f, seed=33)
    X[0] = rng.exponential(size=f).astype(np.float32) ** 6       # heavy tail
    X[1] = np.float32(0.5)
    X[1, ::3] = rng.random(len(range(0, f, 3))).astype(np.float32)
    X[2] = np.where(rng.random(f) < 0.5, 1.0, 2.0).astype(np.float32)
    X[3] = -np.abs(X[3])
    X[4] = datagen.uniform(1, f, seed=4)[0] * np.float32(1e-30)
    X[5, 7] = np.float32(1e30)                                   # one outlier: all else in bucket 0
    X[6] = (rng.random(f) * 1e-40).astype(np.float32)             # subnormals
    X[7] = np.float32(3.0)
    X[7, 100] = np.float32(3.0000002)
    X[8:64] = (rng.standard_normal((56, f)) ** 3).astype(np.float32)
    X[64] = np.where(rng.random(f) < 0.9, 0.0, X[64]).astype(np.float32)  # sparse: tied zeros
    X[65] = np.where(rng.random(f) < 0.5, np.float32(-0.0), np.float32(0.0))
    X[65, :40] = rng.random(40).astype(np.float32)                # -0 / +0 around the middle
    X[66] = np.float32(-2.0)
    X[66, 384:] = np.float32(7.0)                                 # the two middle keys differ
    X[67] = np.sort(X[67])                                        # sorted along the row
    X[68] = np.float32(-np.float32(3.4e38))
    X[68, ::2] = np.float32(3.4e38)                               # the span overflows f32
    tm = {"median": (S.TauMode.Median, O.TAU_MEDIAN, 0.0),
          "pct": (S.TauMode.Percentile(0.77), O.TAU_PERCENTILE, 0.77)}[tau]
    E, G, lam = run(X, ip, ix, iv, 0, tm[0])
    rE, rG, rl = O.energy_rows(X, ip, ix, iv, O.G_TAUMODE, tm[1], tm[2])
    np.testing.assert_allclose(E, rE, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(G, rG, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(lam, rl, rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("tau", ["median", "pct", "mean"])
def test_v2_kernel_matches_v1(tau, monkeypatch):
    """k_energy_rows2 (diagonal from registers, counted tau select, prefetched
    rows) against the round-2 kernel (MN_ENERGY_V1=1) and the oracle on the
    C3 feature Laplacian with an odd row count."""
    import surfface_hip as S
    ip, ix, iv = feature_laplacian()
    X = datagen.uniform(3001, 768, seed=41)
    X[10] = (np.random.default_rng(3).standard_normal(768) ** 3).astype(np.float32)
    tm = {"median": (S.TauMode.Median, O.TAU_MEDIAN, 0.0),
          "pct": (S.TauMode.Percentile(0.1), O.TAU_PERCENTILE, 0.1),
          "mean": (S.TauMode.Mean, O.TAU_MEAN, 0.0)}[tau]
    E2, G2, l2 = run(X, ip, ix, iv, 0, tm[0])
    monkeypatch.setenv("MN_ENERGY_V1", "1")
    with S._lib.use_tuning():  # the tuning build honours the knob
        E1, G1, l1 = run(X, ip, ix, iv, 0, tm[0])
    rE, rG, rl = O.energy_rows(X, ip, ix, iv, O.G_TAUMODE, tm[1], tm[2])
    for a, b, r in ((E2, E1, rE), (G2, G1, rG), (l2, l1, rl)):
        np.testing.assert_allclose(a, b, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(a, r, rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("gm,tau", [(0, "median"), (0, "pct"), (0, "mean"), (0, "fixed"), (1, "median"),
                                    (2, "median")])
def test_v3_single_pass_matches_two_kernel_path(gm, tau, monkeypatch):
    """k_energy_rows3 (round 4: X streamed once, tau selected inline, rows
    staged as f64 pairs, the list-A identity x^T L x = sum (L_cc - dgA_c) x_c^2
    + sum_A w (x_i - x_j)^2 + list B) against the two-kernel path
    (k_row_tau + k_energy_rows2, MN_ENERGY_V3=0) and the oracle: taumode with
    every tau mode, energymaps and Stage D, an odd row count, the heavy-tail /
    constant / zero / tied rows."""
    import surfface_hip as S
    ip, ix, iv = feature_laplacian()
    X = datagen.uniform(4097, 768, seed=43)
    rng = np.random.default_rng(8)
    X[1] = 0.0
    X[2] = np.float32(2.5)
    X[3] = (rng.standard_normal(768) ** 5).astype(np.float32)
    X[4, ::2] = np.float32(0.125)
    X[5] = np.where(rng.random(768) < 0.9, 0.0, X[5]).astype(np.float32)
    tm = {"median": (S.TauMode.Median, O.TAU_MEDIAN, 0.0),
          "pct": (S.TauMode.Percentile(0.3), O.TAU_PERCENTILE, 0.3),
          "mean": (S.TauMode.Mean, O.TAU_MEAN, 0.0),
          "fixed": (S.TauMode.Fixed(0.2), O.TAU_FIXED, 0.2)}[tau]
    E3, G3, l3 = run(X, ip, ix, iv, gm, tm[0])
    monkeypatch.setenv("MN_ENERGY_V3", "0")
    with S._lib.use_tuning():
        E2, G2, l2 = run(X, ip, ix, iv, gm, tm[0])
    if gm == 2:  # Stage D: f32 Burn reference, the oracle within 1e-4 (test_stage_d_*)
        for a, b in ((E3, E2), (G3, G2), (l3, l2)):
            np.testing.assert_allclose(a, b, rtol=RTOL, atol=ATOL)
        return
    rE, rG, rl = O.energy_rows(X, ip, ix, iv, gm, tm[1], tm[2])
    for a, b, r in ((E3, E2, rE), (G3, G2, rG), (l3, l2, rl)):
        np.testing.assert_allclose(a, b, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(a, r, rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("v3", ["2", "3"])
@pytest.mark.parametrize("tau", ["median", "fixed"])
def test_v3_stage_variants_match_oracle(v3, tau, monkeypatch):
    """The f32-stage single pass (MN_ENERGY_V3=2) and the same kernel with the
    host-ordered, LDS-bank-conflict-free entry lists in a bank-balanced column
    order (MN_ENERGY_V3=3, conflict_free_lists) against the oracle at 1e-9."""
    import surfface_hip as S
    ip, ix, iv = feature_laplacian()
    X = datagen.uniform(3001, 768, seed=47)
    X[7] = 0.0
    tm = {"median": (S.TauMode.Median, O.TAU_MEDIAN, 0.0),
          "fixed": (S.TauMode.Fixed(0.2), O.TAU_FIXED, 0.2)}[tau]
    monkeypatch.setenv("MN_ENERGY_V3", v3)
    with S._lib.use_tuning():
        E3, G3, l3 = run(X, ip, ix, iv, 0, tm[0])
    rE, rG, rl = O.energy_rows(X, ip, ix, iv, 0, tm[1], tm[2])
    for a, r in ((E3, rE), (G3, rG), (l3, rl)):
        np.testing.assert_allclose(a, r, rtol=RTOL, atol=ATOL)
