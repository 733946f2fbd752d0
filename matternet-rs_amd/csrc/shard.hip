// shard.hip — the row-sharded multi-GPU kNN build behind one C entry
// (SURVEY.md §8(b) `mn_knn_sharded_f32`, §8(e)) on a caller-owned RCCL
// communicator: one process (or thread) per GPU, each holding its row shard.
//
// Symmetric form (round 4; self kNN, L2^2, the bf16x1 generator applies):
//   1. ncclAllGather of the shards -> X_all resident on every rank;
//   2. stage A: tau0 of the rank's rows against the global phase-1 sample;
//      ncclAllGather of tau0 and the row norms;
//   3. stage B: every rank builds the same Tf order and fp16 copy of all N
//      rows and sweeps ITS share of the symmetric block table (every
//      unordered pair of tiles once over the whole node — half the Gram of
//      the per-shard form), then re-ranks every row in partial mode;
//   4. grouped ncclSend/ncclRecv: each row's owner receives the R partial lists;
//   5. stage C: merge + certify (the certificate of the single-GPU sweep:
//      the union of the parts' admitted candidates is the same set), exact
//      split scan of the rare uncertified rows against X_all.
// Per-shard form (other metrics / generators, or when the symmetric form
// does not apply — decided collectively):
//   exact per-shard top-k of all N queries against the resident shard
//   (mn_knn_f32_qc, query chunks), the exchange, mn_knn_merge_f32.
// Both are exact: bit-identical to a single-GPU mn_knn_f32 of X.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "gram_sweep2.hpp"
#include "shard_sym.hpp"

#define MN_NCCL_TRY(expr)                                                          \
    do {                                                                           \
        ncclResult_t _r = (expr);                                                  \
        if (_r != ncclSuccess) {                                                   \
            mn::set_error("%s failed: %s", #expr, ncclGetErrorString(_r));         \
            return MN_EHIP;                                                        \
        }                                                                          \
    } while (0)

extern "C" {

int mn_rccl_unique_id(void *out_128_bytes) {
    mn::clear_error();
    MN_REQUIRE(out_128_bytes, MN_EINVAL, "mn_rccl_unique_id: NULL");
    ncclUniqueId id;
    MN_NCCL_TRY(ncclGetUniqueId(&id));
    std::memcpy(out_128_bytes, &id, sizeof(id));
    return MN_OK;
}

int mn_rccl_comm_init(const void *unique_id_128_bytes, int32_t world, int32_t rank,
                      void **comm_out) {
    mn::clear_error();
    MN_REQUIRE(unique_id_128_bytes && comm_out && world >= 1 && rank >= 0 && rank < world,
               MN_EINVAL, "mn_rccl_comm_init: bad arguments");
    ncclUniqueId id;
    std::memcpy(&id, unique_id_128_bytes, sizeof(id));
    ncclComm_t c = nullptr;
    MN_NCCL_TRY(ncclCommInitRank(&c, world, id, rank));
    *comm_out = (void *)c;
    return MN_OK;
}

int mn_rccl_comm_destroy(void *comm) {
    mn::clear_error();
    if (!comm) return MN_OK;
    MN_NCCL_TRY(ncclCommDestroy((ncclComm_t)comm));
    return MN_OK;
}

}  // extern "C"

namespace {

using mn::set_error;

struct DevBufs {
    std::vector<void *> v;
    void *get(size_t bytes) {
        void *p = nullptr;
        if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) return nullptr;
        v.push_back(p);
        return p;
    }
    ~DevBufs() {
        for (void *p : v) (void)hipFree(p);
    }
};

bool sym_applies(const mn::ShardPlan &pl, const mn_knn_opts *o) {
    return pl.ok && o->metric == MN_L2SQ && o->exclude_self &&
           (o->algo == MN_KNN_AUTO || o->algo == MN_KNN_BF16X1);
}

// the per-rank status agreement before each collective phase: max over ranks
// of (0 ok, 1 per-shard form, 2 error) — a rank that failed must not leave
// the others waiting in a collective
int agree(ncclComm_t c, hipStream_t s, int *dflag, int mine, int *out) {
    if (hipMemcpyAsync(dflag, &mine, 4, hipMemcpyHostToDevice, s) != hipSuccess) return MN_EHIP;
    if (ncclAllReduce(dflag, dflag, 1, ncclInt32, ncclMax, c, s) != ncclSuccess) {
        set_error("ncclAllReduce of the shard status failed");
        return MN_EHIP;
    }
    if (hipMemcpyAsync(out, dflag, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return MN_EHIP;
    return MN_OK;
}

int status_of(int rc) { return rc == MN_OK ? 0 : rc == 1 ? 1 : 2; }

// rank r's rows of every part list [N][k] go to rank r: part p of the
// receive buffer [R][nl][k] = the list computed on rank p
int exchange(ncclComm_t c, hipStream_t s, int world, int64_t nl, int k, const int32_t *li,
             const float *ld, int32_t *pi, float *pd) {
    if (ncclGroupStart() != ncclSuccess) return MN_EHIP;
    int rc = MN_OK;
    for (int p = 0; p < world && rc == MN_OK; ++p) {
        const size_t cnt = (size_t)nl * k;
        if (ncclSend(li + (size_t)p * cnt, cnt, ncclInt32, p, c, s) != ncclSuccess ||
            ncclSend(ld + (size_t)p * cnt, cnt, ncclFloat32, p, c, s) != ncclSuccess ||
            ncclRecv(pi + (size_t)p * cnt, cnt, ncclInt32, p, c, s) != ncclSuccess ||
            ncclRecv(pd + (size_t)p * cnt, cnt, ncclFloat32, p, c, s) != ncclSuccess)
            rc = MN_EHIP;
    }
    if (ncclGroupEnd() != ncclSuccess || rc != MN_OK) {
        set_error("grouped ncclSend/ncclRecv of the per-shard lists failed");
        return MN_EHIP;
    }
    return MN_OK;
}

}  // namespace

extern "C" {

int mn_knn_sharded_f32(const float *X_shard, int64_t n_local, int32_t d, void *comm,
                       const mn_knn_opts *opts, int64_t query_chunk, int32_t *out_idx,
                       float *out_dist) {
    using namespace mn;
    clear_error();
    MN_REQUIRE(X_shard && comm && opts && out_idx && out_dist, MN_EINVAL,
               "mn_knn_sharded_f32: NULL argument");
    MN_REQUIRE(n_local >= 1 && d >= 1 && opts->k >= 1, MN_EINVAL,
               "mn_knn_sharded_f32: bad shape");
    ncclComm_t c = (ncclComm_t)comm;
    int world = 1, rank = 0;
    MN_NCCL_TRY(ncclCommCount(c, &world));
    MN_NCCL_TRY(ncclCommUserRank(c, &rank));
    hipStream_t s = (hipStream_t)opts->stream;
    const int k = opts->k;
    const int64_t n_tot = n_local * world;
    MN_REQUIRE(n_tot <= INT32_MAX, MN_EINVAL, "mn_knn_sharded_f32: ids must fit int32");
    MN_REQUIRE(world <= 16, MN_ENOTSUP, "mn_knn_sharded_f32: at most 16 ranks (merge width)");
    const size_t part_b = (size_t)world * n_local * k;  // entries of [R][n_local][k]
    // device buffers owned by the call: X_all, the part lists of all rows
    // [N][k], the received parts [R][n_local][k], the per-row arrays
    DevBufs B;
    void *xall = B.get(sizeof(float) * (size_t)n_tot * d);
    int32_t *li = (int32_t *)B.get(4 * (size_t)n_tot * k);
    float *ld = (float *)B.get(4 * (size_t)n_tot * k);
    int32_t *pi = (int32_t *)B.get(4 * part_b);
    float *pd = (float *)B.get(4 * part_b);
    float *rowv = (float *)B.get(4 * (size_t)n_tot * 3 + 64);
    int *dflag = (int *)B.get(64);
    if (!xall || !li || !ld || !pi || !pd || !rowv || !dflag) {
        set_error("mn_knn_sharded_f32: device allocation failed");
        return MN_ENOMEM;
    }
    float *tau0_all = rowv, *qn_all = rowv + n_tot, *tc_all = rowv + 2 * n_tot;
    mn_knn_stats st{};
    st.n_queries = n_local;
    st.algo = MN_KNN_BF16X1;
    Timer tm;
    tm.start(opts->timing != 0, s);
    // 1. all-gather of the shards (rank r's rows at r * n_local)
    MN_NCCL_TRY(ncclAllGather(X_shard, xall, (size_t)n_local * d, ncclFloat32, c, s));
    const float *X_all = (const float *)xall;
    const ShardPlan pl = shard_plan(n_tot, d, k, world);
    bool sym = world > 1 && sym_applies(pl, opts);
    int agreed = 0, rc = MN_OK;
    int64_t ncand = 0;
    int nfb = 0;
    if (sym) {
        // 2. stage A, then every rank's tau0 / norms everywhere
        rc = shard_phase1(X_all, pl, (int64_t)rank * n_local, n_local, s, tau0_all + rank * n_local,
                          qn_all + rank * n_local);
        const int arc = agree(c, s, dflag, status_of(rc), &agreed);
        if (arc != MN_OK) return arc;
        if (agreed == 2) return rc != MN_OK ? rc : MN_EHIP;
        sym = agreed == 0;
    }
    tm.mark();
    if (sym) {
        MN_NCCL_TRY(ncclAllGather(tau0_all + rank * n_local, tau0_all, (size_t)n_local, ncclFloat32,
                                  c, s));
        MN_NCCL_TRY(ncclAllGather(qn_all + rank * n_local, qn_all, (size_t)n_local, ncclFloat32, c,
                                  s));
        // 3. stage B: this rank's share, partial lists of all rows
        rc = shard_share(X_all, pl, tau0_all, qn_all, rank, world, s, li, ld, tc_all,
                         opts->timing ? &ncand : nullptr);
        const int arc = agree(c, s, dflag, status_of(rc), &agreed);
        if (arc != MN_OK) return arc;
        if (agreed == 2) return rc != MN_OK ? rc : MN_EHIP;
        sym = agreed == 0;  // 1: a non-finite threshold anywhere (same on every rank)
    }
    tm.mark();
    if (sym) {
        // 4. the exchange, 5. stage C
        rc = exchange(c, s, world, n_local, k, li, ld, pi, pd);
        if (rc != MN_OK) return rc;
        tm.mark();
        rc = shard_finish(X_all, pl, (int64_t)rank * n_local, n_local, world,
                          (int64_t)n_local * k, pi, pd, tc_all, s, out_idx, out_dist, &nfb);
        if (rc != MN_OK) return rc;
        st.sweep_slices = -1;
    } else {
        // the per-shard form: exact per-shard top-k of every query against
        // this rank's shard, the exchange, the merge
        mn_knn_opts o = *opts;
        o.stream = s;
        const int64_t qc = query_chunk > 0 ? query_chunk : ((int64_t)1 << 21);
        for (int64_t a = 0; a < n_tot && rc == MN_OK; a += qc) {
            const int64_t b = std::min(n_tot, a + qc);
            rc = mn_knn_f32_qc(X_all + a * d, b - a, X_shard, n_local, d, a,
                               (int64_t)rank * n_local, &o, li + a * k, ld + a * k);
        }
        // a failed rank must not leave the others waiting in the exchange
        const int arc = agree(c, s, dflag, rc == MN_OK ? 0 : 2, &agreed);
        if (arc != MN_OK) return arc;
        if (agreed != 0) return rc != MN_OK ? rc : MN_EHIP;
        tm.mark();
        rc = exchange(c, s, world, n_local, k, li, ld, pi, pd);
        if (rc != MN_OK) return rc;
        tm.mark();
        rc = mn_knn_merge_f32(pi, pd, world, n_local, k, out_idx, out_dist, s);
        if (rc != MN_OK) return rc;
        st.algo = MN_KNN_AUTO;
    }
    tm.mark();
    MN_HIP_TRY(hipStreamSynchronize(s));
    st.n_uncertified = nfb;
    st.n_candidates = ncand;
    st.sample_rows = sym ? pl.m0 : 0;
    if (tm.on) {
        st.ms_sample = tm.ms(0, 1);   // all-gather + stage A
        st.ms_sweep = tm.ms(1, 2);    // stage B (per-shard form: the qc passes)
        st.ms_gram = st.ms_sample + st.ms_sweep;
        st.ms_rerank = tm.ms(2, 3);   // the exchange
        st.ms_fallback = tm.ms(3, 4); // stage C / the merge
        st.ms_total = tm.ms(0, 4);
    }
    knn_stats_ref() = st;
    return MN_OK;
}

// Host only: rank `rank`'s share of the node-wide symmetric tile table over
// nbk 256-row blocks (ksw2::sym_block_table_share; entries (I, Jfirst, tiles,
// stride), the empty XCD padding included).  out4 [cap][4] may be NULL to
// query the count; *n_out = entries.  MN_ECAP when cap is too small.
int mn_sym_share_table(int32_t nbk, int32_t rank, int32_t world, int32_t *out4, int64_t cap,
                       int64_t *n_out) {
    using namespace mn;
    clear_error();
    MN_REQUIRE(nbk >= 1 && world >= 1 && rank >= 0 && rank < world && n_out, MN_EINVAL,
               "mn_sym_share_table: bad arguments");
    const std::vector<int4> tab = ksw2::sym_block_table_share(nbk, 256, rank, world);
    *n_out = (int64_t)tab.size();
    if (!out4) return MN_OK;
    MN_REQUIRE((int64_t)tab.size() <= cap, MN_ECAP, "mn_sym_share_table: cap < %zu", tab.size());
    for (size_t i = 0; i < tab.size(); ++i) {
        out4[4 * i] = tab[i].x;
        out4[4 * i + 1] = tab[i].y;
        out4[4 * i + 2] = tab[i].z;
        out4[4 * i + 3] = tab[i].w;
    }
    return MN_OK;
}

// The symmetric sharded build of `world` ranks simulated on ONE device: X_all
// [n_tot][d] (device) stands for the all-gathered shards, the stages of every
// rank run in turn on this device and the exchange is a strided read of the
// part lists.  out [n_tot][k]: the global graph (bit-identical to mn_knn_f32).
// rank_ms [world][3] (host, may be NULL): per rank the stage A, stage B and
// stage C milliseconds (device events) — a rank's share of the real build.
// MN_ENOTSUP when the symmetric form does not apply (see mn_knn_sharded_f32).
int mn_knn_sharded_sim_f32(const float *X_all, int64_t n_tot, int32_t d, int32_t world,
                           const mn_knn_opts *opts, int32_t *out_idx, float *out_dist,
                           float *rank_ms) {
    using namespace mn;
    clear_error();
    MN_REQUIRE(X_all && opts && out_idx && out_dist, MN_EINVAL, "mn_knn_sharded_sim_f32: NULL argument");
    MN_REQUIRE(world >= 1 && world <= 16 && n_tot >= world && n_tot % world == 0 && d >= 1 &&
                   opts->k >= 1 && n_tot <= INT32_MAX,
               MN_EINVAL, "mn_knn_sharded_sim_f32: bad shape (n_tot a multiple of world <= 16)");
    hipStream_t s = (hipStream_t)opts->stream;
    const int k = opts->k;
    const int64_t nl = n_tot / world;
    const ShardPlan pl = shard_plan(n_tot, d, k, world);
    MN_REQUIRE(sym_applies(pl, opts), MN_ENOTSUP,
               "mn_knn_sharded_sim_f32: the symmetric sharded form does not apply");
    DevBufs B;
    int32_t *li = (int32_t *)B.get(4 * (size_t)world * n_tot * k);
    float *ld = (float *)B.get(4 * (size_t)world * n_tot * k);
    float *rowv = (float *)B.get(4 * (size_t)n_tot * 3 + 64);
    MN_REQUIRE(li && ld && rowv, MN_ENOMEM, "mn_knn_sharded_sim_f32: device allocation failed");
    float *tau0_all = rowv, *qn_all = rowv + n_tot, *tc_all = rowv + 2 * n_tot;
    std::vector<float> ms((size_t)world * 3, 0.f);
    int64_t ncand = 0;
    int nfb_tot = 0;
    for (int r = 0; r < world; ++r) {
        Timer t;
        t.start(true, s);
        const int rc = shard_phase1(X_all, pl, r * nl, nl, s, tau0_all + r * nl, qn_all + r * nl);
        MN_REQUIRE(rc != 1, MN_ENOTSUP, "mn_knn_sharded_sim_f32: values too large for the bf16 bound");
        if (rc != MN_OK) return rc;
        t.mark();
        MN_HIP_TRY(hipStreamSynchronize(s));
        ms[(size_t)r * 3] = t.ms(0, 1);
    }
    for (int r = 0; r < world; ++r) {
        Timer t;
        t.start(true, s);
        int64_t nc1 = 0;
        const int rc = shard_share(X_all, pl, tau0_all, qn_all, r, world, s, li + (size_t)r * n_tot * k,
                                   ld + (size_t)r * n_tot * k, tc_all, &nc1);
        MN_REQUIRE(rc != 1, MN_ENOTSUP, "mn_knn_sharded_sim_f32: non-finite thresholds");
        if (rc != MN_OK) return rc;
        t.mark();
        MN_HIP_TRY(hipStreamSynchronize(s));
        ms[(size_t)r * 3 + 1] = t.ms(0, 1);
        ncand += nc1;
    }
    for (int o = 0; o < world; ++o) {
        Timer t;
        t.start(true, s);
        int nfb = 0;
        const int rc = shard_finish(X_all, pl, o * nl, nl, world, n_tot * k, li + (size_t)o * nl * k,
                                    ld + (size_t)o * nl * k, tc_all, s, out_idx + (size_t)o * nl * k,
                                    out_dist + (size_t)o * nl * k, &nfb);
        if (rc != MN_OK) return rc;
        t.mark();
        MN_HIP_TRY(hipStreamSynchronize(s));
        ms[(size_t)o * 3 + 2] = t.ms(0, 1);
        nfb_tot += nfb;
    }
    mn_knn_stats st{};
    st.n_queries = n_tot;
    st.algo = MN_KNN_BF16X1;
    st.n_uncertified = nfb_tot;
    st.n_candidates = ncand;
    st.sample_rows = pl.m0;
    st.sweep_slices = -1;
    for (int r = 0; r < world; ++r) {
        st.ms_sample = std::max(st.ms_sample, ms[(size_t)r * 3]);
        st.ms_sweep = std::max(st.ms_sweep, ms[(size_t)r * 3 + 1]);
        st.ms_fallback = std::max(st.ms_fallback, ms[(size_t)r * 3 + 2]);
    }
    st.ms_gram = st.ms_sample + st.ms_sweep;
    st.ms_total = st.ms_gram + st.ms_fallback;
    knn_stats_ref() = st;
    if (rank_ms) std::memcpy(rank_ms, ms.data(), sizeof(float) * ms.size());
    return MN_OK;
}

}  // extern "C"
