// shard.hip — the row-sharded multi-GPU kNN build behind one C entry
// (SURVEY.md §8(b) `mn_knn_sharded_f32`, §8(e) strategy A) on a caller-owned
// RCCL communicator: one process (or thread) per GPU, each holding its row
// shard of X.
//
//   1. ncclAllGather of the shards -> every rank holds all N query rows;
//   2. exact per-shard top-k of all queries against the resident shard
//      (mn_knn_f32_qc with global offsets), in query chunks;
//   3. grouped ncclSend/ncclRecv: each query's owner receives the R per-shard
//      lists of its rows (the lists of rank r's queries computed on rank s);
//   4. mn_knn_merge_f32 by (dist, id) -> the owner's rows of the global graph.
// The merge is exact: the global top-k is contained in the union of the exact
// per-shard top-k lists, and a pair's distance is the same fold on any shard.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>

#include "common.hpp"

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
    const size_t xall_b = sizeof(float) * (size_t)n_tot * d;
    const size_t part_b = (size_t)world * n_local * k;  // entries of [R][n_local][k]
    // device buffers owned by the call: X_all, the per-shard lists of all
    // queries [N][k], and the received parts [R][n_local][k]
    void *xall = nullptr, *li = nullptr, *ld = nullptr, *pi = nullptr, *pd = nullptr;
    auto cleanup = [&]() {
        for (void *p : {xall, li, ld, pi, pd})
            if (p) (void)hipFree(p);
    };
    if (hipMalloc(&xall, xall_b) != hipSuccess || hipMalloc(&li, 4 * (size_t)n_tot * k) != hipSuccess ||
        hipMalloc(&ld, 4 * (size_t)n_tot * k) != hipSuccess || hipMalloc(&pi, 4 * part_b) != hipSuccess ||
        hipMalloc(&pd, 4 * part_b) != hipSuccess) {
        cleanup();
        set_error("mn_knn_sharded_f32: device allocation failed");
        return MN_ENOMEM;
    }
    int rc = MN_OK;
    do {
        // 1. all-gather of the shards (rank r's rows at r * n_local)
        if (ncclAllGather(X_shard, xall, (size_t)n_local * d, ncclFloat32, c, s) != ncclSuccess) {
            set_error("ncclAllGather of the query rows failed");
            rc = MN_EHIP;
            break;
        }
        // 2. exact per-shard top-k of every query against this rank's shard
        mn_knn_opts o = *opts;
        o.stream = s;
        const int64_t qc = query_chunk > 0 ? query_chunk : ((int64_t)1 << 21);
        for (int64_t a = 0; a < n_tot && rc == MN_OK; a += qc) {
            const int64_t b = std::min(n_tot, a + qc);
            rc = mn_knn_f32_qc((const float *)xall + a * d, b - a, X_shard, n_local, d, a,
                               (int64_t)rank * n_local, &o, (int32_t *)li + a * k,
                               (float *)ld + a * k);
        }
        if (rc != MN_OK) break;
        // 3. the lists of rank r's queries go to rank r; part p of the receive
        //    buffer = the lists computed on rank p
        if (ncclGroupStart() != ncclSuccess) { rc = MN_EHIP; break; }
        for (int p = 0; p < world && rc == MN_OK; ++p) {
            const size_t cnt = (size_t)n_local * k;
            if (ncclSend((const int32_t *)li + (size_t)p * cnt, cnt, ncclInt32, p, c, s) != ncclSuccess ||
                ncclSend((const float *)ld + (size_t)p * cnt, cnt, ncclFloat32, p, c, s) != ncclSuccess ||
                ncclRecv((int32_t *)pi + (size_t)p * cnt, cnt, ncclInt32, p, c, s) != ncclSuccess ||
                ncclRecv((float *)pd + (size_t)p * cnt, cnt, ncclFloat32, p, c, s) != ncclSuccess)
                rc = MN_EHIP;
        }
        if (ncclGroupEnd() != ncclSuccess || rc != MN_OK) {
            set_error("grouped ncclSend/ncclRecv of the per-shard lists failed");
            rc = MN_EHIP;
            break;
        }
        // 4. merge the R exact lists of this rank's queries
        rc = mn_knn_merge_f32((const int32_t *)pi, (const float *)pd, world, n_local, k, out_idx,
                              out_dist, s);
    } while (0);
    if (hipStreamSynchronize(s) != hipSuccess && rc == MN_OK) rc = MN_EHIP;
    cleanup();
    return rc;
}

}  // extern "C"
