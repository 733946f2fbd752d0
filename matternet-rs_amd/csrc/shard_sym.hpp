// shard_sym.hpp — stages of the row-sharded symmetric kNN build (knn_f32.hip
// section 6), driven by shard.hip over RCCL or simulated on one device.
#pragma once
#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>

#include "common.hpp"
#include "matternet_hip.h"

namespace mn {

// ranks of one sharded build (the merge width of k_merge_certify / mn_knn_merge_f32)
constexpr int kMaxShardRanks = 16;

struct ShardPlan {
    int64_t N, m0;  // all rows; the global phase-1 sample
    int d, dp, nkb, k, L1, world;
    bool ok;        // the symmetric form applies (else the per-shard path)
};

constexpr int kShardKMax = 64;  // k limit of the candidate generators (knn::KMAX)

// The plan of an N-row build over `world` ranks (host only): the global
// phase-1 sample m0 (the first N / 24 rows of the golden-ratio order, whole
// 256-row panels) and whether the symmetric form applies (as knn_x1: a corpus
// well past the sample; the sweep's grid and int32 ids bound N).
inline ShardPlan shard_plan(int64_t N, int d, int k, int world) {
    ShardPlan p{};
    p.N = N;
    p.d = d;
    p.dp = (d + 255) / 256 * 256;
    p.nkb = p.dp / 32;
    p.k = k;
    p.world = world;
    p.L1 = std::min(std::max((3 * k + 3) / 8, 12), 48);
    const char *fs = knob("MN_SH_SAMPLE_DIV");  // tuning build: sample = N / div
    const int64_t div = (fs && *fs) ? std::max(2, atoi(fs)) : 24;
    p.m0 = std::max<int64_t>(N / div, (int64_t)64 * p.L1);
    p.m0 = (p.m0 + 255) / 256 * 256;
    p.ok = k >= 1 && k <= kShardKMax && d >= 1 && p.m0 + 4 * 256 <= N && N * 32 < INT_MAX &&
           world >= 1 && world <= kMaxShardRanks;
    return p;
}

// Stage A: tau0_o / qn_o [nl] of rows [row0, row0 + nl) of X_all.  1: the
// symmetric form does not apply (values too large for the bf16 bound).
int shard_phase1(const float *X_all, const ShardPlan &pl, int64_t row0, int64_t nl, hipStream_t s,
                 float *tau0_o, float *qn_o);

// Stage B: this rank's share of the sweep; pidx / pdist [N][k] partial lists
// (global ids), tc_all [N] the rows' certificate thresholds.  1: a non-finite
// threshold (the per-shard path).  n_cand (may be NULL): buffered candidates.
int shard_share(const float *X_all, const ShardPlan &pl, const float *tau0_all,
                const float *qn_all, int rank, int world, hipStream_t s, int32_t *pidx,
                float *pdist, float *tc_all, int64_t *n_cand);

// Stage C: merge + certify the owner's rows [row0, row0 + nl) from `parts`
// partial lists (part p row q at p * part_stride + q * k), exact scan of the
// rest; out_idx / out_dist [nl][k].
int shard_finish(const float *X_all, const ShardPlan &pl, int64_t row0, int64_t nl, int parts,
                 int64_t part_stride, const int32_t *pidx, const float *pdist, const float *tc_all,
                 hipStream_t s, int32_t *out_idx, float *out_dist, int *n_fallback);

// the calling thread's mn_knn_last_stats record
mn_knn_stats &knn_stats_ref();

}  // namespace mn
