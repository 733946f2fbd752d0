// Host-side planners of the kNN path under ASan / UBSan (tests/test_sanitizers.py):
// the symmetric block tables (every order and every rank share), the sweep and
// phase-1 Gram slicing / buffer sizing, and the sharded build's plan.  Every
// invariant the kernels index by is checked; "bad 0" on success.
#include <cstdio>
#include <vector>

#include "gram_bf16.hpp"
#include "gram_sweep2.hpp"
#include "shard_sym.hpp"

int main() {
    long bad = 0, cases = 0;
    using mn::ksw2::BC;
    // plan_sweep: S slices of `chunk` rows cover the sweep's corpus rows,
    // chunk a multiple of the 256-row tile, cap a multiple of 16 >= 64
    for (long nq : {1L, 255L, 256L, 257L, 40000L, 1000000L, 8000000L})
        for (long nc2 : {256L, 1000L, 65536L, 958333L, 7666667L})
            for (double ex : {1.0, 288.0, 5000.0}) {
                const auto p = mn::ksw2::plan_sweep(nq, nc2, ex);
                ++cases;
                if (p.S < 1 || p.chunk < BC || p.chunk % BC || p.S * p.chunk < nc2 ||
                    (p.S - 1) * p.chunk >= nc2 || p.cap < 64 || p.cap % 16)
                    ++bad;
                const long grid = (nq + 255) / 256 * p.S;
                if (grid <= 0) ++bad;
            }
    // plan_gram: slices cover the corpus, chunk a multiple of BN, the re-rank
    // width S * L within the 8-register budget, cap a multiple of 64
    for (long nq : {1L, 64L, 1000L, 1000000L})
        for (long nc : {1L, 100L, 41667L, 1000000L})
            for (int L : {4, 12, 16, 48})
                for (long mins : {1L, 8L})
                    for (long maxs : {0L, 1L}) {
                        const auto p = mn::kb16::plan_gram(nq, nc, L, mins, maxs);
                        ++cases;
                        if (p.S < 1 || p.chunk < mn::kb16::BN || p.chunk % mn::kb16::BN ||
                            p.S * p.chunk < nc || (maxs > 0 && p.S > maxs) || p.cap < 64 ||
                            p.cap % 64 || p.NR < 1 || p.NR > 8 || p.S * L > 8 * 64)
                            ++bad;
                    }
    // shard_plan: whole-panel sample inside the corpus when the symmetric
    // form applies; int32 ids
    for (long N : {1L, 1000L, 2048L, 150000L, 1000000L, 8000000L, 67108863L})
        for (int k : {1, 10, 32, 64, 65})
            for (int world : {1, 2, 3, 8, 16, 17}) {
                const auto p = mn::shard_plan(N, 768, k, world);
                ++cases;
                if (p.m0 % 256 || p.L1 < 12 || p.L1 > 48 || p.nkb * 32 != p.dp) ++bad;
                if (p.ok && (p.m0 + 1024 > N || k > 64 || world > 16 || N * 32 >= INT_MAX)) ++bad;
            }
    // block tables: every upper-triangle tile once over the ranks' shares
    for (int nbk : {1, 2, 9, 64, 257, 3907})
        for (int world : {1, 3, 8})
            for (int gr : {2, 4}) {
                std::vector<unsigned char> seen((size_t)nbk * nbk, 0);
                for (int r = 0; r < world; ++r) {
                    const auto tab = mn::ksw2::sym_block_table_share(nbk, 256, r, world, gr);
                    ++cases;
                    if (tab.size() % 8) ++bad;
                    for (const auto &e : tab)
                        for (int t = 0; t < e.z; ++t) {
                            const int J = e.y + t * e.w;
                            if (e.x < 0 || J < e.x || J >= nbk) { ++bad; continue; }
                            seen[(size_t)e.x * nbk + J]++;
                        }
                }
                for (int I = 0; I < nbk; ++I)
                    for (int J = I; J < nbk; ++J)
                        if (seen[(size_t)I * nbk + J] != 1) ++bad;
            }
    printf("cases %ld bad %ld\n", cases, bad);
    return bad ? 1 : 0;
}
