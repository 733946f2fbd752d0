// Host-side coverage check of ksw2::sym_block_table (tests/test_sweep_table.py).
#include "gram_sweep2.hpp"
#include <cstdio>
#include <algorithm>
#include <vector>
int main() {
    int bad = 0;
    for (int nbk : {1, 2, 3, 5, 8, 13, 31, 32, 33, 100, 257, 1000, 3907}) {
        for (int order : {0, 1, 2}) {
            auto tab = mn::ksw2::sym_block_table(nbk, 256, order);
            std::vector<int> seen((size_t)nbk * nbk, 0);
            long tiles = 0;
            for (auto e : tab) {
                for (int t = 0; t < e.z; ++t) {
                    int J = e.y + t * e.w;
                    if (J < e.x || J >= nbk || e.x >= nbk) { bad++; continue; }
                    if (J == e.x && t != 0) bad++;
                    seen[(size_t)e.x * nbk + J]++;
                    tiles++;
                }
            }
            for (int I = 0; I < nbk; ++I)
                for (int J = I; J < nbk; ++J)
                    if (seen[(size_t)I * nbk + J] != 1) bad++;
            if (order == 2 && tab.size() % 8) bad++;
            if (nbk == 3907) printf("nbk %d order %d entries %zu tiles %ld\n", nbk, order, tab.size(), tiles);
        }
    }
    // rank shares of the order-2 table: together every tile exactly once,
    // each share a multiple of 8 entries, full-group tiles balanced
    for (int nbk : {1, 7, 33, 257, 1000, 3907}) {
        for (int world : {1, 2, 3, 8}) {
            std::vector<int> seen((size_t)nbk * nbk, 0);
            long tmin = -1, tmax = 0;
            for (int r = 0; r < world; ++r) {
                auto tab = mn::ksw2::sym_block_table_share(nbk, 256, r, world);
                if (tab.size() % 8) bad++;
                long tiles = 0;
                for (auto e : tab)
                    for (int t = 0; t < e.z; ++t) {
                        int J = e.y + t * e.w;
                        if (J < e.x || J >= nbk || e.x >= nbk) { bad++; continue; }
                        if (J == e.x && t != 0) bad++;
                        seen[(size_t)e.x * nbk + J]++;
                        tiles++;
                    }
                tmin = tmin < 0 ? tiles : std::min(tmin, tiles);
                tmax = std::max(tmax, tiles);
            }
            for (int I = 0; I < nbk; ++I)
                for (int J = I; J < nbk; ++J)
                    if (seen[(size_t)I * nbk + J] != 1) bad++;
            if (nbk == 3907) {
                printf("nbk %d world %d tiles per rank %ld..%ld\n", nbk, world, tmin, tmax);
                if (tmax > tmin + tmin / 50) bad++;  // within 2%
            }
        }
    }
    auto a = mn::ksw2::sym_block_table(1000, 256, 2);
    auto b = mn::ksw2::sym_block_table_share(1000, 256, 0, 1);
    if (a.size() != b.size()) bad++;
    printf("bad %d\n", bad);
    return bad != 0;
}
