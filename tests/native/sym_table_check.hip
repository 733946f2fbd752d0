// Host-side coverage check of ksw2::sym_block_table (tests/test_sweep_table.py).
#include "gram_sweep2.hpp"
#include <cstdio>
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
    printf("bad %d\n", bad);
    return bad != 0;
}
