// Host check of the XCD-run workgroup map (csrc/reduce_common.hpp xcd_trip / xcd_full): for many
// grid sizes and run lengths it must be a bijection on [0, n), and every remapped block must land
// in a run owned by its XCD (block b runs on XCD b % 8).  Built and run by tests/test_xcd_map_host.py.
#include <cstdio>
#include <vector>
#include "reduce_common.hpp"
int main() {
    int bad = 0;
    for (uint32_t n : {1u, 7u, 8u, 9u, 63u, 64u, 65u, 1000u, 4096u, 100003u})
        for (uint32_t cs = 0; cs <= 10; ++cs) {
            std::vector<int> hit(n, 0);
            const uint32_t full = chr::xcd_full(n, cs);
            for (uint32_t b = 0; b < n; ++b) {
                size_t t = chr::xcd_trip(b, full, cs);
                if (t >= n) { ++bad; continue; }
                ++hit[t];
                if (b < full && (t >> cs) % 8 != b % 8) ++bad;  // run of XCD b % 8
            }
            for (uint32_t t = 0; t < n; ++t) bad += hit[t] != 1;
        }
    std::printf("%d\n", bad);
    return bad != 0;
}
