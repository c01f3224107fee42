// Host check of the XCD-run workgroup map (csrc/reduce_common.hpp xcd_trip / xcd_full / xcd_trip_w):
// for many grid sizes, run lengths and odd-XCD handovers it must be a bijection from the active
// blocks onto [0, n), and every remapped block must land in a run owned by its XCD (block b runs on
// XCD b % 8) or, for an even XCD under a handover, by the odd XCD above it.  Built and run by
// tests/test_xcd_map_host.py.
#include <cstdio>
#include <vector>
#include "reduce_common.hpp"
int main() {
    int bad = 0;
    for (uint32_t n : {1u, 7u, 8u, 9u, 63u, 64u, 65u, 1000u, 4096u, 100003u})
        for (uint32_t cs = 0; cs <= 10; ++cs) {
            const uint32_t full = chr::xcd_full(n, cs), q = full >> 3;
            for (uint32_t hand : {0u, 1u, 2u, q >> 6, q >> 2, q >> 1, q}) {
                if (hand > q) continue;
                std::vector<int> hit(n, 0);
                const uint32_t grid = n + 8u * hand;
                for (uint32_t b = 0; b < grid; ++b) {
                    const size_t t = chr::xcd_trip_w(b, full, cs, hand);
                    if (t == chr::kIdleTrip) {
                        if (b >= full + 8u * hand || (b & 1u) == 0) ++bad;  // only odd XCDs idle, in the region
                        continue;
                    }
                    if (t >= n) { ++bad; continue; }
                    ++hit[t];
                    const uint32_t x = b % 8, owner = (uint32_t)((t >> cs) % 8);
                    if (b < full + 8u * hand && owner != x && !(hand && x % 2 == 0 && owner == x + 1)) ++bad;
                }
                for (uint32_t t = 0; t < n; ++t) bad += hit[t] != 1;
                if (hand == 0)  // the unweighted map itself
                    for (uint32_t b = 0; b < n; ++b) bad += chr::xcd_trip(b, full, cs) != chr::xcd_trip_w(b, full, cs, 0);
            }
        }
    // the policy: 1/64 of each XCD's share, none below 64 trips per XCD, off with shift 0
    bad += chr::xcd_hand(16384, -1) != 32 || chr::xcd_hand(256, -1) != 0 || chr::xcd_hand(16384, 0) != 0;
    std::printf("%d\n", bad);
    return bad != 0;
}
