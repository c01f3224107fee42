// Host-staging probe: how fast can a pageable (malloc'd) host buffer go H2D and come back D2H?
// The reference's contract starts and ends in pageable host memory (its harness mallocs the send
// and recv buffers), so the drop-in path's end-to-end rate is set by these copies.
//
//   seq        one hipMemcpyAsync H2D of the whole buffer, then one D2H (what a single-window call does)
//   conc2      the same two copies issued at once from two host threads, on two streams
//   win2       the buffer in windows: one thread streams the H2D windows, another the D2H windows
//   bounce_T   our own staging: T host threads copy pageable <-> a ring of pinned windows while the
//              DMA engines move the pinned windows, both directions at once
//   pinned2    reference: both directions at once from pinned memory
//   register   hipHostRegister + hipHostUnregister of the whole buffer
//
// Prints one JSON line.  Build: hipcc -O3 -std=c++17 -pthread -o host_stage_probe host_stage_probe.cpp
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

using clk = std::chrono::steady_clock;
static double ms_since(clk::time_point t0) {
    return std::chrono::duration<double, std::milli>(clk::now() - t0).count();
}

// parallel memcpy over T threads (each takes a contiguous share)
static void pcopy(void* dst, const void* src, size_t bytes, int T, std::vector<std::thread>& pool) {
    pool.clear();
    const size_t share = ((bytes + T - 1) / T + 4095) & ~(size_t)4095;
    for (int t = 0; t < T; ++t) {
        const size_t off = (size_t)t * share;
        if (off >= bytes) break;
        const size_t nb = std::min(share, bytes - off);
        pool.emplace_back([=] { std::memcpy((char*)dst + off, (const char*)src + off, nb); });
    }
    for (auto& th : pool) th.join();
}

int main(int argc, char** argv) {
    const size_t bytes = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1024) << 20;
    const size_t win = (argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 32) << 20;
    const int reps = 3;
    CK(hipSetDevice(0));
    char* hs = (char*)std::malloc(bytes);
    char* hr = (char*)std::malloc(bytes);
    std::memset(hs, 1, bytes);
    std::memset(hr, 0, bytes);
    char *ds, *dr;
    CK(hipMalloc(&ds, bytes));
    CK(hipMalloc(&dr, bytes));
    CK(hipMemset(dr, 2, bytes));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    CK(hipDeviceSynchronize());
    std::string out = "{\"bytes\": " + std::to_string(bytes) + ", \"window\": " + std::to_string(win);
    auto row = [&](const char* name, double ms) {
        char b[160];
        std::snprintf(b, sizeof b, ", \"%s_ms\": %.2f", name, ms);
        out += b;
        std::fprintf(stderr, "%-12s %8.2f ms  %6.1f GB/s per direction\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    };
    auto best = [&](auto fn) {
        fn();  // warm
        double m = 1e30;
        for (int r = 0; r < reps; ++r) {
            auto t0 = clk::now();
            fn();
            m = std::min(m, ms_since(t0));
        }
        return m;
    };

    row("seq", best([&] {
            CK(hipMemcpyAsync(ds, hs, bytes, hipMemcpyHostToDevice, s1));
            CK(hipStreamSynchronize(s1));
            CK(hipMemcpyAsync(hr, dr, bytes, hipMemcpyDeviceToHost, s1));
            CK(hipStreamSynchronize(s1));
        }));
    row("conc2", best([&] {
            std::thread a([&] {
                CK(hipMemcpyAsync(ds, hs, bytes, hipMemcpyHostToDevice, s1));
                CK(hipStreamSynchronize(s1));
            });
            std::thread b([&] {
                CK(hipMemcpyAsync(hr, dr, bytes, hipMemcpyDeviceToHost, s2));
                CK(hipStreamSynchronize(s2));
            });
            a.join();
            b.join();
        }));
    row("win2", best([&] {
            std::thread a([&] {
                for (size_t o = 0; o < bytes; o += win)
                    CK(hipMemcpyAsync(ds + o, hs + o, std::min(win, bytes - o), hipMemcpyHostToDevice, s1));
                CK(hipStreamSynchronize(s1));
            });
            std::thread b([&] {
                for (size_t o = 0; o < bytes; o += win)
                    CK(hipMemcpyAsync(hr + o, dr + o, std::min(win, bytes - o), hipMemcpyDeviceToHost, s2));
                CK(hipStreamSynchronize(s2));
            });
            a.join();
            b.join();
        }));

    // own bounce ring: NB pinned windows per direction
    const int NB = 4;
    char *pin_in[NB], *pin_out[NB];
    hipEvent_t ev_in[NB], ev_out[NB];
    for (int i = 0; i < NB; ++i) {
        CK(hipHostMalloc(&pin_in[i], win, hipHostMallocDefault));
        CK(hipHostMalloc(&pin_out[i], win, hipHostMallocDefault));
        CK(hipEventCreateWithFlags(&ev_in[i], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&ev_out[i], hipEventDisableTiming));
    }
    for (int T : {1, 2, 4, 8, 16}) {
        auto fn = [&] {
            const size_t nw = (bytes + win - 1) / win;
            std::thread a([&] {  // H2D: copy into pinned slot, DMA it
                std::vector<std::thread> pool;
                for (size_t j = 0; j < nw; ++j) {
                    const int i = (int)(j % NB);
                    const size_t o = j * win, nb = std::min(win, bytes - o);
                    if (j >= (size_t)NB) CK(hipEventSynchronize(ev_in[i]));
                    pcopy(pin_in[i], hs + o, nb, T, pool);
                    CK(hipMemcpyAsync(ds + o, pin_in[i], nb, hipMemcpyHostToDevice, s1));
                    CK(hipEventRecord(ev_in[i], s1));
                }
                CK(hipStreamSynchronize(s1));
            });
            std::thread b([&] {  // D2H: DMA into pinned slot ahead, copy out when it lands
                std::vector<std::thread> pool;
                size_t issued = 0;
                for (size_t j = 0; j < nw; ++j) {
                    while (issued < nw && issued < j + NB) {
                        const int i = (int)(issued % NB);
                        const size_t o = issued * win, nb = std::min(win, bytes - o);
                        CK(hipMemcpyAsync(pin_out[i], dr + o, nb, hipMemcpyDeviceToHost, s2));
                        CK(hipEventRecord(ev_out[i], s2));
                        ++issued;
                    }
                    const int i = (int)(j % NB);
                    const size_t o = j * win, nb = std::min(win, bytes - o);
                    CK(hipEventSynchronize(ev_out[i]));
                    pcopy(hr + o, pin_out[i], nb, T, pool);
                }
            });
            a.join();
            b.join();
        };
        row(("bounce_" + std::to_string(T)).c_str(), best(fn));
    }
    // correctness of the last bounce round trip: hr must equal dr's fill (2)
    bool ok = true;
    for (size_t o = 0; o < bytes; o += 4099) ok &= hr[o] == 2;
    // host memcpy alone (pageable -> pageable), T threads, for scale
    for (int T : {1, 4, 16}) {
        std::vector<std::thread> pool;
        row(("memcpy_" + std::to_string(T)).c_str(), best([&] { pcopy(hr, hs, bytes, T, pool); }));
    }
    {
        char *ps, *pr;
        CK(hipHostMalloc(&ps, bytes, hipHostMallocDefault));
        CK(hipHostMalloc(&pr, bytes, hipHostMallocDefault));
        std::memset(ps, 1, bytes);
        row("pinned_seq", best([&] {
                CK(hipMemcpyAsync(ds, ps, bytes, hipMemcpyHostToDevice, s1));
                CK(hipMemcpyAsync(pr, dr, bytes, hipMemcpyDeviceToHost, s1));
                CK(hipStreamSynchronize(s1));
            }));
        row("pinned2", best([&] {
                CK(hipMemcpyAsync(ds, ps, bytes, hipMemcpyHostToDevice, s1));
                CK(hipMemcpyAsync(pr, dr, bytes, hipMemcpyDeviceToHost, s2));
                CK(hipStreamSynchronize(s1));
                CK(hipStreamSynchronize(s2));
            }));
        CK(hipHostFree(ps));
        CK(hipHostFree(pr));
    }
    row("register", best([&] {
            CK(hipHostRegister(hs, bytes, hipHostRegisterDefault));
            CK(hipHostUnregister(hs));
        }));
    out += std::string(", \"ok\": ") + (ok ? "true" : "false") + "}";
    std::printf("%s\n", out.c_str());
    return ok ? 0 : 1;
}
