// Serving independent single images from several host threads through the C ABI:
// every thread owns its contexts (each with its own stream, gdp_create on the shared device) and
// builds the pyramid of its own synthetic image `iters` times, rotating over `sets` contexts of that
// image so the job's working set (>= 5 x 514 MB at 4096^2 by default) is far beyond the 256 MB
// Infinity Cache and every rate is an HBM rate, as in bench.py; the threads start together, so
// their launches overlap on the GPU.  Afterwards one context rebuilds every thread's image alone and the
// checksums must agree bit for bit (nothing is shared between contexts).  Plain C++ over
// libgdp.so, no HIP headers:
//   serve_threads <n> <threads> <iters> [sets per thread]     ->  one JSON line
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gdp.h"

namespace {
constexpr uint32_t kSeed = 0x5EED;  // bench.py's synthetic images (first_image = thread id)

struct Gate {  // all threads start their timed builds together
    std::mutex m;
    std::condition_variable cv;
    int waiting = 0, total = 0;
    bool open = false;
    void arrive_and_wait() {
        std::unique_lock<std::mutex> lk(m);
        if (++waiting == total) {
            open = true;
            cv.notify_all();
        }
        cv.wait(lk, [&] { return open; });
    }
};

int check(int rc, gdp_ctx* c, const char* what) {
    if (rc != GDP_OK) std::fprintf(stderr, "serve_threads: %s: %s\n", what, gdp_last_error(c));
    return rc;
}
}  // namespace

int main(int argc, char** argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 4096;
    const int threads = argc > 2 ? std::atoi(argv[2]) : 4;
    const int iters = argc > 3 ? std::atoi(argv[3]) : 50;
    const int sets = argc > 4 ? std::atoi(argv[4]) : (5 + threads - 1) / threads;
    if (n < 16 || threads < 1 || threads > 64 || iters < 1 || sets < 1 || sets > 16) {
        std::fprintf(stderr, "usage: serve_threads <n >= 16> <threads 1..64> <iters >= 1> [sets 1..16]\n");
        return 2;
    }
    std::vector<uint64_t> sums(threads, 0);
    std::vector<int> status(threads, GDP_OK);
    std::vector<std::chrono::steady_clock::time_point> done(threads);
    Gate gate;
    gate.total = threads + 1;
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t) {
        pool.emplace_back([&, t] {
            std::vector<gdp_ctx*> cs(sets, nullptr);
            int rc = GDP_OK;
            for (int k = 0; k < sets && rc == GDP_OK; ++k) {
                rc = check(gdp_create(&cs[k], n, n, 2, 5, 1, 0), nullptr, "gdp_create");
                if (rc == GDP_OK) rc = check(gdp_fill_synthetic(cs[k], kSeed, t, nullptr), cs[k], "gdp_fill_synthetic");
                if (rc == GDP_OK) rc = check(gdp_build(cs[k], nullptr), cs[k], "gdp_build (warm)");
                if (rc == GDP_OK) rc = check(gdp_sync(cs[k]), cs[k], "gdp_sync");
            }
            gate.arrive_and_wait();  // (a thread that failed still arrives, so nobody waits forever)
            for (int k = 0; k < iters && rc == GDP_OK; ++k) rc = check(gdp_build(cs[k % sets], nullptr), cs[k % sets], "gdp_build");
            for (int k = 0; k < sets && rc == GDP_OK; ++k) rc = check(gdp_sync(cs[k]), cs[k], "gdp_sync");
            done[t] = std::chrono::steady_clock::now();  // the timed part ends when these streams drain
            if (rc == GDP_OK) rc = check(gdp_checksum(cs[(iters - 1) % sets], 0, &sums[t]), cs[(iters - 1) % sets], "gdp_checksum");
            status[t] = rc;
            for (gdp_ctx* c : cs) gdp_destroy(c);
        });
    }
    gate.arrive_and_wait();
    const auto t0 = std::chrono::steady_clock::now();
    for (std::thread& th : pool) th.join();
    for (int t = 0; t < threads; ++t)
        if (status[t] != GDP_OK) return 1;
    double wall = 0.0;  // start of the timed builds to the last thread's drained stream
    for (int t = 0; t < threads; ++t) wall = std::max(wall, std::chrono::duration<double>(done[t] - t0).count());
    // every thread's image rebuilt alone on one fresh context
    gdp_ctx* ref = nullptr;
    if (check(gdp_create(&ref, n, n, 2, 5, 1, 0), nullptr, "gdp_create (reference)") != GDP_OK) return 1;
    bool same = true;
    std::string sums_json;
    for (int t = 0; t < threads; ++t) {
        uint64_t want = 0;
        if (check(gdp_fill_synthetic(ref, kSeed, t, nullptr), ref, "fill") != GDP_OK ||
            check(gdp_build(ref, nullptr), ref, "build") != GDP_OK ||
            check(gdp_checksum(ref, 0, &want), ref, "checksum") != GDP_OK)
            return 1;
        same = same && want == sums[t];
        char buf[40];
        std::snprintf(buf, sizeof buf, "%s\"%016llx\"", t ? ", " : "", (unsigned long long)sums[t]);
        sums_json += buf;
    }
    const double bytes_per_image = 4.0 * n * n + (double)gdp_pyramid_bytes(ref);
    gdp_destroy(ref);
    const double images = (double)threads * iters;
    std::printf("{\"n\": %d, \"threads\": %d, \"sets_per_thread\": %d, \"iters\": %d, \"wall_s\": %.6f, \"ms_per_image\": %.6f, "
                "\"mpix_per_s\": %.1f, \"frac_of_8TBps\": %.4f, \"bit_identical_to_one_context\": %s, "
                "\"checksums\": [%s]}\n",
                n, threads, sets, iters, wall, wall * 1e3 / images, images * n * (double)n / wall / 1e6,
                images * bytes_per_image / wall / 8e12, same ? "true" : "false", sums_json.c_str());
    return same ? 0 : 1;
}
