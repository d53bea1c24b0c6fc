// Host-side AddressSanitizer / UBSan run of the C ABI (GPU kernels are not instrumented: only
// -Xarch_host gets -fsanitize).  Exercises every export on small shapes, including the error paths,
// and checks a few invariants (fused build == GaussPyInit + GenerateDoG by checksum, downloads
// agree with each other).  Build + run on the GPU box:  make -C tools/asan run
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gdp.h"

static int failures = 0;
#define EXPECT(cond)                                                                  \
    do {                                                                              \
        if (!(cond)) {                                                                \
            std::fprintf(stderr, "%s:%d: expectation failed: %s\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                               \
        }                                                                             \
    } while (0)
#define OK(call) EXPECT((call) == GDP_OK)

static void exercise(int H, int W, int S, int O, int B, int r0, int r1) {
    gdp_ctx* c = nullptr;
    const bool band = r1 > r0;
    OK(band ? gdp_create_band(&c, H, W, S, O, B, r0, r1, 0) : gdp_create(&c, H, W, S, O, B, 0));
    if (!c) return;
    int gh, gw, gs, go, gb, rows, cols0, first0;
    OK(gdp_get_geometry(c, &gh, &gw, &gs, &go, &gb));
    OK(gdp_level_dims(c, 0, &rows, &cols0, &first0)); // input rows held = octave-0 rows
    std::vector<int32_t> img((size_t)rows * W);
    for (size_t i = 0; i < img.size(); ++i) img[i] = (int32_t)((i * 2654435761u) >> 24);
    std::vector<const int32_t*> rowp(rows);
    for (int r = 0; r < rows; ++r) rowp[r] = img.data() + (size_t)r * W;
    for (int b = 0; b < gb; ++b) {
        OK(gdp_set_input_host(c, b, img.data(), (size_t)W, nullptr));
        OK(gdp_set_input_rows(c, b, rowp.data(), nullptr));
    }
    OK(gdp_build(c, nullptr));
    OK(gdp_sync(c));
    uint64_t built = 0, again = 0;
    OK(gdp_checksum(c, 0, &built));
    OK(gdp_init(c, nullptr));
    OK(gdp_generate_dog(c, nullptr));
    OK(gdp_checksum(c, 0, &again));
    EXPECT(built == again);
    OK(gdp_dog_range(c, 0, go, nullptr));
    EXPECT(gdp_dog_range(c, 1, 1, nullptr) == GDP_ERR_ARG);
    OK(gdp_build_subset(c, nullptr));  // GenerateDoG_nomp_dynamic fused, then in place
    OK(gdp_generate_dog_subset(c, nullptr));
    OK(gdp_sync(c));
    for (int o = 0; o < go; ++o) {
        int lr, lc, first;
        OK(gdp_level_dims(c, o, &lr, &lc, &first));
        std::vector<float> dense((size_t)lr * lc + 1), range((size_t)lr * lc + 1);
        std::vector<std::vector<float>> rws(lr, std::vector<float>(lc));
        std::vector<float*> rp(lr);
        for (int r = 0; r < lr; ++r) rp[r] = rws[r].data();
        for (int s = 0; s < gs + 3; ++s) {
            OK(gdp_download_level(c, 0, o, s, dense.data()));
            OK(gdp_download_level_rows(c, 0, o, s, rp.data()));
            OK(gdp_download_level_range(c, 0, o, s, 0, lr, range.data()));
            for (int r = 0; r < lr; ++r) {
                EXPECT(std::memcmp(rws[r].data(), dense.data() + (size_t)r * lc, (size_t)lc * 4) == 0);
                EXPECT(std::memcmp(range.data() + (size_t)r * lc, dense.data() + (size_t)r * lc, (size_t)lc * 4) == 0);
            }
            EXPECT(gdp_download_level_range(c, 0, o, s, lr, 1, range.data()) != GDP_OK);
        }
        OK(gdp_gauss_octave(c, o, nullptr));
        OK(gdp_dog_octave(c, o, nullptr));
    }
    std::vector<float> packed(gdp_packed_floats(c));
    OK(gdp_download_pyramid(c, 0, packed.data()));
    OK(gdp_upload_pyramid(c, 0, packed.data()));
    {  // round 4: host -> device state (two-way GaussPy) — raw, row-pointer and per-level uploads
        uint64_t before = 0, after = 0;
        OK(gdp_checksum(c, 0, &before));
        std::vector<float> raw(gdp_image_floats(c));
        OK(gdp_download_image_raw(c, 0, raw.data()));
        OK(gdp_upload_image_raw(c, 0, raw.data()));
        std::vector<std::vector<std::vector<float>>> rows_store(go);
        std::vector<std::vector<float*>> rowp(go * (gs + 3));
        std::vector<float**> lev(go * (gs + 3));
        std::vector<float***> oct(go);
        for (int o = 0; o < go; ++o) {
            int lr, lc, first;
            OK(gdp_level_dims(c, o, &lr, &lc, &first));
            for (int s = 0; s < gs + 3; ++s) {
                std::vector<float*>& rp = rowp[o * (gs + 3) + s];
                rows_store[o].emplace_back((size_t)lr * lc + 1);
                for (int r = 0; r < lr; ++r) rp.push_back(rows_store[o].back().data() + (size_t)r * lc);
                if (rp.empty()) rp.push_back(rows_store[o].back().data());
                lev[o * (gs + 3) + s] = rp.data();
            }
            oct[o] = lev.data() + o * (gs + 3);
        }
        OK(gdp_download_pyramid_rows(c, 0, oct.data()));
        OK(gdp_upload_pyramid_rows(c, 0, (const float* const* const* const*)oct.data()));
        for (int o = 0; o < go; ++o)
            for (int s = 0; s < gs + 3; ++s) {
                OK(gdp_upload_level(c, 0, o, s, rows_store[o][s].data()));
                OK(gdp_upload_level_rows(c, 0, o, s, rowp[o * (gs + 3) + s].data()));
            }
        OK(gdp_checksum(c, 0, &after));
        EXPECT(before == after);
        EXPECT(gdp_upload_level(c, 0, go, 0, raw.data()) == GDP_ERR_ARG);
        OK(gdp_gauss_scales(c, 1, 2, 0, go, nullptr));
        EXPECT(gdp_gauss_scales(c, 2, 2, 0, go, nullptr) == GDP_ERR_ARG);
        // round 5: the pipelined mirrored GenerateDoG (pageable and pinned host buffers) == the
        // serial upload + in-place pass + download
        OK(gdp_download_image_raw(c, 0, raw.data()));
        std::vector<float> piped(raw);
        OK(gdp_generate_dog_mirrored(c, 0, piped.data()));
        OK(gdp_upload_image_raw(c, 0, raw.data()));
        OK(gdp_generate_dog(c, nullptr));
        std::vector<float> serial(raw.size());
        OK(gdp_download_image_raw(c, 0, serial.data()));
        for (int o = 0; o < go; ++o)
            for (int s = 0; s < gs + 3; ++s) {
                int lr, lc, first;
                OK(gdp_level_dims(c, o, &lr, &lc, &first));
                const size_t off = gdp_level_offset(c, 0, o, s);
                EXPECT(std::memcmp(piped.data() + off, serial.data() + off, (size_t)lr * lc * 4) == 0);
            }
        void* pinned = nullptr;
        OK(gdp_host_alloc(raw.size() * 4, &pinned));
        std::memcpy(pinned, raw.data(), raw.size() * 4);
        OK(gdp_generate_dog_mirrored(c, 0, static_cast<float*>(pinned)));
        EXPECT(gdp_host_track(pinned, raw.size() * 4) == GDP_ERR_STATE);  // registered memory refused
        gdp_host_free(pinned);
        // round 6: the write-tracked mirror (aliased registered + protected views, SIGSEGV handler)
        void* tv = nullptr;
        if (gdp_host_alloc_tracked(raw.size() * 4, &tv) == GDP_OK) {
            float* t = static_cast<float*>(tv);
            size_t wb = 7;
            OK(gdp_download_image_raw(c, 0, t));
            EXPECT(gdp_host_written_bytes(t, &wb) == GDP_ERR_STATE);
            OK(gdp_host_arm(t));
            OK(gdp_host_written_bytes(t, &wb));
            EXPECT(wb == 0);
            t[3] = -2.5f;  // a write through the protected view: recorded, and it lands
            OK(gdp_host_written_bytes(t, &wb));
            EXPECT(wb > 0 && t[3] == -2.5f);
            OK(gdp_generate_dog_mirrored_written(c, 0, t));
            OK(gdp_host_written_bytes(t, &wb));
            EXPECT(wb == 0);
            t[raw.size() - 1] = 1.0f;
            OK(gdp_upload_image_written(c, 0, t));
            OK(gdp_host_untrack(t));
            t[0] = 2.0f;  // writable, not recorded
            OK(gdp_host_track(t, raw.size() * 4));  // tracking back on (not armed)
            OK(gdp_upload_image_written(c, 0, t));  // not armed: the whole mirror, then armed
            OK(gdp_host_written_bytes(t, &wb));
            // the deferred download: pages fetched on touch (a helper thread's copies), a write
            // recorded, completion by gdp_host_fetch / a whole download / gdp_destroy's settle
            OK(gdp_generate_dog(c, nullptr));
            OK(gdp_host_defer(c, 0, t));
            size_t st = 0, fb = 0;
            uint64_t nf = 0;
            OK(gdp_host_deferred_stats(t, &st, &fb, &nf));
            EXPECT(st >= raw.size() * 4 && fb == 0 && nf == 0);
            std::vector<float> dev(raw.size());
            OK(gdp_download_image_raw(c, 0, dev.data()));
            EXPECT(t[raw.size() / 2] == dev[raw.size() / 2] || (t[raw.size() / 2] != t[raw.size() / 2]));
            t[1] = 4.0f;
            dev[1] = 4.0f;
            OK(gdp_host_written_bytes(t, &wb));
            EXPECT(wb > 0);
            OK(gdp_host_fetch(t));
            OK(gdp_host_deferred_stats(t, &st, &fb, &nf));
            EXPECT(st == 0 && nf > 0);
            EXPECT(std::memcmp(t, dev.data(), raw.size() * 4) == 0);
            OK(gdp_upload_image_written(c, 0, t));
            OK(gdp_host_defer(c, 0, t));
            {  // a sequential read of the whole mirror: growing blocks, read-ahead, tripwires
                double sum = 0;
                for (size_t i = 0; i < raw.size(); ++i) sum += t[i];
                OK(gdp_host_deferred_stats(t, &st, &fb, &nf));
                EXPECT(st == 0 && nf > 0 && sum == sum);
                OK(gdp_download_image_raw(c, 0, dev.data()));
                EXPECT(std::memcmp(t, dev.data(), raw.size() * 4) == 0);
            }
            OK(gdp_host_defer(c, 0, t));
            OK(gdp_download_image_raw(c, 0, t));  // ends the deferral
            OK(gdp_host_deferred_stats(t, &st, nullptr, nullptr));
            EXPECT(st == 0);
            OK(gdp_host_defer(c, 0, t));
            EXPECT(gdp_host_deferred_stats(nullptr, &st, nullptr, nullptr) == GDP_ERR_ARG);
            EXPECT(gdp_host_fetch(nullptr) == GDP_ERR_ARG);
            gdp_host_free(tv);  // freed while deferred
        }
        EXPECT(gdp_generate_dog_mirrored(c, 1 << 20, raw.data()) == GDP_ERR_ARG);
        EXPECT(gdp_generate_dog_mirrored(c, 0, nullptr) == GDP_ERR_ARG);
        int ids[64];
        EXPECT(gdp_build_variants(ids, 64) == gdp_build_variants(nullptr, 0));
    }
    OK(gdp_gauss_range(c, 0, go, nullptr));
    // tuning: every key, valid and invalid values
    for (int key = 1; key <= 11; ++key) {
        int v = -1;
        if (gdp_get_tuning(c, key, &v) == GDP_OK) OK(gdp_set_tuning(c, key, v));
    }
    EXPECT(gdp_set_tuning(c, GDP_TUNE_VARIANT, 99) != GDP_OK);
    EXPECT(gdp_set_tuning(c, GDP_TUNE_CONV_ROWS, 7) != GDP_OK);
    EXPECT(gdp_set_tuning(c, 12345, 0) != GDP_OK);
    {  // every variant the library holds, and a removed id refused
        int ids[64];
        const int nv = gdp_build_variants(ids, 64);
        for (int i = 0; i < nv && i < 64; ++i) OK(gdp_set_tuning(c, GDP_TUNE_VARIANT, ids[i]));
        EXPECT(gdp_set_tuning(c, GDP_TUNE_VARIANT, 1) == GDP_ERR_ARG);
    }
    int bv = -1, bo = -1;
    float bms = 0;
    OK(gdp_autotune(c, 1, nullptr, &bv, &bo, &bms));
    float ms = 0;
    OK(gdp_time_builds(c, 2, nullptr, &ms));
    if (!band) {
        OK(gdp_build_gaussian(c, nullptr));
        OK(gdp_set_tuning(c, GDP_TUNE_CONV_KERNEL, 1));
        OK(gdp_build_gaussian(c, nullptr));
    } else {  // row band: the convolution needs its halo rows first
        int above = -1, below = -1;
        OK(gdp_conv_halo_rows(c, &above, &below));
        EXPECT(above >= 0 && below >= 0 && above + below > 0);
        EXPECT(gdp_build_gaussian(c, nullptr) != GDP_OK);
        void* h[2] = {nullptr, nullptr};
        size_t hp = 0;
        for (int side = 0; side < 2; ++side) OK(gdp_input_halo(c, side, &h[side], &hp));
        EXPECT(hp >= (size_t)W && (h[0] != nullptr) == (above > 0) && (h[1] != nullptr) == (below > 0));
        for (int side = 0; side < 2; ++side) {  // asking again returns the same binding (no re-upload)
            void* again = nullptr;
            size_t hp2 = 0;
            OK(gdp_input_halo(c, side, &again, &hp2));
            EXPECT(again == h[side] && hp2 == hp);
        }
        EXPECT(gdp_input_halo(c, 2, &h[0], &hp) != GDP_OK);
        EXPECT(gdp_bind_input_halo(c, h[0], h[1], (size_t)W + 1, 0) != GDP_OK || above + below == 0);  // pitch % 4
        const void* in = nullptr;
        size_t ip = 0;
        OK(gdp_device_input(c, 0, &in, &ip));
        EXPECT(in != nullptr && ip >= (size_t)W);
        EXPECT(gdp_device_input(c, B, &in, &ip) != GDP_OK);
        if (W % (1 << (go + 1)) == 0)
            OK(gdp_build_gaussian(c, nullptr));  // every octave width a multiple of 4
        else
            EXPECT(gdp_build_gaussian(c, nullptr) != GDP_OK);
    }
    OK(gdp_fill_synthetic(c, 0x5EED, 3, nullptr));
    OK(gdp_set_input_format(c, GDP_INPUT_U8));
    std::vector<uint8_t> u8((size_t)rows * W, 7);
    OK(gdp_set_input_host_u8(c, 0, u8.data(), (size_t)W, nullptr));
    OK(gdp_build(c, nullptr));
    // both window centres (one device table each, built on first use) and the row windows of every
    // octave read back through the layout in use ([row][scale] for non-square images)
    std::vector<float> tap((size_t)std::max(H, W)), tap2((size_t)std::max(H, W));
    OK(gdp_get_taps(c, 0, 0, 0, tap.data()));
    EXPECT(gdp_get_taps(c, 2, 0, 0, tap.data()) != GDP_OK);
    for (int o = 0; o < go; ++o)
        for (int sc = 0; sc < S + 3; ++sc) OK(gdp_get_taps(c, 1, o, sc, tap.data()));
    OK(gdp_get_taps(c, 1, 0, S + 2, tap.data()));
    for (int rep = 0; rep < 3; ++rep) {
        OK(gdp_set_window_centre(c, GDP_CENTRE_INTLEN));
        EXPECT(gdp_get_window_centre(c) == GDP_CENTRE_INTLEN);
        OK(gdp_build(c, nullptr));
        OK(gdp_set_window_centre(c, GDP_CENTRE_SERIAL));
    }
    OK(gdp_get_taps(c, 1, 0, S + 2, tap2.data()));
    EXPECT(std::memcmp(tap.data(), tap2.data(), sizeof(float) * (size_t)H) == 0);  // back to the serial table
    EXPECT(gdp_set_window_centre(c, 7) != GDP_OK);
    // block tiles refuse a (rows, waves) pair with no kernel instance
    OK(gdp_set_tuning(c, GDP_TUNE_CONV_KERNEL, 2));
    OK(gdp_set_tuning(c, GDP_TUNE_CONV_ROWS, 48));
    OK(gdp_set_tuning(c, GDP_TUNE_CONV_WAVES, 8));
    if (!band) EXPECT(gdp_build_gaussian(c, nullptr) == GDP_ERR_STATE);
    OK(gdp_set_tuning(c, GDP_TUNE_CONV_WAVES, 16));
    OK(gdp_set_tuning(c, GDP_TUNE_CONV_ROWS, 32));
    EXPECT(gdp_device_level(c, 0, go, 0) == nullptr);
    OK(gdp_sync(c));
    gdp_destroy(c);
}

int main() {
    std::setvbuf(stdout, nullptr, _IONBF, 0);
    EXPECT(gdp_device_count() >= 1);
    exercise(96, 160, 2, 0, 1, 0, 0);
    exercise(100, 37, 3, 0, 2, 0, 0);
    exercise(7, 5, 0, 0, 1, 0, 0);
    exercise(256, 300, 2, 5, 1, 16, 48);
    exercise(512, 256, 2, 5, 2, 128, 256);
    exercise(1080, 1920, 2, 5, 1, 0, 0);
    gdp_ctx* c = nullptr;
    EXPECT(gdp_create(&c, 0, 10, 2, 0, 1, 0) != GDP_OK);
    EXPECT(gdp_create(&c, 10, 10, 2, 9, 1, 0) != GDP_OK);
    EXPECT(gdp_create_band(&c, 64, 64, 2, 5, 1, 3, 40, 0) != GDP_OK);
    gdp_destroy(nullptr);
    std::printf(failures ? "asan driver: %d failures\n" : "asan driver: ok\n", failures);
    return failures ? 1 : 0;
}
