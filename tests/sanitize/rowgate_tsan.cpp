// rowgate_tsan.cpp -- TEST INFRASTRUCTURE (tests/test_sanitizers.py).  The
// host side of a pipelined run under ThreadSanitizer: a producer thread
// stands in for k_pipeline, filling each picture's MbRecords row by row and
// publishing the picture's row count with a release store (the kernel's
// system-scope release of h_progress[kRowsAt + k], hl_encoder.hip), while
// writer threads serialise the pictures with write_slice behind a RowGate
// whose wait acquires that count (hl_writer.h RowGate, the Gate of
// hl_encoder.hip encode_pictures).  The gated slices must equal slices
// written after the run, and TSan must see no race on the records.
//   rowgate_tsan [relaxed]   relaxed: the count published and read relaxed,
//                            a negative control TSan must flag
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../../hartallo_amd/csrc/hl_writer.h"

using namespace hl;

static bool g_relaxed = false;

struct Gate {
    const int32_t* rows;
    static bool wait(void* ctx, int r)
    {
        const Gate* g = (const Gate*)ctx;
        while ((g_relaxed ? __atomic_load_n(g->rows, __ATOMIC_RELAXED) : __atomic_load_n(g->rows, __ATOMIC_ACQUIRE)) <= r)
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        return true;
    }
};

// a syntactically valid macroblock of a P picture: P_Skip, P_L0_16x16 or
// P_8x8 with motion differences and luma / chroma levels
static void make_record(std::mt19937& rng, MbRecord& m)
{
    memset(&m, 0, sizeof(m));
    const int kind = (int)(rng() % 3);
    if (kind == 0) {
        m.e_type = ET_PSKIP;
        m.flags = FL_INTER | FL_SKIP;
        return;
    }
    m.flags = FL_INTER;
    m.pm0 = PM_L0;
    if (kind == 1) {
        m.e_type = ET_P16x16;
        m.mb_type = 0;
        m.num_part = 1;
        m.mvd[0][0][0] = (int16_t)((int)(rng() % 65) - 32);
        m.mvd[0][0][1] = (int16_t)((int)(rng() % 65) - 32);
    }
    else {
        m.e_type = ET_P8x8;
        m.mb_type = 3;
        m.num_part = 4;
        for (int p = 0; p < 4; ++p) {
            m.num_sub[p] = 1;
            m.mvd[p][0][0] = (int16_t)((int)(rng() % 17) - 8);
            m.mvd[p][0][1] = (int16_t)((int)(rng() % 17) - 8);
        }
    }
    m.cbp_l = (int)(rng() % 16);
    m.cbp_c = (int)(rng() % 3);
    m.cbp = m.cbp_l | (m.cbp_c << 4);
    for (int b = 0; b < 16; ++b) {
        if (!(m.cbp_l & (1 << (b >> 2)))) continue;
        for (int i = 0; i < 16; ++i)
            if (rng() % 4 == 0) m.luma[b][i] = (int16_t)((int)(rng() % 9) - 4);
        m.nc_luma[b] = (int8_t)(rng() % 9);
    }
    if (m.cbp_c) {
        for (int c = 0; c < 2; ++c) {
            m.cbp_cdc[c] = 1;
            m.cdc[c][0] = (int16_t)((int)(rng() % 5) - 2);
        }
        if (m.cbp_c & 2)
            for (int c = 0; c < 2; ++c)
                for (int b = 0; b < 4; ++b) {
                    m.cbp_cac[c] |= 1 << b;
                    m.cac[c][b][0] = 1;
                    m.nc_cac[c][b] = (int8_t)(rng() % 5);
                }
    }
}

int main(int argc, char** argv)
{
    g_relaxed = argc > 1 && !strcmp(argv[1], "relaxed");
    const StreamParams sp{352, 288, 28, 1, 1};
    const int mbw = sp.width / 16, mbh = sp.height / 16, nmb = mbw * mbh, m = 6, nwriters = 4;
    std::vector<MbRecord> recs((size_t)m * nmb);
    std::vector<int32_t> rows(m, 0);
    std::vector<std::vector<uint8_t>> gated(m), after(m);
    std::thread producer([&] {
        std::mt19937 rng(7);
        for (int k = 0; k < m; ++k)
            for (int y = 0; y < mbh; ++y) {
                for (int x = 0; x < mbw; ++x) make_record(rng, recs[(size_t)k * nmb + y * mbw + x]);
                if (g_relaxed) __atomic_store_n(&rows[k], y + 1, __ATOMIC_RELAXED);
                else __atomic_store_n(&rows[k], y + 1, __ATOMIC_RELEASE);
                std::this_thread::sleep_for(std::chrono::microseconds(50));
            }
    });
    std::atomic<int> next{0};
    auto work = [&] {
        std::vector<uint8_t> scratch(slice_scratch_bytes(sp)), out(slice_scratch_bytes(sp) + 64);
        for (int k; (k = next.fetch_add(1)) < m;) {
            Gate g{&rows[k]};
            const RowGate gate{&Gate::wait, &g};
            const SliceState ss{0, k + 1, 0, sp.qp};
            const size_t n = write_slice(sp, ss, recs.data() + (size_t)k * nmb, scratch.data(), out.data(), out.size(), nullptr, &gate);
            gated[k].assign(out.begin(), out.begin() + n);
        }
    };
    std::vector<std::thread> th;
    for (int w = 0; w < nwriters; ++w) th.emplace_back(work);
    for (auto& t : th) t.join();
    producer.join();
    std::vector<uint8_t> scratch(slice_scratch_bytes(sp)), out(slice_scratch_bytes(sp) + 64);
    for (int k = 0; k < m; ++k) {
        const SliceState ss{0, k + 1, 0, sp.qp};
        const size_t n = write_slice(sp, ss, recs.data() + (size_t)k * nmb, scratch.data(), out.data(), out.size());
        if (n == 0 || gated[k].size() != n || memcmp(gated[k].data(), out.data(), n)) {
            fprintf(stderr, "picture %d: gated slice (%zu bytes) differs from the slice written after the run (%zu bytes)\n", k,
                    gated[k].size(), n);
            return 1;
        }
    }
    printf("rowgate ok: %d pictures, %d writers\n", m, nwriters);
    return 0;
}
