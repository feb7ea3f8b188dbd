// hl_emu.hip -- TEST INFRASTRUCTURE.  Runs the product's macroblock kernel
// logic (hartallo_amd/csrc/hl_mbcore.h, hl_filters.h) on the host, one lane
// per workgroup (nthr = 1), in raster order, followed by the product's host
// bitstream writer.  It lets tests/ diff the gfx950 kernel logic against the
// oracle without a GPU.  The product library never links this file; it
// fails loudly without a GPU instead of falling back to it.
#define HL_EMU_BUILD 1
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <memory>
#include <vector>

#include "../../hartallo_amd/csrc/hl_pipeline.h"
#include "../../hartallo_amd/csrc/hl_svc.h"
#include "../../hartallo_amd/csrc/hl_cavlc.h"
#include "../../hartallo_amd/csrc/hl_rc.h"
#include "../../hartallo_amd/csrc/hl_writer.h"

using namespace hl;

#if !defined(__HIP_DEVICE_COMPILE__)
int hl::g_emu_bad_guess = 0;  // intra_helper (hl_mbcore.h): HL_EMU_HELPER=2
int hl::g_emu_bad_guess3 = 0;  // fam3_helper: HL_EMU_HELPER bit 8
#endif

struct EmuEnc {
    int W, H, Wc, Hc, mbw, mbh, nmb, qp, qpc, me_range, deblock, gop, early_term;
    int pstride;
    int max_ref_frame = 1;
    std::vector<uint8_t> pic[2][3];
    std::vector<uint8_t> pl[4];
    std::vector<MbState> st;
    std::vector<MbRecord> rec;
    std::vector<MbChain> chain;
    std::vector<int32_t> spec;
    std::vector<uint8_t> scratch, out, hdr;
    int cur, frame_index, gop_left, pict_count, idr_pic_id, chain_end;
    Shared* S;
    Shared* S2;                        // the intra helper's workgroup image (HL_EMU_HELPER)
    std::vector<IntraSpec> ispec;
    std::vector<int32_t> hstate;
    std::vector<Fam3Out> f3;
    std::vector<int32_t> hstate3;
    long helper_runs = 0, helper3_runs = 0;
    // bits (emu_set_helper, HL_EMU_HELPER): 1 intra helpers, 2 intra helpers
    // with a wrong guess, 4 8x8-family helpers, 8 8x8-family helpers with a
    // wrong guess
    int helper_mode = 0;
    int32_t perr[8] = {};              // FrameArgs::perr: [2] helper Intra4x4 kept, [3] rejected; [5] 8x8 family kept, [6] rejected
    std::unique_ptr<RateControl> rc;  // rate control (hl_rc.h), as in the product
    int last_qp;
};

// k_deblock_rows (hl_encoder.hip) lane by lane: every row's tile, prefetch
// registers and bS chunk as the row's workgroup holds them, the MBs in the
// tightest order the kernel's waits allow -- MB (x, y) in step x + 2y, rows
// of one step bottom-up, i.e. before row y - 1's MB x + 2 of the same step.
static void deblock_rows_emu(const DeblockArgs& D, int mbh)
{
    const int mbw = D.mbw;
    std::vector<DbTile> tiles(mbh);
    std::vector<uint32_t> own_l((size_t)mbh * 64), own_c((size_t)mbh * 64);
    std::vector<int> chunk0(mbh, -kDbChunk);
    for (int y = 0; y < mbh; ++y)
        for (int j = 0; j < 64; ++j) {
            own_l[y * 64 + j] = db_own_luma(D, 0, y, j);
            own_c[y * 64 + j] = j < 32 ? db_own_chroma(D, 0, y, j) : 0u;
        }
    for (int d = 0; d < mbw + 2 * mbh; ++d)
        for (int y = mbh - 1; y >= 0; --y) {
            const int x = d - 2 * y;
            if (x < 0 || x >= mbw) continue;
            DbTile& t = tiles[y];
            if (x - chunk0[y] >= kDbChunk) {
                chunk0[y] = x;
                const int n = std::min(kDbChunk, mbw - x) * 32;
                for (int i = 0; i < n; ++i) t.B[i >> 5][i & 31] = (uint8_t)deblock_edge_bs(D, y * mbw + x + (i >> 5), (i & 31) >> 2, i & 3);
            }
            if (x > 0)
                for (int j = 0; j < 64; ++j) db_shift(t, j);
            for (int j = 0; j < 64; ++j) db_put_own(t, j, own_l[y * 64 + j], own_c[y * 64 + j]);
            if (x + 1 < mbw)
                for (int j = 0; j < 64; ++j) {
                    own_l[y * 64 + j] = db_own_luma(D, x + 1, y, j);
                    if (j < 32) own_c[y * 64 + j] = db_own_chroma(D, x + 1, y, j);
                }
            if (y > 0)
                for (int j = 0; j < 64; ++j) db_load_above(D, t, x, y, j);
            for (int step = 0; step < 8; ++step)
                for (int j = 0; j < 64; ++j) db_tile_step(D, t, t.B[x - chunk0[y]], step, j);
            for (int j = 0; j < db_store_words(); ++j) db_store(D, t, x, y, j);
        }
}

// Randomised check of the tiled row deblocking (k_deblock_rows' code, in
// deblock_rows_emu's order) against the per-MB raster filter
// (deblock_mb_step, the reference's order): random samples (smooth with
// steps, so that every filter branch is taken) and random MB objects (intra,
// skip, 16x16 .. 4x4 partitions, coded blocks, motion).  Returns the number
// of differing samples (-1 if the filter changed no sample at all).
// mode 0: the row kernel's order (deblock_rows_emu); mode 1: k_pipeline's
// per-MB LDS tiles (DbMbTile), MB by MB in the tasks of the pipelined
// schedule (task_blocks), tasks in wavefront order
static void deblock_tasks_emu(const DeblockArgs& D, int mbh)
{
    const int mbw = D.mbw;
    DbMbTile t;
    for (int d = 0; d < mbw + 2 * mbh; ++d)
        for (int y = 0; y < mbh; ++y) {
            const int x = d - 2 * y;
            if (x < 0 || x >= mbw) continue;
            int blk[kMaxTaskBlocks][2];
            const int nd = task_blocks(0, x, y, mbw, mbh, blk);
            for (int i = 0; i < nd; ++i) {
                const int X = blk[i][0], Y = blk[i][1];
                memset(&t, 0xA5, sizeof(t));  // stale scratch: every sample a filter reads must be loaded
                for (int j = 0; j < db_mb_load_words(); ++j) db_mb_load(D, t, X, Y, j);
                for (int l = 0; l < 32; ++l) t.bs[l] = (uint8_t)deblock_edge_bs(D, Y * mbw + X, l >> 2, l & 3);
                for (int step = 0; step < 8; ++step)
                    for (int l = 0; l < 64; ++l) db_tile_step(D, t, t.bs, step, l);
                for (int j = 0; j < db_mb_store_slots(); ++j) db_mb_store(D, t, X, Y, j);
            }
        }
}

extern "C" long emu_deblock_selftest(int W, int H, int qp, unsigned seed, int mode)
{
    uint64_t st = seed * 0x9E3779B97F4A7C15ull + 1;
    auto rnd = [&]() -> uint32_t {
        st ^= st << 13;
        st ^= st >> 7;
        st ^= st << 17;
        return (uint32_t)(st >> 11);
    };
    const int mbw = W / 16, mbh = H / 16, Wc = W / 2, Hc = H / 2;
    std::vector<MbState> mbs((size_t)mbw * mbh);
    for (MbState& m : mbs) {
        m = MbState{};
        const uint32_t k = rnd() % 8;
        if (k == 0) {
            m.e_type = ET_I16;
            m.flags = FL_INTRA;
        }
        else if (k == 1) {
            m.e_type = ET_I_NXN;
            m.flags = FL_INTRA;
        }
        else if (k == 2) {
            m.e_type = ET_P16x16;
            m.flags = FL_SKIP;
        }
        else {
            static const int et[5] = {ET_P16x16, ET_P16x8, ET_P8x16, ET_P8x8, ET_P8x8REF0};
            m.e_type = et[rnd() % 5];
        }
        m.part_w = m.e_type == ET_P16x8 ? 16 : (m.e_type == ET_P8x16 || m.e_type == ET_P8x8 || m.e_type == ET_P8x8REF0 ? 8 : 16);
        m.part_h = m.e_type == ET_P8x16 ? 16 : (m.e_type == ET_P16x8 || m.e_type == ET_P8x8 || m.e_type == ET_P8x8REF0 ? 8 : 16);
        for (int i = 0; i < 4; ++i) {
            m.sub_w[i] = rnd() & 1 ? 4 : 8;
            m.sub_h[i] = rnd() & 1 ? 4 : 8;
        }
        m.cbp_l4x4 = rnd() % 3 == 0 ? 0 : (int)(rnd() & 0xFFFF);
        m.cbp_l = m.cbp_l4x4 ? 1 + (int)(rnd() % 15) : 0;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                for (int c = 0; c < 2; ++c) m.mv[i][j][c] = (int16_t)((int)(rnd() % 13) - 6);
    }
    std::vector<uint8_t> a[3], b[3];
    for (int c = 0; c < 3; ++c) {
        const int w = c ? Wc : W, h = c ? Hc : H;
        a[c].resize((size_t)w * h);
        int base = 128;
        for (int y = 0; y < h; ++y)
            for (int x = 0; x < w; ++x) {
                if ((x & 3) == 0 && rnd() % 5 == 0) base = 40 + (int)(rnd() % 176);  // steps at block edges
                a[c][(size_t)y * w + x] = (uint8_t)clip255(base + (int)(rnd() % 9) - 4);
            }
        b[c] = a[c];
    }
    DeblockArgs D;
    D.W = W;
    D.H = H;
    D.Wc = Wc;
    D.mbw = mbw;
    D.qp = qp;
    D.qpc = kQpToQpc[qp];
    D.st = mbs.data();
    std::vector<uint8_t> orig[3] = {a[0], a[1], a[2]};
    for (int c = 0; c < 3; ++c) D.pic[c] = a[c].data();
    for (int m = 0; m < mbw * mbh; ++m)
        for (int step = 0; step < 8; ++step)
            for (int lane = 0; lane < 32; ++lane) deblock_mb_step(D, m, step, lane);
    for (int c = 0; c < 3; ++c) D.pic[c] = b[c].data();
    if (mode == 1) deblock_tasks_emu(D, mbh);
    else deblock_rows_emu(D, mbh);
    long diff = 0, filtered = 0;
    for (int c = 0; c < 3; ++c)
        for (size_t i = 0; i < a[c].size(); ++i) {
            diff += a[c][i] != b[c][i];
            filtered += a[c][i] != orig[c][i];
        }
    return diff ? diff : (filtered ? 0 : -1);  // -1: the filter changed nothing (a vacuous case)
}

extern "C" void* emu_create(int W, int H, int qp, int me_range, int deblock, int gop, int early_term)
{
    if (W <= 0 || H <= 0 || (W & 15) || (H & 15)) return nullptr;
    EmuEnc* e = new EmuEnc();
    e->W = W;
    e->H = H;
    e->Wc = W / 2;
    e->Hc = H / 2;
    e->mbw = W / 16;
    e->mbh = H / 16;
    e->nmb = e->mbw * e->mbh;
    e->qp = qp;
    e->qpc = kQpToQpc[qp];
    e->me_range = me_range < 1 ? 1 : (me_range > 64 ? 64 : me_range);
    e->deblock = deblock;
    e->gop = gop;
    e->early_term = early_term;
    e->pstride = W + 2 * kPad;
    for (int k = 0; k < 2; ++k)
        for (int c = 0; c < 3; ++c) e->pic[k][c].assign(c ? (size_t)e->Wc * e->Hc : (size_t)W * H, 0);
    for (int i = 0; i < 4; ++i) e->pl[i].assign((size_t)e->pstride * (H + 2 * kPad), 0);
    e->st.assign(e->nmb, MbState{});
    memset(e->st.data(), 0, sizeof(MbState) * e->nmb);
    e->rec.assign(e->nmb, MbRecord{});
    e->chain.assign(e->nmb, MbChain{});
    e->spec.assign(e->mbh, 0);
    const StreamParams sp{W, H, qp, deblock};
    e->scratch.resize(slice_scratch_bytes(sp));
    e->out.resize(slice_scratch_bytes(sp) + 64);
    e->hdr.resize(256);
    e->hdr.resize(write_stream_headers(sp, e->hdr.data(), e->hdr.size()));
    e->S = (Shared*)calloc(1, sizeof(Shared));
    e->S2 = (Shared*)calloc(1, sizeof(Shared));
    e->helper_mode = getenv("HL_EMU_HELPER") ? atoi(getenv("HL_EMU_HELPER")) : 0;
    return e;
}

// hl_codec_t.max_ref_frame before the first frame: the SPS / PPS fields only
// (hl_amd_set_max_ref_frame)
extern "C" int emu_set_max_ref_frame(void* h, int max_ref_frame)
{
    EmuEnc* e = (EmuEnc*)h;
    e->max_ref_frame = max_ref_frame;
    const StreamParams sp{e->W, e->H, e->qp, e->deblock, max_ref_frame};
    e->hdr.resize(256);
    e->hdr.resize(write_stream_headers(sp, e->hdr.data(), e->hdr.size()));
    return 0;
}

extern "C" void emu_destroy(void* h)
{
    EmuEnc* e = (EmuEnc*)h;
    if (!e) return;
    free(e->S);
    free(e->S2);
    delete e;
}
extern "C" long emu_helper_runs(void* h) { return ((EmuEnc*)h)->helper_runs; }
extern "C" int emu_helper_i4(void* h, int rejected) { return ((EmuEnc*)h)->perr[rejected ? 3 : 2]; }
extern "C" int emu_helper_fam3(void* h, int rejected) { return ((EmuEnc*)h)->perr[rejected ? 6 : 5]; }
extern "C" long emu_helper3_runs(void* h) { return ((EmuEnc*)h)->helper3_runs; }
extern "C" void emu_set_helper(void* h, int mode) { ((EmuEnc*)h)->helper_mode = mode; }

// Writes hdr (first frame) + 00 00 01 + slice into out; returns bytes or -1.
// rate control of the product path (hl_amd_set_rate_control)
extern "C" int emu_set_rc(void* h, long long bitrate, int fps_num, int fps_den, int basicunit, int qp_min, int qp_max)
{
    EmuEnc* e = (EmuEnc*)h;
    if (bitrate <= 0) {
        e->rc.reset();
        return 0;
    }
    if (fps_num <= 0 || fps_den / fps_num <= 0) return 1;
    e->rc.reset(new RateControl(RcConfig{bitrate, fps_num, fps_den, basicunit, qp_min, qp_max, e->gop, e->W, e->H}));
    return 0;
}

extern "C" int emu_last_qp(void* h) { return ((EmuEnc*)h)->last_qp; }

extern "C" long emu_encode_frame(void* h, const uint8_t* y, const uint8_t* u, const uint8_t* v, uint8_t* out, long cap)
{
    EmuEnc* e = (EmuEnc*)h;
    const bool intra = e->gop_left <= 0;
    if (intra) e->gop_left = e->gop;
    const int qp = e->rc ? e->rc->begin_picture(intra) : e->qp;
    const int qpc = kQpToQpc[qp];
    auto& cur = e->pic[e->cur];
    auto& ref = e->pic[e->cur ^ 1];
    if (!intra)
        for (int p = 0; p < 4; ++p)
            for (int py = 0; py < e->H + 2 * kPad; ++py)
                for (int px = 0; px < e->W + 2 * kPad; ++px)
                    e->pl[p][(size_t)py * e->pstride + px] = qpel_plane_sample(ref[0].data(), e->W, e->H, p, px - kPad, py - kPad);
    FrameArgs F;
    F.W = e->W;
    F.H = e->H;
    F.Wc = e->Wc;
    F.Hc = e->Hc;
    F.mbw = e->mbw;
    F.mbh = e->mbh;
    F.qp = qp;
    F.qpc = qpc;
    F.is_intra = intra;
    F.me_range = e->me_range;
    F.early_term = e->early_term;
    F.lambda = rdo_lambda(qp);
    F.src[0] = y;
    F.src[1] = u;
    F.src[2] = v;
    for (int c = 0; c < 3; ++c) {
        F.cur[c] = cur[c].data();
        F.ref[c] = ref[c].data();
    }
    for (int i = 0; i < 4; ++i) F.pl[i] = e->pl[i].data();
    F.pstride = e->pstride;
    F.st = e->st.data();
    F.rec = e->rec.data();
    F.chain = e->chain.data();
    F.spec = e->spec.data();
    F.prof = nullptr;
    F.run_done = nullptr;
    F.perr = e->perr;
    // HL_EMU_HELPER=1: every P macroblock's intra helper (hl_mbcore.h
    // intra_helper) runs first, on its own workgroup image, as a pipelined
    // run's helper task would; the macroblock then uses its results
    // (2: the helpers guess the live TotalCoeffs wrongly; emu_set_helper)
    // (4: every P macroblock's 8x8-family partitioning helpers likewise;
    // 8: with a wrong guess of the entry values)
    const int helper = e->helper_mode;
#if !defined(__HIP_DEVICE_COMPILE__)
    g_emu_bad_guess = (helper & 2) != 0;
    g_emu_bad_guess3 = (helper & 8) != 0;
#endif
    F.ispec = nullptr;
    F.hstate = nullptr;
    F.f3 = nullptr;
    F.hstate3 = nullptr;
    if ((helper & 3) && !intra) {
        e->ispec.resize(e->nmb);
        e->hstate.assign(e->nmb, HS_DONE);
        F.ispec = e->ispec.data();
        F.hstate = e->hstate.data();
    }
    if ((helper & 12) && !intra) {
        e->f3.resize(4 * e->nmb);
        e->hstate3.assign(4 * e->nmb, HS_DONE);
        F.f3 = e->f3.data();
        F.hstate3 = e->hstate3.data();
    }
    int chain = e->chain_end;
    // HL_EMU_POISON=<seed>: fill the workgroup's LDS image with pseudo-random
    // bytes before every macroblock (a GPU workgroup finds whatever the
    // previous task or kernel left there); any read-before-write of Shared
    // that matters then changes the output.
    static const char* poison = getenv("HL_EMU_POISON");
    static uint64_t prng = poison ? strtoull(poison, nullptr, 10) * 0x9E3779B97F4A7C15ull + 1 : 0;
    for (int a = 0; a < e->nmb; ++a) {
        if (poison) {
            uint8_t* s = (uint8_t*)e->S;
            for (size_t i = 0; i < sizeof(Shared); ++i) {
                prng ^= prng << 13;
                prng ^= prng >> 7;
                prng ^= prng << 17;
                s[i] = (uint8_t)prng;
            }
        }
        if (F.hstate) {
            intra_helper(F, *e->S2, a, 0, 1, chain, F.ispec + a);
            ++e->helper_runs;
        }
        if (F.hstate3)
            for (int j = 3; j < 7; ++j) {  // as the helper tasks of the 8x8 family's partitionings
                encode_mb(F, *e->S2, a, 0, 1, chain, 1 << 20, 1 << 20, 1, F.f3 + 4 * a + j - 3, j);
                ++e->helper3_runs;
            }
        encode_mb(F, *e->S, a, 0, 1, chain);
        chain = e->chain[a].s_out;
    }
    e->chain_end = chain;
    if (e->deblock) {
        DeblockArgs D;
        D.W = e->W;
        D.H = e->H;
        D.Wc = e->Wc;
        D.mbw = e->mbw;
        D.qp = qp;
        D.qpc = qpc;
        for (int c = 0; c < 3; ++c) D.pic[c] = cur[c].data();
        D.st = e->st.data();
        deblock_rows_emu(D, e->mbh);
    }
    const StreamParams sp{e->W, e->H, e->qp, e->deblock};
    const SliceState ss{intra ? 1 : 0, e->pict_count, e->idr_pic_id, qp};
    size_t n = 0;
    if (e->frame_index == 0) {
        if ((long)e->hdr.size() > cap) return -1;
        memcpy(out, e->hdr.data(), e->hdr.size());
        n = e->hdr.size();
    }
    SliceBits sb{};
    const size_t m = write_slice(sp, ss, e->rec.data(), e->scratch.data(), out + n, (size_t)cap - n, &sb);
    if (!m) return -1;
    if (e->rc) {
        RcPictureStats st{};
        for (int a = 0; a < e->nmb; ++a) st.mad_sum += e->rec[a].mad;
        st.header_bits = sb.header_bits;
        st.texture_bits = sb.texture_bits;
        st.nbits = (int32_t)((m - 3) * 8);
        e->rc->end_picture(intra, st, e->gop_left - 1 <= 0);
        if (getenv("HL_EMU_RC_DEBUG"))
            fprintf(stderr, "%d qp %d hdr %d tex %d mad %lld nbytes %d\n", e->frame_index, qp, st.header_bits, st.texture_bits,
                    (long long)st.mad_sum, st.nbits / 8);
    }
    e->last_qp = qp;
    n += m;
    e->cur ^= 1;
    ++e->pict_count;
    if (intra) ++e->idr_pic_id;
    --e->gop_left;
    ++e->frame_index;
    return (long)n;
}

extern "C" const uint8_t* emu_recon(void* h, int plane)
{
    EmuEnc* e = (EmuEnc*)h;
    return e->pic[e->cur ^ 1][plane].data();
}

extern "C" const void* emu_records(void* h) { return ((EmuEnc*)h)->rec.data(); }
extern "C" int emu_record_size(void) { return (int)sizeof(MbRecord); }
extern "C" const void* emu_states(void* h) { return ((EmuEnc*)h)->st.data(); }
extern "C" int emu_state_size(void) { return (int)sizeof(MbState); }

// unit hooks: GPU-side bit counting vs the writer's table
extern "C" int emu_level_code_len(int sl, int lc) { return level_code_len(sl, lc); }
extern "C" int emu_writer_level_bits(int sl, int lc) { return level_code_bits(sl, lc); }

// The device's table-driven Intra4x4 prediction (kI4Tab, i4_tab_pred; DC from
// i4_dc) against the per-mode definition i4_pred_px on random neighbourhoods,
// every mode and sample: the number of differing samples.
extern "C" long emu_i4_table_check(unsigned seed, int n)
{
    long bad = 0;
    unsigned r = seed * 2654435761u + 1u;
    for (int t = 0; t < n; ++t) {
        int p[13], nb[14];
        for (int k = 0; k < 13; ++k) {
            r = r * 1664525u + 1013904223u;
            p[k] = (int)(r >> 24);
            nb[k] = p[k];
        }
        nb[13] = i4_dc(p);
        for (int m = 0; m < 9; ++m)
            for (int pos = 0; pos < 16; ++pos) {
                const uint32_t e = kI4Tab.e[m][pos];
                bad += i4_tab_pred(e, nb[e & 15], nb[(e >> 4) & 15], nb[(e >> 8) & 15]) != i4_pred_px(m, p, pos & 3, pos >> 2);
            }
    }
    return bad;
}

// The pipelined-run schedule (hl_pipeline.h) for tests/test_pipeline_schedule.py:
// deblocking (kind 0) or plane (kind 1) blocks of task (x, y) as X, Y pairs.
extern "C" int emu_task_blocks(int kind, int x, int y, int mbw, int mbh, int* out)
{
    int b[kMaxTaskBlocks][2];
    const int n = task_blocks(kind, x, y, mbw, mbh, b);
    for (int i = 0; i < n; ++i) {
        out[2 * i] = b[i][0];
        out[2 * i + 1] = b[i][1];
    }
    return n;
}

// Dependencies / successors of pipelined-run tasks (hl_pipeline.h) as
// (f, x, y) triples.
extern "C" int emu_task_deps(int f, int x, int y, int mbw, int mbh, int R, int* out)
{
    int d[3][3];
    const int n = task_deps(f, x, y, mbw, mbh, R, d);
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) out[3 * i + k] = d[i][k];
    return n;
}
extern "C" int emu_task_succ(int f, int x, int y, int mbw, int mbh, int R, int nframes, int* out)
{
    int fo = 0, xo = 0, yo = 0;
    const int n = task_succ(f, x, y, mbw, mbh, R, nframes, -1, fo, xo, yo);
    for (int j = 0; j < n; ++j) {
        task_succ(f, x, y, mbw, mbh, R, nframes, j, fo, xo, yo);
        out[3 * j] = fo;
        out[3 * j + 1] = xo;
        out[3 * j + 2] = yo;
    }
    return n;
}
extern "C" void emu_reach_task(int X, int Y, int mbw, int mbh, int* out)
{
    reach_task(X, Y, mbw, mbh, out[0], out[1]);
}

// ---------------------------------------------------------------------------
// Spatial SVC: the base layer through EmuEnc, every enhancement layer through
// the product's svc_encode_mb (hl_svc.h), one lane, raster order.
// emu_svc_encode() returns what the reference harness (oracle/ref_svc_harness.c)
// writes for the call: header bytes when they changed, and after the last
// layer "00 00 01" + the access unit.
// ---------------------------------------------------------------------------
struct EmuLayer {
    int W, H, Wc, Hc, mbw, mbh, nmb, pstride, level;
    SvcGeom g;
    std::vector<uint8_t> pic[2][3];
    std::vector<uint8_t> pl[4];
    std::vector<MbState> st;
    std::vector<MbRecord> rec;
    std::vector<uint8_t> scratch;
    int cur, pict_count, idr_pic_id;
    SvcShared* S;
};

struct EmuSvc {
    EmuEnc* base;
    int L, qp, deblock;
    std::vector<EmuLayer> el;  // layers 1..L-1
    std::vector<int32_t> ws, hs;
    std::vector<uint8_t> au, slice, hdr;
    int next, hdr_layers, au_intra;
    int32_t unpinned;
    int first, last, gop, gop_left;  // layer-sharded coding (hl_amd_set_layer_range)
    long last_hdr;                   // header bytes at the start of the last emu_svc_encode output
};

extern "C" void* emu_svc_create(int W0, int H0, int L, int qp, int me_range, int deblock, int gop, int early_term)
{
    if (L < 2 || L > 4) return nullptr;
    EmuSvc* s = new EmuSvc();
    s->base = (EmuEnc*)emu_create(W0, H0, qp, me_range, deblock, gop, early_term);
    if (!s->base) {
        delete s;
        return nullptr;
    }
    s->L = L;
    s->qp = qp;
    s->deblock = deblock;
    for (int l = 0; l < L; ++l) {
        s->ws.push_back(W0 << l);
        s->hs.push_back(H0 << l);
    }
    s->el.resize(L - 1);
    for (int l = 1; l < L; ++l) {
        EmuLayer& e = s->el[l - 1];
        e.W = W0 << l;
        e.H = H0 << l;
        e.Wc = e.W / 2;
        e.Hc = e.H / 2;
        e.mbw = e.W / 16;
        e.mbh = e.H / 16;
        e.nmb = e.mbw * e.mbh;
        e.pstride = e.W + 2 * kPad;
        e.g = svc_geom(e.W, e.H, e.W / 2, e.H / 2, stream_level_idc(e.W, e.H));
        for (int k = 0; k < 2; ++k)
            for (int c = 0; c < 3; ++c) e.pic[k][c].assign(c ? (size_t)e.Wc * e.Hc : (size_t)e.W * e.H, 0);
        for (int i = 0; i < 4; ++i) e.pl[i].assign((size_t)e.pstride * (e.H + 2 * kPad), 0);
        e.st.assign(e.nmb, MbState{});
        memset(e.st.data(), 0, sizeof(MbState) * e.nmb);
        e.rec.assign(e.nmb, MbRecord{});
        const StreamParams sp{e.W, e.H, qp, deblock};
        e.scratch.resize(slice_scratch_bytes(sp));
        e.cur = e.pict_count = e.idr_pic_id = 0;
        e.S = (SvcShared*)calloc(1, sizeof(SvcShared));
    }
    s->next = 0;
    s->hdr_layers = 1;
    s->unpinned = 0;
    s->first = 0;
    s->last = L - 1;
    s->gop = gop;
    s->gop_left = 0;
    return s;
}

extern "C" void emu_svc_destroy(void* h)
{
    EmuSvc* s = (EmuSvc*)h;
    if (!s) return;
    emu_destroy(s->base);
    for (auto& e : s->el) free(e.S);
    delete s;
}

extern "C" int emu_svc_unpinned(void* h) { return ((EmuSvc*)h)->unpinned; }
extern "C" int emu_svc_set_max_ref_frame(void* h, int max_ref_frame) { return emu_set_max_ref_frame(((EmuSvc*)h)->base, max_ref_frame); }

extern "C" long emu_svc_encode(void* h, int layer, const uint8_t* y, const uint8_t* u, const uint8_t* v, uint8_t* out, long cap)
{
    EmuSvc* s = (EmuSvc*)h;
    if (layer != s->next || layer < s->first || layer > s->last) return -2;
    size_t n = 0;
    s->last_hdr = 0;
    if (layer == 0) {
        EmuEnc* b = s->base;
        s->au_intra = b->gop_left <= 0;
        const bool first = b->frame_index == 0;
        const size_t hdr = first ? b->hdr.size() : 0;
        s->slice.resize(b->out.size() + 256);
        const long m = emu_encode_frame(b, y, u, v, s->slice.data(), (long)s->slice.size());
        if (m < 0) return -1;
        if (first) {
            memcpy(out, s->slice.data(), hdr);
            n = hdr;
            s->last_hdr = (long)hdr;
        }
        uint8_t pre[5];
        write_prefix_nal(s->au_intra != 0, pre);
        s->au.assign(pre, pre + 5);
        static const uint8_t scp[3] = {0, 0, 1};
        s->au.insert(s->au.end(), scp, scp + 3);
        s->au.insert(s->au.end(), s->slice.data() + hdr + 3, s->slice.data() + m);
        if (s->last == 0) {
            if ((long)(n + 3 + s->au.size()) > cap) return -1;
            memcpy(out + n, scp, 3);
            memcpy(out + n + 3, s->au.data(), s->au.size());
            n += 3 + s->au.size();
            s->next = 0;
        }
        else {
            s->next = 1;
        }
        return (long)n;
    }
    EmuLayer& e = s->el[layer - 1];
    const bool intra = s->au_intra != 0;
    if (layer == s->first) s->au.clear();
    if (layer >= s->hdr_layers) {
        const StreamParams bp{s->ws[0], s->hs[0], s->qp, s->deblock, s->base->max_ref_frame};
        n = write_svc_headers(bp, s->ws.data(), s->hs.data(), layer + 1, out, (size_t)cap);
        s->hdr_layers = layer + 1;
        s->last_hdr = (long)n;
    }
    // reference layer: its current picture and macroblock objects
    const uint8_t* rl[3];
    const MbState* rst;
    if (layer == 1) {
        for (int c = 0; c < 3; ++c) rl[c] = emu_recon(s->base, c);
        rst = s->base->st.data();
    }
    else {
        EmuLayer& r = s->el[layer - 2];
        for (int c = 0; c < 3; ++c) rl[c] = r.pic[r.cur ^ 1][c].data();
        rst = r.st.data();
    }
    auto& cur = e.pic[e.cur];
    auto& ref = e.pic[e.cur ^ 1];
    if (!intra)
        for (int p = 0; p < 4; ++p)
            for (int py = 0; py < e.H + 2 * kPad; ++py)
                for (int px = 0; px < e.W + 2 * kPad; ++px)
                    e.pl[p][(size_t)py * e.pstride + px] = qpel_plane_sample(ref[0].data(), e.W, e.H, p, px - kPad, py - kPad);
    SvcArgs A{};
    A.g = e.g;
    FrameArgs& F = A.F;
    F.W = e.W;
    F.H = e.H;
    F.Wc = e.Wc;
    F.Hc = e.Hc;
    F.mbw = e.mbw;
    F.mbh = e.mbh;
    F.qp = s->qp;
    F.qpc = kQpToQpc[s->qp];
    F.is_intra = intra;
    F.src[0] = y;
    F.src[1] = u;
    F.src[2] = v;
    for (int c = 0; c < 3; ++c) {
        F.cur[c] = cur[c].data();
        F.ref[c] = ref[c].data();
    }
    for (int i = 0; i < 4; ++i) F.pl[i] = e.pl[i].data();
    F.pstride = e.pstride;
    F.st = e.st.data();
    F.rec = e.rec.data();
    for (int c = 0; c < 3; ++c) A.rl[c] = rl[c];
    A.rst = rst;
    A.unpinned = &s->unpinned;
    for (int a = 0; a < e.nmb; ++a) svc_encode_mb(A, *e.S, a, 0, 1);
    if (s->deblock) {
        DeblockArgs D;
        D.W = e.W;
        D.H = e.H;
        D.Wc = e.Wc;
        D.mbw = e.mbw;
        D.qp = s->qp;
        D.qpc = kQpToQpc[s->qp];
        for (int c = 0; c < 3; ++c) D.pic[c] = cur[c].data();
        D.st = e.st.data();
        deblock_rows_emu(D, e.mbh);
    }
    const StreamParams sp{e.W, e.H, s->qp, s->deblock};
    const SvcSliceState ss{intra ? 1 : 0, e.pict_count, e.idr_pic_id, s->qp, layer};
    s->slice.resize(e.scratch.size() + 64);
    size_t m;
    if (getenv("HL_EMU_HOST_WRITER")) {
        m = write_svc_slice(sp, ss, e.rec.data(), e.scratch.data(), s->slice.data(), s->slice.size(), 4);
    }
    else {
        // the product's GPU serialisation (hl_cavlc.h): counts, exclusive scan, writes
        std::vector<int64_t> off(e.nmb + 1, 0);
        for (int a = 0; a < e.nmb; ++a) {
            BitCount bc;
            el_mb_bits(bc, e.rec.data(), a, e.mbw, intra);
            off[a + 1] = off[a] + bc.pos;
        }
        std::vector<uint32_t> words((size_t)(off[e.nmb] >> 5) + 2, 0);
        for (int a = 0; a < e.nmb; ++a) {
            BitOr bo{words.data(), off[a]};
            el_mb_bits(bo, e.rec.data(), a, e.mbw, intra);
        }
        m = write_svc_slice_bits(sp, ss, words.data(), off[e.nmb], e.scratch.data(), s->slice.data(), s->slice.size());
    }
    if (!m) return -1;
    static const uint8_t scp[3] = {0, 0, 1};
    if (layer != s->first) s->au.insert(s->au.end(), scp, scp + 3);
    s->au.insert(s->au.end(), s->slice.data() + 3, s->slice.data() + m);
    e.cur ^= 1;
    ++e.pict_count;
    // idr_pic_id counts IdrPicFlag(nal_unit_type) pictures (encode.c:527-530):
    // type-20 slices never do, so an enhancement layer's stays 0
    if (layer == s->last) {
        if ((long)(n + 3 + s->au.size()) > cap) return -1;
        memcpy(out + n, scp, 3);
        memcpy(out + n + 3, s->au.data(), s->au.size());
        n += 3 + s->au.size();
        s->next = s->first;
        --s->gop_left;
    }
    else {
        s->next = layer + 1;
    }
    return (long)n;
}

// reconstructed (deblocked) picture of a layer after its last encode
extern "C" const uint8_t* emu_svc_recon(void* h, int layer, int plane)
{
    EmuSvc* s = (EmuSvc*)h;
    if (layer == 0) return emu_recon(s->base, plane);
    EmuLayer& e = s->el[layer - 1];
    return e.pic[e.cur ^ 1][plane].data();
}
extern "C" const void* emu_svc_records(void* h, int layer)
{
    EmuSvc* s = (EmuSvc*)h;
    return layer == 0 ? s->base->rec.data() : s->el[layer - 1].rec.data();
}

// layer-sharded coding, as hl_amd_set_layer_range / _export_layer / _import_layer
extern "C" int emu_svc_set_range(void* h, int first, int last)
{
    EmuSvc* s = (EmuSvc*)h;
    if (first < 0 || last < first || last >= s->L) return 1;
    s->first = first;
    s->last = last;
    s->next = first;
    return 0;
}

static void emu_layer_ptrs(EmuSvc* s, int l, int pick, uint8_t** pic, MbState*& st, int& W, int& H, int& n)
{
    if (l == 0) {
        EmuEnc* b = s->base;
        const int k = pick ? b->cur : b->cur ^ 1;
        for (int c = 0; c < 3; ++c) pic[c] = b->pic[k][c].data();
        st = b->st.data();
        W = b->W;
        H = b->H;
        n = b->nmb;
    }
    else {
        EmuLayer& e = s->el[l - 1];
        const int k = pick ? e.cur : e.cur ^ 1;
        for (int c = 0; c < 3; ++c) pic[c] = e.pic[k][c].data();
        st = e.st.data();
        W = e.W;
        H = e.H;
        n = e.nmb;
    }
}

extern "C" long emu_svc_layer_state_bytes(void* h, int layer)
{
    EmuSvc* s = (EmuSvc*)h;
    const long W = s->ws[layer], H = s->hs[layer];
    return W * H * 3 / 2 + (long)sizeof(MbState) * (W / 16) * (H / 16);
}

extern "C" int emu_svc_export(void* h, int layer, uint8_t* dst)
{
    EmuSvc* s = (EmuSvc*)h;
    uint8_t* pic[3];
    MbState* st;
    int W, H, n;
    emu_layer_ptrs(s, layer, 0, pic, st, W, H, n);
    const size_t ys = (size_t)W * H, cs = ys / 4;
    memcpy(dst, pic[0], ys);
    memcpy(dst + ys, pic[1], cs);
    memcpy(dst + ys + cs, pic[2], cs);
    memcpy(dst + ys + 2 * cs, st, sizeof(MbState) * n);
    return 0;
}

extern "C" int emu_svc_import(void* h, int layer, const uint8_t* src)
{
    EmuSvc* s = (EmuSvc*)h;
    if (layer != s->first - 1 || s->next != s->first) return 1;
    uint8_t* pic[3];
    MbState* st;
    int W, H, n;
    emu_layer_ptrs(s, layer, 1, pic, st, W, H, n);
    const size_t ys = (size_t)W * H, cs = ys / 4;
    memcpy(pic[0], src, ys);
    memcpy(pic[1], src + ys, cs);
    memcpy(pic[2], src + ys + cs, cs);
    memcpy(st, src + ys + 2 * cs, sizeof(MbState) * n);
    if (layer == 0) s->base->cur ^= 1;
    else s->el[layer - 1].cur ^= 1;
    s->au_intra = s->gop_left <= 0;
    if (s->au_intra) s->gop_left = s->gop;
    return 0;
}

extern "C" long emu_svc_last_hdr(void* h) { return ((EmuSvc*)h)->last_hdr; }

// diagnostics: seconds per write_svc_slice of layer `layer`'s last records
extern "C" double emu_svc_write_seconds(void* h, int layer, int threads, int reps)
{
    EmuSvc* s = (EmuSvc*)h;
    EmuLayer& e = s->el[layer - 1];
    const StreamParams sp{e.W, e.H, s->qp, s->deblock};
    const SvcSliceState ss{0, 1, 0, s->qp, layer};
    std::vector<uint8_t> out(e.scratch.size() + 64);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) write_svc_slice(sp, ss, e.rec.data(), e.scratch.data(), out.data(), out.size(), threads);
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
}
