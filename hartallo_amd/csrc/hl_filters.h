// hl_filters.h -- picture-level filters of the encode path for gfx950:
//  * the quarter-pel reference planes (full, b, h, j) of 8.4.2.2.1, padded so
//    every motion-search fetch is a plain 2D load (pred_inter.c:339-885 and
//    the clamped index table of interpol.c:74-225 give the edge semantics:
//    every tap coordinate is clamped to the picture independently);
//  * the Baseline deblocking filter of one macroblock (8.7, deblock.c:192-3553),
//    luma and chroma lines in parallel lanes, edges in the reference's order.
#pragma once
#include "hl_mbcore.h"

namespace hl {

HD int tap6(int a, int b, int c, int d, int e, int f) { return a - 5 * (b + e) + 20 * (c + d) + f; }

// One sample of the padded plane `plane` at picture coordinates (x, y).
HD uint8_t qpel_plane_sample(const uint8_t* ref, int W, int H, int plane, int x, int y)
{
    auto S = [&](int xx, int yy) -> int { return ref[clip3(0, H - 1, yy) * W + clip3(0, W - 1, xx)]; };
    auto h1 = [&](int xx) -> int { return tap6(S(xx, y - 2), S(xx, y - 1), S(xx, y), S(xx, y + 1), S(xx, y + 2), S(xx, y + 3)); };
    switch (plane) {
    case 0: return (uint8_t)S(x, y);
    case 1: return (uint8_t)clip255((tap6(S(x - 2, y), S(x - 1, y), S(x, y), S(x + 1, y), S(x + 2, y), S(x + 3, y)) + 16) >> 5);
    case 2: return (uint8_t)clip255((h1(x) + 16) >> 5);
    default: return (uint8_t)clip255((tap6(h1(x - 2), h1(x - 1), h1(x), h1(x + 1), h1(x + 2), h1(x + 3)) + 512) >> 10);
    }
}

#if defined(__HIPCC__)
// Quarter-pel planes (full, b, h, j) of a reference picture, padded by kPad
// (qpel_plane_sample, hl_filters.h: every tap coordinate clamped to the
// picture independently, interpol.c:74-225).  One workgroup per
// (16 kPlSpt) x 16 tile of the padded planes: the clamped source tile with
// its 6-tap apron is staged in LDS as 4-byte words (one aligned global load
// per word inside the picture), then every lane computes kPlSpt consecutive
// samples of one row of each plane from 6 LDS rows and writes them with one
// store per plane.  HBM-bound: 1 B/px read, 4 B per padded pixel written.
#ifndef HL_PL_SPT
#define HL_PL_SPT 8  // samples per lane and plane: 4, 8 or 16 (8: 6.5 us per 1088p picture, 16: 8.0, 4: 8.1, profiles/r05_ab_planes_samples_per_lane.log)
#endif
constexpr int kPlSpt = HL_PL_SPT;
static_assert(kPlSpt == 4 || kPlSpt == 8 || kPlSpt == 16, "a lane's samples are one 4-, 8- or 16-byte store per plane");
constexpr int kPlTileW = 16 * kPlSpt, kPlTileH = 16;
__global__ __launch_bounds__(256) void k_planes(const uint8_t* __restrict__ ref, int W, int H, uint8_t* __restrict__ pl0, int pstride,
                                                int plsz)
{
    constexpr int TWW = (kPlTileW + 8) / 4, TR = kPlTileH + 5;  // words per tile row (apron 2 + 3, alignment 3), rows
    constexpr int NW = kPlSpt / 4;                               // output words per lane and plane
    __shared__ uint32_t T[TR][TWW + 1];
    const int PW = W + 2 * kPad, PH = H + 2 * kPad;
    const int tx = blockIdx.x * kPlTileW, ty = blockIdx.y * kPlTileH;  // tile origin, padded coordinates
    const int xs = tx - kPad - 2, x0 = xs & ~3, o = xs - x0;          // picture x of T column 0 (4-aligned); offset of the first tap
    const int y0 = ty - kPad - 2;                                      // picture y of T row 0
    // every load of the tile in flight at once, then the LDS stores
    constexpr int kIt = (TR * TWW + 255) / 256;
    uint32_t v[kIt];
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
        const int i = threadIdx.x + it * 256, r = min(i / TWW, TR - 1), w = i - (i / TWW) * TWW;
        const uint8_t* row = ref + (size_t)clip3(0, H - 1, y0 + r) * W;
        const int x = x0 + 4 * w;
        if (x >= 0 && x + 3 < W) v[it] = *reinterpret_cast<const uint32_t*>(row + x);
        else
            v[it] = (uint32_t)row[clip3(0, W - 1, x)] | (uint32_t)row[clip3(0, W - 1, x + 1)] << 8 |
                    (uint32_t)row[clip3(0, W - 1, x + 2)] << 16 | (uint32_t)row[clip3(0, W - 1, x + 3)] << 24;
    }
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
        const int i = threadIdx.x + it * 256;
        if (i < TR * TWW) T[i / TWW][i % TWW] = v[it];
    }
    __syncthreads();
    const int tr = threadIdx.x >> 4, tc = threadIdx.x & 15;
    const int py = ty + tr, px = tx + tc * kPlSpt;
    if (py >= PH || px >= PW) return;  // PW is a multiple of 16: a lane's group never straddles it
    // columns tc*kPlSpt + o + j (j = 0..kPlSpt+4) of rows tr..tr+5
    auto byte_at = [&](int r, int j) -> int {
        const int c = tc * kPlSpt + o + j;
        return (int)((T[tr + r][c >> 2] >> (8 * (c & 3))) & 0xffu);
    };
    int vs[kPlSpt + 5];
#pragma unroll
    for (int j = 0; j < kPlSpt + 5; ++j) vs[j] = tap6(byte_at(0, j), byte_at(1, j), byte_at(2, j), byte_at(3, j), byte_at(4, j), byte_at(5, j));
    uint32_t f[NW], b[NW], h[NW], jj[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) f[q] = b[q] = h[q] = jj[q] = 0;
#pragma unroll
    for (int k = 0; k < kPlSpt; ++k) {
        const int sf = byte_at(2, k + 2);
        int vb = (tap6(byte_at(2, k), byte_at(2, k + 1), sf, byte_at(2, k + 3), byte_at(2, k + 4), byte_at(2, k + 5)) + 16) >> 5;
        int vh = (vs[k + 2] + 16) >> 5;
        int vj = (tap6(vs[k], vs[k + 1], vs[k + 2], vs[k + 3], vs[k + 4], vs[k + 5]) + 512) >> 10;
        // opaque: keeps hipcc (ROCm 7.2) from fusing shift + clamp + byte
        // packing into v_ashr_pk_u8_i32, whose result's upper half it then
        // ORs as if zero -- wrong bytes 2 and 3 of every packed pair on gfx950
        // (tests/test_gpu_unit.py::test_planes_kernel)
        asm volatile("" : "+v"(vb), "+v"(vh), "+v"(vj));
        const int sh = 8 * (k & 3), q = k >> 2;
        f[q] |= (uint32_t)sf << sh;
        b[q] |= (uint32_t)clip255(vb) << sh;
        h[q] |= (uint32_t)clip255(vh) << sh;
        jj[q] |= (uint32_t)clip255(vj) << sh;
    }
    const size_t at = (size_t)py * pstride + px;
    auto put = [&](uint8_t* p, const uint32_t* w) {
        if constexpr (NW == 4) *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
        else if constexpr (NW == 2) *reinterpret_cast<uint2*>(p) = make_uint2(w[0], w[1]);
        else *reinterpret_cast<uint32_t*>(p) = w[0];
    };
    put(pl0 + at, f);
    put(pl0 + plsz + at, b);
    put(pl0 + 2 * (size_t)plsz + at, h);
    put(pl0 + 3 * (size_t)plsz + at, jj);
}
#endif

// ---------------------------------------------------------------------------
// Deblocking
// ---------------------------------------------------------------------------
// bS of the 4-sample segment between p (in MB P at (px,py)) and q (in MB Q at
// (qx,qy)), deblock.c:1784-1834.  ref_idx_l0 is never written by the encoder
// (always 0) and predFlagL0 is 1 for every partition of an inter MB.
HD int deblock_bs(const MbState& P, const MbState& Q, int px, int py, int qx, int qy, bool mb_edge)
{
    if ((P.flags & FL_INTRA) || (Q.flags & FL_INTRA)) return mb_edge ? 4 : 3;
    if ((P.cbp_l4x4 & (1 << blk_idx(px, py))) || (Q.cbp_l4x4 & (1 << blk_idx(qx, qy)))) return 2;
    auto part = [](const MbState& m, int x, int y, int& pi, int& spi) {
        pi = (16 / m.part_w) * (y / m.part_h) + (x / m.part_w);
        spi = (m.e_type == ET_P8x8 || m.e_type == ET_P8x8REF0) ? (8 / m.sub_w[pi]) * ((y % 8) / m.sub_h[pi]) + ((x % 8) / m.sub_w[pi]) : 0;
    };
    int pp, ps, qp, qs;
    part(P, px, py, pp, ps);
    part(Q, qx, qy, qp, qs);
    if (iabs(P.mv[pp][ps][0] - Q.mv[qp][qs][0]) >= 4) return 1;
    return iabs(P.mv[pp][ps][1] - Q.mv[qp][qs][1]) >= 4 ? 1 : 0;
}

// Filters one line across an edge; s points at q0, step reaches q1.
HD void deblock_line(uint8_t* s, int step, int bS, bool chroma, int indexA, int alpha, int beta)
{
    const int p0 = s[-step], p1 = s[-2 * step], q0 = s[0], q1 = s[step];
    const int p2 = chroma ? 0 : s[-3 * step], q2 = chroma ? 0 : s[2 * step];
    if (!(iabs(p0 - q0) < alpha && iabs(p1 - p0) < beta && iabs(q1 - q0) < beta)) return;
    const int ap = iabs(p2 - p0), aq = iabs(q2 - q0);
    if (bS < 4) {
        const int tc0 = tc0_of(indexA, bS);
        const int tc = chroma ? tc0 + 1 : tc0 + (ap < beta) + (aq < beta);
        const int delta = clip3(-tc, tc, ((q0 - p0) * 4 + (p1 - q1) + 4) >> 3);
        s[-step] = (uint8_t)clip255(p0 + delta);
        s[0] = (uint8_t)clip255(q0 - delta);
        if (!chroma && ap < beta) s[-2 * step] = (uint8_t)(p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1));
        if (!chroma && aq < beta) s[step] = (uint8_t)(q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1));
    }
    else {
        const int p3 = chroma ? 0 : s[-4 * step], q3 = chroma ? 0 : s[3 * step];
        const bool strong = iabs(p0 - q0) < ((alpha >> 2) + 2);
        if (!chroma && ap < beta && strong) {
            s[-step] = (uint8_t)((p2 + (p1 << 1) + (p0 << 1) + (q0 << 1) + q1 + 4) >> 3);
            s[-2 * step] = (uint8_t)((p2 + p1 + p0 + q0 + 2) >> 2);
            s[-3 * step] = (uint8_t)(((p3 << 1) + (p2 << 1) + p2 + p1 + p0 + q0 + 4) >> 3);
        }
        else {
            s[-step] = (uint8_t)(((p1 << 1) + p0 + q1 + 2) >> 2);
        }
        if (!chroma && aq < beta && strong) {
            s[0] = (uint8_t)((p1 + (p0 << 1) + (q0 << 1) + (q1 << 1) + q2 + 4) >> 3);
            s[step] = (uint8_t)((p0 + q0 + q1 + q2 + 2) >> 2);
            s[2 * step] = (uint8_t)(((q3 << 1) + (q2 << 1) + q2 + q1 + q0 + p0 + 4) >> 3);
        }
        else {
            s[0] = (uint8_t)(((q1 << 1) + q0 + p1 + 2) >> 2);
        }
    }
}

struct DeblockArgs {
    int32_t W, H, Wc, mbw, qp, qpc;
    uint8_t* pic[3];
    const MbState* st;
};

// bS of segment k (0..3) of luma edge e of macroblock addr -- e 0..3 the
// vertical edges 0, 4, 8, 12, e 4..7 the horizontal ones -- or 0 where the
// edge is not filtered (picture border, or an internal edge of a 16x16
// prediction without luma residual).  The chroma edges 0 / 4 use the bS of
// luma edges 0 / 8 (8.7.2.1: chroma bS is the bS of the corresponding luma
// samples).
HD int deblock_edge_bs(const DeblockArgs& D, int addr, int e, int k)
{
    const int mbx = addr % D.mbw, mby = addr / D.mbw;
    const auto& Q = *gmem(D.st + addr);
    const bool vert = e < 4;
    const int edge = (e & 3) * 4;
    const bool mb_edge = edge == 0;
    if (mb_edge && (vert ? mbx == 0 : mby == 0)) return 0;
    const bool internal = !((Q.e_type == ET_P16x16 || (Q.flags & FL_SKIP)) && !Q.cbp_l);
    if (!mb_edge && !internal) return 0;
    const auto& P = *gmem(D.st + (mb_edge ? (vert ? addr - 1 : addr - D.mbw) : addr));
    return vert ? deblock_bs(P, Q, mb_edge ? 12 : edge - 4, k * 4, edge, k * 4, mb_edge)
                : deblock_bs(P, Q, k * 4, mb_edge ? 12 : edge - 4, k * 4, edge, mb_edge);
}

// ---- Deblocking of a macroblock row in an LDS tile (k_deblock_rows) ----
// The tile holds the macroblock and its 4-sample apron above and to the left
// (luma rows / columns -4..15, chroma -4..7), 4-byte words per row.  The left
// apron is the previous macroblock's right columns, carried over in the
// tile; the rows above come from the row above once it has finished the
// macroblock above-right.  Every filter step runs in the tile; the finished
// words go back to the picture afterwards, the right 4 columns (filtered
// again by the next macroblock's left edge) with the next macroblock.
constexpr int kDbL = 20, kDbC = 12, kDbChunk = 256;
struct DbTile {
    uint8_t T[kDbL * kDbL];       // luma
    uint8_t C[2][kDbC * kDbC];    // Cb, Cr
    uint8_t B[kDbChunk][32];      // bS of a chunk of the row's macroblocks, [mb][e * 4 + k]
};

// word j (0..63) of macroblock (x, y)'s own luma rows, and word j (0..31) of
// its chroma rows (comp = j >> 4, row (j >> 1) & 7, word j & 1)
HD uint32_t db_own_luma(const DeblockArgs& D, int x, int y, int j)
{
    return *gmem(reinterpret_cast<const uint32_t*>(D.pic[0] + (size_t)(y * 16 + (j >> 2)) * D.W + x * 16 + (j & 3) * 4));
}
HD uint32_t db_own_chroma(const DeblockArgs& D, int x, int y, int j)
{
    return *gmem(reinterpret_cast<const uint32_t*>(D.pic[1 + (j >> 4)] + (size_t)(y * 8 + ((j >> 1) & 7)) * D.Wc + x * 8 + (j & 1) * 4));
}
HD void db_put_own(DbTile& t, int j, uint32_t luma, uint32_t chroma)
{
    *reinterpret_cast<uint32_t*>(t.T + (4 + (j >> 2)) * kDbL + 4 + (j & 3) * 4) = luma;
    if (j < 32) *reinterpret_cast<uint32_t*>(t.C[j >> 4] + (4 + ((j >> 1) & 7)) * kDbC + 4 + (j & 1) * 4) = chroma;
}
// left apron <- the previous macroblock's right columns (lanes 0..43)
HD void db_shift(DbTile& t, int j)
{
    if (j < kDbL) {
        uint32_t* r = reinterpret_cast<uint32_t*>(t.T + j * kDbL);
        r[0] = r[4];
    }
    else if (j < kDbL + 2 * kDbC) {
        const int c = (j - kDbL) / kDbC, row = (j - kDbL) % kDbC;
        uint32_t* r = reinterpret_cast<uint32_t*>(t.C[c] + row * kDbC);
        r[0] = r[2];
    }
}
// the 4 rows above (lanes 0..31: 16 luma words, 16 chroma words), y > 0
HD void db_load_above(const DeblockArgs& D, DbTile& t, int x, int y, int j)
{
    if (j < 16) {
        const int row = j >> 2, w = j & 3;
        *reinterpret_cast<uint32_t*>(t.T + row * kDbL + 4 + w * 4) =
            *reinterpret_cast<const uint32_t*>(D.pic[0] + (size_t)(y * 16 - 4 + row) * D.W + x * 16 + w * 4);
    }
    else if (j < 32) {
        const int c = (j - 16) >> 3, row = ((j - 16) >> 1) & 3, w = j & 1;
        *reinterpret_cast<uint32_t*>(t.C[c] + row * kDbC + 4 + w * 4) =
            *reinterpret_cast<const uint32_t*>(D.pic[1 + c] + (size_t)(y * 8 - 4 + row) * D.Wc + x * 8 + w * 4);
    }
}
// step (0..7) of the filter of the tile's macroblock for lane 0..31, as
// deblock_mb_step; bs = the macroblock's 32 bS values
template <class Tile>
HD void db_tile_step(const DeblockArgs& D, Tile& t, const uint8_t* bs, int step, int lane)
{
    if (lane < 16) {
        const bool vert = step < 4;
        const int edge = (step & 3) * 4, b = bs[step * 4 + (lane >> 2)];
        if (!b) return;
        const int indexA = clip3(0, 51, D.qp);
        uint8_t* s = vert ? t.T + (4 + lane) * kDbL + 4 + edge : t.T + (4 + edge) * kDbL + 4 + lane;
        deblock_line(s, vert ? 1 : kDbL, b, false, indexA, kAlpha[indexA], kBeta[indexA]);
    }
    else if (lane < 32 && step < 4) {
        const bool vert = step < 2;
        const int edge = (step & 1) * 4, comp = (lane - 16) >> 3, i = (lane - 16) & 7;
        const int b = bs[((vert ? 0 : 4) + (step & 1) * 2) * 4 + (i >> 1)];
        if (!b) return;
        const int indexA = clip3(0, 51, D.qpc);
        uint8_t* s = vert ? t.C[comp] + (4 + i) * kDbC + 4 + edge : t.C[comp] + (4 + edge) * kDbC + 4 + i;
        deblock_line(s, vert ? 1 : kDbC, b, true, indexA, kAlpha[indexA], kBeta[indexA]);
    }
}
// the finished words of macroblock (x, y) back to the picture: columns -4..11
// (-4..15 for the row's last macroblock), rows -4..15 (0..15 in row 0);
// word j < db_store_words()
HD int db_store_words() { return kDbL * 5 + 2 * kDbC * 3; }
HD void db_store(const DeblockArgs& D, const DbTile& t, int x, int y, int j)
{
    const bool last = x == D.mbw - 1;
    if (j < kDbL * 5) {
        const int row = j / 5, w = j % 5;
        if ((y == 0 && row < 4) || (x == 0 && w == 0) || (!last && w == 4)) return;
        *reinterpret_cast<uint32_t*>(D.pic[0] + (size_t)(y * 16 - 4 + row) * D.W + x * 16 - 4 + w * 4) =
            *reinterpret_cast<const uint32_t*>(t.T + row * kDbL + w * 4);
    }
    else {
        j -= kDbL * 5;
        const int c = j / (kDbC * 3), row = (j / 3) % kDbC, w = j % 3;
        if ((y == 0 && row < 4) || (x == 0 && w == 0) || (!last && w == 2)) return;
        *reinterpret_cast<uint32_t*>(D.pic[1 + c] + (size_t)(y * 8 - 4 + row) * D.Wc + x * 8 - 4 + w * 4) =
            *reinterpret_cast<const uint32_t*>(t.C[c] + row * kDbC + w * 4);
    }
}

// ---- Deblocking of one macroblock in an LDS tile (the tasks of k_pipeline) ----
// The tile of DbTile without the row state: the MB and its 4-sample apron,
// loaded in one round (the apron is final: the MBs left of and above it are
// deblocked in earlier tasks, hl_pipeline.h), filtered in LDS, and the
// samples a filter may change (luma: 3 columns left / 3 rows above and the
// MB; chroma: 1 column / 1 row and the MB) stored back byte by byte.
struct DbMbTile {
    uint8_t T[kDbL * kDbL];
    uint8_t C[2][kDbC * kDbC];
    uint8_t bs[32];
};
HD int db_mb_load_words() { return kDbL * 5 + 2 * kDbC * 3; }
// word j of the tile of MB (X, Y) from the picture (words outside it are not read by any filter that runs)
HD void db_mb_load(const DeblockArgs& D, DbMbTile& t, int X, int Y, int j)
{
    if (j < kDbL * 5) {
        const int row = j / 5, w = j % 5, py = Y * 16 - 4 + row, px = X * 16 - 4 + w * 4;
        if (py < 0 || px < 0) return;
        *reinterpret_cast<uint32_t*>(t.T + row * kDbL + w * 4) = *gmem(reinterpret_cast<const uint32_t*>(D.pic[0] + (size_t)py * D.W + px));
    }
    else {
        j -= kDbL * 5;
        const int c = j / (kDbC * 3), row = (j / 3) % kDbC, w = j % 3, py = Y * 8 - 4 + row, px = X * 8 - 4 + w * 4;
        if (py < 0 || px < 0) return;
        *reinterpret_cast<uint32_t*>(t.C[c] + row * kDbC + w * 4) = *gmem(reinterpret_cast<const uint32_t*>(D.pic[1 + c] + (size_t)py * D.Wc + px));
    }
}
// store slot j (< db_mb_store_slots()): one sample a filter of MB (X, Y) may have changed
HD int db_mb_store_slots() { return 16 * 19 + 3 * 16 + 2 * (8 * 9 + 8); }
HD void db_mb_store(const DeblockArgs& D, const DbMbTile& t, int X, int Y, int j)
{
    int tr, tc, comp = -1;  // tile row / column (apron included)
    if (j < 16 * 19) {
        tr = 4 + j / 19;
        tc = 1 + j % 19;  // columns -3..15
    }
    else if ((j -= 16 * 19) < 3 * 16) {
        tr = 1 + j / 16;  // rows -3..-1
        tc = 4 + j % 16;
    }
    else {
        j -= 3 * 16;
        comp = j / 80;
        j %= 80;
        if (j < 72) {
            tr = 4 + j / 9;
            tc = 3 + j % 9;  // columns -1..7
        }
        else {
            tr = 3;  // row -1
            tc = 4 + (j - 72);
        }
    }
    if (comp < 0) {
        const int py = Y * 16 - 4 + tr, px = X * 16 - 4 + tc;
        if (py >= 0 && px >= 0) gmem(D.pic[0])[(size_t)py * D.W + px] = t.T[tr * kDbL + tc];
    }
    else {
        const int py = Y * 8 - 4 + tr, px = X * 8 - 4 + tc;
        if (py >= 0 && px >= 0) gmem(D.pic[1 + comp])[(size_t)py * D.Wc + px] = t.C[comp][tr * kDbC + tc];
    }
}

// Step `step` (0..7) of the deblocking of macroblock `addr` for lane `lane`
// (0..31): lanes 0-15 filter the luma lines of luma edge `step`
// (vertical 0,4,8,12 then horizontal 0,4,8,12), lanes 16-31 the chroma
// lines of chroma edge `step` (vertical 0,4 then horizontal 0,4; steps 0-3).
HD void deblock_mb_step(const DeblockArgs& D, int addr, int step, int lane)
{
    const int mbx = addr % D.mbw, mby = addr / D.mbw;
    const MbState& Q = D.st[addr];
    const bool internal = !((Q.e_type == ET_P16x16 || (Q.flags & FL_SKIP)) && !Q.cbp_l);
    const bool chroma = lane >= 16;
    int vert, edge;
    if (!chroma) {
        vert = step < 4;
        edge = (step & 3) * 4;
    }
    else {
        if (step >= 4) return;
        vert = step < 2;
        edge = (step & 1) * 4;
    }
    const bool mb_edge = edge == 0;
    if (mb_edge && (vert ? mbx == 0 : mby == 0)) return;
    if (!mb_edge && !internal) return;
    const MbState& P = mb_edge ? (vert ? D.st[addr - 1] : D.st[addr - D.mbw]) : Q;
    if (!chroma) {
        const int i = lane, k = i >> 2;
        const int bS = vert ? deblock_bs(P, Q, mb_edge ? 12 : edge - 4, k * 4, edge, k * 4, mb_edge)
                            : deblock_bs(P, Q, k * 4, mb_edge ? 12 : edge - 4, k * 4, edge, mb_edge);
        if (!bS) return;
        const int indexA = clip3(0, 51, D.qp);
        uint8_t* s = vert ? D.pic[0] + (mby * 16 + i) * D.W + mbx * 16 + edge : D.pic[0] + (mby * 16 + edge) * D.W + mbx * 16 + i;
        deblock_line(s, vert ? 1 : D.W, bS, false, indexA, kAlpha[indexA], kBeta[indexA]);
    }
    else {
        const int comp = (lane - 16) >> 3, i = (lane - 16) & 7, k = i >> 1, ledge = edge * 2;
        const int bS = vert ? deblock_bs(P, Q, mb_edge ? 12 : ledge - 4, k * 4, ledge, k * 4, mb_edge)
                            : deblock_bs(P, Q, k * 4, mb_edge ? 12 : ledge - 4, k * 4, ledge, mb_edge);
        if (!bS) return;
        const int indexA = clip3(0, 51, D.qpc);
        uint8_t* s = vert ? D.pic[1 + comp] + (mby * 8 + i) * D.Wc + mbx * 8 + edge : D.pic[1 + comp] + (mby * 8 + edge) * D.Wc + mbx * 8 + i;
        deblock_line(s, vert ? 1 : D.Wc, bS, true, indexA, kAlpha[indexA], kBeta[indexA]);
    }
}

}  // namespace hl
