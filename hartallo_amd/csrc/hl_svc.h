// hl_svc.h -- spatial-SVC enhancement layers (Annex G) of the reference
// encoder, for gfx950.
//
// The reference codes every enhancement-layer macroblock with
// base_mode_flag = 1 (rdo.c:301-461 intra, rdo.c:1273-1521 inter; "for now we
// always reuse prediction from base layer"): there is no search and no mode
// decision.  A macroblock's type, partitioning and motion are inferred from
// the reference layer (G.8.1.5.1, utils.c:1225-1493), its prediction is the
// motion-compensated enhancement-layer reference picture (inter) or the
// resampled reference-layer picture (Intra_Base, G.8.6.2, decode_svc.c:
// 2864-3175), and its residual is transformed and quantised with *intra*
// rounding (rdo.c:1468) without single-coefficient elimination.  Every
// macroblock of a layer is therefore independent of the others: one launch
// covers the whole picture, one workgroup per macroblock.
//
// Scope (what the reference can produce, hl_codec.c:95-131 and
// hl_codec_264_layer.c:104-152): dyadic spatial layers (each twice the one
// below), no cropping, frame coding, one reference picture.  Then
// SpatialResolutionChangeFlag = 1, RestrictedSpatialResolutionChangeFlag = 1
// and CroppingChangeFlag = 0, which removes the partition fix-up and motion
// merging of G.8.6.1.1/G.8.6.1.2 (utils.c:1711-1772, 1928-2004).
//
// Reference-layer intra macroblocks in P pictures are outside the pinned
// scope: the reference then predicts from whatever its scratch buffers
// (hl_memory_blocks) last held (an I_BL macroblock of an EP slice reaches the
// inter path with no motion, rdo.c:1407-1426) or reads a macroblock object
// at index -1 (utils.c:1796-1803).  Such macroblocks are counted
// (SvcArgs::unpinned) and predicted from the co-located reference samples.
#pragma once
#include <math.h>

#include "hl_filters.h"

namespace hl {

// HL_CODEC_264_MB_TYPE_SVC_I_BL (hl_codec_264_defs.h) and I_BL's mb_type
constexpr int32_t ET_SVC_I_BL = 426;
constexpr int32_t kMbTypeIBL = 26;
constexpr int32_t PM_INTRA_BL = 6;  // MbPartPredMode "Intra_BL" (record info only)

// Per-layer constants of the inter-layer derivations (functions of the layer
// sizes and the layer's level_idc only; G.6.1, G.6.3, G.8.6.1.2).
struct SvcGeom {
    int32_t W, H, mbw, mbh;      // this layer
    int32_t rW, rH, rmbw, rmbh;  // reference layer
    int32_t mshX, mshY, mscX, mscY;  // G.6.1: shiftX/Y, scaleX/Y (G-7..G-10)
    int32_t shX[2], shY[2], scX[2], scY[2], addX[2], addY[2], dX[2], dY[2];  // G.6.3 [chromaFlag] (G-43..G-55)
    int32_t mvsX, mvsY;          // G-232, G-233
};

// shiftX/shiftY of G-7/G-43: the reference evaluates Ceil(Log2(refW)) in
// double as (1 / log(2.0)) * log(refW) (hl_math.h:41)
inline int svc_shift(int level_idc, int refdim)
{
    if (level_idc <= 30) return 16;
    const volatile double l2 = (1 / log(2.0)) * log((double)refdim);
    return 31 - (int)ceil(l2);
}

// G.6.1/G.6.3 constants (utils.c:966-1157); no offsets, phases 0 (the SPS
// extension writes chroma_phase_x_plus1_flag = chroma_phase_y_plus1 = 1,
// sps.c:809-813, and the slice inherits them, slice.c:121-129)
inline SvcGeom svc_geom(int W, int H, int rW, int rH, int level_idc)
{
    SvcGeom g{};
    g.W = W;
    g.H = H;
    g.mbw = W / 16;
    g.mbh = H / 16;
    g.rW = rW;
    g.rH = rH;
    g.rmbw = rW / 16;
    g.rmbh = rH / 16;
    g.mshX = svc_shift(level_idc, rW);
    g.mshY = svc_shift(level_idc, rH);
    g.mscX = ((rW << g.mshX) + (W >> 1)) / W;
    g.mscY = ((rH << g.mshY) + (H >> 1)) / H;
    for (int c = 0; c < 2; ++c) {
        const int refW = c ? rW / 2 : rW, refH = c ? rH / 2 : rH, sW = c ? W / 2 : W, sH = c ? H / 2 : H;
        const int phaseX = 0, phaseY = 0, refPhaseX = 0, refPhaseY = 0;
        g.shX[c] = svc_shift(level_idc, refW);
        g.shY[c] = svc_shift(level_idc, refH);
        g.scX[c] = ((refW << g.shX[c]) + (sW >> 1)) / sW;
        g.scY[c] = ((refH << g.shY[c]) + (sH >> 1)) / sH;
        g.addX[c] = (((refW * (2 + phaseX)) << (g.shX[c] - 2)) + (sW >> 1)) / sW + (1 << (g.shX[c] - 5));
        g.addY[c] = (((refH * (2 + phaseY)) << (g.shY[c] - 2)) + (sH >> 1)) / sH + (1 << (g.shY[c] - 5));
        g.dX[c] = 4 * (2 + refPhaseX);
        g.dY[c] = 4 * (2 + refPhaseY);
    }
    g.mvsX = ((W << 16) + (rW >> 1)) / rW;
    g.mvsY = ((H << 16) + (rH >> 1)) / rH;
    return g;
}

// G.8.6.2.3 filters (Table G-9; the chroma table of decode_svc.c:3117)
static constexpr int8_t kRsLuma[16][4] = {{0, 32, 0, 0},   {-1, 32, 2, -1}, {-2, 31, 4, -1}, {-3, 30, 6, -1},
                                          {-3, 28, 8, -1}, {-4, 26, 11, -1}, {-4, 24, 14, -2}, {-3, 22, 16, -3},
                                          {-3, 19, 19, -3}, {-3, 16, 22, -3}, {-2, 14, 24, -4}, {-1, 11, 26, -4},
                                          {-1, 8, 28, -3}, {-1, 6, 30, -3},  {-1, 4, 31, -2},  {-1, 2, 32, -1}};

struct SvcArgs {
    SvcGeom g;
    FrameArgs F;           // this layer: W..mbh, qp, qpc, is_intra, src, cur, ref (chroma), pl/pstride (luma planes)
    const uint8_t* rl[3];  // reference-layer picture (deblocked reconstruction of this access unit)
    const MbState* rst;    // reference-layer macroblock objects of this access unit
    int32_t* unpinned;     // macroblocks outside the pinned scope (see the header)
};

// Reference-layer macroblock types the inter-layer derivations treat as
// intra: HL_CODEC_264_MB_TYPE_IS_I_{PCM,16X16,8X8,4X4,BL} (mb.h:73-77).  In
// I pictures the base layer's MBs are patched to SVC_I_4X4 / SVC_I_16X16
// (mb.c:330-348), enhancement-layer MBs are I_BL: all intra.  In P pictures
// only I_16x16 would match (I_NxN keeps e_type I_NxN); both are unpinned.
HD bool svc_ref_intra(const MbState& m) { return (m.flags & FL_INTRA) != 0; }

// G.6.4 / 6.4.12.4 (mb.h:313-339): (sub-)partition of luma location (x, y) of
// a reference-layer macroblock
HD void svc_part_at(const MbState& m, int x, int y, int& pi, int& spi)
{
    pi = (16 / m.part_w) * (y / m.part_h) + (x / m.part_w);
    if (m.e_type == ET_P8x8 || m.e_type == ET_P8x8REF0) spi = (8 / m.sub_w[pi]) * ((y % 8) / m.sub_h[pi]) + ((x % 8) / m.sub_w[pi]);
    else spi = 0;
}

// Inferred macroblock of an enhancement layer: type, partitioning, motion
// (G.8.1.5.1.1 + G.8.4.1.1 for base_mode_flag = 1)
struct SvcMb {
    int32_t e_type, mb_type, flags, num_part, part_w, part_h;
    int32_t sub_type[4], num_sub[4], sub_w[4], sub_h[4];
    int16_t mv[4][4][2];  // mvL0[mbPartIdx][subMbPartIdx]
    int32_t unpinned;
};

// utils.c:1225-1493 (initialisation), 1677-1709 (G.8.6.1.1 without fix-up),
// 1780-1926 (G.8.6.1.2 without merging), 2010-2216 (G.8.6.1.3, EP),
// 1558-1671 (G.8.4.1.1) for macroblock (mbx, mby) of the layer
HD void svc_derive(const SvcGeom& g, const MbState* rst, bool is_intra_pic, int mbx, int mby, SvcMb& o)
{
    int32_t rmb[4][4], rpi[4][4], rsp[4][4];
    bool intraIL = true, any_intra = false;
    for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) {
            // G.6.1 (G-11..G-15) for (xP, yP) = (4x + 1, 4y + 1)
            const int xC = mbx * 16 + 4 * x + 1, yC = mby * 16 + 4 * y + 1;
            int xRef = (xC * g.mscX + (1 << (g.mshX - 1))) >> g.mshX;
            int yRef = (yC * g.mscY + (1 << (g.mshY - 1))) >> g.mshY;
            xRef = xRef < g.rW - 1 ? xRef : g.rW - 1;
            yRef = yRef < g.rH - 1 ? yRef : g.rH - 1;
            const int a = (yRef >> 4) * g.rmbw + (xRef >> 4);
            rmb[y][x] = a;
            const MbState& m = rst[a];
            if (svc_ref_intra(m)) {
                any_intra = true;
                rpi[y][x] = rsp[y][x] = 0;
            }
            else {
                intraIL = false;
                svc_part_at(m, xRef & 15, yRef & 15, rpi[y][x], rsp[y][x]);
            }
        }
    o.unpinned = (!is_intra_pic && any_intra) ? 1 : 0;
    for (int i = 0; i < 4; ++i) {
        o.sub_type[i] = -1;
        o.num_sub[i] = 1;
        o.sub_w[i] = o.sub_h[i] = 8;
        for (int j = 0; j < 4; ++j) o.mv[i][j][0] = o.mv[i][j][1] = 0;
    }
    if (intraIL) {
        // I_BL (G.8.1.5.1.1 with tcoeff_level_prediction_flag = 0)
        o.e_type = ET_SVC_I_BL;
        o.mb_type = kMbTypeIBL;
        o.flags = FL_INTRA;
        o.num_part = 1;
        o.part_w = o.part_h = 16;
        return;
    }
    // G.8.6.1.2 (RestrictedSpatialResolutionChangeFlag = 1): motion of every
    // 4x4 block from the co-located reference partition, scaled
    int16_t mvIL[4][4][2];
    int32_t refIL[4][4];
    for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) {
            const MbState& m = rst[rmb[y][x]];
            if (svc_ref_intra(m)) {  // unpinned (refLayerPartIdc = -1)
                refIL[y][x] = -1;
                mvIL[y][x][0] = mvIL[y][x][1] = 0;
                continue;
            }
            refIL[y][x] = 0;  // refIdxL0 of a single-reference P picture
            const int ax = m.mv[rpi[y][x]][rsp[y][x]][0], ay = m.mv[rpi[y][x]][rsp[y][x]][1];
            mvIL[y][x][0] = (int16_t)((ax * g.mvsX + 32768) >> 16);  // G-234
            mvIL[y][x][1] = (int16_t)((ay * g.mvsY + 32768) >> 16);  // G-235
        }
    int32_t refP[2][2];
    for (int yP = 0; yP < 2; ++yP)
        for (int xP = 0; xP < 2; ++xP) refP[yP][xP] = refIL[2 * yP][2 * xP];
    // G.8.6.1.3 partition size (utils.c:2030-2123, EP: one list)
    auto same = [&](int x0, int y0, int x1, int y1) -> bool {
        const int vx = mvIL[y0][x0][0], vy = mvIL[y0][x0][1];
        for (int y = y0; y < y1; ++y)
            for (int x = x0; x < x1; ++x)
                if (mvIL[y][x][0] != vx || mvIL[y][x][1] != vy) return false;
        return true;
    };
    int psize = 3;  // 8x8
    if (refP[0][0] == refP[0][1] && refP[0][0] == refP[1][0] && refP[0][0] == refP[1][1] && same(0, 0, 4, 4)) psize = 0;
    else if (refP[0][0] == refP[0][1] && refP[1][0] == refP[1][1] && same(0, 0, 4, 2) && same(0, 2, 4, 4)) psize = 1;
    else if (refP[0][0] == refP[1][0] && refP[0][1] == refP[1][1] && same(0, 0, 2, 4) && same(2, 0, 4, 4)) psize = 2;
    static constexpr int kEt[4] = {ET_P16x16, ET_P16x8, ET_P8x16, ET_P8x8};
    o.e_type = kEt[psize];
    o.mb_type = psize;  // P_L0_16x16, P_L0_L0_16x8, P_L0_L0_8x16, P_8x8 (Table G-7, EP)
    o.flags = FL_INTER;
    o.num_part = psize == 0 ? 1 : (psize == 3 ? 4 : 2);
    o.part_w = (psize == 0 || psize == 1) ? 16 : 8;
    o.part_h = (psize == 0 || psize == 2) ? 16 : 8;
    if (psize == 3) {
        // sub-partition sizes, utils.c:2140-2210; the initialiser
        // "{ HL_CODEC_264_SUBPART_SIZE_4X4 }" sets only [0] to 4x4, so a
        // quadrant matching no shape keeps 8x8 unless it is quadrant 0
        for (int p = 0; p < 4; ++p) {
            const int xO = (p & 1) * 2, yO = (p >> 1) * 2;
            auto eq = [&](int xa, int ya, int xb, int yb) -> bool {
                return mvIL[ya][xa][0] == mvIL[yb][xb][0] && mvIL[ya][xa][1] == mvIL[yb][xb][1];
            };
            int sps = p == 0 ? 3 : 0;
            if (eq(xO, yO, xO + 1, yO) && eq(xO, yO, xO, yO + 1) && eq(xO, yO, xO + 1, yO + 1)) sps = 0;
            else if (eq(xO, yO, xO + 1, yO) && eq(xO, yO + 1, xO + 1, yO + 1)) sps = 1;
            else if (eq(xO, yO, xO, yO + 1) && eq(xO + 1, yO, xO + 1, yO + 1)) sps = 2;
            o.sub_type[p] = sps;  // P_L0_8x8, 8x4, 4x8, 4x4 (Table G-8, EP)
            o.num_sub[p] = sps == 0 ? 1 : (sps == 3 ? 4 : 2);
            o.sub_w[p] = (sps == 0 || sps == 1) ? 8 : 4;
            o.sub_h[p] = (sps == 0 || sps == 2) ? 8 : 4;
        }
    }
    // G.8.4.1.1 (base_mode_flag = 1): mvL0[mbPartIdx][subMbPartIdx] =
    // mvILPredL0 at the (sub-)partition's upper-left 4x4 block (G-93)
    for (int p = 0; p < o.num_part; ++p) {
        const int xP = (p % (16 / o.part_w)) * o.part_w, yP = (p / (16 / o.part_w)) * o.part_h;
        const int ns = psize == 3 ? o.num_sub[p] : 1;
        for (int s = 0; s < ns; ++s) {
            int xS = 0, yS = 0;
            if (psize == 3) {
                xS = (s % (8 / o.sub_w[p])) * o.sub_w[p];
                yS = (s / (8 / o.sub_w[p])) * o.sub_h[p];
            }
            o.mv[p][s][0] = mvIL[(yP + yS) >> 2][(xP + xS) >> 2][0];
            o.mv[p][s][1] = mvIL[(yP + yS) >> 2][(xP + xS) >> 2][1];
        }
        if (refP[yP >> 3][xP >> 3] < 0) o.unpinned = 1;  // predFlagL0 = 0: no prediction in the reference
    }
}

// G.6.3 (utils.c:1067-1157) for chromaFlag c: xRef16 of column xP / yRef16 of
// row yP of macroblock (mbx, mby)
HD int svc_xref16(const SvcGeom& g, int c, int mbx, int xP)
{
    const int xC = xP + ((mbx * 16) >> c);
    return (((xC * g.scX[c] + g.addX[c]) >> (g.shX[c] - 4)) - g.dX[c]);
}
HD int svc_yref16(const SvcGeom& g, int c, int mby, int yP)
{
    const int yC = yP + ((mby * 16) >> c);
    return (((yC * g.scY[c] + g.addY[c]) >> (g.shY[c] - 4)) - g.dY[c]);
}

// One Intra_Base prediction sample (G.8.6.2.2 + G.8.6.2.3 with every
// reference-layer MB intra, so every array sample is available): the
// separable 4-tap (luma) / 2-tap (chroma) interpolation over the reference
// layer's picture with clamped coordinates (G-280, G-281).
HD int svc_resample(const SvcGeom& g, const uint8_t* plane, int c, int mbx, int mby, int x, int y)
{
    const int refW = c ? g.rW / 2 : g.rW, refH = c ? g.rH / 2 : g.rH;
    const int xr16 = svc_xref16(g, c, mbx, x), yr16 = svc_yref16(g, c, mby, y);
    const int xr = xr16 >> 4, yr = yr16 >> 4, xph = xr16 & 15, yph = yr16 & 15;
    auto R = [&](int xx, int yy) -> int { return plane[clip3(0, refH - 1, yy) * refW + clip3(0, refW - 1, xx)]; };
    int v;
    if (c == 0) {
        int acc = 0;
        for (int k = 0; k < 4; ++k) {
            const int xx = xr - 1 + k;
            const int t = kRsLuma[yph][0] * R(xx, yr - 1) + kRsLuma[yph][1] * R(xx, yr) + kRsLuma[yph][2] * R(xx, yr + 1) +
                          kRsLuma[yph][3] * R(xx, yr + 2);
            acc += kRsLuma[xph][k] * t;
        }
        v = (acc + 512) >> 10;
    }
    else {
        const int t0 = (32 - 2 * yph) * R(xr, yr) + 2 * yph * R(xr, yr + 1);
        const int t1 = (32 - 2 * yph) * R(xr + 1, yr) + 2 * yph * R(xr + 1, yr + 1);
        v = ((32 - 2 * xph) * t0 + 2 * xph * t1 + 512) >> 10;
    }
    return clip255(v);
}

// LDS of one enhancement-layer macroblock
struct SvcShared {
    SvcMb mb;
    uint8_t src[256];
    uint8_t srcc[2][64];
    int32_t pred[256];
    int32_t predc[2][64];
    int32_t luma_level[16][16];
    int32_t coded[16];
    int16_t cac[2][4][16];
    int32_t cres_dc[2][4], cres_cac[2][4], cres_cdc[2][4], cres_tc[2][4], cres_sctr[2][4];
    int32_t cbp_cac[2], cbp_cdc[2], cdc_level[2][4];
};

// One enhancement-layer macroblock (rdo.c:1273-1521 / 301-461 and the
// chroma / CBP of rdo.c:2502-2782), lanes tid of nthr.
HD void svc_encode_mb(const SvcArgs& A, SvcShared& S, int addr, int tid, int nthr)
{
    const FrameArgs& F = A.F;
    const int mbx = addr % F.mbw, mby = addr / F.mbw, xL = mbx * 16, yL = mby * 16;
    if (tid == 0) svc_derive(A.g, A.rst, F.is_intra != 0, mbx, mby, S.mb);
    for (int t = tid; t < 256; t += nthr) S.src[t] = F.src[0][(yL + (t >> 4)) * F.W + xL + (t & 15)];
    for (int t = tid; t < 128; t += nthr) {
        const int comp = t >> 6, i = t & 63;
        S.srcc[comp][i] = F.src[1 + comp][((yL >> 1) + (i >> 3)) * F.Wc + (xL >> 1) + (i & 7)];
        // ChromaACLevel of the macroblock object: blocks without residual
        // keep (and the chroma decode reads) the previous picture's levels
        S.cac[comp][(i >> 4) & 3][i & 15] = F.st[addr].cac_level[comp][(i >> 4) & 3][i & 15];
    }
    HL_SYNC();
    const SvcMb& M = S.mb;
    // --- prediction
    if (M.flags & FL_INTRA) {
        // Intra_Base: resampled reference-layer picture (G.8.6.2.1)
        for (int t = tid; t < 256; t += nthr) S.pred[t] = svc_resample(A.g, A.rl[0], 0, mbx, mby, t & 15, t >> 4);
        for (int t = tid; t < 128; t += nthr) {
            const int comp = t >> 6, i = t & 63;
            S.predc[comp][i] = svc_resample(A.g, A.rl[1 + comp], 1, mbx, mby, i & 7, i >> 3);
        }
    }
    else {
        // 8.4.2 with the inferred motion (rdo.c:1350-1445): luma per 4x4
        // block from the quarter-pel planes of the layer's reference picture,
        // the (sub-)partition origin clipped to [-17, W + 17] (interpol.c)
        auto part_of = [&](int lx, int ly, int& pi, int& spi) {
            pi = (16 / M.part_w) * (ly / M.part_h) + (lx / M.part_w);
            spi = M.e_type == ET_P8x8 ? (8 / M.sub_w[pi]) * ((ly % 8) / M.sub_h[pi]) + ((lx % 8) / M.sub_w[pi]) : 0;
        };
        for (int t = tid; t < 16; t += nthr) {
            const int bx = blk_x(t), by = blk_y(t);
            int pi, spi;
            part_of(bx, by, pi, spi);
            const int xP = (pi % (16 / M.part_w)) * M.part_w, yP = (pi / (16 / M.part_w)) * M.part_h;
            int xS = 0, yS = 0;
            if (M.e_type == ET_P8x8) {
                xS = (spi % (8 / M.sub_w[pi])) * M.sub_w[pi];
                yS = (spi / (8 / M.sub_w[pi])) * M.sub_h[pi];
            }
            const int mvx = M.mv[pi][spi][0], mvy = M.mv[pi][spi][1];
            const int X = clip3(-17, F.W + 17, xL + xP + xS + (mvx >> 2)) + bx - xP - xS;
            const int Y = clip3(-17, F.H + 17, yL + yP + yS + (mvy >> 2)) + by - yP - yS;
            int p[16];
            pred_luma4x4(F, X, Y, mvx & 3, mvy & 3, p);
            for (int i = 0; i < 16; ++i) S.pred[(by + (i >> 2)) * 16 + bx + (i & 3)] = p[i];
        }
        // chroma: 8.4.2.2.2 with mvCL0 = mvL0 (8.4.1.4, frame coding)
        for (int t = tid; t < 64; t += nthr) {
            const int cx = t & 7, cy = t >> 3;
            int pi, spi;
            part_of(cx * 2, cy * 2, pi, spi);
            const int mvx = M.mv[pi][spi][0], mvy = M.mv[pi][spi][1];
            const int xi = (xL >> 1) + cx + (mvx >> 3), yi = (yL >> 1) + cy + (mvy >> 3);
            const int xF = mvx & 7, yF = mvy & 7;
            const int xa = clip3(0, F.Wc - 1, xi), xb = clip3(0, F.Wc - 1, xi + 1);
            const int ya = clip3(0, F.Hc - 1, yi), yb = clip3(0, F.Hc - 1, yi + 1);
            for (int comp = 0; comp < 2; ++comp) {
                const uint8_t* r = F.ref[1 + comp];
                S.predc[comp][t] = ((8 - xF) * (8 - yF) * r[ya * F.Wc + xa] + xF * (8 - yF) * r[ya * F.Wc + xb] +
                                    (8 - xF) * yF * r[yb * F.Wc + xa] + xF * yF * r[yb * F.Wc + xb] + 32) >> 6;
            }
        }
    }
    HL_SYNC();
    // --- luma residual (rdo.c:1450-1494): intra rounding, no single-coefficient elimination
    for (int t = tid; t < 16; t += nthr) {
        const int xO = blk_x(t), yO = blk_y(t);
        int res[16];
        bool zero = true;
        for (int i = 0; i < 16; ++i) {
            const int o = (yO + (i >> 2)) * 16 + xO + (i & 3);
            res[i] = (int)S.src[o] - S.pred[o];
            zero = zero && res[i] == 0;
        }
        int q[16];
        bool coded = false;
        if (!zero) {
            int w[16];
            fwd4x4(res, w);
            quant4x4(F.qp, true, w, q);
            bool qz = true;
            for (int i = 0; i < 16; ++i) qz = qz && q[i] == 0;
            coded = !qz;
        }
        for (int i = 0; i < 16; ++i) S.luma_level[t][i] = coded ? q[kZigzag[i]] : 0;
        int r[16];
        if (coded) dequant_idct(F.qp, q, false, r);
        for (int i = 0; i < 16; ++i) {
            const int o = (yO + (i >> 2)) * 16 + xO + (i & 3);
            F.cur[0][(yL + yO + (i >> 2)) * F.W + xL + xO + (i & 3)] = (uint8_t)(coded ? clip255(S.pred[o] + r[i]) : S.pred[o]);
        }
        S.coded[t] = coded;
    }
    // --- chroma (rdo.c:2502-2701): AC with intra rounding, DC with the MB's intra flag
    for (int t = tid; t < 8; t += nthr) {
        const int comp = t >> 2, b = t & 3, xO = (b & 1) * 4, yO = (b >> 1) * 4;
        int res[16];
        bool zero = true;
        for (int i = 0; i < 16; ++i) {
            const int o = (yO + (i >> 2)) * 8 + xO + (i & 3);
            res[i] = (int)S.srcc[comp][o] - S.predc[comp][o];
            zero = zero && res[i] == 0;
        }
        int dc = 0, cacb = 0, cdcb = 0;
        CavlcStat st = {0, 0, 0, -1};
        if (!zero) {
            int w[16], q[16];
            fwd4x4(res, w);
            quant4x4(F.qpc, true, w, q);
            bool az = true;
            for (int i = 1; i < 16; ++i) {
                S.cac[comp][b][i - 1] = (int16_t)q[kZigzag[i]];
                az = az && q[kZigzag[i]] == 0;
            }
            az = az && S.cac[comp][b][15] == 0;  // allzero16 over the 15 AC levels and one more
            dc = w[0];
            cacb = !az;
            cdcb = w[0] != 0;
            if (cacb) st = cavlc_stat(S.cac[comp][b], 16, 15, false);
        }
        S.cres_dc[comp][b] = dc;
        S.cres_cac[comp][b] = cacb;
        S.cres_cdc[comp][b] = cdcb;
        S.cres_tc[comp][b] = st.tc;
        S.cres_sctr[comp][b] = st.sctr;
    }
    HL_SYNC();
    const bool intra = (M.flags & FL_INTRA) != 0;
    int single[2] = {0, 0}, tcs[2] = {0, 0}, cac[2] = {0, 0}, cdc[2] = {0, 0};
    for (int b = 0; b < 4; ++b)
        for (int comp = 0; comp < 2; ++comp) {
            cac[comp] |= S.cres_cac[comp][b] << b;
            cdc[comp] |= S.cres_cdc[comp][b] << b;
            if (single[comp] < 7 && S.cres_cac[comp][b]) {
                single[comp] += S.cres_sctr[comp][b];
                tcs[comp] += S.cres_tc[comp][b];
            }
        }
    for (int comp = 0; comp < 2; ++comp)
        if (single[comp] < 7 && tcs[comp] == 1) cac[comp] = 0;
    int dcl[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    for (int comp = 0; comp < 2; ++comp)
        if (cdc[comp]) {
            const int* D = S.cres_dc[comp];
            const int t00 = D[0] + D[2], t01 = D[1] + D[3], t10 = D[0] - D[2], t11 = D[1] - D[3];
            dcl[comp][0] = quant_dc(F.qpc, intra, t00 + t01);
            dcl[comp][1] = quant_dc(F.qpc, intra, t00 - t01);
            dcl[comp][2] = quant_dc(F.qpc, intra, t10 + t11);
            dcl[comp][3] = quant_dc(F.qpc, intra, t10 - t11);
            cdc[comp] = (dcl[comp][0] ? 1 : 0) | (dcl[comp][1] ? 2 : 0) | (dcl[comp][2] ? 4 : 0) | (dcl[comp][3] ? 8 : 0);
        }
    for (int t = tid; t < 8; t += nthr) {
        const int comp = t >> 2, b = t & 3, xO = (b & 1) * 4, yO = (b >> 1) * 4;
        int r[16];
        bool have = false;
        if (cdc[comp] || cac[comp]) {
            int dcc = 0;
            if (cdc[comp]) {
                const int qP = F.qpc, scale = level_scale(qP % 6, 0, 0);
                const int* L = dcl[comp];
                const int f00 = (L[0] + L[2]) + (L[1] + L[3]), f01 = (L[0] + L[2]) - (L[1] + L[3]);
                const int f10 = (L[0] - L[2]) + (L[1] - L[3]), f11 = (L[0] - L[2]) - (L[1] - L[3]);
                const int f = b == 0 ? f00 : (b == 1 ? f01 : (b == 2 ? f10 : f11));
                dcc = ((f * scale) * (1 << (qP / 6))) >> 5;
            }
            if (dcc || (cac[comp] & (1 << b))) {
                int list[16], m[16];
                list[0] = dcc;
                for (int i = 1; i < 16; ++i) list[i] = S.cac[comp][b][i - 1];
                unscan(list, m);
                dequant_idct(F.qpc, m, true, r);
                have = true;
            }
        }
        for (int i = 0; i < 16; ++i) {
            const int o = (yO + (i >> 2)) * 8 + xO + (i & 3);
            const int v = have ? clip255(S.predc[comp][o] + r[i]) : S.predc[comp][o];
            F.cur[1 + comp][((yL >> 1) + yO + (i >> 2)) * F.Wc + (xL >> 1) + xO + (i & 3)] = (uint8_t)v;
        }
    }
    HL_SYNC();
    // --- CBP (rdo.c:2703-2782), persistent object, record
    MbState& st = F.st[addr];
    MbRecord& R = F.rec[addr];
    for (int t = tid; t < 256; t += nthr) R.luma[t >> 4][t & 15] = (int16_t)S.luma_level[t >> 4][t & 15];
    for (int t = tid; t < 128; t += nthr) {
        R.cac[t >> 6][(t >> 4) & 3][t & 15] = S.cac[t >> 6][(t >> 4) & 3][t & 15];
        st.cac_level[t >> 6][(t >> 4) & 3][t & 15] = S.cac[t >> 6][(t >> 4) & 3][t & 15];
    }
    if (tid == 0) {
        int cbp4 = 0;
        for (int b = 0; b < 16; ++b) cbp4 |= S.coded[b] << b;
        int cbp_l = 0;
        for (int i8 = 0; i8 < 4; ++i8)
            if (cbp4 & (0xF << (i8 * 4))) cbp_l |= 1 << i8;
        int cbp_c;
        if ((cdc[0] || cdc[1]) && (!cac[0] && !cac[1])) cbp_c = 1;
        else if (cac[0] || cac[1]) cbp_c = 2;
        else cbp_c = 0;
        int cbp = (cbp_c << 4) | cbp_l;
        if (cbp > 47) {
            cbp -= 16;
            cbp_c = cbp >> 4;
        }
        st.e_type = M.e_type;
        st.flags = M.flags;
        st.pm0 = intra ? PM_INTRA_BL : PM_L0;
        st.cbp_l = cbp_l;
        st.cbp_c = cbp_c;
        st.cbp_l4x4 = cbp4;
        st.num_part = M.num_part;
        st.part_w = M.part_w;
        st.part_h = M.part_h;
        for (int i = 0; i < 4; ++i) {
            st.sub_w[i] = M.sub_w[i];
            st.sub_h[i] = M.sub_h[i];
            for (int j = 0; j < 4; ++j) {
                st.mv[i][j][0] = M.mv[i][j][0];
                st.mv[i][j][1] = M.mv[i][j][1];
                R.mv[i][j][0] = M.mv[i][j][0];
                R.mv[i][j][1] = M.mv[i][j][1];
                R.mvd[i][j][0] = R.mvd[i][j][1] = 0;
            }
        }
        R.e_type = M.e_type;
        R.mb_type = M.mb_type;
        R.flags = M.flags;
        R.pm0 = st.pm0;
        R.cbp = cbp;
        R.cbp_l = cbp_l;
        R.cbp_c = cbp_c;
        R.cbp_l4x4 = cbp4;
        R.num_part = M.num_part;
        for (int i = 0; i < 4; ++i) {
            R.num_sub[i] = M.num_sub[i];
            R.sub_mb_type[i] = M.sub_type[i];
        }
        for (int comp = 0; comp < 2; ++comp) {
            R.cbp_cac[comp] = cac[comp];
            R.cbp_cdc[comp] = cdc[comp];
            for (int i = 0; i < 4; ++i) R.cdc[comp][i] = (int16_t)dcl[comp][i];
        }
        R.chroma_mode = 0;
        R.i16mode = 0;
        R.mad = 0;
        if (M.unpinned && A.unpinned) {
#if defined(__HIP_DEVICE_COMPILE__)
            atomicAdd(A.unpinned, 1);
#else
            ++*A.unpinned;
#endif
        }
    }
    HL_SYNC();
}

}  // namespace hl
