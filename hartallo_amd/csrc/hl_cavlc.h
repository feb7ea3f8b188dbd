// hl_cavlc.h -- the CAVLC macroblock_layer() of enhancement-layer slices as
// __host__ __device__ code, for serialising a whole slice on the GPU: every
// macroblock's bit count first (BitCount), an exclusive scan of the counts,
// then every macroblock writes its bits at its offset (BitOr, big-endian
// 32-bit words, atomicOr where two macroblocks share a word).  The syntax
// and every table are those of the host writer (hl_writer.cpp write_block,
// write_svc_mb_range; residual.c:587-901, mb.c:543-892).
#pragma once
#include "hl_prims.h"
#include "hl_types.h"

namespace hl {

struct BitCount {
    int64_t pos = 0;
    HD void u(uint32_t, int n) { pos += n; }
};

// n <= 32 bits of v, MSB first, at bit `pos` of a zeroed big-endian word buffer
struct BitOr {
    uint32_t* w;
    int64_t pos;
    HD void orw(uint32_t* p, uint32_t v)
    {
#if defined(__HIP_DEVICE_COMPILE__)
        if (v) atomicOr(p, v);
#else
        *p |= v;
#endif
    }
    HD void u(uint32_t v, int n)
    {
        if (n <= 0) return;
        if (n < 32) v &= (1u << n) - 1u;
        const int off = (int)(pos & 31), room = 32 - off;
        uint32_t* p = w + (pos >> 5);
        if (n <= room) orw(p, v << (room - n));
        else {
            orw(p, v >> (n - room));
            orw(p + 1, v << (32 - (n - room)));
        }
        pos += n;
    }
};

template <class B>
HD void bits_ue(B& b, uint32_t v)
{
    int lz = 0;
    while ((1ull << (lz + 1)) <= (uint64_t)v + 1) ++lz;
    b.u(0, lz);
    b.u(v + 1, lz + 1);
}
template <class B>
HD void bits_se(B& b, int32_t v)
{
    bits_ue(b, v <= 0 ? (uint32_t)(-(int64_t)v) << 1 : ((uint32_t)v << 1) - 1);
}

// level_prefix / level_suffix of the reference's generated table
// (cavlc.c:59-103; hl_writer.cpp init_levels), in closed form
HD void level_code_parts(int sl, int lc, int& prefix, int& size, uint32_t& suffix)
{
    if (sl == 0) {
        if (lc < 14) prefix = lc, size = 0, suffix = 0;
        else if (lc < 30) prefix = 14, size = 4, suffix = (uint32_t)(lc - 14);
        else if (lc <= 4126) prefix = 15, size = 12, suffix = (uint32_t)(lc - 30);
        else prefix = 0, size = 0, suffix = 0;
        return;
    }
    if (lc < (15 << sl)) prefix = lc >> sl, size = sl, suffix = (uint32_t)(lc & ((1 << sl) - 1));
    else if (lc <= (15 << sl) + 4096) prefix = 15, size = 12, suffix = (uint32_t)(lc - (15 << sl));
    else prefix = 0, size = 0, suffix = 0;
}

// coded_block_pattern -> codeNum, inter column of Table 9-4 (hl_writer.cpp kCbpCode)
static constexpr uint8_t kCbpInter[48] = {0,  2,  3,  7,  4,  8,  17, 13, 5,  18, 9,  14, 10, 15, 16, 11, 1,  32, 33, 36, 34, 37, 44, 40,
                                          35, 45, 38, 41, 39, 42, 43, 19, 6,  24, 25, 20, 26, 21, 46, 28, 27, 47, 22, 29, 23, 30, 31, 12};

// residual_block_cavlc (residual.c:587-901, write path)
template <class B, typename T>
HD void cavlc_block(B& bw, const T* coeffLevel, int endIdx, int maxNumCoef, int nC)
{
    int nz[16], run_before[16];
    for (int j = 0; j < 16; ++j) run_before[j] = 0;
    int tc = 0, t1 = 0, total_zeros = 0, k = -1;
    bool countT1 = true, countTZ = false;
    for (int j = 0; j < maxNumCoef; ++j) {
        const int c = coeffLevel[maxNumCoef - 1 - j];
        if (c) {
            nz[tc++] = c;
            countTZ = true;
            ++k;
            if (countT1) {
                if (c == 1 || c == -1) {
                    ++t1;
                    countT1 = t1 < 3;
                }
                else {
                    countT1 = false;
                }
            }
        }
        else if (countTZ) {
            ++run_before[k];
        }
        if (countTZ && c == 0) ++total_zeros;
    }
    if (nC >= 0) {
        if (nC >= 8) bw.u(tc ? (uint32_t)(((tc - 1) << 2) | t1) : 3u, 6);
        else {
            const int vlc = nC < 2 ? 0 : (nC < 4 ? 1 : 2);
            bw.u(kTokCode[vlc][t1][tc], kTokLen[vlc][t1][tc]);
        }
    }
    else {
        bw.u(kTokCdcCode[t1][tc], kTokCdcLen[t1][tc]);
    }
    if (tc == 0) return;
    int suffixLength = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int j = 0; j < tc; ++j) {
        if (j < t1) {
            bw.u((uint32_t)((1 - nz[j]) >> 1) & 1u, 1);
            continue;
        }
        int lc = nz[j] >= 0 ? nz[j] * 2 - 2 : -(nz[j] * 2) - 1;
        if (j == t1 && t1 < 3 && lc >= 2) lc -= 2;
        int prefix, size;
        uint32_t suffix;
        level_code_parts(suffixLength, lc, prefix, size, suffix);
        if (prefix > 0) bw.u(0, prefix);
        bw.u(1, 1);
        if (size) bw.u(suffix, size);
        if (suffixLength == 0) suffixLength = 1;
        const int thr = suffixLength == 1 ? 3 : (suffixLength == 2 ? 6 : (suffixLength == 3 ? 12 : (suffixLength == 4 ? 24 : (suffixLength == 5 ? 48 : 32768))));
        if (iabs(nz[j]) > thr) ++suffixLength;
    }
    int zerosLeft = 0;
    if (tc < endIdx + 1) {
        if (nC >= 0) bw.u(kTzCode[tc - 1][total_zeros], kTzLen[tc - 1][total_zeros]);
        else bw.u(kTzCdcCode[tc - 1][total_zeros], kTzCdcLen[tc - 1][total_zeros]);
        zerosLeft = total_zeros;
    }
    for (k = 0; k < tc - 1 && zerosLeft > 0; ++k) {
        const int row = zerosLeft <= 6 ? zerosLeft - 1 : 6;
        bw.u(kRbCode[row][run_before[k]], kRbLen[row][run_before[k]]);
        zerosLeft -= run_before[k];
    }
}

// TotalCoeff the reference leaves on the macroblock objects for nC
// (residual.c:796-806; uncoded 8x8 / chroma-AC groups count as 0, utils.h:10-20)
HD int el_tc_luma(const MbRecord& m, int blk)
{
    if (!(m.cbp_l & (1 << (blk >> 2)))) return 0;
    int k = 0;
    for (int i = 0; i < 16; ++i) k += m.luma[blk][i] != 0;
    return k;
}
HD int el_tc_cac(const MbRecord& m, int comp, int b)
{
    if (!(m.cbp_c & 2) || !(m.cbp_cac[comp] & (1 << b))) return 0;
    int k = 0;
    for (int i = 0; i < 15; ++i) k += m.cac[comp][b][i] != 0;
    return k;
}

// macroblock_layer_in_scalable_extension of enhancement-layer macroblock a
// (base_mode_flag = 1, mb.c:543-892), as write_svc_mb_range writes it
template <class B>
HD void el_mb_bits(B& bw, const MbRecord* recs, int a, int mbw, bool idr)
{
    static constexpr int16_t kZ[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const MbRecord& m = recs[a];
    const int mbx = a % mbw, mby = a / mbw;
    if (!idr) bw.u(1, 1);  // mb_skip_run ue(0)
    bw.u(1, 1);            // base_mode_flag
    if (!idr) bw.u(0, 1);  // residual_prediction_flag
    bits_ue(bw, kCbpInter[m.cbp]);
    if (!(m.cbp_l > 0 || m.cbp_c > 0)) return;
    bw.u(1, 1);  // mb_qp_delta se(0)
    for (int i8 = 0; i8 < 4; ++i8)
        for (int i4 = 0; i4 < 4; ++i4) {
            if (!(m.cbp_l & (1 << i8))) continue;
            const int blk = i8 * 4 + i4, bx = blk_x(blk), by = blk_y(blk);
            int nA = 0, nB = 0;
            bool aA = true, aB = true;
            if (bx) nA = el_tc_luma(m, blk_idx(bx - 4, by));
            else if (mbx) nA = el_tc_luma(recs[a - 1], blk_idx(12, by));
            else aA = false;
            if (by) nB = el_tc_luma(m, blk_idx(bx, by - 4));
            else if (mby) nB = el_tc_luma(recs[a - mbw], blk_idx(bx, 12));
            else aB = false;
            const int nC = aA && aB ? (nA + nB + 1) >> 1 : (aA ? nA : (aB ? nB : 0));
            cavlc_block(bw, m.luma[blk], 15, 16, nC);
        }
    if (m.cbp_c & 3)
        for (int c = 0; c < 2; ++c) cavlc_block(bw, m.cbp_cdc[c] ? m.cdc[c] : kZ, 3, 4, -1);
    if (m.cbp_c & 2)
        for (int c = 0; c < 2; ++c)
            for (int i4 = 0; i4 < 4; ++i4) {
                int nA = 0, nB = 0;
                bool aA = true, aB = true;
                if (i4 & 1) nA = el_tc_cac(m, c, i4 - 1);
                else if (mbx) nA = el_tc_cac(recs[a - 1], c, i4 + 1);
                else aA = false;
                if (i4 & 2) nB = el_tc_cac(m, c, i4 - 2);
                else if (mby) nB = el_tc_cac(recs[a - mbw], c, i4 + 2);
                else aB = false;
                const int nC = aA && aB ? (nA + nB + 1) >> 1 : (aA ? nA : (aB ? nB : 0));
                cavlc_block(bw, (m.cbp_cac[c] & (1 << i4)) ? m.cac[c][i4] : kZ, 14, 15, nC);
            }
}

}  // namespace hl
