// hl_coop.h -- the 4x4 residual pipeline of the macroblock search with one
// 16-lane DPP row per 4x4 block (gfx950 only).
//
// Lane p of a row holds raster coefficient (r, c) = (p >> 2, p & 3) of the
// block.  The two 1-D passes of every transform are register exchanges:
// the horizontal pass reads the other lanes of the quad (DPP quad_perm), the
// vertical pass the same column of the other quads (DPP row_ror 4/8/12).
// CAVLC statistics come from two 16-bit masks in scan order (non-zero, +-1)
// built with a row OR-reduction; everything except the level_prefix /
// suffix chain (suffixLength adapts level by level) is then closed-form per
// lane.  Results are bit-identical to the scalar reference paths:
//   forward transform      hl_codec_264_transf.c:716-772   (fwd4x4)
//   quantisation           hl_codec_264_quant.c:116-137     (quant4x4)
//   dequant + inverse      hl_codec_264_transf.c:376-458    (dequant_idct)
//   CAVLC bit count        hl_codec_264_residual.c:587-901  (cavlc_stat)
#pragma once
#include "hl_prims.h"

namespace hl {

template <int CTRL>
__device__ __forceinline__ int dpp(int v)
{
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
constexpr int kQ0 = 0x00, kQ1 = 0x55, kQ2 = 0xAA, kQ3 = 0xFF;  // quad_perm broadcast of quad lane j
constexpr int kRor1 = 0x121, kRor2 = 0x122, kRor4 = 0x124, kRor8 = 0x128, kRor12 = 0x12C;

// sum / or / max over the 16 lanes of a DPP row (every lane gets the result)
__device__ __forceinline__ int row_sum(int x)
{
    x += dpp<kRor8>(x);
    x += dpp<kRor4>(x);
    x += dpp<kRor2>(x);
    return x + dpp<kRor1>(x);
}
__device__ __forceinline__ int row_or(int x)
{
    x |= dpp<kRor8>(x);
    x |= dpp<kRor4>(x);
    x |= dpp<kRor2>(x);
    return x | dpp<kRor1>(x);
}
__device__ __forceinline__ int row_max(int x)
{
    x = max(x, dpp<kRor8>(x));
    x = max(x, dpp<kRor4>(x));
    x = max(x, dpp<kRor2>(x));
    return max(x, dpp<kRor1>(x));
}

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v)
{
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)dpp<CTRL>((int)(unsigned)b), hi = (unsigned)dpp<CTRL>((int)(unsigned)(b >> 32));
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double row_min_f64(double x)
{
    x = fmin(x, dpp_f64<kRor8>(x));
    x = fmin(x, dpp_f64<kRor4>(x));
    x = fmin(x, dpp_f64<kRor2>(x));
    return fmin(x, dpp_f64<kRor1>(x));
}

// Per-lane constants.  The coefficient fields are packed 4 bits per source
// (signed 3-bit coefficient + a shift bit for the IDCT's >>1 terms) and
// decoded with bit-field extracts.
struct LaneK {
    int p, s;          // raster position in the block, zig-zag scan index
    uint32_t fwd;      // [0..15] horizontal, [16..31] vertical forward coefficients
    uint32_t inv;      // same for the inverse transform (coef | shift << 3)
    uint32_t had;      // same for the 4x4 Hadamard (I16x16 DC)
    int mf, mfc;       // quant multiplier at qp / qpc for this position
    int ls, lsc;       // dequant level scale at qp / qpc for this position
};

// forward core matrix and the IDCT's (coefficient, shift) for out o, in i
HD int fwd_m(int o, int i)
{
    const int m[4][4] = {{1, 1, 1, 1}, {2, 1, -1, -2}, {1, -1, -1, 1}, {1, -2, 2, -1}};
    return m[o][i];
}
HD int had_m(int o, int i)
{
    const int m[4][4] = {{1, 1, 1, 1}, {1, 1, -1, -1}, {1, -1, -1, 1}, {1, -1, 1, -1}};
    return m[o][i];
}
HD int inv_c(int o, int i)
{
    if (i == 0) return 1;
    if (i == 2) return (o == 0 || o == 3) ? 1 : -1;
    if (i == 1) return o < 2 ? 1 : -1;
    return (o & 1) ? -1 : 1;
}
HD int inv_s(int o, int i)
{
    if (i == 1) return (o == 1 || o == 2) ? 1 : 0;
    if (i == 3) return (o == 0 || o == 3) ? 1 : 0;
    return 0;
}

__device__ __forceinline__ LaneK make_lanek(int tid, int qp, int qpc)
{
    static constexpr uint8_t kZzInv[16] = {0, 1, 5, 6, 2, 4, 7, 12, 3, 8, 11, 13, 9, 10, 14, 15};
    LaneK K;
    const int p = tid & 15, r = p >> 2, c = p & 3;
    K.p = p;
    int s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s = (p == i) ? kZzInv[i] : s;
    K.s = s;
    // source rows the vertical rotations read (direction-agnostic: rotate the row index itself)
    const int rr[4] = {r, dpp<kRor4>(tid & 15) >> 2, dpp<kRor8>(tid & 15) >> 2, dpp<kRor12>(tid & 15) >> 2};
    uint32_t fw = 0, iv = 0, hd = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        fw |= (uint32_t)(fwd_m(c, j) & 0xF) << (4 * j);
        fw |= (uint32_t)(fwd_m(r, rr[j]) & 0xF) << (16 + 4 * j);
        hd |= (uint32_t)(had_m(c, j) & 0xF) << (4 * j);
        hd |= (uint32_t)(had_m(r, rr[j]) & 0xF) << (16 + 4 * j);
        iv |= (uint32_t)((inv_c(c, j) & 7) | (inv_s(c, j) << 3)) << (4 * j);
        iv |= (uint32_t)((inv_c(r, rr[j]) & 7) | (inv_s(r, rr[j]) << 3)) << (16 + 4 * j);
    }
    K.fwd = fw;
    K.inv = iv;
    K.had = hd;
    const int cls = ((r & 1) == 0 && (c & 1) == 0) ? 0 : (((r & 1) && (c & 1)) ? 1 : 2);
    int mf = 0, mfc = 0, ls = 0, lsc = 0;
#pragma unroll
    for (int m = 0; m < 6; ++m)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (m == qp % 6 && k == cls) {
                mf = kQuantMF[m][k];
                ls = 16 * kScaleV[m][k];
            }
            if (m == qpc % 6 && k == cls) {
                mfc = kQuantMF[m][k];
                lsc = 16 * kScaleV[m][k];
            }
        }
    K.mf = mf;
    K.mfc = mfc;
    K.ls = ls;
    K.lsc = lsc;
    return K;
}

__device__ __forceinline__ int fld_s3(uint32_t w, int pos) { return ((int)(w << (29 - pos))) >> 29; }  // signed bits [pos, pos+2]
__device__ __forceinline__ int fld_u1(uint32_t w, int pos) { return (w >> (pos + 3)) & 1; }

// M X M^T for the packed matrix f (exact integer arithmetic), one
// coefficient per lane.
__device__ __forceinline__ int coop_lin(uint32_t f, int x)
{
    const int q0 = dpp<kQ0>(x), q1 = dpp<kQ1>(x), q2 = dpp<kQ2>(x), q3 = dpp<kQ3>(x);
    // |values| < 2^23 on every path (residuals, DC sums), so 24-bit multiplies are exact
    const int h = __mul24(fld_s3(f, 0), q0) + __mul24(fld_s3(f, 4), q1) + __mul24(fld_s3(f, 8), q2) + __mul24(fld_s3(f, 12), q3);
    const int v1 = dpp<kRor4>(h), v2 = dpp<kRor8>(h), v3 = dpp<kRor12>(h);
    return __mul24(fld_s3(f, 16), h) + __mul24(fld_s3(f, 20), v1) + __mul24(fld_s3(f, 24), v2) + __mul24(fld_s3(f, 28), v3);
}
// forward core transform (transf.c:716-772)
__device__ __forceinline__ int coop_fwd(const LaneK& K, int x) { return coop_lin(K.fwd, x); }

// Inverse core transform (rows, then columns, then (x + 32) >> 6).
__device__ __forceinline__ int coop_idct(const LaneK& K, int d)
{
    const int q0 = dpp<kQ0>(d), q1 = dpp<kQ1>(d), q2 = dpp<kQ2>(d), q3 = dpp<kQ3>(d);
    const uint32_t w = K.inv;
    // dequantised coefficients stay below 2^22 in magnitude (level < 2^13, scale <= 464)
    const int f = __mul24(fld_s3(w, 0), q0 >> fld_u1(w, 0)) + __mul24(fld_s3(w, 4), q1 >> fld_u1(w, 4)) +
                  __mul24(fld_s3(w, 8), q2 >> fld_u1(w, 8)) + __mul24(fld_s3(w, 12), q3 >> fld_u1(w, 12));
    const int v1 = dpp<kRor4>(f), v2 = dpp<kRor8>(f), v3 = dpp<kRor12>(f);
    const int h = __mul24(fld_s3(w, 16), f >> fld_u1(w, 16)) + __mul24(fld_s3(w, 20), v1 >> fld_u1(w, 20)) +
                  __mul24(fld_s3(w, 24), v2 >> fld_u1(w, 24)) + __mul24(fld_s3(w, 28), v3 >> fld_u1(w, 28));
    return (h + 32) >> 6;
}

// LDS tables of the cooperative pipeline
struct CoopTables {
    uint8_t tz[15][16];      // total_zeros lengths
    uint8_t tok[3][4][17];   // coeff_token lengths, nC < 8
    uint8_t pad[4];
    uint8_t rb[16][16];      // run_before lengths [zerosLeft][run] (0 for zerosLeft 0 and run > zerosLeft)
    uint32_t tok3[4][17];    // [t1][tc]: the coeff_token lengths of nC classes 0-2 in 5-bit fields, 6 (class 3) at bit 15
};

// CoopTables::rb as a constant (Table 9-10 by zerosLeft and run)
struct RbTab {
    uint8_t v[16][16];
};
constexpr RbTab make_rb_tab()
{
    RbTab t{};
    for (int zl = 1; zl < 16; ++zl)
        for (int run = 0; run <= zl && run < 15; ++run) t.v[zl][run] = kRbLen[zl <= 6 ? zl - 1 : 6][run];
    return t;
}
constexpr RbTab kRbTab = make_rb_tab();
struct Tok3Tab {
    uint32_t v[4][17];
};
constexpr Tok3Tab make_tok3_tab()
{
    Tok3Tab t{};
    for (int t1 = 0; t1 < 4; ++t1)
        for (int tc = 0; tc < 17; ++tc)
            t.v[t1][tc] = (uint32_t)kTokLen[0][t1][tc] | (uint32_t)kTokLen[1][t1][tc] << 5 | (uint32_t)kTokLen[2][t1][tc] << 10 | 6u << 15;
    return t;
}
constexpr Tok3Tab kTok3Tab = make_tok3_tab();

__device__ __forceinline__ void coop_tables_init(CoopTables& T, int tid, int nthr)
{
    for (int i = tid; i < 15 * 16; i += nthr) T.tz[i >> 4][i & 15] = kTzLen[i >> 4][i & 15];
    for (int i = tid; i < 3 * 4 * 17; i += nthr) T.tok[i / 68][(i / 17) % 4][i % 17] = kTokLen[i / 68][(i / 17) % 4][i % 17];
    for (int i = tid; i < 16 * 16; i += nthr) T.rb[i >> 4][i & 15] = kRbTab.v[i >> 4][i & 15];
    for (int i = tid; i < 4 * 17; i += nthr) T.tok3[i / 17][i % 17] = kTok3Tab.v[i / 17][i % 17];
}

__device__ __forceinline__ int coop_token_len(const CoopTables& T, int nC, int tc, int t1)
{
    return nC >= 8 ? 6 : T.tok[nC < 2 ? 0 : (nC < 4 ? 1 : 2)][t1][tc];
}

// run_before length, Table 9-10 (kRbLen) in closed form
__device__ __forceinline__ int rb_len(int zl, int run)
{
    if (zl > 6) return run < 7 ? 3 : run - 3;
    // rows zerosLeft 1..6, two bits per run value
    const uint32_t rows[6] = {0x5u, 0x29u, 0xAAu, 0x3EAu, 0xFFAu, 0x3FFEu};
    uint32_t w = rows[0];
#pragma unroll
    for (int i = 1; i < 6; ++i) w = zl == i + 1 ? rows[i] : w;
    return (w >> (2 * run)) & 3;
}

// level_prefix + level_suffix length (level_code_len of hl_prims.h), branch-free
__device__ __forceinline__ int level_len(int sl, int lc)
{
    const int l0 = lc < 14 ? lc + 1 : (lc < 30 ? 19 : (lc <= 4126 ? 28 : 1));
    const int l1 = lc < (14 << sl) ? (lc >> sl) + 1 + sl : (lc < (15 << sl) ? 15 + sl : (lc <= (15 << sl) + 4096 ? 28 : 1));
    return sl == 0 ? l0 : l1;
}
// suffixLength update after a level of magnitude a (residual.c:813-858)
__device__ __forceinline__ int next_sl(int sl, int a)
{
    const int s1 = sl == 0 ? 1 : sl;
    const int thr = s1 < 6 ? 3 << (s1 - 1) : 32768;
    return s1 + (a > thr ? 1 : 0);
}

struct CoopStat {
    int tc, t1, rest, sctr;  // as CavlcStat (uniform over the row)
};

// CAVLC statistics of the row's block (cavlc_stat with maxNumCoef 16,
// endIdx 15).  L = this lane's level, li = its list index (scan index, or
// scan index - 1 for AC blocks; -1 = not part of the list).  lvs = 16 words
// of LDS scratch owned by this row (16-byte aligned).
__device__ __forceinline__ CoopStat coop_cavlc(const CoopTables& T, int L, int li, int* lvs)
{
    const int aL = L < 0 ? -L : L;
    const bool nzl = li >= 0 && L != 0;
    const uint32_t masks = (uint32_t)row_or(nzl ? (int)((1u << li) | ((uint32_t)(aL == 1) << (li + 16))) : 0);
    const uint32_t nz = masks & 0xFFFFu, ones = masks >> 16;
    CoopStat st;
    const int tc = __popc(nz);
    const int hi = 31 - __clz(nz | 1u);
    const uint32_t big = nz & ~ones;
    const int hb = big ? 31 - __clz(big) : -1;
    const int t1a = __popc(nz >> (hb + 1));
    const int t1 = t1a < 3 ? t1a : 3;
    // total_zeros length (issued early: independent of the level chain)
    const int tzb = (tc > 0 && tc < 16) ? T.tz[tc - 1][hi + 1 - tc] : 0;
    // this lane's order from the top, run_before and level code
    const int lis = li < 0 ? 0 : li;
    const int j = __popc(nz >> (lis + 1));
    const uint32_t lower = nz & ((1u << lis) - 1u);
    const int zl = lis - __popc(lower);
    const int run = lower ? lis - 1 - (31 - __clz(lower)) : lis;
    const int rb = (nzl && j < tc - 1 && zl > 0) ? rb_len(zl, run) : 0;
    const int m = j - t1;
    int lc = L > 0 ? (L << 1) - 2 : -(L << 1) - 1;
    lc -= (m == 0 && t1 < 3 && lc >= 2) ? 2 : 0;
    const bool lvl = nzl && m >= 0;  // a level coded with level_prefix/suffix
    const int sl0 = (tc > 10 && t1 < 3) ? 1 : 0;
    // Fast path: no level above 3 in magnitude.  suffixLength is then sl0 for
    // the first level and 1 for every later one (it only grows past 1 for
    // |level| > 3), so every length is known without the chain:
    // suffixLength 0: lc + 1 (lc < 14), 1: (lc >> 1) + 2 (lc < 28).
    const int row_in_wave = (__lane_id() >> 4) & 3;
    const bool slow = ((__ballot(lvl && aL > 3) >> (16 * row_in_wave)) & 0xFFFFull) != 0;  // uniform per row
    const int len = (lvl && !slow) ? ((m == 0 && sl0 == 0) ? lc + 1 : (lc >> 1) + 2) : 0;
    int bits = t1 + tzb + row_sum(rb + len);
    if (slow) {
        if (lvl) lvs[m] = (lc << 16) | aL;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        int sl = sl0;
        for (int k = 0; k < tc - t1; ++k) {
            const int v = lvs[k];
            bits += level_len(sl, v >> 16);
            sl = next_sl(sl, v & 0xFFFF);
        }
    }
    st.tc = tc;
    st.t1 = tc ? t1 : 0;
    st.rest = tc ? bits : 0;
    st.sctr = tc == 0 ? -1 : ((tc == 1 && ones == nz) ? (hi == 0 ? 3 : (hi < 3 ? 2 : (hi < 6 ? 1 : 0))) : 9);
    return st;
}

// quantisation of one coefficient: f = 2^qbits / 3 (intra) or / 6 (inter)
__device__ __forceinline__ int coop_quant(int w, int mf, int qbits, int f)
{
    const int v = (int)((__umul24((unsigned)(w < 0 ? -w : w), (unsigned)mf) + (unsigned)f) >> qbits);  // < 2^32
    return w >= 0 ? v : -v;
}
__device__ __forceinline__ int coop_dequant(int c, int ls, int qP)
{
    const int q6 = qP / 6;
    const int p = __mul24(c, ls);
    return qP >= 24 ? p * (1 << (q6 - 4)) : (p + (1 << (3 - q6))) >> (4 - q6);
}

}  // namespace hl
