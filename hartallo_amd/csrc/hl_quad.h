// hl_quad.h -- the 4x4 residual pipeline of the macroblock search with one
// 4-lane quad per 4x4 block (gfx950 only).
//
// Lane r of a quad holds row r of the block, its four samples / coefficients
// in registers.  A 64-lane wave therefore evaluates 16 blocks per
// instruction stream (the 16-lane rows of hl_coop.h: 4), and a 512-lane
// workgroup 128 blocks per round -- a whole 16x16 step (9 candidates x 16
// blocks) in two rounds instead of five.  Row passes of the transforms are
// register arithmetic; column passes read the other rows of the quad with
// DPP quad_perm broadcasts; block sums / ORs are two quad_perm exchanges.
// CAVLC statistics: the scan-order masks OR-reduced over the quad, then the
// same closed forms as hl_coop.h per coefficient, summed in the lane and over
// the quad.  Results are bit-identical to the scalar reference paths
// (hl_prims.h fwd4x4 / quant4x4 / dequant_idct / cavlc_stat):
//   forward transform      hl_codec_264_transf.c:716-772
//   quantisation           hl_codec_264_quant.c:116-137
//   dequant + inverse      hl_codec_264_transf.c:376-458
//   CAVLC bit count        hl_codec_264_residual.c:587-901
#pragma once
#include "hl_coop.h"

namespace hl {

constexpr int kQX1 = 0xB1, kQX2 = 0x4E, kQX3 = 0x1B;  // quad_perm lane ^ 1, lane ^ 2, lane ^ 3

// A DPP read kept as its own v_mov_b32_dpp: the empty asm stops LLVM's DPP
// combiner from folding it into the subtraction that consumes it.  On the
// MI355X a folded v_subrev_u32_dpp returned src1 - src0 of the lane's own
// src0, without the permutation (tests/test_gpu_unit.py, quad, every QP: the
// odd rows of the forward transform's first column); the column passes below
// subtract DPP operands, so they read them through this.
template <int CTRL>
__device__ __forceinline__ int dpp_x(int v)
{
    // mov_dpp (no "old" operand: every lane of a quad is written, so no
    // zero-initialised destination has to be materialised first)
    int r = __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
    asm volatile("" : "+v"(r));
    return r;
}

__device__ __forceinline__ int quad_sum(int x)
{
    x += dpp<kQX1>(x);
    return x + dpp<kQX2>(x);
}
__device__ __forceinline__ int quad_or(int x)
{
    x |= dpp<kQX1>(x);
    return x | dpp<kQX2>(x);
}

// Per-lane constants of the quad pipeline at one QP.
struct LaneQ {
    int r;          // the block row this lane holds (samples and residual)
    // the rest belong to coefficient row quad_coef_row(r)
    int mfE, mfO;   // quantisation multipliers of the row's even / odd columns
    int lsE, lsO;   // dequantisation level scales, same
    uint32_t zz;    // scan index of (r, c) in bits [4c, 4c + 3]
};

// The coefficient row lane r of a quad holds between quad_fwd and quad_idct:
// the two-stage butterflies below leave rows 1 and 2 swapped (0, 2, 1, 3).
__device__ __forceinline__ int quad_coef_row(int r) { return ((r & 1) << 1) | (r >> 1); }

// kZzInv[r * 4 + c]: scan index of raster position (r, c)
constexpr uint64_t kZzRows = 0xFEA9DB83C7426510ull;  // rows of {0,1,5,6},{2,4,7,12},{3,8,11,13},{9,10,14,15}, 4 bits each

// LaneQ::zz recomputed from an opaque copy of the lane's row where a phase
// starts: a zz held from the MB's start was spilled across the searches
__device__ __forceinline__ uint32_t laneq_zz_fresh(int r)
{
    asm volatile("" : "+v"(r));
    return (uint32_t)(kZzRows >> (16 * quad_coef_row(r))) & 0xFFFFu;
}

__device__ __forceinline__ LaneQ make_laneq(int tid, int qp)
{
    LaneQ Q;
    Q.r = tid & 3;
    const int r = quad_coef_row(Q.r);  // the quantiser's, scan's and dequantiser's row
    Q.zz = (uint32_t)(kZzRows >> (16 * r)) & 0xFFFFu;
    const int m = qp % 6;
    const int clsE = (r & 1) ? 2 : 0, clsO = (r & 1) ? 1 : 2;
    int mfE = 0, mfO = 0, lsE = 0, lsO = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k)
        if (k == m) {
            mfE = clsE == 0 ? kQuantMF[k][0] : kQuantMF[k][2];
            mfO = clsO == 1 ? kQuantMF[k][1] : kQuantMF[k][2];
            lsE = 16 * (clsE == 0 ? kScaleV[k][0] : kScaleV[k][2]);
            lsO = 16 * (clsO == 1 ? kScaleV[k][1] : kScaleV[k][2]);
        }
    Q.mfE = mfE;
    Q.mfO = mfO;
    // the level scales pre-shifted by 8.5.12.1's left shift at qp >= 24
    // (quad_idct then only adds its rounding and shifts right below 24)
    const int sa = qp >= 24 ? qp / 6 - 4 : 0;
    Q.lsE = lsE << sa;
    Q.lsO = lsO << sa;
    return Q;
}

// Forward core transform Cf X Cf^T: x = row r of the residual, y = row
// quad_coef_row(r) of the coefficients.  Exact integer arithmetic: the pass
// order does not matter.  The column pass is two butterfly stages with one
// DPP read each (rows a, b, e, d = 0..3):
//   stage 1, partner r ^ 3: a + d | b + e | b - e | a - d   (p + s1 x)
//   stage 2, partner r ^ 1: y0 = (a+d) + (b+e), y2 = (a+d) - (b+e),
//                           y1 = 2 (a-d) + (b-e), y3 = (a-d) - 2 (b-e)
// |values| <= 9180 (8-bit residuals), so the 24-bit multiplies are exact.
// A per-lane weight the compiler must treat as unknown: it otherwise turns
// each multiply by a +-1 select into a negate and a select (two instructions
// per use instead of one multiply-add).
__device__ __forceinline__ int opaque_w(int w)
{
    asm volatile("" : "+v"(w));
    return w;
}

__device__ __forceinline__ void quad_fwd(const LaneQ& Q, const int x[4], int y[4])
{
    const int s03 = x[0] + x[3], d03 = x[0] - x[3], s12 = x[1] + x[2], d12 = x[1] - x[2];
    const int h[4] = {s03 + s12, (d03 << 1) + d12, s03 - s12, d03 - (d12 << 1)};
    const int s1 = opaque_w(Q.r < 2 ? 1 : -1), kx = opaque_w(Q.r == 1 ? -1 : 1), kp = opaque_w(Q.r < 2 ? 1 : (Q.r == 2 ? 2 : -2));
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int t = __mul24(h[c], s1) + dpp_x<kQX3>(h[c]);
        y[c] = __mul24(dpp_x<kQX1>(t), kp) + __mul24(t, kx);
    }
}

// AC quantisation of one coefficient: f = 2^qbits / 3 (intra) or / 6 (inter)
__device__ __forceinline__ int quad_q1(int w, int mf, int qbits, int f)
{
    const int v = (int)((__umul24((unsigned)(w < 0 ? -w : w), (unsigned)mf) + (unsigned)f) >> qbits);  // < 2^32
    return w >= 0 ? v : -v;
}

// Dequantisation (8.5.12.1) and inverse transform (rows first, then columns,
// then (x + 32) >> 6, transf.c:376-458): q = coefficient row
// quad_coef_row(r) of the levels (raster), out = row r of the residual.  The
// column pass as two butterfly stages (input rows f0, f2, f1, f3 in lanes
// 0..3):
//   stage 1, partner r ^ 1: g0 = f0 + f2 | g1 = f0 - f2 | g2 = (f1 >> 1) - f3 | g3 = f1 + (f3 >> 1)
//   stage 2, partner r ^ 3: h0 = g0 + g3 | h1 = g1 + g2 | h2 = g1 - g2 | h3 = g0 - g3
// Dequantised values stay below 2^18 and every sum below 2^22 for levels of
// 8-bit residuals at any QP, so the 24-bit multiplies are exact.
// keep_dc: coefficient (0, 0) is dcv, already scaled (Intra16x16 luma and
// chroma: dequant_idct's keep_dc), in the lane holding coefficient row 0
__device__ __forceinline__ void quad_idct(const LaneQ& Q, const int q[4], int qP, int out[4], bool keep_dc = false, int dcv = 0)
{
    // 8.5.12.1 as ((p << a) + r) >> b with a, r, b uniform: qP >= 24 shifts
    // left by q6 - 4, below it rounds and shifts right by 4 - q6
    // (the left shift at qP >= 24 is folded into Q's level scales, make_laneq)
    const int q6 = qP / 6;
    const int sr = qP >= 24 ? 0 : 1 << (3 - q6), sb = qP >= 24 ? 0 : 4 - q6;
    int d[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) d[c] = (__mul24(q[c], (c & 1) ? Q.lsO : Q.lsE) + sr) >> sb;
    if (keep_dc && Q.r == 0) d[0] = dcv;
    const int e0 = d[0] + d[2], e1 = d[0] - d[2], e2 = (d[1] >> 1) - d[3], e3 = d[1] + (d[3] >> 1);
    const int f[4] = {e0 + e3, e1 + e2, e1 - e2, e0 - e3};
    const int kx = opaque_w(Q.r == 1 ? -1 : 1), sh = Q.r >> 1, kp = opaque_w(Q.r == 2 ? -1 : 1), s1 = opaque_w(Q.r < 2 ? 1 : -1);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int g = __mul24(f[c] >> sh, kx) + __mul24(dpp_x<kQX1>(f[c]), kp);
        out[c] = (__mul24(g, s1) + dpp_x<kQX3>(g) + 32) >> 6;
    }
}

// run_before length, Table 9-10, zerosLeft 1..6 as one 54-bit constant
// (2 bits per run value, row zl at bit zl * zl + zl - 2), zerosLeft > 6
// closed form
__device__ __forceinline__ int quad_rb_len(int zl, int run)
{
    constexpr uint64_t kRb = 0x5ull | (0x29ull << 4) | (0xAAull << 10) | (0x3EAull << 18) | (0xFFAull << 28) | (0x3FFEull << 40);
    const int sh = min(max(zl * zl + zl - 2 + 2 * run, 0), 62);
    const int v = (int)((kRb >> sh) & 3);
    return zl > 6 ? (run < 7 ? 3 : run - 3) : v;
}

// CAVLC statistics of the quad's block (cavlc_stat with maxNumCoef 16,
// endIdx 15, the block's levels in scan order): L = this lane's row of
// levels (raster), ac = 1 for an AC list (scan positions 1..15 at list
// index 0..14, position 0 not in the list).  lvs = 16 words of LDS scratch
// owned by this quad.
__device__ __forceinline__ CoopStat quad_cavlc(const CoopTables& T, const LaneQ& Q, const int L[4], int ac, int* lvs)
{
    // Branch-free throughout: every condition is a select on bitwise-combined
    // flags (a short-circuit && here compiled to an exec-mask branch per
    // coefficient), and shift counts are masked so both arms are defined.
    int li[4], aL[4], nzl[4];
    int mb = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        li[c] = (int)((Q.zz >> (4 * c)) & 15) - ac;
        aL[c] = L[c] < 0 ? -L[c] : L[c];
        nzl[c] = (int)(li[c] >= 0) & (int)(L[c] != 0);
        const uint32_t sh = (uint32_t)li[c] & 15u;
        const uint32_t bits = (aL[c] == 1 ? 0x10001u : 1u) << sh;  // nonzero, and magnitude 1 (bit + 16)
        mb |= nzl[c] ? (int)bits : 0;
    }
    const uint32_t masks = (uint32_t)quad_or(mb);
    const uint32_t nz = masks & 0xFFFFu, ones = masks >> 16;
    CoopStat st;
    const int tc = __popc(nz);
    const int hi = 31 - __clz(nz | 1u);
    const uint32_t big = nz & ~ones;
    const int hb = 31 - __clz(big);  // -1 when big == 0 (__clz(0) = 32)
    const int t1a = __popc(nz >> (hb + 1));
    const int t1 = t1a < 3 ? t1a : 3;
    const int tzi = ((tc - 1) & 15) * 16 + ((hi + 1 - tc) & 15);
    const int tzv = (&T.tz[0][0])[tzi < 15 * 16 ? tzi : 0];
    const int tzb = ((int)(tc > 0) & (int)(tc < 16)) ? tzv : 0;  // total_zeros length
    const int sl0 = ((int)(tc > 10) & (int)(t1 < 3)) ? 1 : 0;
    // the first level coded with level_prefix/suffix: list index pf, the
    // highest nonzero below the t1 trailing ones (-1: none)
    // (with at most three trailing ones that is the highest coefficient above
    // magnitude 1, hb; with more, the fourth nonzero from the top)
    uint32_t rest = nz;
#pragma unroll
    for (int k = 0; k < 3; ++k) rest &= ~(1u << ((31 - __clz(rest)) & 31));
    const int pf = t1a <= 3 ? hb : 31 - __clz(rest);
    int rbs = 0, absum = 0, amax = 0, lf = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int lis = li[c] < 0 ? 0 : li[c];
        const uint32_t lower = nz & ((1u << lis) - 1u);
        const int zl = lis - __popc(lower);
        const int run = lis - 1 - (31 - __clz(lower));  // lis when lower == 0 (__clz(0) = 32)
        // run_before length from the LDS table (zerosLeft 0 reads 0)
        const int rbv = T.rb[zl & 15][run & 15];
        rbs += (nzl[c] & (int)(lower != 0)) ? rbv : 0;
        const int am = nzl[c] ? aL[c] : 0;
        absum += am;
        amax = max(amax, am);
        lf = (nzl[c] & (int)(li[c] == pf)) ? L[c] : lf;
    }
    const bool qslow = quad_or((int)(amax > 3)) != 0;  // uniform per quad (a trailing one has magnitude 1)
    int bits;
    if (!qslow) {
        // fast path (no level above 3 in the block): suffixLength is sl0 for
        // the first level and 1 after it, where a level of magnitude a takes
        // a + 1 bits; so the levels take (sum of magnitudes + tc) - 2 t1 (the
        // trailing ones' share) with the first level's own length in place of
        // its a + 1.  The first level (one lane of the quad) rides in the
        // upper half of the sum.
        const int q = quad_sum(rbs + absum + (lf << 16));
        const int lo16 = q & 0xFFFF, lfq = (q - lo16) >> 16;
        const int af = lfq < 0 ? -lfq : lfq;
        int l = lfq > 0 ? (lfq << 1) - 2 : -(lfq << 1) - 1;
        l -= ((int)(t1 < 3) & (int)(l >= 2)) ? 2 : 0;
        const int lenf = sl0 == 0 ? l + 1 : (l >> 1) + 2;  // 0: lc + 1 (lc < 14), 1: (lc >> 1) + 2 (lc < 28)
        bits = t1 + tzb + lo16 + tc - 2 * t1 + (tc > t1 ? lenf - (af + 1) : 0);
    }
    else {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int lis = li[c] < 0 ? 0 : li[c];
            const int m = __popc(nz >> (lis + 1)) - t1;  // order from the top, past the trailing ones
            int l = L[c] > 0 ? (L[c] << 1) - 2 : -(L[c] << 1) - 1;
            l -= ((int)(m == 0) & (int)(t1 < 3) & (int)(l >= 2)) ? 2 : 0;
            if (nzl[c] & (int)(m >= 0)) lvs[m] = (l << 16) | aL[c];  // a level coded with level_prefix/suffix
        }
        bits = t1 + tzb + quad_sum(rbs);
        // the suffixLength chain over the block's levels, in order (residual.c:813-858)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        int sl = sl0;
        // the 16 words in registers at once (four ds_read_b128 in flight), then
        // the chain over them unrolled: no LDS round trip per level
        const int4 w0 = reinterpret_cast<const int4*>(lvs)[0], w1 = reinterpret_cast<const int4*>(lvs)[1];
        const int4 w2 = reinterpret_cast<const int4*>(lvs)[2], w3 = reinterpret_cast<const int4*>(lvs)[3];
        const int v[16] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, w2.x, w2.y, w2.z, w2.w, w3.x, w3.y, w3.z, w3.w};
        const int n = tc - t1;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (__ballot(k < n) == 0) break;  // (wave-uniform exit)
            if (k < n) {
                bits += level_len(sl, v[k] >> 16);
                sl = next_sl(sl, v[k] & 0xFFFF);
            }
        }
    }
    st.tc = tc;
    st.t1 = tc ? t1 : 0;
    st.rest = tc ? bits : 0;
    // single-coefficient counter: 3 / 2 / 1 / 0 for a lone +-1 at list index
    // 0 / 1-2 / 3-5 / 6+, 2 bits per index in 0x56B; 9 otherwise; -1 if none
    // (selects only: the nested conditional became branches)
    const int lone = (int)((0x56Bu >> (2 * hi)) & 3u);
    const int sc = (int)(tc == 1) & (int)(ones == nz) ? lone : 9;
    st.sctr = tc ? sc : -1;
    return st;
}

// 4 consecutive bytes at p + off (any alignment) from two aligned words
__device__ __forceinline__ uint32_t ld_u8x4(const __attribute__((address_space(1))) uint8_t* p, int off)
{
    const auto w = reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(p + (off & ~3));
    return __builtin_amdgcn_alignbyte(w[1], w[0], (unsigned)(off & 3));
}
// the same from LDS
__device__ __forceinline__ uint32_t ld_lds_u8x4(const uint8_t* p, int off)
{
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p + (off & ~3));
    return __builtin_amdgcn_alignbyte(w[1], w[0], (unsigned)(off & 3));
}
// per byte (a + b + 1) >> 1
__device__ __forceinline__ uint32_t avg_u8x4(uint32_t a, uint32_t b) { return (a | b) - (((a ^ b) & 0xFEFEFEFEu) >> 1); }

}  // namespace hl
