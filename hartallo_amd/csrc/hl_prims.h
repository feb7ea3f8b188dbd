// hl_prims.h -- integer primitives of the H.264 Baseline macroblock path for
// gfx950: 4x4 forward/inverse core transform, quantisation, dequantisation,
// CAVLC bit counting and the constant tables they use.
//
// Every function is __host__ __device__: the same source runs in the HIP
// kernels (one lane per 4x4 block) and in the host-side CAVLC writer.
// Semantics follow the reference's scalar C paths (paths relative to the
// reference root, source/h264/):
//   forward transform   hl_codec_264_transf.c:716-772
//   Hadamard 4x4 / 2x2  hl_codec_264_transf.c:774-869
//   quantisation        hl_codec_264_quant.c:116-189, tables hl_codec_264_tables.c:9-44
//   dequant + IDCT      hl_codec_264_transf.c:376-458, hl_codec_264_quant.c:68-111
//   CAVLC tables        hl_codec_264_cavlc.c:59-103, 652-836 (H.264 tables 9-5..9-10)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hl {

#define HD __host__ __device__ __forceinline__

// Exact IEEE double arithmetic with no contraction: the reference's RDO costs
// are double (me_ds.c:287, rdo.c:1785) and must round identically.
HD double dadd(double a, double b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __dadd_rn(a, b);
#else
    return a + b;
#endif
}
HD double dmul(double a, double b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __dmul_rn(a, b);
#else
    return a * b;
#endif
}

// Global-memory view of a pointer the kernels hold as a generic one (picture
// planes, MB objects, records): its loads and stores become global_* instead
// of flat_* instructions, which also count against the LDS counter (every
// LDS wait then waits for them too) and, aliasing LDS as far as the compiler
// knows, force values it already loaded to be reloaded after every LDS store.
#if defined(__HIP_DEVICE_COMPILE__)
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gmem(T* p)
{
    return (__attribute__((address_space(1))) T*)p;
}
#else
template <typename T>
__host__ __device__ inline T* gmem(T* p)
{
    return p;
}
#endif

// Values every lane computes identically from LDS: tell the compiler they
// are wave-uniform (SGPRs, scalar branches) instead of divergent VGPRs.
HD int uni(int v)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_readfirstlane(v);
#else
    return v;
#endif
}
HD double uni(double v)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)b);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32));
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
#else
    return v;
#endif
}

HD int iabs(int x) { return x < 0 ? -x : x; }
HD int isign(int x) { return x >= 0 ? 1 : -1; }
HD int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
HD int clip255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// --------------------------------------------------------------------------
// Tables (H.264 spec values)
// --------------------------------------------------------------------------
static constexpr int32_t kQuantMF[6][3] = {{13107, 5243, 8066}, {11916, 4660, 7490}, {10082, 4194, 6554},
                                           {9362, 3647, 5825},  {8192, 3355, 5243},  {7282, 2893, 4559}};
static constexpr int32_t kScaleV[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
// position class in a 4x4 matrix: 0 = (even,even), 1 = (odd,odd), 2 = mixed
HD int pos_class(int i, int j) { return ((i & 1) == 0 && (j & 1) == 0) ? 0 : (((i & 1) && (j & 1)) ? 1 : 2); }
HD int32_t quant_mf(int qpm6, int i, int j) { return kQuantMF[qpm6][pos_class(i, j)]; }
HD int32_t level_scale(int qpm6, int i, int j) { return 16 * kScaleV[qpm6][pos_class(i, j)]; }

// zig-zag scan: scan index -> raster index (row*4+col) of the 4x4 matrix
static constexpr uint8_t kZigzag[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
// luma 4x4 block index -> (x, y) offset inside the macroblock (6.4.3)
static constexpr uint8_t kBlkX[16] = {0, 4, 0, 4, 8, 12, 8, 12, 0, 4, 0, 4, 8, 12, 8, 12};
static constexpr uint8_t kBlkY[16] = {0, 0, 4, 4, 0, 0, 4, 4, 8, 8, 12, 12, 8, 8, 12, 12};
// I16x16 DC matrix position of luma block idx (raster index into 4x4 DC matrix)
static constexpr uint8_t kDcPos[16] = {0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15};
HD int blk_idx(int x, int y) { return 8 * (y >> 3) + 4 * (x >> 3) + 2 * ((y & 7) >> 2) + ((x & 7) >> 2); }
// kBlkX / kBlkY as bit arithmetic (no table load for lane-varying indices)
HD int blk_x(int bi) { return ((bi >> 2) & 1) * 8 + (bi & 1) * 4; }
HD int blk_y(int bi) { return ((bi >> 3) & 1) * 8 + ((bi >> 1) & 1) * 4; }

static constexpr uint8_t kQpToQpc[52] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
                                         18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 32, 33,
                                         34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};
static constexpr uint8_t kAlpha[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,   0,   0,   0,   0,   4,   4,
                                       5,  6,  7,  8,  9,  10, 12, 13, 15, 17, 20, 22,  25,  28,  32,  36,  40,  45,
                                       50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
static constexpr uint8_t kBeta[52] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  2,  2,  2,  3,  3,  3,  3,  4,  4,  4,
                                      6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
static constexpr uint8_t kTc0[52][3] = {
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1},
    {0, 0, 1}, {0, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2},
    {1, 1, 2}, {1, 2, 3}, {1, 2, 3}, {2, 2, 3}, {2, 2, 4}, {2, 3, 4}, {2, 3, 4}, {3, 3, 5}, {3, 4, 6}, {3, 4, 6},
    {4, 5, 7}, {4, 5, 8}, {4, 6, 9}, {5, 7, 10}, {6, 8, 11}, {6, 8, 13}, {7, 10, 14}, {8, 11, 16}, {9, 12, 18},
    {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};
// tc0 for bS 1..3 (bS 4 uses the strong filter)
HD int tc0_of(int indexA, int bS) { return kTc0[indexA][bS - 1]; }

// lambda_mode = HL_CODEC_264_RDO_LAMBDA_FACT_ALL * (1 << ((QP - 12) / 3)) as
// the reference's x86 build computes it (slice.c:1766): the int shift count
// is negative below QP 10, and x86's SHL uses its low 5 bits -- QP 0-2 give
// 2^28 / 2^29, QP 3-6 2^30, QP 7-9 (int)(1u << 31) = INT_MIN, a negative
// lambda.  Written with that masking explicit (a negative shift count is
// undefined in C++).
HD double rdo_lambda(int qp) { return 0.852 * (double)(int32_t)(1u << (((qp - 12) / 3) & 31)); }

// coeff_token lengths, Table 9-5: [vlc 0..2][TrailingOnes][TotalCoeff]
static constexpr uint8_t kTokLen[3][4][17] = {
    {{1, 6, 8, 9, 10, 11, 13, 13, 13, 14, 14, 15, 15, 16, 16, 16, 16},
     {0, 2, 6, 8, 9, 10, 11, 13, 13, 14, 14, 15, 15, 15, 16, 16, 16},
     {0, 0, 3, 7, 8, 9, 10, 11, 13, 13, 14, 14, 15, 15, 16, 16, 16},
     {0, 0, 0, 5, 6, 7, 8, 9, 10, 11, 13, 14, 14, 15, 15, 16, 16}},
    {{2, 6, 6, 7, 8, 8, 9, 11, 11, 12, 12, 12, 13, 13, 13, 14, 14},
     {0, 2, 5, 6, 6, 7, 8, 9, 11, 11, 12, 12, 13, 13, 14, 14, 14},
     {0, 0, 3, 6, 6, 7, 8, 9, 11, 11, 12, 12, 13, 13, 13, 14, 14},
     {0, 0, 0, 4, 4, 5, 6, 6, 7, 9, 11, 11, 12, 13, 13, 13, 14}},
    {{4, 6, 6, 6, 7, 7, 7, 7, 8, 8, 9, 9, 9, 10, 10, 10, 10},
     {0, 4, 5, 5, 5, 5, 6, 6, 7, 8, 8, 9, 9, 9, 10, 10, 10},
     {0, 0, 4, 5, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 10},
     {0, 0, 0, 4, 4, 4, 4, 4, 5, 6, 7, 8, 8, 9, 10, 10, 10}}};
static constexpr uint8_t kTokCode[3][4][17] = {
    {{1, 5, 7, 7, 7, 7, 15, 11, 8, 15, 11, 15, 11, 15, 11, 7, 4},
     {0, 1, 4, 6, 6, 6, 6, 14, 10, 14, 10, 14, 10, 1, 14, 10, 6},
     {0, 0, 1, 5, 5, 5, 5, 5, 13, 9, 13, 9, 13, 9, 13, 9, 5},
     {0, 0, 0, 3, 3, 4, 4, 4, 4, 4, 12, 12, 8, 12, 8, 12, 8}},
    {{3, 11, 7, 7, 7, 4, 7, 15, 11, 15, 11, 8, 15, 11, 7, 9, 7},
     {0, 2, 7, 10, 6, 6, 6, 6, 14, 10, 14, 10, 14, 10, 11, 8, 6},
     {0, 0, 3, 9, 5, 5, 5, 5, 13, 9, 13, 9, 13, 9, 6, 10, 5},
     {0, 0, 0, 5, 4, 6, 8, 4, 4, 4, 12, 8, 12, 12, 8, 1, 4}},
    {{15, 15, 11, 8, 15, 11, 9, 8, 15, 11, 15, 11, 8, 13, 9, 5, 1},
     {0, 14, 15, 12, 10, 8, 14, 10, 14, 14, 10, 14, 10, 7, 12, 8, 4},
     {0, 0, 13, 14, 11, 9, 13, 9, 13, 10, 13, 9, 13, 9, 11, 7, 3},
     {0, 0, 0, 12, 11, 10, 9, 8, 13, 12, 12, 12, 8, 12, 10, 6, 2}}};
// chroma DC (nC == -1) coeff_token, [TrailingOnes][TotalCoeff 0..4]
static constexpr uint8_t kTokCdcLen[4][5] = {{2, 6, 6, 6, 6}, {0, 1, 6, 7, 8}, {0, 0, 3, 7, 8}, {0, 0, 0, 6, 7}};
static constexpr uint8_t kTokCdcCode[4][5] = {{1, 7, 4, 3, 2}, {0, 1, 6, 3, 3}, {0, 0, 1, 2, 2}, {0, 0, 0, 5, 0}};
// total_zeros, Tables 9-7/9-8 [TotalCoeff-1][total_zeros]
static constexpr uint8_t kTzLen[15][16] = {
    {1, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 9}, {3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 6, 6, 6, 6},
    {4, 3, 3, 3, 4, 4, 3, 3, 4, 5, 5, 6, 5, 6},       {5, 3, 4, 4, 3, 3, 3, 4, 3, 4, 5, 5, 5},
    {4, 4, 4, 3, 3, 3, 3, 3, 4, 5, 4, 5},             {6, 5, 3, 3, 3, 3, 3, 3, 4, 3, 6},
    {6, 5, 3, 3, 3, 2, 3, 4, 3, 6},                   {6, 4, 5, 3, 2, 2, 3, 3, 6},
    {6, 6, 4, 2, 2, 3, 2, 5},                         {5, 5, 3, 2, 2, 2, 4},
    {4, 4, 3, 3, 1, 3},                               {4, 4, 2, 1, 3},
    {3, 3, 1, 2},                                     {2, 2, 1},
    {1, 1}};
static constexpr uint8_t kTzCode[15][16] = {
    {1, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 1}, {7, 6, 5, 4, 3, 5, 4, 3, 2, 3, 2, 3, 2, 1, 0},
    {5, 7, 6, 5, 4, 3, 4, 3, 2, 3, 2, 1, 1, 0},       {3, 7, 5, 4, 6, 5, 4, 3, 3, 2, 2, 1, 0},
    {5, 4, 3, 7, 6, 5, 4, 3, 2, 1, 1, 0},             {1, 1, 7, 6, 5, 4, 3, 2, 1, 1, 0},
    {1, 1, 5, 4, 3, 3, 2, 1, 1, 0},                   {1, 1, 1, 3, 3, 2, 2, 1, 0},
    {1, 0, 1, 3, 2, 1, 1, 1},                         {1, 0, 1, 3, 2, 1, 1},
    {0, 1, 1, 2, 1, 3},                               {0, 1, 1, 1, 1},
    {0, 1, 1, 1},                                     {0, 1, 1},
    {0, 1}};
static constexpr uint8_t kTzCdcLen[3][4] = {{1, 2, 3, 3}, {1, 2, 2, 0}, {1, 1, 0, 0}};
static constexpr uint8_t kTzCdcCode[3][4] = {{1, 1, 1, 0}, {1, 1, 0, 0}, {1, 0, 0, 0}};
// run_before, Table 9-10 [min(zerosLeft,7)-1][run_before]
static constexpr uint8_t kRbLen[7][15] = {{1, 1}, {1, 2, 2}, {2, 2, 2, 2}, {2, 2, 2, 3, 3}, {2, 2, 3, 3, 3, 3},
                                          {2, 3, 3, 3, 3, 3, 3}, {3, 3, 3, 3, 3, 3, 3, 4, 5, 6, 7, 8, 9, 10, 11}};
static constexpr uint8_t kRbCode[7][15] = {{1, 0}, {1, 1, 0}, {3, 2, 1, 0}, {3, 2, 1, 1, 0}, {3, 2, 3, 2, 1, 0},
                                           {3, 0, 1, 3, 2, 5, 4}, {7, 6, 5, 4, 3, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1}};

// coeff_token length for a luma-type block with context nC >= 0
HD int token_len(int nC, int tc, int t1)
{
    if (nC >= 8) return 6;
    return kTokLen[nC < 2 ? 0 : (nC < 4 ? 1 : 2)][t1][tc];
}

// Length of one level_prefix/level_suffix code as the reference's generated
// table gives it (cavlc.c:59-103, including its inclusive suffix bound and the
// never-written entries beyond level_prefix 15 that emit a single bit).
HD int level_code_len(int sl, int lc)
{
    if (sl == 0) {
        if (lc < 14) return lc + 1;
        if (lc < 30) return 19;
        if (lc <= 4126) return 28;
        return 1;
    }
    if (lc < (14 << sl)) return (lc >> sl) + 1 + sl;
    if (lc < (15 << sl)) return 15 + sl;
    if (lc <= (15 << sl) + 4096) return 28;
    return 1;
}

// CAVLC statistics of one residual block, everything except coeff_token
// (residual.c:587-901 without the bit writer).  coeffLevel has maxNumCoef
// entries in scan order.  rest = bits of trailing-one signs, levels,
// total_zeros and run_before; sctr = the JVT-O079 single-coefficient counter
// the reference leaves in pc_esd->rdo.Single_ctr when TotalCoeff > 0.
struct CavlcStat {
    int tc, t1, rest, sctr;
};

template <typename T>
HD CavlcStat cavlc_stat(const T* coeffLevel, int maxNumCoef, int endIdx, bool chroma_dc)
{
    CavlcStat s;
    int nz[16];
    int run_before[16];
    int tc = 0, t1 = 0, total_zeros = 0, k = -1;
    bool countT1 = true, countTZ = false;
#pragma unroll
    for (int j = 0; j < 16; ++j) run_before[j] = 0;
    for (int j = 0; j < maxNumCoef; ++j) {
        int c = coeffLevel[maxNumCoef - 1 - j];
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
    int bits = 0, zerosLeft = 0;
    if (tc > 0) {
        int suffixLength = (tc > 10 && t1 < 3) ? 1 : 0;
        for (int j = 0; j < tc; ++j) {
            if (j < t1) {
                bits += 1;
            }
            else {
                int lc = nz[j] >= 0 ? nz[j] * 2 - 2 : -(nz[j] * 2) - 1;
                if (j == t1 && t1 < 3 && lc >= 2) lc -= 2;
                bits += level_code_len(suffixLength, lc);
                if (suffixLength == 0) suffixLength = 1;
                const int thr = suffixLength == 1 ? 3 : (suffixLength == 2 ? 6 : (suffixLength == 3 ? 12 : (suffixLength == 4 ? 24 : (suffixLength == 5 ? 48 : 32768))));
                if (iabs(nz[j]) > thr) ++suffixLength;
            }
        }
        if (tc < endIdx + 1) {
            bits += chroma_dc ? kTzCdcLen[tc - 1][total_zeros] : kTzLen[tc - 1][total_zeros];
            zerosLeft = total_zeros;
        }
        for (int kk = 0; kk < tc - 1 && zerosLeft > 0; ++kk) {
            int row = zerosLeft <= 6 ? zerosLeft - 1 : 6;
            bits += kRbLen[row][run_before[kk]];
            zerosLeft -= run_before[kk];
        }
        s.sctr = 9;
        if (tc == 1 && iabs(nz[0]) == 1) {
            int run = zerosLeft > 0 ? run_before[0] : 0;
            s.sctr = run == 0 ? 3 : (run < 3 ? 2 : (run < 6 ? 1 : 0));
        }
    }
    else {
        s.sctr = -1;
    }
    s.tc = tc;
    s.t1 = t1;
    s.rest = bits;
    return s;
}

// --------------------------------------------------------------------------
// Transforms (matrices are int[16], raster order row*4+col)
// --------------------------------------------------------------------------
HD void fwd4x4(const int* in, int* out)
{
    int t[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int a = in[0 * 4 + i], b = in[1 * 4 + i], c = in[2 * 4 + i], d = in[3 * 4 + i];
        t[0 * 4 + i] = a + b + c + d;
        t[1 * 4 + i] = a * 2 + b - c - d * 2;
        t[2 * 4 + i] = a - b - c + d;
        t[3 * 4 + i] = a - b * 2 + c * 2 - d;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int a = t[i * 4 + 0], b = t[i * 4 + 1], c = t[i * 4 + 2], d = t[i * 4 + 3];
        out[i * 4 + 0] = a + b + c + d;
        out[i * 4 + 1] = a * 2 + b - c - d * 2;
        out[i * 4 + 2] = a - b - c + d;
        out[i * 4 + 3] = a - b * 2 + c * 2 - d;
    }
}

HD void hadamard4x4_fwd(const int* in, int* out)
{
    int t[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int a = in[0 * 4 + i], b = in[1 * 4 + i], c = in[2 * 4 + i], d = in[3 * 4 + i];
        t[0 * 4 + i] = a + b + c + d;
        t[1 * 4 + i] = a + b - c - d;
        t[2 * 4 + i] = a - b - c + d;
        t[3 * 4 + i] = a - b + c - d;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int a = t[i * 4 + 0], b = t[i * 4 + 1], c = t[i * 4 + 2], d = t[i * 4 + 3];
        out[i * 4 + 0] = (a + b + c + d) >> 1;
        out[i * 4 + 1] = (a + b - c - d) >> 1;
        out[i * 4 + 2] = (a - b - c + d) >> 1;
        out[i * 4 + 3] = (a - b + c - d) >> 1;
    }
}

HD void idct4x4(const int* d, int* r)
{
    int f[16], h[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int e0 = d[i * 4 + 0] + d[i * 4 + 2];
        const int e1 = d[i * 4 + 0] - d[i * 4 + 2];
        const int e2 = (d[i * 4 + 1] >> 1) - d[i * 4 + 3];
        const int e3 = d[i * 4 + 1] + (d[i * 4 + 3] >> 1);
        f[i * 4 + 0] = e0 + e3;
        f[i * 4 + 1] = e1 + e2;
        f[i * 4 + 2] = e1 - e2;
        f[i * 4 + 3] = e0 - e3;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int g0 = f[0 * 4 + j] + f[2 * 4 + j];
        const int g1 = f[0 * 4 + j] - f[2 * 4 + j];
        const int g2 = (f[1 * 4 + j] >> 1) - f[3 * 4 + j];
        const int g3 = f[1 * 4 + j] + (f[3 * 4 + j] >> 1);
        h[0 * 4 + j] = g0 + g3;
        h[1 * 4 + j] = g1 + g2;
        h[2 * 4 + j] = g1 - g2;
        h[3 * 4 + j] = g0 - g3;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = (h[i] + 32) >> 6;
}

// AC quantisation (quant.c:116-137); intra rounding f = 2^qbits/3, inter /6
HD void quant4x4(int qp, bool intra, const int* w, int* z)
{
    const int qbits = 15 + qp / 6, qm = qp % 6;
    const int f = (1 << qbits) / (intra ? 3 : 6);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int v = (iabs(w[i]) * quant_mf(qm, i >> 2, i & 3) + f) >> qbits;
        z[i] = w[i] >= 0 ? v : -v;
    }
}
// DC quantisation (quant.c:141-189)
HD int quant_dc(int qp, bool intra, int w)
{
    const int qbits = 15 + qp / 6;
    const int f = (1 << qbits) / (intra ? 3 : 6);
    const int v = (iabs(w) * kQuantMF[qp % 6][0] + (f << 1)) >> (qbits + 1);
    return w >= 0 ? v : -v;
}

// 8.5.12: scaling of a 4x4 coefficient matrix c (raster) and inverse
// transform; keep_dc leaves c[0] unscaled (Intra16x16 luma and chroma).
HD void dequant_idct(int qP, const int* c, bool keep_dc, int* r)
{
    int d[16];
    const int qm = qP % 6, q6 = qP / 6;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int ls = level_scale(qm, i >> 2, i & 3);
        d[i] = qP >= 24 ? (c[i] * ls) * (1 << (q6 - 4)) : (c[i] * ls + (1 << (3 - q6))) >> (4 - q6);
    }
    if (keep_dc) d[0] = c[0];
    idct4x4(d, r);
}

// scan order list (16 entries) -> raster matrix
template <typename T>
HD void unscan(const T* list, int* m)
{
#pragma unroll
    for (int i = 0; i < 16; ++i) m[kZigzag[i]] = list[i];
}

// Inter-workgroup flags (agent scope, see hl_pipeline.h)
typedef __attribute__((address_space(1))) int32_t gi32;

// Scopes of the inter-workgroup release / acquire fences of pipelined runs
// (hl_pipeline.h).  Agent scope is the documented gfx950 form
// (cdna_hip_programming.md, Guideline 16); diagnostic builds may override.
#ifndef HL_ACQ_SCOPE
#define HL_ACQ_SCOPE "agent"
#endif
// memory order of the successor-counter decrements of a pipelined task
#ifndef HL_CNT_ORDER
#define HL_CNT_ORDER __ATOMIC_ACQ_REL
#endif
// 1: tasks that copy their records to host memory release at system scope
#ifndef HL_HOSTREC_SYS
#define HL_HOSTREC_SYS 1
#endif
#ifndef HL_REL_SCOPE
#define HL_REL_SCOPE "agent"
#endif

__device__ __forceinline__ int32_t ld_relaxed(const int32_t* p)
{
    return __hip_atomic_load((gi32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(int32_t* p, int32_t v)
{
    __hip_atomic_store((gi32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One lane polls until *flag >= want (bounded: a few seconds, then counts an
// error; the host then re-encodes the run picture by picture).
__device__ __forceinline__ void spin_ge(const int32_t* flag, int32_t want, int32_t* err)
{
    for (unsigned i = 0; ld_relaxed(flag) < want; ++i) {
        __builtin_amdgcn_s_sleep(2);
        if (i > (1u << 26)) {
            atomicAdd(err, 1);
            return;
        }
    }
}


}  // namespace hl
