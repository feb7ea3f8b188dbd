/*
 * hl_oracle.c -- CPU restatement of allweax/hartallo's H.264 Baseline encoder
 * (the per-macroblock RDO encode loop, CAVLC, deblocking and the stream
 * syntax around it).
 *
 * TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the checker.  The product never links it.
 *
 * Parity is pinned against the reference itself (oracle/_ref/ref_enc built
 * from /root/reference by oracle/Makefile) on the committed fixtures in
 * tests/golden/.  Every stateful quirk of the reference that changes
 * decisions or bits is reproduced (see DESIGN.md "Reference quirks").
 * Function comments cite the reference file:line each piece restates
 * (paths relative to the reference root, source/h264/ unless noted).
 */
#include "hl_oracle.h"
#include "mbrec.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* Enumerations (numeric values mirror include/hartallo/h264/hl_codec_264_defs.h
 * :399-540 and hl_codec_264_mb.h:38-54 so that dumps are comparable).        */
/* ------------------------------------------------------------------------- */
enum {
    ET_I_NXN = 101, ET_I16 = 102,
    ET_P16x16 = 301, ET_P16x8 = 302, ET_P8x16 = 303, ET_P8x8 = 304, ET_P8x8REF0 = 305, ET_PSKIP = 306
};
enum {
    FL_INTRA = 1, FL_INTER = 2, FL_SKIP = 4,
    FL_INTRA4 = 1 | (1 << 7), FL_INTRA16 = 1 | (1 << 8), FL_INTER_P = 2 | (1 << 10)
};
enum { PM_NA = -1, PM_L0 = 1, PM_I4 = 2, PM_I16 = 3 };
enum { SUB_NA = -1, SUB_8x8 = 101, SUB_8x4 = 102, SUB_4x8 = 103, SUB_4x4 = 104 };
enum { MODE_16x16 = 0, MODE_16x8, MODE_8x16, MODE_8x8_8x8, MODE_8x8_8x4, MODE_8x8_4x8, MODE_8x8_4x4 };
enum { RES_LUMA = 0, RES_I16_DC, RES_I16_AC, RES_CHROMA_DC, RES_CHROMA_AC };

#define NOT_AVAIL ((int32_t)0xFFFF0000) /* HL_CODEC_264_SAMPLE_NOT_AVAIL, defs.h:82 */
#define RDO_BUFFER_BITS (2048 * 8)      /* HL_CODEC_264_RDO_BUFFER_MAX_SIZE, defs.h:53 */
#define LAMBDA_FACT 0.852               /* HL_CODEC_264_RDO_LAMBDA_FACT_ALL, defs.h:54 */

#define CLIP3(lo, hi, v) ((v) < (lo) ? (lo) : ((v) > (hi) ? (hi) : (v)))
#define ABS(x) ((x) < 0 ? -(x) : (x))
#define SIGN(x) ((x) >= 0 ? 1 : -1)

typedef struct { int32_t x, y; } mv_t;

/* ------------------------------------------------------------------------- */
/* Tables (H.264 spec values; same numbers as source/h264/hl_codec_264_tables.c
 * and include/hartallo/h264/hl_codec_264_tables.h).                         */
/* ------------------------------------------------------------------------- */
static const int32_t QUANT_MF[6][4][4] = {
    {{13107, 8066, 13107, 8066}, {8066, 5243, 8066, 5243}, {13107, 8066, 13107, 8066}, {8066, 5243, 8066, 5243}},
    {{11916, 7490, 11916, 7490}, {7490, 4660, 7490, 4660}, {11916, 7490, 11916, 7490}, {7490, 4660, 7490, 4660}},
    {{10082, 6554, 10082, 6554}, {6554, 4194, 6554, 4194}, {10082, 6554, 10082, 6554}, {6554, 4194, 6554, 4194}},
    {{9362, 5825, 9362, 5825}, {5825, 3647, 5825, 3647}, {9362, 5825, 9362, 5825}, {5825, 3647, 5825, 3647}},
    {{8192, 5243, 8192, 5243}, {5243, 3355, 5243, 3355}, {8192, 5243, 8192, 5243}, {5243, 3355, 5243, 3355}},
    {{7282, 4559, 7282, 4559}, {4559, 2893, 4559, 2893}, {7282, 4559, 7282, 4559}, {4559, 2893, 4559, 2893}}};
static const int32_t SCALE_V[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
static const int32_t ZZ[16][2] = {{0, 0}, {0, 1}, {1, 0}, {2, 0}, {1, 1}, {0, 2}, {0, 3}, {1, 2},
                                  {2, 1}, {3, 0}, {3, 1}, {2, 2}, {1, 3}, {2, 3}, {3, 2}, {3, 3}};
static const int32_t BLK_XY[16][2] = {{0, 0}, {4, 0}, {0, 4}, {4, 4}, {8, 0}, {12, 0}, {8, 4}, {12, 4},
                                      {0, 8}, {4, 8}, {0, 12}, {4, 12}, {8, 8}, {12, 8}, {8, 12}, {12, 12}};
static const int32_t DCYIJ[16][2] = {{0, 0}, {0, 1}, {1, 0}, {1, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3},
                                     {2, 0}, {2, 1}, {3, 0}, {3, 1}, {2, 2}, {2, 3}, {3, 2}, {3, 3}};
static const int32_t QPI2QPC[52] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17,
                                    18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 32, 33,
                                    34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};
static const int32_t DEBLOCK_ALPHA[52] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 4, 4,
                                          5, 6, 7, 8, 9, 10, 12, 13, 15, 17, 20, 22, 25, 28, 32, 36, 40, 45,
                                          50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
static const int32_t DEBLOCK_BETA[52] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 2, 2, 3,
                                         3, 3, 3, 4, 4, 4, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12,
                                         13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
static const int32_t DEBLOCK_TC0[52][5] = {
    {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0},
    {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0},
    {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, 0, 1, 1},
    {0, 0, 0, 1, 1}, {0, 0, 0, 1, 1}, {0, 0, 0, 1, 1}, {0, 0, 1, 1, 1}, {0, 0, 1, 1, 1}, {0, 1, 1, 1, 1},
    {0, 1, 1, 1, 1}, {0, 1, 1, 1, 1}, {0, 1, 1, 1, 1}, {0, 1, 1, 2, 2}, {0, 1, 1, 2, 2}, {0, 1, 1, 2, 2},
    {0, 1, 1, 2, 2}, {0, 1, 2, 3, 3}, {0, 1, 2, 3, 3}, {0, 2, 2, 3, 3}, {0, 2, 2, 4, 4}, {0, 2, 3, 4, 4},
    {0, 2, 3, 4, 4}, {0, 3, 3, 5, 5}, {0, 3, 4, 6, 6}, {0, 3, 4, 6, 6}, {0, 4, 5, 7, 7}, {0, 4, 5, 8, 8},
    {0, 4, 6, 9, 9}, {0, 5, 7, 10, 10}, {0, 6, 8, 11, 11}, {0, 6, 8, 13, 13}, {0, 7, 10, 14, 14},
    {0, 8, 11, 16, 16}, {0, 9, 12, 18, 18}, {0, 10, 13, 20, 20}, {0, 11, 15, 23, 23}, {0, 13, 17, 25, 25}};

/* coeff_token (Table 9-5): [vlc 0..2][TrailingOnes][TotalCoeff] = {len, code};
 * cavlc.c:652-706 (nC>=8 is the 6-bit FLC). */
static const uint8_t COEFF_TOKEN[3][4][17][2] = {
    {{{1, 1}, {6, 5}, {8, 7}, {9, 7}, {10, 7}, {11, 7}, {13, 15}, {13, 11}, {13, 8}, {14, 15}, {14, 11}, {15, 15}, {15, 11}, {16, 15}, {16, 11}, {16, 7}, {16, 4}},
     {{0, 0}, {2, 1}, {6, 4}, {8, 6}, {9, 6}, {10, 6}, {11, 6}, {13, 14}, {13, 10}, {14, 14}, {14, 10}, {15, 14}, {15, 10}, {15, 1}, {16, 14}, {16, 10}, {16, 6}},
     {{0, 0}, {0, 0}, {3, 1}, {7, 5}, {8, 5}, {9, 5}, {10, 5}, {11, 5}, {13, 13}, {13, 9}, {14, 13}, {14, 9}, {15, 13}, {15, 9}, {16, 13}, {16, 9}, {16, 5}},
     {{0, 0}, {0, 0}, {0, 0}, {5, 3}, {6, 3}, {7, 4}, {8, 4}, {9, 4}, {10, 4}, {11, 4}, {13, 12}, {14, 12}, {14, 8}, {15, 12}, {15, 8}, {16, 12}, {16, 8}}},
    {{{2, 3}, {6, 11}, {6, 7}, {7, 7}, {8, 7}, {8, 4}, {9, 7}, {11, 15}, {11, 11}, {12, 15}, {12, 11}, {12, 8}, {13, 15}, {13, 11}, {13, 7}, {14, 9}, {14, 7}},
     {{0, 0}, {2, 2}, {5, 7}, {6, 10}, {6, 6}, {7, 6}, {8, 6}, {9, 6}, {11, 14}, {11, 10}, {12, 14}, {12, 10}, {13, 14}, {13, 10}, {14, 11}, {14, 8}, {14, 6}},
     {{0, 0}, {0, 0}, {3, 3}, {6, 9}, {6, 5}, {7, 5}, {8, 5}, {9, 5}, {11, 13}, {11, 9}, {12, 13}, {12, 9}, {13, 13}, {13, 9}, {13, 6}, {14, 10}, {14, 5}},
     {{0, 0}, {0, 0}, {0, 0}, {4, 5}, {4, 4}, {5, 6}, {6, 8}, {6, 4}, {7, 4}, {9, 4}, {11, 12}, {11, 8}, {12, 12}, {13, 12}, {13, 8}, {13, 1}, {14, 4}}},
    {{{4, 15}, {6, 15}, {6, 11}, {6, 8}, {7, 15}, {7, 11}, {7, 9}, {7, 8}, {8, 15}, {8, 11}, {9, 15}, {9, 11}, {9, 8}, {10, 13}, {10, 9}, {10, 5}, {10, 1}},
     {{0, 0}, {4, 14}, {5, 15}, {5, 12}, {5, 10}, {5, 8}, {6, 14}, {6, 10}, {7, 14}, {8, 14}, {8, 10}, {9, 14}, {9, 10}, {9, 7}, {10, 12}, {10, 8}, {10, 4}},
     {{0, 0}, {0, 0}, {4, 13}, {5, 14}, {5, 11}, {5, 9}, {6, 13}, {6, 9}, {7, 13}, {7, 10}, {8, 13}, {8, 9}, {9, 13}, {9, 9}, {10, 11}, {10, 7}, {10, 3}},
     {{0, 0}, {0, 0}, {0, 0}, {4, 12}, {4, 11}, {4, 10}, {4, 9}, {4, 8}, {5, 13}, {6, 12}, {7, 12}, {8, 12}, {8, 8}, {9, 12}, {10, 10}, {10, 6}, {10, 2}}}};
static const uint8_t COEFF_TOKEN_CDC[4][5][2] = {
    {{2, 1}, {6, 7}, {6, 4}, {6, 3}, {6, 2}},
    {{0, 0}, {1, 1}, {6, 6}, {7, 3}, {8, 3}},
    {{0, 0}, {0, 0}, {3, 1}, {7, 2}, {8, 2}},
    {{0, 0}, {0, 0}, {0, 0}, {6, 5}, {7, 0}}};
/* total_zeros (Tables 9-7/9-8), cavlc.c:727-773 */
static const uint8_t TZ_LEN[15][16] = {
    {1, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 9}, {3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 6, 6, 6, 6},
    {4, 3, 3, 3, 4, 4, 3, 3, 4, 5, 5, 6, 5, 6}, {5, 3, 4, 4, 3, 3, 3, 4, 3, 4, 5, 5, 5},
    {4, 4, 4, 3, 3, 3, 3, 3, 4, 5, 4, 5}, {6, 5, 3, 3, 3, 3, 3, 3, 4, 3, 6},
    {6, 5, 3, 3, 3, 2, 3, 4, 3, 6}, {6, 4, 5, 3, 2, 2, 3, 3, 6}, {6, 6, 4, 2, 2, 3, 2, 5},
    {5, 5, 3, 2, 2, 2, 4}, {4, 4, 3, 3, 1, 3}, {4, 4, 2, 1, 3}, {3, 3, 1, 2}, {2, 2, 1}, {1, 1}};
static const uint8_t TZ_CODE[15][16] = {
    {1, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 1}, {7, 6, 5, 4, 3, 5, 4, 3, 2, 3, 2, 3, 2, 1, 0},
    {5, 7, 6, 5, 4, 3, 4, 3, 2, 3, 2, 1, 1, 0}, {3, 7, 5, 4, 6, 5, 4, 3, 3, 2, 2, 1, 0},
    {5, 4, 3, 7, 6, 5, 4, 3, 2, 1, 1, 0}, {1, 1, 7, 6, 5, 4, 3, 2, 1, 1, 0},
    {1, 1, 5, 4, 3, 3, 2, 1, 1, 0}, {1, 1, 1, 3, 3, 2, 2, 1, 0}, {1, 0, 1, 3, 2, 1, 1, 1},
    {1, 0, 1, 3, 2, 1, 1}, {0, 1, 1, 2, 1, 3}, {0, 1, 1, 1, 1}, {0, 1, 1, 1}, {0, 1, 1}, {0, 1}};
static const uint8_t TZ_CDC_LEN[3][4] = {{1, 2, 3, 3}, {1, 2, 2, 0}, {1, 1, 0, 0}};
static const uint8_t TZ_CDC_CODE[3][4] = {{1, 1, 1, 0}, {1, 1, 0, 0}, {1, 0, 0, 0}};
/* run_before (Table 9-10), cavlc.c:800-836 */
static const uint8_t RB_LEN[7][16] = {{1, 1}, {1, 2, 2}, {2, 2, 2, 2}, {2, 2, 2, 3, 3}, {2, 2, 3, 3, 3, 3},
                                      {2, 3, 3, 3, 3, 3, 3}, {3, 3, 3, 3, 3, 3, 3, 4, 5, 6, 7, 8, 9, 10, 11}};
static const uint8_t RB_CODE[7][16] = {{1, 0}, {1, 1, 0}, {3, 2, 1, 0}, {3, 2, 1, 1, 0}, {3, 2, 3, 2, 1, 0},
                                       {3, 0, 1, 3, 2, 5, 4}, {7, 6, 5, 4, 3, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1}};
/* me(v) mapping coded_block_pattern -> codeNum (Table 9-4), bits.h:845-876 */
static const uint8_t CBP2CODE[48][2] = {
    {3, 0}, {29, 2}, {30, 3}, {17, 7}, {31, 4}, {18, 8}, {37, 17}, {8, 13}, {32, 5}, {38, 18}, {19, 9}, {9, 14},
    {20, 10}, {10, 15}, {11, 16}, {2, 11}, {16, 1}, {33, 32}, {34, 33}, {21, 36}, {35, 34}, {22, 37}, {39, 44}, {4, 40},
    {36, 35}, {40, 45}, {23, 38}, {5, 41}, {24, 39}, {6, 42}, {7, 43}, {1, 19}, {41, 6}, {42, 24}, {43, 25}, {25, 20},
    {44, 26}, {26, 21}, {46, 46}, {12, 28}, {45, 27}, {47, 47}, {27, 22}, {13, 29}, {28, 23}, {14, 30}, {15, 31}, {0, 12}};

/* CAVLC level VLC table built exactly like hl_codec_264_cavlc_InitEncodingTable
 * (cavlc.c:59-103), including its inclusive level_suffix bound. */
#define MAX_LEVEL_CODE 62545
typedef struct { uint16_t prefix, size; uint32_t suffix; } lvl_t;
static lvl_t (*g_levels)[MAX_LEVEL_CODE + 1];

static void init_level_table(void)
{
    int lp, sl, ls, lc, size;
    if (g_levels) return;
    g_levels = (lvl_t(*)[MAX_LEVEL_CODE + 1])calloc(7, sizeof(*g_levels));
    for (lp = 0; lp <= 15; ++lp) {
        for (sl = 0; sl <= 6; ++sl) {
            size = sl;
            if (lp == 14 && sl == 0) size = 4;
            else if (lp >= 15) size = lp - 3;
            for (ls = 0; ls <= (1 << size); ++ls) {
                lc = ((lp < 15 ? lp : 15) << sl);
                if (sl > 0 || lp >= 14) lc += ls;
                if (lp >= 15 && sl == 0) lc += 15;
                g_levels[sl][lc].prefix = (uint16_t)lp;
                g_levels[sl][lc].suffix = (uint32_t)ls;
                g_levels[sl][lc].size = (uint16_t)size;
            }
        }
    }
}

/* ------------------------------------------------------------------------- */
/* Bit writer (include/hartallo/h264/hl_codec_264_bits.h).  A writer with a
 * NULL buffer only counts bits (the RDO buffer of 2 KiB never fills at the
 * QPs used; overflows are counted and must stay zero).                      */
/* ------------------------------------------------------------------------- */
typedef struct {
    uint8_t* buf;
    size_t cap;
    int64_t nbits;
    int64_t limit; /* last writable byte index (pc_end - pc_start), 0 = none */
} bw_t;

static void bw_init(bw_t* b, uint8_t* buf, size_t cap) { b->buf = buf; b->cap = cap; b->nbits = 0; b->limit = 0; }

static void bw_u(bw_t* b, uint32_t v, int n)
{
    if (b->buf) {
        int i;
        for (i = n - 1; i >= 0; --i) {
            int64_t pos = b->nbits;
            if (b->limit && (pos >> 3) > b->limit) return; /* EoB: bits_write_u1 drops (bits.h:236-246) */
            size_t byte = (size_t)(pos >> 3);
            int bit = 7 - (int)(pos & 7);
            if (byte < b->cap) {
                if ((v >> i) & 1) b->buf[byte] |= (uint8_t)(1 << bit);
                else b->buf[byte] &= (uint8_t)~(1 << bit);
            }
            b->nbits++;
        }
    }
    else {
        b->nbits += n;
    }
}
static void bw_u1(bw_t* b, uint32_t v) { bw_u(b, v & 1, 1); }
static int ue_len(uint32_t v)
{
    int lz = 0;
    while ((1u << (lz + 1)) <= v + 1) ++lz;
    return 2 * lz + 1;
}
static void bw_ue(bw_t* b, uint32_t v)
{
    int lz = (ue_len(v) - 1) / 2;
    bw_u(b, 0, lz);
    bw_u(b, v + 1, lz + 1);
}
static uint32_t se2ue(int32_t n) { return (n <= 0) ? (uint32_t)(-n) << 1 : ((uint32_t)n << 1) - 1; }
static void bw_se(bw_t* b, int32_t n) { bw_ue(b, se2ue(n)); }
static int se_len(int32_t n) { return ue_len(se2ue(n)); }

/* rbsp_trailing_bits with the reference's quirk (rbsp.c:162-170): nothing is
 * written when the stream is byte aligned and the last byte ends in a 1. */
static void bw_trailing(bw_t* b)
{
    int aligned = (b->nbits & 7) == 0;
    if (!aligned || !(b->buf[(b->nbits >> 3) - 1] & 1)) {
        int left = 8 - (int)(b->nbits & 7);
        bw_u(b, 1u << (left - 1), left);
    }
}

/* ------------------------------------------------------------------------- */
/* Per-address macroblock state (hl_codec_264_mb_t, mb.h:99-269).  Objects
 * persist across frames exactly like pc_layer->pp_list_macroblocks[]; all
 * fields the encode path reads while stale are kept.                       */
/* ------------------------------------------------------------------------- */
typedef struct {
    int32_t addrA, blkA, addrB, blkB;
} nb4_t;

typedef struct {
    int32_t used;
    int32_t addr, mbx, mby, xL, yL, xC, yC, xL_Idx, yL_Idx;
    int32_t e_type, flags, MbPartPredMode[4];
    int32_t nA, nB, nC, nD; /* neighbour addresses or -1 */
    int32_t prev_flag[16], rem_mode[16];
    int32_t mb_type, sub_mb_type[4];
    int32_t QPy, QPyprime, QPc[2], QPprimeC[2];
    int32_t cbp, CbpL, CbpC, CbpL4x4, CbpCDC[2], CbpCAC[2];
    int32_t chroma_mode, I16Mode, I4Mode[16];
    int32_t RefIdxL0[4], refIdxL0[4], PredFlagL0[4], predFlagL0[4];
    mv_t mvL0[4][4], mvd_l0[4][4], MvL0[4][4];
    int32_t SubMbPredType[4], NumMbPart, NumSubMbPart[4], SubMbPartWidth[4], SubMbPartHeight[4];
    int32_t partWidth[4][4], partHeight[4][4], partWidthC[4][4], partHeightC[4][4];
    int32_t MbPartWidth, MbPartHeight;
    int32_t TCLuma[16], TCChromaAC[2][16];
    int32_t ChromaDCLevel[2][16], ChromaACLevel[2][4][16], I16DC[16], I16AC[16][16], LumaLevel[16][16];
    nb4_t nbL[16], nbC[4];
    int32_t dbInternal, dbLeft, dbTop;
} mb_t;

/* ME scratch (pc_esd->rdo.me, encode.h:41-69) */
typedef struct {
    mv_t mvBest[4][4], mvpLX[4][4];
    double best_cost[4][4];
    int32_t best_dist[4][4], single_ctr[4][4], best_cbp4x4[4][4];
    int32_t xP[4][4], yP[4][4], xS[4][4], yS[4][4], xL_Idx[4][4], yL_Idx[4][4];
    int32_t left, right, top, bottom;
    int32_t me_range, probably_pskip;
} me_t;

struct hlo_enc_s {
    hlo_params_t p;
    int32_t W, H, Wc, Hc, mbw, mbh, nmb;
    mb_t* mbs;
    uint8_t* cur[3];   /* picture being reconstructed (pc_fs_curr)            */
    uint8_t* ref[3];   /* RefPicList0[0]                                      */
    const uint8_t* src[3];
    int32_t frame_index, gop_left, pict_count, idr_pic_id;
    int32_t max_ref_frame; /* hl_codec_t.max_ref_frame (hl_codec.c:36, default 1) */
    int32_t is_intra_slice, qp;
    double lambda_mode, last_best_intra_cost;
    int32_t rdo_single_ctr; /* pc_esd->rdo.Single_ctr (persists, residual.c:883) */
    int32_t skip_run;
    int64_t rdo_overflows;
    me_t me;
    uint8_t* slice_buf;
    size_t slice_cap;
    int32_t level_scale[6][4][4]; /* LevelScale4x4 (flat lists), pps.c:30-80 */
};

/* ------------------------------------------------------------------------- */
/* Small helpers                                                             */
/* ------------------------------------------------------------------------- */
static int is_intra(const mb_t* m) { return (m->flags & FL_INTRA) != 0; }
static int inv_raster(int a, int b, int c, int d, int e) { return e == 0 ? (a % (d / b)) * b : (a / (d / b)) * c; }
static int luma_blk_idx(int x, int y) { return 8 * (y / 8) + 4 * (x / 8) + 2 * ((y % 8) / 4) + ((x % 8) / 4); }
static int sad4x4(const uint8_t* a, int sa, const uint8_t* b, int sb)
{
    int s = 0, i, j;
    for (j = 0; j < 4; ++j)
        for (i = 0; i < 4; ++i) s += ABS((int)a[j * sa + i] - (int)b[j * sb + i]);
    return s;
}
static int allzero16(const int32_t* v)
{
    int i;
    for (i = 0; i < 16; ++i)
        if (v[i]) return 0;
    return 1;
}

/* ------------------------------------------------------------------------- */
/* Transform / quantisation (transf.c:376-869, quant.c:68-189)               */
/* ------------------------------------------------------------------------- */
static void fwd4x4(const int32_t in[4][4], int32_t out[4][4]) /* transf.c:716-772 */
{
    int32_t t[4][4];
    int i;
    for (i = 0; i < 4; ++i) {
        t[0][i] = in[0][i] + in[1][i] + in[2][i] + in[3][i];
        t[1][i] = (in[0][i] << 1) + in[1][i] - in[2][i] - (in[3][i] << 1);
        t[2][i] = in[0][i] - in[1][i] - in[2][i] + in[3][i];
        t[3][i] = in[0][i] - (in[1][i] << 1) + (in[2][i] << 1) - in[3][i];
    }
    for (i = 0; i < 4; ++i) {
        out[i][0] = t[i][0] + t[i][1] + t[i][2] + t[i][3];
        out[i][1] = (t[i][0] << 1) + t[i][1] - t[i][2] - (t[i][3] << 1);
        out[i][2] = t[i][0] - t[i][1] - t[i][2] + t[i][3];
        out[i][3] = t[i][0] - (t[i][1] << 1) + (t[i][2] << 1) - t[i][3];
    }
}
static void hadamard4x4(const int32_t in[4][4], int32_t out[4][4]) /* transf.c:774-840 */
{
    int32_t t[4][4];
    int i;
    for (i = 0; i < 4; ++i) {
        t[0][i] = in[0][i] + in[1][i] + in[2][i] + in[3][i];
        t[1][i] = in[0][i] + in[1][i] - in[2][i] - in[3][i];
        t[2][i] = in[0][i] - in[1][i] - in[2][i] + in[3][i];
        t[3][i] = in[0][i] - in[1][i] + in[2][i] - in[3][i];
    }
    for (i = 0; i < 4; ++i) {
        out[i][0] = (t[i][0] + t[i][1] + t[i][2] + t[i][3]) >> 1;
        out[i][1] = (t[i][0] + t[i][1] - t[i][2] - t[i][3]) >> 1;
        out[i][2] = (t[i][0] - t[i][1] - t[i][2] + t[i][3]) >> 1;
        out[i][3] = (t[i][0] - t[i][1] + t[i][2] - t[i][3]) >> 1;
    }
}
static void quant_ac(int qp, int intra, const int32_t in[4][4], int32_t out[4][4]) /* quant.c:116-137 */
{
    int qbits = 15 + qp / 6, i, j;
    int32_t f = (1 << qbits) / (intra ? 3 : 6);
    for (i = 0; i < 4; ++i)
        for (j = 0; j < 4; ++j) {
            int32_t z = (ABS(in[i][j]) * QUANT_MF[qp % 6][i][j] + f) >> qbits;
            out[i][j] = z * SIGN(in[i][j]);
        }
}
static int32_t quant_dc1(int qp, int intra, int32_t v) /* quant.c:141-189 */
{
    int qbits = 15 + qp / 6;
    int32_t f = (1 << qbits) / (intra ? 3 : 6);
    int32_t z = (ABS(v) * QUANT_MF[qp % 6][0][0] + (f << 1)) >> (qbits + 1);
    return z * SIGN(v);
}
static void idct4x4(const int32_t d[4][4], int32_t r[4][4]) /* transf.c:420-456 */
{
    int32_t e[4][4], f[4][4], g[4][4], h[4][4];
    int i, j;
    for (i = 0; i < 4; ++i) {
        e[i][0] = d[i][0] + d[i][2];
        e[i][1] = d[i][0] - d[i][2];
        e[i][2] = (d[i][1] >> 1) - d[i][3];
        e[i][3] = d[i][1] + (d[i][3] >> 1);
    }
    for (i = 0; i < 4; ++i) {
        f[i][0] = e[i][0] + e[i][3];
        f[i][1] = e[i][1] + e[i][2];
        f[i][2] = e[i][1] - e[i][2];
        f[i][3] = e[i][0] - e[i][3];
    }
    for (j = 0; j < 4; ++j) {
        g[0][j] = f[0][j] + f[2][j];
        g[1][j] = f[0][j] - f[2][j];
        g[2][j] = (f[1][j] >> 1) - f[3][j];
        g[3][j] = f[1][j] + (f[3][j] >> 1);
    }
    for (j = 0; j < 4; ++j) {
        h[0][j] = g[0][j] + g[3][j];
        h[1][j] = g[1][j] + g[2][j];
        h[2][j] = g[1][j] - g[2][j];
        h[3][j] = g[0][j] - g[3][j];
    }
    for (i = 0; i < 4; ++i)
        for (j = 0; j < 4; ++j) r[i][j] = (h[i][j] + 32) >> 6;
}
/* 8.5.12 scaling + inverse transform, transf.c:376-418 + quant.c:68-111.
 * dc_is_scaled: (luma && Intra16x16) || !luma keep c[0][0]. */
static void scale_residual(const hlo_enc_t* e, int qP, const int32_t c[4][4], int dc_is_scaled, int32_t r[4][4])
{
    int32_t d[4][4];
    int i, j;
    for (i = 0; i < 4; ++i)
        for (j = 0; j < 4; ++j) {
            if (qP >= 24) d[i][j] = (c[i][j] * e->level_scale[qP % 6][i][j]) << (qP / 6 - 4);
            else d[i][j] = (c[i][j] * e->level_scale[qP % 6][i][j] + (1 << (3 - qP / 6))) >> (4 - qP / 6);
        }
    if (dc_is_scaled) d[0][0] = c[0][0];
    idct4x4(d, r);
}
static void inverse_scan(const int32_t* in16, int32_t out[4][4])
{
    int i;
    for (i = 0; i < 16; ++i) out[ZZ[i][0]][ZZ[i][1]] = in16[i];
}
static void scan_l(const int32_t in[4][4], int32_t* out16, int ac_only) /* utils.h:168-183 */
{
    int i;
    if (ac_only) {
        for (i = 1; i < 16; ++i) out16[i - 1] = in[ZZ[i][0]][ZZ[i][1]];
    }
    else {
        for (i = 0; i < 16; ++i) out16[i] = in[ZZ[i][0]][ZZ[i][1]];
    }
}
/* 8.5.10, transf.c:498-608 */
static void scale_luma_dc(const hlo_enc_t* e, const mb_t* m, const int32_t c[4][4], int32_t dcY[4][4])
{
    int32_t d[4][4], f[4][4];
    int i, j;
    int qP = m->QPyprime;
    for (j = 0; j < 4; ++j) {
        d[0][j] = c[0][j] + c[1][j] + c[2][j] + c[3][j];
        d[1][j] = c[0][j] + c[1][j] - c[2][j] - c[3][j];
        d[2][j] = c[0][j] - c[1][j] - c[2][j] + c[3][j];
        d[3][j] = c[0][j] - c[1][j] + c[2][j] - c[3][j];
    }
    for (i = 0; i < 4; ++i) {
        f[i][0] = d[i][0] + d[i][1] + d[i][2] + d[i][3];
        f[i][1] = d[i][0] + d[i][1] - d[i][2] - d[i][3];
        f[i][2] = d[i][0] - d[i][1] - d[i][2] + d[i][3];
        f[i][3] = d[i][0] - d[i][1] + d[i][2] - d[i][3];
    }
    {
        int32_t scale = e->level_scale[m->QPy % 6][0][0];
        for (i = 0; i < 4; ++i)
            for (j = 0; j < 4; ++j) {
                if (m->QPy >= 36) dcY[i][j] = (f[i][j] * scale) << (qP / 6 - 6);
                else dcY[i][j] = (f[i][j] * scale + (1 << (5 - qP / 6))) >> (6 - qP / 6);
            }
    }
}

/* ------------------------------------------------------------------------- */
/* CAVLC residual block (residual.c:587-901).  nC is supplied by the caller
 * (computed from the live MB state as residual.c:625-755 does).  Returns
 * TotalCoeffs; updates *single_ctr exactly like pc_esd->rdo.Single_ctr.     */
/* ------------------------------------------------------------------------- */
static int cavlc_block(bw_t* bw, const int32_t* coeffLevel, int startIdx, int endIdx, int maxNumCoef, int nC, int b_rdo,
                       int32_t* single_ctr)
{
    static const int32_t thr[7] = {0, 3, 6, 12, 24, 48, 1 << 15};
    int32_t nz[16], run_before[16] = {0};
    int TotalCoeffs = 0, TrailingOnes = 0, total_zeros = 0, k = -1, j;
    int countT1 = 1, countTZ = 0;
    for (j = 0; j < maxNumCoef; ++j) {
        int32_t coeff = coeffLevel[maxNumCoef - 1 - j];
        if (coeff) {
            nz[TotalCoeffs++] = coeff;
            countTZ = 1;
            ++k;
            if (countT1) {
                if (coeff == 1 || coeff == -1) {
                    ++TrailingOnes;
                    countT1 = (TrailingOnes < 3);
                }
                else {
                    countT1 = 0;
                }
            }
        }
        else if (countTZ) {
            ++run_before[k];
        }
        if (countTZ && coeff == 0) ++total_zeros;
    }
    /* coeff_token */
    if (nC >= 0) {
        if (nC >= 8) {
            bw_u(bw, TotalCoeffs ? (uint32_t)(((TotalCoeffs - 1) << 2) | TrailingOnes) : 3u, 6);
        }
        else {
            int vlc = nC < 2 ? 0 : (nC < 4 ? 1 : 2);
            bw_u(bw, COEFF_TOKEN[vlc][TrailingOnes][TotalCoeffs][1], COEFF_TOKEN[vlc][TrailingOnes][TotalCoeffs][0]);
        }
    }
    else {
        bw_u(bw, COEFF_TOKEN_CDC[TrailingOnes][TotalCoeffs][1], COEFF_TOKEN_CDC[TrailingOnes][TotalCoeffs][0]);
    }
    if (TotalCoeffs > 0) {
        int suffixLength = (TotalCoeffs > 10 && TrailingOnes < 3) ? 1 : 0;
        int zerosLeft;
        for (j = 0; j < TotalCoeffs; ++j) {
            if (j < TrailingOnes) {
                bw_u1(bw, (uint32_t)((1 - nz[j]) >> 1));
            }
            else {
                int32_t levelCode = (nz[j] >= 0) ? (nz[j] << 1) - 2 : -(nz[j] << 1) - 1;
                const lvl_t* L;
                if ((j == TrailingOnes && TrailingOnes < 3) && levelCode >= 2) levelCode -= 2;
                L = &g_levels[suffixLength][levelCode];
                if (L->prefix > 0) bw_u(bw, 0, L->prefix);
                bw_u1(bw, 1);
                if (L->size) bw_u(bw, L->suffix, L->size);
                if (suffixLength == 0) suffixLength = 1;
                if (ABS(nz[j]) > thr[suffixLength]) ++suffixLength;
            }
        }
        if (TotalCoeffs < endIdx - startIdx + 1) {
            if (nC >= 0) bw_u(bw, TZ_CODE[TotalCoeffs - 1][total_zeros], TZ_LEN[TotalCoeffs - 1][total_zeros]);
            else bw_u(bw, TZ_CDC_CODE[TotalCoeffs - 1][total_zeros], TZ_CDC_LEN[TotalCoeffs - 1][total_zeros]);
            zerosLeft = total_zeros;
        }
        else {
            zerosLeft = 0;
        }
        for (k = 0; (k < TotalCoeffs - 1) && (zerosLeft > 0); ++k) {
            int row = zerosLeft <= 6 ? zerosLeft - 1 : 6;
            bw_u(bw, RB_CODE[row][run_before[k]], RB_LEN[row][run_before[k]]);
            zerosLeft -= run_before[k];
        }
        if (b_rdo) { /* JVT-O079 2.3, residual.c:881-897 */
            *single_ctr = 9;
            if (TotalCoeffs == 1) {
                int32_t a = ABS(nz[0]);
                int run = zerosLeft > 0 ? run_before[0] : 0;
                if (a == 1) {
                    static const int32_t T[6] = {3, 2, 2, 1, 1, 1};
                    *single_ctr = run < 6 ? T[run] : 0;
                }
            }
        }
    }
    return TotalCoeffs;
}

/* nC for luma-type blocks (LUMA / I16 DC / I16 AC), residual.c:640-755 with
 * utils.h:9-20 (is_all_neighbouringblocks_zero reads CodedBlockPatternLuma,
 * also of the *current* MB, whose value may be stale). */
static int nc_luma(const hlo_enc_t* e, const mb_t* m, int blk)
{
    const nb4_t* nb = &m->nbL[blk];
    int availA = nb->addrA >= 0, availB = nb->addrB >= 0;
    int nA = 0, nB = 0;
    if (availA) {
        const mb_t* a = &e->mbs[nb->addrA];
        if (a->e_type == ET_PSKIP || (a->CbpL & (1 << (nb->blkA >> 2))) == 0) nA = 0;
        else nA = a->TCLuma[nb->blkA];
    }
    if (availB) {
        const mb_t* b = &e->mbs[nb->addrB];
        if (b->e_type == ET_PSKIP || (b->CbpL & (1 << (nb->blkB >> 2))) == 0) nB = 0;
        else nB = b->TCLuma[nb->blkB];
    }
    if (availA && availB) return (nA + nB + 1) >> 1;
    if (availA) return nA;
    if (availB) return nB;
    return 0;
}
static int nc_chroma_ac(const hlo_enc_t* e, const mb_t* m, int iCbCr, int blk)
{
    const nb4_t* nb = &m->nbC[blk];
    int availA = nb->addrA >= 0, availB = nb->addrB >= 0;
    int nA = 0, nB = 0;
    if (availA) {
        const mb_t* a = &e->mbs[nb->addrA];
        if (a->e_type == ET_PSKIP || (a->CbpC & 2) == 0) nA = 0;
        else nA = a->TCChromaAC[iCbCr][nb->blkA];
    }
    if (availB) {
        const mb_t* b = &e->mbs[nb->addrB];
        if (b->e_type == ET_PSKIP || (b->CbpC & 2) == 0) nB = 0;
        else nB = b->TCChromaAC[iCbCr][nb->blkB];
    }
    if (availA && availB) return (nA + nB + 1) >> 1;
    if (availA) return nA;
    if (availB) return nB;
    return 0;
}

/* write_block for a luma-type block: nC from state, TotalCoeffsLuma[idx]
 * update (residual.c:796-806; I16 DC writes index 0). */
static int wb_luma(hlo_enc_t* e, mb_t* m, bw_t* bw, int type, int blk, const int32_t* lv, int s, int en, int maxc, int b_rdo)
{
    int idx = (type == RES_I16_DC) ? 0 : blk;
    int nC = nc_luma(e, m, idx);
    int tc = cavlc_block(bw, lv, s, en, maxc, nC, b_rdo, &e->rdo_single_ctr);
    m->TCLuma[idx] = tc;
    return tc;
}
static int wb_chroma_ac(hlo_enc_t* e, mb_t* m, bw_t* bw, int iCbCr, int blk, const int32_t* lv, int s, int en, int maxc, int b_rdo)
{
    int nC = nc_chroma_ac(e, m, iCbCr, blk);
    int tc = cavlc_block(bw, lv, s, en, maxc, nC, b_rdo, &e->rdo_single_ctr);
    m->TCChromaAC[iCbCr][blk] = tc;
    return tc;
}

/* ------------------------------------------------------------------------- */
/* Neighbour derivation (utils.c:61-230, utils.h:53-108)                     */
/* ------------------------------------------------------------------------- */
static int nb_location(const mb_t* m, int xN, int yN, int maxW, int maxH, int* xW, int* yW)
{
    int a;
    if (xN >= 0 && xN <= maxW - 1 && yN >= 0 && yN <= maxH - 1) a = m->addr;
    else if (xN >= 0 && xN <= maxW - 1 && yN < 0) a = m->nB;
    else if (xN > maxW - 1 && yN < 0) a = m->nC;
    else if (xN < 0 && yN < 0) a = m->nD;
    else if (xN < 0 && yN >= 0 && yN <= maxH - 1) a = m->nA;
    else a = -1;
    *xW = (xN + maxW) % maxW;
    *yW = (yN + maxH) % maxH;
    return a;
}

static void init_mb(hlo_enc_t* e, int addr) /* utils.c:61-230 */
{
    mb_t* m = &e->mbs[addr];
    int b, xW, yW;
    m->addr = addr;
    m->CbpL4x4 = 0;
    m->CbpCAC[0] = m->CbpCAC[1] = 0;
    m->CbpCDC[0] = m->CbpCDC[1] = 0;
    m->mbx = addr % e->mbw;
    m->mby = addr / e->mbw;
    m->nA = m->nB = m->nC = m->nD = -1;
    if (m->mbx) {
        m->nA = addr - 1;
        if (m->mby) m->nD = addr - e->mbw - 1;
    }
    if (m->mby) {
        m->nB = addr - e->mbw;
        if (m->mbx < e->mbw - 1) m->nC = addr - e->mbw + 1;
    }
    m->xL = m->mbx * 16;
    m->yL = m->mby * 16;
    m->xC = m->xL >> 1;
    m->yC = m->yL >> 1;
    for (b = 0; b < 4; ++b) { /* 6.4.10.5 */
        int x = (b & 1) * 4, y = (b >> 1) * 4;
        int a = nb_location(m, x - 1, y, 8, 8, &xW, &yW);
        m->nbC[b].addrA = a;
        m->nbC[b].blkA = a >= 0 ? (yW / 4) * 2 + (xW / 4) : -1;
        a = nb_location(m, x, y - 1, 8, 8, &xW, &yW);
        m->nbC[b].addrB = a;
        m->nbC[b].blkB = a >= 0 ? (yW / 4) * 2 + (xW / 4) : -1;
    }
    for (b = 0; b < 16; ++b) { /* 6.4.10.4 */
        int x = BLK_XY[b][0], y = BLK_XY[b][1];
        int a = nb_location(m, x - 1, y, 16, 16, &xW, &yW);
        m->nbL[b].addrA = a;
        m->nbL[b].blkA = a >= 0 ? luma_blk_idx(xW, yW) : -1;
        a = nb_location(m, x, y - 1, 16, 16, &xW, &yW);
        m->nbL[b].addrB = a;
        m->nbL[b].blkB = a >= 0 ? luma_blk_idx(xW, yW) : -1;
    }
}

static void set_quant(hlo_enc_t* e, mb_t* m) /* mb.c:375-422 (mb_qp_delta is always 0) */
{
    int c;
    m->QPy = e->qp;
    m->QPyprime = m->QPy;
    for (c = 0; c < 2; ++c) {
        int qPI = CLIP3(0, 51, m->QPy);
        m->QPc[c] = QPI2QPC[qPI];
        m->QPprimeC[c] = m->QPc[c];
    }
}

/* ------------------------------------------------------------------------- */
/* Motion vector prediction (mb.c:426-541, utils.c:708-963)                  */
/* ------------------------------------------------------------------------- */
static int is_8x8_type(int et) { return et == ET_P8x8 || et == ET_P8x8REF0; }

static void sub_part_indices(const mb_t* n, int xW, int yW, int* mbPartIdx, int* subMbPartIdx) /* mb.h:313-339 */
{
    if (is_intra(n)) *mbPartIdx = 0;
    else *mbPartIdx = (16 / n->MbPartWidth) * (yW / n->MbPartHeight) + (xW / n->MbPartWidth);
    if (!is_8x8_type(n->e_type)) *subMbPartIdx = 0;
    else {
        int p = *mbPartIdx;
        *subMbPartIdx = (8 / n->SubMbPartWidth[p]) * ((yW % 8) / n->SubMbPartHeight[p]) + ((xW % 8) / n->SubMbPartWidth[p]);
    }
}

/* Neighbouring partitions A,B,C,D -> (addr, mbPartIdx, subMbPartIdx). */
static void nb_partitions(const hlo_enc_t* e, const mb_t* m, int mbPartIdx, int subMbPartIdx, int out[4][3])
{
    static const int XD[4] = {-1, 0, -1, -1}, YD[4] = {0, -1, -1, -1};
    int x = inv_raster(mbPartIdx, m->MbPartWidth, m->MbPartHeight, 16, 0);
    int y = inv_raster(mbPartIdx, m->MbPartWidth, m->MbPartHeight, 16, 1);
    int xS = 0, yS = 0, predPartWidth, N;
    if (is_8x8_type(m->e_type)) {
        xS = inv_raster(subMbPartIdx, m->SubMbPartWidth[mbPartIdx], m->SubMbPartHeight[mbPartIdx], 8, 0);
        yS = inv_raster(subMbPartIdx, m->SubMbPartWidth[mbPartIdx], m->SubMbPartHeight[mbPartIdx], 8, 1);
    }
    if (m->e_type == ET_PSKIP) predPartWidth = 16;
    else if (is_8x8_type(m->e_type)) predPartWidth = m->SubMbPartWidth[mbPartIdx];
    else predPartWidth = m->MbPartWidth;
    for (N = 0; N < 4; ++N) {
        int xD = (N == 2) ? predPartWidth : XD[N];
        int xW, yW;
        int a = nb_location(m, x + xS + xD, y + yS + YD[N], 16, 16, &xW, &yW);
        out[N][0] = a;
        if (a >= 0) {
            int pi, spi;
            sub_part_indices(&e->mbs[a], xW, yW, &pi, &spi);
            out[N][1] = pi;
            out[N][2] = spi;
            if (a == m->addr && (pi > mbPartIdx || (pi == mbPartIdx && spi > subMbPartIdx))) {
                out[N][0] = out[N][1] = out[N][2] = -1;
            }
        }
        else {
            out[N][1] = out[N][2] = -1;
        }
    }
}

static void nb_motion(const hlo_enc_t* e, const mb_t* m, int mbPartIdx, int subMbPartIdx, int nb[4][3], mv_t mv[4], int ref[4])
{
    int N;
    nb_partitions(e, m, mbPartIdx, subMbPartIdx, nb);
    if (nb[2][0] < 0 || nb[2][1] < 0 || nb[2][2] < 0) {
        nb[2][0] = nb[3][0];
        nb[2][1] = nb[3][1];
        nb[2][2] = nb[3][2];
    }
    for (N = 0; N < 4; ++N) {
        const mb_t* n = nb[N][0] < 0 ? NULL : &e->mbs[nb[N][0]];
        if (!n || is_intra(n) || n->predFlagL0[nb[N][1]] == 0) {
            mv[N].x = mv[N].y = 0;
            ref[N] = -1;
        }
        else {
            mv[N] = n->MvL0[nb[N][1]][nb[N][2]];
            ref[N] = n->RefIdxL0[nb[N][1]];
        }
    }
}

static int median3(int a, int b, int c)
{
    int mx = a > b ? (a > c ? a : c) : (b > c ? b : c);
    int mn = a < b ? (a < c ? a : c) : (b < c ? b : c);
    return a + b + c - mx - mn;
}

static mv_t mvp(const hlo_enc_t* e, const mb_t* m, int mbPartIdx, int subMbPartIdx) /* utils.c:751-831 */
{
    int nb[4][3], ref[4], refIdx = 0;
    mv_t mv[4], r;
    nb_motion(e, m, mbPartIdx, subMbPartIdx, nb, mv, ref);
    if (m->MbPartWidth == 16 && m->MbPartHeight == 8 && mbPartIdx == 0 && ref[1] == refIdx) return mv[1];
    if (m->MbPartWidth == 16 && m->MbPartHeight == 8 && mbPartIdx == 1 && ref[0] == refIdx) return mv[0];
    if (m->MbPartWidth == 8 && m->MbPartHeight == 16 && mbPartIdx == 0 && ref[0] == refIdx) return mv[0];
    if (m->MbPartWidth == 8 && m->MbPartHeight == 16 && mbPartIdx == 1 && ref[2] == refIdx) return mv[2];
    if ((nb[1][0] < 0 || nb[1][1] < 0 || nb[1][2] < 0) && (nb[2][0] < 0 || nb[2][1] < 0 || nb[2][2] < 0) &&
        (nb[0][0] >= 0 && nb[0][1] >= 0 && nb[0][2] >= 0)) {
        mv[1] = mv[2] = mv[0];
        ref[1] = ref[2] = ref[0];
    }
    if (ref[0] == refIdx && ref[1] != refIdx && ref[2] != refIdx) return mv[0];
    if (ref[1] == refIdx && ref[2] != refIdx && ref[0] != refIdx) return mv[1];
    if (ref[2] == refIdx && ref[1] != refIdx && ref[0] != refIdx) return mv[2];
    r.x = median3(mv[0].x, mv[1].x, mv[2].x);
    r.y = median3(mv[0].y, mv[1].y, mv[2].y);
    return r;
}

static mv_t skip_mv(const hlo_enc_t* e, const mb_t* m) /* utils.c:709-748 */
{
    int nb[4][3], ref[4];
    mv_t mv[4], z = {0, 0};
    nb_motion(e, m, 0, 0, nb, mv, ref);
    if (nb[0][0] < 0 || nb[1][0] < 0 || (ref[0] == 0 && !mv[0].x && !mv[0].y) || (ref[1] == 0 && !mv[1].x && !mv[1].y))
        return z;
    return mvp(e, m, 0, 0);
}

/* ------------------------------------------------------------------------- */
/* Inter prediction samples (pred_inter.c:339-885, interpol.c:74-392)        */
/* ------------------------------------------------------------------------- */
static inline int tap6(int E, int F, int G, int H, int I, int J) { return E - 5 * (F + I) + 20 * (G + H) + J; }

/* One luma prediction sample for integer position (x,y) of the clipped
 * origin + fraction; coordinates are clamped (index table interpol.c:108-131). */
typedef struct { const uint8_t* p; int W, H; } plane_t;
static inline int S(const plane_t* P, int x, int y) { return P->p[CLIP3(0, P->H - 1, y) * P->W + CLIP3(0, P->W - 1, x)]; }
static inline int b1_at(const plane_t* P, int x, int y) { return tap6(S(P, x - 2, y), S(P, x - 1, y), S(P, x, y), S(P, x + 1, y), S(P, x + 2, y), S(P, x + 3, y)); }
static inline int h1_at(const plane_t* P, int x, int y) { return tap6(S(P, x, y - 2), S(P, x, y - 1), S(P, x, y), S(P, x, y + 1), S(P, x, y + 2), S(P, x, y + 3)); }
static inline int clip255(int v) { return CLIP3(0, 255, v); }
static inline int half_b(const plane_t* P, int x, int y) { return clip255((b1_at(P, x, y) + 16) >> 5); }
static inline int half_h(const plane_t* P, int x, int y) { return clip255((h1_at(P, x, y) + 16) >> 5); }
static inline int half_j(const plane_t* P, int x, int y)
{
    int j1 = tap6(h1_at(P, x - 2, y), h1_at(P, x - 1, y), h1_at(P, x, y), h1_at(P, x + 1, y), h1_at(P, x + 2, y), h1_at(P, x + 3, y));
    return clip255((j1 + 512) >> 10);
}
static int luma_qpel(const plane_t* P, int x, int y, int xF, int yF)
{
    switch ((yF << 2) | xF) {
    case 0: return S(P, x, y);
    case 1: return (S(P, x, y) + half_b(P, x, y) + 1) >> 1;
    case 2: return half_b(P, x, y);
    case 3: return (S(P, x + 1, y) + half_b(P, x, y) + 1) >> 1;
    case 4: return (S(P, x, y) + half_h(P, x, y) + 1) >> 1;
    case 5: return (half_b(P, x, y) + half_h(P, x, y) + 1) >> 1;
    case 6: return (half_b(P, x, y) + half_j(P, x, y) + 1) >> 1;
    case 7: return (half_b(P, x, y) + half_h(P, x + 1, y) + 1) >> 1;
    case 8: return half_h(P, x, y);
    case 9: return (half_h(P, x, y) + half_j(P, x, y) + 1) >> 1;
    case 10: return half_j(P, x, y);
    case 11: return (half_j(P, x, y) + half_h(P, x + 1, y) + 1) >> 1;
    case 12: return (S(P, x, y + 1) + half_h(P, x, y) + 1) >> 1;
    case 13: return (half_h(P, x, y) + half_b(P, x, y + 1) + 1) >> 1;
    case 14: return (half_j(P, x, y) + half_b(P, x, y + 1) + 1) >> 1;
    default: return (half_h(P, x + 1, y) + half_b(P, x, y + 1) + 1) >> 1;
    }
}
/* Prediction of a partition (pw x ph) at luma origin (xL_Idx,yL_Idx) with
 * motion vector mv into out[16][16] (row-major, stride 16). */
static void pred_luma(const hlo_enc_t* e, int xL_Idx, int yL_Idx, mv_t mv, int pw, int ph, uint8_t out[16][16])
{
    plane_t P = {e->ref[0], e->W, e->H};
    int X = CLIP3(-17, e->W + 17, xL_Idx + (mv.x >> 2));
    int Y = CLIP3(-17, e->H + 17, yL_Idx + (mv.y >> 2));
    int xF = mv.x & 3, yF = mv.y & 3, x, y;
    for (y = 0; y < ph; ++y)
        for (x = 0; x < pw; ++x) out[y][x] = (uint8_t)luma_qpel(&P, X + x, Y + y, xF, yF);
}
/* Chroma 4:2:0 prediction, written in the reference's 4x4 block pattern
 * (interpol.c:337-385 always fills whole 4x4 blocks). */
static void pred_chroma_part(const hlo_enc_t* e, int xL_Idx, int yL_Idx, mv_t mvC, int pwC, int phC, int32_t outCb[16][16],
                             int32_t outCr[16][16], int ox, int oy)
{
    int xIntC = (xL_Idx >> 1) + (mvC.x >> 3), yIntC = (yL_Idx >> 1) + (mvC.y >> 3);
    int xF = mvC.x & 7, yF = mvC.y & 7, xC, yC, x, y, c;
    for (yC = 0; yC < phC; yC += 4)
        for (xC = 0; xC < pwC; xC += 4)
            for (y = 0; y < 4; ++y)
                for (x = 0; x < 4; ++x) {
                    int xa = CLIP3(0, e->Wc - 1, xIntC + xC + x), xb = CLIP3(0, e->Wc - 1, xIntC + xC + x + 1);
                    int ya = CLIP3(0, e->Hc - 1, yIntC + yC + y), yb = CLIP3(0, e->Hc - 1, yIntC + yC + y + 1);
                    int oyy = oy + yC + y, oxx = ox + xC + x;
                    for (c = 0; c < 2; ++c) {
                        const uint8_t* r = e->ref[1 + c];
                        int v = ((8 - xF) * (8 - yF) * r[ya * e->Wc + xa] + xF * (8 - yF) * r[ya * e->Wc + xb] +
                                 (8 - xF) * yF * r[yb * e->Wc + xa] + xF * yF * r[yb * e->Wc + xb] + 32) >> 6;
                        if (oyy < 16 && oxx < 16) (c ? outCr : outCb)[oyy][oxx] = v;
                    }
                }
}

/* ------------------------------------------------------------------------- */
/* Intra prediction (pred_intra.c:326-1220)                                  */
/* ------------------------------------------------------------------------- */
static int sample_cur(const hlo_enc_t* e, int plane, int x, int y)
{
    int W = plane ? e->Wc : e->W;
    return e->cur[plane][y * W + x];
}

static void nb4x4L(const hlo_enc_t* e, const mb_t* m, int blk, int p[13]) /* pred_intra.c:326-376 */
{
    static const int X[13] = {-1, -1, -1, -1, -1, 0, 1, 2, 3, 4, 5, 6, 7};
    static const int Y[13] = {-1, 0, 1, 2, 3, -1, -1, -1, -1, -1, -1, -1, -1};
    int i, xO = BLK_XY[blk][0], yO = BLK_XY[blk][1], x47_na = 1;
    for (i = 0; i < 13; ++i) {
        int xW, yW;
        int a = nb_location(m, xO + X[i], yO + Y[i], 16, 16, &xW, &yW);
        if (a < 0 || (X[i] > 3 && (blk == 3 || blk == 11))) {
            p[i] = NOT_AVAIL;
        }
        else {
            const mb_t* n = &e->mbs[a];
            if (x47_na && Y[i] == -1 && X[i] >= 4 && X[i] <= 7) x47_na = 0;
            p[i] = sample_cur(e, 0, n->xL + xW, n->yL + yW);
        }
    }
    if (x47_na && p[8] != NOT_AVAIL) p[9] = p[10] = p[11] = p[12] = p[8];
}
static void nb16x16L(const hlo_enc_t* e, const mb_t* m, int p[33]) /* pred_intra.c:379-413 */
{
    int i;
    for (i = 0; i < 33; ++i) {
        int x = i < 17 ? -1 : i - 17, y = i < 17 ? i - 1 : -1, xW, yW;
        int a = nb_location(m, x, y, 16, 16, &xW, &yW);
        if (a < 0) p[i] = NOT_AVAIL;
        else p[i] = sample_cur(e, 0, e->mbs[a].xL + xW, e->mbs[a].yL + yW);
    }
}
static void nbC(const hlo_enc_t* e, const mb_t* m, int pCb[17], int pCr[17]) /* pred_intra.c:416-457 */
{
    int i;
    for (i = 0; i < 17; ++i) {
        int x = i < 9 ? -1 : i - 9, y = i < 9 ? i - 1 : -1, xW, yW;
        int a = nb_location(m, x, y, 8, 8, &xW, &yW);
        if (a < 0) pCb[i] = pCr[i] = NOT_AVAIL;
        else {
            const mb_t* n = &e->mbs[a];
            int xM = (n->xL >> 4) * 8, yM = (n->yL >> 4) * 8 + (n->yL & 1);
            pCb[i] = sample_cur(e, 1, xM + xW, yM + yW);
            pCr[i] = sample_cur(e, 2, xM + xW, yM + yW);
        }
    }
}
#define P4(x, y) p[(x) == -1 ? (y) + 1 : (x) + 5]
static void pred4x4(int mode, const int p[13], int32_t pr[4][4]) /* pred_intra.c:617-853 */
{
    int x, y;
    switch (mode) {
    case 0:
        for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) pr[y][x] = p[5 + x];
        break;
    case 1:
        for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) pr[y][x] = p[1 + y];
        break;
    case 2: {
        int xa = !(p[5] == NOT_AVAIL || p[6] == NOT_AVAIL || p[7] == NOT_AVAIL || p[8] == NOT_AVAIL);
        int ya = !(p[1] == NOT_AVAIL || p[2] == NOT_AVAIL || p[3] == NOT_AVAIL || p[4] == NOT_AVAIL);
        int r;
        if (xa && ya) r = (p[5] + p[6] + p[7] + p[8] + p[1] + p[2] + p[3] + p[4] + 4) >> 3;
        else if (!xa && ya) r = (p[1] + p[2] + p[3] + p[4] + 2) >> 2;
        else if (!ya && xa) r = (p[5] + p[6] + p[7] + p[8] + 2) >> 2;
        else r = 128;
        for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) pr[y][x] = r;
        break;
    }
    case 3:
        for (y = 0; y < 4; ++y)
            for (x = 0; x < 4; ++x) pr[y][x] = (P4(x + y, -1) + 2 * P4(x + y + 1, -1) + P4(x + y + 2, -1) + 2) >> 2;
        pr[3][3] = (p[11] + 3 * p[12] + 2) >> 2;
        break;
    case 4:
        for (y = 0; y < 4; ++y)
            for (x = 0; x < 4; ++x) {
                if (x > y) pr[y][x] = (P4(x - y - 2, -1) + (P4(x - y - 1, -1) << 1) + P4(x - y, -1) + 2) >> 2;
                else if (x < y) pr[y][x] = (P4(-1, y - x - 2) + (P4(-1, y - x - 1) << 1) + P4(-1, y - x) + 2) >> 2;
                else pr[y][x] = (p[5] + (P4(-1, -1) << 1) + p[1] + 2) >> 2;
            }
        break;
    case 5:
        for (y = 0; y < 4; ++y)
            for (x = 0; x < 4; ++x) {
                int z = 2 * x - y;
                if (z >= 0 && !(z & 1)) pr[y][x] = (P4(x - (y >> 1) - 1, -1) + P4(x - (y >> 1), -1) + 1) >> 1;
                else if (z >= 0) pr[y][x] = (P4(x - (y >> 1) - 2, -1) + (P4(x - (y >> 1) - 1, -1) << 1) + P4(x - (y >> 1), -1) + 2) >> 2;
                else if (z == -1) pr[y][x] = (p[1] + (P4(-1, -1) << 1) + p[5] + 2) >> 2;
                else pr[y][x] = (P4(-1, y - 1) + (P4(-1, y - 2) << 1) + P4(-1, y - 3) + 2) >> 2;
            }
        break;
    case 6:
        for (y = 0; y < 4; ++y)
            for (x = 0; x < 4; ++x) {
                int z = 2 * y - x;
                if (z >= 0 && !(z & 1)) pr[y][x] = (P4(-1, y - (x >> 1) - 1) + P4(-1, y - (x >> 1)) + 1) >> 1;
                else if (z >= 0) pr[y][x] = (P4(-1, y - (x >> 1) - 2) + 2 * P4(-1, y - (x >> 1) - 1) + P4(-1, y - (x >> 1)) + 2) >> 2;
                else if (z == -1) pr[y][x] = (p[1] + 2 * P4(-1, -1) + p[5] + 2) >> 2;
                else pr[y][x] = (P4(x - 1, -1) + 2 * P4(x - 2, -1) + P4(x - 3, -1) + 2) >> 2;
            }
        break;
    case 7:
        for (x = 0; x < 4; ++x) {
            pr[0][x] = (P4(x, -1) + P4(x + 1, -1) + 1) >> 1;
            pr[2][x] = (P4(x + 1, -1) + P4(x + 2, -1) + 1) >> 1;
            pr[1][x] = (P4(x, -1) + 2 * P4(x + 1, -1) + P4(x + 2, -1) + 2) >> 2;
            pr[3][x] = (P4(x + 1, -1) + 2 * P4(x + 2, -1) + P4(x + 3, -1) + 2) >> 2;
        }
        break;
    default:
        for (x = 0; x < 4; ++x)
            for (y = 0; y < 4; ++y) {
                int z = x + 2 * y;
                if (z == 0 || z == 2 || z == 4) pr[y][x] = (P4(-1, y + (x >> 1)) + P4(-1, y + (x >> 1) + 1) + 1) >> 1;
                else if (z == 1 || z == 3) pr[y][x] = (P4(-1, y + (x >> 1)) + 2 * P4(-1, y + (x >> 1) + 1) + P4(-1, y + (x >> 1) + 2) + 2) >> 2;
                else if (z == 5) pr[y][x] = (p[3] + 3 * p[4] + 2) >> 2;
                else pr[y][x] = p[4];
            }
        break;
    }
}
static void pred16x16(int mode, const int p[33], int32_t pr[16][16]) /* pred_intra.c:855-1041 */
{
    int x, y;
    if (mode == 0) {
        for (y = 0; y < 16; ++y) for (x = 0; x < 16; ++x) pr[y][x] = p[17 + x];
    }
    else if (mode == 1) {
        for (y = 0; y < 16; ++y) for (x = 0; x < 16; ++x) pr[y][x] = p[1 + y];
    }
    else if (mode == 2) {
        int xa = 1, ya = 1, xs = 0, ys = 0, r;
        for (x = 0; x < 16; ++x) {
            if (p[17 + x] == NOT_AVAIL) { xa = 0; break; }
            xs += p[17 + x];
        }
        for (y = 0; y < 16; ++y) {
            if (p[1 + y] == NOT_AVAIL) { ya = 0; break; }
            ys += p[1 + y];
        }
        if (xa && ya) r = (xs + ys + 16) >> 5;
        else if (!xa && ya) r = (ys + 8) >> 4;
        else if (!ya && xa) r = (xs + 8) >> 4;
        else r = 128;
        for (y = 0; y < 16; ++y) for (x = 0; x < 16; ++x) pr[y][x] = r;
    }
    else {
        int H = 0, V = 0, a, b, c, i;
        for (i = 0; i < 7; ++i) {
            H += (i + 1) * (p[25 + i] - p[23 - i]);
            V += (i + 1) * (p[9 + i] - p[7 - i]);
        }
        H += 8 * (p[32] - p[0]);
        V += 8 * (p[16] - p[0]);
        a = (p[16] + p[32]) << 4;
        b = (5 * H + 32) >> 6;
        c = (5 * V + 32) >> 6;
        for (y = 0; y < 16; ++y)
            for (x = 0; x < 16; ++x) pr[y][x] = clip255((a + b * (x - 7) + c * (y - 7) + 16) >> 5);
    }
}
static void predChroma(int mode, const int p[17], int32_t pr[16][16]) /* pred_intra.c:1043-1220 */
{
    int x, y;
    const int* px = &p[9];
    const int* py = &p[1];
    if (mode == 0) {
        int xa = 1, ya = 1, b; /* availability flags are not reset per block (pred_intra.c:1046) */
        for (b = 0; b < 4; ++b) {
            int xO = (b & 1) * 4, yO = (b >> 1) * 4, xs = 0, ys = 0, t = 128;
            for (x = 0; x < 4; ++x) {
                if (px[xO + x] == NOT_AVAIL) { xa = 0; break; }
                xs += px[xO + x];
            }
            for (y = 0; y < 4; ++y) {
                if (py[yO + y] == NOT_AVAIL) { ya = 0; break; }
                ys += py[yO + y];
            }
            if ((xO == 0 && yO == 0) || (xO > 0 && yO > 0)) {
                if (xa && ya) t = (xs + ys + 4) >> 3;
                else if (!xa && ya) t = (ys + 2) >> 2;
                else if (!ya && xa) t = (xs + 2) >> 2;
            }
            else if (xO > 0 && yO == 0) {
                if (xa) t = (xs + 2) >> 2;
                else if (ya) t = (ys + 2) >> 2;
            }
            else {
                if (ya) t = (ys + 2) >> 2;
                else if (xa) t = (xs + 2) >> 2;
            }
            for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) pr[yO + y][xO + x] = t;
        }
    }
    else if (mode == 1) {
        for (y = 0; y < 8; ++y) for (x = 0; x < 8; ++x) pr[y][x] = py[y];
    }
    else if (mode == 2) {
        for (y = 0; y < 8; ++y) for (x = 0; x < 8; ++x) pr[y][x] = px[x];
    }
    else {
        int H = 0, V = 0, a, b, c, i;
        for (i = 0; i < 3; ++i) {
            H += (i + 1) * (p[13 + i] - p[11 - i]);
            V += (i + 1) * (p[5 + i] - p[3 - i]);
        }
        H += 4 * (p[16] - p[0]);
        V += 4 * (p[8] - p[0]);
        a = (p[8] + p[16]) << 4;
        b = (34 * H + 32) >> 6;
        c = (34 * V + 32) >> 6;
        for (y = 0; y < 8; ++y)
            for (x = 0; x < 8; ++x) pr[y][x] = clip255((a + b * (x - 3) + c * (y - 3) + 16) >> 5);
    }
}

/* picture construction (pict.c:223-303) */
static void put_luma4x4(hlo_enc_t* e, const mb_t* m, int blk, const int32_t* s, int stride)
{
    int x, y, xO = m->xL + BLK_XY[blk][0], yO = m->yL + BLK_XY[blk][1];
    for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) e->cur[0][(yO + y) * e->W + xO + x] = (uint8_t)s[y * stride + x];
}
static void put_chroma8x8(hlo_enc_t* e, const mb_t* m, int c, const int32_t u[16][16])
{
    int x, y;
    for (y = 0; y < 8; ++y) for (x = 0; x < 8; ++x) e->cur[1 + c][(m->yC + y) * e->Wc + m->xC + x] = (uint8_t)u[y][x];
}

/* ------------------------------------------------------------------------- */
/* Chroma transform decoding (transf.c:161-294)                              */
/* ------------------------------------------------------------------------- */
static void decode_chroma(hlo_enc_t* e, mb_t* m, const int32_t predC[16][16], int c)
{
    int32_t dcC[2][2] = {{0, 0}, {0, 0}}, rMb[16][16], u[16][16];
    int b, x, y;
    if (m->CbpCDC[c] == 0 && m->CbpCAC[c] == 0) {
        put_chroma8x8(e, m, c, predC);
        return;
    }
    memset(rMb, 0, sizeof(rMb));
    if (m->CbpCDC[c] != 0) { /* 8.5.11 */
        int32_t cc[2][2], t[2][2], f[2][2];
        int qP = m->QPprimeC[c], scale = e->level_scale[qP % 6][0][0];
        cc[0][0] = m->ChromaDCLevel[c][0];
        cc[0][1] = m->ChromaDCLevel[c][1];
        cc[1][0] = m->ChromaDCLevel[c][2];
        cc[1][1] = m->ChromaDCLevel[c][3];
        t[0][0] = cc[0][0] + cc[1][0];
        t[0][1] = cc[0][1] + cc[1][1];
        t[1][0] = cc[0][0] - cc[1][0];
        t[1][1] = cc[0][1] - cc[1][1];
        f[0][0] = t[0][0] + t[0][1];
        f[0][1] = t[0][0] - t[0][1];
        f[1][0] = t[1][0] + t[1][1];
        f[1][1] = t[1][0] - t[1][1];
        for (y = 0; y < 2; ++y)
            for (x = 0; x < 2; ++x) dcC[y][x] = ((f[y][x] * scale) << (qP / 6)) >> 5;
    }
    for (b = 0; b < 4; ++b) {
        int32_t list[16];
        list[0] = dcC[b >> 1][b & 1];
        if (list[0] || (m->CbpCAC[c] & (1 << b))) {
            int32_t cf[4][4], r[4][4];
            memcpy(&list[1], &m->ChromaACLevel[c][b][0], 15 * sizeof(int32_t));
            inverse_scan(list, cf);
            scale_residual(e, m->QPprimeC[c], cf, 1, r);
            for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) rMb[(b >> 1) * 4 + y][(b & 1) * 4 + x] = r[y][x];
        }
    }
    for (y = 0; y < 8; ++y) for (x = 0; x < 8; ++x) u[y][x] = clip255(predC[y][x] + rMb[y][x]);
    put_chroma8x8(e, m, c, u);
}

/* _hl_codec_264_rdo_mb_reconstruct_chroma, rdo.c:2502-2701 */
static void reconstruct_chroma(hlo_enc_t* e, mb_t* m, const int32_t predCb[16][16], const int32_t predCr[16][16])
{
    int32_t single[2] = {0, 0}, tcs[2] = {0, 0}, DC[2][2][2];
    int isIntra = is_intra(m), b, c, x, y;
    bw_t bw;
    bw_init(&bw, NULL, 0);
    m->CbpCAC[0] = m->CbpCAC[1] = 0;
    m->CbpCDC[0] = m->CbpCDC[1] = 0;
    for (b = 0; b < 4; ++b) {
        int xO = (b & 1) * 4, yO = (b >> 1) * 4;
        for (c = 0; c < 2; ++c) {
            const int32_t(*pred)[16] = c ? predCr : predCb;
            const uint8_t* src = e->src[1 + c] + (m->yC + yO) * e->Wc + m->xC + xO;
            int32_t res[4][4], t[4][4], q[4][4];
            for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) res[y][x] = (int32_t)src[y * e->Wc + x] - pred[yO + y][xO + x];
            if (!allzero16(&res[0][0])) {
                int az;
                fwd4x4(res, t);
                quant_ac(m->QPc[c], 1, t, q); /* intra rounding for every MB (rdo.c:2588,2618) */
                scan_l(q, m->ChromaACLevel[c][b], 1);
                az = allzero16(m->ChromaACLevel[c][b]);
                DC[c][yO >> 2][xO >> 2] = t[0][0];
                m->CbpCAC[c] |= az ? 0 : (1 << b);
                m->CbpCDC[c] |= t[0][0] ? (1 << b) : 0;
            }
            else {
                DC[c][yO >> 2][xO >> 2] = 0;
            }
            if (single[c] < 7 && (m->CbpCAC[c] & (1 << b))) {
                wb_chroma_ac(e, m, &bw, c, b, m->ChromaACLevel[c][b], 0, 15, 16, 1);
                single[c] += e->rdo_single_ctr;
                tcs[c] += m->TCChromaAC[c][b];
            }
        }
    }
    for (c = 0; c < 2; ++c)
        if (single[c] < 7 && tcs[c] == 1) m->CbpCAC[c] = 0;
    if (m->CbpCDC[0] || m->CbpCDC[1]) {
        for (c = 0; c < 2; ++c) {
            if (m->CbpCDC[c]) {
                int32_t t[2][2], o[2][2];
                t[0][0] = DC[c][0][0] + DC[c][1][0];
                t[0][1] = DC[c][0][1] + DC[c][1][1];
                t[1][0] = DC[c][0][0] - DC[c][1][0];
                t[1][1] = DC[c][0][1] - DC[c][1][1];
                o[0][0] = quant_dc1(m->QPc[c], isIntra, t[0][0] + t[0][1]);
                o[0][1] = quant_dc1(m->QPc[c], isIntra, t[0][0] - t[0][1]);
                o[1][0] = quant_dc1(m->QPc[c], isIntra, t[1][0] + t[1][1]);
                o[1][1] = quant_dc1(m->QPc[c], isIntra, t[1][0] - t[1][1]);
                m->ChromaDCLevel[c][0] = o[0][0];
                m->ChromaDCLevel[c][1] = o[0][1];
                m->ChromaDCLevel[c][2] = o[1][0];
                m->ChromaDCLevel[c][3] = o[1][1];
                m->CbpCDC[c] = (o[0][0] ? 1 : 0) | (o[0][1] ? 2 : 0) | (o[1][0] ? 4 : 0) | (o[1][1] ? 8 : 0);
            }
        }
    }
    decode_chroma(e, m, predCb, 0);
    decode_chroma(e, m, predCr, 1);
}

static void guess_cbp(mb_t* m) /* rdo.c:2703-2782 */
{
    if ((m->flags & FL_INTRA16) == FL_INTRA16) {
        m->CbpL = m->CbpL4x4 ? 15 : 0;
    }
    else {
        int i8;
        m->CbpL = 0;
        for (i8 = 0; i8 < 4; ++i8)
            if (m->CbpL4x4 & (0xF << (i8 * 4))) m->CbpL |= 1 << i8;
    }
    if ((m->CbpCDC[0] || m->CbpCDC[1]) && (!m->CbpCAC[0] && !m->CbpCAC[1])) m->CbpC = 1;
    else if (m->CbpCAC[0] || m->CbpCAC[1]) m->CbpC = 2;
    else m->CbpC = 0;
    m->cbp = (m->CbpC << 4) | m->CbpL;
    if (m->cbp > 47) {
        m->cbp -= 16;
        m->CbpC = m->cbp >> 4;
    }
}

/* ------------------------------------------------------------------------- */
/* Intra RDO (rdo.c:99-299, 1526-2136)                                       */
/* ------------------------------------------------------------------------- */
static void guess_intra16x16(hlo_enc_t* e, mb_t* m, double lambda, int32_t* cbp4x4_out, int32_t* best_dist, double* best_cost)
{
    int p[33], mode, blk, x, y;
    const uint8_t* eS = e->src[0] + m->yL * e->W + m->xL;
    *best_cost = DBL_MAX;
    *cbp4x4_out = 0;
    m->e_type = ET_I16;
    m->flags = FL_INTRA16;
    m->MbPartPredMode[0] = PM_I16;
    m->I16Mode = 2;
    nb16x16L(e, m, p);
    for (mode = 0; mode < 4; ++mode) {
        int32_t pred[16][16], DCc[4][4], AC[16][16], DCl[16];
        int32_t bcbp = 0, single = 0;
        double dist = 0, rate, cost;
        bw_t bw;
        if (mode == 0 && p[17] == NOT_AVAIL) continue;
        if (mode == 1 && p[1] == NOT_AVAIL) continue;
        if (mode == 3 && p[0] == NOT_AVAIL) continue;
        bw_init(&bw, NULL, 0);
        pred16x16(mode, p, pred);
        for (blk = 0; blk < 16; ++blk) {
            int xO = BLK_XY[blk][0], yO = BLK_XY[blk][1];
            int32_t res[4][4], t[4][4], q[4][4];
            for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) res[y][x] = (int32_t)eS[(yO + y) * e->W + xO + x] - pred[yO + y][xO + x];
            fwd4x4(res, t);
            quant_ac(m->QPy, 1, t, q);
            scan_l(q, AC[blk], 1);
            AC[blk][15] = 0;
            if (!allzero16(&q[0][0])) {
                wb_luma(e, m, &bw, RES_I16_AC, blk, AC[blk], 0, 15, 16, 1);
                bcbp |= 1 << blk;
                single += e->rdo_single_ctr;
            }
            DCc[yO >> 2][xO >> 2] = t[0][0];
        }
        if (bcbp && single < 6) bcbp = 0;
        if (bcbp) {
            int32_t h[4][4], q[4][4], c[4][4], dcY[4][4], rMb[16][16], u[16][16];
            hadamard4x4(DCc, h);
            for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) q[y][x] = quant_dc1(m->QPy, 1, h[y][x]);
            scan_l(q, DCl, 0);
            wb_luma(e, m, &bw, RES_I16_DC, 0, DCl, 0, 15, 16, 1);
            inverse_scan(DCl, c);
            scale_luma_dc(e, m, c, dcY);
            memset(rMb, 0, sizeof(rMb));
            for (blk = 0; blk < 16; ++blk) {
                int32_t list[16];
                list[0] = dcY[DCYIJ[blk][0]][DCYIJ[blk][1]];
                memcpy(&list[1], AC[blk], 15 * sizeof(int32_t));
                if (!allzero16(list)) {
                    int32_t cf[4][4], r[4][4];
                    inverse_scan(list, cf);
                    scale_residual(e, m->QPyprime, cf, 1, r);
                    for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) rMb[BLK_XY[blk][1] + y][BLK_XY[blk][0] + x] = r[y][x];
                }
            }
            for (y = 0; y < 16; ++y) for (x = 0; x < 16; ++x) u[y][x] = clip255(pred[y][x] + rMb[y][x]);
            for (blk = 0; blk < 16; ++blk) {
                uint8_t t8[16];
                int xO = BLK_XY[blk][0], yO = BLK_XY[blk][1];
                for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) t8[y * 4 + x] = (uint8_t)u[yO + y][xO + x];
                dist += sad4x4(eS + yO * e->W + xO, e->W, t8, 4);
            }
        }
        else {
            memset(DCl, 0, sizeof(DCl));
            for (blk = 0; blk < 16; ++blk) {
                uint8_t t8[16];
                int xO = BLK_XY[blk][0], yO = BLK_XY[blk][1];
                for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) t8[y * 4 + x] = (uint8_t)pred[yO + y][xO + x];
                dist += sad4x4(eS + yO * e->W + xO, e->W, t8, 4);
            }
        }
        if (bw.nbits > RDO_BUFFER_BITS) e->rdo_overflows++;
        rate = (double)bw.nbits;
        cost = dist + lambda * rate;
        if (cost < *best_cost) {
            *best_cost = cost;
            *best_dist = (int32_t)dist;
            *cbp4x4_out = bcbp;
            m->I16Mode = mode;
            memcpy(m->I16AC, AC, sizeof(AC));
            memcpy(m->I16DC, DCl, sizeof(DCl));
        }
    }
}

static void guess_intra4x4(hlo_enc_t* e, mb_t* m, double lambda, int32_t* cbp4x4_out, int32_t* best_dist, double* best_cost)
{
    int blk, mode, x, y;
    int32_t bestPred[16][4][4], single = 0, bestSingle = 0;
    const uint8_t* eS0 = e->src[0] + m->yL * e->W + m->xL;
    *best_cost = 0;
    *best_dist = 0;
    *cbp4x4_out = 0;
    m->e_type = ET_I_NXN;
    m->flags = FL_INTRA4;
    m->MbPartPredMode[0] = PM_I4;
    for (blk = 0; blk < 16; ++blk) {
        int p[13], xO = BLK_XY[blk][0], yO = BLK_XY[blk][1];
        const uint8_t* eS = eS0 + yO * e->W + xO;
        double dmin_cost = DBL_MAX, dmin_dist = 0;
        int best_all_zeros = 0;
        int32_t lv[16];
        m->I4Mode[blk] = 2;
        nb4x4L(e, m, blk, p);
        for (mode = 0; mode < 9; ++mode) {
            int32_t pred[4][4], res[4][4];
            double dist = 0, cost = 0;
            int isAllZeros;
            if ((mode == 0 || mode == 3 || mode == 7) && p[5] == NOT_AVAIL) continue;
            if ((mode == 1 || mode == 8) && p[1] == NOT_AVAIL) continue;
            if ((mode == 4 || mode == 5 || mode == 6) && p[0] == NOT_AVAIL) continue;
            pred4x4(mode, p, pred);
            for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) res[y][x] = (int32_t)eS[y * e->W + x] - pred[y][x];
            isAllZeros = allzero16(&res[0][0]);
            if (isAllZeros) { /* exact match: stop searching (rdo.c:1949-1958) */
                dmin_cost = 0;
                dmin_dist = 0;
                m->I4Mode[blk] = mode;
                best_all_zeros = 1;
                memcpy(bestPred[blk], pred, sizeof(pred));
                memset(m->LumaLevel[blk], 0, sizeof(m->LumaLevel[blk]));
                break;
            }
            else {
                int32_t t[4][4], q[4][4];
                uint8_t t8[16];
                bw_t bw;
                bw_init(&bw, NULL, 0);
                fwd4x4(res, t);
                quant_ac(m->QPy, 1, t, q);
                scan_l(q, lv, 0);
                isAllZeros = allzero16(lv);
                if (!isAllZeros) {
                    int32_t cf[4][4], r[4][4];
                    wb_luma(e, m, &bw, RES_LUMA, blk, lv, 0, 15, 16, 1);
                    inverse_scan(lv, cf);
                    scale_residual(e, m->QPyprime, cf, 0, r);
                    for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) t8[y * 4 + x] = (uint8_t)clip255(pred[y][x] + r[y][x]);
                }
                else {
                    for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) t8[y * 4 + x] = (uint8_t)pred[y][x];
                }
                dist = sad4x4(eS, e->W, t8, 4);
                if (bw.nbits > RDO_BUFFER_BITS) e->rdo_overflows++;
                cost = dist + lambda * (double)bw.nbits;
            }
            if (cost < dmin_cost) {
                dmin_cost = cost;
                dmin_dist = dist;
                m->I4Mode[blk] = mode;
                best_all_zeros = isAllZeros;
                bestSingle = isAllZeros ? 0 : e->rdo_single_ctr;
                memcpy(bestPred[blk], pred, sizeof(pred));
                memcpy(m->LumaLevel[blk], lv, sizeof(lv));
            }
        }
        *best_cost = *best_cost + dmin_cost;
        *best_dist = (int32_t)(*best_dist + dmin_dist);
        if (!best_all_zeros) {
            *cbp4x4_out |= 1 << blk;
            single += bestSingle;
        }
        if (*cbp4x4_out & (1 << blk)) {
            int32_t cf[4][4], r[4][4], u[4][4];
            inverse_scan(m->LumaLevel[blk], cf);
            scale_residual(e, m->QPyprime, cf, 0, r);
            for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) u[y][x] = clip255(bestPred[blk][y][x] + r[y][x]);
            put_luma4x4(e, m, blk, &u[0][0], 4);
        }
        else {
            put_luma4x4(e, m, blk, &bestPred[blk][0][0], 4);
        }
    }
    (void)single;
}

static void pred_modes_4x4(const hlo_enc_t* e, mb_t* m) /* pred_intra.c:541-615 */
{
    int blk;
    for (blk = 0; blk < 16; ++blk) {
        const nb4_t* nb = &m->nbL[blk];
        const mb_t* A = nb->addrA >= 0 ? &e->mbs[nb->addrA] : NULL;
        const mb_t* B = nb->addrB >= 0 ? &e->mbs[nb->addrB] : NULL;
        int dcf = (!A || !B), mA, mB, pred;
        if (dcf || A->MbPartPredMode[0] != PM_I4) mA = 2;
        else mA = A->I4Mode[nb->blkA];
        if (dcf || B->MbPartPredMode[0] != PM_I4) mB = 2;
        else mB = B->I4Mode[nb->blkB];
        pred = mA < mB ? mA : mB;
        if (pred == m->I4Mode[blk]) m->prev_flag[blk] = 1;
        else {
            m->prev_flag[blk] = 0;
            m->rem_mode[blk] = m->I4Mode[blk] < pred ? m->I4Mode[blk] : m->I4Mode[blk] - 1;
        }
    }
}

/* transf.c:298-373 via rdo.c:2100-2136 */
static void reconstruct_intra16x16_luma(hlo_enc_t* e, mb_t* m)
{
    int p[33], x, y, blk;
    int32_t pred[16][16], u[16][16];
    nb16x16L(e, m, p);
    pred16x16(m->I16Mode, p, pred);
    if (!m->CbpL4x4) {
        for (y = 0; y < 16; ++y) for (x = 0; x < 16; ++x) e->cur[0][(m->yL + y) * e->W + m->xL + x] = (uint8_t)pred[y][x];
        return;
    }
    {
        int32_t c[4][4], dcY[4][4], rMb[16][16];
        inverse_scan(m->I16DC, c);
        scale_luma_dc(e, m, c, dcY);
        memset(rMb, 0, sizeof(rMb));
        for (blk = 0; blk < 16; ++blk) {
            int32_t list[16];
            list[0] = dcY[DCYIJ[blk][0]][DCYIJ[blk][1]];
            memcpy(&list[1], m->I16AC[blk], 15 * sizeof(int32_t));
            if (!allzero16(list)) {
                int32_t cf[4][4], r[4][4];
                inverse_scan(list, cf);
                scale_residual(e, m->QPyprime, cf, 1, r);
                for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) rMb[BLK_XY[blk][1] + y][BLK_XY[blk][0] + x] = r[y][x];
            }
        }
        for (y = 0; y < 16; ++y) for (x = 0; x < 16; ++x) u[y][x] = clip255(pred[y][x] + rMb[y][x]);
        for (y = 0; y < 16; ++y) for (x = 0; x < 16; ++x) e->cur[0][(m->yL + y) * e->W + m->xL + x] = (uint8_t)u[y][x];
    }
}

/* hl_codec_264_rdo_mb_guess_best_intra_pred_avc, rdo.c:99-299 */
static void guess_intra(hlo_enc_t* e, mb_t* m)
{
    double c16, c4, lambda = e->lambda_mode;
    int32_t cbp16, cbp4 = 0, d16, d4;
    guess_intra16x16(e, m, lambda, &cbp16, &d16, &c16);
    if (c16 == 0) {
        d4 = INT_MAX;
        c4 = DBL_MAX;
    }
    else {
        guess_intra4x4(e, m, lambda, &cbp4, &d4, &c4);
    }
    switch (m->I16Mode) {
    case 0: m->chroma_mode = 2; break;
    case 3: m->chroma_mode = 3; break;
    case 1: m->chroma_mode = 1; break;
    case 2: m->chroma_mode = 0; break;
    }
    if (c4 < c16) {
        int rbc, blk, nz = 0;
        m->mb_type = 0;
        m->e_type = ET_I_NXN;
        m->flags = FL_INTRA4;
        m->MbPartPredMode[0] = PM_I4;
        m->CbpL4x4 = cbp4;
        pred_modes_4x4(e, m);
        for (blk = 0; blk < 16; ++blk) nz += !m->prev_flag[blk];
        rbc = 16 + nz * 3;
        c4 += lambda * rbc;
    }
    if (c16 <= c4) {
        m->mb_type = 1;
        m->e_type = ET_I16;
        m->flags = FL_INTRA16;
        m->MbPartPredMode[0] = PM_I16;
        m->CbpL4x4 = cbp16;
    }
    e->last_best_intra_cost = c16 < c4 ? c16 : c4;
    {
        int pCb[17], pCr[17];
        int32_t predCb[16][16], predCr[16][16];
        nbC(e, m, pCb, pCr);
        predChroma(m->chroma_mode, pCb, predCb);
        predChroma(m->chroma_mode, pCr, predCr);
        reconstruct_chroma(e, m, predCb, predCr);
    }
    if ((m->flags & FL_INTRA16) == FL_INTRA16) reconstruct_intra16x16_luma(e, m);
    guess_cbp(m);
    if ((m->flags & FL_INTRA16) == FL_INTRA16) m->mb_type += (m->CbpC << 2) + m->I16Mode + (m->CbpL ? 12 : 0);
    if (!e->is_intra_slice) m->mb_type += 5;
}

/* ------------------------------------------------------------------------- */
/* Motion estimation: diamond search with full RDO cost (me_ds.c:104-688)     */
/* ------------------------------------------------------------------------- */
typedef struct {
    int NumMbPart, NumSubMbPart[4], SubMbPartWidth[4], SubMbPartHeight[4], SubMbPredType[4];
    int MbPartWidth, MbPartHeight, NumHeaderBits, Mode;
} part_t;

static const part_t PART_16x16 = {1, {1}, {16}, {16}, {SUB_NA}, 16, 16, 3, MODE_16x16};
static const part_t PART_16x8 = {2, {1, 1}, {16, 16}, {8, 8}, {SUB_NA, SUB_NA}, 16, 8, 5, MODE_16x8};
static const part_t PART_8x16 = {2, {1, 1}, {8, 8}, {16, 16}, {SUB_NA, SUB_NA}, 8, 16, 5, MODE_8x16};
static const part_t PART_8x8[4] = {
    {4, {1, 1, 1, 1}, {8, 8, 8, 8}, {8, 8, 8, 8}, {SUB_8x8, SUB_8x8, SUB_8x8, SUB_8x8}, 8, 8, 11, MODE_8x8_8x8},
    {4, {2, 2, 2, 2}, {8, 8, 8, 8}, {4, 4, 4, 4}, {SUB_8x4, SUB_8x4, SUB_8x4, SUB_8x4}, 8, 8, 19, MODE_8x8_8x4},
    {4, {2, 2, 2, 2}, {4, 4, 4, 4}, {8, 8, 8, 8}, {SUB_4x8, SUB_4x8, SUB_4x8, SUB_4x8}, 8, 8, 19, MODE_8x8_4x8},
    {4, {4, 4, 4, 4}, {4, 4, 4, 4}, {4, 4, 4, 4}, {SUB_4x4, SUB_4x4, SUB_4x4, SUB_4x4}, 8, 8, 27, MODE_8x8_4x4}};

/* compute_cost_mode, me_ds.c:527-688 (+ rdo.c:2784-2830) */
static void cost_mode(hlo_enc_t* e, mb_t* m, int pi, int spi, mv_t mv, int32_t* single, int32_t* rbc, int32_t* dist, int32_t* cbp4x4)
{
    me_t* me = &e->me;
    uint8_t pred[16][16];
    int pw = m->partWidth[pi][spi], ph = m->partHeight[pi][spi], hx, hy, x, y;
    bw_t bw;
    bw_init(&bw, NULL, 0);
    *single = 0;
    *rbc = 0;
    *dist = 0;
    *cbp4x4 = 0;
    m->xL_Idx = me->xL_Idx[pi][spi];
    m->yL_Idx = me->yL_Idx[pi][spi];
    pred_luma(e, m->xL_Idx, m->yL_Idx, mv, pw, ph, pred);
    for (hy = 0; hy < (ph >> 2); ++hy) {
        const uint8_t* src = e->src[0] + (m->yL_Idx + (hy << 2)) * e->W + m->xL_Idx;
        for (hx = 0; hx < (pw >> 2); ++hx) {
            int blk = luma_blk_idx(me->xP[pi][spi] + me->xS[pi][spi] + (hx << 2), me->yP[pi][spi] + me->yS[pi][spi] + (hy << 2));
            int32_t res[4][4], lv[16];
            int zeros;
            const uint8_t* pp = &pred[hy << 2][hx << 2];
            for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) res[y][x] = (int32_t)src[y * e->W + x] - pp[y * 16 + x];
            zeros = allzero16(&res[0][0]);
            if (!zeros) {
                int32_t t[4][4], q[4][4];
                fwd4x4(res, t);
                quant_ac(m->QPy, 0, t, q);
                scan_l(q, lv, 0);
                zeros = allzero16(lv);
            }
            if (!zeros) {
                int32_t cf[4][4], r[4][4];
                uint8_t t8[16];
                wb_luma(e, m, &bw, RES_LUMA, blk, lv, 0, 15, 16, 1);
                inverse_scan(lv, cf);
                scale_residual(e, m->QPyprime, cf, 0, r);
                for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) t8[y * 4 + x] = (uint8_t)clip255(pp[y * 16 + x] + r[y][x]);
                *dist += sad4x4(src, e->W, t8, 4);
                *single += e->rdo_single_ctr;
                *cbp4x4 |= 1 << blk;
            }
            else {
                *dist += sad4x4(src, e->W, pp, 16);
            }
            src += 4;
        }
    }
    if (bw.nbits > RDO_BUFFER_BITS) e->rdo_overflows++;
    *rbc = (int32_t)bw.nbits;
}

#define SET_COST(pi, spi, c, s, d, cb, mv_) \
    do {                                     \
        me->single_ctr[pi][spi] = (s);       \
        me->best_cost[pi][spi] = (c);        \
        me->best_dist[pi][spi] = (d);        \
        me->mvBest[pi][spi] = (mv_);         \
        me->best_cbp4x4[pi][spi] = (cb);     \
    } while (0)

static void find_best_cost(hlo_enc_t* e, mb_t* m, const part_t* part) /* me_ds.c:104-477 */
{
    static const int DS_INT[9][2] = {{0, 2}, {-1, 1}, {1, 1}, {-2, 0}, {0, 0}, {2, 0}, {-1, -1}, {1, -1}, {0, -2}};
    static const int DS_HALF[5][2] = {{0, 1}, {-1, 0}, {0, -1}, {1, 0}, {0, 0}};
    static const int DS_QUAR[9][2] = {{-1, 1}, {0, 1}, {1, 1}, {-1, 0}, {0, 0}, {1, 0}, {-1, -1}, {0, -1}, {1, -1}};
    /* skip masks, me_ds.c:385-465 (bit i = candidate i) */
    static const int MASK_INT[9] = {
        ~(16 | 64 | 256 | 128), ~(16 | 32 | 256), ~(16 | 2 | 8 | 64 | 256 | 128), ~(16 | 4 | 32 | 128), ~0,
        ~(16 | 2 | 8 | 64), ~(16 | 1 | 2 | 128 | 32 | 4), ~(16 | 1 | 2 | 8 | 64 | 4), ~(16 | 4 | 1 | 2)};
    static const int MASK_HALF[5] = {~(16 | 4), ~(16 | 8), ~(16 | 1), ~(16 | 2), ~0};
    static const int MASK_QUAR[9] = {
        ~(16 | 32 | 256 | 128), ~(16 | 8 | 64 | 128 | 256 | 32), ~(16 | 8 | 1 | 2 | 4 | 32), ~(16 | 2 | 4 | 32 | 256 | 128), ~0,
        ~(16 | 1 | 2 | 8 | 64 | 128), ~(16 | 2 | 4 | 32), ~(16 | 1 | 2 | 4 | 8 | 32), ~(16 | 1 | 2 | 8)};
    me_t* me = &e->me;
    int pi, spi;
    int32_t single, rbc, dist, cbp4, rbc_mv;
    double cost;
    mv_t mv;

    m->NumMbPart = part->NumMbPart;
    m->MbPartWidth = part->MbPartWidth;
    m->MbPartHeight = part->MbPartHeight;
    for (pi = 0; pi < part->NumMbPart; ++pi) {
        m->predFlagL0[pi] = 1;
        m->MbPartPredMode[pi] = PM_L0;
        m->SubMbPredType[pi] = part->SubMbPredType[pi];
        m->NumSubMbPart[pi] = part->NumSubMbPart[pi];
        m->SubMbPartWidth[pi] = part->SubMbPartWidth[pi];
        m->SubMbPartHeight[pi] = part->SubMbPartHeight[pi];
        for (spi = 0; spi < m->NumSubMbPart[pi]; ++spi) {
            m->partWidth[pi][spi] = m->SubMbPartWidth[pi];
            m->partHeight[pi][spi] = m->SubMbPartHeight[pi];
            m->partWidthC[pi][spi] = m->partWidth[pi][spi] >> 1;
            m->partHeightC[pi][spi] = m->partHeight[pi][spi] >> 1;
            if (pi == 0 && spi == 0) {
                me->xL_Idx[0][0] = m->xL;
                me->yL_Idx[0][0] = m->yL;
                me->xP[0][0] = me->yP[0][0] = me->xS[0][0] = me->yS[0][0] = 0;
            }
            else {
                me->xP[pi][spi] = inv_raster(pi, m->MbPartWidth, m->MbPartHeight, 16, 0);
                me->yP[pi][spi] = inv_raster(pi, m->MbPartWidth, m->MbPartHeight, 16, 1);
                if (is_8x8_type(m->e_type)) {
                    me->xS[pi][spi] = inv_raster(spi, m->SubMbPartWidth[pi], m->SubMbPartHeight[pi], 8, 0);
                    me->yS[pi][spi] = inv_raster(spi, m->SubMbPartWidth[pi], m->SubMbPartHeight[pi], 8, 1);
                }
                else {
                    me->xS[pi][spi] = (spi & 1) * 4; /* InverseRasterScan16_4x4[spi][8] */
                    me->yS[pi][spi] = (spi >> 1) * 4;
                }
                me->xL_Idx[pi][spi] = m->xL + me->xP[pi][spi] + me->xS[pi][spi];
                me->yL_Idx[pi][spi] = m->yL + me->yP[pi][spi] + me->yS[pi][spi];
            }
            me->single_ctr[pi][spi] = 9;
            me->best_dist[pi][spi] = INT_MAX;
            me->best_cost[pi][spi] = DBL_MAX;
        }
    }
    me->probably_pskip = 0;

    if (part->Mode == MODE_16x16) { /* P-skip probe, me_ds.c:229-261 */
        mv_t smv = skip_mv(e, m);
        mv_t pmv = mvp(e, m, 0, 0);
        me->mvpLX[0][1] = pmv;
        if (pmv.x == smv.x && pmv.y == smv.y) {
            cost_mode(e, m, 0, 0, pmv, &single, &rbc, &dist, &cbp4);
            if (rbc == 0 || single < 6) {
                me->probably_pskip = 1;
                SET_COST(0, 0, 0.0, single, dist, cbp4, pmv);
            }
        }
    }

    for (pi = 0; pi < m->NumMbPart; ++pi) {
        for (spi = 0; spi < m->NumSubMbPart[pi]; ++spi) {
            const int(*idx)[2] = DS_INT;
            int count = 9, shift = 2, flags = 0xFFFFFF, cx, cy;
            mv_t pmv = mvp(e, m, pi, spi);
            me->mvpLX[pi][spi] = pmv;
            cost_mode(e, m, pi, spi, pmv, &single, &rbc, &dist, &cbp4);
            rbc_mv = se_len(0) + se_len(0);
            cost = dist + ((rbc + rbc_mv) * e->lambda_mode);
            if (cost < me->best_cost[pi][spi]) SET_COST(pi, spi, cost, single, dist, cbp4, pmv);
            if (pmv.x != 0 || pmv.y != 0) {
                mv.x = mv.y = 0;
                cost_mode(e, m, pi, spi, mv, &single, &rbc, &dist, &cbp4);
                rbc_mv = se_len(mv.x - pmv.x) + se_len(mv.y - pmv.y);
                cost = dist + ((rbc + rbc_mv) * e->lambda_mode);
                if (cost < me->best_cost[pi][spi]) SET_COST(pi, spi, cost, single, dist, cbp4, mv);
            }
            cx = me->mvBest[pi][spi].x >> 2;
            cy = me->mvBest[pi][spi].y >> 2;
            me->left = cx - me->me_range;
            me->right = cx + me->me_range;
            me->top = cy - me->me_range;
            me->bottom = cy + me->me_range;
            for (;;) {
                int best = -1, i;
                for (i = 0; i < count; ++i) {
                    if (!(flags & (1 << i))) continue;
                    mv.x = cx + idx[i][0];
                    mv.y = cy + idx[i][1];
                    if (mv.x < me->left || mv.x > me->right) continue;
                    if (mv.y < me->top || mv.y > me->bottom) continue;
                    mv.x <<= shift;
                    mv.y <<= shift;
                    cost_mode(e, m, pi, spi, mv, &single, &rbc, &dist, &cbp4);
                    rbc_mv = se_len(mv.x - pmv.x) + se_len(mv.y - pmv.y);
                    cost = dist + ((rbc + rbc_mv) * e->lambda_mode);
                    if (cost < me->best_cost[pi][spi]) {
                        best = i;
                        SET_COST(pi, spi, cost, single, dist, cbp4, mv);
                    }
                }
                flags = 0xFFFFFF;
                if (shift == 2 && best == -1) {
                    shift = 1;
                    idx = DS_HALF;
                    count = 5;
                    cx = me->mvBest[pi][spi].x >> 2; /* integer-pel value reused as half-pel centre (me_ds.c:360) */
                    cy = me->mvBest[pi][spi].y >> 2;
                }
                else if ((shift == 1 || shift == 0) && best == -1) {
                    if (shift == 1) {
                        shift = 0;
                        idx = DS_QUAR;
                        count = 9;
                        cx = me->mvBest[pi][spi].x;
                        cy = me->mvBest[pi][spi].y;
                    }
                    else {
                        break;
                    }
                }
                else {
                    cx = me->mvBest[pi][spi].x >> shift;
                    cy = me->mvBest[pi][spi].y >> shift;
                    if (shift == 2) flags &= MASK_INT[best];
                    else if (shift == 1) flags &= MASK_HALF[best];
                    else flags &= MASK_QUAR[best];
                    continue;
                }
                me->left = cx - me->me_range;
                me->right = cx + me->me_range;
                me->top = cy - me->me_range;
                me->bottom = cy + me->me_range;
            }
            m->MvL0[pi][spi] = me->mvBest[pi][spi];
        }
    }
}

/* ------------------------------------------------------------------------- */
/* Inter reconstruction (rdo.c:2138-2500)                                    */
/* ------------------------------------------------------------------------- */
static void chroma_pred_16x16(hlo_enc_t* e, mb_t* m, mv_t mv, int32_t predCb[16][16], int32_t predCr[16][16])
{
    pred_chroma_part(e, m->xL_Idx, m->yL_Idx, mv, m->partWidthC[0][0], m->partHeightC[0][0], predCb, predCr, 0, 0);
}

static int is_zeros_inter16x16_chroma(hlo_enc_t* e, mb_t* m, mv_t mv) /* rdo.c:2140-2215 */
{
    int32_t predCb[16][16], predCr[16][16];
    chroma_pred_16x16(e, m, mv, predCb, predCr);
    reconstruct_chroma(e, m, predCb, predCr);
    return !m->CbpCAC[0] && !m->CbpCAC[1] && !m->CbpCDC[0] && !m->CbpCDC[1];
}

static void reconstruct_luma_pskip(hlo_enc_t* e, mb_t* m, mv_t mv) /* rdo.c:2217-2269 */
{
    uint8_t pred[16][16];
    int x, y;
    pred_luma(e, m->xL_Idx, m->yL_Idx, mv, m->partWidth[0][0], m->partHeight[0][0], pred);
    for (y = 0; y < 16; ++y) for (x = 0; x < 16; ++x) e->cur[0][(m->yL + y) * e->W + m->xL + x] = pred[y][x];
}

static void reconstruct_inter(hlo_enc_t* e, mb_t* m, int32_t single_luma) /* rdo.c:2274-2500 */
{
    int32_t predL[16][16], predCb[16][16], predCr[16][16];
    int pi, spi, x, y, blk;
    const uint8_t* eS = e->src[0] + m->yL * e->W + m->xL;
    m->CbpL4x4 = 0;
    memset(predCb, 0, sizeof(predCb));
    memset(predCr, 0, sizeof(predCr));
    for (pi = 0; pi < m->NumMbPart; ++pi) {
        int xP = inv_raster(pi, m->MbPartWidth, m->MbPartHeight, 16, 0);
        int yP = inv_raster(pi, m->MbPartWidth, m->MbPartHeight, 16, 1);
        for (spi = 0; spi < m->NumSubMbPart[pi]; ++spi) {
            int xS = 0, yS = 0;
            uint8_t pl[16][16];
            if (!(pi == 0 && spi == 0)) {
                if (is_8x8_type(m->e_type)) {
                    xS = inv_raster(spi, m->SubMbPartWidth[pi], m->SubMbPartHeight[pi], 8, 0);
                    yS = inv_raster(spi, m->SubMbPartWidth[pi], m->SubMbPartHeight[pi], 8, 1);
                }
                else {
                    xS = (spi & 1) * 4;
                    yS = (spi >> 1) * 4;
                }
            }
            m->xL_Idx = m->xL + xP + xS;
            m->yL_Idx = m->yL + yP + yS;
            pred_luma(e, m->xL_Idx, m->yL_Idx, m->mvL0[pi][spi], m->partWidth[pi][spi], m->partHeight[pi][spi], pl);
            for (y = 0; y < m->partHeight[pi][spi]; ++y)
                for (x = 0; x < m->partWidth[pi][spi]; ++x) predL[yP + yS + y][xP + xS + x] = pl[y][x];
            pred_chroma_part(e, m->xL_Idx, m->yL_Idx, m->mvL0[pi][spi], m->partWidthC[pi][spi], m->partHeightC[pi][spi], predCb, predCr,
                             (xP >> 1) + (xS >> 1), (yP >> 1) + (yS >> 1));
        }
    }
    if (single_luma < 6) {
        for (blk = 0; blk < 16; ++blk) {
            int32_t t[16];
            for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) t[y * 4 + x] = predL[BLK_XY[blk][1] + y][BLK_XY[blk][0] + x];
            put_luma4x4(e, m, blk, t, 4);
        }
    }
    else {
        for (blk = 0; blk < 16; ++blk) {
            int xO = BLK_XY[blk][0], yO = BLK_XY[blk][1], az;
            int32_t res[4][4], t[4][4], q[4][4], u[16];
            for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) res[y][x] = (int32_t)eS[(yO + y) * e->W + xO + x] - predL[yO + y][xO + x];
            az = allzero16(&res[0][0]);
            if (!az) {
                fwd4x4(res, t);
                quant_ac(m->QPy, 0, t, q);
                az = allzero16(&q[0][0]);
                if (!az) {
                    scan_l(q, m->LumaLevel[blk], 0);
                    m->CbpL4x4 |= 1 << blk;
                }
            }
            if (az) memset(m->LumaLevel[blk], 0, sizeof(m->LumaLevel[blk]));
            if (m->CbpL4x4 & (1 << blk)) {
                int32_t cf[4][4], r[4][4];
                inverse_scan(m->LumaLevel[blk], cf);
                scale_residual(e, m->QPyprime, cf, 0, r);
                for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) u[y * 4 + x] = clip255(predL[yO + y][xO + x] + r[y][x]);
            }
            else {
                for (y = 0; y < 4; ++y) for (x = 0; x < 4; ++x) u[y * 4 + x] = predL[yO + y][xO + x];
            }
            put_luma4x4(e, m, blk, u, 4);
        }
    }
    reconstruct_chroma(e, m, predCb, predCr);
}

/* hl_math_homogeneousity8x8_u8_cpp, hl_math.c:470-486 (JVT-O079 eq. 2-35):
 * Sobel-like edge energy of the 8x8 block at p (p must not lie on the picture
 * border: the taps reach one sample beyond the block on every side). */
static int32_t homogeneity8x8(const uint8_t* p, int stride)
{
    int32_t i, j, ret = 0;
    for (j = 0; j < 8; ++j) {
        const uint8_t* u = p + stride * j;
        const uint8_t* um = u - stride;
        const uint8_t* up = u + stride;
        for (i = 0; i < 8; ++i) {
            const int32_t dx = up[i - 1] + (up[i] << 1) + up[i + 1] - um[i - 1] - (um[i] << 1) - um[i + 1];
            const int32_t dy = um[i + 1] + (u[i + 1] << 1) + up[i + 1] - um[i - 1] - (u[i - 1] << 1) - up[i - 1];
            ret += (dx < 0 ? -dx : dx) + (dy < 0 ? -dy : dy);
        }
    }
    return ret;
}

/* Early termination (me_early_term_flag), rdo.c:888-931: the partition
 * modes left enabled after the 16x16 search, from the homogeneity of the
 * four 8x8 quadrants of the source MB (JVT-O079 2.1.3.4.3.1).  Bit k+1 =
 * MODE_ k (reference numbering HL_CODEC_264_MODE_16X16 = 1 ...). */
#define HOMO_TH16X16 20000 /* HL_CODEC_264_RDO_HOMOGENEOUSITY_TH16X16, defs.h:61 */
#define HOMO_TH8X8 5000    /* defs.h:62 */
#define HOMO_TH8X4 7500    /* defs.h:63 */
static int early_term_modes(const hlo_enc_t* e, const mb_t* m)
{
    const int W = e->W, H = e->H;
    const int xs = m->xL == 0 ? 1 : (m->xL == W - 16 ? W - 17 : m->xL);
    const int ys = m->yL == 0 ? 1 : (m->yL == H - 16 ? H - 17 : m->yL);
    int32_t h[4];
    int k;
    for (k = 0; k < 4; ++k) h[k] = homogeneity8x8(e->src[0] + (xs + (k & 1) * 8) + (ys + (k >> 1) * 8) * W, W);
    if (h[0] < HOMO_TH8X8 && h[1] < HOMO_TH8X8 && h[2] < HOMO_TH8X8 && h[3] < HOMO_TH8X8) return 1 << 1;
    if (h[0] + h[1] + h[2] + h[3] < HOMO_TH16X16) {
        if (h[0] < HOMO_TH8X8 && h[1] < HOMO_TH8X8) return (1 << 1) | (1 << 2);
        return (1 << 1) | (1 << 3);
    }
    if (h[0] < HOMO_TH8X4 && h[1] < HOMO_TH8X4 && h[2] < HOMO_TH8X4 && h[3] < HOMO_TH8X4) return 0x7E; /* every mode but the 4x4 sub-partitions */
    return 0xFFFF;
}

/* hl_codec_264_rdo_mb_guess_best_inter_pred_avc, rdo.c:678-1271 */
static void guess_inter(hlo_enc_t* e, mb_t* m)
{
    typedef struct { int mbType; const part_t* parts; int count; } pdef_t;
    static const pdef_t DEFS[4] = {{ET_P16x16, &PART_16x16, 1}, {ET_P16x8, &PART_16x8, 1}, {ET_P8x16, &PART_8x16, 1}, {ET_P8x8REF0, PART_8x8, 4}};
    me_t* me = &e->me;
    double best_cost = DBL_MAX;
    int32_t best_single = 9, bestRef[4][4];
    mv_t bestMv[4][4], bestMvp[4][4], MVP[4][4];
    const part_t* bestPart = NULL;
    const pdef_t* bestDef = NULL;
    int best_found = 0, pskip = 0, probably = 0, i, j, pi, spi;
    int mode_flags = 0xFFFF; /* rdo.c:874 (one reference picture) */

    me->me_range = CLIP3(1, 64, e->p.me_range);
    m->flags = FL_INTER_P;
    for (i = 0; i < 4 && !best_found; ++i) {
        const pdef_t* def = &DEFS[i];
        m->e_type = def->mbType;
        for (j = 0; j < def->count; ++j) {
            const part_t* part = &def->parts[j];
            double cost_sum = 0;
            int32_t dist_sum = 0, single_sum = 0;
            /* modes disabled by early termination are skipped; `probably`
             * then keeps the value of the last mode searched (rdo.c:883-885) */
            if (!((1 << (part->Mode + 1)) & mode_flags)) continue;
            if (e->p.early_term && part->Mode == MODE_16x16) mode_flags = early_term_modes(e, m);
            find_best_cost(e, m, part);
            probably = me->probably_pskip;
            for (pi = 0; pi < m->NumMbPart; ++pi)
                for (spi = 0; spi < m->NumSubMbPart[pi]; ++spi) {
                    cost_sum += me->best_cost[pi][spi];
                    dist_sum += me->best_dist[pi][spi];
                    single_sum += me->single_ctr[pi][spi];
                    m->MvL0[pi][spi] = me->mvBest[pi][spi];
                    MVP[pi][spi] = me->mvpLX[pi][spi];
                }
            if (!probably && cost_sum && single_sum < 6) {
                if (m->e_type == ET_P16x16) {
                    mv_t smv = skip_mv(e, m);
                    probably = (smv.x == MVP[0][0].x && smv.y == MVP[0][0].y) && (m->MvL0[0][0].x == MVP[0][0].x && m->MvL0[0][0].y == MVP[0][0].y);
                }
            }
            cost_sum += e->lambda_mode * part->NumHeaderBits;
            if (cost_sum < best_cost) {
                best_cost = cost_sum;
                best_single = single_sum;
                bestPart = part;
                bestDef = def;
                for (pi = 0; pi < part->NumMbPart; ++pi)
                    for (spi = 0; spi < m->NumSubMbPart[pi]; ++spi) {
                        bestRef[pi][spi] = 0;
                        bestMv[pi][spi] = m->MvL0[pi][spi];
                        bestMvp[pi][spi] = MVP[pi][spi];
                    }
            }
        }
        if ((pskip = probably)) pskip = is_zeros_inter16x16_chroma(e, m, bestMv[0][0]);
        best_found |= (best_cost == 0) || pskip;
    }

    if (!pskip) {
        guess_intra(e, m);
        if (e->last_best_intra_cost <= best_cost) return;
    }

    m->flags = FL_INTER;
    for (pi = 0; pi < 4; ++pi) {
        m->refIdxL0[pi] = m->RefIdxL0[pi] = 0;
        m->predFlagL0[pi] = m->PredFlagL0[pi] = 0;
    }
    m->e_type = bestDef->mbType;
    m->mb_type = m->e_type - 301;
    m->NumMbPart = bestPart->NumMbPart;
    m->MbPartWidth = bestPart->MbPartWidth;
    m->MbPartHeight = bestPart->MbPartHeight;
    for (pi = 0; pi < m->NumMbPart; ++pi) {
        m->RefIdxL0[pi] = m->refIdxL0[pi] = bestRef[pi][0];
        m->PredFlagL0[pi] = m->predFlagL0[pi] = 1;
        m->MbPartPredMode[pi] = PM_L0;
        m->SubMbPredType[pi] = bestPart->SubMbPredType[pi];
        m->NumSubMbPart[pi] = bestPart->NumSubMbPart[pi];
        m->SubMbPartWidth[pi] = bestPart->SubMbPartWidth[pi];
        m->SubMbPartHeight[pi] = bestPart->SubMbPartHeight[pi];
        m->sub_mb_type[pi] = (uint32_t)(m->SubMbPredType[pi] - 100 - 1);
        for (spi = 0; spi < m->NumSubMbPart[pi]; ++spi) {
            m->mvL0[pi][spi] = bestMv[pi][spi];
            m->partWidth[pi][spi] = m->SubMbPartWidth[pi];
            m->partHeight[pi][spi] = m->SubMbPartHeight[pi];
            m->partWidthC[pi][spi] = m->partWidth[pi][spi] >> 1;
            m->partHeightC[pi][spi] = m->partHeight[pi][spi] >> 1;
            m->mvd_l0[pi][spi].x = m->mvL0[pi][spi].x - bestMvp[pi][spi].x;
            m->mvd_l0[pi][spi].y = m->mvL0[pi][spi].y - bestMvp[pi][spi].y;
            m->MvL0[pi][spi] = m->mvL0[pi][spi];
        }
    }
    if (pskip) {
        reconstruct_luma_pskip(e, m, m->mvL0[0][0]);
        m->e_type = ET_PSKIP;
        m->flags |= FL_SKIP;
        m->mb_type = m->e_type - 301;
        m->cbp = 0;
        m->CbpC = 0;
        m->CbpL4x4 = 0;
        m->CbpL = 0;
    }
    else {
        reconstruct_inter(e, m, best_single);
        guess_cbp(m);
    }
    if (!(m->flags & FL_SKIP) && m->cbp == 0 && m->e_type == ET_P16x16 && m->mvd_l0[0][0].x == 0 && m->mvd_l0[0][0].y == 0) {
        mv_t smv = skip_mv(e, m);
        if (smv.x == bestMvp[0][0].x && smv.y == bestMvp[0][0].y) {
            m->e_type = ET_PSKIP;
            m->mb_type = m->e_type - 301;
        }
    }
}

/* ------------------------------------------------------------------------- */
/* Macroblock layer writer (mb.c:543-892, residual.c:903-1094)               */
/* ------------------------------------------------------------------------- */
static void write_mb(hlo_enc_t* e, mb_t* m, bw_t* bw)
{
    static const int32_t zeros[16] = {0};
    int pi, spi;
    if (!e->is_intra_slice) {
        if (m->e_type == ET_PSKIP) {
            ++e->skip_run;
            if (m->addr == e->nmb - 1) bw_ue(bw, (uint32_t)e->skip_run);
            return;
        }
        bw_ue(bw, (uint32_t)e->skip_run);
        e->skip_run = 0;
    }
    bw_ue(bw, (uint32_t)m->mb_type);
    if (m->e_type != ET_I_NXN && m->MbPartPredMode[0] != PM_I16 && m->NumMbPart == 4 && !is_intra(m)) {
        for (pi = 0; pi < 4; ++pi) bw_ue(bw, (uint32_t)m->sub_mb_type[pi]);
        for (pi = 0; pi < 4; ++pi)
            for (spi = 0; spi < m->NumSubMbPart[pi]; ++spi) {
                bw_se(bw, m->mvd_l0[pi][spi].x);
                bw_se(bw, m->mvd_l0[pi][spi].y);
            }
    }
    else if (m->MbPartPredMode[0] == PM_I4 || m->MbPartPredMode[0] == PM_I16) {
        if (m->MbPartPredMode[0] == PM_I4) {
            int blk;
            for (blk = 0; blk < 16; ++blk) {
                bw_u1(bw, (uint32_t)m->prev_flag[blk]);
                if (!m->prev_flag[blk]) bw_u(bw, (uint32_t)m->rem_mode[blk], 3);
            }
        }
        bw_ue(bw, (uint32_t)m->chroma_mode);
    }
    else {
        for (pi = 0; pi < m->NumMbPart; ++pi) {
            bw_se(bw, m->mvd_l0[pi][0].x);
            bw_se(bw, m->mvd_l0[pi][0].y);
        }
    }
    if (m->MbPartPredMode[0] != PM_I16) bw_ue(bw, CBP2CODE[m->cbp][m->MbPartPredMode[0] == PM_I4 ? 0 : 1]);
    if (m->CbpL > 0 || m->CbpC > 0 || m->MbPartPredMode[0] == PM_I16) {
        int i8, i4, c;
        bw_se(bw, 0); /* mb_qp_delta */
        if (m->MbPartPredMode[0] == PM_I16) wb_luma(e, m, bw, RES_I16_DC, 0, m->I16DC, 0, 15, 16, 0);
        for (i8 = 0; i8 < 4; ++i8)
            for (i4 = 0; i4 < 4; ++i4)
                if (m->CbpL & (1 << i8)) {
                    int blk = i8 * 4 + i4;
                    if (m->MbPartPredMode[0] == PM_I16) wb_luma(e, m, bw, RES_I16_AC, blk, m->I16AC[blk], 0, 14, 15, 0);
                    else wb_luma(e, m, bw, RES_LUMA, blk, m->LumaLevel[blk], 0, 15, 16, 0);
                }
        if (m->CbpC & 3) {
            for (c = 0; c < 2; ++c)
                cavlc_block(bw, m->CbpCDC[c] ? m->ChromaDCLevel[c] : zeros, 0, 3, 4, -1, 0, &e->rdo_single_ctr);
        }
        for (c = 0; c < 2; ++c)
            for (i4 = 0; i4 < 4; ++i4)
                if (m->CbpC & 2)
                    wb_chroma_ac(e, m, bw, c, i4, (m->CbpCAC[c] & (1 << i4)) ? m->ChromaACLevel[c][i4] : zeros, 0, 14, 15, 0);
    }
}

/* ------------------------------------------------------------------------- */
/* Deblocking (deblock.c:192-3553, baseline path)                            */
/* ------------------------------------------------------------------------- */
static int bs_luma(const mb_t* P, const mb_t* Q, int px, int py, int qx, int qy, int mb_edge) /* deblock.c:1784-1834 */
{
    int pb, qb, pPi, pSpi, qPi, qSpi, d;
    if (is_intra(Q) || is_intra(P)) return mb_edge ? 4 : 3;
    pb = luma_blk_idx(px, py);
    qb = luma_blk_idx(qx, qy);
    if ((P->CbpL4x4 & (1 << pb)) || (Q->CbpL4x4 & (1 << qb))) return 2;
    sub_part_indices(P, px, py, &pPi, &pSpi);
    sub_part_indices(Q, qx, qy, &qPi, &qSpi);
    if (P->predFlagL0[pPi] != Q->predFlagL0[qPi]) return 1; /* ref_idx_l0 is always 0 (never written) */
    if (P->predFlagL0[pPi] && Q->predFlagL0[qPi]) {
        d = P->mvL0[pPi][pSpi].x - Q->mvL0[qPi][qSpi].x;
        if (ABS(d) >= 4) return 1;
        d = P->mvL0[pPi][pSpi].y - Q->mvL0[qPi][qSpi].y;
        return ABS(d) >= 4 ? 1 : 0;
    }
    return 0;
}

/* Filters one line of samples across an edge; s points at q0, step to q1. */
static void filter_line(uint8_t* s, int step, int bS, int chroma, int indexA, int alpha, int beta)
{
    int p0 = s[-step], p1 = s[-2 * step], q0 = s[0], q1 = s[step];
    int p2 = chroma ? 0 : s[-3 * step], q2 = chroma ? 0 : s[2 * step];
    if (!(ABS(p0 - q0) < alpha && ABS(p1 - p0) < beta && ABS(q1 - q0) < beta)) return;
    if (bS < 4) {
        int tc0 = DEBLOCK_TC0[indexA][bS], tc, delta;
        int ap = ABS(p2 - p0), aq = ABS(q2 - q0);
        tc = chroma ? tc0 + 1 : tc0 + (ap < beta) + (aq < beta);
        delta = CLIP3(-tc, tc, ((((q0 - p0) << 2) + (p1 - q1) + 4) >> 3));
        s[-step] = (uint8_t)clip255(p0 + delta);
        s[0] = (uint8_t)clip255(q0 - delta);
        if (!chroma && ap < beta) s[-2 * step] = (uint8_t)(p1 + CLIP3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1));
        if (!chroma && aq < beta) s[step] = (uint8_t)(q1 + CLIP3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1));
    }
    else {
        int p3 = chroma ? 0 : s[-4 * step], q3 = chroma ? 0 : s[3 * step];
        int ap = ABS(p2 - p0), aq = ABS(q2 - q0);
        int strong = ABS(p0 - q0) < ((alpha >> 2) + 2);
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

static void deblock_edge(hlo_enc_t* e, const mb_t* P, const mb_t* Q, int vertical, int edge /* 0,4,8,12 in luma units */, int mb_edge)
{
    int bS[4], k, c, any = 0;
    for (k = 0; k < 4; ++k) {
        if (vertical) bS[k] = bs_luma(P, Q, mb_edge ? 12 : edge - 4, k * 4, edge, k * 4, mb_edge);
        else bS[k] = bs_luma(P, Q, k * 4, mb_edge ? 12 : edge - 4, k * 4, edge, mb_edge);
        any |= bS[k];
    }
    if (!any) return;
    { /* luma */
        int qPav = (P->QPy + Q->QPy + 1) >> 1;
        int indexA = CLIP3(0, 51, qPav), indexB = CLIP3(0, 51, qPav);
        int alpha = DEBLOCK_ALPHA[indexA], beta = DEBLOCK_BETA[indexB], i;
        for (i = 0; i < 16; ++i) {
            uint8_t* s;
            if (!bS[i >> 2]) continue;
            if (vertical) s = e->cur[0] + (Q->yL + i) * e->W + Q->xL + edge;
            else s = e->cur[0] + (Q->yL + edge) * e->W + Q->xL + i;
            filter_line(s, vertical ? 1 : e->W, bS[i >> 2], 0, indexA, alpha, beta);
        }
    }
    (void)c;
}

static void deblock_edge_chroma(hlo_enc_t* e, const mb_t* P, const mb_t* Q, int vertical, int edge /* 0 or 4 chroma */, int mb_edge)
{
    int bS[4], k, c, any = 0, ledge = edge * 2;
    for (k = 0; k < 4; ++k) {
        if (vertical) bS[k] = bs_luma(P, Q, mb_edge ? 12 : ledge - 4, k * 4, ledge, k * 4, mb_edge);
        else bS[k] = bs_luma(P, Q, k * 4, mb_edge ? 12 : ledge - 4, k * 4, ledge, mb_edge);
        any |= bS[k];
    }
    if (!any) return;
    for (c = 0; c < 2; ++c) {
        int qPav = (P->QPc[c] + Q->QPc[c] + 1) >> 1;
        int indexA = CLIP3(0, 51, qPav), indexB = CLIP3(0, 51, qPav);
        int alpha = DEBLOCK_ALPHA[indexA], beta = DEBLOCK_BETA[indexB], i;
        for (i = 0; i < 8; ++i) {
            uint8_t* s;
            if (!bS[i >> 1]) continue;
            if (vertical) s = e->cur[1 + c] + (Q->yC + i) * e->Wc + Q->xC + edge;
            else s = e->cur[1 + c] + (Q->yC + edge) * e->Wc + Q->xC + i;
            filter_line(s, vertical ? 1 : e->Wc, bS[i >> 1], 1, indexA, alpha, beta);
        }
    }
}

static void deblock_picture(hlo_enc_t* e) /* deblock.c:192-284, 573-651 */
{
    int a;
    for (a = 0; a < e->nmb; ++a) {
        mb_t* m = &e->mbs[a];
        const mb_t* L = m->mbx ? &e->mbs[a - 1] : NULL;
        const mb_t* T = m->mby ? &e->mbs[a - e->mbw] : NULL;
        int internal = !((m->e_type == ET_P16x16 || (m->flags & FL_SKIP)) && !m->CbpL);
        if (L) deblock_edge(e, L, m, 1, 0, 1);
        if (internal) {
            deblock_edge(e, m, m, 1, 4, 0);
            deblock_edge(e, m, m, 1, 8, 0);
            deblock_edge(e, m, m, 1, 12, 0);
        }
        if (T) deblock_edge(e, T, m, 0, 0, 1);
        if (internal) {
            deblock_edge(e, m, m, 0, 4, 0);
            deblock_edge(e, m, m, 0, 8, 0);
            deblock_edge(e, m, m, 0, 12, 0);
        }
        if (L) deblock_edge_chroma(e, L, m, 1, 0, 1);
        if (internal) deblock_edge_chroma(e, m, m, 1, 4, 0);
        if (T) deblock_edge_chroma(e, T, m, 0, 0, 1);
        if (internal) deblock_edge_chroma(e, m, m, 0, 4, 0);
    }
}

/* ------------------------------------------------------------------------- */
/* Stream syntax (sps.c:535-800, pps.c:265-400, slice.c:660-900, rbsp.c)     */
/* ------------------------------------------------------------------------- */
static int guess_level(int w, int h) /* utils.c:14-58 */
{
    static const int L[16][3] = {{10, 128, 96}, {9, 128, 96}, {11, 176, 144}, {12, 320, 240}, {13, 352, 288}, {20, 352, 288},
                                 {21, 352, 480}, {22, 352, 480}, {30, 720, 480}, {31, 1280, 720}, {32, 1280, 720}, {40, 2048, 1024},
                                 {41, 2048, 1024}, {42, 2048, 1080}, {50, 2560, 1920}, {51, 3840, 2160}};
    int i;
    for (i = 0; i < 16; ++i)
        if (L[i][1] >= w && L[i][2] >= h) return L[i][0];
    return 51;
}

/* max_num_ref_frames = min(MaxDpbMbs[level] / PicSizeInMbs, max_ref_frame),
 * sps.c:620-636; MaxDpbMbs is Table A-1 (tables.h:143) indexed as
 * HL_CODEC_264_LEVEL_TO_ZERO_BASED_INDEX (tables.h:151) maps level_idc */
static int max_num_ref_frames(const hlo_enc_t* e)
{
    static const int lv[16] = {10, 9, 11, 12, 13, 20, 21, 22, 30, 31, 32, 40, 41, 42, 50, 51};
    static const int dpb[16] = {396, 396, 900, 2376, 2376, 2376, 4752, 8100, 8100, 18000, 20480, 32768, 32768, 34816, 110400, 184320};
    const int level = guess_level(e->W, e->H);
    int i, n;
    for (i = 0; i < 15 && lv[i] != level; ++i) {
    }
    n = dpb[i] / (e->mbw * e->mbh);
    return n < e->max_ref_frame ? n : e->max_ref_frame;
}

static size_t write_headers(const hlo_enc_t* e, uint8_t* out)
{
    const int nref = max_num_ref_frames(e);
    uint8_t buf[256];
    bw_t bw;
    size_t n = 0;
    memset(buf, 0, sizeof(buf));
    bw_init(&bw, buf, sizeof(buf));
    /* SPS */
    bw_u(&bw, 0, 1);
    bw_u(&bw, 1, 2);
    bw_u(&bw, 7, 5);
    bw_u(&bw, 66, 8);
    bw_u1(&bw, 1);
    bw_u1(&bw, 1);
    bw_u1(&bw, 1);
    bw_u1(&bw, 0);
    bw_u1(&bw, 0);
    bw_u1(&bw, 0);
    bw_u(&bw, 0, 2);
    bw_u(&bw, (uint32_t)guess_level(e->W, e->H), 8);
    bw_ue(&bw, 0);
    bw_ue(&bw, 4); /* log2_max_frame_num_minus4 */
    bw_ue(&bw, 2); /* pic_order_cnt_type */
    bw_ue(&bw, (uint32_t)nref); /* max_num_ref_frames (sps.c:620-636) */
    bw_u1(&bw, 0);
    bw_ue(&bw, (uint32_t)(e->mbw - 1));
    bw_ue(&bw, (uint32_t)(e->mbh - 1));
    bw_u1(&bw, 1);
    bw_u1(&bw, 0);
    bw_u1(&bw, 0);
    bw_u1(&bw, 0);
    bw_trailing(&bw);
    out[n++] = 0;
    out[n++] = 0;
    out[n++] = 1;
    memcpy(out + n, buf, (size_t)(bw.nbits >> 3));
    n += (size_t)(bw.nbits >> 3);
    /* PPS */
    memset(buf, 0, sizeof(buf));
    bw_init(&bw, buf, sizeof(buf));
    bw_u(&bw, 0, 1);
    bw_u(&bw, 1, 2);
    bw_u(&bw, 8, 5);
    bw_ue(&bw, 0);
    bw_ue(&bw, 0);
    bw_u1(&bw, 0);
    bw_u1(&bw, 0);
    bw_ue(&bw, 0); /* num_slice_groups_minus1 */
    bw_ue(&bw, (uint32_t)(nref > 0 ? nref - 1 : 0)); /* num_ref_idx_l0_default_active_minus1, pps.c:291 */
    bw_ue(&bw, 0);
    bw_u1(&bw, 0);
    bw_u(&bw, 0, 2);
    bw_se(&bw, e->p.qp - 26);
    bw_se(&bw, 0);
    bw_se(&bw, 0);
    bw_u1(&bw, 1);
    bw_u1(&bw, 0);
    bw_u1(&bw, 0);
    bw_trailing(&bw);
    out[n++] = 0;
    out[n++] = 0;
    out[n++] = 1;
    memcpy(out + n, buf, (size_t)(bw.nbits >> 3));
    n += (size_t)(bw.nbits >> 3);
    return n;
}

static void write_slice_header(hlo_enc_t* e, bw_t* bw)
{
    int idr = e->is_intra_slice;
    bw_u(bw, 0, 1);
    bw_u(bw, 1, 2);
    bw_u(bw, idr ? 5 : 1, 5);
    bw_ue(bw, 0);                /* first_mb_in_slice */
    bw_ue(bw, idr ? 2 : 0);      /* slice_type */
    bw_ue(bw, 0);                /* pic_parameter_set_id */
    bw_u(bw, (uint32_t)e->pict_count & 0xFF, 8); /* frame_num, never reset (encode.c:251,527) */
    if (idr) bw_ue(bw, (uint32_t)e->idr_pic_id);
    if (!idr) {
        bw_u1(bw, 1);            /* num_ref_idx_active_override_flag */
        bw_ue(bw, 0);
        bw_u1(bw, 0);            /* ref_pic_list_modification_flag_l0 */
    }
    if (idr) {
        bw_u1(bw, 0);
        bw_u1(bw, 0);
    }
    else {
        bw_u1(bw, 0);
    }
    bw_se(bw, 0);                /* slice_qp_delta */
    bw_ue(bw, e->p.deblock ? 0 : 1);
    if (e->p.deblock) {
        bw_se(bw, 0);
        bw_se(bw, 0);
    }
}

/* rbsp.c:609-632: escapes only 00 00 01 and never updates the caller's
 * length (encode.c:443-444), so each escape drops the last byte.  size is
 * the slice buffer size (encode.c:192). */
static int escape_inplace(uint8_t* p, size_t n, size_t size)
{
    size_t i, zeros = 0;
    for (i = 0; i < n; ++i) {
        if (zeros == 2) {
            if (p[i] == 0x01) {
                if (n + 1 >= size) return -1; /* HL_ERROR_TOOSHORT (rbsp.c:617-620) */
                memmove(&p[i + 1], &p[i], n - i + 1);
                n++;
                p[i++] = 0x03;
            }
            zeros = 0;
        }
        zeros = p[i] ? 0 : zeros + 1;
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Public API                                                                */
/* ------------------------------------------------------------------------- */
hlo_enc_t* hlo_create(const hlo_params_t* p)
{
    hlo_enc_t* e;
    int c, m, i, j;
    if (!p || p->width <= 0 || p->height <= 0 || (p->width & 15) || (p->height & 15)) return NULL;
    init_level_table();
    e = (hlo_enc_t*)calloc(1, sizeof(*e));
    e->p = *p;
    e->max_ref_frame = 1;
    e->W = p->width;
    e->H = p->height;
    e->Wc = e->W / 2;
    e->Hc = e->H / 2;
    e->mbw = e->W / 16;
    e->mbh = e->H / 16;
    e->nmb = e->mbw * e->mbh;
    e->mbs = (mb_t*)calloc((size_t)e->nmb, sizeof(mb_t));
    for (c = 0; c < 3; ++c) {
        size_t sz = c ? (size_t)e->Wc * e->Hc : (size_t)e->W * e->H;
        e->cur[c] = (uint8_t*)calloc(sz, 1);
        e->ref[c] = (uint8_t*)calloc(sz, 1);
    }
    e->slice_cap = (size_t)e->W * e->H * 3 / 2 + 4096 + ((size_t)e->nmb << 8);
    e->slice_buf = (uint8_t*)malloc(e->slice_cap);
    for (m = 0; m < 6; ++m)
        for (i = 0; i < 4; ++i)
            for (j = 0; j < 4; ++j) {
                int v = ((i & 1) == 0 && (j & 1) == 0) ? SCALE_V[m][0] : (((i & 1) == 1 && (j & 1) == 1) ? SCALE_V[m][1] : SCALE_V[m][2]);
                e->level_scale[m][i][j] = 16 * v;
            }
    return e;
}

void hlo_destroy(hlo_enc_t* e)
{
    int c;
    if (!e) return;
    for (c = 0; c < 3; ++c) {
        free(e->cur[c]);
        free(e->ref[c]);
    }
    free(e->mbs);
    free(e->slice_buf);
    free(e);
}

int hlo_encode_frame(hlo_enc_t* e, const uint8_t* y, const uint8_t* u, const uint8_t* v, uint8_t* out, size_t out_cap, size_t* out_len)
{
    bw_t bw;
    size_t n = 0, slice_len;
    int a, c;
    if (!e || !y || !u || !v || !out) return -1;
    if (out_cap < 64 + e->slice_cap) return -2;
    e->src[0] = y;
    e->src[1] = u;
    e->src[2] = v;
    /* encoding type (hl_codec_264.c:704-718) */
    if (e->gop_left <= 0) {
        e->is_intra_slice = 1;
        e->gop_left = e->p.gop_size;
    }
    else {
        e->is_intra_slice = 0;
    }
    if (e->frame_index == 0) n += write_headers(e, out);
    e->qp = e->p.qp;
    /* slice.c:1766 as the reference's x86 build computes it: below QP 10 the
     * int shift count (QP - 12) / 3 is negative and SHL uses its low 5 bits
     * (QP 7-9: (int)(1u << 31) = INT_MIN, a negative lambda) */
    e->lambda_mode = LAMBDA_FACT * (double)(int32_t)(1u << (((e->qp - 12) / 3) & 31));
    e->skip_run = 0;
    memset(e->slice_buf, 0, e->slice_cap);
    bw_init(&bw, e->slice_buf, e->slice_cap);
    /* the slice NAL is built in a (mb_count << 8) + 4096 byte buffer
     * (encode.c:192); writes past its end are dropped (bits.h:236-246) */
    bw.limit = ((int64_t)e->nmb << 8) + 4096;
    write_slice_header(e, &bw);
    for (a = 0; a < e->nmb; ++a) {
        mb_t* m = &e->mbs[a];
        m->used = 1;
        init_mb(e, a);
        set_quant(e, m);
        if (e->is_intra_slice) guess_intra(e, m);
        else guess_inter(e, m);
        write_mb(e, m, &bw);
    }
    if (e->p.deblock) deblock_picture(e);
    bw_trailing(&bw);
    slice_len = (size_t)((bw.nbits + 7) >> 3);
    if (escape_inplace(e->slice_buf, slice_len, (size_t)bw.limit)) return -3;
    out[n++] = 0;
    out[n++] = 0;
    out[n++] = 1;
    memcpy(out + n, e->slice_buf, slice_len);
    n += slice_len;
    *out_len = n;
    /* DPB: the reconstructed picture becomes RefPicList0[0] */
    for (c = 0; c < 3; ++c) {
        uint8_t* t = e->ref[c];
        e->ref[c] = e->cur[c];
        e->cur[c] = t;
    }
    ++e->pict_count;
    if (e->is_intra_slice) ++e->idr_pic_id;
    --e->gop_left;
    ++e->frame_index;
    return 0;
}

const uint8_t* hlo_recon(const hlo_enc_t* e, int plane) { return (e && plane >= 0 && plane < 3) ? e->ref[plane] : NULL; }

int64_t hlo_rdo_overflows(const hlo_enc_t* e) { return e ? e->rdo_overflows : -1; }

void hlo_dump_mbs(const hlo_enc_t* e, int32_t* recs)
{
    int a, i, j, c;
    for (a = 0; a < e->nmb; ++a) {
        const mb_t* m = &e->mbs[a];
        int32_t* r = recs + (size_t)a * MBR_STRIDE;
        memset(r, 0, sizeof(int32_t) * MBR_STRIDE);
        r[MBR_FLAGS] = ((m->flags & FL_INTRA) ? 1 : 0) | ((m->flags & FL_INTER) ? 2 : 0) | ((m->flags & FL_SKIP) ? 4 : 0) |
                       (m->MbPartPredMode[0] == PM_I16 ? 8 : 0) | (m->MbPartPredMode[0] == PM_I4 ? 16 : 0);
        r[MBR_MB_TYPE] = m->mb_type;
        for (i = 0; i < 4; ++i) r[MBR_SUB_MB_TYPE + i] = m->sub_mb_type[i];
        r[MBR_NUM_MB_PART] = m->NumMbPart;
        for (i = 0; i < 4; ++i)
            for (j = 0; j < 4; ++j) {
                r[MBR_MVL0 + (i * 4 + j) * 2] = m->mvL0[i][j].x;
                r[MBR_MVL0 + (i * 4 + j) * 2 + 1] = m->mvL0[i][j].y;
                r[MBR_MVD + (i * 4 + j) * 2] = m->mvd_l0[i][j].x;
                r[MBR_MVD + (i * 4 + j) * 2 + 1] = m->mvd_l0[i][j].y;
                r[MBR_MVL0_CAP + (i * 4 + j) * 2] = m->MvL0[i][j].x;
                r[MBR_MVL0_CAP + (i * 4 + j) * 2 + 1] = m->MvL0[i][j].y;
            }
        r[MBR_CBP_L4x4] = m->CbpL4x4;
        r[MBR_CBP] = m->cbp;
        r[MBR_CBP_L] = m->CbpL;
        r[MBR_CBP_C] = m->CbpC;
        for (c = 0; c < 2; ++c) {
            r[MBR_CBP_CAC + c] = m->CbpCAC[c];
            r[MBR_CBP_CDC + c] = m->CbpCDC[c];
        }
        r[MBR_I16_MODE] = m->I16Mode;
        for (i = 0; i < 16; ++i) {
            r[MBR_I4_MODE + i] = m->I4Mode[i];
            r[MBR_PREV_FLAG + i] = m->prev_flag[i];
            r[MBR_REM_MODE + i] = m->rem_mode[i];
            r[MBR_TC_LUMA + i] = m->TCLuma[i];
            r[MBR_I16_DC + i] = m->I16DC[i];
            for (j = 0; j < 16; ++j) {
                r[MBR_LUMA_LEVEL + i * 16 + j] = m->LumaLevel[i][j];
                r[MBR_I16_AC + i * 16 + j] = m->I16AC[i][j];
            }
        }
        r[MBR_CHROMA_MODE] = m->chroma_mode;
        r[MBR_QPY] = m->QPy;
        for (c = 0; c < 2; ++c)
            for (i = 0; i < 4; ++i) {
                r[MBR_TC_CAC + c * 4 + i] = m->TCChromaAC[c][i];
                r[MBR_CHROMA_DC + c * 4 + i] = m->ChromaDCLevel[c][i];
                for (j = 0; j < 16; ++j) r[MBR_CHROMA_AC + (c * 4 + i) * 16 + j] = m->ChromaACLevel[c][i][j];
            }
        r[MBR_ETYPE] = m->e_type;
    }
}

/* hl_codec_t.max_ref_frame, before the first frame (only the SPS / PPS read it) */
int hlo_set_max_ref_frame(hlo_enc_t* e, int max_ref_frame)
{
    if (!e || max_ref_frame < 0 || e->frame_index) return -1; /* any value: the SPS carries min(MaxDpbMbs / PicSizeInMbs, it) (sps.c:635-636) */
    e->max_ref_frame = max_ref_frame;
    return 0;
}
