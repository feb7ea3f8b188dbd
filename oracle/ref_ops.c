/*
 * ref_ops.c -- TEST INFRASTRUCTURE.  Drives the reference's own per-block
 * kernels (oracle/_ref/libhl.a, the reference sources compiled by
 * oracle/Makefile) on vectors from a file, so that the gfx950 kernels can be
 * pinned op by op (tests/golden/make_op_golden.py -> tests/golden/ops_*.npz,
 * tests/test_gpu_ops.py).  Never linked into the product.
 *
 *   ref_ops <op> <in.bin> <out.bin>
 *
 * A small reference encoder is created first and codes one I and one P
 * picture (96x64, QP 28, hl_codec_encode as test_encoder.c does): that
 * initialises the reference's function tables (transf.c:42, quant.c:26,
 * deblock.c:3575, interpol.h) and gives a live codec, PPS (LevelScale4x4),
 * DPB interpolation index table and macroblock objects to call them with.
 *
 * ops (records little-endian, int32 unless noted):
 *   xform  in {u8 src[16], u8 pred[16], qp, intra}            (raster 4x4)
 *          out {q[16] raster levels, u8 rec[16]}
 *          hl_math_sub4x4 -> transf_frw_residual4x4 (transf.c:716-772)
 *          -> quant_frw4x4_scale_ac(qp, intra) (quant.c:116-139)
 *          -> quant_scale_residual4x4 (quant.c:68-112, the PPS's flat
 *          LevelScale4x4) -> transf_inverse_residual4x4 (transf.c:420-458)
 *          -> Clip1(pred + r), as rdo.c:2784-2830 and the reconstruction do.
 *   cavlc  in {kind, nC, level[16]}  kind 0 luma 4x4 (16 coefficients),
 *          1 Intra16x16 AC (15), 2 chroma DC (4, nC -1), 3 chroma AC (15),
 *          4 Intra16x16 AC as the RDO prices it: 15 levels and a zero written
 *          with startIdx 0, endIdx 15, maxNumCoef 16 (rdo.c:1676, 2601)
 *          out {nbits, u8 bits[96]}: residual_block_cavlc as
 *          hl_codec_264_residual_write_block_cavlc (residual.c:587-901)
 *          writes it, nC through the macroblock's own neighbour derivation
 *          (residual.c:640-760: block A is a block of the same macroblock
 *          whose TotalCoeff is nC, block B unavailable).
 *   lpred  in {W, H, u8 luma[W*H]} then records {mbx, mby, mvx, mvy}
 *          out u8 pred[256]: hl_codec_264_interpol_luma (pred_inter.c:
 *          339-885) of a 16x16 partition at MB (mbx, mby), quarter-pel
 *          motion (mvx, mvy), from the W x H picture (the codec's index table
 *          for that size: the encode above is made at W x H).
 *   dblk   in {u8 p[4][8], u8 q[4][8], bS, indexA, chroma}  (p[k] = pk
 *          of 8 lines across one edge)
 *          out {u8 p[3][8], u8 q[3][8]}: the baseline u8 edge filter as
 *          the macroblock filters compose it (deblock.c:2760-2810):
 *          indexA / alpha / beta (deblock.c:1836-1843, Table 8-16),
 *          get_threshold8samples (deblock.c:1847-1880),
 *          filter8samples0_bs_lt4 / _bs_eq4 (deblock.c:2245-2420, with
 *          tc0 from Table 8-17), the unfiltered samples bypassed.
 *
 * deblock.c is compiled into this file (it is not linked from libhl.a) so
 * that its static tables and static inline filter steps are reachable; no
 * reference source is copied or changed.
 */
#include <hartallo/hl_api.h>
#include <hartallo/hl_frame.h>
#include <hartallo/hl_codec.h>
#include <hartallo/hl_object.h>
#include <hartallo/hl_debug.h>
#include <hartallo/hl_memory.h>
#include <hartallo/h264/hl_codec_264.h>
#include <hartallo/h264/hl_codec_264_layer.h>
#include <hartallo/h264/hl_codec_264_mb.h>
#include <hartallo/h264/hl_codec_264_dpb.h>
#include <hartallo/h264/hl_codec_264_pict.h>
#include <hartallo/h264/hl_codec_264_bits.h>
#include <hartallo/h264/hl_codec_264_transf.h>
#include <hartallo/h264/hl_codec_264_quant.h>
#include <hartallo/h264/hl_codec_264_residual.h>
#include <hartallo/h264/hl_codec_264_nal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "h264/hl_codec_264_deblock.c"

HL_ERROR_T hl_codec_264_interpol_luma(hl_codec_264_t* p_codec, hl_codec_264_mb_t* p_mb, int32_t mbPartIdx, int32_t subMbPartIdx,
                                      const hl_codec_264_mv_xt* mvLX, const hl_pixel_t* cSL, void* predPartLXL16x16,
                                      int32_t predPartLXLSampleSize);

static struct hl_codec_s* open_codec(int W, int H)
{
    const struct hl_codec_plugin_def_s* pl = 0;
    struct hl_codec_s* c = 0;
    struct hl_codec_result_s* r = 0;
    hl_frame_video_t* f = 0;
    hl_debug_set_level(HL_DEBUG_LEVEL_ERROR);
    hl_engine_set_cpu_flags(kCpuFlagAll);
    if (hl_engine_init()) return 0;
    hl_codec_plugin_find(HL_CODEC_TYPE_H264, &pl);
    hl_codec_create(pl, &c);
    hl_codec_result_create(&r);
    hl_frame_video_create(&f);
    c->gop_size = 30; c->me_range = 8; c->qp = 28; c->fps.num = 1; c->fps.den = 15;
    c->rc_bitrate = -1; c->deblock_flag = 1; c->threads_count = 1; c->max_ref_frame = 1;
    c->distortion_mesure_type = HL_VIDEO_DISTORTION_MESURE_TYPE_SAD;
    c->me_type = (HL_VIDEO_ME_TYPE_INTEGER | HL_VIDEO_ME_TYPE_HALF | HL_VIDEO_ME_TYPE_QUATER);
    c->me_part_types = HL_VIDEO_ME_PART_TYPE_ALL;
    c->me_subpart_types = HL_VIDEO_ME_SUBPART_TYPE_ALL;
    size_t fs = (size_t)W * H * 3 / 2;
    uint8_t* buf = (uint8_t*)malloc(fs);
    for (int k = 0; k < 2; ++k) {
        for (size_t i = 0; i < fs; ++i) buf[i] = (uint8_t)((i * 7 + (i / W) * 3 + k * 5) & 255);
        hl_frame_video_fill(f, HL_VIDEO_CHROMA_YUV420, W, H, buf, fs);
        f->encoding = HL_VIDEO_ENCODING_TYPE_AUTO;
        if (hl_codec_encode(c, (hl_frame_t*)f, r)) return 0;
    }
    free(buf);
    return c;
}

static void* slurp(const char* path, size_t* n)
{
    FILE* fp = fopen(path, "rb");
    if (!fp) return 0;
    fseek(fp, 0, SEEK_END);
    *n = (size_t)ftell(fp);
    fseek(fp, 0, SEEK_SET);
    void* b = malloc(*n + 1);
    if (fread(b, 1, *n, fp) != *n) return 0;
    fclose(fp);
    return b;
}

struct XIn { uint8_t src[16], pred[16]; int32_t qp, intra; };
struct XOut { int32_t q[16]; uint8_t rec[16]; };

static int op_xform(hl_codec_264_t* p, const struct XIn* in, size_t n, struct XOut* out)
{
    hl_codec_264_mb_t* mb = p->layers.pc_active->pp_list_macroblocks[0];
    for (size_t i = 0; i < n; ++i) {
        HL_ALIGN(16) int32_t res[4][4], w[4][4], c[4][4], d[4][4], r[4][4];
        for (int k = 0; k < 16; ++k) res[k >> 2][k & 3] = (int32_t)in[i].src[k] - (int32_t)in[i].pred[k];
        hl_codec_264_transf_frw_residual4x4(res, w);
        hl_codec_264_quant_frw4x4_scale_ac(in[i].qp, in[i].intra ? HL_TRUE : HL_FALSE, w, c);
        /* the dequantiser reads the PPS's LevelScale4x4[inter][Y]: the MB type picks the (flat) list */
        mb->e_type = in[i].intra ? HL_CODEC_264_MB_TYPE_I_NXN : HL_CODEC_264_MB_TYPE_P_L0_16X16;
        mb->flags_type = in[i].intra ? HL_CODEC_264_MB_TYPE_FLAGS_INTRA : HL_CODEC_264_MB_TYPE_FLAGS_INTER;
        hl_codec_264_quant_scale_residual4x4(p, mb, 8, in[i].qp, (const int32_t (*)[4])c, HL_TRUE, HL_FALSE, 0, d);
        hl_codec_264_transf_inverse_residual4x4(8, d, r);
        for (int k = 0; k < 16; ++k) {
            int v = (int)in[i].pred[k] + r[k >> 2][k & 3];
            out[i].q[k] = c[k >> 2][k & 3];
            out[i].rec[k] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
        }
    }
    return 0;
}

struct CIn { int32_t kind, nC, level[16]; };
struct COut { int32_t nbits; uint8_t bits[96]; };

static int op_cavlc(hl_codec_264_t* p, const struct CIn* in, size_t n, struct COut* out)
{
    hl_codec_264_layer_t* L = p->layers.pc_active;
    hl_codec_264_mb_t* mb = L->pp_list_macroblocks[0];
    static uint8_t buf[4096];
    hl_codec_264_bits_t* bits = 0;
    if (hl_codec_264_bits_create(&bits, buf, sizeof(buf))) return 5;
    /* a non-skip, non-PCM macroblock with every coded-block-pattern bit set,
     * so that the neighbour's TotalCoeff is what nA reads (utils.h:10-20) */
    mb->e_type = HL_CODEC_264_MB_TYPE_P_L0_16X16;
    mb->flags_type = HL_CODEC_264_MB_TYPE_FLAGS_INTER;
    mb->CodedBlockPatternLuma = 15;
    mb->CodedBlockPatternChroma = 2;
    for (size_t i = 0; i < n; ++i) {
        hl_codec_264_residual_inv_xt inv;
        memset(&inv, 0, sizeof(inv));
        int32_t lv[16];
        memcpy(lv, in[i].level, sizeof(lv));
        int start = 0, end = 15, maxn = 16;
        switch (in[i].kind) {
        case 0: inv.e_type = HL_CODEC_264_RESISUAL_INV_TYPE_LUMA_LEVEL; break;
        case 1: inv.e_type = HL_CODEC_264_RESISUAL_INV_TYPE_INTRA16X16_ACLEVEL; end = 14; maxn = 15; break;
        case 2: inv.e_type = HL_CODEC_264_RESISUAL_INV_TYPE_CHROMA_DCLEVEL; end = 3; maxn = 4; break;
        case 3: inv.e_type = HL_CODEC_264_RESISUAL_INV_TYPE_CHROMA_ACLEVEL; end = 14; maxn = 15; break;
        default: inv.e_type = HL_CODEC_264_RESISUAL_INV_TYPE_INTRA16X16_ACLEVEL; break; /* (0, 15, 16): the RDO's call, rdo.c:1676 */
        }
        if (in[i].kind == 3) {
            inv.i_cbr4x4BlkIdx = 0;
            mb->neighbouringChromaBlock4x4[0].i_addr_A = (int32_t)mb->u_addr;
            mb->neighbouringChromaBlock4x4[0].i_blk_idx_A = 3;
            mb->neighbouringChromaBlock4x4[0].i_addr_B = -1;
            mb->neighbouringChromaBlock4x4[0].i_blk_idx_B = -1;
            mb->TotalCoeffsChromaACCbCr[0][3] = in[i].nC;
        }
        else if (in[i].kind != 2) {
            inv.i_luma4x4BlkIdx = 0;
            mb->neighbouringLumaBlock4x4[0].i_addr_A = (int32_t)mb->u_addr;
            mb->neighbouringLumaBlock4x4[0].i_blk_idx_A = 15;
            mb->neighbouringLumaBlock4x4[0].i_addr_B = -1;
            mb->neighbouringLumaBlock4x4[0].i_blk_idx_B = -1;
            mb->TotalCoeffsLuma[15] = in[i].nC;
        }
        memset(buf, 0, sizeof(buf));
        hl_codec_264_bits_reset(bits, buf, sizeof(buf));
        if (hl_codec_264_residual_write_block_cavlc(&inv, p, mb, bits, lv, start, end, maxn)) return 6;
        out[i].nbits = (int32_t)hl_codec_264_bits_get_stream_index(bits);
        if (out[i].nbits > 96 * 8) return 7;
        memcpy(out[i].bits, buf, 96);
    }
    hl_object_unref(bits);
    return 0;
}

struct PIn { int32_t mbx, mby, mvx, mvy; };

static int op_lpred(hl_codec_264_t* p, int W, int H, const uint8_t* luma, const struct PIn* in, size_t n, uint8_t* out)
{
    hl_codec_264_mb_t* mb = p->layers.pc_active->pp_list_macroblocks[0];
    HL_ALIGN(16) uint8_t pred[16][16];
    mb->partWidth[0][0] = 16;
    mb->partHeight[0][0] = 16;
    for (size_t i = 0; i < n; ++i) {
        hl_codec_264_mv_xt mv;
        mv.x = (int16_t)in[i].mvx;
        mv.y = (int16_t)in[i].mvy;
        mb->xL_Idx = 16 * in[i].mbx;
        mb->yL_Idx = 16 * in[i].mby;
        if (in[i].mbx < 0 || in[i].mby < 0 || 16 * in[i].mbx >= W || 16 * in[i].mby >= H) return 8;
        if (hl_codec_264_interpol_luma(p, mb, 0, 0, &mv, luma, pred, sizeof(uint8_t))) return 9;
        memcpy(out + 256 * i, pred, 256);
    }
    return 0;
}

struct DIn { uint8_t p[4][8], q[4][8]; int32_t bS, indexA, chroma; };
struct DOut { uint8_t p[3][8], q[3][8]; };

static int op_dblk(const struct DIn* in, size_t n, struct DOut* out)
{
    for (size_t i = 0; i < n; ++i) {
        struct DIn x = in[i];
        int16_t indexA, alpha, beta, bS[4], flags[8];
        const int16_t qp = (int16_t)x.indexA;
        hl_codec_264_deblock_avc_baseline_get_indexA_alpha_and_beta_u8(qp, qp, 0, 0, &indexA, &alpha, &beta);
        for (int k = 0; k < 4; ++k) bS[k] = (int16_t)x.bS;
        if (x.chroma)
            hl_codec_264_deblock_avc_baseline_get_threshold8samples_chroma_u8(x.p[0], x.q[0], x.p[1], x.q[1], bS, alpha, beta, flags);
        else
            hl_codec_264_deblock_avc_baseline_get_threshold8samples_luma_u8(x.p[0], x.q[0], x.p[1], x.q[1], bS, alpha, beta, flags);
        HL_ALIGN(16) uint8_t pf[3][8], qf[3][8];
        if (x.bS < 4)
            hl_codec_264_deblock_avc_baseline_filter8samples0_bs_lt4_u8(x.p[0], x.p[1], x.p[2], x.q[0], x.q[1], x.q[2], x.chroma ? 1 : 0, bS,
                                                                         indexA, beta, flags, pf[0], pf[1], pf[2], qf[0], qf[1], qf[2]);
        else
            hl_codec_264_deblock_avc_baseline_filter8samples0_bs_eq4_u8(x.p[0], x.p[1], x.p[2], x.p[3], x.q[0], x.q[1], x.q[2], x.q[3],
                                                                         x.chroma ? 1 : 0, indexA, alpha, beta, flags, pf[0], pf[1], pf[2],
                                                                         qf[0], qf[1], qf[2]);
        memcpy(out[i].p, pf, sizeof(pf));
        memcpy(out[i].q, qf, sizeof(qf));
    }
    return 0;
}

int main(int argc, char** argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: %s xform|cavlc|lpred|dblk in.bin out.bin\n", argv[0]);
        return 1;
    }
    size_t nb = 0;
    uint8_t* in = (uint8_t*)slurp(argv[2], &nb);
    if (!in) return 2;
    int W = 96, H = 64;
    const uint8_t* recs = in;
    if (!strcmp(argv[1], "lpred")) {
        W = ((int32_t*)in)[0];
        H = ((int32_t*)in)[1];
        recs = in + 8 + (size_t)W * H;
        nb -= 8 + (size_t)W * H;
    }
    hl_codec_264_t* p = (hl_codec_264_t*)open_codec(W, H);
    if (!p) return 3;
    void* out = 0;
    size_t osz = 0, n = 0;
    int rc = 4;
    if (!strcmp(argv[1], "xform")) {
        n = nb / sizeof(struct XIn);
        out = calloc(n + 1, osz = sizeof(struct XOut));
        rc = op_xform(p, (const struct XIn*)recs, n, (struct XOut*)out);
    }
    else if (!strcmp(argv[1], "cavlc")) {
        n = nb / sizeof(struct CIn);
        out = calloc(n + 1, osz = sizeof(struct COut));
        rc = op_cavlc(p, (const struct CIn*)recs, n, (struct COut*)out);
    }
    else if (!strcmp(argv[1], "lpred")) {
        n = nb / sizeof(struct PIn);
        out = calloc(n + 1, osz = 256);
        rc = op_lpred(p, W, H, in + 8, (const struct PIn*)recs, n, (uint8_t*)out);
    }
    else if (!strcmp(argv[1], "dblk")) {
        n = nb / sizeof(struct DIn);
        out = calloc(n + 1, osz = sizeof(struct DOut));
        rc = op_dblk((const struct DIn*)recs, n, (struct DOut*)out);
    }
    if (rc) {
        fprintf(stderr, "%s failed: %d\n", argv[1], rc);
        return rc;
    }
    FILE* fo = fopen(argv[3], "wb");
    if (!fo || fwrite(out, osz, n, fo) != n) return 10;
    fclose(fo);
    return 0;
}
