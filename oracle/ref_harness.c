/*
 * ref_harness.c -- TEST INFRASTRUCTURE.  Drives the *reference* encoder
 * (allweax/hartallo, compiled by oracle/Makefile into oracle/_ref/libhl.a)
 * through its public API exactly like source/test_encoder.c:135-146 does
 * (threads_count=1, SAD distortion, rc off, max_ref_frame=1) and dumps, per
 * frame:
 *   <prefix>.264      Annex-B stream (hdr bytes + 00 00 01 + slice bytes,
 *                     as test_encoder.c:220-236 writes it)
 *   <prefix>.rec.yuv  the reconstructed (deblocked) reference picture
 *   <prefix>.mbs      one mbrec.h record per macroblock
 * The dumps are read back through the reference's own structures
 * (hl_codec_264_t / hl_codec_264_layer_t / hl_codec_264_mb_t).
 *
 * and <prefix>.idx, the byte offset in <prefix>.264 where each frame's
 * output ends (one decimal number per line).
 *
 * usage: ref_enc W H N qp me_range deblock gop early_term in.yuv out_prefix [quiet|rec]
 * rate control (rc_bitrate > 0, hl_codec_264.c:719-742) from the environment:
 *   HL_REF_RC_BITRATE, HL_REF_RC_BASICUNIT, HL_REF_RC_QP_MIN, HL_REF_RC_QP_MAX
 *   quiet: no .rec.yuv / .mbs dumps (timing runs); rec: .rec.yuv but no .mbs
 */
#include <hartallo/hl_api.h>
#include <hartallo/hl_frame.h>
#include <hartallo/hl_codec.h>
#include <hartallo/hl_object.h>
#include <hartallo/hl_debug.h>
#include <hartallo/hl_cpu.h>
#include <hartallo/h264/hl_codec_264.h>
#include <hartallo/h264/hl_codec_264_layer.h>
#include <hartallo/h264/hl_codec_264_mb.h>
#include <hartallo/h264/hl_codec_264_dpb.h>
#include <hartallo/h264/hl_codec_264_pict.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "mbrec.h"
#include "ref_mbdump.h"

int main(int argc, char** argv)
{
    if (argc < 11) {
        fprintf(stderr, "usage: %s W H N qp me_range deblock gop early_term in.yuv out_prefix [quiet]\n", argv[0]);
        return 1;
    }
    int W = atoi(argv[1]), H = atoi(argv[2]), N = atoi(argv[3]), qp = atoi(argv[4]);
    int mer = atoi(argv[5]), db = atoi(argv[6]), gop = atoi(argv[7]), et = atoi(argv[8]);
    const char* in = argv[9];
    const char* pre = argv[10];
    int quiet = argc > 11 && strcmp(argv[11], "rec") != 0;
    int no_mbs = argc > 11;
    char path[1024];

    hl_debug_set_level(HL_DEBUG_LEVEL_ERROR);
    hl_engine_set_cpu_flags(kCpuFlagAll);
    if (hl_engine_init()) return 2;

    const struct hl_codec_plugin_def_s* pl = 0;
    struct hl_codec_s* c = 0;
    struct hl_codec_result_s* r = 0;
    hl_frame_video_t* f = 0;
    hl_codec_plugin_find(HL_CODEC_TYPE_H264, &pl);
    hl_codec_create(pl, &c);
    hl_codec_result_create(&r);
    hl_frame_video_create(&f);
    c->gop_size = gop; c->me_range = mer; c->qp = qp; c->fps.num = 1; c->fps.den = 15;
    c->rc_bitrate = -1; c->deblock_flag = db; c->threads_count = 1; c->max_ref_frame = 1;
    if (getenv("HL_REF_MAX_REF_FRAME")) c->max_ref_frame = atoi(getenv("HL_REF_MAX_REF_FRAME")); /* SPS/PPS only */
    c->distortion_mesure_type = HL_VIDEO_DISTORTION_MESURE_TYPE_SAD;
    c->me_type = (HL_VIDEO_ME_TYPE_INTEGER | HL_VIDEO_ME_TYPE_HALF | HL_VIDEO_ME_TYPE_QUATER);
    c->me_part_types = HL_VIDEO_ME_PART_TYPE_ALL;
    c->me_subpart_types = HL_VIDEO_ME_SUBPART_TYPE_ALL;
    c->me_early_term_flag = et;
    /* rate control (hl_codec_264.c:719-742): HL_REF_RC_BITRATE=<bits/s> turns it on */
    if (getenv("HL_REF_RC_BITRATE")) c->rc_bitrate = atoi(getenv("HL_REF_RC_BITRATE"));
    if (getenv("HL_REF_RC_BASICUNIT")) c->rc_basicunit = atoi(getenv("HL_REF_RC_BASICUNIT"));
    if (getenv("HL_REF_RC_QP_MIN")) c->rc_qp_min = atoi(getenv("HL_REF_RC_QP_MIN"));
    if (getenv("HL_REF_RC_QP_MAX")) c->rc_qp_max = atoi(getenv("HL_REF_RC_QP_MAX"));

    size_t fs = (size_t)W * H * 3 / 2;
    uint8_t* buf = (uint8_t*)malloc(fs);
    FILE* fi = fopen(in, "rb");
    if (!fi) { fprintf(stderr, "cannot open %s\n", in); return 3; }
    snprintf(path, sizeof(path), "%s.264", pre);
    FILE* fo = fopen(path, "wb");
    FILE* frec = 0;
    FILE* fmb = 0;
    if (!quiet) {
        snprintf(path, sizeof(path), "%s.rec.yuv", pre);
        frec = fopen(path, "wb");
    }
    if (!no_mbs) {
        snprintf(path, sizeof(path), "%s.mbs", pre);
        fmb = fopen(path, "wb");
    }
    snprintf(path, sizeof(path), "%s.idx", pre);
    FILE* fidx = fopen(path, "wb");
    static const uint8_t scp[3] = { 0, 0, 1 };
    int32_t rec[MBR_STRIDE];
    int n = 0;
    double tot = 0, tp = 0;  /* tp: time of the P pictures (every picture after the first) */
    while (n < N && fread(buf, 1, fs, fi) == fs) {
        struct timespec t0, t1;
        hl_frame_video_fill(f, HL_VIDEO_CHROMA_YUV420, W, H, buf, fs);
        f->encoding = HL_VIDEO_ENCODING_TYPE_AUTO;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        int e = hl_codec_encode(c, (hl_frame_t*)f, r);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        if (e) { fprintf(stderr, "encode err %d at frame %d\n", e, n); return 4; }
        const double dt = (t1.tv_sec - t0.tv_sec) + (t1.tv_nsec - t0.tv_nsec) * 1e-9;
        tot += dt;
        if (n > 0) tp += dt;
        if (r->type & HL_CODEC_RESULT_TYPE_HDR) fwrite(c->hdr_bytes, 1, c->hdr_bytes_count, fo);
        if (r->type & HL_CODEC_RESULT_TYPE_DATA) { fwrite(scp, 1, 3, fo); fwrite(r->data_ptr, 1, r->data_size, fo); }
        if (fidx) fprintf(fidx, "%ld\n", ftell(fo));
        if (!quiet) {
            hl_codec_264_t* p264 = (hl_codec_264_t*)c;
            hl_codec_264_layer_t* L = p264->layers.pc_active;
            const hl_codec_264_pict_t* pict = L->pc_fs_curr->p_pict;
            fwrite(pict->pc_data_y, 1, (size_t)W * H, frec);
            fwrite(pict->pc_data_u, 1, (size_t)W * H / 4, frec);
            fwrite(pict->pc_data_v, 1, (size_t)W * H / 4, frec);
            for (size_t a = 0; fmb && a < L->u_list_macroblocks_count; ++a) {
                dump_mb(L->pp_list_macroblocks[a], rec);
                fwrite(rec, sizeof(int32_t), MBR_STRIDE, fmb);
            }
        }
        n++;
    }
    fclose(fo);
    if (frec) fclose(frec);
    if (fmb) fclose(fmb);
    if (fidx) fclose(fidx);
    printf("{\"frames\": %d, \"seconds\": %.6f, \"fps\": %.4f, \"mb_per_s\": %.1f, \"p_seconds\": %.6f, \"p_fps\": %.4f}\n",
           n, tot, n / tot, (double)n * (W / 16) * (H / 16) / tot, tp, n > 1 ? (n - 1) / tp : 0.0);
    return 0;
}
