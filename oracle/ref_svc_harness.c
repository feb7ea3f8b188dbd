/*
 * ref_svc_harness.c -- TEST INFRASTRUCTURE.  Drives the *reference* encoder
 * (oracle/_ref/libhl.a) as a spatial-SVC encoder the way
 * source/test_encoder.c:151-202 does with HL_TEST_ENCODER_SVC_ENABLED: one
 * hl_codec_add_layer per layer (increasing, dyadic sizes), then per frame one
 * hl_codec_encode per layer, base first.  Settings as ref_harness.c
 * (test_encoder.c:135-146 with threads_count=1, max_ref_frame=1).
 *
 * usage: ref_svc L W0 H0 N qp me_range deblock gop early_term out_prefix in0.yuv .. in{L-1}.yuv
 *   layer l is (W0<<l) x (H0<<l); in<l>.yuv holds N frames of that size.
 * writes
 *   <prefix>.264          Annex-B stream (hdr bytes once, then per access unit
 *                         00 00 01 + the result bytes of the last layer's call)
 *   <prefix>.idx          byte offset in .264 where each access unit ends
 *   <prefix>.L<l>.rec.yuv the layer's reconstructed picture after each frame
 *   <prefix>.L<l>.mbs     the layer's mbrec.h macroblock records (unless quiet)
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
#include "ref_mbdump.h"

int main(int argc, char** argv)
{
    if (argc < 12) {
        fprintf(stderr, "usage: %s L W0 H0 N qp me_range deblock gop early_term out_prefix in0.yuv .. [quiet]\n", argv[0]);
        return 1;
    }
    int L = atoi(argv[1]), W0 = atoi(argv[2]), H0 = atoi(argv[3]), N = atoi(argv[4]);
    int qp = atoi(argv[5]), mer = atoi(argv[6]), db = atoi(argv[7]), gop = atoi(argv[8]), et = atoi(argv[9]);
    const char* pre = argv[10];
    if (L < 1 || L > 4 || argc < 11 + L) { fprintf(stderr, "bad layer count\n"); return 1; }
    int quiet = argc > 11 + L;
    char path[1024];

    hl_debug_set_level(HL_DEBUG_LEVEL_ERROR);
    hl_engine_set_cpu_flags(kCpuFlagAll);
    if (hl_engine_init()) return 2;

    const struct hl_codec_plugin_def_s* pl = 0;
    struct hl_codec_s* c = 0;
    struct hl_codec_result_s* r = 0;
    hl_frame_video_t* f = 0;
    hl_codec_plugin_find(HL_CODEC_TYPE_H264_SVC, &pl);
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
    for (int l = 0; l < L; ++l) {
        int e = hl_codec_add_layer(c, (uint32_t)(W0 << l), (uint32_t)(H0 << l), 0, 0);
        if (e) { fprintf(stderr, "add_layer %d err %d\n", l, e); return 5; }
    }

    FILE* fi[4] = {0};
    FILE* frec[4] = {0};
    FILE* fmb[4] = {0};
    uint8_t* buf[4] = {0};
    size_t fs[4];
    for (int l = 0; l < L; ++l) {
        fs[l] = (size_t)(W0 << l) * (H0 << l) * 3 / 2;
        buf[l] = (uint8_t*)malloc(fs[l]);
        fi[l] = fopen(argv[11 + l], "rb");
        if (!fi[l]) { fprintf(stderr, "cannot open %s\n", argv[11 + l]); return 3; }
        snprintf(path, sizeof(path), "%s.L%d.rec.yuv", pre, l);
        frec[l] = fopen(path, "wb");
        if (!quiet) {
            snprintf(path, sizeof(path), "%s.L%d.mbs", pre, l);
            fmb[l] = fopen(path, "wb");
        }
    }
    snprintf(path, sizeof(path), "%s.264", pre);
    FILE* fo = fopen(path, "wb");
    snprintf(path, sizeof(path), "%s.idx", pre);
    FILE* fidx = fopen(path, "wb");
    static const uint8_t scp[3] = { 0, 0, 1 };
    int32_t rec[MBR_STRIDE];
    int n = 0;
    double tot = 0, tot_p = 0;  /* all access units; those after the first */
    for (; n < N; ++n) {
        int ok = 1;
        for (int l = 0; l < L; ++l) ok &= fread(buf[l], 1, fs[l], fi[l]) == fs[l];
        if (!ok) break;
        for (int l = 0; l < L; ++l) {
            struct timespec t0, t1;
            const int W = W0 << l, H = H0 << l;
            hl_frame_video_fill(f, HL_VIDEO_CHROMA_YUV420, W, H, buf[l], fs[l]);
            f->encoding = HL_VIDEO_ENCODING_TYPE_AUTO;
            clock_gettime(CLOCK_MONOTONIC, &t0);
            int e = hl_codec_encode(c, (hl_frame_t*)f, r);
            clock_gettime(CLOCK_MONOTONIC, &t1);
            if (e) { fprintf(stderr, "encode err %d at frame %d layer %d\n", e, n, l); return 4; }
            tot += (t1.tv_sec - t0.tv_sec) + (t1.tv_nsec - t0.tv_nsec) * 1e-9;
            if (n > 0) tot_p += (t1.tv_sec - t0.tv_sec) + (t1.tv_nsec - t0.tv_nsec) * 1e-9;
            if (r->type & HL_CODEC_RESULT_TYPE_HDR) fwrite(c->hdr_bytes, 1, c->hdr_bytes_count, fo);
            if (l == L - 1 && (r->type & HL_CODEC_RESULT_TYPE_DATA)) {
                fwrite(scp, 1, 3, fo);
                fwrite(r->data_ptr, 1, r->data_size, fo);
            }
            hl_codec_264_t* p264 = (hl_codec_264_t*)c;
            hl_codec_264_layer_t* Ly = p264->layers.pc_active;
            const hl_codec_264_pict_t* pict = Ly->pc_fs_curr->p_pict;
            fwrite(pict->pc_data_y, 1, (size_t)W * H, frec[l]);
            fwrite(pict->pc_data_u, 1, (size_t)W * H / 4, frec[l]);
            fwrite(pict->pc_data_v, 1, (size_t)W * H / 4, frec[l]);
            for (size_t a = 0; fmb[l] && a < Ly->u_list_macroblocks_count; ++a) {
                dump_mb(Ly->pp_list_macroblocks[a], rec);
                fwrite(rec, sizeof(int32_t), MBR_STRIDE, fmb[l]);
            }
        }
        fprintf(fidx, "%ld\n", ftell(fo));
    }
    fclose(fo);
    fclose(fidx);
    for (int l = 0; l < L; ++l) {
        fclose(fi[l]);
        fclose(frec[l]);
        if (fmb[l]) fclose(fmb[l]);
    }
    printf("{\"frames\": %d, \"layers\": %d, \"seconds\": %.6f, \"fps\": %.4f, \"p_seconds\": %.6f}\n", n, L, tot, n / tot, tot_p);
    return 0;
}
