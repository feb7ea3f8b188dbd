/*
 * drop_in_harness.c -- TEST INFRASTRUCTURE.  Drives the reference's own
 * codec API (allweax/hartallo, oracle/_ref/libhl.a) with the gfx950 plugin
 * (integration/hl_codec_264_gfx950.c) installed in place of the stock H.264
 * plugin: hl_engine_init, hl_codec_264_gfx950_install (unregister +
 * register, hl_codec.c:161-212), hl_codec_plugin_find, hl_codec_create and
 * hl_codec_encode with the settings of source/test_encoder.c:135-146.  Every
 * frame is encoded by libhartallo_amd.so on the GPU; the output is written
 * as test_encoder.c:220-236 writes it.
 *
 * usage: drop_in_enc W H N qp me_range deblock gop early_term in.yuv out.264
 * decoding after install: drop_in_dec dec in.264 out.yuv
 *   hl_codec_decode through the installed plugin (it forwards to a stock
 *   codec it owns), driven like source/test_decoder.c:43-115 and
 *   oracle/ref_decode.c; then one hl_codec_encode on the same object, which
 *   the stock plugin refuses (hl_codec_264.c:447-452).  drop_in_dec is this
 *   file linked with the reference library whose bit reader works
 *   (oracle/Makefile, libhl_dec.a)
 *   early_term -1 keeps the hl_codec_create default (hl_types.h:67)
 * spatial SVC: drop_in_enc svc L W0 H0 N qp me_range deblock gop early_term out_prefix in0.yuv .. in{L-1}.yuv
 *   hl_codec_add_layer per layer (W0 << l, H0 << l), then per frame one
 *   hl_codec_encode per layer, base first (test_encoder.c:151-202); writes
 *   out_prefix.264 as oracle/ref_svc_harness.c does and out_prefix.idx (the
 *   stream's size after every access unit)
 */
#include <hartallo/hl_api.h>
#include <hartallo/hl_codec.h>
#include <hartallo/hl_cpu.h>
#include <hartallo/hl_debug.h>
#include <hartallo/hl_frame.h>
#include <hartallo/hl_object.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

extern const hl_codec_plugin_def_t hl_codec_264_gfx950_plugin_def_s;
HL_ERROR_T hl_codec_264_gfx950_install(void);
HL_ERROR_T hl_codec_264_gfx950_flush(hl_codec_t* codec, hl_codec_result_t* result);

static int run_svc(int argc, char** argv);
static int run_dec(int argc, char** argv);

int main(int argc, char** argv)
{
    if (argc > 1 && !strcmp(argv[1], "svc")) return run_svc(argc - 1, argv + 1);
    if (argc > 1 && !strcmp(argv[1], "dec")) return run_dec(argc - 1, argv + 1);
    if (argc < 11) {
        fprintf(stderr, "usage: %s W H N qp me_range deblock gop early_term in.yuv out.264\n", argv[0]);
        return 1;
    }
    int W = atoi(argv[1]), H = atoi(argv[2]), N = atoi(argv[3]), qp = atoi(argv[4]);
    int mer = atoi(argv[5]), db = atoi(argv[6]), gop = atoi(argv[7]), et = atoi(argv[8]);
    hl_debug_set_level(HL_DEBUG_LEVEL_ERROR);
    if (hl_engine_init()) return 2;
    if (hl_codec_264_gfx950_install()) return 3;
    const struct hl_codec_plugin_def_s* pl = 0;
    struct hl_codec_s* c = 0;
    struct hl_codec_result_s* r = 0;
    hl_frame_video_t* f = 0;
    if (hl_codec_plugin_find(HL_CODEC_TYPE_H264, &pl) || pl != &hl_codec_264_gfx950_plugin_def_s) {
        fprintf(stderr, "the gfx950 plugin is not the one hl_codec_plugin_find returns\n");
        return 4;
    }
    hl_codec_create(pl, &c);
    hl_codec_result_create(&r);
    hl_frame_video_create(&f);
    c->gop_size = gop; c->me_range = mer; c->qp = qp; c->fps.num = 1; c->fps.den = 15;
    c->rc_bitrate = -1; c->deblock_flag = db; c->threads_count = 1; c->max_ref_frame = 1;
    if (getenv("HL_REF_MAX_REF_FRAME")) c->max_ref_frame = atoi(getenv("HL_REF_MAX_REF_FRAME")); /* SPS/PPS only */
    c->distortion_mesure_type = HL_VIDEO_DISTORTION_MESURE_TYPE_SAD;
    if (et >= 0) c->me_early_term_flag = et;
    /* rate control set on the hl_codec_t as a hartallo caller would */
    if (getenv("HL_REF_RC_BITRATE")) c->rc_bitrate = atoi(getenv("HL_REF_RC_BITRATE"));
    if (getenv("HL_REF_RC_BASICUNIT")) c->rc_basicunit = atoi(getenv("HL_REF_RC_BASICUNIT"));
    if (getenv("HL_REF_RC_QP_MIN")) c->rc_qp_min = atoi(getenv("HL_REF_RC_QP_MIN"));
    if (getenv("HL_REF_RC_QP_MAX")) c->rc_qp_max = atoi(getenv("HL_REF_RC_QP_MAX"));
    size_t fs = (size_t)W * H * 3 / 2;
    uint8_t* buf = (uint8_t*)malloc(fs);
    FILE* fi = fopen(argv[9], "rb");
    FILE* fo = fopen(argv[10], "wb");
    if (!fi || !fo) return 5;
    static const uint8_t scp[3] = {0, 0, 1};
    int n = 0;
    double* ms = (double*)calloc(N > 0 ? N : 1, sizeof(double)); /* wall time of each hl_codec_encode call */
    while (n < N && fread(buf, 1, fs, fi) == fs) {
        hl_frame_video_fill(f, HL_VIDEO_CHROMA_YUV420, W, H, buf, fs);
        f->encoding = HL_VIDEO_ENCODING_TYPE_AUTO;
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        int e = hl_codec_encode(c, (hl_frame_t*)f, r);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        ms[n] = (t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_nsec - t0.tv_nsec) * 1e-6;
        if (e) {
            fprintf(stderr, "encode err %d at frame %d\n", e, n);
            return 6;
        }
        if (r->type & HL_CODEC_RESULT_TYPE_HDR) fwrite(c->hdr_bytes, 1, c->hdr_bytes_count, fo);
        if (r->type & HL_CODEC_RESULT_TYPE_DATA) {
            fwrite(scp, 1, 3, fo);
            fwrite(r->data_ptr, 1, r->data_size, fo);
        }
        ++n;
    }
    /* the plugin's look-ahead (HL_AMD_LOOKAHEAD): the frames it still holds */
    struct timespec tf0, tf1;
    clock_gettime(CLOCK_MONOTONIC, &tf0);
    for (;;) {
        int e = hl_codec_264_gfx950_flush(c, r);
        if (e) {
            fprintf(stderr, "flush err %d\n", e);
            return 6;
        }
        if (!(r->type & (HL_CODEC_RESULT_TYPE_HDR | HL_CODEC_RESULT_TYPE_DATA))) break;
        if (r->type & HL_CODEC_RESULT_TYPE_HDR) fwrite(c->hdr_bytes, 1, c->hdr_bytes_count, fo);
        if (r->type & HL_CODEC_RESULT_TYPE_DATA) {
            fwrite(scp, 1, 3, fo);
            fwrite(r->data_ptr, 1, r->data_size, fo);
        }
    }
    clock_gettime(CLOCK_MONOTONIC, &tf1);
    fclose(fo);
    fclose(fi);
    hl_object_unref(r);
    hl_object_unref(c);
    hl_object_unref(f);
    printf("{\"frames\": %d, \"encode_ms\": [", n);
    for (int i = 0; i < n; ++i) printf("%s%.3f", i ? ", " : "", ms[i]);
    printf("], \"flush_ms\": %.3f}\n", (tf1.tv_sec - tf0.tv_sec) * 1e3 + (tf1.tv_nsec - tf0.tv_nsec) * 1e-6);
    free(ms);
    return 0;
}

/* argv: svc L W0 H0 N qp me_range deblock gop early_term out_prefix in0.yuv .. */
static int run_svc(int argc, char** argv)
{
    if (argc < 11) {
        fprintf(stderr, "usage: drop_in_enc svc L W0 H0 N qp me_range deblock gop early_term out_prefix in0.yuv ..\n");
        return 1;
    }
    int L = atoi(argv[1]), W0 = atoi(argv[2]), H0 = atoi(argv[3]), N = atoi(argv[4]), qp = atoi(argv[5]);
    int mer = atoi(argv[6]), db = atoi(argv[7]), gop = atoi(argv[8]), et = atoi(argv[9]);
    const char* pre = argv[10];
    if (L < 2 || L > 4 || argc < 11 + L) return 1;
    hl_debug_set_level(HL_DEBUG_LEVEL_ERROR);
    if (hl_engine_init()) return 2;
    if (hl_codec_264_gfx950_install()) return 3;
    const struct hl_codec_plugin_def_s* pl = 0;
    struct hl_codec_s* c = 0;
    struct hl_codec_result_s* r = 0;
    hl_frame_video_t* f = 0;
    if (hl_codec_plugin_find(HL_CODEC_TYPE_H264_SVC, &pl) || pl != &hl_codec_264_gfx950_plugin_def_s) return 4;
    hl_codec_create(pl, &c);
    hl_codec_result_create(&r);
    hl_frame_video_create(&f);
    c->gop_size = gop; c->me_range = mer; c->qp = qp; c->fps.num = 1; c->fps.den = 15;
    c->rc_bitrate = -1; c->deblock_flag = db; c->threads_count = 1; c->max_ref_frame = 1;
    if (getenv("HL_REF_MAX_REF_FRAME")) c->max_ref_frame = atoi(getenv("HL_REF_MAX_REF_FRAME")); /* SPS/PPS only */
    c->distortion_mesure_type = HL_VIDEO_DISTORTION_MESURE_TYPE_SAD;
    if (et >= 0) c->me_early_term_flag = et;
    for (int l = 0; l < L; ++l)
        if (hl_codec_add_layer(c, (uint32_t)(W0 << l), (uint32_t)(H0 << l), 0, 0)) return 5;
    FILE* fi[4] = {0};
    uint8_t* buf[4] = {0};
    size_t fs[4];
    char path[4096];
    for (int l = 0; l < L; ++l) {
        fs[l] = (size_t)(W0 << l) * (H0 << l) * 3 / 2;
        buf[l] = (uint8_t*)malloc(fs[l]);
        if (!(fi[l] = fopen(argv[11 + l], "rb"))) return 5;
    }
    snprintf(path, sizeof(path), "%s.264", pre);
    FILE* fo = fopen(path, "wb");
    snprintf(path, sizeof(path), "%s.idx", pre);
    FILE* fidx = fopen(path, "wb");
    if (!fo || !fidx) return 5;
    static const uint8_t scp[3] = {0, 0, 1};
    int n = 0;
    for (; n < N; ++n) {
        int ok = 1;
        for (int l = 0; l < L; ++l) ok &= fread(buf[l], 1, fs[l], fi[l]) == fs[l];
        if (!ok) break;
        for (int l = 0; l < L; ++l) {
            hl_frame_video_fill(f, HL_VIDEO_CHROMA_YUV420, W0 << l, H0 << l, buf[l], fs[l]);
            f->encoding = HL_VIDEO_ENCODING_TYPE_AUTO;
            int e = hl_codec_encode(c, (hl_frame_t*)f, r);
            if (e) {
                fprintf(stderr, "encode err %d at frame %d layer %d\n", e, n, l);
                return 6;
            }
            if (r->type & HL_CODEC_RESULT_TYPE_HDR) fwrite(c->hdr_bytes, 1, c->hdr_bytes_count, fo);
            if (l == L - 1 && (r->type & HL_CODEC_RESULT_TYPE_DATA)) {
                fwrite(scp, 1, 3, fo);
                fwrite(r->data_ptr, 1, r->data_size, fo);
            }
        }
        fprintf(fidx, "%ld\n", ftell(fo));
    }
    fclose(fo);
    fclose(fidx);
    for (int l = 0; l < L; ++l) {
        fclose(fi[l]);
        free(buf[l]);
    }
    hl_object_unref(r);
    hl_object_unref(c);
    hl_object_unref(f);
    printf("{\"frames\": %d, \"layers\": %d}\n", n, L);
    return 0;
}

/* argv: dec in.264 out.yuv; prints {"frames", "width", "height", "errors",
 * "plugin_is_gfx950", "encode_after_decode"} */
static int run_dec(int argc, char** argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: drop_in_dec dec in.264 out.yuv\n");
        return 1;
    }
    FILE* fi = fopen(argv[1], "rb");
    FILE* fo = fopen(argv[2], "wb");
    if (!fi || !fo) return 1;
    fseek(fi, 0, SEEK_END);
    const long n = ftell(fi);
    fseek(fi, 0, SEEK_SET);
    uint8_t* buf = (uint8_t*)calloc((size_t)n + 16, 1); /* the parser reads one byte past the last NAL */
    if (!buf || fread(buf, 1, (size_t)n, fi) != (size_t)n) return 1;
    fclose(fi);
    hl_debug_set_level(HL_DEBUG_LEVEL_ERROR);
    hl_engine_set_cpu_flags(kCpuFlagAll); /* as oracle/ref_decode.c */
    if (hl_engine_init()) return 2;
    if (hl_codec_264_gfx950_install()) return 3;
    const struct hl_parser_plugin_def_s* ppl = 0;
    struct hl_parser_s* parser = 0;
    const struct hl_codec_plugin_def_s* cpl = 0;
    struct hl_codec_s* codec = 0;
    struct hl_codec_result_s* res = 0;
    if (hl_parser_plugin_find(HL_CODEC_TYPE_H264_SVC, &ppl) || hl_parser_create(ppl, &parser) || hl_codec_result_create(&res) ||
        hl_codec_plugin_find(HL_CODEC_TYPE_H264_SVC, &cpl) || hl_codec_create(cpl, &codec))
        return 4;
    codec->threads_count = 1;
    int frames = 0, errors = 0, w = 0, h = 0;
    hl_size_t start, end, count = (hl_size_t)n;
    const uint8_t* p = buf;
    while (count && hl_parser_find_bounds(parser, p, count, &start, &end) == HL_ERROR_SUCCESS) {
        res->type = HL_CODEC_RESULT_TYPE_NONE;
        if (hl_codec_decode(codec, &p[start], end - start + 1, res) != HL_ERROR_SUCCESS) ++errors;
        if (res->type & HL_CODEC_RESULT_TYPE_DATA) {
            fwrite(res->data_ptr, 1, res->data_size, fo);
            w = (int)res->width;
            h = (int)res->height;
            ++frames;
        }
        p += end;
        count -= end;
    }
    fclose(fo);
    /* the object has decoded: encoding on it is refused, as by the stock plugin */
    hl_frame_video_t* f = 0;
    hl_frame_video_create(&f);
    uint8_t* pic = (uint8_t*)calloc(16 * 16 * 3 / 2, 1);
    hl_frame_video_fill(f, HL_VIDEO_CHROMA_YUV420, 16, 16, pic, 16 * 16 * 3 / 2);
    const int enc_err = hl_codec_encode(codec, (hl_frame_t*)f, res);
    printf("{\"frames\": %d, \"width\": %d, \"height\": %d, \"errors\": %d, \"plugin_is_gfx950\": %d, "
           "\"encode_after_decode\": %d, \"invalid_operation\": %d}\n",
           frames, w, h, errors, cpl == &hl_codec_264_gfx950_plugin_def_s, enc_err, (int)HL_ERROR_INVALID_OPERATION);
    HL_OBJECT_SAFE_FREE(f);
    HL_OBJECT_SAFE_FREE(parser);
    HL_OBJECT_SAFE_FREE(codec);
    HL_OBJECT_SAFE_FREE(res);
    free(pic);
    free(buf);
    return 0;
}
