/*
 * ref_decode.c -- TEST INFRASTRUCTURE.  The reference's own H.264 decoder
 * (allweax/hartallo, compiled from its sources by oracle/Makefile into
 * oracle/_ref/libhl_dec.a) as a conformance gate for the streams this
 * repository's encoder produces.  Driven like
 * source/test_decoder.c:43-115: the H.264 parser plugin splits the Annex-B
 * stream into NAL units (hl_parser_find_bounds), each goes to
 * hl_codec_decode, and every decoded picture (result type DATA: planar
 * Y|U|V, hl_codec_264.c:378-386) is appended to out.yuv.
 *
 * usage: ref_dec in.264 out.yuv
 * prints one JSON line {"frames": n, "width": w, "height": h, "errors": e}
 */
#include <hartallo/hl_api.h>
#include <hartallo/hl_codec.h>
#include <hartallo/hl_object.h>
#include <hartallo/hl_debug.h>
#include <hartallo/hl_cpu.h>
#include <stdio.h>
#include <stdlib.h>

int main(int argc, char** argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s in.264 out.yuv\n", argv[0]);
        return 1;
    }
    FILE* fi = fopen(argv[1], "rb");
    FILE* fo = fopen(argv[2], "wb");
    if (!fi || !fo) return 1;
    fseek(fi, 0, SEEK_END);
    const long n = ftell(fi);
    fseek(fi, 0, SEEK_SET);
    /* the parser reads one byte past the last NAL (hl_parser_264.c:42-43) */
    uint8_t* buf = (uint8_t*)calloc((size_t)n + 16, 1);
    if (!buf || fread(buf, 1, (size_t)n, fi) != (size_t)n) return 1;
    fclose(fi);

    hl_debug_set_level(HL_DEBUG_LEVEL_ERROR);
    hl_engine_set_cpu_flags(kCpuFlagAll);
    if (hl_engine_init()) return 2;
    const struct hl_parser_plugin_def_s* ppl = 0;
    struct hl_parser_s* parser = 0;
    const struct hl_codec_plugin_def_s* cpl = 0;
    struct hl_codec_s* codec = 0;
    struct hl_codec_result_s* res = 0;
    if (hl_parser_plugin_find(HL_CODEC_TYPE_H264_SVC, &ppl) || hl_parser_create(ppl, &parser) || hl_codec_result_create(&res) ||
        hl_codec_plugin_find(HL_CODEC_TYPE_H264_SVC, &cpl) || hl_codec_create(cpl, &codec))
        return 3;
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
    printf("{\"frames\": %d, \"width\": %d, \"height\": %d, \"errors\": %d}\n", frames, w, h, errors);
    HL_OBJECT_SAFE_FREE(parser);
    HL_OBJECT_SAFE_FREE(codec);
    HL_OBJECT_SAFE_FREE(res);
    free(buf);
    return 0;
}
