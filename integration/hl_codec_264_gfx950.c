/*
 * hl_codec_264_gfx950.c -- the hartallo-side plugin that drops the MI355X
 * (gfx950) encode path in behind hartallo's codec API.  This is the file a
 * maintainer adds to hartallo (source/h264/); it is compiled here against
 * the reference's own headers and linked with the reference's own library
 * by oracle/Makefile (oracle/_ref/drop_in_enc, tests/test_drop_in.py), so
 * the drop-in is exercised through hl_codec_encode exactly as
 * source/test_encoder.c:135-146 calls it.
 *
 * The plugin ABI is hl_codec_plugin_def_t (include/hartallo/hl_codec.h:
 * 173-184); its encode slot is called by hl_codec_encode (source/hl_codec.c:
 * 152-159), which refuses a plugin whose decode slot is NULL (:154).  The
 * codec object must start with hl_codec_t (HL_DECLARE_CODEC, hl_codec.h:171)
 * because the API reads and writes its fields directly.
 */
#include <hartallo/hl_codec.h>
#include <hartallo/hl_frame.h>
#include <hartallo/hl_object.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include "hartallo_amd.h" /* include/hartallo_amd.h of the gfx950 library */

extern const hl_codec_plugin_def_t* hl_codec_264_plugin_def_t; /* the stock plugin (hl_codec_264.c:1186) */

/* what a codec object has been used for: the stock plugin refuses to switch
 * between encoding and decoding (hl_codec_264.c:100-109, 447-457) */
enum { GFX950_UNUSED = 0, GFX950_ENCODING, GFX950_DECODING };

typedef struct hl_codec_264_gfx950_s {
    HL_DECLARE_CODEC; /* first member (hl_codec.h:171) */
    hl_amd_encoder_t* enc;
    hl_size_t width, height; /* the encoder's (base layer's) size */
    hl_size_t layers;        /* spatial layers the encoder was opened with (0: AVC) */
    int input_type;          /* GFX950_* */
    hl_codec_t* dec;         /* stock H.264 codec that decodes for this object (created on the first decode) */
} hl_codec_264_gfx950_t;

static hl_object_t* gfx950_ctor(hl_object_t* self, va_list* app)
{
    (void)app;
    return self;
}

static hl_object_t* gfx950_dtor(hl_object_t* self)
{
    hl_codec_264_gfx950_t* p = (hl_codec_264_gfx950_t*)self;
    if (p && p->enc) {
        hl_amd_encoder_destroy(p->enc);
        p->enc = NULL;
    }
    if (p) HL_OBJECT_SAFE_FREE(p->dec);
    return self;
}

static int gfx950_cmp(const hl_object_t* a, const hl_object_t* b) { return (int)((const char*)a - (const char*)b); }

static const hl_object_def_t gfx950_def_s = {sizeof(hl_codec_264_gfx950_t), gfx950_ctor, gfx950_dtor, gfx950_cmp, HL_TRUE};

/* (re)opens the gfx950 encoder at W x H with the hl_codec_t settings */
static HL_ERROR_T gfx950_open(hl_codec_264_gfx950_t* self, hl_codec_t* base, hl_size_t W, hl_size_t H)
{
    hl_amd_params_t p;
    int32_t err;
    if (self->enc) {
        hl_amd_encoder_destroy(self->enc);
        self->enc = NULL;
    }
    self->layers = 0;
    p.width = (int32_t)W;
    p.height = (int32_t)H;
    p.qp = base->qp;
    p.me_range = base->me_range;
    p.deblock = base->deblock_flag;
    p.gop_size = base->gop_size;
    p.me_early_term = base->me_early_term_flag;
    /* the HIP device: HL_AMD_DEVICE, read at every open (a process that
     * drives several GPUs through this API sets it before hl_codec_encode
     * opens the codec's encoder), else 0 (one process per GPU) */
    {
        const char* dv = getenv("HL_AMD_DEVICE");
        p.device = dv ? atoi(dv) : 0;
    }
    if ((err = hl_amd_encoder_create(&p, &self->enc))) return (HL_ERROR_T)err; /* HL_ERROR_T values (hl_types.h:101-122) */
    /* look-ahead (opt-in, no reference counterpart): HL_AMD_LOOKAHEAD=k codes
     * every k frames as one pipelined run; each hl_codec_encode then returns
     * the result of the frame k - 1 calls earlier (NONE while the first ones
     * queue) and the caller drains the rest with hl_codec_264_gfx950_flush.
     * AVC only: an SVC encoder (layers added after the open) ignores it. */
    {
        const char* la = getenv("HL_AMD_LOOKAHEAD");
        if (la && atoi(la) > 1 && (err = hl_amd_set_lookahead(self->enc, atoi(la)))) return (HL_ERROR_T)err;
    }
    /* SPS max_num_ref_frames / PPS num_ref_idx_l0_default_active_minus1
     * (hl_codec_264_sps.c:620-636, hl_codec_264_pps.c:291) */
    if ((err = hl_amd_set_max_ref_frame(self->enc, base->max_ref_frame))) return (HL_ERROR_T)err;

    /* rate control: the hl_codec_t fields hl_codec_264.c:719-742 reads */
    if (base->rc_bitrate > 0 &&
        (err = hl_amd_set_rate_control(self->enc, base->rc_bitrate, base->fps.num, base->fps.den, base->rc_basicunit,
                                       base->rc_qp_min, base->rc_qp_max)))
        return (HL_ERROR_T)err;
    self->width = W;
    self->height = H;
    return HL_ERROR_SUCCESS;
}

/* the encoder's result as hl_codec_264.c returns it */
static void gfx950_result(hl_codec_t* base, const hl_amd_result_t* r, hl_codec_result_t* result)
{
    result->type = HL_CODEC_RESULT_TYPE_NONE;
    if (r->type & HL_AMD_RESULT_TYPE_HDR) { /* hl_codec_264.c:675-686 */
        base->hdr_bytes = r->hdr;
        base->hdr_bytes_count = r->hdr_size;
        result->type |= HL_CODEC_RESULT_TYPE_HDR;
    }
    if (r->type & HL_AMD_RESULT_TYPE_DATA) { /* hl_codec_264.c:1000-1006 */
        result->type |= HL_CODEC_RESULT_TYPE_DATA;
        result->data_ptr = r->data; /* owned by the encoder, valid until the next call */
        result->data_size = r->data_size;
    }
}

/* plugin encode(): one planar YUV420 frame in host memory -> headers + one
 * slice NAL, as the stock plugin's _hl_codec_264_encode (hl_codec_264.c:
 * 404-1038) returns them.  With layers added (hl_codec_add_layer,
 * hl_codec.c:95-131) it is one layer of an SVC access unit: the caller
 * encodes the layers of a frame base first, the frame's size selects the
 * layer (hl_codec_264.c:470-481), and the last layer's DATA is the access
 * unit. */
static HL_ERROR_T gfx950_encode(hl_codec_t* base, const hl_frame_t* frame, hl_codec_result_t* result)
{
    hl_codec_264_gfx950_t* self = (hl_codec_264_gfx950_t*)base;
    const hl_frame_video_t* f = (const hl_frame_video_t*)frame;
    hl_amd_result_t r;
    int32_t err;
    hl_size_t l, L;
    if (!self || !f || !result) return HL_ERROR_INVALID_PARAMETER;
    if (self->input_type == GFX950_DECODING) return HL_ERROR_INVALID_OPERATION; /* hl_codec_264.c:447-452 */
    if (base->threads_count > 1) {
        /* the stock plugin cuts every picture into threads_count slices
         * (hl_codec_264.c:571, encode.c:488-495); hl_codec_create defaults
         * threads_count to the core count (hl_codec.c:33).  This plugin codes
         * one slice per picture: refused rather than a different stream. */
        fprintf(stderr, "hl_codec_264_gfx950: threads_count %d (%d slices per picture) is not implemented; set threads_count = 1\n",
                (int)base->threads_count, (int)base->threads_count);
        return HL_ERROR_NOT_IMPLEMENTED;
    }
    self->input_type = GFX950_ENCODING;
    L = base->layers_active_count;
    if (L > 1) {
        if (base->rc_bitrate > 0) {
            /* known gap: no reference golden pins rate control of
             * an SVC stream, and the gfx950 encoder does not implement it; refused
             * before any layer is coded */
            fprintf(stderr, "hl_codec_264_gfx950: spatial SVC with rate control (rc_bitrate > 0) is not implemented\n");
            return HL_ERROR_NOT_IMPLEMENTED;
        }
        if (!self->enc || self->layers != L || self->width != base->layers[0].u_width || self->height != base->layers[0].u_height) {
            if ((err = gfx950_open(self, base, base->layers[0].u_width, base->layers[0].u_height))) return (HL_ERROR_T)err;
            for (l = 0; l < L; ++l)
                if ((err = hl_amd_add_layer(self->enc, (int32_t)base->layers[l].u_width, (int32_t)base->layers[l].u_height)))
                    return (HL_ERROR_T)err;
            self->layers = L;
        }
        if ((err = hl_amd_encode_layer(self->enc, (int32_t)f->data_width[0], (int32_t)f->data_height[0], f->data_ptr[0],
                                       f->data_ptr[1], f->data_ptr[2], 0, &r)))
            return (HL_ERROR_T)err;
    }
    else {
        if (!self->enc || self->layers || f->data_width[0] != self->width || f->data_height[0] != self->height)
            if ((err = gfx950_open(self, base, f->data_width[0], f->data_height[0]))) return (HL_ERROR_T)err;
        if ((err = hl_amd_encode(self->enc, f->data_ptr[0], f->data_ptr[1], f->data_ptr[2], &r)))
            return (HL_ERROR_T)err;
    }
    gfx950_result(base, &r, result);
    result->width = f->data_width[0];
    result->height = f->data_height[0];
    return HL_ERROR_SUCCESS;
}

/* Look-ahead (HL_AMD_LOOKAHEAD, gfx950_open): codes the frames still queued
 * and returns the next result, one per call, NONE once none is left.  A
 * caller that opted in calls it after its last hl_codec_encode until NONE;
 * without look-ahead it returns NONE at once. */
HL_ERROR_T hl_codec_264_gfx950_flush(hl_codec_t* base, hl_codec_result_t* result)
{
    hl_codec_264_gfx950_t* self = (hl_codec_264_gfx950_t*)base;
    hl_amd_result_t r;
    int32_t err;
    if (!self || !result) return HL_ERROR_INVALID_PARAMETER;
    result->type = HL_CODEC_RESULT_TYPE_NONE;
    if (!self->enc || self->layers) return HL_ERROR_SUCCESS;
    if ((err = hl_amd_flush(self->enc, &r))) return (HL_ERROR_T)err;
    gfx950_result(base, &r, result);
    result->width = self->width;
    result->height = self->height;
    return HL_ERROR_SUCCESS;
}

static HL_ERROR_T gfx950_set_option(hl_codec_t* base, const struct hl_option_s* opt)
{
    return hl_codec_264_plugin_def_t->set_option(base, opt);
}

/* plugin decode(): decoding stays on the CPU, in the stock H.264 plugin
 * (hl_codec_264.c:79-402).  install() takes the stock plugin out of the
 * registry, so hl_codec_decode on a codec created after install lands here;
 * it is forwarded to a stock codec this object owns, created on the first
 * call with this object's settings.  Like the stock plugin, an object that
 * has encoded does not decode (hl_codec_264.c:100-106). */
static HL_ERROR_T gfx950_decode(hl_codec_t* base, const void* data, hl_size_t size, hl_codec_result_t* result)
{
    hl_codec_264_gfx950_t* self = (hl_codec_264_gfx950_t*)base;
    HL_ERROR_T err;
    if (!self) return HL_ERROR_INVALID_PARAMETER;
    if (self->input_type == GFX950_ENCODING) return HL_ERROR_INVALID_OPERATION;
    if (!self->dec) {
        if ((err = hl_codec_create(hl_codec_264_plugin_def_t, &self->dec))) return err;
        self->dec->threads_count = base->threads_count;
        self->dec->dqid_min = base->dqid_min;
        self->dec->dqid_max = base->dqid_max;
    }
    self->input_type = GFX950_DECODING;
    return hl_codec_decode(self->dec, data, size, result);
}

const hl_codec_plugin_def_t hl_codec_264_gfx950_plugin_def_s = {
    &gfx950_def_s, HL_CODEC_TYPE_H264, HL_MEDIA_TYPE_VIDEO, "H.264 AVC encoder (MI355X gfx950)", gfx950_set_option, gfx950_decode, gfx950_encode,
};

/* After hl_engine_init(): make this the plugin hl_codec_plugin_find(H264)
 * returns (hl_codec.c:161-229: register adds at the first free slot, find
 * returns the first match). */
HL_ERROR_T hl_codec_264_gfx950_install(void)
{
    HL_ERROR_T err = hl_codec_plugin_unregister(hl_codec_264_plugin_def_t);
    if (err) return err;
    return hl_codec_plugin_register(&hl_codec_264_gfx950_plugin_def_s);
}
