/*
 * hartallo_amd.h -- C ABI of the MI355X (gfx950) H.264 encode path.
 *
 * Drop-in boundary.  hartallo reaches an encoder through one plugin slot:
 *
 *   HL_ERROR_T (*encode)(struct hl_codec_s*, const struct hl_frame_s*,
 *                        struct hl_codec_result_s*);
 *     include/hartallo/hl_codec.h:173-184 (hl_codec_plugin_def_t.encode),
 *     called by hl_codec_encode, source/hl_codec.c:152-159.
 *
 * The H.264 plugin behind it (hl_codec_264_encode, source/h264/
 * hl_codec_264.c:637-1006) turns one planar YUV420 frame into headers +
 * one slice NAL.  The functions below are that operation with plain C types:
 * a maintainer registers a plugin def whose encode() forwards here (see
 * INTEGRATION.md), and hartallo's public API is unchanged.
 *
 * Semantics follow the reference:
 *   - parameters are the hl_codec_t fields the encoder reads
 *     (hl_codec.h:33-80): qp, gop_size, me_range, deblock_flag,
 *     me_early_term_flag; max_ref_frame through hl_amd_set_max_ref_frame;
 *     threads_count is 1 (the reference cuts a picture into threads_count
 *     slices, hl_codec_264.c:571; one slice per picture here);
 *   - width and height must be multiples of 16 (1088, not 1080 -- the
 *     reference rejects cropping, hl_codec_264.c:430-438);
 *   - result.type carries HL_CODEC_RESULT_TYPE_DATA / _HDR bits
 *     (hl_types.h:158-163); result.hdr holds "00 00 01"-prefixed SPS+PPS
 *     on the first frame (hl_codec_264.c:675-686), result.data the slice
 *     NAL without its start code (hl_codec_264.c:1000-1006);
 *   - the output buffers are owned by the encoder and valid until the next
 *     call (hl_codec_264.c:1000-1006);
 *   - errors are HL_ERROR_T values (hl_types.h:101-122).
 * Output is bit-identical to the reference encoder on the same input.
 */
#ifndef HARTALLO_AMD_H
#define HARTALLO_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* HL_ERROR_T values, hl_types.h:101-122 */
enum {
    HL_AMD_SUCCESS = 0,
    HL_AMD_ERROR_INVALID_PARAMETER = 1,
    HL_AMD_ERROR_INVALID_STATE = 3,
    HL_AMD_ERROR_INVALID_FORMAT = 4,
    HL_AMD_ERROR_NOT_FOUND = 6,
    HL_AMD_ERROR_NOT_IMPLEMENTED = 7,
    HL_AMD_ERROR_OUTOFMEMMORY = 8,
    HL_AMD_ERROR_OUTOFCAPACITY = 10,
    HL_AMD_ERROR_SYSTEM = 13,
    HL_AMD_ERROR_TOOSHORT = 15
};

/* HL_CODEC_RESULT_TYPE_T bits, hl_types.h:158-163 */
enum { HL_AMD_RESULT_TYPE_DATA = 1, HL_AMD_RESULT_TYPE_HDR = 2 };

typedef struct hl_amd_params_s {
    int32_t width;          /* hl_codec_t.width  (multiple of 16) */
    int32_t height;         /* hl_codec_t.height (multiple of 16) */
    int32_t qp;             /* hl_codec_t.qp, 0..51 */
    int32_t me_range;       /* hl_codec_t.me_range, clipped to [1,64] (rdo.c:847) */
    int32_t deblock;        /* hl_codec_t.deblock_flag */
    int32_t gop_size;       /* hl_codec_t.gop_size */
    int32_t me_early_term;  /* hl_codec_t.me_early_term_flag (homogeneity mode masks,
                               rdo.c:888-931); 1 needs width and height >= 32 */
    int32_t device;         /* HIP device ordinal */
} hl_amd_params_t;

typedef struct hl_amd_result_s {
    int32_t type;            /* HL_AMD_RESULT_TYPE_* bits */
    const uint8_t* hdr;      /* SPS + PPS with start codes, when type & HDR */
    size_t hdr_size;
    const uint8_t* data;     /* slice NAL without start code, when type & DATA */
    size_t data_size;
} hl_amd_result_t;

typedef struct hl_amd_encoder_s hl_amd_encoder_t;

/* hl_codec_create + option setting for HL_CODEC_TYPE_H264 (hl_codec.c:24-150) */
int32_t hl_amd_encoder_create(const hl_amd_params_t* params, hl_amd_encoder_t** encoder);
void hl_amd_encoder_destroy(hl_amd_encoder_t* encoder);

/* plugin encode() for a planar YUV420 frame in host memory
 * (hl_frame_video_t data_ptr[0..2], hl_frame.h:278-291) */
int32_t hl_amd_encode(hl_amd_encoder_t* encoder, const uint8_t* y, const uint8_t* u, const uint8_t* v,
                      hl_amd_result_t* result);

/* Look-ahead for per-frame callers (no reference interface: hl_codec_encode,
 * hl_codec.c:152-159, codes one frame per call and has no flush).  With
 * frames = k > 1, set before the first frame: hl_amd_encode queues each host
 * frame in device memory and codes every k queued frames as one
 * hl_amd_encode_batch (a frame-pipelined run); each call hands out the next
 * coded result in order -- type 0 (nothing) while the first k - 1 frames
 * queue, so a frame's bytes come k - 1 calls later -- and hl_amd_flush codes
 * what is still queued and hands out the remaining results, one per call,
 * type 0 once none is left.  The bytes are those of k separate calls.  An
 * error is reported by the call that codes the batch.  k = 1: off (the
 * default).  AVC only (adding a layer turns it off).  While frames are
 * queued, hl_amd_encode_device and hl_amd_encode_batch are refused
 * (HL_AMD_ERROR_INVALID_STATE): flush first. */
int32_t hl_amd_set_lookahead(hl_amd_encoder_t* encoder, int32_t frames);
int32_t hl_amd_flush(hl_amd_encoder_t* encoder, hl_amd_result_t* result);

/* same, with the planes already resident in device memory (HBM) */
int32_t hl_amd_encode_device(hl_amd_encoder_t* encoder, const uint8_t* y, const uint8_t* u, const uint8_t* v,
                             hl_amd_result_t* result);

/* n consecutive frames of the stream (planes resident in device memory),
 * encoded as if by n calls of hl_amd_encode_device, with results[i] the
 * i-th call's result (bitstreams identical).  Runs of P pictures are encoded
 * in one frame-pipelined launch: picture f+1 starts as soon as picture f has
 * finished the region its motion search can reach.  The data of every
 * result stays valid until the next call on this encoder.  No reference
 * interface: a throughput entry point for callers that hold several frames
 * (hl_codec_encode takes one frame per call, hl_codec.c:152-159). */
int32_t hl_amd_encode_batch(hl_amd_encoder_t* encoder, int32_t n, const uint8_t* const* y, const uint8_t* const* u,
                            const uint8_t* const* v, hl_amd_result_t* results);

/* n frames of each of `count` independent streams (1..16 encoders, one per
 * stream: the same picture size and device, no rate control, no spatial
 * layers) in shared pipelined runs: one persistent launch holds every
 * stream's pictures, so the streams' macroblock tasks share the device's
 * workgroups and one stream's wavefront ramp and tail overlap the others'
 * work (several streams per GPU without processes time-slicing the device).
 * y[s * n + i] = frame i of stream s (device memory, as hl_amd_encode_batch);
 * results[s * n + i] its result, valid until the next call on that encoder;
 * each stream's results are those of hl_amd_encode_batch on its encoder
 * alone (the reference serves N streams as N hl_codec_t instances,
 * hl_codec.c:24-150).  The diagnostics of every encoder (stats, timing)
 * describe the shared launches, and encoder 0's pipeline settings
 * (hl_amd_set_pipeline, hl_amd_set_intra_helpers, hl_amd_set_timing) govern
 * them.  The streams advance together: an error before any stream commits
 * leaves every encoder as it was; a stream whose picture-by-picture fallback
 * fails after others committed leaves every encoder of the call unusable
 * (HL_AMD_ERROR_INVALID_STATE from then on).  No reference interface. */
int32_t hl_amd_encode_streams(hl_amd_encoder_t* const* encoders, int32_t count, int32_t n, const uint8_t* const* y,
                              const uint8_t* const* u, const uint8_t* const* v, hl_amd_result_t* results);

/* rate control (hl_codec_t.rc_bitrate > 0; hl_codec_264.c:719-742, 1018-1031,
 * model hl_codec_264_rc.c): bitrate in bits/s, frame rate fps_den / fps_num
 * (hl_codec_t.fps, integer quotient), rc_basicunit (<= 0: the picture),
 * rc_qp_min / rc_qp_max (-1: 0 / 51).  Call before the first frame;
 * bitrate <= 0 turns it off.  Each picture's QP then follows the previous
 * pictures' bits, so hl_amd_encode_batch codes the pictures one by one. */
int32_t hl_amd_set_rate_control(hl_amd_encoder_t* encoder, int64_t bitrate, int32_t fps_num, int32_t fps_den,
                                int32_t basicunit, int32_t qp_min, int32_t qp_max);

/* hl_codec_t.max_ref_frame (hl_codec.c:36, default 1): the SPS's
 * max_num_ref_frames = min(MaxDpbMbs / PicSizeInMbs, max_ref_frame)
 * (hl_codec_264_sps.c:620-636) and the PPS's
 * num_ref_idx_l0_default_active_minus1 (hl_codec_264_pps.c:291), for every
 * (subset) SPS / PPS of the stream.  The reference's P slices override the
 * active references to one (slice.c:289, encode.c:269), so only the headers
 * change.  Any value >= 0 (the reference takes any and writes the clamped
 * one: 720p with 32 gives 5); HL_AMD_ERROR_INVALID_PARAMETER only when the
 * clamped value is above 16.  Call before the first frame (the reference
 * reads it when it builds the first SPS), else HL_AMD_ERROR_INVALID_STATE. */
int32_t hl_amd_set_max_ref_frame(hl_amd_encoder_t* encoder, int32_t max_ref_frame);

/* SliceQPY of the last encoded picture (the rate-controlled QP), or -1 */
int32_t hl_amd_last_qp(hl_amd_encoder_t* encoder);

/* pipelined-run scheduling: persistent workgroups (0 = one per resident
 * workgroup slot of the device, <= 4096), the reference reach R in MBs
 * (0..16) that a macroblock task of picture f+1 waits for in picture f
 * before it becomes ready, and the pictures (1..64, from the oldest
 * unfinished one) a workgroup looks at for ready tasks; defaults 0, 2, 64.
 * Results do not depend on these. */
int32_t hl_amd_set_pipeline(hl_amd_encoder_t* encoder, int32_t workgroups, int32_t reach, int32_t window);

/* resident workgroups per CU of the pipelined kernel (HIP occupancy query;
 * geometry tuning), or -1 */
int32_t hl_amd_pipeline_occupancy(void);

/* reconstructed (deblocked) picture of the last encoded frame, i.e. the
 * reference picture the next frame predicts from (dpb.c:160-170) */
int32_t hl_amd_get_recon(hl_amd_encoder_t* encoder, uint8_t* y, uint8_t* u, uint8_t* v);

/* Time of the last encode call, in milliseconds, split by stage.
 * Per-picture calls: [0] quarter-pel planes kernel, [1] macroblock-decision
 * kernels (sum over the wavefront launches, re-runs included), [2]
 * deblocking kernels, [3] the frame's device timeline from planes to
 * deblock end (host validation gaps included).
 * Pipelined runs (hl_amd_encode_batch): [0] planes of the picture before
 * the run, [1] the pipelined kernel, [2] the copy of the run's records to
 * the host, [3] host slice writing (wall time).  Filled only when timing is
 * on. */
int32_t hl_amd_set_timing(hl_amd_encoder_t* encoder, int32_t enable);
int32_t hl_amd_get_timing(hl_amd_encoder_t* encoder, float* ms4);

/* number of row-start re-runs the last frame needed (rdo.Single_ctr
 * speculation) -- diagnostics */
int32_t hl_amd_last_reruns(hl_amd_encoder_t* encoder);

/* number of in-kernel rdo.Single_ctr walks (resolve_chain: a row start
 * read the counter while its value was still speculated) in the last
 * pipelined run -- diagnostics */
int32_t hl_amd_last_chain_walks(hl_amd_encoder_t* encoder);

/* Diagnostics: `iters` launches of the quarter-pel plane kernel on the
 * encoder's current reference picture; *ms = average ms per launch (the
 * HBM-bound kernel's own roofline line in bench.py).  No reference interface. */
int32_t hl_amd_bench_planes(hl_amd_encoder_t* encoder, int32_t iters, float* ms);

/* number of macroblock-decision kernel launches of the last frame */
int32_t hl_amd_last_mb_launches(hl_amd_encoder_t* encoder);

/* How the last encode call (hl_amd_encode*, or one base-layer chunk of
 * hl_amd_encode_layers_batch) ran -- diagnostics, no reference interface:
 * out5[0] pipelined runs launched, [1] pictures coded on the per-picture
 * wavefront path, [2] runs that fell back to it (re-encoded picture by
 * picture), [3] bounded waits that gave up, [4] in-kernel rdo.Single_ctr
 * walks.  A healthy call has [1] = [2] = [3] = 0. */
int32_t hl_amd_last_batch_stats(hl_amd_encoder_t* encoder, int32_t* out5);

/* Intra helper tasks (pipelined runs, on by default; also HL_AMD_HELPERS=0
 * at create): a P macroblock's intra fallback (rdo.c:1161-1167) is prepared
 * by a second workgroup beside the macroblock's inter search -- every
 * Intra16x16 mode's transform, quantisation, CAVLC statistics and
 * reconstruction, and the Intra4x4 decision under a guess of the live
 * TotalCoeffs that the macroblock verifies; and, in a run
 * of one picture (the per-frame path), a third workgroup searches the
 * macroblock's P8x8 partitionings from its MB-start live TotalCoeffs while
 * the macroblock searches the larger ones, proven by nC-class intervals
 * before the macroblock takes them (HL_AMD_FAM3=0 at create
 * turns that part off).  Results do not depend on it.  No reference
 * interface. */
int32_t hl_amd_set_intra_helpers(hl_amd_encoder_t* encoder, int32_t enable);

/* How the intra fallbacks of the last encode call ran -- diagnostics:
 * out3[0] P macroblocks that kept their helper's Intra4x4 decision, [1]
 * that rejected it (an nC class differed: decided again), [2] whose helper
 * no workgroup had claimed in time (the macroblock decided intra itself). */
int32_t hl_amd_last_helper_stats(hl_amd_encoder_t* encoder, int32_t* out3);

/* How the 8x8-family helpers of the last encode call ran -- diagnostics:
 * out2[0] P macroblocks that took their helper's P8x8 searches, [1] that
 * found them unproven for their entry state (searched again). */
int32_t hl_amd_last_fam3_stats(hl_amd_encoder_t* encoder, int32_t* out2);

/* per-phase shader-clock counters of the macroblock kernel; filled only by
 * the profiling build (make profile); out[2k] = cycles, out[2k+1] = calls
 * for k < 32, then out[64 + addr] = cycles of macroblock addr in the last
 * frame (n <= 64 + macroblocks).  The phase counters are cleared by the call. */
int32_t hl_amd_profile_counters(hl_amd_encoder_t* encoder, unsigned long long* out, int32_t n);

/* diagnostics: the macroblock records (syntax handed to the slice writer,
 * hartallo_amd/csrc/hl_types.h MbRecord) of picture k of the last encode
 * call, bytes = macroblocks * hl_amd_record_size(); INVALID_STATE when the
 * call did not keep them (a run re-encoded picture by picture) */
int32_t hl_amd_debug_records(hl_amd_encoder_t* encoder, int32_t k, void* out, size_t bytes);
int32_t hl_amd_record_size(void);

/* diagnostics: the rdo.Single_ctr chain records (hl_types.h MbChain, 20 bytes
 * per macroblock) and the reconstructed (deblocked) planes of picture k of
 * the last encode call */
int32_t hl_amd_debug_chain(hl_amd_encoder_t* encoder, int32_t k, void* out, size_t bytes);
int32_t hl_amd_debug_recon(hl_amd_encoder_t* encoder, int32_t k, uint8_t* y, uint8_t* u, uint8_t* v);

/* ---- Spatial SVC (Annex G) ----
 * hl_codec_add_layer (source/hl_codec.c:95-131): layers in increasing order,
 * the first one of the encoder's own size; each further layer twice the one
 * below (the reference accepts any power-of-two ratio, its encoder is only
 * exercised dyadic; other ratios return NOT_IMPLEMENTED).  At most 4 layers
 * (HL_ENCODER_MAX_LAYERS, OUTOFCAPACITY).  Call before the first frame. */
int32_t hl_amd_add_layer(hl_amd_encoder_t* encoder, int32_t width, int32_t height);

/* plugin encode() of a frame of the given size (hl_frame_video_t.data_width /
 * data_height[0]): with layers, the frame's size selects the layer
 * (hl_codec_264.c:470-483, NOT_FOUND otherwise) and the layers of an access
 * unit come in increasing order (INVALID_STATE otherwise).  Like the
 * reference, result.type has HDR whenever the header set grew (the first
 * frame of each layer; result.hdr then holds every SPS, subset SPS and PPS)
 * and DATA only with the access unit's last layer (result.data = prefix NAL,
 * base slice and enhancement slices, "00 00 01"-separated, no leading start
 * code; hl_codec_264.c:999-1017).  on_device: planes in HBM (else host).
 * Without layers this is hl_amd_encode / hl_amd_encode_device. */
int32_t hl_amd_encode_layer(hl_amd_encoder_t* encoder, int32_t width, int32_t height, const uint8_t* y, const uint8_t* u,
                            const uint8_t* v, int32_t on_device, hl_amd_result_t* result);

/* reconstructed (deblocked) picture of layer `layer` after its last frame */
int32_t hl_amd_get_layer_recon(hl_amd_encoder_t* encoder, int32_t layer, uint8_t* y, uint8_t* u, uint8_t* v);

/* enhancement-layer macroblocks coded so far whose reference-layer macroblock
 * was intra in a P picture: the reference's output there depends on its
 * uninitialised scratch memory (hartallo_amd/csrc/hl_svc.h), so they are
 * outside the bit-exact guarantee; 0 on every pinned workload */
int32_t hl_amd_svc_unpinned(hl_amd_encoder_t* encoder);

/* Layer-sharded coding (one process / GPU per layer).  An encoder with all
 * layers added codes only layers [first, last] (no reference interface: the
 * reference codes every layer in one hl_codec_t).  Per access unit the rank
 * coding the layer below `first` exports that layer's state -- picture
 * Y|U|V and macroblock objects, hl_amd_layer_state_bytes() bytes -- into a
 * device buffer (hl_amd_export_layer, after its last call of the access
 * unit), the buffer travels (RCCL over xGMI), and this encoder imports it
 * (hl_amd_import_layer) before coding `first`.  The DATA of the call for
 * `last` then holds only layers [first, last] ("00 00 01"-separated); the
 * access unit is the ranks' parts joined with "00 00 01" in layer order. */
int32_t hl_amd_set_layer_range(hl_amd_encoder_t* encoder, int32_t first, int32_t last);
size_t hl_amd_layer_state_bytes(hl_amd_encoder_t* encoder, int32_t layer);
int32_t hl_amd_export_layer(hl_amd_encoder_t* encoder, int32_t layer, void* dst_device);
int32_t hl_amd_import_layer(hl_amd_encoder_t* encoder, int32_t layer, const void* src_device);

/* n access units of every layer (planes in HBM; planes[(l * n + i) * 3 + c]
 * = plane c of layer l's frame of access unit i), as if by the
 * hl_amd_encode_layer calls for them: the base-layer pictures are coded
 * frame-pipelined (hl_amd_encode_batch), then every enhancement layer.
 * results[i] = access unit i: HDR with every header set those calls signal,
 * in order, and DATA; valid until the next call.  Needs every layer coded by
 * this encoder (no layer range).  No reference interface: a throughput entry
 * point like hl_amd_encode_batch.  A call that fails part-way leaves the
 * layers of its access units inconsistent: every later call then returns
 * HL_AMD_ERROR_INVALID_STATE, and destroying and re-creating the encoder is
 * the only reset. */
int32_t hl_amd_encode_layers_batch(hl_amd_encoder_t* encoder, int32_t n, int32_t layers, const uint8_t* const* planes,
                                   hl_amd_result_t* results);

/* device time (ms) of the enhancement layers of the last access unit (with
 * hl_amd_set_timing on) */
float hl_amd_svc_layer_ms(hl_amd_encoder_t* encoder);

const char* hl_amd_version(void);

#ifdef __cplusplus
}
#endif

#endif
