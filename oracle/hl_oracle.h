/*
 * hl_oracle.h -- CPU restatement of allweax/hartallo's H.264 encoder hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product
 * (hartallo_amd/, libhartallo_amd.so) never links it.
 *
 * It restates, single-threaded and in plain C, the reference's encode path
 * (source/h264/hl_codec_264_{slice,mb,rdo,me_ds,residual,cavlc,transf,quant,
 * interpol,pred_inter,pred_intra,utils,deblock,encode,sps,pps,rbsp}.c) with
 * every stateful quirk needed for bit-identical output, and is pinned against
 * the reference itself (oracle/_ref/ref_enc) and the committed golden
 * fixtures in tests/golden/.
 */
#ifndef HL_ORACLE_H
#define HL_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hlo_params_s {
    int32_t width;        /* luma width, multiple of 16 (hl_codec_264.c:430) */
    int32_t height;       /* luma height, multiple of 16 (hl_codec_264.c:433) */
    int32_t qp;           /* hl_codec_t.qp                                   */
    int32_t me_range;     /* hl_codec_t.me_range (clipped to [1,64])         */
    int32_t deblock;      /* hl_codec_t.deblock_flag                         */
    int32_t gop_size;     /* hl_codec_t.gop_size                             */
    int32_t early_term;   /* hl_codec_t.me_early_term_flag (rdo.c:888-931)   */
} hlo_params_t;

typedef struct hlo_enc_s hlo_enc_t;

hlo_enc_t* hlo_create(const hlo_params_t* params);
void hlo_destroy(hlo_enc_t* enc);

/* hl_codec_t.max_ref_frame (default 1), before the first frame: the SPS's
 * max_num_ref_frames and the PPS's num_ref_idx_l0_default_active_minus1
 * (sps.c:620-636, pps.c:291).  0 on success. */
int hlo_set_max_ref_frame(hlo_enc_t* enc, int max_ref_frame);

/* Encodes one planar YUV420 frame.  Writes into out exactly the bytes the
 * reference harness writes for that frame: the SPS/PPS header bytes on the
 * first frame, then 00 00 01 + the (escaped) slice NAL.  Returns 0 on
 * success, <0 on error. */
int hlo_encode_frame(hlo_enc_t* enc, const uint8_t* y, const uint8_t* u, const uint8_t* v,
                     uint8_t* out, size_t out_cap, size_t* out_len);

/* Reconstructed (deblocked) reference picture of the last encoded frame. */
const uint8_t* hlo_recon(const hlo_enc_t* enc, int plane);

/* Per-MB records (oracle/mbrec.h layout, MBR_STRIDE int32 each). */
void hlo_dump_mbs(const hlo_enc_t* enc, int32_t* recs);

/* Counter of RDO bit-buffer overflows (must stay 0; see residual.c:587). */
int64_t hlo_rdo_overflows(const hlo_enc_t* enc);

#ifdef __cplusplus
}
#endif

#endif
