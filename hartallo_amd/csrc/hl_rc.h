// hl_rc.h -- frame-level rate control of the encoder (rc_bitrate > 0).
//
// The reference enables a JM-style quadratic rate controller when
// hl_codec_t.rc_bitrate > 0 (source/h264/hl_codec_264.c:719-742,
// 1018-1031; model in source/h264/hl_codec_264_rc.c, update mode 0, no B
// pictures, frame coding).  Its only effect on the bitstream is the QP of
// each picture (slice_qp_delta, lambda, quantisers, deblocking), chosen
// before the picture from the statistics of the pictures before it:
//   - per picture: the bits of its slice NAL, the slice-header + MB-header
//     bits and the residual ("texture") bits (mb.c:543-892 split);
//   - per macroblock: the RDO distortion of the chosen mode, summed as the
//     picture MAD (rdo.c:211-228, 1266-1268).
// The macroblock-level QP hook of the reference is compiled out
// (slice.c:1806-1816), so a basic unit smaller than the picture only
// changes the model bookkeeping, never the QP inside a picture.
//
// Everything here runs on the host between pictures; arithmetic types
// (float vs double vs int64) follow the reference exactly because the
// chosen QP depends on their rounding.
#pragma once
#include <stdint.h>

#include <vector>

namespace hl {

struct RcConfig {
    int64_t bitrate;     // hl_codec_t.rc_bitrate (> 0 enables the controller)
    int32_t fps_num;     // hl_codec_t.fps (frame rate = den / num, integer)
    int32_t fps_den;
    int32_t basicunit;   // hl_codec_t.rc_basicunit (<= 0: whole picture)
    int32_t qp_min;      // hl_codec_t.rc_qp_min (< 0: 0)
    int32_t qp_max;      // hl_codec_t.rc_qp_max (outside [0, 51]: 51)
    int32_t gop_size;    // hl_codec_t.gop_size (IDR period)
    int32_t width, height;
};

// Statistics of one encoded picture, as the reference accumulates them.
struct RcPictureStats {
    int64_t mad_sum;      // sum over macroblocks of the chosen mode's distortion
    int32_t header_bits;  // slice header (NAL header byte included) + all MB headers
    int32_t texture_bits; // residual() bits
    int32_t nbits;        // bits of the slice NAL as stored (escaped bytes * 8)
};

class RateControl {
public:
    // hl_codec_264_rc_init (rc.c:288-327) + _rc_init_seq (rc.c:1886-2021)
    explicit RateControl(const RcConfig& cfg);
    // QP of the next picture: hl_codec_264_rc_start_gop at an IDR
    // (rc.c:355-370) and hl_codec_264_rc_start_frame (rc.c:383-399)
    int32_t begin_picture(bool idr);
    // hl_codec_264_rc_end_frame (rc.c:445-457) and, after the last picture
    // of a GOP, hl_codec_264_rc_end_gop (rc.c:372-381)
    void end_picture(bool idr, const RcPictureStats& st, bool gop_end);

private:
    void init_gop(int np, int nb);
    void init_picture(bool p_slice);
    int32_t update_qp(bool p_slice);
    int32_t model_qp(int bits);
    void update_model();
    void update_mad_model();
    void estimate_rd(int n, const bool* rejected);
    void estimate_mad(int n, const bool* rejected);

    RcConfig cfg_;
    int32_t pic_mbs_, mb_per_row_, size_, frame_rate_i_;
    int32_t basicunit_, min_qp_, max_qp_, seinitial_qp_;
    int32_t number_, curr_frm_idx_, qp_;
    bool frame_level_;
    // generic state (RCGeneric, rc.c:82-110)
    int32_t hdr_bits_, tex_bits_, bu_hdr_bits_, bu_tex_bits_;
    int32_t n_gop_;
    int64_t bu_mad_sum_, buffer_fullness_, remaining_bits_;
    int64_t frame_mad_sum_;
    // quadratic model state (RCQuadratic, rc.c:112-207)
    float bit_rate_, frame_rate_, prev_bit_rate_;
    double gamma_p_, beta_p_, gop_target_level_, target_level_, ave_wp_;
    int32_t initial_qp_, p_average_qp_;
    double prev_picture_mad_, mad_c1_, mad_c2_, p_mad_c1_, p_mad_c2_;
    double p_picture_mad_[21], picture_mad_[21], reference_mad_[21];
    double rg_qp_[21], rg_rp_[21], p_rg_qp_[21], p_rg_rp_[21];
    double x1_, x2_, p_x1_, p_x2_;
    int32_t p_qp_, mad_window_, rd_window_, qc_;
    int32_t p_pre_header_, prev_last_qp_, curr_last_qp_;
    int32_t total_frame_qp_, n_basic_unit_, p_ave_hdr1_, p_ave_hdr2_, p_ave_hdr3_, p_ave_frame_qp_;
    int32_t total_basic_units_, coded_basic_units_;
    int32_t coded_p_frames_, total_qp_p_, n_p_pictures_;
    double curr_frame_mad_, total_bu_mad_, prev_frame_mad_;
    int32_t ddquant_, qp_last_p_frame_, qp_last_gop_;
    std::vector<double> bu_prev_mad_, bu_curr_mad_;
    bool gop_overdue_;
    int32_t xp_, target_, np_, nb_;
    int32_t upper1_, upper2_, lower_;
    double wp_, wb_, delta_p_;
    int32_t total_p_frames_, max_qp_change_;
};

}  // namespace hl
