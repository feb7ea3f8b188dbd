// hl_rc.cpp -- frame-level quadratic rate control (see hl_rc.h).
//
// Follows source/h264/hl_codec_264_rc.c of the reference with its build
// constants folded in: update mode 0 (rc.c:220), no B pictures (:221), frame
// coding without MBAFF (:224-225), constant channel (:226), at most 4 QP
// steps between pictures (:232), SPS frame_mbs_only_flag = 1.  Each member
// function names the reference function it restates.  Operand types mirror
// the reference (float rates, double model, int64 buffers) so that every
// intermediate rounds the same way.
#include "hl_rc.h"

#include <limits.h>
#include <math.h>
#include <string.h>

#include <algorithm>

namespace hl {

namespace {
constexpr int kHist = 21;                // RC_MODEL_HISTORY, rc.c:56
constexpr float kOmega = 0.9F;           // rc.c:217
constexpr float kMinValue = 4.0F;        // rc.c:218
constexpr int kQcifPix = 25344, kCifPix = 101376;  // rc.c:49-51

inline int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

// _QP2Qstep, rc.c:1781-1793
double qp_to_qstep(int qp)
{
    static const double kBase[6] = {0.625, 0.6875, 0.8125, 0.875, 1.0, 1.125};
    double q = kBase[qp % 6];
    for (int i = 0; i < qp / 6; ++i) q *= 2;
    return q;
}

// _Qstep2QP, rc.c:1737-1779
int qstep_to_qp(double q)
{
    if (q < qp_to_qstep(0)) return 0;
    if (q > qp_to_qstep(51)) return 51;
    int per = 0;
    while (q > qp_to_qstep(5)) {
        q /= 2.0;
        ++per;
    }
    static const double kEdge[5] = {0.65625, 0.75, 0.84375, 0.9375, 1.0625};
    int rem = 5;
    for (int i = 0; i < 5; ++i)
        if (q <= kEdge[i]) {
            rem = i;
            break;
        }
    return per * 6 + rem;
}
}  // namespace

RateControl::RateControl(const RcConfig& c) : cfg_(c)
{
    pic_mbs_ = (c.width / 16) * (c.height / 16);
    mb_per_row_ = c.width / 16;
    size_ = c.width * c.height;
    frame_rate_i_ = c.fps_den / c.fps_num;
    basicunit_ = c.basicunit > 0 ? c.basicunit : pic_mbs_;
    min_qp_ = c.qp_min >= 0 ? c.qp_min : 0;                        // rc.c:713
    max_qp_ = (c.qp_max >= 0 && c.qp_max <= 51) ? c.qp_max : 51;   // rc.c:714
    frame_level_ = basicunit_ == pic_mbs_;
    number_ = curr_frm_idx_ = 0;
    qp_ = 0;
    hdr_bits_ = tex_bits_ = bu_hdr_bits_ = bu_tex_bits_ = 0;
    n_gop_ = 0;
    bu_mad_sum_ = buffer_fullness_ = remaining_bits_ = frame_mad_sum_ = 0;
    ave_wp_ = 0.0;
    initial_qp_ = p_average_qp_ = 0;
    prev_picture_mad_ = mad_c1_ = mad_c2_ = 0.0;
    memset(picture_mad_, 0, sizeof(picture_mad_));
    memset(reference_mad_, 0, sizeof(reference_mad_));
    memset(rg_qp_, 0, sizeof(rg_qp_));
    memset(rg_rp_, 0, sizeof(rg_rp_));
    x1_ = x2_ = 0.0;
    qc_ = 0;
    prev_last_qp_ = curr_last_qp_ = 0;
    total_frame_qp_ = n_basic_unit_ = p_ave_hdr2_ = p_ave_frame_qp_ = 0;
    coded_basic_units_ = 0;
    total_qp_p_ = n_p_pictures_ = 0;
    total_bu_mad_ = 0.0;
    // _rc_alloc_quadratic (rc.c:571-587): the model starts with unit MADs and
    // unbounded HRD limits; the struct is malloc'ed, and QPLastPFrame, read by
    // the second GOP (rc.c:866) but only written by the basic-unit path, is
    // taken as the zero of fresh heap memory
    curr_frame_mad_ = prev_frame_mad_ = 1.0;
    qp_last_p_frame_ = qp_last_gop_ = 0;
    gop_overdue_ = false;
    xp_ = target_ = np_ = nb_ = 0;
    upper1_ = upper2_ = INT_MAX;
    lower_ = 0;
    wp_ = wb_ = delta_p_ = 0.0;
    total_p_frames_ = 0;
    target_level_ = 0.0;

    // _rc_init_seq, rc.c:1886-2021
    bit_rate_ = (float)c.bitrate;
    frame_rate_ = (float)(double)frame_rate_i_;
    prev_bit_rate_ = bit_rate_;
    const int bu = std::min(basicunit_, pic_mbs_);
    total_basic_units_ = bu < pic_mbs_ ? pic_mbs_ / bu : 1;
    buffer_fullness_ = 0;
    gop_target_level_ = (double)buffer_fullness_;
    rd_window_ = mad_window_ = 0;
    coded_p_frames_ = 0;
    remaining_bits_ = 0;
    gamma_p_ = 0.5;
    beta_p_ = 0.5;
    p_pre_header_ = 0;
    p_x1_ = bit_rate_ * 1.0;
    p_x2_ = 0.0;
    p_mad_c1_ = 1.0;
    p_mad_c2_ = 0.0;
    for (int i = 0; i < kHist; ++i) {
        p_rg_qp_[i] = 0;
        p_rg_rp_[i] = 0.0;
        p_picture_mad_[i] = 0.0;
    }
    max_qp_change_ = 4;
    p_ave_hdr1_ = p_ave_hdr3_ = 0;
    ddquant_ = total_basic_units_ >= 9 ? 1 : 2;
    bu_prev_mad_.assign(std::max(1, pic_mbs_ / basicunit_), 0.0);
    bu_curr_mad_.assign(bu_prev_mad_.size(), 0.0);
    // initial QP from the bits per pixel (rc.c:1983-2015)
    const double bpp = 1.0 * bit_rate_ / (frame_rate_ * (float)(size_t)size_);
    double l1, l2, l3;
    if (size_ <= kQcifPix) {
        l1 = 0.1;
        l2 = 0.3;
        l3 = 0.6;
    }
    else if (size_ <= kCifPix) {
        l1 = 0.2;
        l2 = 0.6;
        l3 = 1.2;
    }
    else {
        l1 = 0.6;
        l2 = 1.4;
        l3 = 2.4;
    }
    seinitial_qp_ = bpp <= l1 ? 35 : (bpp <= l2 ? 25 : (bpp <= l3 ? 20 : 10));
}

// _rc_init_gop_params (rc.c:632-697, mode 0 with an IDR period) and
// _rc_init_GOP (rc.c:699-889)
void RateControl::init_gop(int np, int nb)
{
    lower_ = (int)(remaining_bits_ + bit_rate_ / frame_rate_);
    upper1_ = (int)(remaining_bits_ + (bit_rate_ * 2.048));
    const int64_t alloc = (int64_t)floor((1 + np + nb) * bit_rate_ / frame_rate_ + 0.5);
    remaining_bits_ += alloc;
    np_ = np;
    nb_ = nb;
    gop_overdue_ = false;
    total_p_frames_ = np;
    ++n_gop_;
    if (n_gop_ == 1) {
        initial_qp_ = seinitial_qp_;
        curr_last_qp_ = initial_qp_ - 1;
        qp_last_gop_ = initial_qp_;
        p_ave_frame_qp_ = initial_qp_;
        qc_ = p_ave_frame_qp_;
        p_average_qp_ = p_ave_frame_qp_;
    }
    else {
        p_average_qp_ = (int)(1.0 * total_qp_p_ / n_p_pictures_ + 0.5);
        int gdq = (int)((1.0 * (np + nb + 1) / 15.0) + 0.5);
        if (gdq > 2) gdq = 2;
        p_average_qp_ -= gdq;
        if (p_average_qp_ > (qp_last_p_frame_ - 2)) p_average_qp_--;
        p_average_qp_ = clip3(qp_last_gop_ - 2, qp_last_gop_ + 2, p_average_qp_);
        p_average_qp_ = clip3(min_qp_, max_qp_, p_average_qp_);
        initial_qp_ = p_average_qp_;
        p_qp_ = p_average_qp_;
        p_ave_frame_qp_ = p_average_qp_;
        qp_last_gop_ = initial_qp_;
        prev_last_qp_ = curr_last_qp_;
        curr_last_qp_ = initial_qp_ - 1;
    }
    total_qp_p_ = 0;
    n_p_pictures_ = 0;
}

// _rc_init_pict with fieldpic = 1, topfield = 0, targetcomputation = 1,
// mult = 1 (rc.c:891-1120)
void RateControl::init_picture(bool p_slice)
{
    const int tnbu = pic_mbs_ / basicunit_;
    if (p_slice) {
        if (frame_level_) {
            if (n_p_pictures_ == 1) {
                target_level_ = (double)buffer_fullness_;
                delta_p_ = (buffer_fullness_ - gop_target_level_) / (total_p_frames_ - 1);
                target_level_ -= delta_p_;
            }
            else if (n_p_pictures_ > 1) {
                target_level_ -= delta_p_;
            }
        }
        else {
            if (coded_p_frames_ > 0) std::copy(bu_curr_mad_.begin(), bu_curr_mad_.begin() + tnbu, bu_prev_mad_.begin());
            if (n_gop_ == 1) {
                if (n_p_pictures_ == 1) {
                    target_level_ = (double)buffer_fullness_;
                    delta_p_ = (buffer_fullness_ - gop_target_level_) / (total_p_frames_ - 1);
                    target_level_ -= delta_p_;
                }
                else if (n_p_pictures_ > 1) {
                    target_level_ -= delta_p_;
                }
            }
            else if (n_gop_ > 1) {
                if (n_p_pictures_ == 0) {
                    target_level_ = (double)buffer_fullness_;
                    delta_p_ = (buffer_fullness_ - gop_target_level_) / total_p_frames_;
                    target_level_ -= delta_p_;
                }
                else if (n_p_pictures_ > 0) {
                    target_level_ -= delta_p_;
                }
            }
        }
        if (coded_p_frames_ == 1) ave_wp_ = wp_;
        if (coded_p_frames_ < 8 && coded_p_frames_ > 1) ave_wp_ = (ave_wp_ + wp_ * (coded_p_frames_ - 1)) / coded_p_frames_;
        else if (coded_p_frames_ > 1) ave_wp_ = (wp_ + 7 * ave_wp_) / 8;
        // target bits of the picture
        const bool compute = frame_level_ ? coded_p_frames_ > 0 : ((n_gop_ == 1 && coded_p_frames_ > 0) || n_gop_ > 1);
        if (compute) {
            target_ = (int)floor(wp_ * remaining_bits_ / (np_ * wp_ + nb_ * wb_) + 0.5);
            const int t = std::max(0, (int)floor(bit_rate_ / frame_rate_ - gamma_p_ * (buffer_fullness_ - target_level_) + 0.5));
            target_ = (int)floor(beta_p_ * (target_ - t) + t + 0.5);
        }
        target_ = (int)(1.0F * target_);
        target_ = clip3(lower_, upper2_, target_);
    }
    hdr_bits_ = 0;
    tex_bits_ = 0;
    if (!frame_level_) {
        total_frame_qp_ = 0;
        bu_hdr_bits_ = 0;
        bu_tex_bits_ = 0;
        bu_mad_sum_ = 0;
        n_basic_unit_ = total_basic_units_;
    }
}

// _updateModelQPFrame, rc.c:1462-1476
int32_t RateControl::model_qp(int bits)
{
    double qstep;
    const double d = curr_frame_mad_ * x1_ * curr_frame_mad_ * x1_ + 4 * x2_ * curr_frame_mad_ * bits;
    if (x2_ == 0.0 || d < 0 || (sqrt(d) - x1_ * curr_frame_mad_) <= 0.0) qstep = (float)(x1_ * curr_frame_mad_ / (double)bits);
    else qstep = (float)((2 * x2_ * curr_frame_mad_) / (sqrt(d) - x1_ * curr_frame_mad_));
    return qstep_to_qp(qstep);
}

// _updateQPRC0, rc.c:1165-1417 (top field / frame, FieldControl = 0)
int32_t RateControl::update_qp(bool p_slice)
{
    if (!p_slice) {
        qc_ = initial_qp_;
        return qc_;
    }
    if (frame_level_) {
        if (n_p_pictures_ != 0) {
            x1_ = p_x1_;
            x2_ = p_x2_;
            mad_c1_ = p_mad_c1_;
            mad_c2_ = p_mad_c2_;
            prev_picture_mad_ = p_picture_mad_[0];
            const int qp = p_qp_, hp = p_pre_header_;
            curr_frame_mad_ = mad_c1_ * prev_picture_mad_ + mad_c2_;
            if (target_ < 0) {
                qc_ = clip3(min_qp_, max_qp_, qp + max_qp_change_);
            }
            else {
                int bits = target_ - hp;
                bits = std::max(bits, (int)(bit_rate_ / (kMinValue * frame_rate_)));
                qc_ = model_qp(bits);
                qc_ = clip3(min_qp_, max_qp_, qc_);
                qc_ = clip3(qp - max_qp_change_, qp + max_qp_change_, qc_);
            }
        }
        else {
            qc_ = initial_qp_;
        }
        // _updateQPNonPicAFF, rc.c:1435-1447
        total_qp_p_ += qc_;
        prev_last_qp_ = curr_last_qp_;
        curr_last_qp_ = qc_;
        p_qp_ = qc_;
        return qc_;
    }
    // basic-unit model: only the first unit's QP is ever asked for
    if (n_gop_ == 1 && n_p_pictures_ == 0) {  // _updateFirstP, rc.c:1493-1526
        qc_ = initial_qp_;
        bu_hdr_bits_ = 0;
        bu_tex_bits_ = 0;
        n_basic_unit_--;
        if (n_basic_unit_ == 0) {  // a one-unit picture (topfield = 0)
            total_qp_p_ += qc_;
            prev_last_qp_ = curr_last_qp_;
            curr_last_qp_ = qc_;
            p_ave_frame_qp_ = qc_;
            p_ave_hdr3_ = p_ave_hdr2_;
        }
        p_qp_ = qc_;
        total_frame_qp_ += qc_;
        return qc_;
    }
    x1_ = p_x1_;
    x2_ = p_x2_;
    mad_c1_ = p_mad_c1_;
    mad_c2_ = p_mad_c2_;
    // _updateFirstBU, rc.c:1528-1570
    if (target_ <= 0) {
        qc_ = p_ave_frame_qp_ + 2;
        if (cfg_.qp_max >= 0 && qc_ > cfg_.qp_max) qc_ = cfg_.qp_max;
        gop_overdue_ = true;
    }
    else {
        qc_ = p_ave_frame_qp_;
    }
    total_frame_qp_ += qc_;
    n_basic_unit_--;
    p_qp_ = p_ave_frame_qp_;
    return qc_;
}

int32_t RateControl::begin_picture(bool idr)
{
    if (idr) {
        // rc_start_gop: np = n - 1 P pictures of an n-picture GOP (rc.c:673-690)
        const int n = cfg_.gop_size;
        const int np = curr_frm_idx_ == 0 ? 1 + (n - 2) : (n - 1);
        init_gop(np, n - np - 1);
    }
    // _rc_init_frame, rc.c:1122-1163
    init_picture(!idr);
    qp_ = update_qp(!idr);
    return qp_;
}

// _RCModelEstimator, rc.c:2189-2251
void RateControl::estimate_rd(int n, const bool* rej)
{
    int real = n;
    for (int i = 0; i < n; ++i)
        if (rej[i]) real--;
    x1_ = x2_ = 0.0;
    double one = 0;
    bool second = false;
    for (int i = 0; i < n; ++i)
        if (!rej[i]) one = rg_qp_[i];
    for (int i = 0; i < n; ++i) {
        if (rg_qp_[i] != one && !rej[i]) second = true;
        if (!rej[i]) x1_ += (rg_qp_[i] * rg_rp_[i]) / real;
    }
    if (real >= 1 && second) {
        double a00 = 0.0, a01 = 0.0, a10 = 0.0, a11 = 0.0, b0 = 0.0, b1 = 0.0;
        for (int i = 0; i < n; ++i)
            if (!rej[i]) {
                a00 = a00 + 1.0;
                a01 += 1.0 / rg_qp_[i];
                a10 = a01;
                a11 += 1.0 / (rg_qp_[i] * rg_qp_[i]);
                b0 += rg_qp_[i] * rg_rp_[i];
                b1 += rg_rp_[i];
            }
        const double det = a00 * a11 - a01 * a10;
        if (fabs(det) > 0.000001) {
            x1_ = (b0 * a11 - b1 * a01) / det;
            x2_ = (b1 * a00 - b0 * a10) / det;
        }
        else {
            x1_ = b0 / a00;
            x2_ = 0.0;
        }
    }
    p_x1_ = x1_;
    p_x2_ = x2_;
}

// _MADModelEstimator, rc.c:2253-2316
void RateControl::estimate_mad(int n, const bool* rej)
{
    int real = n;
    for (int i = 0; i < n; ++i)
        if (rej[i]) real--;
    mad_c1_ = mad_c2_ = 0.0;
    double one = 0.0;
    bool second = false;
    for (int i = 0; i < n; ++i)
        if (!rej[i]) one = picture_mad_[i];
    for (int i = 0; i < n; ++i) {
        if (picture_mad_[i] != one && !rej[i]) second = true;
        if (!rej[i]) mad_c1_ += picture_mad_[i] / (reference_mad_[i] * real);
    }
    if (real >= 1 && second) {
        double a00 = 0.0, a01 = 0.0, a10 = 0.0, a11 = 0.0, b0 = 0.0, b1 = 0.0;
        for (int i = 0; i < n; ++i)
            if (!rej[i]) {
                a00 = a00 + 1.0;
                a01 += reference_mad_[i];
                a10 = a01;
                a11 += reference_mad_[i] * reference_mad_[i];
                b0 += picture_mad_[i];
                b1 += picture_mad_[i] * reference_mad_[i];
            }
        const double det = a00 * a11 - a01 * a10;
        if (fabs(det) > 0.000001) {
            mad_c2_ = (b0 * a11 - b1 * a01) / det;
            mad_c1_ = (b1 * a00 - b0 * a10) / det;
        }
        else {
            mad_c1_ = b0 / a01;
            mad_c2_ = 0.0;
        }
    }
    p_mad_c1_ = mad_c1_;
    p_mad_c2_ = mad_c2_;
}

// _updateMADModel, rc.c:2318-2404
void RateControl::update_mad_model()
{
    if (coded_p_frames_ <= 0) return;
    const int nc = frame_level_ ? coded_p_frames_ : coded_p_frames_ * total_basic_units_ + coded_basic_units_;
    for (int i = kHist - 2; i > 0; --i) {
        p_picture_mad_[i] = p_picture_mad_[i - 1];
        picture_mad_[i] = p_picture_mad_[i];
        reference_mad_[i] = reference_mad_[i - 1];
    }
    p_picture_mad_[0] = curr_frame_mad_;
    picture_mad_[0] = p_picture_mad_[0];
    reference_mad_[0] = frame_level_ ? picture_mad_[1] : bu_prev_mad_[total_basic_units_ - 1 - n_basic_unit_];
    mad_c1_ = p_mad_c1_;
    mad_c2_ = p_mad_c2_;
    int n = curr_frame_mad_ > prev_frame_mad_ ? (int)((float)(kHist - 1) * prev_frame_mad_ / curr_frame_mad_)
                                               : (int)((float)(kHist - 1) * curr_frame_mad_ / prev_frame_mad_);
    n = clip3(1, nc - 1, n);
    n = std::min(n, std::min(20, mad_window_ + 1));
    mad_window_ = n;
    bool rej[kHist] = {false};
    prev_frame_mad_ = curr_frame_mad_;
    estimate_mad(n, rej);
    double err[kHist], sq = 0.0;
    for (int i = 0; i < n; ++i) {
        err[i] = mad_c1_ * reference_mad_[i] + mad_c2_ - picture_mad_[i];
        sq += err[i] * err[i];
    }
    const double thr = n == 2 ? 0 : sqrt(sq / n);
    for (int i = 0; i < n; ++i)
        if (fabs(err[i]) > thr) rej[i] = true;
    rej[0] = false;
    estimate_mad(n, rej);
}

// _updateRCModel, rc.c:2406-2538 (P pictures)
void RateControl::update_model()
{
    int nc;
    if (frame_level_) {
        curr_frame_mad_ = (double)frame_mad_sum_ / (256.0 * (double)pic_mbs_);  // _ComputeFrameMAD, rc.c:2156-2168
        nc = coded_p_frames_;
    }
    else {
        curr_frame_mad_ = (double)((bu_mad_sum_ >> 8) / basicunit_);
        bu_mad_sum_ = 0;
        coded_basic_units_ = total_basic_units_ - n_basic_unit_;
        if (coded_basic_units_ > 0) {
            p_ave_hdr1_ = (int)((double)(p_ave_hdr1_ * (coded_basic_units_ - 1) + bu_hdr_bits_) / coded_basic_units_ + 0.5);
            if (p_ave_hdr3_ == 0) p_ave_hdr2_ = p_ave_hdr1_;
            else
                p_ave_hdr2_ = (int)((double)(p_ave_hdr1_ * coded_basic_units_ + p_ave_hdr3_ * n_basic_unit_) / total_basic_units_ + 0.5);
        }
        bu_curr_mad_[total_basic_units_ - 1 - n_basic_unit_] = curr_frame_mad_;
        nc = n_basic_unit_ != 0 ? coded_p_frames_ * total_basic_units_ + coded_basic_units_
                                : (coded_p_frames_ - 1) * total_basic_units_ + coded_basic_units_;
    }
    const bool mad_model = nc > 1;
    p_pre_header_ = hdr_bits_;
    for (int i = kHist - 2; i > 0; --i) {
        p_rg_qp_[i] = p_rg_qp_[i - 1];
        rg_qp_[i] = p_rg_qp_[i];
        p_rg_rp_[i] = p_rg_rp_[i - 1];
        rg_rp_[i] = p_rg_rp_[i];
    }
    p_rg_qp_[0] = qp_to_qstep(qc_);
    p_rg_rp_[0] = (frame_level_ ? tex_bits_ : bu_tex_bits_) * 1.0 / curr_frame_mad_;
    rg_qp_[0] = p_rg_qp_[0];
    rg_rp_[0] = p_rg_rp_[0];
    x1_ = p_x1_;
    x2_ = p_x2_;
    int n = curr_frame_mad_ > prev_frame_mad_ ? (int)(prev_frame_mad_ / curr_frame_mad_ * (kHist - 1))
                                               : (int)(curr_frame_mad_ / prev_frame_mad_ * (kHist - 1));
    n = clip3(1, nc, n);
    n = std::min(n, rd_window_ + 1);
    n = std::min(n, kHist - 1);
    rd_window_ = n;
    bool rej[kHist] = {false};
    estimate_rd(n, rej);
    n = rd_window_;
    double err[kHist], sq = 0.0;
    for (int i = 0; i < n; ++i) {
        err[i] = x1_ / rg_qp_[i] + x2_ / (rg_qp_[i] * rg_qp_[i]) - rg_rp_[i];
        sq += err[i] * err[i];
    }
    const double thr = n == 2 ? 0 : sqrt(sq / n);
    for (int i = 0; i < n; ++i)
        if (fabs(err[i]) > thr) rej[i] = true;
    rej[0] = false;
    estimate_rd(n, rej);
    if (mad_model) update_mad_model();
    else p_picture_mad_[0] = curr_frame_mad_;
}

void RateControl::end_picture(bool idr, const RcPictureStats& st, bool gop_end)
{
    const bool p_slice = !idr;
    // per-macroblock and slice-header accumulation (rc.c:423-443, 2024-2045)
    hdr_bits_ += st.header_bits;
    tex_bits_ += st.texture_bits;
    frame_mad_sum_ = st.mad_sum;
    if (!frame_level_) {
        bu_mad_sum_ += st.mad_sum;
        bu_hdr_bits_ += st.header_bits;
        bu_tex_bits_ += st.texture_bits;
    }
    // _rc_update_pict_frame, rc.c:2073-2128 (mode 0)
    int complexity = 0;
    if (frame_level_) complexity = (int)floor(st.nbits * qc_ + 0.5);
    else if (p_slice) complexity = (int)floor(st.nbits * ((double)total_frame_qp_ / (double)total_basic_units_) + 0.5);
    if (p_slice) {  // _updatePparams, rc.c:2170-2178
        xp_ = complexity;
        np_--;
        wp_ = xp_;
        coded_p_frames_++;
        n_p_pictures_++;
    }
    // _rc_update_pict, rc.c:2047-2066
    const int delta = st.nbits - (int)floor(bit_rate_ / frame_rate_ + 0.5F);
    remaining_bits_ -= st.nbits;
    buffer_fullness_ += delta;
    lower_ -= delta;
    upper1_ -= delta;
    upper2_ = (int)(kOmega * upper1_);
    if (p_slice) update_model();
    number_++;
    curr_frm_idx_++;
    if (gop_end) {
        number_ = 0;
        curr_frm_idx_ = 0;
    }
}

}  // namespace hl
