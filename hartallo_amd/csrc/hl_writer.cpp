// hl_writer.cpp -- see hl_writer.h.
#include "hl_writer.h"

#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <thread>
#include <vector>

#include "hl_prims.h"

namespace hl {

BitWriter::BitWriter(uint8_t* buf, size_t cap, int64_t limit)
    : buf_(buf), cap_(cap), limit_(limit < 0 ? (int64_t)cap - 1 : limit), nbits_(0), overflow_(false)
{
}

void BitWriter::u(uint32_t v, int n)
{
    if (n <= 0) return;
    // fast path: the whole write lies below the limit and inside the buffer;
    // up to one byte per step
    const int64_t last = (nbits_ + n - 1) >> 3;
    if (last <= limit_ && (uint64_t)last < (uint64_t)cap_) {
        while (n > 0) {
            const int room = 8 - (int)(nbits_ & 7);
            const int take = n < room ? n : room;
            const uint32_t chunk = (v >> (n - take)) & ((1u << take) - 1u);
            const int shift = room - take;
            uint8_t& b = buf_[nbits_ >> 3];
            const uint32_t mask = ((1u << take) - 1u) << shift;
            b = (uint8_t)((b & ~mask) | (chunk << shift));
            nbits_ += take;
            n -= take;
        }
        return;
    }
    for (int i = n - 1; i >= 0; --i) {
        if ((nbits_ >> 3) > limit_) {
            overflow_ = true;
            return;
        }
        const size_t byte = (size_t)(nbits_ >> 3);
        const int bit = 7 - (int)(nbits_ & 7);
        if (byte < cap_) {
            if ((v >> i) & 1u) buf_[byte] |= (uint8_t)(1u << bit);
            else buf_[byte] &= (uint8_t)~(1u << bit);
        }
        else {
            overflow_ = true;
        }
        ++nbits_;
    }
}

void BitWriter::ue(uint32_t v)
{
    int lz = 0;
    while ((1ull << (lz + 1)) <= (uint64_t)v + 1) ++lz;
    u(0, lz);
    u(v + 1, lz + 1);
}

void BitWriter::se(int32_t v) { ue(v <= 0 ? (uint32_t)(-(int64_t)v) << 1 : ((uint32_t)v << 1) - 1); }

void BitWriter::trailing()
{
    const bool aligned = (nbits_ & 7) == 0;
    if (!aligned || !(buf_[(nbits_ >> 3) - 1] & 1)) {
        const int left = 8 - (int)(nbits_ & 7);
        u(1u << (left - 1), left);
    }
}

// ---------------------------------------------------------------------------
// CAVLC level table, generated exactly like cavlc.c:59-103 (inclusive suffix
// bound; entries past the generated range stay {0,0,0}).
// ---------------------------------------------------------------------------
namespace {

constexpr int kMaxLevelCode = 62545;
struct LevelCode {
    uint16_t prefix, size;
    uint32_t suffix;
};
std::vector<LevelCode>* g_levels = nullptr;
std::once_flag g_levels_once;

void init_levels()
{
    g_levels = new std::vector<LevelCode>(7 * (kMaxLevelCode + 1), LevelCode{0, 0, 0});
    for (int lp = 0; lp <= 15; ++lp)
        for (int sl = 0; sl <= 6; ++sl) {
            int size = sl;
            if (lp == 14 && sl == 0) size = 4;
            else if (lp >= 15) size = lp - 3;
            for (int ls = 0; ls <= (1 << size); ++ls) {
                int lc = (lp < 15 ? lp : 15) << sl;
                if (sl > 0 || lp >= 14) lc += ls;
                if (lp >= 15 && sl == 0) lc += 15;
                (*g_levels)[(size_t)sl * (kMaxLevelCode + 1) + lc] = LevelCode{(uint16_t)lp, (uint16_t)size, (uint32_t)ls};
            }
        }
}

const LevelCode& level_code(int sl, int lc)
{
    std::call_once(g_levels_once, init_levels);
    if (lc > kMaxLevelCode) lc = kMaxLevelCode;
    return (*g_levels)[(size_t)sl * (kMaxLevelCode + 1) + lc];
}

// me(v) coded_block_pattern -> codeNum, Table 9-4 [cbp][0 = Intra_4x4, 1 = Inter]
constexpr uint8_t kCbpCode[48][2] = {
    {3, 0},   {29, 2},  {30, 3},  {17, 7},  {31, 4},  {18, 8},  {37, 17}, {8, 13},  {32, 5},  {38, 18}, {19, 9},  {9, 14},
    {20, 10}, {10, 15}, {11, 16}, {2, 11},  {16, 1},  {33, 32}, {34, 33}, {21, 36}, {35, 34}, {22, 37}, {39, 44}, {4, 40},
    {36, 35}, {40, 45}, {23, 38}, {5, 41},  {24, 39}, {6, 42},  {7, 43},  {1, 19},  {41, 6},  {42, 24}, {43, 25}, {25, 20},
    {44, 26}, {26, 21}, {46, 46}, {12, 28}, {45, 27}, {47, 47}, {27, 22}, {13, 29}, {28, 23}, {14, 30}, {15, 31}, {0, 12}};

// residual_block_cavlc, residual.c:587-901 (write path)
template <typename T>
void write_block(BitWriter& bw, const T* coeffLevel, int endIdx, int maxNumCoef, int nC)
{
    static constexpr int32_t kThr[7] = {0, 3, 6, 12, 24, 48, 1 << 15};
    int nz[16], run_before[16] = {0};
    int tc = 0, t1 = 0, total_zeros = 0, k = -1;
    bool countT1 = true, countTZ = false;
    for (int j = 0; j < maxNumCoef; ++j) {
        const int c = coeffLevel[maxNumCoef - 1 - j];
        if (c) {
            nz[tc++] = c;
            countTZ = true;
            ++k;
            if (countT1) {
                if (c == 1 || c == -1) {
                    ++t1;
                    countT1 = t1 < 3;
                }
                else {
                    countT1 = false;
                }
            }
        }
        else if (countTZ) {
            ++run_before[k];
        }
        if (countTZ && c == 0) ++total_zeros;
    }
    if (nC >= 0) {
        if (nC >= 8) bw.u(tc ? (uint32_t)(((tc - 1) << 2) | t1) : 3u, 6);
        else {
            const int vlc = nC < 2 ? 0 : (nC < 4 ? 1 : 2);
            bw.u(kTokCode[vlc][t1][tc], kTokLen[vlc][t1][tc]);
        }
    }
    else {
        bw.u(kTokCdcCode[t1][tc], kTokCdcLen[t1][tc]);
    }
    if (tc == 0) return;
    int suffixLength = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int j = 0; j < tc; ++j) {
        if (j < t1) {
            bw.u1((uint32_t)((1 - nz[j]) >> 1));
            continue;
        }
        int lc = nz[j] >= 0 ? nz[j] * 2 - 2 : -(nz[j] * 2) - 1;
        if (j == t1 && t1 < 3 && lc >= 2) lc -= 2;
        const LevelCode& L = level_code(suffixLength, lc);
        if (L.prefix > 0) bw.u(0, L.prefix);
        bw.u1(1);
        if (L.size) bw.u(L.suffix, L.size);
        if (suffixLength == 0) suffixLength = 1;
        if (iabs(nz[j]) > kThr[suffixLength]) ++suffixLength;
    }
    int zerosLeft = 0;
    if (tc < endIdx + 1) {
        if (nC >= 0) bw.u(kTzCode[tc - 1][total_zeros], kTzLen[tc - 1][total_zeros]);
        else bw.u(kTzCdcCode[tc - 1][total_zeros], kTzCdcLen[tc - 1][total_zeros]);
        zerosLeft = total_zeros;
    }
    for (k = 0; k < tc - 1 && zerosLeft > 0; ++k) {
        const int row = zerosLeft <= 6 ? zerosLeft - 1 : 6;
        bw.u(kRbCode[row][run_before[k]], kRbLen[row][run_before[k]]);
        zerosLeft -= run_before[k];
    }
}

// levels in the reference's guess order (utils.c:14-58); the position is
// also the level's zero-based index into the Table A-1 arrays
// (HL_CODEC_264_LEVEL_TO_ZERO_BASED_INDEX, tables.h:151: 10 -> 0, 9 -> 1, ...)
const int kLevels[16][3] = {{10, 128, 96},   {9, 128, 96},    {11, 176, 144},  {12, 320, 240},  {13, 352, 288},  {20, 352, 288},
                            {21, 352, 480},  {22, 352, 480},  {30, 720, 480},  {31, 1280, 720}, {32, 1280, 720}, {40, 2048, 1024},
                            {41, 2048, 1024}, {42, 2048, 1080}, {50, 2560, 1920}, {51, 3840, 2160}};

int guess_level_index(int w, int h)
{
    for (int i = 0; i < 16; ++i)
        if (kLevels[i][1] >= w && kLevels[i][2] >= h) return i;
    return 15;  // 51
}

int guess_level(int w, int h) { return kLevels[guess_level_index(w, h)][0]; }  // utils.c:14-58

size_t put_nal(uint8_t* out, size_t cap, const uint8_t* rbsp, size_t n)
{
    if (cap < n + 3) return 0;
    out[0] = 0;
    out[1] = 0;
    out[2] = 1;
    memcpy(out + 3, rbsp, n);
    return n + 3;
}

}  // namespace

int sps_max_num_ref_frames(int width, int height, int max_ref_frame)
{
    static const int kMaxDpbMbs[16] = {396, 396, 900, 2376, 2376, 2376, 4752, 8100, 8100, 18000, 20480, 32768, 32768, 34816, 110400, 184320};
    const int dpb = kMaxDpbMbs[guess_level_index(width, height)] / ((width / 16) * (height / 16));
    return dpb < max_ref_frame ? dpb : max_ref_frame;
}

int level_code_bits(int suffix_length, int code)
{
    const LevelCode& L = level_code(suffix_length, code);
    return L.prefix + 1 + L.size;
}

size_t write_stream_headers(const StreamParams& p, uint8_t* out, size_t cap)
{
    uint8_t buf[64];
    size_t n = 0;
    const int nref = sps_max_num_ref_frames(p.width, p.height, p.max_ref_frame);
    {
        memset(buf, 0, sizeof(buf));
        BitWriter bw(buf, sizeof(buf));
        bw.u(0, 1);
        bw.u(1, 2);
        bw.u(7, 5);     // nal_unit_type SPS
        bw.u(66, 8);    // profile_idc Baseline
        bw.u1(1);       // constraint_set0..2 = 1 (sps.c:555-560)
        bw.u1(1);
        bw.u1(1);
        bw.u1(0);
        bw.u1(0);
        bw.u1(0);
        bw.u(0, 2);
        bw.u((uint32_t)guess_level(p.width, p.height), 8);
        bw.ue(0);  // seq_parameter_set_id
        bw.ue(4);  // log2_max_frame_num_minus4
        bw.ue(2);  // pic_order_cnt_type
        bw.ue((uint32_t)nref);  // max_num_ref_frames (sps.c:620-636)
        bw.u1(0);
        bw.ue((uint32_t)(p.width / 16 - 1));
        bw.ue((uint32_t)(p.height / 16 - 1));
        bw.u1(1);  // frame_mbs_only_flag
        bw.u1(0);  // direct_8x8_inference_flag
        bw.u1(0);  // frame_cropping_flag
        bw.u1(0);  // vui_parameters_present_flag
        bw.trailing();
        n += put_nal(out + n, cap - n, buf, bw.bytes());
    }
    {
        memset(buf, 0, sizeof(buf));
        BitWriter bw(buf, sizeof(buf));
        bw.u(0, 1);
        bw.u(1, 2);
        bw.u(8, 5);  // nal_unit_type PPS
        bw.ue(0);
        bw.ue(0);
        bw.u1(0);    // entropy_coding_mode_flag (CAVLC)
        bw.u1(0);
        bw.ue(0);    // num_slice_groups_minus1
        bw.ue((uint32_t)(nref > 0 ? nref - 1 : 0));  // num_ref_idx_l0_default_active_minus1 (pps.c:291)
        bw.ue(0);
        bw.u1(0);
        bw.u(0, 2);
        bw.se(p.qp - 26);
        bw.se(0);
        bw.se(0);
        bw.u1(1);  // deblocking_filter_control_present_flag
        bw.u1(0);
        bw.u1(0);
        bw.trailing();
        n += put_nal(out + n, cap - n, buf, bw.bytes());
    }
    return n;
}

size_t slice_scratch_bytes(const StreamParams& p)
{
    const size_t nmb = (size_t)(p.width / 16) * (p.height / 16);
    return (size_t)p.width * p.height * 3 / 2 + 4096 + (nmb << 8);
}

size_t write_slice(const StreamParams& p, const SliceState& s, const MbRecord* recs, uint8_t* scratch, uint8_t* out, size_t cap,
                   SliceBits* bits, const RowGate* gate)
{
    static const int16_t kZeros[16] = {0};
    const size_t scap = slice_scratch_bytes(p);
    const int nmb = (p.width / 16) * (p.height / 16);
    // the reference builds the slice NAL in a (mb_count << 8) + 4096 byte
    // buffer (encode.c:192) and drops writes past its end
    const size_t esd_size = ((size_t)nmb << 8) + 4096;
    memset(scratch, 0, scap);
    BitWriter bw(scratch, scap, (int64_t)esd_size);
    // slice header, slice.c:660-900
    bw.u(0, 1);
    bw.u(1, 2);
    bw.u(s.idr ? 5 : 1, 5);
    bw.ue(0);                // first_mb_in_slice
    bw.ue(s.idr ? 2 : 0);    // slice_type I / P
    bw.ue(0);                // pic_parameter_set_id
    bw.u((uint32_t)s.frame_num & 0xFF, 8);
    if (s.idr) bw.ue((uint32_t)s.idr_pic_id);
    if (!s.idr) {
        bw.u1(1);            // num_ref_idx_active_override_flag
        bw.ue(0);
        bw.u1(0);            // ref_pic_list_modification_flag_l0
        bw.u1(0);            // adaptive_ref_pic_marking_mode_flag
    }
    else {
        bw.u1(0);            // no_output_of_prior_pics_flag
        bw.u1(0);            // long_term_reference_flag
    }
    bw.se(s.qp - p.qp);      // slice_qp_delta (encode.c:257, 274)
    bw.ue(p.deblock ? 0 : 1);
    if (p.deblock) {
        bw.se(0);
        bw.se(0);
    }
    // slice_data, mb.c:543-892
    int skip_run = 0;
    int64_t texture = 0;
    const int mbw = p.width / 16;
    for (int a = 0; a < nmb; ++a) {
        if (gate && a % mbw == 0 && !gate->wait(gate->ctx, a / mbw)) return 0;
        const MbRecord& m = recs[a];
        if (!s.idr) {
            if (m.e_type == ET_PSKIP) {
                ++skip_run;
                if (a == nmb - 1) bw.ue((uint32_t)skip_run);
                continue;
            }
            bw.ue((uint32_t)skip_run);
            skip_run = 0;
        }
        bw.ue((uint32_t)m.mb_type);
        const bool intra = (m.flags & FL_INTRA) != 0;
        if (m.e_type != ET_I_NXN && m.pm0 != PM_I16 && m.num_part == 4 && !intra) {
            for (int pi = 0; pi < 4; ++pi) bw.ue((uint32_t)m.sub_mb_type[pi]);
            for (int pi = 0; pi < 4; ++pi)
                for (int spi = 0; spi < m.num_sub[pi]; ++spi) {
                    bw.se(m.mvd[pi][spi][0]);
                    bw.se(m.mvd[pi][spi][1]);
                }
        }
        else if (m.pm0 == PM_I4 || m.pm0 == PM_I16) {
            if (m.pm0 == PM_I4)
                for (int b = 0; b < 16; ++b) {
                    bw.u1((uint32_t)m.prev_flag[b]);
                    if (!m.prev_flag[b]) bw.u((uint32_t)m.rem_mode[b], 3);
                }
            bw.ue((uint32_t)m.chroma_mode);
        }
        else {
            for (int pi = 0; pi < m.num_part; ++pi) {
                bw.se(m.mvd[pi][0][0]);
                bw.se(m.mvd[pi][0][1]);
            }
        }
        if (m.pm0 != PM_I16) bw.ue(kCbpCode[m.cbp][m.pm0 == PM_I4 ? 0 : 1]);
        if (m.cbp_l > 0 || m.cbp_c > 0 || m.pm0 == PM_I16) {
            bw.se(0);  // mb_qp_delta
            const int64_t t0 = bw.bits();
            if (m.pm0 == PM_I16) write_block(bw, m.i16dc, 15, 16, m.nc_dc);
            for (int i8 = 0; i8 < 4; ++i8)
                for (int i4 = 0; i4 < 4; ++i4)
                    if (m.cbp_l & (1 << i8)) {
                        const int blk = i8 * 4 + i4;
                        if (m.pm0 == PM_I16) write_block(bw, m.luma[blk], 14, 15, m.nc_luma[blk]);
                        else write_block(bw, m.luma[blk], 15, 16, m.nc_luma[blk]);
                    }
            if (m.cbp_c & 3)
                for (int c = 0; c < 2; ++c) write_block(bw, m.cbp_cdc[c] ? m.cdc[c] : kZeros, 3, 4, -1);
            for (int c = 0; c < 2; ++c)
                for (int i4 = 0; i4 < 4; ++i4)
                    if (m.cbp_c & 2) write_block(bw, (m.cbp_cac[c] & (1 << i4)) ? m.cac[c][i4] : kZeros, 14, 15, m.nc_cac[c][i4]);
            texture += bw.bits() - t0;
        }
    }
    if (bits) {
        bits->texture_bits = (int32_t)texture;
        bits->header_bits = (int32_t)(bw.bits() - texture);
    }
    bw.trailing();
    size_t n = bw.bytes();
    // emulation prevention, rbsp.c:609-632: only 00 00 01 is escaped and the
    // caller keeps the unescaped length (encode.c:443-444)
    {
        size_t zeros = 0, len = n;
        for (size_t i = 0; i < len; ++i) {
            if (zeros == 2) {
                if (scratch[i] == 0x01) {
                    if (len + 1 >= esd_size) return 0;  // HL_ERROR_TOOSHORT, rbsp.c:617-620
                    memmove(&scratch[i + 1], &scratch[i], len - i + 1);
                    len++;
                    scratch[i++] = 0x03;
                }
                zeros = 0;
            }
            zeros = scratch[i] ? 0 : zeros + 1;
        }
    }
    return put_nal(out, cap, scratch, n);
}

// ---------------------------------------------------------------------------
// Spatial SVC
// ---------------------------------------------------------------------------
namespace {

// pps.c:265-400 as write_stream_headers writes it, for pic_parameter_set_id =
// seq_parameter_set_id = id (hl_codec_264.c:607-617)
size_t put_pps(int id, int qp, int nref, uint8_t* out, size_t cap)
{
    uint8_t buf[64];
    memset(buf, 0, sizeof(buf));
    BitWriter bw(buf, sizeof(buf));
    bw.u(0, 1);
    bw.u(1, 2);
    bw.u(8, 5);
    bw.ue((uint32_t)id);
    bw.ue((uint32_t)id);
    bw.u1(0);
    bw.u1(0);
    bw.ue(0);
    bw.ue((uint32_t)(nref > 0 ? nref - 1 : 0));  // num_ref_idx_l0_default_active_minus1 of SPS id (pps.c:291)
    bw.ue(0);
    bw.u1(0);
    bw.u(0, 2);
    bw.se(qp - 26);
    bw.se(0);
    bw.se(0);
    bw.u1(1);
    bw.u1(0);
    bw.u1(0);
    bw.trailing();
    return put_nal(out, cap, buf, bw.bytes());
}

// subset_seq_parameter_set_rbsp of an enhancement layer (sps.c:535-860):
// Scalable Baseline (83) with constraint_set0 only, the High-profile fields
// profile 83 carries, and the SVC extension the encoder sets (sps.c:799-851)
size_t put_subset_sps(int id, int w, int h, int nref, uint8_t* out, size_t cap)
{
    uint8_t buf[64];
    memset(buf, 0, sizeof(buf));
    BitWriter bw(buf, sizeof(buf));
    bw.u(0, 1);
    bw.u(1, 2);
    bw.u(15, 5);    // nal_unit_type subset SPS
    bw.u(83, 8);    // profile_idc Scalable Baseline
    bw.u1(1);       // constraint_set0_flag
    bw.u(0, 7);     // constraint_set1..5, reserved_zero_2bits
    bw.u((uint32_t)guess_level(w, h), 8);
    bw.ue((uint32_t)id);
    bw.ue(1);       // chroma_format_idc 4:2:0
    bw.ue(0);       // bit_depth_luma_minus8
    bw.ue(0);       // bit_depth_chroma_minus8
    bw.u1(0);       // qpprime_y_zero_transform_bypass_flag
    bw.u1(0);       // seq_scaling_matrix_present_flag
    bw.ue(4);       // log2_max_frame_num_minus4
    bw.ue(2);       // pic_order_cnt_type
    bw.ue((uint32_t)nref);  // max_num_ref_frames (sps.c:620-636)
    bw.u1(0);
    bw.ue((uint32_t)(w / 16 - 1));
    bw.ue((uint32_t)(h / 16 - 1));
    bw.u1(1);       // frame_mbs_only_flag
    bw.u1(0);       // direct_8x8_inference_flag
    bw.u1(0);       // frame_cropping_flag
    bw.u1(0);       // vui_parameters_present_flag
    // seq_parameter_set_svc_extension() (G.7.3.2.1.4)
    bw.u1(1);       // inter_layer_deblocking_filter_control_present_flag
    bw.u(0, 2);     // extended_spatial_scalability_idc
    bw.u1(1);       // chroma_phase_x_plus1_flag
    bw.u(1, 2);     // chroma_phase_y_plus1
    bw.u1(0);       // seq_tcoeff_level_prediction_flag
    bw.u1(0);       // slice_header_restriction_flag
    bw.u1(0);       // svc_vui_parameters_present_flag
    bw.u1(0);       // additional_extension2_flag
    bw.trailing();
    return put_nal(out, cap, buf, bw.bytes());
}

// TotalCoeff of the blocks the writer codes, as the reference leaves them on
// the macroblock objects during the final write (residual.c:796-806); blocks
// of uncoded 8x8 / chroma-AC groups count as 0 (utils.h:10-20)
int tc_luma(const MbRecord& m, int blk)
{
    if (!(m.cbp_l & (1 << (blk >> 2)))) return 0;
    int k = 0;
    for (int i = 0; i < 16; ++i) k += m.luma[blk][i] != 0;
    return k;
}
int tc_cac(const MbRecord& m, int comp, int b)
{
    if (!(m.cbp_c & 2) || !(m.cbp_cac[comp] & (1 << b))) return 0;
    int k = 0;
    for (int i = 0; i < 15; ++i) k += m.cac[comp][b][i] != 0;
    return k;
}

}  // namespace

int stream_level_idc(int width, int height) { return guess_level(width, height); }

size_t write_svc_headers(const StreamParams& base, const int32_t* widths, const int32_t* heights, int n, uint8_t* out, size_t cap)
{
    // SPS 0 and PPS 0 are write_stream_headers' two NAL units
    uint8_t avc[256];
    const StreamParams b0{widths[0], heights[0], base.qp, base.deblock, base.max_ref_frame};
    const size_t na = write_stream_headers(b0, avc, sizeof(avc));
    size_t sps0 = 3;
    while (sps0 + 2 < na && !(avc[sps0] == 0 && avc[sps0 + 1] == 0 && avc[sps0 + 2] == 1)) ++sps0;
    size_t k = 0;
    if (cap < na) return 0;
    memcpy(out, avc, sps0);
    k = sps0;
    for (int l = 1; l < n; ++l) {
        const size_t m = put_subset_sps(l, widths[l], heights[l], sps_max_num_ref_frames(widths[l], heights[l], base.max_ref_frame),
                                        out + k, cap - k);
        if (!m) return 0;
        k += m;
    }
    for (int l = 0; l < n; ++l) {
        const size_t m = put_pps(l, base.qp, sps_max_num_ref_frames(widths[l], heights[l], base.max_ref_frame), out + k, cap - k);
        if (!m) return 0;
        k += m;
    }
    return k;
}

size_t write_prefix_nal(bool idr, uint8_t* out)
{
    out[0] = 0x2E;                          // nal_ref_idc 1, nal_unit_type 14
    out[1] = (uint8_t)(0x80 | (idr ? 0x40 : 0));  // svc_extension_flag, idr_flag, priority_id 0
    out[2] = 0x80;                          // no_inter_layer_pred_flag 1, dependency_id 0, quality_id 0
    out[3] = 0x07;                          // temporal_id 0, use_ref_base 0, discardable 0, output 1, reserved 3
    out[4] = 32;                            // store_ref_base_pic_flag 0, additional flag 0, trailing (encode.c:355)
    return 5;
}

namespace {
// NAL header + nal_unit_header_svc_extension (encode.c:296-328) and
// slice_header_in_scalable_extension (slice.c:722-988)
void svc_slice_header(BitWriter& bw, const StreamParams& p, const SvcSliceState& s)
{
    bw.u(0, 1);
    bw.u(1, 2);
    bw.u(20, 5);
    bw.u1(1);                           // svc_extension_flag
    bw.u1((uint32_t)s.idr);             // idr_flag
    bw.u(0, 6);                         // priority_id
    bw.u1(0);                           // no_inter_layer_pred_flag
    bw.u((uint32_t)s.dependency_id, 3);
    bw.u(0, 4);                         // quality_id
    bw.u(0, 3);                         // temporal_id
    bw.u1(0);                           // use_ref_base_pic_flag
    bw.u1(0);                           // discardable_flag
    bw.u1(1);                           // output_flag
    bw.u(3, 2);                         // reserved_three_2bits
    bw.ue(0);                           // first_mb_in_slice
    bw.ue(s.idr ? 2 : 0);               // slice_type EI / EP
    bw.ue((uint32_t)s.dependency_id);   // pic_parameter_set_id
    bw.u((uint32_t)s.frame_num & 0xFF, 8);
    if (s.idr) bw.ue((uint32_t)s.idr_pic_id);
    if (!s.idr) {
        bw.u1(1);                       // num_ref_idx_active_override_flag
        bw.ue(0);
        bw.u1(0);                       // ref_pic_list_modification_flag_l0
        bw.u1(0);                       // adaptive_ref_pic_marking_mode_flag
    }
    else {
        bw.u1(0);                       // no_output_of_prior_pics_flag
        bw.u1(0);                       // long_term_reference_flag
    }
    bw.u1(0);                           // store_ref_base_pic_flag
    bw.se(s.qp - p.qp);                 // slice_qp_delta
    bw.ue(p.deblock ? 0 : 1);
    if (p.deblock) {
        bw.se(0);
        bw.se(0);
    }
    bw.ue((uint32_t)((s.dependency_id - 1) << 4));  // ref_layer_dq_id
    bw.ue(0);                           // disable_inter_layer_deblocking_filter_idc (deblock_inter_layer_flag = 1)
    bw.se(0);
    bw.se(0);
    bw.u1(0);                           // constrained_intra_resampling_flag
    bw.u1(0);                           // slice_skip_flag
    bw.u1(1);                           // adaptive_base_mode_flag
    bw.u1(1);                           // adaptive_motion_prediction_flag
    bw.u1(1);                           // adaptive_residual_prediction_flag
    bw.u(0, 4);                         // scan_idx_start
    bw.u(15, 4);                        // scan_idx_end
}

// trailing bits, emulation prevention (only 00 00 01, the unescaped length
// kept: rbsp.c:609-632, encode.c:443-444) and the start code
size_t svc_slice_finish(BitWriter& bw, uint8_t* scratch, size_t esd_size, uint8_t* out, size_t cap)
{
    bw.trailing();
    size_t n = bw.bytes();
    size_t zeros = 0, len = n;
    for (size_t i = 0; i < len; ++i) {
        if (zeros == 2) {
            if (scratch[i] == 0x01) {
                if (len + 1 >= esd_size) return 0;
                memmove(&scratch[i + 1], &scratch[i], len - i + 1);
                len++;
                scratch[i++] = 0x03;
            }
            zeros = 0;
        }
        zeros = scratch[i] ? 0 : zeros + 1;
    }
    return put_nal(out, cap, scratch, n);
}
}  // namespace

size_t write_svc_slice(const StreamParams& p, const SvcSliceState& s, const MbRecord* recs, uint8_t* scratch, uint8_t* out, size_t cap,
                       int threads)
{
    const size_t scap = slice_scratch_bytes(p);
    const int nmb = (p.width / 16) * (p.height / 16);
    const size_t esd_size = ((size_t)nmb << 8) + 4096;
    BitWriter bw(scratch, scap, (int64_t)esd_size);
    svc_slice_header(bw, p, s);
    write_svc_mbs(bw, p, s, recs, 0, nmb, threads);
    return svc_slice_finish(bw, scratch, esd_size, out, cap);
}

size_t write_svc_slice_bits(const StreamParams& p, const SvcSliceState& s, const uint32_t* words, int64_t data_bits, uint8_t* scratch,
                            uint8_t* out, size_t cap)
{
    const size_t scap = slice_scratch_bytes(p);
    const int nmb = (p.width / 16) * (p.height / 16);
    const size_t esd_size = ((size_t)nmb << 8) + 4096;
    BitWriter bw(scratch, scap, (int64_t)esd_size);
    svc_slice_header(bw, p, s);
    const int64_t full = data_bits >> 5;
    for (int64_t i = 0; i < full; ++i) bw.u(words[i], 32);
    if (data_bits & 31) bw.u(words[full] >> (32 - (int)(data_bits & 31)), (int)(data_bits & 31));
    return svc_slice_finish(bw, scratch, esd_size, out, cap);
}

namespace {
// macroblock_layer_in_scalable_extension of macroblocks [a0, a1) (mb.c:543-892)
void write_svc_mb_range(BitWriter& bw, const StreamParams& p, const SvcSliceState& s, const MbRecord* recs, int a0, int a1)
{
    static const int16_t kZeros[16] = {0};
    const int mbw = p.width / 16;
    for (int a = a0; a < a1; ++a) {
        const MbRecord& m = recs[a];
        const int mbx = a % mbw, mby = a / mbw;
        if (!s.idr) bw.ue(0);           // mb_skip_run (no skipped macroblocks)
        bw.u1(1);                       // base_mode_flag
        if (!s.idr) bw.u1(0);           // residual_prediction_flag
        bw.ue(kCbpCode[m.cbp][1]);      // coded_block_pattern, inter mapping (MbPartPredMode is not Intra_4x4)
        if (!(m.cbp_l > 0 || m.cbp_c > 0)) continue;
        bw.se(0);                       // mb_qp_delta
        for (int i8 = 0; i8 < 4; ++i8)
            for (int i4 = 0; i4 < 4; ++i4) {
                if (!(m.cbp_l & (1 << i8))) continue;
                const int blk = i8 * 4 + i4, bx = blk_x(blk), by = blk_y(blk);
                int nA = 0, nB = 0;
                bool aA = true, aB = true;
                if (bx) nA = tc_luma(m, blk_idx(bx - 4, by));
                else if (mbx) nA = tc_luma(recs[a - 1], blk_idx(12, by));
                else aA = false;
                if (by) nB = tc_luma(m, blk_idx(bx, by - 4));
                else if (mby) nB = tc_luma(recs[a - mbw], blk_idx(bx, 12));
                else aB = false;
                const int nC = aA && aB ? (nA + nB + 1) >> 1 : (aA ? nA : (aB ? nB : 0));
                write_block(bw, m.luma[blk], 15, 16, nC);
            }
        if (m.cbp_c & 3)
            for (int c = 0; c < 2; ++c) write_block(bw, m.cbp_cdc[c] ? m.cdc[c] : kZeros, 3, 4, -1);
        if (m.cbp_c & 2)
            for (int c = 0; c < 2; ++c)
                for (int i4 = 0; i4 < 4; ++i4) {
                    int nA = 0, nB = 0;
                    bool aA = true, aB = true;
                    if (i4 & 1) nA = tc_cac(m, c, i4 - 1);
                    else if (mbx) nA = tc_cac(recs[a - 1], c, i4 + 1);
                    else aA = false;
                    if (i4 & 2) nB = tc_cac(m, c, i4 - 2);
                    else if (mby) nB = tc_cac(recs[a - mbw], c, i4 + 2);
                    else aB = false;
                    const int nC = aA && aB ? (nA + nB + 1) >> 1 : (aA ? nA : (aB ? nB : 0));
                    write_block(bw, (m.cbp_cac[c] & (1 << i4)) ? m.cac[c][i4] : kZeros, 14, 15, nC);
                }
    }
}
}  // namespace

// The enhancement-layer macroblocks have no skip runs and their nC contexts
// come from the records, so ranges of macroblocks are written independently
// (one bit buffer per thread) and concatenated.
void write_svc_mbs(BitWriter& bw, const StreamParams& p, const SvcSliceState& s, const MbRecord* recs, int a0, int a1, int threads)
{
    const int n = a1 - a0;
    if (threads <= 1 || n < 64 * threads) {
        write_svc_mb_range(bw, p, s, recs, a0, a1);
        return;
    }
    struct Part {
        std::vector<uint8_t> buf;
        int64_t bits = 0;
        bool overflow = false;
    };
    std::vector<Part> parts(threads);
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            const int b0 = a0 + (int)((int64_t)n * t / threads), b1 = a0 + (int)((int64_t)n * (t + 1) / threads);
            Part& P = parts[t];
            P.buf.assign(((size_t)(b1 - b0) << 9) + 4096, 0);
            BitWriter w(P.buf.data(), P.buf.size());
            write_svc_mb_range(w, p, s, recs, b0, b1);
            P.bits = w.bits();
            P.overflow = w.overflow();
        });
    for (auto& x : th) x.join();
    for (const Part& P : parts) {
        if (P.overflow) {  // a range outgrew its buffer: write serially
            write_svc_mb_range(bw, p, s, recs, a0, a1);
            return;
        }
    }
    for (const Part& P : parts) {
        const int64_t full = P.bits >> 3;
        for (int64_t i = 0; i < full; ++i) bw.u(P.buf[i], 8);
        const int rest = (int)(P.bits & 7);
        if (rest) bw.u((uint32_t)P.buf[full] >> (8 - rest), rest);
    }
}

}  // namespace hl
