// hl_writer.h -- host-side H.264 Baseline bitstream writer of the encoder:
// SPS/PPS (sps.c:535-800, pps.c:265-400), slice header (slice.c:660-900),
// macroblock_layer() + CAVLC residual (mb.c:543-892, residual.c:587-1094),
// rbsp trailing bits and emulation prevention (rbsp.c:162-170, 609-632).
//
// The GPU hands over one MbRecord per macroblock with every syntax value and
// every nC context already resolved, so this pass is serialisation only.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "hl_types.h"

namespace hl {

struct StreamParams {
    int32_t width, height, qp, deblock;
    int32_t max_ref_frame = 1;  // hl_codec_t.max_ref_frame (hl_codec.c:36 default 1): SPS/PPS only
};

// max_num_ref_frames the reference writes in a SPS of this picture size:
// min(MaxDpbMbs / PicSizeInMbs, max_ref_frame) (sps.c:620-636, the level
// from utils.c:14-58, MaxDpbMbs from tables.h:143-151)
int sps_max_num_ref_frames(int width, int height, int max_ref_frame);

class BitWriter {
public:
    // limit: last writable byte index; bits beyond it are dropped like the
    // reference's end-of-buffer handling (bits.h:236-246, 612-626); -1 = cap
    BitWriter(uint8_t* buf, size_t cap, int64_t limit = -1);
    void u(uint32_t v, int n);
    void u1(uint32_t v) { u(v & 1u, 1); }
    void ue(uint32_t v);
    void se(int32_t v);
    void trailing();  // rbsp_trailing_bits with the reference's aligned-stream quirk
    size_t bytes() const { return (size_t)((nbits_ + 7) >> 3); }
    int64_t bits() const { return nbits_; }
    bool overflow() const { return overflow_; }

private:
    uint8_t* buf_;
    size_t cap_;
    int64_t limit_;
    int64_t nbits_;
    bool overflow_;
};

// Writes the 00 00 01-prefixed SPS and PPS NAL units; returns bytes written.
// The PPS's num_ref_idx_l0_default_active_minus1 follows the SPS's
// max_num_ref_frames (pps.c:291); P slices still override it to one active
// reference (slice.c:289, encode.c:269).
size_t write_stream_headers(const StreamParams& p, uint8_t* out, size_t cap);

struct SliceState {
    int32_t idr, frame_num, idr_pic_id;
    int32_t qp;  // SliceQPY (rate control may move it off the PPS value; slice_qp_delta = qp - p.qp)
};

// Bit counts of a written slice as the reference's rate control takes them
// (slice.c:994-995, mb.c:580-886): header = slice header (NAL header byte
// included) + every macroblock's header syntax, texture = residual().
struct SliceBits {
    int32_t header_bits, texture_bits;
};

// Writes "00 00 01" + one escaped slice NAL for the frame's MB records.
// scratch must hold at least slice_scratch_bytes(); returns bytes written to
// out, or 0 when out is too small or the reference would fail the frame with
// HL_ERROR_TOOSHORT (an escape that does not fit its slice buffer).
size_t slice_scratch_bytes(const StreamParams& p);

// Bits of one level code (level_prefix + 1 + level_suffix) from the table the
// writer serialises with; the GPU bit counter (hl_prims.h level_code_len)
// must agree with it for every (suffixLength, levelCode).
int level_code_bits(int suffix_length, int level_code);
// gate (optional): wait(ctx, r) returns once the records of MB row r may be
// read, or false to give up (write_slice then returns 0) -- a pipelined run
// publishes a picture's records row by row while it is still coding it.
struct RowGate {
    bool (*wait)(void* ctx, int row);
    void* ctx;
};
size_t write_slice(const StreamParams& p, const SliceState& s, const MbRecord* recs, uint8_t* scratch, uint8_t* out, size_t cap,
                   SliceBits* bits = nullptr, const RowGate* gate = nullptr);

// ---------------------------------------------------------------------------
// Spatial SVC (Annex G), the reference's encoder syntax (hl_codec_264.c:
// 577-687, encode.c:281-365, slice.c:660-1002, mb.c:543-892)
// ---------------------------------------------------------------------------
// Header NAL units once layers [0, n) exist: SPS of layer 0 (the AVC SPS),
// subset SPS of layers 1..n-1, then PPS 0..n-1, each with "00 00 01".
// level_idc the encoder writes for a picture size (utils.c:14-58)
int stream_level_idc(int width, int height);

size_t write_svc_headers(const StreamParams& base, const int32_t* widths, const int32_t* heights, int n, uint8_t* out, size_t cap);

// Prefix NAL unit of a base-layer slice (encode.c:296-365), without start
// code: 5 bytes.
size_t write_prefix_nal(bool idr, uint8_t* out);

struct SvcSliceState {
    int32_t idr, frame_num, idr_pic_id, qp;
    int32_t dependency_id;  // layer index (DQId >> 4)
};

// "00 00 01" + one escaped enhancement-layer slice NAL (type 20) of the
// layer's MB records; every macroblock has base_mode_flag = 1 and the nC of
// each residual block is derived here from the neighbours' levels
// (residual.c:587-755).  Same return convention as write_slice.
// threads > 1: ranges of macroblocks are serialised in parallel
// (write_svc_mbs) and concatenated.
size_t write_svc_slice(const StreamParams& p, const SvcSliceState& s, const MbRecord* recs, uint8_t* scratch, uint8_t* out, size_t cap,
                       int threads = 1);
void write_svc_mbs(BitWriter& bw, const StreamParams& p, const SvcSliceState& s, const MbRecord* recs, int a0, int a1, int threads);
// Same slice from its macroblock_layer() bits serialised elsewhere (the GPU,
// hl_cavlc.h): data_bits bits in big-endian 32-bit words.
size_t write_svc_slice_bits(const StreamParams& p, const SvcSliceState& s, const uint32_t* words, int64_t data_bits, uint8_t* scratch,
                            uint8_t* out, size_t cap);

}  // namespace hl
