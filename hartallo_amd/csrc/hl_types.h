// hl_types.h -- data layouts shared by the gfx950 macroblock kernels, the
// host CAVLC writer and the C-ABI.
//
// MbState is the per-address macroblock object that persists across frames,
// like the reference's pc_layer->pp_list_macroblocks[] (hl_codec_264_mb_t,
// include/hartallo/h264/hl_codec_264_mb.h:99-269).  Only the members the
// encode path reads back (from neighbours, or stale from the previous frame
// at the same address) are kept.
//
// MbRecord is what one macroblock hands to the host bitstream writer: the
// macroblock_layer() syntax values (mb.c:543-892) plus the nC context of
// every residual block, so that the host pass is pure serialisation.
#pragma once
#include <stdint.h>

namespace hl {

// e_type values mirror HL_CODEC_264_MB_TYPE_* (hl_codec_264_defs.h:399-540)
enum : int32_t {
    ET_I_NXN = 101,
    ET_I16 = 102,
    ET_P16x16 = 301,
    ET_P16x8 = 302,
    ET_P8x16 = 303,
    ET_P8x8 = 304,
    ET_P8x8REF0 = 305,
    ET_PSKIP = 306
};
// flags (hl_codec_264_mb.h:38-54)
enum : int32_t { FL_INTRA = 1, FL_INTER = 2, FL_SKIP = 4 };
// MbPartPredMode[0]
enum : int32_t { PM_L0 = 1, PM_I4 = 2, PM_I16 = 3 };

struct alignas(16) MbState {  // 432 bytes: whole 16-byte words (mb_begin loads neighbours as uint4)
    int32_t e_type, flags, pm0;
    int32_t cbp_l, cbp_c, cbp_l4x4;
    int32_t num_part, part_w, part_h;
    int32_t sub_w[4], sub_h[4];
    int16_t mv[4][4][2];          // MvL0 of the final decision
    int8_t i4mode[16];
    int8_t tc_luma[16];           // TotalCoeffsLuma
    int8_t tc_cac[2][4];          // TotalCoeffsChromaACCbCr
    int16_t cac_level[2][4][16];  // ChromaACLevel (read stale by decode_chroma)
    int32_t pad;
};
static_assert(sizeof(MbState) % 16 == 0, "MbState in whole 16-byte words");

struct MbRecord {
    int32_t e_type, mb_type, flags, pm0;
    int32_t cbp, cbp_l, cbp_c, cbp_l4x4;
    int32_t cbp_cdc[2], cbp_cac[2];
    int32_t num_part, num_sub[4], sub_mb_type[4];
    int32_t chroma_mode, i16mode;
    int16_t mvd[4][4][2];
    int16_t mv[4][4][2];
    int8_t prev_flag[16], rem_mode[16], i4mode[16];
    int8_t nc_luma[16];   // nC of each luma / I16 AC block write
    int8_t nc_cac[2][4];  // nC of each chroma AC block write
    int8_t nc_dc, pad0[3];
    int16_t luma[16][16];       // LumaLevel, or Intra16x16ACLevel (15 used)
    int16_t i16dc[16];
    int16_t cdc[2][4];
    int16_t cac[2][4][16];      // ChromaACLevel as written (15 used)
    int32_t mad;                // distortion of the chosen mode (rate control, rdo.c:211-228, 1266-1268)
    int32_t pad1;               // 1120 bytes: whole 16-byte words (the pipelined run copies records to the host)
#if defined(HL_DIAG_INPUTS)
    uint32_t dbg[8];            // diagnostic builds: digests of the MB's inputs (hl_mbcore.h mb_begin)
#endif
};

// Per-MB record of the rdo.Single_ctr chain (the reference keeps one
// encoder-global counter, residual.c:881-897, read stale by the I16x16 RDO).
struct MbChain {
    int32_t s_in;    // value seen on entry
    int32_t s_out;   // value left on exit
    int32_t dep;     // 1 = a stale read of the entry value happened before any fresh write
    int32_t fresh;   // 1 = the MB wrote the counter at least once
    int32_t spec;    // 1 = s_out is still a row-start speculation (no fresh write or resolution since)
};

}  // namespace hl
