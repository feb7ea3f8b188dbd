/*
 * ref_mbdump.h -- TEST INFRASTRUCTURE.  One mbrec.h record per reference
 * macroblock object (hl_codec_264_mb_t, mb.h:99-269), shared by the reference
 * drivers ref_harness.c and ref_svc_harness.c.
 */
#ifndef REF_MBDUMP_H
#define REF_MBDUMP_H
#include "mbrec.h"

static void dump_mb(const hl_codec_264_mb_t* m, int32_t* r)
{
    int i, j, c;
    memset(r, 0, sizeof(int32_t) * MBR_STRIDE);
    r[MBR_FLAGS] = ((m->flags_type & HL_CODEC_264_MB_TYPE_FLAGS_INTRA) ? 1 : 0)
                 | ((m->flags_type & HL_CODEC_264_MB_TYPE_FLAGS_INTER) ? 2 : 0)
                 | ((m->flags_type & HL_CODEC_264_MB_TYPE_FLAGS_SKIP) ? 4 : 0)
                 | ((m->MbPartPredMode[0] == HL_CODEC_264_MB_MODE_INTRA_16X16) ? 8 : 0)
                 | ((m->MbPartPredMode[0] == HL_CODEC_264_MB_MODE_INTRA_4X4) ? 16 : 0);
    r[MBR_MB_TYPE] = (int32_t)m->mb_type;
    for (i = 0; i < 4; ++i) r[MBR_SUB_MB_TYPE + i] = (int32_t)m->sub_mb_type[i];
    r[MBR_NUM_MB_PART] = m->NumMbPart;
    for (i = 0; i < 4; ++i) for (j = 0; j < 4; ++j) {
        r[MBR_MVL0 + (i * 4 + j) * 2 + 0] = m->mvL0[i][j].x;
        r[MBR_MVL0 + (i * 4 + j) * 2 + 1] = m->mvL0[i][j].y;
        r[MBR_MVD + (i * 4 + j) * 2 + 0] = m->mvd_l0[i][j].x;
        r[MBR_MVD + (i * 4 + j) * 2 + 1] = m->mvd_l0[i][j].y;
        r[MBR_MVL0_CAP + (i * 4 + j) * 2 + 0] = m->MvL0[i][j].x;
        r[MBR_MVL0_CAP + (i * 4 + j) * 2 + 1] = m->MvL0[i][j].y;
    }
    r[MBR_CBP_L4x4] = (int32_t)m->CodedBlockPatternLuma4x4;
    r[MBR_CBP] = (int32_t)m->coded_block_pattern;
    r[MBR_CBP_L] = (int32_t)m->CodedBlockPatternLuma;
    r[MBR_CBP_C] = (int32_t)m->CodedBlockPatternChroma;
    for (c = 0; c < 2; ++c) {
        r[MBR_CBP_CAC + c] = (int32_t)m->CodedBlockPatternChromaAC4x4[c];
        r[MBR_CBP_CDC + c] = (int32_t)m->CodedBlockPatternChromaDC4x4[c];
    }
    r[MBR_I16_MODE] = m->Intra16x16PredMode;
    for (i = 0; i < 16; ++i) {
        r[MBR_I4_MODE + i] = m->Intra4x4PredMode[i];
        r[MBR_PREV_FLAG + i] = m->prev_intra4x4_pred_mode_flag[i];
        r[MBR_REM_MODE + i] = m->rem_intra4x4_pred_mode[i];
        r[MBR_TC_LUMA + i] = m->TotalCoeffsLuma[i];
        r[MBR_I16_DC + i] = m->Intra16x16DCLevel[i];
        for (j = 0; j < 16; ++j) {
            r[MBR_LUMA_LEVEL + i * 16 + j] = m->LumaLevel[i][j];
            r[MBR_I16_AC + i * 16 + j] = m->Intra16x16ACLevel[i][j];
        }
    }
    r[MBR_CHROMA_MODE] = m->intra_chroma_pred_mode;
    r[MBR_QPY] = m->QPy;
    for (c = 0; c < 2; ++c) for (i = 0; i < 4; ++i) {
        r[MBR_TC_CAC + c * 4 + i] = m->TotalCoeffsChromaACCbCr[c][i];
        r[MBR_CHROMA_DC + c * 4 + i] = m->ChromaDCLevel[c][i];
        for (j = 0; j < 16; ++j) r[MBR_CHROMA_AC + (c * 4 + i) * 16 + j] = m->ChromaACLevel[c][i][j];
    }
    r[MBR_ETYPE] = m->e_type;
}

#endif
