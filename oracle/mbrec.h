/*
 * mbrec.h -- per-macroblock decision/state record used to diff the C
 * restatement (hl_oracle.c) and the HIP encoder against the reference
 * encoder MB by MB.  TEST INFRASTRUCTURE: the layout is ours; the fields
 * mirror members of the reference's hl_codec_264_mb_t
 * (include/hartallo/h264/hl_codec_264_mb.h:99-269) that the encode path
 * reads or writes.
 */
#ifndef HL_MBREC_H
#define HL_MBREC_H

enum {
    MBR_FLAGS = 0,            /* 1=intra 2=inter 4=skip 8=I16x16 16=I4x4 */
    MBR_MB_TYPE = 1,          /* mb_type syntax value                       */
    MBR_SUB_MB_TYPE = 2,      /* [4]                                        */
    MBR_NUM_MB_PART = 6,
    MBR_MVL0 = 7,             /* mvL0[4][4][2] (lower-case: final MVs)      */
    MBR_MVD = 39,             /* mvd_l0[4][4][2]                            */
    MBR_CBP_L4x4 = 71,
    MBR_CBP = 72,             /* coded_block_pattern                        */
    MBR_CBP_L = 73,
    MBR_CBP_C = 74,
    MBR_CBP_CAC = 75,         /* [2]                                        */
    MBR_CBP_CDC = 77,         /* [2]                                        */
    MBR_I16_MODE = 79,
    MBR_I4_MODE = 80,         /* [16]                                       */
    MBR_CHROMA_MODE = 96,
    MBR_PREV_FLAG = 97,       /* [16]                                       */
    MBR_REM_MODE = 113,       /* [16]                                       */
    MBR_QPY = 129,
    MBR_TC_LUMA = 130,        /* TotalCoeffsLuma[16]                        */
    MBR_TC_CAC = 146,         /* TotalCoeffsChromaACCbCr[2][4]              */
    MBR_LUMA_LEVEL = 154,     /* LumaLevel[16][16]                          */
    MBR_I16_DC = 410,         /* Intra16x16DCLevel[16]                      */
    MBR_I16_AC = 426,         /* Intra16x16ACLevel[16][16]                  */
    MBR_CHROMA_DC = 682,      /* ChromaDCLevel[2][4]                        */
    MBR_CHROMA_AC = 690,      /* ChromaACLevel[2][4][16]                    */
    MBR_ETYPE = 818,          /* reference e_type enum value (info only)    */
    MBR_MVL0_CAP = 819,       /* MvL0[4][4][2] (search state)               */
    MBR_COUNT = 851,
    MBR_STRIDE = 864          /* int32 per record in the dump files         */
};

#endif
