// hl_pipeline.h -- frame-pipelined encoding of a run of P pictures in one
// persistent launch (gfx950).
//
// The reference encodes picture after picture, and inside a picture macroblock
// after macroblock in raster order (slice.c:1701-1932), deblocking the whole
// picture afterwards (slice.c:1868-1880).  Its results only depend on that
// order through data dependencies, which this schedule keeps:
//
//  * inside a picture, MB (x, y) needs (x-1, y) and (x+1, y-1) (intra
//    neighbours, MV predictors, nC, and the rdo.Single_ctr chain along the
//    row);
//  * one task per MB: decide(x, y), then the deblocking of the MBs whose last
//    unfiltered-sample reader that decision was (trig_db), then the
//    quarter-pel plane blocks whose 3x3 deblocked neighbourhood is then final
//    (trig_pl).  tests/test_pipeline_schedule.py model-checks these rules:
//    deblocking stays in raster causality (deblock.c order) and never filters
//    a sample an intra prediction still has to read unfiltered;
//  * picture f+1 reads picture f's quarter-pel planes and chroma, and the
//    per-address MbState objects that persist across pictures
//    (hl_codec_264_mb_t, mb.h:99-269).  Task (f+1, x, y) waits until picture
//    f has finished every task in the staircase below (x+R+3, y+R+2): that
//    covers the planes of MBs up to (x+R, y+R) and every reader of the
//    MbState it overwrites.  A partition search whose motion window reaches
//    further waits for more (reach_wait in hl_mbcore.h).
//
// Frames are spread over S slots of W workgroups each (slot = frame mod S);
// picture f only ever waits for picture f-1, so the slots cannot deadlock
// once the grid (S x W <= 256 workgroups, one per CU) is resident.
// Hand-offs between workgroups use the agent-scope release/acquire protocol
// of the gfx950 guide (cdna_hip_programming.md, Guideline 16): payload
// stores, s_waitcnt vmcnt(0) in every wave, barrier, one lane's release
// fence, then a relaxed agent-scope flag store; consumers poll the flag
// relaxed, then one agent-scope acquire.  Every spin is bounded.
#pragma once
#include "hl_filters.h"

namespace hl {

// deblocking of MB (X, Y) runs in the task of MB trig_db(X, Y)
HD void trig_db(int X, int Y, int mbw, int mbh, int& x, int& y)
{
    if (Y < mbh - 1) {
        x = X + 1 < mbw - 1 ? X + 1 : mbw - 1;
        y = Y + 1;
    }
    else {
        x = X + 2 < mbw - 1 ? X + 2 : mbw - 1;
        y = mbh - 1;
    }
}
// quarter-pel planes of MB (X, Y) (and the padding it owns) run right after
// the deblocking of MB (min(X+1), min(Y+1)), in that deblocking's task
HD void trig_pl(int X, int Y, int mbw, int mbh, int& x, int& y)
{
    trig_db(X + 1 < mbw - 1 ? X + 1 : mbw - 1, Y + 1 < mbh - 1 ? Y + 1 : mbh - 1, mbw, mbh, x, y);
}

// Deblocking (kind 0) or plane (kind 1) blocks of task (x, y), in raster
// order; returns the count (at most 5 deblocks and 11 plane blocks, at the
// bottom-right corner).
constexpr int kMaxTaskBlocks = 16;
HD int task_blocks(int kind, int x, int y, int mbw, int mbh, int out[kMaxTaskBlocks][2])
{
    int n = 0;
    const int y0 = y - (kind ? 3 : 1), x0 = x - (kind ? 4 : 2);
    for (int Y = y0 < 0 ? 0 : y0; Y <= y; ++Y)
        for (int X = x0 < 0 ? 0 : x0; X <= x; ++X) {
            int tx, ty;
            if (kind) trig_pl(X, Y, mbw, mbh, tx, ty);
            else trig_db(X, Y, mbw, mbh, tx, ty);
            if (tx == x && ty == y && n < kMaxTaskBlocks) {
                out[n][0] = X;
                out[n][1] = Y;
                ++n;
            }
        }
    return n;
}

// Quarter-pel plane samples owned by MB (X, Y): its 16x16 pixels plus, for
// border MBs, the kPad-wide padding beside / above / below them (and the
// corners).  Each sample: qpel_plane_sample of all four planes.
HD void plane_block(const uint8_t* ref, int W, int H, int mbw, int mbh, uint8_t* pl0, int pstride, int plsz, int X, int Y,
                    int tid, int nthr)
{
    const int x0 = X == 0 ? -kPad : X * 16, x1 = X == mbw - 1 ? W + kPad : X * 16 + 16;
    const int y0 = Y == 0 ? -kPad : Y * 16, y1 = Y == mbh - 1 ? H + kPad : Y * 16 + 16;
    const int bw = x1 - x0, n = bw * (y1 - y0);
    for (int t = tid; t < n; t += nthr) {
        const int px = x0 + t % bw, py = y0 + t / bw;
        const int o = (py + kPad) * pstride + px + kPad;
        for (int p = 0; p < 4; ++p) pl0[p * plsz + o] = qpel_plane_sample(ref, W, H, p, px, py);
    }
}

// One picture of a pipelined run
struct PipeFrame {
    FrameArgs F;
    DeblockArgs D;
    uint8_t* pl_out;  // this picture's quarter-pel planes (plane p at pl_out + p * F.plsz)
    int32_t deblock;  // deblocking enabled (disable_deblocking_filter_idc 0)
};

struct PipeArgs {
    const PipeFrame* fr;
    int32_t nframes, slots;
    const int32_t* order;  // MB addresses in wavefront (anti-diagonal) order
    int32_t* done;         // [slots][nmb]: picture index + 1 once the task of MB addr finished
    int32_t* next;         // [slots] task counters
    int32_t* err;          // [0] = number of bounded spins that gave up
    int32_t reach;         // guaranteed reference reach R in MBs
};

}  // namespace hl
