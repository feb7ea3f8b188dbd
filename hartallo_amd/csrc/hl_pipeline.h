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
//    f has finished every task in the staircase below (x+R+2, y+R+2): that
//    covers the planes of MBs up to (x+R, y+R) and every reader of the
//    MbState it overwrites.  A partition search whose motion window reaches
//    further waits for more (reach_wait in hl_mbcore.h).
//
// Scheduling is readiness-driven: every task (picture f, MB) has a counter
// of unfinished dependencies (task_deps); the workgroup that finishes a task
// decrements the counters of its successors (task_succ, the exact inverse)
// and pushes those that reach zero onto their picture's ready queue.
// Workgroups pop ready tasks, oldest picture first, so they never hold a task
// that cannot run yet.  The waits left inside a task (reach_wait, for motion
// windows beyond the guaranteed reach; resolve_chain, for an exact
// rdo.Single_ctr at a row start) only ever wait for tasks earlier in run
// order (picture, then raster address).  Workgroup 0 claims tasks in exactly
// that order instead of popping, so the earliest unfinished task is always
// held by a running workgroup that does not wait: the run progresses with
// any number of workgroups.
// Hand-offs between workgroups use the agent-scope release/acquire protocol
// of the gfx950 guide (cdna_hip_programming.md, Guideline 16): payload
// stores, s_waitcnt vmcnt(0) in every wave, barrier, one wave's release
// fence, then the counter / queue / flag atomics; consumers acquire once
// before reading.  Every wait is bounded.
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
    uint8_t* pl_out;    // this picture's quarter-pel planes (plane p at pl_out + p * F.plsz)
    int32_t deblock;    // deblocking enabled (disable_deblocking_filter_idc 0)
    int32_t* progress;  // host-mapped count of its stream's published pictures, or null
    int32_t* rows;      // host-mapped count of this picture's published MB rows, or null
};

// Dependencies of task (f, x, y) inside a run: the wavefront neighbours
// (x-1, y) and (x+1, y-1) (or (x, y-1) in the last column) and, from the
// second picture of the run on, the task of picture f-1 that completes the
// planes of MBs up to (x+R, y+R) (reach_task: (x+R+2, y+R+2) inside the
// picture), which also covers every reader of the MB state it overwrites.
HD int task_deps(int f, int x, int y, int mbw, int mbh, int R, int out[3][3])
{
    int n = 0;
    if (x > 0) {
        out[n][0] = f, out[n][1] = x - 1, out[n][2] = y;
        ++n;
    }
    if (y > 0) {
        out[n][0] = f, out[n][1] = x + 1 < mbw ? x + 1 : x, out[n][2] = y - 1;
        ++n;
    }
    if (f > 0) {
        out[n][0] = f - 1;
        reach_task(x + R, y + R, mbw, mbh, out[n][1], out[n][2]);
        ++n;
    }
    return n;
}

// Successors of task (f, X, Y): the tasks whose task_deps name it.  Returns
// their number and, for j below it, the j-th in (fo, xo, yo): in-picture ones
// first, then a rectangle of picture f+1 (several tasks at the right and
// bottom edges, where the staircase corner is clamped).
HD int task_succ(int f, int X, int Y, int mbw, int mbh, int R, int nframes, int j, int& fo, int& xo, int& yo)
{
    int n = 0;
    if (X + 1 < mbw) {  // (X+1, Y) waits on its left neighbour
        if (j == n) fo = f, xo = X + 1, yo = Y;
        ++n;
    }
    if (Y + 1 < mbh) {
        if (X > 0) {  // (X-1, Y+1) waits on its top-right neighbour
            if (j == n) fo = f, xo = X - 1, yo = Y + 1;
            ++n;
        }
        if (X == mbw - 1) {  // in the last column, on the one above
            if (j == n) fo = f, xo = X, yo = Y + 1;
            ++n;
        }
    }
    if (f + 1 < nframes) {
        const int k = Y == mbh - 1 ? 3 : 2;
        const int xa = X < mbw - 1 ? X - R - k : (mbw - 1 - R - k > 0 ? mbw - 1 - R - k : 0);
        const int ya = Y < mbh - 1 ? Y - R - 2 : (mbh - 1 - R - 2 > 0 ? mbh - 1 - R - 2 : 0);
        const int nx = X < mbw - 1 ? (xa >= 0 ? 1 : 0) : mbw - xa, ny = Y < mbh - 1 ? (ya >= 0 ? 1 : 0) : mbh - ya;
        if (j >= n && j < n + nx * ny) fo = f + 1, xo = xa + (j - n) % nx, yo = ya + (j - n) / nx;
        n += nx * ny;
    }
    return n;
}

// A run holds nstreams independent streams of spp consecutive pictures each:
// picture k of stream s is slot s * spp + k; task_deps / task_succ apply to
// the pictures of one stream (k), offset by the stream's first slot.
constexpr int kHelperQ = 16;  // helper FIFOs (PipeArgs::hq)

struct PipeArgs {
    const PipeFrame* fr;
    int32_t nframes;  // slots: nstreams * spp
    int32_t spp, nstreams;
    int32_t reach;   // guaranteed reference reach R in MBs
    int32_t window;  // pictures a workgroup looks at for ready tasks (from the oldest unfinished)
    int32_t hop;     // pop order: < 0 oldest picture first; else longest remaining path first, a picture
                     // boundary counting hop wavefront steps (pop_task)
    int32_t* cnt;    // [nframes][nmb] unfinished dependencies
    int32_t* claim;  // [nframes][nmb] 1 once a workgroup holds the task
    int32_t* done;   // [nframes][nmb] 1 once the task finished (reach_wait polls it)
    int32_t* queue;  // [nframes][kSubQ][nmb] ready tasks, MB address + 1 (0 = slot not yet written)
    // helper tasks (hl_mbcore.h intra_helper, guess_inter with f3out): a
    // ready P macroblock also queues its helpers, in kHelperQ FIFOs that
    // workgroups take from only when no macroblock is ready (ramp and tail of
    // a run, a lone picture).  Helper kind k of task g = f * nmb + addr goes
    // to FIFO (5 g + k) % kHelperQ: a bijection of [0, 5 nframes nmb), so no
    // FIFO holds more than ceil(5 nframes nmb / kHelperQ) entries
    int32_t helpers; // 1 = queue them
    int32_t* hstate; // [nframes][nmb] intra helper task states (HS_*)
    int32_t* hstate3; // [nframes][nmb][4] states of the 8x8 family's partitioning helpers (j = 3..6); HS_MAIN
                      // unless they were queued
    int32_t fam3;    // 1 = queue the partitioning helpers too, for pictures k < f3_first or k >= spp - f3_last of each
                     // stream (the ramp and tail of a run; every picture of a lone one)
    int32_t f3_first, f3_last;
    int32_t* hq;     // [kHelperQ][hq_cap] helper FIFOs, kind << 27 | (f * nmb + MB address + 1) (0 = slot not yet written)
    int32_t hq_cap;
    int32_t* hq_head;  // [kHelperQ]
    int32_t* hq_tail;  // [kHelperQ]
    int32_t* head;   // [nframes][kSubQ] next queue slot to pop
    int32_t* tail;   // [nframes][kSubQ] next queue slot to push
    int32_t* oldest; // [nstreams] first unfinished picture of each stream
    int32_t* err;    // [0] number of bounded waits that gave up
    unsigned long long* pub_clock;  // diagnostics: device wall clock at each picture's publication, or null
};

}  // namespace hl
