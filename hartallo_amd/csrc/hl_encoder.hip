// hl_encoder.hip -- the gfx950 encode path behind include/hartallo_amd.h.
//
// Per frame (hl_codec_264_encode_frame, encode.c:144-527, restated):
//   1. k_planes      quarter-pel planes of the reference picture (HBM-bound)
//   2. k_mb_diag     macroblock decisions on an anti-diagonal wavefront:
//                    MB (x, y) runs after (x-1, y) and (x+1, y-1), i.e. in
//                    launch d = x + 2y; one 512-lane workgroup per MB
//   3. row-start validation of the rdo.Single_ctr speculation (host), with a
//      re-run of the wavefront from the first mispredicted row
//   4. k_deblock_rows the in-place Baseline deblocking in one launch (one
//                    workgroup per MB row, LDS tiles, raster causality)
//   5. host CAVLC serialisation of the MB records (hl_writer.cpp)
// Runs of pictures: k_pipeline (hl_pipeline.h), one persistent launch.
// Spatial SVC layers: k_svc_mb, k_deblock_rows, k_el_count / k_el_write.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <future>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#if !defined(HL_KERNELS_ONLY)
#include "../../include/hartallo_amd.h"
#include "hl_rc.h"
#endif
#include "hl_pipeline.h"
#if !defined(HL_KERNELS_ONLY)
#include "hl_svc.h"
#include "hl_cavlc.h"
#include "hl_writer.h"
#endif

using namespace hl;

#define HL_HIP_CHECK(x)                                                                  \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "hartallo_amd: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return HL_AMD_ERROR_SYSTEM;                                                  \
        }                                                                                \
    } while (0)


// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
#if !defined(HL_KERNELS_ONLY)
static void launch_planes(hl_amd_encoder_t* e, const uint8_t* ref_y);
#endif

#if defined(HL_POISON_LDS)
// Debug builds (-DHL_POISON_LDS=<salt>): the workgroup's LDS image (bytes
// [HL_POISON_LO, HL_POISON_HI) of Shared, default all of it) is filled with a
// pattern derived from the task before every macroblock, so that any read of
// Shared before this macroblock wrote it changes the output.
#ifndef HL_POISON_LO
#define HL_POISON_LO 0
#endif
#ifndef HL_POISON_HI
#define HL_POISON_HI sizeof(Shared)
#endif
__device__ void poison_lds(Shared& S, uint32_t seed)
{
    uint32_t* w = reinterpret_cast<uint32_t*>(&S);
    const uint32_t lo = (uint32_t)(HL_POISON_LO) / 4, hi = ((uint32_t)(HL_POISON_HI) + 3) / 4;
    for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        uint32_t h = (i + 1u) * 2654435761u ^ (seed + (uint32_t)HL_POISON_LDS) * 0x9E3779B9u;
        h ^= h >> 15;
        h *= 0x2C1B3C6Du;
        h ^= h >> 12;
        w[i] = h;
    }
    __syncthreads();
}
#define HL_POISON(S, seed) poison_lds(S, seed)
#else
#define HL_POISON(S, seed) ((void)0)
#endif

// macroblocks (x, y) with x + 2 * (y - row0) == diag
__device__ __forceinline__ void diag_mb(int mbw, int mbh, int row0, int diag, int k, int& x, int& y)
{
    const int ylo = std::max(0, (diag - mbw + 2) / 2);
    const int yy = ylo + k;
    y = row0 + yy;
    x = diag - 2 * yy;
}

// The frame arguments of a macroblock task, copied into LDS: their fields are
// then LDS reads the compiler knows cannot alias the global stores and the
// LDS stores of the decision (read through a generic pointer, every field
// was reloaded with a flat load after each store).
__device__ __forceinline__ void frame_args_to_lds(FrameArgs& dst, const FrameArgs& src, int tid)
{
    static_assert(sizeof(FrameArgs) % 4 == 0 && sizeof(FrameArgs) / 4 <= kMbThreads, "FrameArgs copied one word per lane");
    if (tid < (int)(sizeof(FrameArgs) / 4))
        reinterpret_cast<uint32_t*>(&dst)[tid] = gmem(reinterpret_cast<const uint32_t*>(&src))[tid];
    __syncthreads();
}

#if !defined(HL_KERNELS_ONLY)
__global__ __launch_bounds__(kMbThreads, 2) void k_mb_diag(FrameArgs F, int diag, int row0)
{
    __shared__ Shared S;
    __shared__ FrameArgs sF;
    int x, y;
    diag_mb(F.mbw, F.mbh, row0, diag, blockIdx.x, x, y);
    const int addr = y * F.mbw + x;
    const int s_in = x == 0 ? F.spec[y] : F.chain[addr - 1].s_out;
    HL_POISON(S, (uint32_t)addr * 7919u + (uint32_t)diag);
    if (threadIdx.x < (int)(sizeof(FrameArgs) / 4)) reinterpret_cast<uint32_t*>(&sF)[threadIdx.x] = reinterpret_cast<const uint32_t*>(&F)[threadIdx.x];
    __syncthreads();
    encode_mb(sF, S, addr, threadIdx.x, kMbThreads, s_in);
}
#endif

#if !defined(HL_KERNELS_ONLY)
// Deblocking of a whole picture in one launch: one 64-lane workgroup per MB
// row, its MBs left to right; MB (x, y) waits until row y - 1 has finished
// MB x + 1 -- the order of the anti-diagonal launches d = x + 2y, so every
// edge sees the samples the reference's raster-order filter sees
// (deblock.c:192-284).  Each MB is filtered in an LDS tile (DbTile,
// hl_filters.h): its own rows are prefetched into registers during the
// previous MB, the left apron is carried over, only the 4 rows above wait for
// the row above; the bS values of the whole row (up to 256 MBs)
// are computed before its first wait, off the chain of rows.  Hand-offs as
// in k_pipeline: stores drained, a release fence, a relaxed flag; the
// consumer acquires.
__global__ __launch_bounds__(64) void k_deblock_rows(DeblockArgs D, int32_t* row_done, int32_t* err)
{
    __shared__ DbTile t;
    const int y = blockIdx.x, tid = threadIdx.x, mbw = D.mbw;
    uint32_t own_l = db_own_luma(D, 0, y, tid), own_c = tid < 32 ? db_own_chroma(D, 0, y, tid) : 0u;
    int chunk0 = -kDbChunk;
    for (int x = 0; x < mbw; ++x) {
        __syncthreads();  // the previous MB's stores have read the tile
        if (x - chunk0 >= kDbChunk) {
            chunk0 = x;
            const int n = min(kDbChunk, mbw - x) * 32;
            for (int i = tid; i < n; i += 64) t.B[i >> 5][i & 31] = (uint8_t)deblock_edge_bs(D, y * mbw + x + (i >> 5), (i & 31) >> 2, i & 3);
        }
        if (x > 0) db_shift(t, tid);
        __syncthreads();
        db_put_own(t, tid, own_l, own_c);
        if (x + 1 < mbw) {  // the next MB's own rows, in flight during this one
            own_l = db_own_luma(D, x + 1, y, tid);
            if (tid < 32) own_c = db_own_chroma(D, x + 1, y, tid);
        }
        if (y > 0) {
            if (tid == 0) spin_ge(row_done + y - 1, min(x + 2, mbw), err);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            __syncthreads();
            db_load_above(D, t, x, y, tid);
        }
        __syncthreads();
        const uint8_t* bs = t.B[x - chunk0];
        for (int step = 0; step < 8; ++step) {
            db_tile_step(D, t, bs, step, tid);
            __syncthreads();
        }
        for (int j = tid; j < db_store_words(); j += 64) db_store(D, t, x, y, j);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (tid == 0) st_relaxed(row_done + y, x + 1);
    }
}
#endif

// 1: the task's plane and deblocked-sample stores non-temporal
// Deblocking and plane blocks of task (x, y) (hl_pipeline.h).
// The deblocking of one MB in the LDS tile (DbMbTile, hl_filters.h) that
// aliases the decision's prediction scratch (free once the MB is decided):
// one load round, the eight edges by wave 0 in LDS, one store round.
__device__ void deblock_mb_lds(const DeblockArgs& D, int X, int Y, int tid, DbMbTile& t)
{
    for (int j = tid; j < db_mb_load_words(); j += kMbThreads) db_mb_load(D, t, X, Y, j);
    if (tid < 32) t.bs[tid] = (uint8_t)deblock_edge_bs(D, Y * D.mbw + X, tid >> 2, tid & 3);
    __syncthreads();
    if (tid < 64)
        for (int step = 0; step < 8; ++step) {
            db_tile_step(D, t, t.bs, step, tid);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: the next edge reads what this one wrote
        }
    __syncthreads();
    for (int j = tid; j < db_mb_store_slots(); j += kMbThreads) db_mb_store(D, t, X, Y, j);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// Quarter-pel plane samples of an interior MB (no padding to own, every tap
// inside the picture): the 21x21 source neighbourhood and its vertical 6-tap
// sums staged in LDS, then 64 lanes write 4 samples of each plane as one
// 4-byte store per plane.  Same values as plane_block / qpel_plane_sample.
__device__ void plane_block_lds(const uint8_t* ref, int W, uint8_t* pl0, int pstride, int plsz, int X, int Y, int tid, uint8_t* T,
                                int16_t* V)
{
    constexpr int TS = 24;  // T row stride
    const int x0 = X * 16 - 2, y0 = Y * 16 - 2;
    for (int i = tid; i < 21 * 21; i += kMbThreads) {
        const int r = i / 21, c = i - r * 21;
        T[r * TS + c] = gmem(ref)[(size_t)(y0 + r) * W + x0 + c];
    }
    __syncthreads();
    for (int i = tid; i < 16 * 21; i += kMbThreads) {
        const int r = i / 21, c = i - r * 21;
        const uint8_t* t = T + r * TS + c;
        V[r * 21 + c] = (int16_t)tap6(t[0], t[TS], t[2 * TS], t[3 * TS], t[4 * TS], t[5 * TS]);
    }
    __syncthreads();
    if (tid < 64) {
        const int r = tid >> 2, c0 = (tid & 3) * 4;
        uint32_t f = 0, b = 0, h = 0, j = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint8_t* t = T + (r + 2) * TS + c0 + k;  // t[2]: the sample itself
            const int16_t* v = V + r * 21 + c0 + k;        // v[2]: its vertical sum
            int vb = (tap6(t[0], t[1], t[2], t[3], t[4], t[5]) + 16) >> 5;
            int vh = (v[2] + 16) >> 5;
            int vj = (tap6(v[0], v[1], v[2], v[3], v[4], v[5]) + 512) >> 10;
            // opaque: keeps hipcc from fusing shift + clamp + packing into
            // v_ashr_pk_u8_i32 (miscompiled on gfx950, see k_planes)
            asm volatile("" : "+v"(vb), "+v"(vh), "+v"(vj));
            f |= (uint32_t)t[2] << (8 * k);
            b |= (uint32_t)clip255(vb) << (8 * k);
            h |= (uint32_t)clip255(vh) << (8 * k);
            j |= (uint32_t)clip255(vj) << (8 * k);
        }
        const size_t o = (size_t)(Y * 16 + r + kPad) * pstride + X * 16 + c0 + kPad;
        *gmem(reinterpret_cast<uint32_t*>(pl0 + o)) = f;
        *gmem(reinterpret_cast<uint32_t*>(pl0 + plsz + o)) = b;
        *gmem(reinterpret_cast<uint32_t*>(pl0 + 2 * (size_t)plsz + o)) = h;
        *gmem(reinterpret_cast<uint32_t*>(pl0 + 3 * (size_t)plsz + o)) = j;
    }
    __syncthreads();  // the scratch is reused by the next block
}

__device__ void task_filters(const PipeFrame& PF, Shared& S, int x, int y, int mbw, int mbh, int tid)
{
    static_assert(sizeof(DbMbTile) <= sizeof(S.pred), "the tile aliases Shared::pred");
    int blk[kMaxTaskBlocks][2];
    const int nd = PF.deblock ? task_blocks(0, x, y, mbw, mbh, blk) : 0;
    DbMbTile& tile = *reinterpret_cast<DbMbTile*>(S.pred);
    for (int i = 0; i < nd; ++i) deblock_mb_lds(PF.D, blk[i][0], blk[i][1], tid, tile);
    const int np = task_blocks(1, x, y, mbw, mbh, blk);
    static_assert(21 * 24 <= sizeof(S.pred) && 16 * 21 * sizeof(int16_t) <= sizeof(S.i16_ac), "plane scratch");
    uint8_t* T = reinterpret_cast<uint8_t*>(S.pred);      // free once the MB is decided
    int16_t* V = reinterpret_cast<int16_t*>(S.i16_ac);
    for (int i = 0; i < np; ++i) {
        const int X = blk[i][0], Y = blk[i][1];
        if (X > 0 && Y > 0 && X < mbw - 1 && Y < mbh - 1)
            plane_block_lds(PF.F.cur[0], PF.F.W, PF.pl_out, PF.F.pstride, PF.F.plsz, X, Y, tid, T, V);
        else
            plane_block(PF.F.cur[0], PF.F.W, PF.F.H, mbw, mbh, PF.pl_out, PF.F.pstride, PF.F.plsz, X, Y, tid, kMbThreads);
    }
}

// a / d for 0 <= a < 2^24 and quotients below 2^20 from a float reciprocal
// of d (correctly rounded or the 1-ulp v_rcp_f32: the product is within one
// of the quotient) and one correction each way (exact; the scheduler's
// quotients are pictures, rows and streams): integer division by a runtime value is a
// long VALU sequence, and the scheduler divides by the picture width, the MB
// count and the stream and picture counts on every pop and task
__device__ __forceinline__ int udiv_small(int a, int d, float inv)
{
    int q = (int)((float)a * inv);
    q -= q * d > a ? 1 : 0;
    q += (q + 1) * d <= a ? 1 : 0;
    return q;
}
// 1: scheduler reciprocals in LDS, task coordinates and the wave's first
// lane index in SGPRs (k_pipeline): VGPR spills 15 -> 13, but 0.4 % slower
// (profiles/r05_ab_sched_lds_sgpr_coords_not_kept.log)
__device__ __forceinline__ int uni(int v) { return v; }
struct SchedRecip {
    float mbw, nmb, S, spp;  // 1 / (MBs per row, MBs per picture, streams, pictures per stream)
};

// Every picture's ready queue is split into kSubQ sub-queues (column bands
// of MBs) with their own heads: a workgroup prefers its own sub-queue
// (blockIdx % kSubQ) among tasks of similar priority, so that hundreds of
// idle workgroups do not all race for one queue head (one head serialised
// the pops: 19 attempts per task, 18 lost, profiles/r04_pipe_profile_pops.log).
#ifndef HL_SUBQ
#define HL_SUBQ 4
#endif
constexpr int kSubQ = HL_SUBQ;
// head entries each lane of pop_task examines: kScan * 64 / kSubQ pictures in view
#ifndef HL_SCAN
#define HL_SCAN 4
#endif
constexpr int kScan = HL_SCAN;

#if !defined(HL_KERNELS_ONLY)
// Dependency counters and ready queues of a run (hl_pipeline.h): only task
// (0, 0) of every stream's first picture starts ready.
__global__ __launch_bounds__(256) void k_pipe_init(PipeArgs P, int mbw, int mbh)
{
    const int nmb = mbw * mbh, i = blockIdx.x * 256 + threadIdx.x;
    if (i < P.nframes * nmb) {
        const int f = i / nmb, a = i - f * nmb, k = f % P.spp;  // picture k of its stream
        int d[3][3];
        P.cnt[i] = task_deps(k, a % mbw, a / mbw, mbw, mbh, P.reach, d);
        P.done[i] = 0;
        for (int q = 0; q < kSubQ; ++q) P.queue[(f * kSubQ + q) * nmb + a] = k == 0 && a == 0 && q == 0 ? 1 : 0;  // every stream's first task
        P.claim[i] = 0;
        P.hstate[i] = HS_FREE;
        for (int j = 0; j < 4; ++j) P.hstate3[4 * i + j] = HS_MAIN;  // (HS_FREE once queued)
        for (int j = 0; j < 5; ++j) P.hq[j * P.nframes * nmb + i] = 0;
    }
    if (i < kHelperQ) P.hq[5 * P.nframes * nmb + i] = 0;  // (kHelperQ * hq_cap < 5 nframes nmb + kHelperQ; the grid has >= 256 threads)
    if (i < P.nframes * kSubQ) {
        P.head[i] = 0;
        P.tail[i] = (i / kSubQ) % P.spp == 0 && i % kSubQ == 0 ? 1 : 0;
    }
    if (i < P.nstreams) P.oldest[i] = 0;
    if (i < kHelperQ) {
        P.hq_head[i] = 0;
        P.hq_tail[i] = 0;
    }
    if (i == 0) {
        for (int k = 0; k < 8; ++k) P.err[k] = 0;  // give-ups, chain walks, helper I4 kept / rejected / taken over, -, 8x8 family kept / rejected
    }
}
#endif

// Wave 0 takes the next ready task and claims it: f * nmb + addr, or -1 once
// the run has finished (or after ~10 s without a task: a wait gave up
// somewhere and the host re-encodes the run).  A queue entry whose claim
// fails was taken by workgroup 0 (claim_next) and is skipped.
//
// Which picture's queue head: with P.hop < 0 the oldest picture's; else the
// head with the longest remaining dependency path to the end of the run
// (highest level first), ties to the older picture.  Inside a picture the
// path from MB (x, y) to the last MB is (mbw-1-x) + 2 (mbh-1-y) wavefront
// steps; each later picture adds the lag of task_deps' staircase, about
// 3 (R+2) steps (P.hop).  The oldest-first order lets the newest pictures'
// wavefronts start late, and the run ends on their critical path.
#if defined(HL_PROFILE)
#define HL_POPSTAT(i) (++pst[i])
#else
#define HL_POPSTAT(i) ((void)0)
#endif
// olc: lane s < S holds stream s's oldest unfinished picture as the previous
// call read it (-1: none yet); the scan uses it while this call's read is in
// flight (a stale value only shifts the window late: its first pictures are
// finished ones, with empty queues)
__device__ int pop_task(const PipeArgs& P, int nmb, int mbw, int mbh, int& olc, const SchedRecip& rc
#if defined(HL_PROFILE)
                        , unsigned long long* pst  // profiling: [0] attempts on a macroblock, [1] lost, [2] empty rounds
#endif
)
{
    const int lane = __lane_id();
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    int empty = 0;
    for (;;) {
        // entry e = lane + 64 i (kScan per lane) = (sub-queue e % kSubQ,
        // stream r % S, its picture oldest + r / S) with r = e / kSubQ: the
        // window of each stream's first unfinished pictures
        const int S = P.nstreams;
        int oln = 0;
        if (lane < S) oln = ld_relaxed(P.oldest + lane);
        const int ol = P.nframes > 1 && olc >= 0 ? olc : oln;  // (a lone picture: idle workgroups poll at the read's pace)
        int fl[kScan], ql[kScan], hs[kScan], ts[kScan], js[kScan], sqs[kScan];
        bool ins[kScan];
#pragma unroll
        for (int i = 0; i < kScan; ++i) {
            const int e = lane + 64 * i, sq = e % kSubQ, rr = e / kSubQ, j = udiv_small(rr, S, rc.S), sj = rr - j * S;
            const int k = __shfl(ol, sj, 64) + j;
            ins[i] = j < max(1, P.window / S) && k < P.spp;
            fl[i] = sj * P.spp + k;  // picture slot, its sub-queue
            ql[i] = fl[i] * kSubQ + sq;
            js[i] = j;
            sqs[i] = sq;
            hs[i] = ts[i] = 0;
            if (ins[i]) {
                hs[i] = ld_relaxed(P.head + ql[i]);
                ts[i] = ld_relaxed(P.tail + ql[i]);
            }
        }
        olc = oln;
        if (__ballot(lane < S && oln < P.spp) == 0) return -1;  // every stream finished
        int i0 = -1, hh = 0, v = 0, bfl = 0, bql = 0;
        if (P.hop < 0) {
            // oldest first: the first non-empty entry
            unsigned long long bal = 0;
            int bh = 0;
#pragma unroll
            for (int i = 0; i < kScan && !bal; ++i) {
                bal = __ballot(ins[i] && hs[i] < ts[i]);
                if (bal) {
                    i0 = __ffsll((long long)bal) - 1;
                    bh = __builtin_amdgcn_readlane(hs[i], i0);
                    bfl = __builtin_amdgcn_readlane(fl[i], i0);
                    bql = __builtin_amdgcn_readlane(ql[i], i0);
                }
            }
            hh = bh;
        }
        else {
            // the head entries themselves (0: pushed, not yet written); each
            // lane keeps its best, then the wave's best
            int qv[kScan];
#pragma unroll
            for (int i = 0; i < kScan; ++i) {
                qv[i] = 0;
                if (ins[i] && hs[i] < ts[i]) qv[i] = ld_relaxed(P.queue + ql[i] * nmb + hs[i]);
            }
            int key = -1, lh = 0, lq = 0, lfl = 0, lql = 0;
#pragma unroll
            for (int i = 0; i < kScan; ++i) {
                if (qv[i] > 0) {
                    const int a = qv[i] - 1, y = udiv_small(a, mbw, rc.mbw), x = a - y * mbw;
                    // preference for the workgroup's sub-queue, in wavefront steps of priority (one stream's
                    // column bands 30: +0.5 / +0.9 %, profiles/r06_ab_column_bands.log; several streams 12)
                    const int own = sqs[i] == (int)(blockIdx.x % kSubQ) ? (S == 1 ? 30 : 12) : 0;
                    const int kk = (((mbw - 1 - x) + 2 * (mbh - 1 - y) - P.hop * js[i] + own + 4096) << 6) | (63 - lane);
                    if (kk > key) {
                        key = kk;
                        lh = hs[i];
                        lq = qv[i];
                        lfl = fl[i];
                        lql = ql[i];
                    }
                }
            }
            for (int s2 = 1; s2 < 64; s2 <<= 1) key = max(key, __shfl_xor(key, s2, 64));
            key = __builtin_amdgcn_readfirstlane(key);
            if (key >= 0) {
                i0 = 63 - (key & 63);
                hh = __builtin_amdgcn_readlane(lh, i0);
                v = __builtin_amdgcn_readlane(lq, i0);
                bfl = __builtin_amdgcn_readlane(lfl, i0);
                bql = __builtin_amdgcn_readlane(lql, i0);
            }
            // else: empty, or only pushes between their tail and slot stores
        }
        if (i0 >= 0) {
            HL_POPSTAT(0);
            const int f = bfl, qf = bql;
            int r = 0;
            if (lane == 0 && atomicCAS(P.head + qf, hh, hh + 1) == hh) {
                r = v;
                // the slot is pushed right after the tail moved
                for (unsigned k = 0; r == 0 && (r = ld_relaxed(P.queue + qf * nmb + hh)) == 0; ++k)
                    if (k > (1u << 26)) {
                        atomicAdd(P.err, 1);
                        r = -1;
                        break;
                    }
                if (r > 0 && atomicCAS(P.claim + f * nmb + r - 1, 0, 1) != 0) r = 0;
            }
            r = __builtin_amdgcn_readfirstlane(r);
            if (r < 0) return -1;
            if (r > 0) {
                return f * nmb + r - 1;
            }
            HL_POPSTAT(1);
            // another workgroup took it: retry, except beside a lone picture
            // (the 8x8 family's helpers on), where ~200 idle workgroups race for
            // each ready macroblock and the losers take a helper task instead
            // (in runs, measured: no gain, profiles/r06_ab_partitioning_helpers_in_runs.log)
            if (!P.fam3 || P.nframes > 1) continue;
        }
        if (P.helpers) {  // no macroblock ready: a helper task, unless its macroblock took it over
            // lane q reads FIFO q; the workgroup's own FIFO first, then the
            // next non-empty one after it
            int qh = 0, qt = 0;
            if (lane < kHelperQ) {
                qh = ld_relaxed(P.hq_head + lane);
                qt = ld_relaxed(P.hq_tail + lane);
            }
            const unsigned ne = (unsigned)__ballot(lane < kHelperQ && qh < qt);
            if (ne) {
                const int own = (int)(blockIdx.x % kHelperQ);
                const unsigned rot = ((ne >> own) | (ne << (kHelperQ - own))) & ((1u << kHelperQ) - 1u);
                const int q = (own + __builtin_ctz(rot)) % kHelperQ;
                const int hh = __builtin_amdgcn_readlane(qh, q);
                int r = 0;
                int kind = 0;
                if (lane == 0 && atomicCAS(P.hq_head + q, hh, hh + 1) == hh) {
                    for (unsigned k = 0; (r = ld_relaxed(P.hq + q * P.hq_cap + hh)) == 0; ++k)
                        if (k > (1u << 26)) {
                            atomicAdd(P.err, 1);
                            r = -1;
                            break;
                        }
                    if (r > 0) {
                        kind = r >> 27;
                        r &= (1 << 27) - 1;
                        if (atomicCAS(kind ? P.hstate3 + 4 * (r - 1) + kind - 1 : P.hstate + r - 1, HS_FREE, HS_CLAIMED) != HS_FREE) r = 0;
                    }
                }
                r = __builtin_amdgcn_readfirstlane(r);
                kind = __builtin_amdgcn_readfirstlane(kind);
                if (r < 0) return -1;
                if (r > 0) {
                    return (1 + kind) * P.nframes * nmb + r - 1;  // intra helpers, then the 8x8 family's partitionings 3..6
                }
                continue;
            }
        }
        HL_POPSTAT(2);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 1000000000ull) {  // 10 s at 100 MHz
            if (lane == 0) atomicAdd(P.err, 1);
            return -1;
        }
        // nothing ready: back off (fewer scans of the queue words while tasks run)
#ifndef HL_IDLE_SLEEP
#define HL_IDLE_SLEEP 16
#endif
        if (++empty < 4) __builtin_amdgcn_s_sleep(4);
        else __builtin_amdgcn_s_sleep(HL_IDLE_SLEEP);
    }
}

// Workgroup 0 claims tasks in run order (picture, then raster address)
// instead of popping ready ones, and waits for the claimed task's
// dependencies.  Every wait inside a task (reach_wait, resolve_chain) and
// every dependency targets a task earlier in run order, and every earlier
// task is claimed, i.e. held by a running workgroup or done; so the earliest
// unfinished task never waits, and the run completes with any number of
// workgroups (one included) -- no geometry can deadlock.
__device__ int claim_next(const PipeArgs& P, int nmb, int& cursor)
{
    const int lane = __lane_id(), total = P.nframes * nmb;
    for (;; ++cursor) {
        if (cursor >= total) return -1;
        int c = 0;
        if (lane == 0) c = atomicCAS(P.claim + cursor, 0, 1);
        if (__builtin_amdgcn_readfirstlane(c) == 0) break;
    }
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (ld_relaxed(P.cnt + cursor) != 0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 1000000000ull) {  // 10 s at 100 MHz
            if (lane == 0) atomicAdd(P.err, 1);
            return -1;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    return cursor++;
}

// Pipelined run of P pictures (hl_pipeline.h): persistent workgroups taking
// ready tasks (decision, then the deblocking and plane blocks it completes)
// until the run has finished.
// waves per SIMD the register allocation of k_pipeline must allow (the
// second __launch_bounds__ argument is waves per EU on AMDGPU): 2 = one
// 512-lane workgroup per CU with up to 256 VGPRs, 4 = two workgroups with 128
#ifndef HL_PIPE_WAVES_PER_EU
#define HL_PIPE_WAVES_PER_EU 2
#endif
// 1: successor-counter decrements relaxed behind the task's release fence,
// an acquire fence only before a push (0: acq_rel decrements)
__global__ __launch_bounds__(kMbThreads, HL_PIPE_WAVES_PER_EU) void k_pipeline(PipeArgs Pk, int mbw, int mbh)
{
    const PipeArgs& P0 = Pk;  // (the prologue's reads; the loop reads P, below)
    __shared__ Shared S;
    __shared__ FrameArgs sF;  // the task's frame arguments (frame_args_to_lds)
    __shared__ int32_t s_task;
    const int nmb = mbw * mbh;
    const bool in_order = blockIdx.x == 0;  // claims tasks in run order (claim_next)
    // wave 0's loop state per lane in LDS (claim_next's cursor, pop_task's
    // oldest pictures of the previous call): held in VGPRs, the two were
    // spilled in the prologue
    __shared__ int s_sched[2][64];
    if (threadIdx.x < 64) {
        s_sched[0][threadIdx.x] = 0;
        s_sched[1][threadIdx.x] = -1;
    }
#define HL_RC rc
    // the wave's first lane index in an SGPR (the work-item index VGPR was
    // spilled in the prologue and reloaded per task)
    const int wbase = __builtin_amdgcn_readfirstlane(threadIdx.x) & ~63;
#define HL_WAVE0 (wbase == 0)
#define HL_TID (wbase + (int)__lane_id())
#if defined(HL_PRIO_YOUNG)
    // the second-dispatched half of the workgroup (waves 4-7) loses every VALU
    // arbitration to its SIMD partner at equal priority (MI355X_MICROARCH.md,
    // two waves per SIMD, item 4): static priority for it
    if (threadIdx.x >= kMbThreads / 2) __builtin_amdgcn_s_setprio(HL_PRIO_YOUNG);
#endif
#if defined(HL_PROFILE)
    // per-workgroup totals (profiling build): prof[40..44] = waits for a ready
    // task, decisions, filters, tasks, workgroup lifetime (shader clock)
    unsigned long long pw_wait = 0, pw_mb = 0, pw_filt = 0, pw_n = 0, pw_hlp = 0, pw_hn = 0, pw_phlp = 0, pw_phn = 0;
    unsigned long long pst[3] = {0, 0, 0};  // pop_task rounds (wave 0)
    unsigned long long ptail[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // after the filters: barrier, release fence, successors' release; early release; its fence, release, spin, acquire
    const unsigned long long pw_t0 = __builtin_readcyclecounter();
    unsigned long long* prof = P0.fr[0].F.prof;
#endif
    for (;;) {
        // the run's arguments read from the kernel-argument segment in every
        // task (scalar loads through a pointer the compiler cannot follow),
        // not held in registers across the task body (spilled in the prologue)
        using KArgs = __attribute__((address_space(4))) const PipeArgs;
        KArgs* pk = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(pk));
        const PipeArgs& P = *(const PipeArgs*)pk;
        // the scheduler's reciprocals per task, from opaque copies (hoisted,
        // they were held across the body too); udiv_small corrects the
        // approximate reciprocal's quotient
        int iw = mbw, in = nmb;
        asm volatile("" : "+s"(iw), "+s"(in));
        const SchedRecip rc{__builtin_amdgcn_rcpf((float)iw), __builtin_amdgcn_rcpf((float)in), __builtin_amdgcn_rcpf((float)P.nstreams),
                            __builtin_amdgcn_rcpf((float)P.spp)};
#if defined(HL_PROFILE)
        const unsigned long long pt0 = __builtin_readcyclecounter();
#endif
        if (HL_WAVE0) {
            int ln = __lane_id();
            asm volatile("" : "+v"(ln));  // (its LDS address computed here, not held)
            int cursor = s_sched[0][ln], olc = s_sched[1][ln];
            const int t = in_order ? claim_next(P, nmb, cursor) : pop_task(P, nmb, mbw, mbh, olc, HL_RC
#if defined(HL_PROFILE)
                                                                                           , pst
#endif
            );
            s_sched[0][ln] = cursor;
            s_sched[1][ln] = olc;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, HL_ACQ_SCOPE);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate completes before the barrier
            if (__lane_id() == 0) s_task = t;
        }
        __syncthreads();
        int t = __builtin_amdgcn_readfirstlane(s_task);
        if (t < 0) break;
#if defined(HL_PROFILE)
        const unsigned long long pw_start = wall_clock64();  // (the task's timeline, below)
#endif
        // helper tasks (hl_mbcore.h): 1 = intra_helper, 2..5 = the 8x8 family's
        // partitioning hk + 1 (guess_inter)
        int hk = 0;
        while (t >= P.nframes * nmb) {
            t -= P.nframes * nmb;
            ++hk;
        }
        hk = uni(hk);
        const bool helper = hk > 0;
#if defined(HL_DIAG) && HL_DIAG == 1
        __syncthreads();
#endif
        // opaque per task: keeps the compiler from hoisting encode_mb's
        // lane-index arithmetic out of the task loop and holding it live
        // across the whole body (160 spilled VGPRs without this)
        int tid = HL_TID;
        asm volatile("" : "+v"(tid));
        // (the task's coordinates are uniform: computed on the VALU (float
        // reciprocals), held in SGPRs across the macroblock body)
        const int f = uni(udiv_small(t, nmb, rc.nmb)), addr = t - f * nmb;
        const PipeFrame& PF = P.fr[f];
        const int y = uni(udiv_small(addr, mbw, rc.mbw)), x = addr - y * mbw;
        const int fq = uni(udiv_small(f, P.spp, rc.spp)), fk = f - fq * P.spp, fb = f - fk;  // picture fk of the stream whose first slot is fb
        int gx = 1 << 20, gy = 1 << 20;
        if (fk > 0) {  // the reference is a picture of this run (of the same stream)
            gx = min(x + P.reach, mbw - 1);
            gy = min(y + P.reach, mbh - 1);
        }
#if defined(HL_PROFILE)
        const unsigned long long pt1 = __builtin_readcyclecounter();
#endif
        // the left neighbour's chain record was written by another workgroup:
        // vector loads behind the pop's acquire (never the scalar cache)
        const int s_in = uni(x == 0 ? PF.F.spec[y] : ld_relaxed(&PF.F.chain[addr - 1].s_out));
        const int spec_in = uni(x == 0 ? 1 : ld_relaxed(&PF.F.chain[addr - 1].spec));
        HL_POISON(S, (uint32_t)t * 7919u + blockIdx.x);
#if defined(HL_DIAG) && HL_DIAG == 2
        __syncthreads();
#elif defined(HL_DIAG) && HL_DIAG == 3
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#elif defined(HL_DIAG) && HL_DIAG == 4
        __builtin_amdgcn_s_sleep(20);
#elif defined(HL_DIAG) && HL_DIAG == 6
        if (threadIdx.x < 64) __builtin_amdgcn_s_sleep(20);
#endif
        frame_args_to_lds(sF, PF.F, tid);
        // (one call site of encode_mb: the macroblock and its 8x8-family helper
        // share the inlined search)
        if (hk == 1) intra_helper(sF, S, addr, tid, kMbThreads, s_in, PF.F.ispec + addr);
        else encode_mb(sF, S, addr, tid, kMbThreads, s_in, gx, gy, spec_in, hk >= 2 ? PF.F.f3 + addr * 4 + (hk - 2) : nullptr, hk + 1);
        if (helper) {
            // results, every wave's stores drained, barrier, one release, the state
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid < 64) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, HL_REL_SCOPE);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (tid == 0) st_relaxed(hk == 1 ? P.hstate + t : P.hstate3 + 4 * t + hk - 2, HS_DONE);
            }
#if defined(HL_PROFILE)
            pw_hlp += __builtin_readcyclecounter() - pt1;
            ++pw_hn;
            if (hk >= 2) {  // of which the 8x8 family's partitioning helpers
                pw_phlp += __builtin_readcyclecounter() - pt1;
                ++pw_phn;
            }
#endif
            continue;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#if defined(HL_PROFILE)
        if (f == 0 && tid == 0 && prof) {
            prof[64 + nmb + 3 * addr] = pw_start;
            prof[64 + nmb + 3 * addr + 1] = wall_clock64();
        }
#endif
        // (encode_mb stored the record into host memory, PF.F.hrec; the publish fence below is system scope)
#if defined(HL_PROFILE)
        const unsigned long long pt2 = __builtin_readcyclecounter();
#endif
        // Releases successors (Guideline 16: every wave drained, barrier, ONE
        // release whose own wait is explicit, then relaxed atomics: the L2
        // write-back of the release fence covers the payload, and every
        // consumer acquires after its pop): those of this picture (phase 0),
        // of the next one (1), or all (2).  Those whose last dependency this
        // was are queued (with their intra helpers, in P pictures).
        // (two dependent round trips per successor: its counter, then the
        // queue and helper FIFO tails together; the successor picture's kind
        // is read before them)
        auto release = [&](int phase) {
            int fo = 0, xo = 0, yo = 0;
            const int ns = task_succ(fk, x, y, mbw, mbh, P.reach, P.spp, -1, fo, xo, yo);
            for (int j = tid; j < ns; j += 64) {
                task_succ(fk, x, y, mbw, mbh, P.reach, P.spp, j, fo, xo, yo);
                if (phase != 2 && (fo == fk) != (phase == 0)) continue;
                const bool hlp = P.helpers && !(fo == fk ? sF.is_intra : ld_relaxed(&P.fr[fo + fb].F.is_intra));
                const bool h3 = hlp && P.fam3 && (fo < P.f3_first || fo >= P.spp - P.f3_last);
                fo += fb;
                const int a = yo * mbw + xo;
                // the release half is the fence before release(); the acquire
                // half (the other dependencies' writes happen before the push)
                // only where this decrement was the last
                if (__hip_atomic_fetch_add(P.cnt + fo * nmb + a, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 1) continue;
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, HL_ACQ_SCOPE);
                // one stream: sub-queue = the successor's column band (kSubQ
                // bands of MB columns): a workgroup prefers its own (blockIdx %
                // kSubQ), so a band's macroblocks, the plane blocks they write and
                // the reference planes they search stay on two XCDs' L2s.  Several
                // streams: MB address % kSubQ (the bands' preference bent the
                // streams' priorities: 8 streams -4.5 %, profiles/r06_ab_column_bands.log)
                const int qf = fo * kSubQ + (P.nstreams == 1 ? xo * kSubQ / mbw : a % kSubQ);
                const int pos = __hip_atomic_fetch_add(P.tail + qf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // helper kinds: 0 = intra, 1..4 = the 8x8 family's partitioning kind + 2
                const int g = fo * nmb + a, nk = hlp ? (h3 ? 5 : 1) : 0;
                if (h3) {  // the partitioning helpers' states, before the macroblock's push (its pop reads them)
                    int32_t* st = P.hstate3 + 4 * g;
                    st_relaxed(st, HS_FREE);
                    st_relaxed(st + 1, HS_FREE);
                    st_relaxed(st + 2, HS_FREE);
                    st_relaxed(st + 3, HS_FREE);
                }
                int hq[5], hp[5];
#pragma unroll
                for (int k = 0; k < 5; ++k) {
                    hq[k] = (5 * g + k) % kHelperQ;
                    hp[k] = k < nk ? __hip_atomic_fetch_add(P.hq_tail + hq[k], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
                }
                __hip_atomic_store(P.queue + qf * nmb + pos, a + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                for (int k = 0; k < 5; ++k)
                    if (k < nk) __hip_atomic_store(P.hq + hq[k] * P.hq_cap + hp[k], (k << 27) | (g + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
        };
        // This picture's successors need the decision (its reconstruction, MB
        // object, chain record), not this task's deblocking and plane blocks:
        // they are released before those.  The filters then wait for the
        // filters of the in-picture predecessors, which keeps the deblocking
        // in the reference's raster causality (tests/test_pipeline_schedule.py
        // models both events); the next picture still waits for `done`, set
        // after the filters.
        if (tid < 64) {
#if defined(HL_PROFILE)
            const unsigned long long pe0 = __builtin_readcyclecounter();
#endif
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, HL_REL_SCOPE);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if defined(HL_PROFILE)
            const unsigned long long pe1 = __builtin_readcyclecounter();
#endif
            // the predecessors' flags are read before the release's atomics
            // return (their round trips overlap); polled after it if unset
            const int32_t* dA = P.done + t - 1;
            const int32_t* dB = P.done + f * nmb + (y - 1) * mbw + min(x + 1, mbw - 1);
            int vA = 1, vB = 1;
            if (tid == 0) {
                if (x > 0) vA = ld_relaxed(dA);
                if (y > 0) vB = ld_relaxed(dB);
            }
            release(0);
#if defined(HL_PROFILE)
            if (f == 0 && tid == 0 && prof) prof[64 + nmb + 3 * addr + 2] = wall_clock64();
            const unsigned long long pe2 = __builtin_readcyclecounter();
#endif
            if (tid == 0) {
                if (vA < 1) spin_ge(dA, 1, P.err);
                if (vB < 1) spin_ge(dB, 1, P.err);
            }
#if defined(HL_PROFILE)
            const unsigned long long pe3 = __builtin_readcyclecounter();
#endif
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, HL_ACQ_SCOPE);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if defined(HL_PROFILE)
            const unsigned long long pe4 = __builtin_readcyclecounter();
            ptail[4] += pe1 - pe0;
            ptail[5] += pe2 - pe1;
            ptail[6] += pe3 - pe2;
            ptail[7] += pe4 - pe3;
#endif
        }
        __syncthreads();
#if defined(HL_PROFILE)
        const unsigned long long pt2e = __builtin_readcyclecounter();
#endif
        // deblocking, then quarter-pel planes, this decision completed
        task_filters(PF, S, x, y, mbw, mbh, tid);
#if defined(HL_PROFILE)
        pw_wait += pt1 - pt0;
        pw_mb += pt2 - pt1;
        const unsigned long long pw_filt_last = __builtin_readcyclecounter() - pt2;
        pw_filt += pw_filt_last;
        ++pw_n;
#endif
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#if defined(HL_PROFILE)
        const unsigned long long pt3 = __builtin_readcyclecounter();
        unsigned long long pt4 = pt3;
#endif
        if (tid < 64) {
#if HL_HOSTREC_SYS
            if (PF.progress) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // host-visible records (system scope)
            else
#endif
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, HL_REL_SCOPE);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if defined(HL_PROFILE)
            pt4 = __builtin_readcyclecounter();
#endif
            if (tid == 0) {
                st_relaxed(P.done + t, 1);
                // the row's records are in host memory: every MB of rows <= y
                // set its done flag after its system-scope release, and this
                // task's filters waited for (x-1, y) and (x, y-1) (the slice
                // writers consume the picture row by row)
                if (x == mbw - 1 && PF.rows) __hip_atomic_store(PF.rows, y + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            release(1);
            // a stream's pictures finish in order: the last MB depends on every
            // other one and on the previous picture's last MB
            if (tid == 0 && addr == nmb - 1) {
                __hip_atomic_store(P.oldest + fq, fk + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                // every record of the picture is in host memory (each task released at system scope)
                if (PF.progress) __hip_atomic_store(PF.progress, fk + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                if (P.pub_clock) P.pub_clock[f] = wall_clock64();
            }
        }
#if defined(HL_PROFILE)
        {
            const unsigned long long pt5 = __builtin_readcyclecounter();
            ptail[0] += pt3 - pt2 - (pw_filt_last);
            ptail[1] += pt4 - pt3;
            ptail[2] += pt5 - pt4;
            ptail[3] += pt2e - pt2;
        }
#endif
    }
#if defined(HL_PROFILE)
    if (threadIdx.x == 0 && prof) {
        atomicAdd(prof + 40, pw_wait);
        atomicAdd(prof + 41, pw_mb);
        atomicAdd(prof + 42, pw_filt);
        atomicAdd(prof + 43, pw_n);
        atomicAdd(prof + 44, __builtin_readcyclecounter() - pw_t0);
        atomicAdd(prof + 45, pw_hlp);  // intra helper tasks: cycles, count
        atomicAdd(prof + 46, pw_hn);
        atomicAdd(prof + 58, pw_phlp);
        atomicAdd(prof + 59, pw_phn);
        for (int i = 0; i < 3; ++i) atomicAdd(prof + 47 + i, pst[i]);  // pops: attempts, lost, empty rounds
        for (int i = 0; i < 8; ++i) atomicAdd(prof + 50 + i, ptail[i]);  // filters' barrier, release fence, successors, early release (fence, release, spin, acquire)
    }
#endif
}
#undef HL_RC
#undef HL_WAVE0
#undef HL_TID

#if !defined(HL_KERNELS_ONLY)  // (hl_encoder_fam3.hip compiles the kernels above again, with HL_FAM3=1)
extern "C" hipError_t hl_fam3_launch_pipeline(const void* args, size_t psz, int mbw, int mbh, int workgroups, hipStream_t stream);
extern "C" hipError_t hl_fam3_pipeline_occupancy(int* per_cu);
static int diag_count(int mbw, int rows, int diag)
{
    const int ylo = std::max(0, (diag - mbw + 2) / 2);
    const int yhi = std::min(rows - 1, diag / 2);
    return yhi >= ylo ? yhi - ylo + 1 : 0;
}

// ---------------------------------------------------------------------------
// encoder context
// ---------------------------------------------------------------------------
constexpr int kMaxRun = 128;  // pictures per pipelined launch and stream (bench.py MAX_RUN)
#if defined(HL_PROFILE) && defined(HL_BAR_PROF) && HL_BAR_PROF >= 2
constexpr int kProfExtra = 2 * kBarSites;  // per barrier site after the timeline (hl_mbcore.h)
#else
constexpr int kProfExtra = 0;
#endif
constexpr int kRowsAt = 16;   // h_progress word of picture 0's row count

struct hl_amd_encoder_s {
    hl_amd_params_t p;
    int W, H, Wc, Hc, mbw, mbh, nmb, qpc, pstride;
    hipStream_t stream;
    uint8_t* d_in[3];
    uint8_t* d_pic[2][3];  // [cur/ref swap][plane]
    int cur;
    uint8_t* d_pl[4];  // one allocation: d_pl[i] = d_pl[0] + i * plsz
    size_t plsz;
    MbState *d_st, *d_snap;
    MbRecord* d_rec;
    MbChain* d_chain;
    int32_t* d_spec;
    MbRecord* h_rec;
    MbChain* h_chain;
    int32_t* h_spec;
    std::vector<uint8_t> hdr, out, scratch;
    int32_t frame_index, gop_left, pict_count, idr_pic_id, chain_end, reruns;
    int32_t chain_walks;  // resolve_chain walks of the last pipelined run
    bool timing;
    hipEvent_t ev[6];
    float ms[4];
    int32_t mb_launches;
    unsigned long long* d_prof;  // phase counters (HL_PROFILE builds)
    // pipelined runs of P pictures (hl_pipeline.h)
    int pipe_wg, reach, window;  // workgroups (0: one per resident slot), R in MBs, pictures looked at
    int hop;                     // pop order (PipeArgs::hop)
    int bcap;                    // pictures the run buffers hold
    int scap = 0;                // picture slots the scheduler state holds (ensure_sched)
    uint8_t *d_bpic, *d_bpl;     // per picture: recon (Y|U|V), quarter-pel planes
    MbRecord *d_brec, *h_brec, *dh_brec;  // dh_brec: device address of the pinned h_brec (the run writes it)
    int32_t* h_progress;                  // pinned: pictures of the running run whose records are in h_brec;
                                          // [4, 12) the run's error words; [kRowsAt + k] MB rows of picture k
    std::atomic<int> run_live{0};         // 1 while a pipelined run is on the GPU (h_progress counts its pictures)
    std::chrono::steady_clock::time_point run_t0;  // launch time of the running run (writer tracing)
    MbChain *d_bchain, *h_bchain;
    int32_t *d_bspec, *d_err;
    int32_t *d_cnt, *d_done, *d_queue, *d_head;  // scheduler state (cnt: [cnt | claim], head: [head | tail | oldest])
    int32_t* d_hstate = nullptr;                 // intra helper task states [picture][MB] (HS_*)
    IntraSpec* d_ispec = nullptr;                // intra helper results, per MB address
    bool helpers = true;                         // P macroblocks of pipelined runs get intra helper tasks
    int32_t helper_kept = 0, helper_rejected = 0, helper_self = 0;  // hl_amd_last_helper_stats
    int fam3 = 1;                                // ... and 8x8-family helper tasks (HL_AMD_FAM3: 0 off, 2 runs too)
    int32_t fam3_kept = 0, fam3_rejected = 0;    // hl_amd_last_fam3_stats
    Fam3Out* d_f3 = nullptr;                     // 8x8-family partitioning helper results [MB][4] ([slot][MB][4] with HL_AMD_FAM3=2)
    PipeFrame *d_pf, *h_pf;
    std::vector<std::vector<uint8_t>> bout;  // bitstreams of the last hl_amd_encode_batch
    int nwriters;                            // host slice writer threads of a run
    int32_t max_ref_frame = 1;               // hl_codec_t.max_ref_frame: SPS/PPS fields only (hl_amd_set_max_ref_frame)
    std::vector<std::vector<uint8_t>> wscratch, wout;
    std::vector<int32_t> run_intra, run_idr_id;  // per picture of the run: IDR, idr_pic_id
    std::vector<int32_t> run_qp;                 // per picture of the run: SliceQPY (rate control: one picture per run)
    std::vector<SliceBits> run_bits;             // per picture of the run: header / texture bits (rate control)
    // accounting of the last encode call (hl_amd_last_batch_stats)
    int32_t calls_runs = 0, calls_per_picture = 0, calls_fallbacks = 0, calls_gave_up = 0, calls_walks = 0;
    bool run_fallback = false;                   // the last run was re-encoded picture by picture
    bool broken = false;                         // a failed layers batch left the encoder unusable
    // SVC batches: the enhancement-layer thread consumes pictures of a live
    // run; a run that falls back stops it (run_aborted) and waits for the
    // picture it is queuing (el_mu) before the run's buffers are rewritten
    std::atomic<bool> run_aborted{false};
    std::mutex el_mu;
    std::vector<const MbRecord*> last_recs;      // host records per picture of the last encode call (diagnostics)
    std::vector<const MbChain*> last_chain;      // host chain records, same
    std::vector<const uint8_t*> last_pic;        // device recon (Y|U|V planes contiguous) or null = the current reference
    std::unique_ptr<hl::RateControl> rc;         // rate control (rc_bitrate > 0), hl_rc.h
    hl::RcConfig rc_cfg;
    int32_t last_qp;                             // SliceQPY of the last encoded picture
    struct SvcState* svc = nullptr;              // spatial SVC layers (hl_amd_add_layer), else null
    int32_t* d_rows = nullptr;                   // k_deblock_rows: per-row progress [mbh], spin failures [mbh]
    // look-ahead (hl_amd_set_lookahead): host frames queued in device memory
    // and coded `lookahead` at a time as one hl_amd_encode_batch; results
    // handed out one per call, in order
    struct LaOut {
        int32_t type = 0;
        std::vector<uint8_t> hdr, data;
    };
    int32_t lookahead = 1;
    uint8_t* d_la = nullptr;                     // [lookahead] frames, Y | U | V each
    int32_t la_n = 0;                            // frames queued, not yet coded
    std::vector<LaOut> la_out;                   // coded results not yet handed out, from la_head
    size_t la_head = 0;
    LaOut la_cur;                                // the result the last call handed out (valid until the next call)
};

static void svc_free(hl_amd_encoder_t* e);
static hipError_t svc_drain_el(hl_amd_encoder_t* e);
static bool svc_started(const hl_amd_encoder_t* e);

static void free_all(hl_amd_encoder_t* e)
{
    svc_free(e);
    for (int c = 0; c < 3; ++c) {
        (void)hipFree(e->d_in[c]);
        (void)hipFree(e->d_pic[0][c]);
        (void)hipFree(e->d_pic[1][c]);
    }
    (void)hipFree(e->d_pl[0]);
    (void)hipFree(e->d_st);
    (void)hipFree(e->d_snap);
    (void)hipFree(e->d_rec);
    (void)hipFree(e->d_chain);
    (void)hipFree(e->d_spec);
    (void)hipFree(e->d_prof);
    (void)hipFree(e->d_rows);
    (void)hipFree(e->d_la);
    (void)hipFree(e->d_bpic);
    (void)hipFree(e->d_bpl);
    (void)hipFree(e->d_brec);
    (void)hipFree(e->d_bchain);
    (void)hipFree(e->d_bspec);
    (void)hipFree(e->d_err);
    (void)hipFree(e->d_cnt);
    (void)hipFree(e->d_done);
    (void)hipFree(e->d_queue);
    (void)hipFree(e->d_head);
    (void)hipFree(e->d_hstate);
    (void)hipFree(e->d_f3);
    (void)hipFree(e->d_ispec);
    (void)hipFree(e->d_pf);
    (void)hipHostFree(e->h_brec);
    (void)hipHostFree(e->h_bchain);
    (void)hipHostFree(e->h_pf);
    (void)hipHostFree(e->h_rec);
    (void)hipHostFree(e->h_chain);
    (void)hipHostFree(e->h_spec);
    (void)hipHostFree(e->h_progress);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    for (int i = 0; i < 6; ++i)
        if (e->ev[i]) (void)hipEventDestroy(e->ev[i]);
}

extern "C" int32_t hl_amd_encoder_create(const hl_amd_params_t* p, hl_amd_encoder_t** out)
{
    if (!p || !out) return HL_AMD_ERROR_INVALID_PARAMETER;
    *out = nullptr;
    if (p->width <= 0 || p->height <= 0 || (p->width & 15) || (p->height & 15)) return HL_AMD_ERROR_INVALID_FORMAT;
    if (p->qp < 0 || p->qp > 51) return HL_AMD_ERROR_INVALID_PARAMETER;
    // early termination reads the source one sample around the MB quadrants
    // (rdo.c:895-896): the picture needs two MB rows and columns
    if (p->me_early_term && (p->width < 32 || p->height < 32)) return HL_AMD_ERROR_INVALID_FORMAT;
    HL_HIP_CHECK(hipSetDevice(p->device));
    hl_amd_encoder_t* e = new hl_amd_encoder_s();
    e->p = *p;
    e->W = p->width;
    e->H = p->height;
    e->Wc = e->W / 2;
    e->Hc = e->H / 2;
    e->mbw = e->W / 16;
    e->mbh = e->H / 16;
    e->nmb = e->mbw * e->mbh;
    e->qpc = kQpToQpc[p->qp];
    e->pstride = (e->W + 2 * kPad + 63) & ~63;
    const size_t pls = (size_t)e->pstride * (e->H + 2 * kPad);
    // All work of an encoder runs on its own non-blocking stream, which does
    // not order against the null stream: the initial state is written on
    // that stream and synchronised before create returns.
    bool ok = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) == hipSuccess;
    for (int c = 0; c < 3 && ok; ++c) {
        const size_t sz = c ? (size_t)e->Wc * e->Hc : (size_t)e->W * e->H;
        ok = hipMalloc(&e->d_in[c], sz) == hipSuccess && hipMalloc(&e->d_pic[0][c], sz) == hipSuccess &&
             hipMalloc(&e->d_pic[1][c], sz) == hipSuccess && hipMemsetAsync(e->d_pic[0][c], 0, sz, e->stream) == hipSuccess &&
             hipMemsetAsync(e->d_pic[1][c], 0, sz, e->stream) == hipSuccess;
    }
    e->plsz = pls;
    ok = ok && hipMalloc(&e->d_pl[0], 4 * pls) == hipSuccess;
    for (int i = 1; i < 4 && ok; ++i) e->d_pl[i] = e->d_pl[0] + i * pls;
    ok = ok && hipMalloc(&e->d_st, sizeof(MbState) * e->nmb) == hipSuccess && hipMalloc(&e->d_snap, sizeof(MbState) * e->nmb) == hipSuccess &&
         hipMalloc(&e->d_rec, sizeof(MbRecord) * e->nmb) == hipSuccess && hipMalloc(&e->d_chain, sizeof(MbChain) * e->nmb) == hipSuccess &&
         hipMalloc(&e->d_spec, sizeof(int32_t) * e->mbh) == hipSuccess &&
         hipHostMalloc(&e->h_rec, sizeof(MbRecord) * e->nmb, hipHostMallocDefault) == hipSuccess &&
         hipHostMalloc(&e->h_chain, sizeof(MbChain) * e->nmb, hipHostMallocDefault) == hipSuccess &&
         hipHostMalloc(&e->h_spec, sizeof(int32_t) * e->mbh, hipHostMallocDefault) == hipSuccess &&
         hipHostMalloc(&e->h_progress, sizeof(int32_t) * (kRowsAt + kMaxRun), hipHostMallocCoherent) == hipSuccess;
    ok = ok && hipMalloc(&e->d_rows, sizeof(int32_t) * (e->mbh + 1)) == hipSuccess &&
         hipMemsetAsync(e->d_rows, 0, sizeof(int32_t) * (e->mbh + 1), e->stream) == hipSuccess;
    // the per-address MB objects start zeroed (calloc'd by the reference, mb.c)
    ok = ok && hipMemsetAsync(e->d_st, 0, sizeof(MbState) * e->nmb, e->stream) == hipSuccess;
#if defined(HL_PROFILE)
    // 64 phase counters, the cycles of every macroblock of the last frame,
    // then the timeline of the first picture of the last pipelined run (per
    // MB: task start, decision end, in-picture successors released; wall clock)
    ok = ok && hipMalloc(&e->d_prof, (64 + 4 * e->nmb + kProfExtra) * sizeof(unsigned long long)) == hipSuccess &&
         hipMemsetAsync(e->d_prof, 0, (64 + 4 * e->nmb + kProfExtra) * sizeof(unsigned long long), e->stream) == hipSuccess;
#endif
    ok = ok && hipStreamSynchronize(e->stream) == hipSuccess;
    for (int i = 0; i < 6 && ok; ++i) ok = hipEventCreate(&e->ev[i]) == hipSuccess;
    if (!ok) {
        free_all(e);
        delete e;
        return HL_AMD_ERROR_OUTOFMEMMORY;
    }
    {
        const char* wt = getenv("HL_AMD_WRITER_THREADS");
        const unsigned hc = std::thread::hardware_concurrency();
        e->nwriters = wt ? std::max(1, atoi(wt)) : (int)std::max(1u, std::min(16u, hc));
    }
    e->pipe_wg = 0;
    {
        const char* h = getenv("HL_AMD_HELPERS");  // A/B knob (hl_amd_set_intra_helpers)
        e->helpers = !(h && atoi(h) == 0);
        const char* h3 = getenv("HL_AMD_FAM3");  // A/B knob
        e->fam3 = h3 ? atoi(h3) : 1;  // 0 off, 1 lone pictures, 2 runs of one stream too (their first / last pictures, HL_AMD_F3_EDGE)
    }
    e->reach = 2;
    e->window = 64;
    {
        const char* h = getenv("HL_AMD_PIPE_HOP");  // A/B knob of the pop order
        e->hop = h ? atoi(h) : 3 * (e->reach + 2) + 6;  // the staircase lag plus two MB rows (tools/gpu_hop.sh)
    }
    const StreamParams sp{e->W, e->H, p->qp, p->deblock, e->max_ref_frame};
    e->scratch.resize(slice_scratch_bytes(sp));
    e->out.resize(slice_scratch_bytes(sp) + 64);
    e->hdr.resize(256);
    e->hdr.resize(write_stream_headers(sp, e->hdr.data(), e->hdr.size()));
    *out = e;
    return HL_AMD_SUCCESS;
}

extern "C" void hl_amd_encoder_destroy(hl_amd_encoder_t* e)
{
    if (!e) return;
    (void)hipStreamSynchronize(e->stream);
    free_all(e);
    delete e;
}

static void launch_planes(hl_amd_encoder_t* e, const uint8_t* ref_y)
{
    const dim3 grid((e->W + 2 * kPad + kPlTileW - 1) / kPlTileW, (e->H + 2 * kPad + kPlTileH - 1) / kPlTileH);
    k_planes<<<grid, 256, 0, e->stream>>>(ref_y, e->W, e->H, e->d_pl[0], e->pstride, (int)e->plsz);
}

// Launches the MB wavefront for rows [row0, mbh).
static hipError_t run_wavefront(hl_amd_encoder_t* e, const FrameArgs& F, int row0)
{
    const int rows = e->mbh - row0;
    const int ndiag = (e->mbw - 1) + 2 * (rows - 1) + 1;
    for (int d = 0; d < ndiag; ++d) {
        const int n = diag_count(e->mbw, rows, d);
        if (!n) continue;
        k_mb_diag<<<n, kMbThreads, 0, e->stream>>>(F, d, row0);
        ++e->mb_launches;
    }
    return hipGetLastError();
}

// Checks the row-start speculation of rdo.Single_ctr; returns the first row
// to re-run (and fixes its speculated value) or -1 when the frame is exact.
static int validate_chain(hl_amd_encoder_t* e, int row0, int& chain_end)
{
    int carry = e->h_spec[row0];
    for (int y = row0; y < e->mbh; ++y) {
        const MbChain* row = e->h_chain + (size_t)y * e->mbw;
        if (y > row0 && e->h_spec[y] != carry) {
            for (int x = 0; x < e->mbw; ++x) {
                if (row[x].dep) {
                    e->h_spec[y] = carry;
                    return y;
                }
                if (row[x].fresh) break;
            }
        }
        bool any_fresh = false;
        for (int x = 0; x < e->mbw && !any_fresh; ++x) any_fresh = row[x].fresh != 0;
        if (any_fresh) carry = row[e->mbw - 1].s_out;
    }
    chain_end = carry;
    return -1;
}

// The per-picture path: one k_mb_diag launch per anti-diagonal.  It is the
// fallback of a pipelined run (encode_run) whose bounded waits gave up.
// qp_set >= 0: the picture's QP was already taken from the rate controller
// (by the run that fell back); the picture's statistics still go back to it.
static int32_t encode_frame(hl_amd_encoder_t* e, const uint8_t* y, const uint8_t* u, const uint8_t* v, hl_amd_result_t* r,
                            int qp_set = -1)
{
    const bool intra = e->gop_left <= 0;
    if (intra) e->gop_left = e->p.gop_size;
    // rate control picks the picture's QP before it is coded (hl_codec_264.c:719-742)
    const int qp = qp_set >= 0 ? qp_set : (e->rc ? e->rc->begin_picture(intra) : e->p.qp);
    const int qpc = kQpToQpc[qp];
    uint8_t** cur = e->d_pic[e->cur];
    uint8_t** ref = e->d_pic[e->cur ^ 1];
    FrameArgs F{};  // ref_done = null: the per-picture path needs no reference waits
    F.W = e->W;
    F.H = e->H;
    F.Wc = e->Wc;
    F.Hc = e->Hc;
    F.mbw = e->mbw;
    F.mbh = e->mbh;
    F.qp = qp;
    F.qpc = qpc;
    F.is_intra = intra;
    F.me_range = std::min(64, std::max(1, e->p.me_range));
    F.early_term = e->p.me_early_term != 0;
    F.lambda = rdo_lambda(qp);  // slice.c:1766
    F.src[0] = y;
    F.src[1] = u;
    F.src[2] = v;
    for (int c = 0; c < 3; ++c) {
        F.cur[c] = cur[c];
        F.ref[c] = ref[c];
    }
    for (int i = 0; i < 4; ++i) F.pl[i] = e->d_pl[i];
    F.pstride = e->pstride;
    F.plsz = (int32_t)e->plsz;
    F.st = e->d_st;
    F.rec = e->d_rec;
    F.hrec = nullptr;
    F.rec_dev = 1;
    F.chain = e->d_chain;
    F.spec = e->d_spec;
    F.prof = e->d_prof;

    if (e->timing) HL_HIP_CHECK(hipEventRecord(e->ev[0], e->stream));
    if (!intra) {
        launch_planes(e, ref[0]);
        HL_HIP_CHECK(hipGetLastError());
    }
    if (e->timing) HL_HIP_CHECK(hipEventRecord(e->ev[1], e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(e->d_snap, e->d_st, sizeof(MbState) * e->nmb, hipMemcpyDeviceToDevice, e->stream));
    e->h_spec[0] = e->chain_end;
    for (int yy = 1; yy < e->mbh; ++yy) e->h_spec[yy] = 9;
    int row0 = 0, chain_end = 0;
    e->reruns = 0;
    e->mb_launches = 0;
    e->ms[1] = 0.f;
    for (;;) {
        HL_HIP_CHECK(hipMemcpyAsync(e->d_spec, e->h_spec, sizeof(int32_t) * e->mbh, hipMemcpyHostToDevice, e->stream));
        if (e->timing) HL_HIP_CHECK(hipEventRecord(e->ev[4], e->stream));
        HL_HIP_CHECK(run_wavefront(e, F, row0));
        if (e->timing) HL_HIP_CHECK(hipEventRecord(e->ev[5], e->stream));
        HL_HIP_CHECK(hipMemcpyAsync(e->h_chain, e->d_chain, sizeof(MbChain) * e->nmb, hipMemcpyDeviceToHost, e->stream));
        HL_HIP_CHECK(hipStreamSynchronize(e->stream));
        if (e->timing) {
            float t = 0.f;
            (void)hipEventElapsedTime(&t, e->ev[4], e->ev[5]);
            e->ms[1] += t;
        }
        const int bad = validate_chain(e, row0, chain_end);
        if (bad < 0) break;
        ++e->reruns;
        const size_t off = (size_t)bad * e->mbw;
        HL_HIP_CHECK(hipMemcpyAsync(e->d_st + off, e->d_snap + off, sizeof(MbState) * (e->nmb - off), hipMemcpyDeviceToDevice, e->stream));
        row0 = bad;
    }
    e->chain_end = chain_end;
    if (e->timing) HL_HIP_CHECK(hipEventRecord(e->ev[2], e->stream));
    if (e->p.deblock) {
        DeblockArgs D;
        D.W = e->W;
        D.H = e->H;
        D.Wc = e->Wc;
        D.mbw = e->mbw;
        D.qp = qp;
        D.qpc = qpc;
        for (int c = 0; c < 3; ++c) D.pic[c] = cur[c];
        D.st = e->d_st;
        HL_HIP_CHECK(hipMemsetAsync(e->d_rows, 0, sizeof(int32_t) * e->mbh, e->stream));
        k_deblock_rows<<<e->mbh, 64, 0, e->stream>>>(D, e->d_rows, e->d_rows + e->mbh);
        HL_HIP_CHECK(hipGetLastError());
    }
    if (e->timing) HL_HIP_CHECK(hipEventRecord(e->ev[3], e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(e->h_rec, e->d_rec, sizeof(MbRecord) * e->nmb, hipMemcpyDeviceToHost, e->stream));
    HL_HIP_CHECK(hipStreamSynchronize(e->stream));
    if (e->timing) {
        (void)hipEventElapsedTime(&e->ms[0], e->ev[0], e->ev[1]);
        (void)hipEventElapsedTime(&e->ms[2], e->ev[2], e->ev[3]);
        (void)hipEventElapsedTime(&e->ms[3], e->ev[0], e->ev[3]);
    }
    const StreamParams sp{e->W, e->H, e->p.qp, e->p.deblock};
    const SliceState ss{intra ? 1 : 0, e->pict_count, e->idr_pic_id, qp};
    SliceBits sb{};
    const size_t n = write_slice(sp, ss, e->h_rec, e->scratch.data(), e->out.data(), e->out.size(), &sb);
    ++e->calls_per_picture;  // pictures coded on this path (hl_amd_last_batch_stats)
    if (!n) return HL_AMD_ERROR_TOOSHORT;
    if (e->rc) {  // hl_codec_264_rc_end_frame / _end_gop, hl_codec_264.c:1018-1031
        RcPictureStats st{};
        for (int a = 0; a < e->nmb; ++a) st.mad_sum += e->h_rec[a].mad;
        st.header_bits = sb.header_bits;
        st.texture_bits = sb.texture_bits;
        st.nbits = (int32_t)((n - 3) * 8);
        e->rc->end_picture(intra, st, e->gop_left - 1 <= 0);
    }
    e->last_qp = qp;
    r->type = HL_AMD_RESULT_TYPE_DATA;
    r->data = e->out.data() + 3;
    r->data_size = n - 3;
    r->hdr = e->hdr.data();
    r->hdr_size = e->hdr.size();
    if (e->frame_index == 0) r->type |= HL_AMD_RESULT_TYPE_HDR;
    // the reconstructed picture becomes RefPicList0[0]
    e->cur ^= 1;
    ++e->pict_count;
    if (intra) ++e->idr_pic_id;
    --e->gop_left;
    ++e->frame_index;
    return HL_AMD_SUCCESS;
}

// ---------------------------------------------------------------------------
// pipelined runs of P pictures
// ---------------------------------------------------------------------------
constexpr int kMaxStreams = 16;  // streams per launch (hl_amd_encode_streams)

static hipError_t ensure_batch(hl_amd_encoder_t* e, int n)
{
    if (n <= e->bcap) return hipSuccess;
    const size_t pic = (size_t)e->W * e->H * 3 / 2, nmb = e->nmb;
    // Sized for a whole run of kMaxRun pictures at the first batch when that
    // fits in 4 GB of HBM (about 22 MB per 1088p picture, 2.8 GB at 1088p),
    // so that later, longer batches never reallocate between runs.  One
    // picture per call (the plugin path) allocates for one picture.
    // device copies of the records only in diagnostic builds (runs write them
    // to pinned host memory, F.hrec)
#if defined(HL_DIAG_INPUTS)
    const size_t drec = sizeof(MbRecord);
#else
    const size_t drec = 0;
#endif
    const size_t per_pic = pic + 4 * e->plsz + (drec + sizeof(MbChain) + 5 * sizeof(int32_t)) * nmb;
    if (n > 1 && per_pic * kMaxRun <= (4ull << 30)) n = std::max(n, kMaxRun);
    // free and forget every run buffer first, so that a failed allocation
    // below never leaves a dangling pointer for free_all or a later retry
    auto dfree = [](auto*& p) {
        (void)hipFree(p);
        p = nullptr;
    };
    auto hfree = [](auto*& p) {
        (void)hipHostFree(p);
        p = nullptr;
    };
    dfree(e->d_bpic);
    dfree(e->d_bpl);
    dfree(e->d_brec);
    dfree(e->d_bchain);
    dfree(e->d_bspec);
    dfree(e->d_ispec);
    hfree(e->h_brec);
    hfree(e->h_bchain);
    e->bcap = 0;
    hipError_t r;
    if ((r = hipMalloc(&e->d_bpic, pic * n)) || (r = hipMalloc(&e->d_bpl, 4 * e->plsz * n)) ||
        (drec && (r = hipMalloc(&e->d_brec, drec * nmb * n))) || (r = hipMalloc(&e->d_bchain, sizeof(MbChain) * nmb * n)) ||
        (r = hipMalloc(&e->d_bspec, sizeof(int32_t) * e->mbh * n)) ||
        (r = hipHostMalloc(&e->h_brec, sizeof(MbRecord) * nmb * n, hipHostMallocDefault)) ||
        (r = hipHostMalloc(&e->h_bchain, sizeof(MbChain) * nmb * n, hipHostMallocDefault)) ||
        (r = hipMalloc(&e->d_ispec, sizeof(IntraSpec) * nmb)) || (r = hipHostGetDevicePointer((void**)&e->dh_brec, e->h_brec, 0)))
        return r;
    if (!e->d_err && (r = hipMalloc(&e->d_err, sizeof(int32_t) * 8))) return r;
    // defined contents from the start (nothing reads a run buffer before the
    // run writes it; this keeps any such read deterministic)
    if ((r = hipMemsetAsync(e->d_bpic, 0, pic * n, e->stream)) || (r = hipMemsetAsync(e->d_bpl, 0, 4 * e->plsz * n, e->stream)) ||
        (drec && (r = hipMemsetAsync(e->d_brec, 0, drec * nmb * n, e->stream))) ||
        (r = hipMemsetAsync(e->d_bchain, 0, sizeof(MbChain) * nmb * n, e->stream)))
        return r;
    std::vector<int32_t> spec((size_t)e->mbh * n, 9);  // speculated rdo.Single_ctr at every row start
    if ((r = hipMemcpyAsync(e->d_bspec, spec.data(), sizeof(int32_t) * spec.size(), hipMemcpyHostToDevice, e->stream))) return r;
    if ((r = hipStreamSynchronize(e->stream))) return r;
    e->bcap = n;
    return hipSuccess;
}

// The scheduler state of a pipelined launch (hl_pipeline.h) for `slots`
// pictures (of one or several streams), owned by the encoder that launches.
static hipError_t ensure_sched(hl_amd_encoder_t* e, int slots)
{
    if (slots <= e->scap) return hipSuccess;
    const size_t nmb = e->nmb;
    if (slots > 1) slots = std::max(slots, kMaxRun);
    auto dfree = [](auto*& p) {
        (void)hipFree(p);
        p = nullptr;
    };
    dfree(e->d_pf);
    dfree(e->d_cnt);
    dfree(e->d_done);
    dfree(e->d_queue);
    dfree(e->d_head);
    dfree(e->d_hstate);
    dfree(e->d_f3);
    (void)hipHostFree(e->h_pf);
    e->h_pf = nullptr;
    e->scap = 0;
    hipError_t r;
    // (helper states: intra [slot][MB], then the 8x8 family's [slot][MB][4];
    // the helper FIFO sits after the ready queues, five entries per MB)
    if ((r = hipMalloc(&e->d_pf, sizeof(PipeFrame) * slots)) || (r = hipHostMalloc(&e->h_pf, sizeof(PipeFrame) * slots, hipHostMallocDefault)) ||
        (r = hipMalloc(&e->d_cnt, sizeof(int32_t) * 2 * nmb * slots)) || (r = hipMalloc(&e->d_done, sizeof(int32_t) * nmb * slots)) ||
        (r = hipMalloc(&e->d_queue, sizeof(int32_t) * ((kSubQ + 5) * nmb * slots + kHelperQ))) ||
        (r = hipMalloc(&e->d_head, sizeof(int32_t) * (2 * kSubQ * slots + kMaxStreams + 2 * kHelperQ))) ||
        (r = hipMalloc(&e->d_hstate, sizeof(int32_t) * 5 * nmb * slots)) ||
        (r = hipMalloc(&e->d_f3, sizeof(Fam3Out) * 4 * nmb * (e->fam3 >= 2 ? slots : 1))))
        return r;
    if (!e->d_err && (r = hipMalloc(&e->d_err, sizeof(int32_t) * 8))) return r;
    e->scap = slots;
    return hipSuccess;
}

// Exact rdo.Single_ctr walk of one picture whose row starts were speculated
// as `spec`; false when a macroblock read a mispredicted value.
static bool validate_rows(const MbChain* ch, int mbw, int mbh, int spec, int32_t& carry)
{
    for (int y = 0; y < mbh; ++y) {
        const MbChain* row = ch + (size_t)y * mbw;
        if (spec != carry)
            for (int x = 0; x < mbw; ++x) {
                if (row[x].dep) return false;
                if (row[x].fresh) break;
            }
        bool any_fresh = false;
        for (int x = 0; x < mbw && !any_fresh; ++x) any_fresh = row[x].fresh != 0;
        if (any_fresh) carry = row[mbw - 1].s_out;
    }
    return true;
}

static FrameArgs frame_args(hl_amd_encoder_t* e, bool intra, int qp)
{
    FrameArgs F{};
    F.W = e->W;
    F.H = e->H;
    F.Wc = e->Wc;
    F.Hc = e->Hc;
    F.mbw = e->mbw;
    F.mbh = e->mbh;
    F.qp = qp;
    F.qpc = kQpToQpc[qp];
    F.is_intra = intra;
    F.me_range = std::min(64, std::max(1, e->p.me_range));
    F.early_term = e->p.me_early_term != 0;
    F.lambda = rdo_lambda(qp);  // slice.c:1766
    F.pstride = e->pstride;
    F.plsz = (int32_t)e->plsz;
    F.st = e->d_st;
    F.prof = e->d_prof;
    return F;
}

static void store_result(hl_amd_encoder_t* e, int i, const hl_amd_result_t& src, hl_amd_result_t* dst)
{
    e->bout[i].assign((const uint8_t*)src.data, (const uint8_t*)src.data + src.data_size);
    *dst = src;
    dst->data = e->bout[i].data();
}

// Slice writers of a pipelined run: the run's records are in h_brec; worker
// threads serialise its pictures in parallel, each with its own scratch
// buffers, into bout[base + k].  Returns the bytes written per picture
// (start code included; 0 = output buffer too short).
static std::vector<size_t> write_run(hl_amd_encoder_t* e, int m, int base, const std::atomic<bool>* abort = nullptr, int nw = 0)
{
    const int n = std::max(1, std::min(m, nw > 0 ? nw : e->nwriters));
    const StreamParams sp{e->W, e->H, e->p.qp, e->p.deblock};
    if ((int)e->wscratch.size() < n) {
        e->wscratch.resize(n);
        e->wout.resize(n);
    }
    for (int w = 0; w < n; ++w) {
        e->wscratch[w].resize(slice_scratch_bytes(sp));
        e->wout[w].resize(slice_scratch_bytes(sp) + 64);
    }
    std::vector<size_t> size(m, 0);
    std::atomic<int> next{0};
    // during a run: a row of picture k is read once the kernel has put its
    // records in host memory (h_progress[kRowsAt + k] counts the rows)
    struct Gate {
        const int32_t* rows;
        const std::atomic<bool>* abort;
        static bool wait(void* ctx, int r)
        {
            const Gate* g = (const Gate*)ctx;
            while (__atomic_load_n(g->rows, __ATOMIC_ACQUIRE) <= r) {
                if (g->abort->load()) return false;
                std::this_thread::sleep_for(std::chrono::microseconds(20));
            }
            return true;
        }
    };
    auto work = [&](int w) {
        for (int k; (k = next.fetch_add(1)) < m;) {
            Gate g{e->h_progress + kRowsAt + k, abort};
            const RowGate gate{&Gate::wait, &g};
            if (abort && !Gate::wait(&g, 0)) return;
            const SliceState ss{e->run_intra[k], e->pict_count + k, e->run_idr_id[k], e->run_qp[k]};
            uint8_t* out = e->wout[w].data();
            static const bool trace = getenv("HL_AMD_TRACE_WRITERS") != nullptr;
            const auto tk = std::chrono::steady_clock::now();
            const size_t nb = write_slice(sp, ss, e->h_brec + (size_t)e->nmb * k, e->wscratch[w].data(), out, e->wout[w].size(),
                                          &e->run_bits[k], abort ? &gate : nullptr);
            if (!nb && abort && abort->load()) return;
            if (trace)
                fprintf(stderr, "writer %d picture %d: start %.2f ms, write %.2f ms\n", w, k,
                        std::chrono::duration<double, std::milli>(tk - e->run_t0).count(),
                        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tk).count());
            size[k] = nb;
            if (nb) e->bout[base + k].assign(out + 3, out + nb);
        }
    };
    std::vector<std::thread> th;
    for (int w = 1; w < n; ++w) th.emplace_back(work, w);
    work(0);
    for (auto& t : th) t.join();
    return size;
}

// m consecutive pictures (IDR and P, in GOP order) of each of S streams
// (encoders es[s], frames Y[s][k]; the same picture size) in one pipelined
// launch (a single picture too: one persistent launch instead of a launch
// per anti-diagonal): the streams' tasks share the device's workgroups, so
// one stream's ramp and tail overlap the others' work.  Each stream's
// results are those of its own run.  A stream falls back to the per-picture
// path when a row-start speculation turned out to matter (resolve_chain
// makes that exact inside a run), every stream when a bounded wait gave up.
// Under rate control S and m are 1 and the picture's QP comes from the rate
// controller.
static int32_t encode_group(hl_amd_encoder_t* const* es, int S, int m, const uint8_t* const* const* Y, const uint8_t* const* const* U,
                            const uint8_t* const* const* V, hl_amd_result_t* const* res, int base)
{
    hl_amd_encoder_t* e0 = es[0];
    const size_t pic = (size_t)e0->W * e0->H * 3 / 2, nmb = e0->nmb;
    const int slots = S * m;
    // a lone picture runs the kernel built with the 8x8-family helper tasks
    // (hl_encoder_fam3.hip): most workgroups would idle beside its wavefront
    const bool fam3 = e0->helpers && (slots == 1 ? e0->fam3 != 0 : S == 1 && e0->fam3 >= 2);
    for (int si = 0; si < S; ++si) {
        hl_amd_encoder_t* e = es[si];
        if (e->rc && (m != 1 || S != 1)) return HL_AMD_ERROR_INVALID_STATE;
        HL_HIP_CHECK(ensure_batch(e, m));
        // picture types, idr_pic_id and QP of the run, as m encode_frame calls would set them
        e->run_intra.resize(m);
        e->run_idr_id.resize(m);
        e->run_qp.assign(m, e->p.qp);
        e->run_bits.assign(m, SliceBits{});
        for (int k = 0, gl = e->gop_left, idr = e->idr_pic_id; k < m; ++k) {
            const bool intra = gl <= 0;
            if (intra) gl = e->p.gop_size;
            e->run_intra[k] = intra;
            e->run_idr_id[k] = idr;
            idr += intra;
            --gl;
        }
        // rate control picks the picture's QP before it is coded (hl_codec_264.c:719-742)
        if (e->rc) e->run_qp[0] = e->rc->begin_picture(e->run_intra[0] != 0);
        e->run_fallback = false;
        e->run_aborted.store(false, std::memory_order_release);
        if (e->timing) HL_HIP_CHECK(hipEventRecord(e->ev[0], e->stream));
        launch_planes(e, e->d_pic[e->cur ^ 1][0]);  // quarter-pel planes of the picture before the run
        HL_HIP_CHECK(hipGetLastError());
        if (e->timing) HL_HIP_CHECK(hipEventRecord(e->ev[1], e->stream));
        HL_HIP_CHECK(hipMemcpyAsync(e->d_snap, e->d_st, sizeof(MbState) * nmb, hipMemcpyDeviceToDevice, e->stream));
    }
    HL_HIP_CHECK(ensure_sched(e0, slots));
    for (int si = 0; si < S; ++si) HL_HIP_CHECK(hipStreamSynchronize(es[si]->stream));  // (h_pf may still be read by a previous copy)
    struct RunLive {  // cleared on every way out of the run (an error return included),
                      // built before any stream's run_live is set
        hl_amd_encoder_t* const* es;
        int S;
        ~RunLive()
        {
            for (int si = 0; si < S; ++si) es[si]->run_live.store(0, std::memory_order_release);
        }
    } run_live_guard{es, S};
    for (int si = 0; si < S; ++si) {
        hl_amd_encoder_t* e = es[si];
        uint8_t** ref0 = e->d_pic[e->cur ^ 1];
        int32_t* d_progress = nullptr;
        HL_HIP_CHECK(hipHostGetDevicePointer((void**)&d_progress, e->h_progress, 0));
        for (int k = 0; k < m; ++k) {
            const int slot = si * m + k;
            PipeFrame& pf = e0->h_pf[slot];
            pf = PipeFrame{};
            FrameArgs& F = pf.F;
            F = frame_args(e, e->run_intra[k] != 0, e->run_qp[k]);
            uint8_t* cur = e->d_bpic + pic * k;
            F.src[0] = Y[si][k];
            F.src[1] = U[si][k];
            F.src[2] = V[si][k];
            F.cur[0] = cur;
            F.cur[1] = cur + (size_t)e->W * e->H;
            F.cur[2] = cur + (size_t)e->W * e->H * 5 / 4;
            if (k == 0)
                for (int c = 0; c < 3; ++c) F.ref[c] = ref0[c];
            else {
                const uint8_t* rp = e->d_bpic + pic * (k - 1);
                F.ref[0] = rp;
                F.ref[1] = rp + (size_t)e->W * e->H;
                F.ref[2] = rp + (size_t)e->W * e->H * 5 / 4;
            }
            const uint8_t* plb = k == 0 ? e->d_pl[0] : e->d_bpl + 4 * e->plsz * (k - 1);
            for (int i = 0; i < 4; ++i) F.pl[i] = plb + i * e->plsz;
            F.rec = e->d_brec ? e->d_brec + nmb * k : nullptr;
            F.hrec = e->dh_brec + nmb * k;  // the slice writers read the records from host memory during the run
#if defined(HL_DIAG_INPUTS)
            F.rec_dev = 1;
#else
            F.rec_dev = 0;
#endif
            F.chain = e->d_bchain + nmb * k;
            F.spec = e->d_bspec + e->mbh * k;
            F.ref_done = k == 0 ? nullptr : e0->d_done + (slot - 1) * nmb;
            F.ref_epoch = 1;
            F.perr = e0->d_err;
            F.run_done = e0->d_done + (size_t)si * m * nmb;  // this stream's picture 0
            F.run_chain = e->d_bchain;
            F.run_pos = k;
            F.carry_in = e->chain_end;
            if (e0->helpers && !e->run_intra[k]) {
                F.ispec = e->d_ispec;
                F.hstate = e0->d_hstate + nmb * slot;
                if (fam3) {
                    // per MB address and partitioning; per picture too in runs
                    // (a helper may still run after its macroblock ended)
                    F.f3 = e0->d_f3 + (e0->fam3 >= 2 ? (size_t)4 * nmb * slot : 0);
                    F.hstate3 = e0->d_hstate + (size_t)nmb * slots + (size_t)4 * nmb * slot;
                }
            }
            pf.D.W = e->W;
            pf.D.H = e->H;
            pf.D.Wc = e->Wc;
            pf.D.mbw = e->mbw;
            pf.D.qp = F.qp;
            pf.D.qpc = F.qpc;
            for (int c = 0; c < 3; ++c) pf.D.pic[c] = F.cur[c];
            pf.D.st = e->d_st;
            pf.pl_out = e->d_bpl + 4 * e->plsz * k;
            pf.deblock = e->p.deblock;
            pf.progress = d_progress;
            pf.rows = d_progress + kRowsAt + k;
            __atomic_store_n(e->h_progress + kRowsAt + k, 0, __ATOMIC_RELAXED);
        }
        __atomic_store_n(e->h_progress, 0, __ATOMIC_RELEASE);
        e->run_live.store(1, std::memory_order_release);
    }
    HL_HIP_CHECK(hipMemcpyAsync(e0->d_pf, e0->h_pf, sizeof(PipeFrame) * slots, hipMemcpyHostToDevice, e0->stream));
    PipeArgs P;
    P.fr = e0->d_pf;
    P.nframes = slots;
    P.spp = m;
    P.nstreams = S;
    P.reach = e0->reach;
    P.window = e0->window;
    P.hop = e0->hop;
    P.cnt = e0->d_cnt;
    P.claim = e0->d_cnt + nmb * slots;
    P.done = e0->d_done;
    P.queue = e0->d_queue;
    P.hstate = e0->d_hstate;
    P.hstate3 = e0->d_hstate + (size_t)nmb * slots;
    P.helpers = e0->helpers ? 1 : 0;
    P.fam3 = fam3 ? 1 : 0;
    {  // the pictures of a run whose macroblocks get partitioning helpers (every picture of a lone one)
        const char* fe = getenv("HL_AMD_F3_EDGE");  // A/B knob: "first,last" (default 1,2)
        int a = 1, b = 2;
        if (fe) sscanf(fe, "%d,%d", &a, &b);
        P.f3_first = m == 1 ? 1 : a;
        P.f3_last = m == 1 ? 1 : b;
    }
    P.hq = e0->d_queue + kSubQ * nmb * slots;
    P.head = e0->d_head;
    P.tail = e0->d_head + kSubQ * slots;
    P.oldest = e0->d_head + 2 * kSubQ * slots;
    P.hq_cap = (5 * slots * nmb + kHelperQ - 1) / kHelperQ;
    P.hq_head = e0->d_head + 2 * kSubQ * slots + kMaxStreams;
    P.hq_tail = e0->d_head + 2 * kSubQ * slots + kMaxStreams + kHelperQ;
    P.err = e0->d_err;
    static const bool trace = getenv("HL_AMD_TRACE_WRITERS") != nullptr;
    static unsigned long long* h_clock = nullptr;
    P.pub_clock = nullptr;
    if (trace && slots <= 1024) {
        if (!h_clock) HL_HIP_CHECK(hipHostMalloc((void**)&h_clock, sizeof(unsigned long long) * 1024, hipHostMallocCoherent));
        HL_HIP_CHECK(hipHostGetDevicePointer((void**)&P.pub_clock, h_clock, 0));
    }
    // one thread per task, and at least one per sub-queue head / tail and
    // stream word: pictures of fewer than kSubQ macroblocks have more heads
    // than tasks
    const size_t init_threads = std::max({nmb * slots, (size_t)kSubQ * slots, (size_t)kMaxStreams});
    k_pipe_init<<<(unsigned)((init_threads + 255) / 256), 256, 0, e0->stream>>>(P, e0->mbw, e0->mbh);
    HL_HIP_CHECK(hipGetLastError());
    static const int env_wg = getenv("HL_AMD_PIPE_WG") ? atoi(getenv("HL_AMD_PIPE_WG")) : 0;  // experiments
    int wgs = e0->pipe_wg > 0 ? e0->pipe_wg : env_wg;
    if (wgs <= 0) {  // one workgroup per resident slot of the device
        int dev = 0, cus = 0, occ = 0;
        HL_HIP_CHECK(hipGetDevice(&dev));
        HL_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        if (fam3) HL_HIP_CHECK(hl_fam3_pipeline_occupancy(&occ));  // the build that is launched
        else HL_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_pipeline, kMbThreads, 0));
        wgs = std::max(1, cus * occ);
    }
    if (e0->timing) HL_HIP_CHECK(hipEventRecord(e0->ev[4], e0->stream));
    for (int si = 0; si < S; ++si) es[si]->run_t0 = std::chrono::steady_clock::now();
    if (fam3) HL_HIP_CHECK(hl_fam3_launch_pipeline(&P, sizeof(P), e0->mbw, e0->mbh, wgs, e0->stream));
    else k_pipeline<<<wgs, kMbThreads, 0, e0->stream>>>(P, e0->mbw, e0->mbh);
    HL_HIP_CHECK(hipGetLastError());
    if (e0->timing) HL_HIP_CHECK(hipEventRecord(e0->ev[5], e0->stream));
    // The kernel stores every finished MB's record into pinned host memory and
    // counts each stream's finished pictures in a host-mapped word: writer
    // threads serialise each picture's slice as soon as it is complete, while
    // the run goes on.  The chain records and the give-up counter come back
    // after the run (pinned: the copies are asynchronous -- a copy into
    // pageable memory blocks the host until the kernel ends, and with it the
    // writers).
    int32_t* errw = e0->h_progress + 4;  // bounded waits that gave up, resolve_chain walks, helper counts
    for (int si = 0; si < S; ++si)
        HL_HIP_CHECK(hipMemcpyAsync(es[si]->h_bchain, es[si]->d_bchain, sizeof(MbChain) * nmb * m, hipMemcpyDeviceToHost, e0->stream));
    HL_HIP_CHECK(hipMemcpyAsync(errw, e0->d_err, 8 * sizeof(int32_t), hipMemcpyDeviceToHost, e0->stream));
    if (e0->timing) HL_HIP_CHECK(hipEventRecord(e0->ev[2], e0->stream));
    std::vector<std::atomic<bool>> abort(S);
    std::vector<std::vector<size_t>> wsize(S);
    std::vector<std::thread> writers;
    for (int si = 0; si < S; ++si) {
        abort[si] = false;
        writers.emplace_back([&, si] { wsize[si] = write_run(es[si], m, base, &abort[si], std::max(1, es[si]->nwriters / S)); });
    }
    const hipError_t serr = hipStreamSynchronize(e0->stream);
    for (int si = 0; si < S; ++si) es[si]->run_live.store(0, std::memory_order_release);
    const auto tw0 = std::chrono::steady_clock::now();
    bool aborted = false;
    for (int si = 0; si < S; ++si)
        if (serr != hipSuccess || __atomic_load_n(es[si]->h_progress, __ATOMIC_ACQUIRE) < m) {
            abort[si] = true;
            aborted = true;
        }
    for (auto& w : writers) w.join();
    if (e0->timing) e0->ms[3] = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - tw0).count();
    if (trace && P.pub_clock)
        for (int f = 0; f < slots; ++f) fprintf(stderr, "picture %d published at device clock +%.2f ms\n", f, (h_clock[f] - h_clock[0]) * 1e-5);
    HL_HIP_CHECK(serr);
    if (aborted) {
        fprintf(stderr, "hartallo_amd: pipelined run ended before every picture was published\n");
        return HL_AMD_ERROR_SYSTEM;
    }
    if (e0->timing) {
        (void)hipEventElapsedTime(&e0->ms[0], e0->ev[0], e0->ev[1]);
        (void)hipEventElapsedTime(&e0->ms[1], e0->ev[4], e0->ev[5]);
        (void)hipEventElapsedTime(&e0->ms[2], e0->ev[5], e0->ev[2]);
    }
    const int32_t err = errw[0];
    if (err) fprintf(stderr, "hartallo_amd: pipelined run: %d bounded waits gave up; re-encoding the run picture by picture\n", err);
    const bool force_fb = getenv("HL_AMD_FORCE_FALLBACK")  // (read per run: tests set it per case)
                           && atoi(getenv("HL_AMD_FORCE_FALLBACK")) > 0;
    // which streams keep their run (else they are re-coded picture by
    // picture below), and every kept stream's slices fit, before any stream
    // commits: the streams of a group advance together or not at all
    std::vector<char> keep(S);
    std::vector<int32_t> carry_out(S);
    for (int si = 0; si < S; ++si) {
        int32_t carry = es[si]->chain_end;
        bool ok = err == 0;
        for (int k = 0; k < m && ok; ++k) ok = validate_rows(es[si]->h_bchain + nmb * k, es[si]->mbw, es[si]->mbh, 9, carry);
        if (force_fb) ok = false;  // diagnostics: HL_AMD_FORCE_FALLBACK=1 takes the fallback below for every run (tests)
        keep[si] = ok;
        carry_out[si] = carry;
        for (int k = 0; k < m && ok; ++k)
            if (!wsize[si][k]) return HL_AMD_ERROR_TOOSHORT;
    }
    // a stream whose fallback fails after earlier streams committed leaves
    // the group out of step: every encoder of the group is then unusable
    struct GroupGuard {
        hl_amd_encoder_t* const* es;
        int S;
        bool done = false;
        ~GroupGuard()
        {
            if (!done && S > 1)
                for (int si = 0; si < S; ++si) es[si]->broken = true;
        }
    } group_guard{es, S};
    for (int si = 0; si < S; ++si) {
        hl_amd_encoder_t* e = es[si];
        // the launch's counters (shared by its streams)
        e->chain_walks = errw[1];
        e->mb_launches = 1;
        e->reruns = 0;
        ++e->calls_runs;
        e->calls_gave_up += err;
        e->calls_walks += errw[1];
        e->helper_kept += errw[2];
        e->helper_rejected += errw[3];
        e->helper_self += errw[4];
        e->fam3_kept += errw[5];
        e->fam3_rejected += errw[6];
        if (si) {
            e->ms[1] = e0->ms[1];
            e->ms[3] = e0->ms[3];
        }
        const int32_t carry = carry_out[si];
        if (!keep[si]) {  // a speculated row start mattered (or a wait gave up): redo the stream's run picture by picture
            e->run_fallback = true;
            ++e->calls_fallbacks;
            // an SVC batch's enhancement-layer thread may be coding from this
            // run's pictures: stop it and drain what it queued before they are
            // rewritten (hl_amd_encode_layers_batch re-codes those layers)
            e->run_aborted.store(true, std::memory_order_release);
            {
                std::lock_guard<std::mutex> lk(e->el_mu);
                HL_HIP_CHECK(svc_drain_el(e));
            }
            HL_HIP_CHECK(hipMemcpyAsync(e->d_st, e->d_snap, sizeof(MbState) * nmb, hipMemcpyDeviceToDevice, e->stream));
            for (int k = 0; k < m; ++k) {
                hl_amd_result_t rr;
                // under rate control the run's picture already has its QP (m == 1)
                const int32_t rc = encode_frame(e, Y[si][k], U[si][k], V[si][k], &rr, e->rc ? e->run_qp[k] : -1);
                if (rc) return rc;
                store_result(e, base + k, rr, &res[si][k]);
                // keep every picture's records and reconstruction in the run
                // buffers, as the pipelined run would (diagnostics, and the
                // reference layer of hl_amd_encode_layers_batch)
                memcpy(e->h_brec + nmb * k, e->h_rec, sizeof(MbRecord) * nmb);
                memcpy(e->h_bchain + nmb * k, e->h_chain, sizeof(MbChain) * nmb);
                uint8_t* dst = e->d_bpic + pic * k;
                const size_t ys = (size_t)e->W * e->H, cs = ys / 4;
                uint8_t** rp = e->d_pic[e->cur ^ 1];
                HL_HIP_CHECK(hipMemcpyAsync(dst, rp[0], ys, hipMemcpyDeviceToDevice, e->stream));
                HL_HIP_CHECK(hipMemcpyAsync(dst + ys, rp[1], cs, hipMemcpyDeviceToDevice, e->stream));
                HL_HIP_CHECK(hipMemcpyAsync(dst + ys + cs, rp[2], cs, hipMemcpyDeviceToDevice, e->stream));
                e->last_recs[base + k] = e->h_brec + nmb * k;
                e->last_chain[base + k] = e->h_bchain + nmb * k;
                e->last_pic[base + k] = dst;
            }
            e->reruns = 1;
            continue;
        }
        for (int k = 0; k < m; ++k) {
            e->last_recs[base + k] = e->h_brec + nmb * k;
            e->last_chain[base + k] = e->h_bchain + nmb * k;
            e->last_pic[base + k] = e->d_bpic + pic * k;
        }
        for (int k = 0; k < m; ++k) {
            hl_amd_result_t& o = res[si][k];
            o.type = HL_AMD_RESULT_TYPE_DATA;
            o.data = e->bout[base + k].data();
            o.data_size = e->bout[base + k].size();
            o.hdr = e->hdr.data();
            o.hdr_size = e->hdr.size();
            if (e->frame_index == 0) o.type |= HL_AMD_RESULT_TYPE_HDR;
            if (e->run_intra[k]) e->gop_left = e->p.gop_size;  // encode_frame's bookkeeping, picture by picture
            if (e->rc) {  // hl_codec_264_rc_end_frame / _end_gop, hl_codec_264.c:1018-1031
                RcPictureStats st{};
                const MbRecord* rr = e->h_brec + nmb * k;
                for (size_t a = 0; a < nmb; ++a) st.mad_sum += rr[a].mad;
                st.header_bits = e->run_bits[k].header_bits;
                st.texture_bits = e->run_bits[k].texture_bits;
                st.nbits = (int32_t)((wsize[si][k] - 3) * 8);
                e->rc->end_picture(e->run_intra[k] != 0, st, e->gop_left - 1 <= 0);
            }
            e->last_qp = e->run_qp[k];
            ++e->pict_count;
            if (e->run_intra[k]) ++e->idr_pic_id;
            --e->gop_left;
            ++e->frame_index;
        }
        e->chain_end = carry;
        // the last picture of the run becomes the reference
        uint8_t** dst = e->d_pic[e->cur];
        const uint8_t* last = e->d_bpic + pic * (m - 1);
        HL_HIP_CHECK(hipMemcpyAsync(dst[0], last, (size_t)e->W * e->H, hipMemcpyDeviceToDevice, e->stream));
        HL_HIP_CHECK(hipMemcpyAsync(dst[1], last + (size_t)e->W * e->H, (size_t)e->Wc * e->Hc, hipMemcpyDeviceToDevice, e->stream));
        HL_HIP_CHECK(hipMemcpyAsync(dst[2], last + (size_t)e->W * e->H * 5 / 4, (size_t)e->Wc * e->Hc, hipMemcpyDeviceToDevice, e->stream));
        HL_HIP_CHECK(hipStreamSynchronize(e->stream));
        e->cur ^= 1;
    }
    group_guard.done = true;
    return HL_AMD_SUCCESS;
}

static int32_t encode_run(hl_amd_encoder_t* e, int m, const uint8_t* const* Y, const uint8_t* const* U, const uint8_t* const* V,
                          hl_amd_result_t* res, int base)
{
    return encode_group(&e, 1, m, &Y, &U, &V, &res, base);
}

static void begin_call(hl_amd_encoder_t* e, int n)
{
    e->bout.resize(n);
    e->last_recs.assign(n, nullptr);
    e->last_chain.assign(n, nullptr);
    e->last_pic.assign(n, nullptr);
    e->calls_runs = e->calls_per_picture = e->calls_fallbacks = e->calls_gave_up = e->calls_walks = 0;
    e->helper_kept = e->helper_rejected = e->helper_self = 0;
    e->fam3_kept = e->fam3_rejected = 0;
}

// n consecutive pictures of the stream, every one through a pipelined run:
// runs span GOPs (IDR pictures included), kMaxRun bounds the run's buffers
// (~22 MB of HBM and 9 MB of pinned host memory per 1088p picture); under
// rate control every run is one picture (its QP needs the previous
// picture's bits).  Results are those of n per-picture calls.
static int32_t encode_pictures(hl_amd_encoder_t* e, int n, const uint8_t* const* y, const uint8_t* const* u, const uint8_t* const* v,
                               hl_amd_result_t* results)
{
    if (e->broken) return HL_AMD_ERROR_INVALID_STATE;
    begin_call(e, n);
    for (int i = 0; i < n;) {
        const int m = e->rc ? 1 : std::min(n - i, kMaxRun);
        const int32_t rc = encode_run(e, m, y + i, u + i, v + i, results + i, i);
        if (rc) return rc;
        i += m;
    }
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_encode_streams(hl_amd_encoder_t* const* encoders, int32_t count, int32_t n, const uint8_t* const* y,
                                         const uint8_t* const* u, const uint8_t* const* v, hl_amd_result_t* results)
{
    if (!encoders || count <= 0 || count > kMaxStreams || n <= 0 || !y || !u || !v || !results) return HL_AMD_ERROR_INVALID_PARAMETER;
    for (int i = 0; i < count * n; ++i)
        if (!y[i] || !u[i] || !v[i]) return HL_AMD_ERROR_INVALID_PARAMETER;
    for (int s = 0; s < count; ++s) {
        hl_amd_encoder_t* e = encoders[s];
        if (!e) return HL_AMD_ERROR_INVALID_PARAMETER;
        for (int t = 0; t < s; ++t)
            if (encoders[t] == e) return HL_AMD_ERROR_INVALID_PARAMETER;
        if (e->W != encoders[0]->W || e->H != encoders[0]->H || e->p.device != encoders[0]->p.device) return HL_AMD_ERROR_INVALID_FORMAT;
        if (e->rc || e->svc || e->broken) return HL_AMD_ERROR_INVALID_STATE;
    }
    for (int s = 0; s < count; ++s) begin_call(encoders[s], n);
    std::vector<const uint8_t* const*> Y(count), U(count), V(count);
    std::vector<hl_amd_result_t*> R(count);
    for (int i = 0; i < n;) {
        const int m = std::min(n - i, kMaxRun);
        for (int s = 0; s < count; ++s) {
            Y[s] = y + (size_t)s * n + i;
            U[s] = u + (size_t)s * n + i;
            V[s] = v + (size_t)s * n + i;
            R[s] = results + (size_t)s * n + i;
        }
        const int32_t rc = encode_group(encoders, count, m, Y.data(), U.data(), V.data(), R.data(), i);
        if (rc) return rc;
        i += m;
    }
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_last_batch_stats(hl_amd_encoder_t* e, int32_t* out5)
{
    if (!e || !out5) return HL_AMD_ERROR_INVALID_PARAMETER;
    out5[0] = e->calls_runs;
    out5[1] = e->calls_per_picture;
    out5[2] = e->calls_fallbacks;
    out5[3] = e->calls_gave_up;
    out5[4] = e->calls_walks;
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_last_fam3_stats(hl_amd_encoder_t* e, int32_t* out2)
{
    if (!e || !out2) return HL_AMD_ERROR_INVALID_PARAMETER;
    out2[0] = e->fam3_kept;
    out2[1] = e->fam3_rejected;
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_last_helper_stats(hl_amd_encoder_t* e, int32_t* out3)
{
    if (!e || !out3) return HL_AMD_ERROR_INVALID_PARAMETER;
    out3[0] = e->helper_kept;
    out3[1] = e->helper_rejected;
    out3[2] = e->helper_self;
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_set_intra_helpers(hl_amd_encoder_t* e, int32_t enable)
{
    if (!e) return HL_AMD_ERROR_INVALID_PARAMETER;
    e->helpers = enable != 0;
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_encode_batch(hl_amd_encoder_t* e, int32_t n, const uint8_t* const* y, const uint8_t* const* u,
                                       const uint8_t* const* v, hl_amd_result_t* results)
{
    if (!e || n <= 0 || !y || !u || !v || !results) return HL_AMD_ERROR_INVALID_PARAMETER;
    for (int i = 0; i < n; ++i)
        if (!y[i] || !u[i] || !v[i]) return HL_AMD_ERROR_INVALID_PARAMETER;
    if (e->la_n) return HL_AMD_ERROR_INVALID_STATE;  // frames still queued by the look-ahead come first (hl_amd_flush)
    return encode_pictures(e, n, y, u, v, results);
}

extern "C" int32_t hl_amd_set_max_ref_frame(hl_amd_encoder_t* e, int32_t max_ref_frame)
{
    // any value: the SPS carries min(MaxDpbMbs / PicSizeInMbs, max_ref_frame)
    // (sps.c:635-636); refused only when that value itself is above 16 (the
    // enhancement layers are larger pictures: their value is never higher)
    if (!e || max_ref_frame < 0 || sps_max_num_ref_frames(e->W, e->H, max_ref_frame) > 16) return HL_AMD_ERROR_INVALID_PARAMETER;
    // the reference reads it once, when it builds the first SPS (sps.c:620-636)
    if (e->frame_index != 0 || svc_started(e)) return HL_AMD_ERROR_INVALID_STATE;
    e->max_ref_frame = max_ref_frame;
    const StreamParams sp{e->W, e->H, e->p.qp, e->p.deblock, e->max_ref_frame};
    e->hdr.resize(256);
    e->hdr.resize(write_stream_headers(sp, e->hdr.data(), e->hdr.size()));
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_set_rate_control(hl_amd_encoder_t* e, int64_t bitrate, int32_t fps_num, int32_t fps_den,
                                           int32_t basicunit, int32_t qp_min, int32_t qp_max)
{
    if (!e) return HL_AMD_ERROR_INVALID_PARAMETER;
    if (e->frame_index != 0) return HL_AMD_ERROR_INVALID_STATE;  // the model starts with the first GOP
    if (bitrate <= 0) {
        e->rc.reset();
        return HL_AMD_SUCCESS;
    }
    if (fps_num <= 0 || fps_den <= 0 || fps_den / fps_num <= 0) return HL_AMD_ERROR_INVALID_PARAMETER;
    e->rc_cfg = hl::RcConfig{bitrate, fps_num, fps_den, basicunit, qp_min, qp_max, e->p.gop_size, e->W, e->H};
    e->rc.reset(new hl::RateControl(e->rc_cfg));
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_last_qp(hl_amd_encoder_t* e) { return e ? e->last_qp : -1; }

extern "C" int32_t hl_amd_set_pipeline(hl_amd_encoder_t* e, int32_t workgroups, int32_t reach, int32_t window)
{
    if (!e || workgroups < 0 || workgroups > 4096 || reach < 0 || reach > 16 || window < 1 || window > 64)
        return HL_AMD_ERROR_INVALID_PARAMETER;
    e->pipe_wg = workgroups;
    e->reach = reach;
    e->window = window;
    return HL_AMD_SUCCESS;
}

// Resident workgroups per CU of the pipelined kernel (HIP occupancy query).
extern "C" int32_t hl_amd_pipeline_occupancy(void)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_pipeline, kMbThreads, 0) != hipSuccess) return -1;
    return n;
}

// One picture per call (the plugin's encode(), hl_codec.c:152-159): a
// pipelined run of one picture -- one persistent launch whose workgroups take
// the picture's macroblocks as they become ready, with deblocking and the
// next reference's quarter-pel planes fused into the tasks.
extern "C" int32_t hl_amd_encode_device(hl_amd_encoder_t* e, const uint8_t* y, const uint8_t* u, const uint8_t* v, hl_amd_result_t* r)
{
    if (!e || !y || !u || !v || !r) return HL_AMD_ERROR_INVALID_PARAMETER;
    if (e->la_n) return HL_AMD_ERROR_INVALID_STATE;  // frames still queued by the look-ahead come first (hl_amd_flush)
    return encode_pictures(e, 1, &y, &u, &v, r);
}

// Look-ahead: the queued frames as one batch; every result copied out (a
// batch's result data is valid only until the next call)
static int32_t la_run(hl_amd_encoder_t* e)
{
    const int n = e->la_n;
    if (!n) return HL_AMD_SUCCESS;
    e->la_n = 0;
    const size_t ny = (size_t)e->W * e->H, nc = (size_t)e->Wc * e->Hc;
    std::vector<const uint8_t*> y(n), u(n), v(n);
    for (int i = 0; i < n; ++i) {
        y[i] = e->d_la + (ny + 2 * nc) * i;
        u[i] = y[i] + ny;
        v[i] = u[i] + nc;
    }
    std::vector<hl_amd_result_t> res(n);
    const int32_t rc = encode_pictures(e, n, y.data(), u.data(), v.data(), res.data());
    if (rc) return rc;
    if (e->la_head == e->la_out.size()) {
        e->la_out.clear();
        e->la_head = 0;
    }
    for (const hl_amd_result_t& r : res) {
        hl_amd_encoder_s::LaOut o;
        o.type = r.type;
        if (r.type & HL_AMD_RESULT_TYPE_HDR) o.hdr.assign(r.hdr, r.hdr + r.hdr_size);
        if (r.type & HL_AMD_RESULT_TYPE_DATA) o.data.assign(r.data, r.data + r.data_size);
        e->la_out.push_back(std::move(o));
    }
    return HL_AMD_SUCCESS;
}

// the next coded result, or TYPE 0 (nothing yet)
static void la_pop(hl_amd_encoder_t* e, hl_amd_result_t* r)
{
    memset(r, 0, sizeof(*r));
    if (e->la_head == e->la_out.size()) return;
    e->la_cur = std::move(e->la_out[e->la_head++]);
    r->type = e->la_cur.type;
    if (r->type & HL_AMD_RESULT_TYPE_HDR) {
        r->hdr = e->la_cur.hdr.data();
        r->hdr_size = e->la_cur.hdr.size();
    }
    if (r->type & HL_AMD_RESULT_TYPE_DATA) {
        r->data = e->la_cur.data.data();
        r->data_size = e->la_cur.data.size();
    }
}

extern "C" int32_t hl_amd_set_lookahead(hl_amd_encoder_t* e, int32_t frames)
{
    if (!e || frames < 1 || frames > 128) return HL_AMD_ERROR_INVALID_PARAMETER;
    if (e->frame_index != 0 || e->la_n || svc_started(e) || e->svc) return HL_AMD_ERROR_INVALID_STATE;  // before the first frame, AVC only
    (void)hipFree(e->d_la);
    e->d_la = nullptr;
    e->lookahead = frames;
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_flush(hl_amd_encoder_t* e, hl_amd_result_t* r)
{
    if (!e || !r) return HL_AMD_ERROR_INVALID_PARAMETER;
    const int32_t rc = la_run(e);
    if (rc) return rc;
    la_pop(e, r);
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_encode(hl_amd_encoder_t* e, const uint8_t* y, const uint8_t* u, const uint8_t* v, hl_amd_result_t* r)
{
    if (!e || !y || !u || !v || !r) return HL_AMD_ERROR_INVALID_PARAMETER;
    if (e->lookahead > 1) {  // queue the frame (copied: the caller may reuse its buffer), code a full queue
        const size_t ny = (size_t)e->W * e->H, nc = (size_t)e->Wc * e->Hc, fb = ny + 2 * nc;
        if (!e->d_la) HL_HIP_CHECK(hipMalloc(&e->d_la, fb * e->lookahead));
        uint8_t* d = e->d_la + fb * e->la_n;
        HL_HIP_CHECK(hipMemcpyAsync(d, y, ny, hipMemcpyHostToDevice, e->stream));
        HL_HIP_CHECK(hipMemcpyAsync(d + ny, u, nc, hipMemcpyHostToDevice, e->stream));
        HL_HIP_CHECK(hipMemcpyAsync(d + ny + nc, v, nc, hipMemcpyHostToDevice, e->stream));
        HL_HIP_CHECK(hipStreamSynchronize(e->stream));
        if (++e->la_n == e->lookahead) {
            const int32_t rc = la_run(e);
            if (rc) return rc;
        }
        la_pop(e, r);
        return HL_AMD_SUCCESS;
    }
    HL_HIP_CHECK(hipMemcpyAsync(e->d_in[0], y, (size_t)e->W * e->H, hipMemcpyHostToDevice, e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(e->d_in[1], u, (size_t)e->Wc * e->Hc, hipMemcpyHostToDevice, e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(e->d_in[2], v, (size_t)e->Wc * e->Hc, hipMemcpyHostToDevice, e->stream));
    const uint8_t *dy = e->d_in[0], *du = e->d_in[1], *dv = e->d_in[2];
    return encode_pictures(e, 1, &dy, &du, &dv, r);
}

extern "C" int32_t hl_amd_get_recon(hl_amd_encoder_t* e, uint8_t* y, uint8_t* u, uint8_t* v)
{
    if (!e || !y || !u || !v) return HL_AMD_ERROR_INVALID_PARAMETER;
    uint8_t** ref = e->d_pic[e->cur ^ 1];
    HL_HIP_CHECK(hipMemcpyAsync(y, ref[0], (size_t)e->W * e->H, hipMemcpyDeviceToHost, e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(u, ref[1], (size_t)e->Wc * e->Hc, hipMemcpyDeviceToHost, e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(v, ref[2], (size_t)e->Wc * e->Hc, hipMemcpyDeviceToHost, e->stream));
    HL_HIP_CHECK(hipStreamSynchronize(e->stream));
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_set_timing(hl_amd_encoder_t* e, int32_t enable)
{
    if (!e) return HL_AMD_ERROR_INVALID_PARAMETER;
    e->timing = enable != 0;
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_get_timing(hl_amd_encoder_t* e, float* ms4)
{
    if (!e || !ms4) return HL_AMD_ERROR_INVALID_PARAMETER;
    memcpy(ms4, e->ms, sizeof(e->ms));
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_last_reruns(hl_amd_encoder_t* e) { return e ? e->reruns : -1; }
extern "C" int32_t hl_amd_last_chain_walks(hl_amd_encoder_t* e) { return e ? e->chain_walks : -1; }

// k_planes alone (the HBM-bound kernel of the path): `iters` launches on the
// encoder's current reference picture and stream, timed with HIP events;
// *ms = average milliseconds per launch.  Diagnostics, no reference interface.
extern "C" int32_t hl_amd_bench_planes(hl_amd_encoder_t* e, int32_t iters, float* ms)
{
    if (!e || iters <= 0 || !ms) return HL_AMD_ERROR_INVALID_PARAMETER;
    hipEvent_t a, b;
    HL_HIP_CHECK(hipEventCreate(&a));
    HL_HIP_CHECK(hipEventCreate(&b));
    const uint8_t* ref = e->d_pic[e->cur ^ 1][0];
    launch_planes(e, ref);  // warm
    HL_HIP_CHECK(hipEventRecord(a, e->stream));
    for (int i = 0; i < iters; ++i) launch_planes(e, ref);
    HL_HIP_CHECK(hipEventRecord(b, e->stream));
    HL_HIP_CHECK(hipGetLastError());
    HL_HIP_CHECK(hipEventSynchronize(b));
    float t = 0.f;
    (void)hipEventElapsedTime(&t, a, b);
    *ms = t / iters;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_last_mb_launches(hl_amd_encoder_t* e) { return e ? e->mb_launches : -1; }

// Phase cycle counters of HL_PROFILE builds (zeros otherwise): 64 phase
// counters, then (n > 64) the cycles of each macroblock of the last frame.
extern "C" int32_t hl_amd_profile_counters(hl_amd_encoder_t* e, unsigned long long* out, int32_t n)
{
    if (!e || !out || n < 0 || n > 64 + 4 * e->nmb + kProfExtra) return HL_AMD_ERROR_INVALID_PARAMETER;
    memset(out, 0, sizeof(unsigned long long) * n);
    if (!e->d_prof) return HL_AMD_SUCCESS;
    HL_HIP_CHECK(hipMemcpy(out, e->d_prof, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost));
    HL_HIP_CHECK(hipMemset(e->d_prof, 0, sizeof(unsigned long long) * 64));
    if (kProfExtra) HL_HIP_CHECK(hipMemset(e->d_prof + 64 + 4 * e->nmb, 0, sizeof(unsigned long long) * kProfExtra));
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_debug_records(hl_amd_encoder_t* e, int32_t k, void* out, size_t bytes)
{
    if (!e || !out || k < 0) return HL_AMD_ERROR_INVALID_PARAMETER;
    if (k >= (int)e->last_recs.size() || !e->last_recs[k]) return HL_AMD_ERROR_INVALID_STATE;
    if (bytes != sizeof(MbRecord) * (size_t)e->nmb) return HL_AMD_ERROR_INVALID_PARAMETER;
    memcpy(out, e->last_recs[k], bytes);
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_record_size(void) { return (int32_t)sizeof(MbRecord); }

extern "C" int32_t hl_amd_debug_chain(hl_amd_encoder_t* e, int32_t k, void* out, size_t bytes)
{
    if (!e || !out || k < 0) return HL_AMD_ERROR_INVALID_PARAMETER;
    if (k >= (int)e->last_chain.size() || !e->last_chain[k]) return HL_AMD_ERROR_INVALID_STATE;
    if (bytes != sizeof(MbChain) * (size_t)e->nmb) return HL_AMD_ERROR_INVALID_PARAMETER;
    memcpy(out, e->last_chain[k], bytes);
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_debug_recon(hl_amd_encoder_t* e, int32_t k, uint8_t* y, uint8_t* u, uint8_t* v)
{
    if (!e || !y || !u || !v || k < 0) return HL_AMD_ERROR_INVALID_PARAMETER;
    if (k >= (int)e->last_pic.size()) return HL_AMD_ERROR_INVALID_STATE;
    const uint8_t* p = e->last_pic[k];
    if (!p) {
        if (k != (int)e->last_pic.size() - 1) return HL_AMD_ERROR_INVALID_STATE;
        return hl_amd_get_recon(e, y, u, v);
    }
    const size_t ny = (size_t)e->W * e->H, nc = (size_t)e->Wc * e->Hc;
    HL_HIP_CHECK(hipMemcpyAsync(y, p, ny, hipMemcpyDeviceToHost, e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(u, p + ny, nc, hipMemcpyDeviceToHost, e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(v, p + ny + nc, nc, hipMemcpyDeviceToHost, e->stream));
    HL_HIP_CHECK(hipStreamSynchronize(e->stream));
    return HL_AMD_SUCCESS;
}

extern "C" const char* hl_amd_version(void) { return "hartallo_amd 0.1 (gfx950)"; }

// ---------------------------------------------------------------------------
// Spatial SVC (hl_svc.h).  The encoder codes layer 0 as the AVC base layer
// (encode_frame, plus a prefix NAL unit) and every enhancement layer with one
// k_svc_mb launch over all its macroblocks, then deblocking.  Like the
// reference (hl_codec_264.c:470-1018) the caller passes one frame per layer
// and access unit, base first; the access unit's bytes come back with the
// last layer's call.  For layer-sharded runs (one rank per layer) an encoder
// codes only layers [first, last] and imports the layer below first from the
// rank that coded it (hl_amd_export_layer / hl_amd_import_layer).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_svc_mb(SvcArgs A)
{
    __shared__ SvcShared S;
    svc_encode_mb(A, S, blockIdx.x, threadIdx.x, 64);
}

// Enhancement-layer slice data on the GPU (hl_cavlc.h): bit count of every
// macroblock_layer(), an exclusive scan, then every macroblock writes its
// bits at its offset.  One lane per macroblock.
__global__ __launch_bounds__(64) void k_el_count(const MbRecord* __restrict__ rec, int nmb, int mbw, int idr, int64_t* len)
{
    const int a = blockIdx.x * 64 + threadIdx.x;
    if (a >= nmb) return;
    BitCount bc;
    el_mb_bits(bc, rec, a, mbw, idr != 0);
    len[a] = bc.pos;
}

// in-place exclusive scan of v[0, n), v[n] = the total (one workgroup)
__global__ __launch_bounds__(1024) void k_scan_excl(int64_t* v, int n)
{
    __shared__ int64_t part[1024];
    const int t = threadIdx.x, per = (n + 1023) / 1024, lo = t * per, hi = lo + per < n ? lo + per : n;
    int64_t sum = 0;
    for (int i = lo; i < hi; ++i) sum += v[i];
    part[t] = sum;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele scan of the partial sums
        const int64_t x = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    int64_t run = t ? part[t - 1] : 0;
    for (int i = lo; i < hi; ++i) {
        const int64_t x = v[i];
        v[i] = run;
        run += x;
    }
    if (t == 1023) v[n] = part[1023];
}

__global__ __launch_bounds__(64) void k_el_write(const MbRecord* __restrict__ rec, int nmb, int mbw, int idr, const int64_t* off,
                                                 uint32_t* words)
{
    const int a = blockIdx.x * 64 + threadIdx.x;
    if (a >= nmb) return;
    BitOr bo{words, off[a]};
    el_mb_bits(bo, rec, a, mbw, idr != 0);
}

struct SvcLayerDev {
    int W, H, Wc, Hc, mbw, mbh, nmb, pstride;
    size_t plsz;
    SvcGeom g;
    uint8_t* d_in[3];
    uint8_t* d_pic[2][3];
    int cur;
    uint8_t* d_pl;
    MbState* d_st;
    MbRecord *d_rec, *h_rec;
    int pict_count;
    std::vector<uint8_t> scratch, out;
    hipEvent_t ev_rec = nullptr, ev_t0 = nullptr, ev_t1 = nullptr;  // slice bits on the host; kernel span (timing)
    int64_t* d_len;                 // per MB bit counts, scanned in place; [nmb] = the total
    uint32_t *d_words, *h_words;    // slice data bits (big-endian words), device / pinned copy of the first esd_size bytes
    int64_t* h_total;               // pinned: total data bits
    int32_t* d_rows;                // k_deblock_rows progress [mbh] + spin failures
    size_t words_bytes, esd_size;
    std::future<size_t> writing;  // the slice, written by a host thread while the GPU codes the next layer
    uint8_t* d_snap;              // the reference picture at the start of a layers batch (its redo after a base re-encode)
};

struct SvcState {
    std::vector<int32_t> w, h;       // layer sizes, [0] = the encoder's own
    std::vector<SvcLayerDev> el;     // layers 1.. (allocated when the first frame is coded)
    int first = 0, last = -1;        // layers coded here; the layer below first is imported
    int next = 0;                    // layer the next call must code
    int hdr_layers = 0;              // layers whose header NAL units were signalled
    int gop_left = 0;                // access-unit GOP counter when the base layer is imported
    bool au_intra = false;
    bool started = false;
    std::vector<uint8_t> au, hdr;
    int32_t* d_unpinned = nullptr;
    int32_t unpinned = 0;
    float ms_el = 0.f;               // enhancement-layer device time of the last access unit
    // hl_amd_encode_layers_batch: the base layer of access unit i as the
    // reference layer (picture of the base run, MB objects from its records)
    uint8_t* ref0_pic[3] = {nullptr, nullptr, nullptr};
    const MbState* ref0_st = nullptr;
    // MB objects of a batch's base pictures (device, pinned staging)
    MbState *d_bst = nullptr, *h_bst = nullptr;
    size_t bst_cap = 0;
    std::vector<std::vector<uint8_t>> bau, bhdr;    // access units / header bytes of the last batch
    std::vector<std::vector<uint8_t>> elau, elhdr;  // their enhancement-layer slices / header NAL units
    // the enhancement layers run on a stream of their own; `linked`: every
    // enhancement-layer picture is ordered after the work queued on the
    // encoder's stream and before what is queued there next (one stream's
    // semantics, hl_amd_encode_layer); hl_amd_encode_layers_batch unlinks
    // them to code access unit i's enhancement layers while the base run
    // goes on with the pictures after i
    hipStream_t est = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_base = nullptr;
    bool linked = true;
    int pipe_wg = 128;  // workgroups of a batch's base run: the rest of the device codes the enhancement layers
};

static bool svc_started(const hl_amd_encoder_t* e) { return e->svc && e->svc->started; }

static void svc_free(hl_amd_encoder_t* e)
{
    SvcState* s = e->svc;
    if (!s) return;
    for (SvcLayerDev& L : s->el) {
        for (int c = 0; c < 3; ++c) {
            (void)hipFree(L.d_in[c]);
            (void)hipFree(L.d_pic[0][c]);
            (void)hipFree(L.d_pic[1][c]);
        }
        (void)hipFree(L.d_pl);
        (void)hipFree(L.d_st);
        (void)hipFree(L.d_snap);
        if (L.writing.valid()) L.writing.wait();
        (void)hipFree(L.d_len);
        (void)hipFree(L.d_rows);
        (void)hipFree(L.d_words);
        (void)hipHostFree(L.h_words);
        (void)hipHostFree(L.h_total);
        (void)hipFree(L.d_rec);
        (void)hipHostFree(L.h_rec);
        if (L.ev_rec) (void)hipEventDestroy(L.ev_rec);
        if (L.ev_t0) (void)hipEventDestroy(L.ev_t0);
        if (L.ev_t1) (void)hipEventDestroy(L.ev_t1);
    }
    (void)hipFree(s->d_unpinned);
    (void)hipFree(s->d_bst);
    (void)hipHostFree(s->h_bst);
    if (s->ev_base) (void)hipEventDestroy(s->ev_base);
    if (s->ev_fork) (void)hipEventDestroy(s->ev_fork);
    if (s->ev_join) (void)hipEventDestroy(s->ev_join);
    if (s->est) (void)hipStreamDestroy(s->est);
    delete s;
    e->svc = nullptr;
}

// waits for the enhancement-layer work queued on the layers' own stream
static hipError_t svc_drain_el(hl_amd_encoder_t* e)
{
    return e->svc && e->svc->est ? hipStreamSynchronize(e->svc->est) : hipSuccess;
}

static int32_t svc_alloc(hl_amd_encoder_t* e)
{
    SvcState* s = e->svc;
    s->el = std::vector<SvcLayerDev>(s->w.size() - 1);  // value-initialised: null pointers until allocated
    bool ok = hipMalloc(&s->d_unpinned, sizeof(int32_t)) == hipSuccess &&
              hipMemsetAsync(s->d_unpinned, 0, sizeof(int32_t), e->stream) == hipSuccess &&
              hipStreamCreateWithFlags(&s->est, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&s->ev_fork, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&s->ev_join, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&s->ev_base, hipEventDisableTiming) == hipSuccess;
    for (size_t l = 1; l < s->w.size() && ok; ++l) {
        SvcLayerDev& L = s->el[l - 1];
        L.W = s->w[l];
        L.H = s->h[l];
        L.Wc = L.W / 2;
        L.Hc = L.H / 2;
        L.mbw = L.W / 16;
        L.mbh = L.H / 16;
        L.nmb = L.mbw * L.mbh;
        L.pstride = (L.W + 2 * kPad + 63) & ~63;
        L.plsz = (size_t)L.pstride * (L.H + 2 * kPad);
        L.g = svc_geom(L.W, L.H, s->w[l - 1], s->h[l - 1], stream_level_idc(L.W, L.H));
        for (int c = 0; c < 3 && ok; ++c) {
            const size_t sz = c ? (size_t)L.Wc * L.Hc : (size_t)L.W * L.H;
            ok = hipMalloc(&L.d_in[c], sz) == hipSuccess && hipMalloc(&L.d_pic[0][c], sz) == hipSuccess &&
                 hipMalloc(&L.d_pic[1][c], sz) == hipSuccess && hipMemsetAsync(L.d_pic[0][c], 0, sz, e->stream) == hipSuccess &&
                 hipMemsetAsync(L.d_pic[1][c], 0, sz, e->stream) == hipSuccess;
        }
        ok = ok && hipMalloc(&L.d_pl, 4 * L.plsz) == hipSuccess && hipMalloc(&L.d_st, sizeof(MbState) * L.nmb) == hipSuccess &&
             hipMemsetAsync(L.d_st, 0, sizeof(MbState) * L.nmb, e->stream) == hipSuccess &&
             hipMalloc(&L.d_rec, sizeof(MbRecord) * L.nmb) == hipSuccess &&
             hipHostMalloc(&L.h_rec, sizeof(MbRecord) * L.nmb, hipHostMallocDefault) == hipSuccess &&
             hipEventCreateWithFlags(&L.ev_rec, hipEventDisableTiming) == hipSuccess && hipEventCreate(&L.ev_t0) == hipSuccess &&
             hipEventCreate(&L.ev_t1) == hipSuccess;
        // slice data: at most ~1.5 KB per macroblock (16 luma + 10 chroma
        // CAVLC blocks); the reference's slice buffer holds (nmb << 8) + 4096
        // bytes (encode.c:192), bits past it are dropped (write_svc_slice_bits)
        L.esd_size = ((size_t)L.nmb << 8) + 4096;
        L.words_bytes = (size_t)L.nmb * 2048 + 4096;
        ok = ok && hipMalloc(&L.d_len, sizeof(int64_t) * (L.nmb + 1)) == hipSuccess && hipMalloc(&L.d_words, L.words_bytes) == hipSuccess &&
             hipHostMalloc(&L.h_words, L.esd_size + 64, hipHostMallocDefault) == hipSuccess &&
             hipHostMalloc(&L.h_total, sizeof(int64_t), hipHostMallocDefault) == hipSuccess &&
             hipMalloc(&L.d_rows, sizeof(int32_t) * (L.mbh + 1)) == hipSuccess &&
             hipMalloc(&L.d_snap, (size_t)L.W * L.H * 3 / 2) == hipSuccess &&
             hipMemsetAsync(L.d_rows, 0, sizeof(int32_t) * (L.mbh + 1), e->stream) == hipSuccess;
        const StreamParams sp{L.W, L.H, e->p.qp, e->p.deblock};
        L.scratch.resize(slice_scratch_bytes(sp));
        L.out.resize(slice_scratch_bytes(sp) + 64);
        L.cur = 0;
        L.pict_count = 0;
    }
    ok = ok && hipStreamSynchronize(e->stream) == hipSuccess;
    return ok ? HL_AMD_SUCCESS : HL_AMD_ERROR_OUTOFMEMMORY;
}

// current (deblocked) picture and macroblock objects of layer l
static void svc_layer_ptrs(hl_amd_encoder_t* e, int l, uint8_t* const*& pic, MbState*& st, int& W, int& H, int& nmb)
{
    if (l == 0 && e->svc->ref0_st) {
        pic = e->svc->ref0_pic;
        st = const_cast<MbState*>(e->svc->ref0_st);
        W = e->W;
        H = e->H;
        nmb = e->nmb;
    }
    else if (l == 0) {
        pic = e->d_pic[e->cur ^ 1];
        st = e->d_st;
        W = e->W;
        H = e->H;
        nmb = e->nmb;
    }
    else {
        SvcLayerDev& L = e->svc->el[l - 1];
        pic = L.d_pic[L.cur ^ 1];
        st = L.d_st;
        W = L.W;
        H = L.H;
        nmb = L.nmb;
    }
}

// one enhancement-layer picture: planes, k_svc_mb, deblocking, records, slice
static int32_t svc_encode_el(hl_amd_encoder_t* e, int l, const uint8_t* y, const uint8_t* u, const uint8_t* v)
{
    SvcState* s = e->svc;
    SvcLayerDev& L = s->el[l - 1];
    const bool intra = s->au_intra;
    const int qp = e->p.qp, qpc = kQpToQpc[qp];
    uint8_t** cur = L.d_pic[L.cur];
    uint8_t** ref = L.d_pic[L.cur ^ 1];
    uint8_t* const* rpic;
    MbState* rst;
    int rW, rH, rn;
    svc_layer_ptrs(e, l - 1, rpic, rst, rW, rH, rn);
    if (rW * 2 != L.W || rH * 2 != L.H) return HL_AMD_ERROR_INVALID_STATE;
    hipStream_t st = s->est;
    if (s->linked) {
        HL_HIP_CHECK(hipEventRecord(s->ev_fork, e->stream));
        HL_HIP_CHECK(hipStreamWaitEvent(st, s->ev_fork, 0));
    }
    HL_HIP_CHECK(hipEventRecord(L.ev_t0, st));
    if (!intra) {
        const dim3 grid((L.W + 2 * kPad + kPlTileW - 1) / kPlTileW, (L.H + 2 * kPad + kPlTileH - 1) / kPlTileH);
        k_planes<<<grid, 256, 0, st>>>(ref[0], L.W, L.H, L.d_pl, L.pstride, (int)L.plsz);
        HL_HIP_CHECK(hipGetLastError());
    }
    SvcArgs A{};
    A.g = L.g;
    FrameArgs& F = A.F;
    F.W = L.W;
    F.H = L.H;
    F.Wc = L.Wc;
    F.Hc = L.Hc;
    F.mbw = L.mbw;
    F.mbh = L.mbh;
    F.qp = qp;
    F.qpc = qpc;
    F.is_intra = intra;
    F.src[0] = y;
    F.src[1] = u;
    F.src[2] = v;
    for (int c = 0; c < 3; ++c) {
        F.cur[c] = cur[c];
        F.ref[c] = ref[c];
        A.rl[c] = rpic[c];
    }
    for (int i = 0; i < 4; ++i) F.pl[i] = L.d_pl + i * L.plsz;
    F.pstride = L.pstride;
    F.plsz = (int32_t)L.plsz;
    F.st = L.d_st;
    F.rec = L.d_rec;
    A.rst = rst;
    A.unpinned = s->d_unpinned;
    k_svc_mb<<<L.nmb, 64, 0, st>>>(A);
    HL_HIP_CHECK(hipGetLastError());
    if (e->p.deblock) {
        DeblockArgs D;
        D.W = L.W;
        D.H = L.H;
        D.Wc = L.Wc;
        D.mbw = L.mbw;
        D.qp = qp;
        D.qpc = qpc;
        for (int c = 0; c < 3; ++c) D.pic[c] = cur[c];
        D.st = L.d_st;
        HL_HIP_CHECK(hipMemsetAsync(L.d_rows, 0, sizeof(int32_t) * L.mbh, st));
        k_deblock_rows<<<L.mbh, 64, 0, st>>>(D, L.d_rows, L.d_rows + L.mbh);
        HL_HIP_CHECK(hipGetLastError());
    }
    // slice data serialised on the GPU (hl_cavlc.h)
    {
        const int nb = (L.nmb + 63) / 64;
        HL_HIP_CHECK(hipMemsetAsync(L.d_words, 0, L.words_bytes, st));
        k_el_count<<<nb, 64, 0, st>>>(L.d_rec, L.nmb, L.mbw, intra, L.d_len);
        k_scan_excl<<<1, 1024, 0, st>>>(L.d_len, L.nmb);
        k_el_write<<<nb, 64, 0, st>>>(L.d_rec, L.nmb, L.mbw, intra, L.d_len, L.d_words);
        HL_HIP_CHECK(hipGetLastError());
    }
    HL_HIP_CHECK(hipEventRecord(L.ev_t1, st));
    HL_HIP_CHECK(hipMemcpyAsync(L.h_total, L.d_len + L.nmb, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HL_HIP_CHECK(hipMemcpyAsync(L.h_words, L.d_words, L.esd_size + 64, hipMemcpyDeviceToHost, st));
    HL_HIP_CHECK(hipMemcpyAsync(&s->unpinned, s->d_unpinned, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HL_HIP_CHECK(hipEventRecord(L.ev_rec, st));
    if (s->linked) {
        HL_HIP_CHECK(hipEventRecord(s->ev_join, st));
        HL_HIP_CHECK(hipStreamWaitEvent(e->stream, s->ev_join, 0));
    }
    // the header, trailing bits and escaping are added by a host thread once
    // the bits arrived, while the GPU codes the layers above; joined by the
    // access unit's last call
    const StreamParams sp{L.W, L.H, qp, e->p.deblock};
    const SvcSliceState ss{intra ? 1 : 0, L.pict_count, 0, qp, l};  // idr_pic_id: encode.c:527-530 counts type-5 slices only
    const int threads = e->nwriters;
    L.writing = std::async(std::launch::async, [&L, sp, ss, threads]() -> size_t {
        if (hipEventSynchronize(L.ev_rec) != hipSuccess) return 0;
        const int64_t bits = *L.h_total;
        if ((bits >> 3) + 64 < (int64_t)L.esd_size)
            return write_svc_slice_bits(sp, ss, L.h_words, bits, L.scratch.data(), L.out.data(), L.out.size());
        // a slice past the reference's slice buffer: the host writer reproduces its truncation
        if (hipMemcpy(L.h_rec, L.d_rec, sizeof(MbRecord) * L.nmb, hipMemcpyDeviceToHost) != hipSuccess) return 0;
        return write_svc_slice(sp, ss, L.h_rec, L.scratch.data(), L.out.data(), L.out.size(), threads);
    });
    L.cur ^= 1;
    ++L.pict_count;
    return HL_AMD_SUCCESS;
}

// joins the slice writers of layers [first, last] of the access unit and
// appends their slices to it
static int32_t svc_join(hl_amd_encoder_t* e, int upto)
{
    SvcState* s = e->svc;
    static const uint8_t scp[3] = {0, 0, 1};
    int32_t rc = HL_AMD_SUCCESS;
    for (int l = std::max(1, s->first); l <= upto; ++l) {
        SvcLayerDev& L = s->el[l - 1];
        if (!L.writing.valid()) continue;
        const size_t n = L.writing.get();
        if (!n) {
            rc = HL_AMD_ERROR_TOOSHORT;
            continue;
        }
        if (!s->au.empty()) s->au.insert(s->au.end(), scp, scp + 3);
        s->au.insert(s->au.end(), L.out.data() + 3, L.out.data() + n);
        if (e->timing) {
            float t = 0.f;
            (void)hipEventElapsedTime(&t, L.ev_t0, L.ev_t1);
            s->ms_el += t;
        }
    }
    return rc;
}

extern "C" int32_t hl_amd_add_layer(hl_amd_encoder_t* e, int32_t width, int32_t height)
{
    if (!e || width <= 0 || height <= 0) return HL_AMD_ERROR_INVALID_PARAMETER;
    if (e->frame_index > 0 || e->la_n || (e->svc && e->svc->started)) return HL_AMD_ERROR_INVALID_STATE;
    e->lookahead = 1;  // (the look-ahead is AVC only: an encoder with layers ignores it)
    if (!e->svc) e->svc = new SvcState();
    SvcState* s = e->svc;
    if ((int)s->w.size() >= 4) return HL_AMD_ERROR_OUTOFCAPACITY;  // HL_ENCODER_MAX_LAYERS
    if (s->w.empty()) {
        if (width != e->W || height != e->H) return HL_AMD_ERROR_INVALID_PARAMETER;  // the base layer is the encoder's size
    }
    else {
        const int pw = s->w.back(), ph = s->h.back();
        if (pw >= width || ph >= height) return HL_AMD_ERROR_INVALID_PARAMETER;  // increasing (hl_codec.c:107-112)
        const int rw = width / pw, rh = height / ph;
        if ((rw & (rw - 1)) || (rh & (rh - 1))) return HL_AMD_ERROR_INVALID_PARAMETER;  // power of 2 (hl_codec.c:113-121)
        if (width != 2 * pw || height != 2 * ph || (width & 15) || (height & 15)) return HL_AMD_ERROR_NOT_IMPLEMENTED;  // dyadic only
    }
    s->w.push_back(width);
    s->h.push_back(height);
    s->last = (int)s->w.size() - 1;
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_set_layer_range(hl_amd_encoder_t* e, int32_t first, int32_t last)
{
    if (!e || !e->svc) return HL_AMD_ERROR_INVALID_STATE;
    SvcState* s = e->svc;
    if (s->started) return HL_AMD_ERROR_INVALID_STATE;
    if (first < 0 || last < first || last >= (int)s->w.size()) return HL_AMD_ERROR_INVALID_PARAMETER;
    s->first = first;
    s->last = last;
    return HL_AMD_SUCCESS;
}

static int32_t svc_start(hl_amd_encoder_t* e)
{
    SvcState* s = e->svc;
    if (s->started) return HL_AMD_SUCCESS;
    if (e->rc) return HL_AMD_ERROR_NOT_IMPLEMENTED;
    const int32_t rc = svc_alloc(e);
    if (rc != HL_AMD_SUCCESS) return rc;
    s->started = true;
    s->next = s->first;
    s->hdr_layers = 0;
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_encode_layer(hl_amd_encoder_t* e, int32_t width, int32_t height, const uint8_t* y, const uint8_t* u,
                                       const uint8_t* v, int32_t on_device, hl_amd_result_t* r)
{
    if (!e || !y || !u || !v || !r) return HL_AMD_ERROR_INVALID_PARAMETER;
    SvcState* s = e->svc;
    if (!s || s->w.size() < 2) {
        if (width != e->W || height != e->H) return HL_AMD_ERROR_INVALID_FORMAT;
        return on_device ? hl_amd_encode_device(e, y, u, v, r) : hl_amd_encode(e, y, u, v, r);
    }
    int l = -1;
    for (size_t i = 0; i < s->w.size(); ++i)
        if (s->w[i] == width && s->h[i] == height) l = (int)i;
    if (l < 0) return HL_AMD_ERROR_NOT_FOUND;  // hl_codec_264.c:470-481
    int32_t rc = svc_start(e);
    if (rc != HL_AMD_SUCCESS) return rc;
    if (l != s->next || l < s->first || l > s->last) return HL_AMD_ERROR_INVALID_STATE;
    r->type = 0;
    r->data = nullptr;
    r->data_size = 0;
    r->hdr = nullptr;
    r->hdr_size = 0;
    if (l == 0) {
        s->au_intra = e->gop_left <= 0;
        s->ms_el = 0.f;
        hl_amd_result_t b{};
        rc = on_device ? hl_amd_encode_device(e, y, u, v, &b) : hl_amd_encode(e, y, u, v, &b);
        if (rc != HL_AMD_SUCCESS) return rc;
        if (b.type & HL_AMD_RESULT_TYPE_HDR) {
            s->hdr.assign(b.hdr, b.hdr + b.hdr_size);
            s->hdr_layers = 1;
            r->type |= HL_AMD_RESULT_TYPE_HDR;
        }
        uint8_t pre[5];
        write_prefix_nal(s->au_intra, pre);
        s->au.assign(pre, pre + 5);
        static const uint8_t scp[3] = {0, 0, 1};
        s->au.insert(s->au.end(), scp, scp + 3);
        s->au.insert(s->au.end(), b.data, b.data + b.data_size);
        // encode_frame counted this picture against the GOP; the reference
        // decrements gop_left once per access unit, at its last layer
        ++e->gop_left;
    }
    else {
        SvcLayerDev& L = s->el[l - 1];
        if (!on_device) {
            HL_HIP_CHECK(hipMemcpyAsync(L.d_in[0], y, (size_t)L.W * L.H, hipMemcpyHostToDevice, e->stream));
            HL_HIP_CHECK(hipMemcpyAsync(L.d_in[1], u, (size_t)L.Wc * L.Hc, hipMemcpyHostToDevice, e->stream));
            HL_HIP_CHECK(hipMemcpyAsync(L.d_in[2], v, (size_t)L.Wc * L.Hc, hipMemcpyHostToDevice, e->stream));
            y = L.d_in[0];
            u = L.d_in[1];
            v = L.d_in[2];
        }
        if (l == s->first) s->au.clear();
        rc = svc_encode_el(e, l, y, u, v);
        if (rc != HL_AMD_SUCCESS) return rc;
        if (l >= s->hdr_layers) {  // hl_codec_264.c:577-687: a new (subset) SPS and PPS
            s->hdr.resize(1024);
            const StreamParams bp{s->w[0], s->h[0], e->p.qp, e->p.deblock, e->max_ref_frame};
            s->hdr.resize(write_svc_headers(bp, s->w.data(), s->h.data(), l + 1, s->hdr.data(), s->hdr.size()));
            s->hdr_layers = l + 1;
            r->type |= HL_AMD_RESULT_TYPE_HDR;
        }
    }
    if (r->type & HL_AMD_RESULT_TYPE_HDR) {
        r->hdr = s->hdr.data();
        r->hdr_size = s->hdr.size();
    }
    if (l == s->last) {
        rc = svc_join(e, l);
        if (rc != HL_AMD_SUCCESS) return rc;
        r->type |= HL_AMD_RESULT_TYPE_DATA;
        r->data = s->au.data();
        r->data_size = s->au.size();
        s->next = s->first;
        if (s->first == 0) --e->gop_left;
        else --s->gop_left;
    }
    else {
        s->next = l + 1;
    }
    return HL_AMD_SUCCESS;
}

extern "C" int32_t hl_amd_svc_unpinned(hl_amd_encoder_t* e) { return e && e->svc ? e->svc->unpinned : -1; }

extern "C" int32_t hl_amd_get_layer_recon(hl_amd_encoder_t* e, int32_t layer, uint8_t* y, uint8_t* u, uint8_t* v)
{
    if (!e || !y || !u || !v) return HL_AMD_ERROR_INVALID_PARAMETER;
    if (layer == 0) return hl_amd_get_recon(e, y, u, v);
    if (!e->svc || !e->svc->started || layer < 1 || layer >= (int)e->svc->w.size()) return HL_AMD_ERROR_INVALID_PARAMETER;
    uint8_t* const* pic;
    MbState* st;
    int W, H, n;
    svc_layer_ptrs(e, layer, pic, st, W, H, n);
    HL_HIP_CHECK(hipMemcpyAsync(y, pic[0], (size_t)W * H, hipMemcpyDeviceToHost, e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(u, pic[1], (size_t)W * H / 4, hipMemcpyDeviceToHost, e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(v, pic[2], (size_t)W * H / 4, hipMemcpyDeviceToHost, e->stream));
    HL_HIP_CHECK(hipStreamSynchronize(e->stream));
    return HL_AMD_SUCCESS;
}

// state a layer hands to the layer above: its picture (Y|U|V) and its
// macroblock objects
extern "C" size_t hl_amd_layer_state_bytes(hl_amd_encoder_t* e, int32_t layer)
{
    if (!e || !e->svc || layer < 0 || layer >= (int)e->svc->w.size()) return 0;
    const size_t W = e->svc->w[layer], H = e->svc->h[layer];
    return W * H * 3 / 2 + sizeof(MbState) * (W / 16) * (H / 16);
}

extern "C" int32_t hl_amd_export_layer(hl_amd_encoder_t* e, int32_t layer, void* dst)
{
    if (!e || !dst || !hl_amd_layer_state_bytes(e, layer)) return HL_AMD_ERROR_INVALID_PARAMETER;
    int32_t rc = svc_start(e);
    if (rc != HL_AMD_SUCCESS) return rc;
    uint8_t* const* pic;
    MbState* st;
    int W, H, n;
    svc_layer_ptrs(e, layer, pic, st, W, H, n);
    uint8_t* d = (uint8_t*)dst;
    const size_t ys = (size_t)W * H, cs = ys / 4;
    HL_HIP_CHECK(hipMemcpyAsync(d, pic[0], ys, hipMemcpyDeviceToDevice, e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(d + ys, pic[1], cs, hipMemcpyDeviceToDevice, e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(d + ys + cs, pic[2], cs, hipMemcpyDeviceToDevice, e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(d + ys + 2 * cs, st, sizeof(MbState) * n, hipMemcpyDeviceToDevice, e->stream));
    HL_HIP_CHECK(hipStreamSynchronize(e->stream));
    return HL_AMD_SUCCESS;
}

// The layer below `first` of this access unit, coded elsewhere: it becomes
// that layer's current picture and macroblock objects, and starts the
// access unit (its IDR decision follows the GOP like the base layer's).
extern "C" int32_t hl_amd_import_layer(hl_amd_encoder_t* e, int32_t layer, const void* src)
{
    if (!e || !src || !e->svc || !hl_amd_layer_state_bytes(e, layer)) return HL_AMD_ERROR_INVALID_PARAMETER;
    SvcState* s = e->svc;
    int32_t rc = svc_start(e);
    if (rc != HL_AMD_SUCCESS) return rc;
    if (layer != s->first - 1 || s->next != s->first) return HL_AMD_ERROR_INVALID_STATE;
    int W, H, n;
    uint8_t** pic;
    MbState* st;
    if (layer == 0) {
        pic = e->d_pic[e->cur];
        st = e->d_st;
        W = e->W;
        H = e->H;
        n = e->nmb;
        e->cur ^= 1;
    }
    else {
        SvcLayerDev& L = s->el[layer - 1];
        pic = L.d_pic[L.cur];
        st = L.d_st;
        W = L.W;
        H = L.H;
        n = L.nmb;
        L.cur ^= 1;
    }
    const uint8_t* d = (const uint8_t*)src;
    const size_t ys = (size_t)W * H, cs = ys / 4;
    HL_HIP_CHECK(hipMemcpyAsync(pic[0], d, ys, hipMemcpyDeviceToDevice, e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(pic[1], d + ys, cs, hipMemcpyDeviceToDevice, e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(pic[2], d + ys + cs, cs, hipMemcpyDeviceToDevice, e->stream));
    HL_HIP_CHECK(hipMemcpyAsync(st, d + ys + 2 * cs, sizeof(MbState) * n, hipMemcpyDeviceToDevice, e->stream));
    s->au_intra = s->gop_left <= 0;
    if (s->au_intra) s->gop_left = e->p.gop_size;
    s->ms_el = 0.f;
    return HL_AMD_SUCCESS;
}

extern "C" float hl_amd_svc_layer_ms(hl_amd_encoder_t* e) { return e && e->svc ? e->svc->ms_el : -1.f; }

// The fields of a macroblock object the inter-layer derivations read
// (hl_svc.h svc_derive), from the macroblock's record
static void state_from_record(const MbRecord& r, MbState& m)
{
    memset(&m, 0, sizeof(m));
    m.e_type = r.e_type;
    m.flags = r.flags;
    m.pm0 = r.pm0;
    m.cbp_l = r.cbp_l;
    m.cbp_c = r.cbp_c;
    m.cbp_l4x4 = r.cbp_l4x4;
    m.num_part = r.num_part;
    const bool p16x8 = r.e_type == ET_P16x8, p8x16 = r.e_type == ET_P8x16, p8x8 = r.e_type == ET_P8x8 || r.e_type == ET_P8x8REF0;
    m.part_w = (p8x16 || p8x8) ? 8 : 16;
    m.part_h = (p16x8 || p8x8) ? 8 : 16;
    for (int i = 0; i < 4; ++i) {
        const int st = p8x8 ? r.sub_mb_type[i] : 0;
        m.sub_w[i] = (st == 2 || st == 3) ? 4 : 8;
        m.sub_h[i] = (st == 1 || st == 3) ? 4 : 8;
        for (int j = 0; j < 4; ++j) {
            m.mv[i][j][0] = r.mv[i][j][0];
            m.mv[i][j][1] = r.mv[i][j][1];
        }
    }
}

// n access units of every layer, planes resident in HBM:
// planes[(l * n + i) * 3 + c] is plane c of layer l's frame of access unit
// i.  The base pictures are coded frame-pipelined (hl_amd_encode_batch, one
// run on part of the device); a host thread codes access unit i's
// enhancement layers on their own stream as soon as the run has published
// base picture i (its records in host memory, its picture in the run's
// buffers), while the run goes on.  If the run is re-encoded picture by
// picture (encode_run), the enhancement layers are rolled back and coded
// again from the final base pictures.  results[i] = access unit i as the
// calls of hl_amd_encode_layer would give it: HDR with every header set
// those calls signal, in order, and DATA.  No reference interface (a
// throughput entry point, like hl_amd_encode_batch).
extern "C" int32_t hl_amd_encode_layers_batch(hl_amd_encoder_t* e, int32_t n, int32_t layers, const uint8_t* const* planes,
                                              hl_amd_result_t* results)
{
    if (!e || n <= 0 || !planes || !results) return HL_AMD_ERROR_INVALID_PARAMETER;
    SvcState* s = e->svc;
    if (!s || (int)s->w.size() != layers || layers < 2) return HL_AMD_ERROR_INVALID_STATE;
    for (int i = 0; i < 3 * n * layers; ++i)
        if (!planes[i]) return HL_AMD_ERROR_INVALID_PARAMETER;
    int32_t rc = svc_start(e);
    if (rc != HL_AMD_SUCCESS) return rc;
    if (s->first != 0 || s->last != layers - 1 || s->next != 0) return HL_AMD_ERROR_INVALID_STATE;
    // under rate control every base picture takes the per-picture path and no
    // run keeps the pictures' records: code such streams with hl_amd_encode_layer
    if (e->rc) return HL_AMD_ERROR_NOT_IMPLEMENTED;
    const size_t nmb0 = e->nmb, ys = (size_t)e->W * e->H, cs = ys / 4, pic = ys + 2 * cs;
    const int chunk = std::min(n, kMaxRun);
    if (s->bst_cap < (size_t)chunk) {
        (void)hipFree(s->d_bst);
        (void)hipHostFree(s->h_bst);
        s->d_bst = s->h_bst = nullptr;
        s->bst_cap = 0;
        if (hipMalloc(&s->d_bst, sizeof(MbState) * nmb0 * chunk) != hipSuccess ||
            hipHostMalloc(&s->h_bst, sizeof(MbState) * nmb0 * chunk, hipHostMallocDefault) != hipSuccess)
            return HL_AMD_ERROR_OUTOFMEMMORY;
        s->bst_cap = chunk;
    }
    s->bau.assign(n, {});
    s->bhdr.assign(n, {});
    s->elau.assign(n, {});
    s->elhdr.assign(n, {});
    // picture types of the batch, as the base encoder will choose them
    std::vector<uint8_t> intra(n);
    for (int i = 0, gl = e->gop_left; i < n; ++i) {
        intra[i] = gl <= 0;
        if (intra[i]) gl = e->p.gop_size;
        --gl;
    }
    if (e->broken) return HL_AMD_ERROR_INVALID_STATE;
    // what the caller queued on the encoder's stream before comes first
    HL_HIP_CHECK(hipEventRecord(s->ev_fork, e->stream));
    HL_HIP_CHECK(hipStreamWaitEvent(s->est, s->ev_fork, 0));
    s->linked = false;
    // Every way out (error returns included) restores the encoder's
    // single-call state: the run geometry, the stream linking, the reference
    // layer pointers into this batch, and the order of the two streams.  A
    // batch that fails part-way has advanced the enhancement layers for
    // access units whose base picture did not finish: only then is the
    // encoder marked unusable (INVALID_STATE from then on); an error before
    // any enhancement layer of an unfinished chunk was coded leaves it usable.
    std::atomic<bool> el_ahead{false};  // enhancement layers coded for a chunk that has not completed
    struct Restore {
        hl_amd_encoder_t* e;
        SvcState* s;
        int saved_wg;
        std::atomic<bool>& el_ahead;
        bool ok = false;
        ~Restore()
        {
            e->pipe_wg = saved_wg;
            s->linked = true;
            s->ref0_st = nullptr;
            for (int c = 0; c < 3; ++c) s->ref0_pic[c] = nullptr;
            // what is queued on the encoder's stream next sees the enhancement layers
            bool joined = hipEventRecord(s->ev_join, s->est) == hipSuccess && hipStreamWaitEvent(e->stream, s->ev_join, 0) == hipSuccess;
            if (!joined || (!ok && el_ahead.load())) e->broken = true;
        }
    } restore{e, s, e->pipe_wg, el_ahead};
    std::atomic<bool> base_done{false};
    constexpr int32_t kAborted = -1;  // the run fell back while the thread coded from it
    // the enhancement layers of access units [i0, i0 + m) (base pictures
    // k = i - i0 of the current chunk): from the running run while it is
    // live, else from the chunk's final results
    auto el_chunk = [&](int i0, int m, bool wait_run) -> int32_t {
        int32_t r = HL_AMD_SUCCESS;
        for (int k = 0; k < m && r == HL_AMD_SUCCESS; ++k) {
            const int i = i0 + k;
            const MbRecord* recs;
            const uint8_t* bp;
            for (;;) {
                if (wait_run && e->run_aborted.load(std::memory_order_acquire)) return kAborted;
                if (base_done.load(std::memory_order_acquire)) {
                    recs = e->last_recs[k];
                    bp = e->last_pic[k];
                    break;
                }
                if (wait_run && e->run_live.load(std::memory_order_acquire) && __atomic_load_n(e->h_progress, __ATOMIC_ACQUIRE) > k) {
                    recs = e->h_brec + nmb0 * k;
                    bp = e->d_bpic + pic * k;
                    break;
                }
                std::this_thread::sleep_for(std::chrono::microseconds(20));
            }
            // a run that falls back takes this lock before it rewrites the
            // pictures this one reads (encode_run)
            std::unique_lock<std::mutex> lk(e->el_mu, std::defer_lock);
            if (wait_run) {
                lk.lock();
                if (e->run_aborted.load(std::memory_order_acquire)) return kAborted;
            }
            if (!recs) return HL_AMD_ERROR_INVALID_STATE;
            MbState* hs = s->h_bst + nmb0 * k;
            for (size_t a = 0; a < nmb0; ++a) state_from_record(recs[a], hs[a]);
            HL_HIP_CHECK(hipMemcpyAsync(s->d_bst + nmb0 * k, hs, sizeof(MbState) * nmb0, hipMemcpyHostToDevice, s->est));
            if (bp) {
                s->ref0_pic[0] = const_cast<uint8_t*>(bp);
                s->ref0_pic[1] = const_cast<uint8_t*>(bp) + ys;
                s->ref0_pic[2] = const_cast<uint8_t*>(bp) + ys + cs;
            }
            else
                for (int c = 0; c < 3; ++c) s->ref0_pic[c] = e->d_pic[e->cur ^ 1][c];  // a lone picture: the base encoder's current reference
            s->ref0_st = s->d_bst + nmb0 * k;
            s->au_intra = intra[i] != 0;
            s->au.clear();
            s->ms_el = 0.f;
            std::vector<uint8_t>& hdr = s->elhdr[i];
            hdr.clear();
            el_ahead.store(true);
            for (int l = 1; l < layers && r == HL_AMD_SUCCESS; ++l) {
                const uint8_t* const* p = planes + ((size_t)l * n + i) * 3;
                r = svc_encode_el(e, l, p[0], p[1], p[2]);
                if (r == HL_AMD_SUCCESS && l >= s->hdr_layers) {  // hl_codec_264.c:577-687: a new (subset) SPS and PPS
                    std::vector<uint8_t> h(1024);
                    const StreamParams bp0{s->w[0], s->h[0], e->p.qp, e->p.deblock, e->max_ref_frame};
                    h.resize(write_svc_headers(bp0, s->w.data(), s->h.data(), l + 1, h.data(), h.size()));
                    hdr.insert(hdr.end(), h.begin(), h.end());
                    s->hdr_layers = l + 1;
                }
            }
            if (r == HL_AMD_SUCCESS) r = svc_join(e, layers - 1);
            s->elau[i].swap(s->au);
        }
        return r;
    };
    const char* wenv = getenv("HL_AMD_PIPE_WG");
    if (e->pipe_wg == 0 && !(wenv && atoi(wenv) > 0)) e->pipe_wg = s->pipe_wg;
    std::vector<const uint8_t*> Y(chunk), U(chunk), V(chunk);
    std::vector<hl_amd_result_t> br(chunk);
    static const uint8_t scp[3] = {0, 0, 1};
    for (int i0 = 0; i0 < n && rc == HL_AMD_SUCCESS; i0 += chunk) {
        const int m = std::min(chunk, n - i0);
        for (int k = 0; k < m; ++k) {
            Y[k] = planes[(i0 + k) * 3 + 0];
            U[k] = planes[(i0 + k) * 3 + 1];
            V[k] = planes[(i0 + k) * 3 + 2];
        }
        // the enhancement layers' cross-access-unit state, for a redo
        struct Snap {
            int cur, pict_count;
        };
        std::vector<Snap> snap(layers - 1);
        const int hdr_layers0 = s->hdr_layers;
        for (int l = 1; l < layers && rc == HL_AMD_SUCCESS; ++l) {
            SvcLayerDev& L = s->el[l - 1];
            snap[l - 1] = {L.cur, L.pict_count};
            const size_t ly = (size_t)L.W * L.H, lc = ly / 4;
            uint8_t** ref = L.d_pic[L.cur ^ 1];
            if (hipMemcpyAsync(L.d_snap, ref[0], ly, hipMemcpyDeviceToDevice, s->est) != hipSuccess ||
                hipMemcpyAsync(L.d_snap + ly, ref[1], lc, hipMemcpyDeviceToDevice, s->est) != hipSuccess ||
                hipMemcpyAsync(L.d_snap + ly + lc, ref[2], lc, hipMemcpyDeviceToDevice, s->est) != hipSuccess)
                rc = HL_AMD_ERROR_SYSTEM;
        }
        if (rc != HL_AMD_SUCCESS) break;
        base_done.store(false, std::memory_order_release);
        // a flag left set by an earlier run that fell back must not stop this
        // chunk's thread before this chunk's run starts (encode_run clears it
        // again, and sets it only when this run falls back)
        e->run_aborted.store(false, std::memory_order_release);
        std::future<int32_t> el = std::async(std::launch::async, el_chunk, i0, m, true);
        rc = hl_amd_encode_batch(e, m, Y.data(), U.data(), V.data(), br.data());
        base_done.store(true, std::memory_order_release);
        int32_t rel = el.get();
        if (rc != HL_AMD_SUCCESS) break;
        if ((rel == HL_AMD_SUCCESS || rel == kAborted) && e->calls_fallbacks) {
            // the run was re-encoded picture by picture: roll the enhancement
            // layers back and code them again from the final base pictures
            if (hipStreamSynchronize(s->est) != hipSuccess) {
                rc = HL_AMD_ERROR_SYSTEM;
                break;
            }
            for (int l = 1; l < layers; ++l) {  // the slice writers of the discarded pictures
                SvcLayerDev& L = s->el[l - 1];
                if (L.writing.valid()) L.writing.wait();
            }
            for (int l = 1; l < layers; ++l) {
                SvcLayerDev& L = s->el[l - 1];
                L.cur = snap[l - 1].cur;
                L.pict_count = snap[l - 1].pict_count;
                const size_t ly = (size_t)L.W * L.H, lc = ly / 4;
                uint8_t** ref = L.d_pic[L.cur ^ 1];
                HL_HIP_CHECK(hipMemcpyAsync(ref[0], L.d_snap, ly, hipMemcpyDeviceToDevice, s->est));
                HL_HIP_CHECK(hipMemcpyAsync(ref[1], L.d_snap + ly, lc, hipMemcpyDeviceToDevice, s->est));
                HL_HIP_CHECK(hipMemcpyAsync(ref[2], L.d_snap + ly + lc, lc, hipMemcpyDeviceToDevice, s->est));
            }
            s->hdr_layers = hdr_layers0;
            HL_HIP_CHECK(hipEventRecord(s->ev_base, e->stream));
            HL_HIP_CHECK(hipStreamWaitEvent(s->est, s->ev_base, 0));
            rel = el_chunk(i0, m, false);
        }
        rc = rel == kAborted ? HL_AMD_ERROR_SYSTEM : rel;
        // access unit = prefix NAL unit, base slice, enhancement-layer slices
        for (int k = 0; k < m && rc == HL_AMD_SUCCESS; ++k) {
            const int i = i0 + k;
            const hl_amd_result_t& b = br[k];
            uint8_t pre[5];
            write_prefix_nal(intra[i] != 0, pre);
            std::vector<uint8_t>& au = s->bau[i];
            au.assign(pre, pre + 5);
            au.insert(au.end(), scp, scp + 3);
            au.insert(au.end(), b.data, b.data + b.data_size);
            au.insert(au.end(), scp, scp + 3);
            au.insert(au.end(), s->elau[i].begin(), s->elau[i].end());
            std::vector<uint8_t>& hdr = s->bhdr[i];
            if (b.type & HL_AMD_RESULT_TYPE_HDR) hdr.assign(b.hdr, b.hdr + b.hdr_size);
            hdr.insert(hdr.end(), s->elhdr[i].begin(), s->elhdr[i].end());
            results[i].type = HL_AMD_RESULT_TYPE_DATA | (hdr.empty() ? 0 : HL_AMD_RESULT_TYPE_HDR);
            results[i].hdr = hdr.empty() ? nullptr : hdr.data();
            results[i].hdr_size = hdr.size();
            results[i].data = au.data();
            results[i].data_size = au.size();
        }
        if (rc == HL_AMD_SUCCESS) el_ahead.store(false);  // this chunk's base and enhancement layers are consistent
    }
    restore.ok = rc == HL_AMD_SUCCESS;
    return rc;
}
#endif  // !HL_KERNELS_ONLY
