// hl_mbcore.h -- one macroblock of the reference's RDO encode loop, written
// for one gfx950 workgroup per macroblock.
//
// Scope (reference paths relative to source/h264/):
//   P-MB decision      hl_codec_264_rdo.c:678-1271   guess_inter()
//   diamond search     hl_codec_264_me_ds.c:104-477  search_partition()
//   candidate cost     hl_codec_264_me_ds.c:527-688  eval_candidates()
//   intra decision     hl_codec_264_rdo.c:99-299, 1526-2136 guess_intra()
//   reconstruction     hl_codec_264_rdo.c:2140-2782
//   MV prediction      hl_codec_264_utils.c:709-963, hl_codec_264_mb.c:426-541
//
// Execution model.  Control flow is uniform: every lane runs the same loop
// nest (partitions, diamond steps, intra modes) and computes the same scalar
// decisions from LDS, so they live in SGPRs.  Data-parallel phases are
// strided loops over (candidate x 4x4 block), (mode x block) or pixels,
// separated by HL_SYNC().  Built for the host with nthr = 1 the same code
// runs serially; that build is only used by tests/ to diff the kernel logic
// against the oracle without a GPU.
//
// Order-dependent reference state is reproduced exactly:
//  * TotalCoeffsLuma of the live MB is rewritten by every trial CAVLC call
//    (residual.c:796-806); the nC a candidate sees depends on all candidates
//    evaluated before it.  eval_candidates() resolves this with a
//    last-writer lookup over the candidates of the step.
//  * CodedBlockPatternLuma of the live MB is stale (previous frame) during
//    the search (utils.h:9-20).
//  * pc_esd->rdo.Single_ctr is one encoder-global counter read stale by the
//    I16x16 RDO; it is carried in Ctx::chain and recorded in MbChain so the
//    host can validate row-start speculation.
#pragma once
#include <stddef.h>
#include <string.h>

#include "hl_coop.h"
#include "hl_prims.h"
#include "hl_quad.h"
#include "hl_types.h"

namespace hl {

constexpr int kBarSites = 2560;  // HL_BAR_PROF=2: barrier sites (source line / 2)
#if defined(__HIP_DEVICE_COMPILE__) && defined(HL_PROFILE) && defined(HL_BAR_PROF)
// profiling build: every wave's cycles inside the macroblock's barriers
// (lane 0 of each wave adds to its own word; encode_mb reports them)
__shared__ unsigned long long g_bar_acc[8][2];
#if HL_BAR_PROF >= 2
// HL_BAR_PROF=2: per barrier site (source line / 2): wait cycles summed over
// the waves, and wave 0's count; added to FrameArgs::prof after the timeline
__shared__ unsigned long long g_bar_site[kBarSites];
__shared__ unsigned g_bar_cnt[kBarSites];
#endif
__device__ __forceinline__ void hl_sync_prof(int line)
{
    const unsigned long long t0 = __builtin_readcyclecounter();
    __syncthreads();
    const unsigned long long dt = __builtin_readcyclecounter() - t0;
    if ((threadIdx.x & 63) == 0) {
        g_bar_acc[threadIdx.x >> 6][0] += dt;
        g_bar_acc[threadIdx.x >> 6][1] += 1;
#if HL_BAR_PROF >= 2
        const int k = min(line >> 1, kBarSites - 1);
        atomicAdd(&g_bar_site[k], dt);
        if (threadIdx.x == 0) g_bar_cnt[k] += 1;
#endif
    }
}
#define HL_SYNC() hl_sync_prof(__LINE__)
#elif defined(__HIP_DEVICE_COMPILE__)
#define HL_SYNC() __syncthreads()
#else
#define HL_SYNC() ((void)0)
#endif

// Optional phase timing (profiling build only, -DHL_PROFILE): every wave
// accumulates shader-clock cycles per phase in registers (Ctx::pacc); lane 0
// adds them to FrameArgs::prof once per macroblock.
#if defined(HL_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
#define HL_PROF_T(v) const unsigned long long v = __builtin_readcyclecounter()
#define HL_PROF_ADD(c, slot, t0)                                 \
    do {                                                         \
        (c).pacc[slot] += __builtin_readcyclecounter() - (t0);   \
        (c).pcnt[slot] += 1;                                     \
    } while (0)
#if !defined(HL_STEP_PROF) && !defined(HL_I4_PROF) && !defined(HL_NBLK_PROF) && !defined(HL_BAR_PROF)
#define HL_PROF_MISC 1  // slots 14, 15, 18: chroma reconstruction, the intra decision's tail, inter prediction
#endif
constexpr int kProfSlots = 20;  // prof[2 * slot], prof[2 * slot + 1] (< 40: the pipelined kernel uses 40-44)
#else
#define HL_PROF_T(v) const unsigned long long v = 0
#define HL_PROF_ADD(c, slot, t0) ((void)(t0))
#endif

constexpr int kPad = 40;  // padding of the luma reference planes (origin clip is +-17, block 16, tap 3)
constexpr int kMaxWaves = 8;   // waves of the macroblock workgroup
// lanes of the macroblock workgroup.  512 (one workgroup per CU) is the
// product.  The 256-lane build (two workgroups per CU) is bit-exact too
// (every parity case, round 4), but gains only 4 % where the device is full
// and loses 35 % of macroblock latency, which the ramp, the tail and lone
// pictures pay (profiles/r04_ab_256_lanes_two_wg_per_cu.log).
#ifndef HL_MB_THREADS
#define HL_MB_THREADS 512
#endif
constexpr int kMbThreads = HL_MB_THREADS;
constexpr int kMbRows = kMbThreads / 16;           // 16-lane rows
// Candidates of one evaluation pass: a chain of up to four search steps
// (MVP/(0,0), then the first integer, half and quarter steps), the later ones
// speculative (see search_partition); at most kMaxPass rows per lane.
constexpr int kMaxCand = 32;
constexpr int kMaxSeg = 4;
// partitions whose passes chain speculative steps: with the quad pipeline a
// pass holds 256 blocks, so even a 16x16 chain (MVP/(0,0) + integer + half
// step, 16 candidates) fits one pass
#ifndef HL_SPEC_MAX_BLOCKS
#define HL_SPEC_MAX_BLOCKS 16
#endif
constexpr int kMaxPass = (9 * 16 + kMbRows - 1) / kMbRows;  // rows per lane for the largest step
// Candidate evaluation with one 4-lane quad per 4x4 block (hl_quad.h, the
// default) or one 16-lane row per block (hl_coop.h): blocks a pass can hold.
// quad rounds per pass: 2 x 128 blocks at 512 lanes; smaller workgroups take
// enough rounds for the largest non-speculative step (9 16x16 candidates)
#ifndef HL_QPASS
#define HL_QPASS 2  // quad rounds a 512-lane pass holds (3: a 16x16 pass holds two steps)
#endif
constexpr int kQPass = kMbThreads >= 512 ? HL_QPASS : (9 * 16 + (kMbThreads >> 2) - 1) / (kMbThreads >> 2);
constexpr int kPassItems = kQPass * (kMbThreads >> 2);
constexpr int kSpecMaxBlocks = HL_SPEC_MAX_BLOCKS;

// One candidate of a step: plane offsets of its quarter-pel prediction
// (second plane = first when the phase needs no average) and its MV.
struct alignas(16) CandSlot {
    int32_t off1, off2;
    int16_t mvx, mvy;
    int32_t pad;
};
constexpr int kNA = -1;   // not-available sample marker

// The intra fallback of a P macroblock (rdo.c:1161-1167 -> rdo.c:99-299)
// split into what only depends on the MB's source and its final neighbours
// and what depends on the live state its inter search leaves behind (the
// TotalCoeffs of quirk 1 and rdo.Single_ctr).  The first part -- prediction,
// transform, quantisation, CAVLC statistics and reconstruction of every
// Intra16x16 mode, and the whole Intra4x4 decision under a guess of the live
// TotalCoeffs -- runs in a helper task beside the MB's inter search
// (intra_helper; pipelined runs, hl_encoder.hip); the MB then resolves the
// Intra16x16 modes against its live state (i16_light) and keeps the helper's
// Intra4x4 decision if every nC class it used is the one the live state gives
// (i4_verify), else decides Intra4x4 itself.  IntraHead is the small part the
// MB reads first (whole 16-byte words; also the LDS image, Shared::ih).
struct alignas(16) IntraHead {
    int32_t blk[4][16];  // I16 mode m, block t: coded | TotalCoeff << 1 | TrailingOnes << 6 | (single + 1) << 8 | rest bits << 16
    int32_t dcs[4][4];   // I16 mode m, DC block: bits (coeff_token included), TotalCoeff, single counter, -
    int32_t dist[4][2];  // I16 mode m: distortion with the residual / of the prediction alone
    int8_t i4_ncls[16];  // I4 block: nC class its mode costs used (-1: no cost used an nC)
    int8_t i4_lwtc[16];  // I4 block: TotalCoeff its resolution wrote to the live state (-1: none)
    int8_t i4_mode[16];  // I4 block: chosen mode
    int32_t i4_cbp, i4_dist, i4_sct, i4_valid;  // coded blocks, distortion, last counter write (-1: none), 1 = present
    double i4_cost;      // the Intra4x4 cost (z-order sum)
    int32_t pad[2];
};
static_assert(sizeof(IntraHead) % 16 == 0, "IntraHead in whole 16-byte words");
struct alignas(16) IntraSpec {
    IntraHead h;
    uint8_t rec[4][256];   // I16 mode m: reconstruction with the residual
    uint8_t pred[4][256];  // I16 mode m: prediction
    int16_t ac[4][16][16]; // I16 mode m: Intra16x16ACLevel per block (15 used)
    int16_t dcl[4][16];    // I16 mode m: DC levels (scan order)
    uint8_t i4_rec[256];   // I4: reconstruction of the chosen modes
    int16_t i4_lv[16][16]; // I4: LumaLevel of the chosen modes
};
static_assert(sizeof(IntraSpec) % 16 == 0, "IntraSpec in whole 16-byte words");
// helper task state (FrameArgs::hstate[addr])
enum : int32_t { HS_FREE = 0, HS_CLAIMED = 1, HS_MAIN = 2, HS_DONE = 3 };

// A partitioning helper task's results (FrameArgs::f3[addr * 4 + j - 3]): P8x8
// partitioning j (kParts[3..6], rdo.c:745-760) searched from the MB-start live
// TotalCoeffs while the macroblock searches 16x16 / 16x8 / 8x16, with the
// intervals of the entry values under which every nC class it used holds
// (f3_verify), and the state the partitioning leaves behind (the per-
// partitioning arrays hold j's entry only).
struct Fam3Out {
    double cost[4];               // partitioning j = 3..6: sum of the partitions' best costs (header bits not added)
    int32_t single[4], dist[4];
    int32_t done_mask;            // bit j - 3: partitioning j searched (mode_flags)
    int32_t wmask;                // blocks whose live TotalCoeff the family wrote
    int32_t chain, fresh;         // rdo.Single_ctr after the family; fresh = the family wrote it
    int32_t e_last;               // the last partitioning searched
    int32_t pad0[3];
    int8_t tc[16];                // live TotalCoeffs after the family (blocks in wmask)
    int8_t lo[32], hi[32];        // [b]: entry value of block b; [16 + b]: sum of block b's inside neighbours' entry values
    int16_t bmv[4][4][4][2], bmvp[4][4][4][2];  // per partitioning: best MVs and MVPs
    int16_t nbmv[4][4][2];        // MvL0 of the partitions (Shared::nb[0].mv) after the family
    int32_t mvg[6][6];            // motion grid after the family
    int8_t mvs[6][6];
    int8_t pad1[12];
};
static_assert(sizeof(Fam3Out) % 16 == 0, "Fam3Out in whole 16-byte words");

struct FrameArgs {
    int32_t W, H, Wc, Hc, mbw, mbh;
    int32_t qp, qpc, is_intra, me_range;
    int32_t early_term;     // hl_codec_t.me_early_term_flag (rdo.c:888-931)
    double lambda;
    const uint8_t* src[3];
    uint8_t* cur[3];
    const uint8_t* ref[3];  // ref[0] unused (luma goes through pl[])
    const uint8_t* pl[4];   // padded luma reference: full, half-h (b), half-v (h), centre (j)
    int32_t pstride;
    int32_t plsz;           // pl[i] = pl[0] + i * plsz (device buffers)
    MbState* st;
    MbRecord* rec;
    MbRecord* hrec;         // host-mapped copy of the records (pipelined runs: the slice writers read it), or null
    int32_t rec_dev;        // 1 = write the records to rec (device memory) too
    MbChain* chain;
    const int32_t* spec;  // speculated Single_ctr at each row start
    unsigned long long* prof;  // phase cycle counters (profiling build), may be null
    // pipelined runs (hl_pipeline.h); ref_done is null in the per-picture path
    const int32_t* ref_done;  // task flags of the reference picture's slot
    int32_t ref_epoch;        // flag value once a task of the reference picture finished
    int32_t* perr;            // [0] bounded-spin failures, [1] resolve_chain walks
    // exact rdo.Single_ctr for stale reads of a speculated value (resolve_chain);
    // run_done is null in the per-picture path (the host re-runs rows instead)
    const int32_t* run_done;  // task flags of picture 0 of the run ([pos * mbw * mbh + addr])
    const MbChain* run_chain; // chain records of picture 0 of the run (same layout)
    int32_t run_pos;          // this picture's position in the run
    int32_t carry_in;         // exact counter value entering picture 0 of the run
    // intra helper tasks (P pictures of pipelined runs; null otherwise): the
    // per-address results and this picture's task states (HS_*)
    IntraSpec* ispec;
    int32_t* hstate;
    // 8x8-family helper tasks (the same pictures): this picture's results and states
    Fam3Out* f3;       // [addr * 4 + j - 3]
    int32_t* hstate3;  // [addr * 4 + j - 3]
};

struct NbInfo {
    int32_t avail, intra, e_type, part_w, part_h;
    int32_t sub_w[4], sub_h[4];
    int16_t mv[4][4][2];
};

struct PartDef {
    int8_t num_part, num_sub, sub_w, sub_h, part_w, part_h, hdr_bits, sub_type;
};
// Partition families searched by guess_inter (rdo.c:731-760), in order.
static constexpr PartDef kParts[7] = {
    {1, 1, 16, 16, 16, 16, 3, -1}, {2, 1, 16, 8, 16, 8, 5, -1}, {2, 1, 8, 16, 8, 16, 5, -1},
    {4, 1, 8, 8, 8, 8, 11, 0},     {4, 2, 8, 4, 8, 8, 19, 1},   {4, 2, 4, 8, 8, 8, 19, 2},
    {4, 4, 4, 4, 8, 8, 27, 3}};

struct Shared {
    MbState nbst[5];  // MB start (device): the MB objects of the current address, A, B, C, D as loaded;
                      // nbst[0] becomes the MB's new object at the MB end
    MbRecord recb;    // MB end (device): the record, assembled before its 16-byte stores
    int8_t tcn[16], tccn[2][4];  // MB end (device): TotalCoeffs after the final CAVLC write
    NbInfo nb[5];  // 0 = current MB (live search state), 1 = A, 2 = B, 3 = C, 4 = D
    int32_t mvg[5][6];  // motion grid, see MvN
    int8_t mvs[5][6];
    int32_t nb_pm0[3];
    int8_t nb_i4[3][16];
    int8_t extA[16], extB[16];  // luma nC from the neighbouring MB (-1 = not available, -2 = inside MB)
    int8_t extCA[4], extCB[4];  // chroma AC nC from neighbouring MBs
    uint8_t src[256];
    uint8_t srcc[2][64];
    alignas(16) uint8_t rec[256];// current MB luma recon (intra neighbours read it)
    int16_t top[25];      // luma row y=-1, x=-1..23 (kNA when not available)
    int16_t left[16];     // luma column x=-1
    int16_t ctop[2][9];   // chroma row y=-1, x=-1..7
    int16_t cleft[2][8];
    int8_t tc[16];        // live TotalCoeffsLuma
    int8_t tcc[2][4];     // live TotalCoeffsChromaACCbCr
    int16_t cac[2][4][16];// live ChromaACLevel
    int32_t cbp_l, cbp_c; // live CodedBlockPattern{Luma,Chroma}
    // --- candidate step scratch
    CandSlot wc[kMaxWaves][kMaxCand];  // candidates of the step, one copy per wave (each wave writes its own)
    int32_t be_nz[kMaxCand][16], be_tc[kMaxCand][16], be_t1[kMaxCand][16], be_sctr[kMaxCand][16], be_bits[kMaxCand][16],
        be_dist[kMaxCand][16];
    alignas(16) int4 be_w[kMaxCand][16];  // packed block statistics (device path): w0, w1, w2 of eval_candidates, -
    // Per-step results are double-buffered by step parity (Ctx::par): after a
    // step's last barrier, waves still read its results (the candidate scan,
    // the live TotalCoeffs update, the Single_ctr chain) while faster waves
    // already write the next step's -- a step only reuses the buffer of the
    // step before the previous one, whose readers all passed a barrier since.
    alignas(16) uint8_t be_tcb[2][16][kMaxCand];         // TotalCoeff [parity][block][candidate]
    uint32_t be_tcm[3][16];  // candidates with a nonzero TotalCoeff [pass mod 3][block]
    alignas(16) int32_t lvs[kMaxWaves * 4][16];          // per-row level scratch of coop_cavlc
    alignas(16) int32_t lvq[kMaxWaves * 16][16];         // per-quad level scratch of quad_cavlc
    CoopTables ct;
    uint32_t qtab[16];                                   // packed quarter-pel phase table
    alignas(8) int2 qoff[16];  // per phase: plane offsets of the two prediction samples relative to (X, Y) (put_cand)
    struct CandRes {
        double cost[kMaxCand];
        int32_t bits[kMaxCand], dist[kMaxCand], single[kMaxCand], cbp[kMaxCand], last[kMaxCand];
    } cd[2];  // per candidate of a step [parity]
    // --- per (sub)partition search results
    double bcost[4][4];
    int32_t bdist[4][4], bsingle[4][4], bcbp[4][4];
    int16_t bmv[4][4][2], bmvp[4][4][2];
    // --- best inter decision
    int16_t best_mv[4][4][2], best_mvp[4][4][2];
    // --- intra scratch
    alignas(16) int32_t pred[256];
    int32_t i16_ac[16][16], i16_dcc[64];  // (i16_ac: scratch of the pipelined task's plane blocks)
    int32_t i16_called[16], i16_bits[16], i16_dist[32], i16_distz[32];  // (i16_dcc / _dist / _distz: two modes' rows)
    alignas(16) int16_t i16_best_ac[16][16];
    alignas(16) int16_t i16_best_dc[16];
    alignas(16) uint8_t i16_best_rec[256];
    // Intra16x16 statistics of every mode and the Intra4x4 verification record
    // (IntraHead: computed here by i16_heavy / guess_i4, or imported from the
    // MB's intra helper task), and the modes' bulk results (i16_heavy)
    IntraHead ih;
    alignas(16) uint8_t ih_rec[4][256];
    alignas(16) uint8_t ih_pred[4][256];
    alignas(16) int16_t ih_ac[4][16][16];
    alignas(16) int16_t ih_dcl[4][16];
    // I4x4 trials of up to two blocks at once [wavefront slot][mode] (device) / [0][mode] (host)
    int32_t i4_cost_ok[2][9], i4_exact[2][9], i4_nz[2][9], i4_tc[2][9], i4_sctr[2][9], i4_dist[2][9];
    double i4_cost[2][9];
    int16_t i4_lv[2][9][16];
    uint8_t i4_rec[2][9][16];
    double i4r_dmin[16];       // per block, in z-order accumulation after the wavefront
    int32_t i4r_dist[16], i4r_sct[16], i4r_zero[16];
    int32_t luma_level[16][16];
    int32_t dcY[64];             // I16x16: scaled DC per DC-matrix position (per mode)
    int32_t chain_x;             // resolve_chain result
    int32_t hs_x;                // intra helper state seen by the MB (HS_*)
    int32_t hs3_x;               // 8x8-family helper state seen by the MB
    int32_t f3lo[32], f3hi[32];  // fam3_helper: entry-value intervals being recorded (see Fam3Out)
    int32_t f3w;                 // fam3_helper: blocks whose live TotalCoeff the family wrote so far
    int8_t f3pad0[16];
    int16_t f3pad1[64];          // (unused: they keep the later fields' LDS offsets, which the register allocation follows)
    double f3pad2;
    int32_t f3b[8];              // the partitioning helper: [0] partitionings searched (mode_flags)
    int32_t homo[4];             // early termination: homogeneity of the four 8x8 source quadrants
    int32_t predc[2][64];
    int32_t cres_dc[2][4], cres_cac[2][4], cres_cdc[2][4], cres_tc[2][4], cres_sctr[2][4];
    int32_t cdc_level[2][4];
    // --- live MB decision fields
    int32_t flags, pm0, e_type, mb_type, i16mode, chroma_mode, cbp, cbp_l4x4, cbp_cac[2], cbp_cdc[2];
    int32_t num_part, num_sub[4], sub_type[4];
    int8_t i4mode[16], prev_flag[16], rem_mode[16];
    int16_t mvd[4][4][2];
    int8_t nc_luma[16], nc_cac[2][4], nc_dc;
    int32_t mad;  // distortion of the chosen mode (rate control MAD, rdo.c:211-228, 1266-1268)
    // per-lane constants of the 16-lane block pipeline at this MB's QP, by
    // lane position (tid & 15): read from LDS where used instead of held in 9
    // VGPRs for the whole MB (which the compiler spilled to scratch: those
    // scratch stores were most of k_pipeline's HBM writes)
    LaneK lk[16];
};

// 8x8-family helper tasks (guess_inter): 1 = built in.  Off
// in the product: the recording in the search's hot loop and the import
// path cost the macroblock decision more registers (VGPR spills 19 -> 34)
// than the helpers win in the ramp and tail (profiles/r04_ab_fam3_helpers.log);
// the CPU emulator builds it (tests/emu) and `make variant` can.
#ifndef HL_FAM3
#define HL_FAM3 0
#endif
#ifndef HL_F3REC_ON
#define HL_F3REC_ON 1
#endif
#define HL_F3REC(c) (HL_FAM3 && HL_F3REC_ON && REC && (c).f3rec)  // (REC: the search's template argument)
// A fresh, opaque copy of the lane index at the entry of each phase: the
// compiler cannot compute the phase's lane-dependent addresses earlier and
// hold them (spilled) across the partition searches.
#if defined(__HIP_DEVICE_COMPILE__)
#define HL_FRESH_TID(c) \
    do { \
        int t_ = (c).tid; \
        asm volatile("" : "+v"(t_)); \
        (c).tid = t_; \
    } while (0)
#else
#define HL_FRESH_TID(c) ((void)0)
#endif
#ifndef HL_FRESH_MASK
#define HL_FRESH_MASK 0xFFE
#endif
// the quad pipeline's scan-order word (LaneQ::zz) recomputed at the start
// of the evaluation pass (bit 0) / of the later phases (bit 1) instead of held
// from the MB's start
#ifndef HL_FRESH_ZZ
#define HL_FRESH_ZZ 2
#endif
#define HL_FRESH_TID_K(c, k) \
    do { \
        if ((HL_FRESH_MASK >> (k)) & 1) HL_FRESH_TID(c); \
    } while (0)
struct Ctx {
    const FrameArgs& F;
    Shared& S;
    int tid, nthr;
    int addr, mbx, mby, xL, yL;
    int chain, fresh, dep;  // rdo.Single_ctr emulation (uniform)
    // per-lane constants of the 16-lane block pipeline (Shared::lk), addressed
    // from the phase's lane index at each use (an address held from the MB's
    // start was spilled across the partition searches)
    __host__ __device__ const LaneK& k() const { return S.lk[tid & 15]; }
#if defined(__HIP_DEVICE_COMPILE__)
    LaneQ Q{};              // per-lane constants of the quad block pipeline (registers: the search loop reads them every pass)
#endif
    int gx, gy;             // reference planes known complete for MBs (X <= gx, Y <= gy) (pipelined runs)
    int spec = 0;           // 1 = chain is still a row-start speculation (uniform)
    int par = 0;            // buffer parity of the last candidate step (Shared::cd, be_tcb)
    int p3 = 0;             // the last candidate step's slot of Shared::be_tcm (pass mod 3)
    int f3rec = 0;          // 1 = fam3_helper: record entry-value intervals and written blocks (Shared::f3*)
#if defined(HL_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
    unsigned long long pacc[kProfSlots] = {};
    unsigned pcnt[kProfSlots] = {};
#endif
};

// --------------------------------------------------------------------------
// small helpers
// --------------------------------------------------------------------------
// ue(v) length 2 floor(log2(v + 1)) + 1, closed form (a per-lane loop here
// ran in every lane of the cost phase); v + 1 < 2^31 for every MV difference
HD int ue_len(unsigned v)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return 2 * (31 - __clz((int)(v + 1))) + 1;
#else
    int lz = 0;
    while ((1u << (lz + 1)) <= v + 1) ++lz;
    return 2 * lz + 1;
#endif
}
HD int se_len(int n) { return ue_len(n <= 0 ? (unsigned)(-n) << 1 : ((unsigned)n << 1) - 1); }

HD void chain_write(Ctx& c, int sctr)
{
    c.chain = sctr;
    c.fresh = 1;
    c.spec = 0;
}

// Luma 4x4 prediction from the padded quarter-pel planes for integer origin
// (X, Y) and fraction (xF, yF) -- the 16 cases of 8.4.2.2.1 as computed by
// interpol.h:162-925 (planes: 0 full, 1 b, 2 h, 3 j).
static constexpr int8_t kQpelTab[16][6] = {
    {0, 0, 0, -1, 0, 0}, {0, 0, 0, 1, 0, 0}, {1, 0, 0, -1, 0, 0}, {0, 1, 0, 1, 0, 0},
    {0, 0, 0, 2, 0, 0},  {1, 0, 0, 2, 0, 0}, {1, 0, 0, 3, 0, 0},  {1, 0, 0, 2, 1, 0},
    {2, 0, 0, -1, 0, 0}, {2, 0, 0, 3, 0, 0}, {3, 0, 0, -1, 0, 0}, {3, 0, 0, 2, 1, 0},
    {0, 0, 1, 2, 0, 0},  {2, 0, 0, 1, 0, 1}, {3, 0, 0, 1, 0, 1},  {2, 1, 0, 1, 0, 1}};

HD void pred_luma4x4(const FrameArgs& F, int X, int Y, int xF, int yF, int* p)
{
    const int ph = (yF << 2) | xF;
    const int s = F.pstride;
    const auto p1 = gmem(F.pl[kQpelTab[ph][0]]) + (Y + kPad + kQpelTab[ph][2]) * s + X + kPad + kQpelTab[ph][1];
    if (kQpelTab[ph][3] < 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) p[j * 4 + i] = p1[j * s + i];
    }
    else {
        const auto p2 = gmem(F.pl[kQpelTab[ph][3]]) + (Y + kPad + kQpelTab[ph][5]) * s + X + kPad + kQpelTab[ph][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) p[j * 4 + i] = (p1[j * s + i] + p2[j * s + i] + 1) >> 1;
    }
}

// --------------------------------------------------------------------------
// neighbour derivation (6.4.12, utils.c:61-230)
// --------------------------------------------------------------------------
// Which MB holds luma/chroma location (xN, yN) relative to the current MB:
// 0 current, 1 A, 2 B, 3 C, 4 D, -1 not available.
HD int nb_loc(const Shared& S, int xN, int yN, int maxW, int maxH, int& xW, int& yW)
{
    int w;
    if (xN >= 0 && xN < maxW && yN >= 0 && yN < maxH) w = 0;
    else if (xN >= 0 && xN < maxW && yN < 0) w = 2;
    else if (xN >= maxW && yN < 0) w = 3;
    else if (xN < 0 && yN < 0) w = 4;
    else if (xN < 0 && yN >= 0 && yN < maxH) w = 1;
    else w = -1;
    if (w > 0 && !S.nb[w].avail) w = -1;
    xW = (xN + maxW) % maxW;
    yW = (yN + maxH) % maxH;
    return w;
}

HD bool is8x8(int et) { return et == ET_P8x8 || et == ET_P8x8REF0; }

// log2 of a power of two (partition sizes 4, 8, 16): divisions by a
// runtime partition size compile to long VALU sequences; shifts do not
HD int lg2(int v)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return 31 - __clz(v);
#else
    return 31 - __builtin_clz((unsigned)v);
#endif
}
// origin of partition pi of a 16x16 MB split into pw x ph partitions
HD int part_x(int pi, int pw) { return (pi & ((16 >> lg2(pw)) - 1)) << lg2(pw); }
HD int part_y(int pi, int pw, int ph) { return (pi >> (4 - lg2(pw))) << lg2(ph); }
// origin of sub-partition spi of an 8x8 partition split into sw x sh
HD int sub_x(int spi, int sw) { return (spi & ((8 >> lg2(sw)) - 1)) << lg2(sw); }
HD int sub_y(int spi, int sw, int sh) { return (spi >> (3 - lg2(sw))) << lg2(sh); }

HD void sub_part_idx(const NbInfo& n, int xW, int yW, int& pi, int& spi)  // mb.h:313-339
{
    if (n.intra) pi = 0;
    else pi = ((yW >> lg2(n.part_h)) << (4 - lg2(n.part_w))) + (xW >> lg2(n.part_w));
    if (!is8x8(n.e_type)) spi = 0;
    else spi = (((yW & 7) >> lg2(n.sub_h[pi])) << (3 - lg2(n.sub_w[pi]))) + ((xW & 7) >> lg2(n.sub_w[pi]));
}

// Motion of the 4x4 blocks around and inside the current MB, in LDS:
// S.mvg / S.mvs [by + 1][bx + 1] for block coordinates bx -1..4, by -1..3
// (row -1 = MBs D, B, C; column -1 = MB A; inside = partitions of the
// current partitioning already searched).  State 0 = not available,
// 1 = available intra (refIdx -1), 2 = inter (refIdx 0).  This is the
// neighbour derivation of 8.4.1.3.2 (utils.c:854-963) with the partition
// lookup done once per MB instead of per predictor.
struct MvN {
    int st, mv[2];
};

HD MvN mv_at(const Shared& S, int bx, int by)
{
    MvN n;
    n.st = S.mvs[by + 1][bx + 1];
    const int v = S.mvg[by + 1][bx + 1];
    n.mv[0] = n.st == 2 ? (int)(int16_t)(v & 0xFFFF) : 0;
    n.mv[1] = n.st == 2 ? (v >> 16) : 0;
    return n;
}

// A, B, C (C replaced by D when not available) of the (sub)partition at
// luma (x, y) of width ppw; all four cells are read in one batch
HD void nb_motion(const Shared& S, int x, int y, int ppw, MvN nb[3])
{
    const int bx = x >> 2, by = y >> 2;
    const int cx = (x + ppw) >> 2;
    const bool c_in = cx <= 4 && !(cx == 4 && by > 0);
    const MvN a = mv_at(S, bx - 1, by), b = mv_at(S, bx, by - 1), d = mv_at(S, bx - 1, by - 1);
    const MvN cc = mv_at(S, c_in ? cx : bx - 1, by - 1);
    nb[0] = a;
    nb[1] = b;
    nb[2] = (c_in && cc.st != 0) ? cc : d;
}

HD int median3(int a, int b, int c)
{
    const int mx = a > b ? (a > c ? a : c) : (b > c ? b : c);
    const int mn = a < b ? (a < c ? a : c) : (b < c ? b : c);
    return a + b + c - mx - mn;
}

// shape of the partitioning being searched (registers, not LDS)
struct PartShape {
    int part_w, part_h, sub_w, sub_h, is8;
};

// 8.4.1.3 (utils.c:751-831) for partition (pi, spi) of partitioning ps
HD void mvp(const Shared& S, const PartShape& ps, int pi, int spi, int out[2])
{
    const int x = part_x(pi, ps.part_w);
    const int y = part_y(pi, ps.part_w, ps.part_h);
    int xS = 0, yS = 0, ppw = ps.part_w;
    if (ps.is8) {
        xS = sub_x(spi, ps.sub_w);
        yS = sub_y(spi, ps.sub_w, ps.sub_h);
        ppw = ps.sub_w;
    }
    MvN nb[3];
    nb_motion(S, x + xS, y + yS, ppw, nb);
#if defined(__HIP_DEVICE_COMPILE__)
    {
        // 8.4.1.3 as selects (the values are uniform but live in VGPRs: every
        // branch on them would be an exec-mask branch)
        const MvN A = nb[0], B = nb[1], C = nb[2];
        const bool a2 = A.st == 2, b2 = B.st == 2, c2 = C.st == 2;
        const bool p168 = ps.part_w == 16 && ps.part_h == 8, p816 = ps.part_w == 8 && ps.part_h == 16;
        int sel = (p168 && pi == 0 && b2) ? 1 : ((p168 && pi == 1 && a2) ? 0 : ((p816 && pi == 0 && a2) ? 0 : ((p816 && pi == 1 && c2) ? 2 : -1)));
        const bool rep = B.st == 0 && C.st == 0 && A.st != 0;  // B and C replaced by A
        const bool eb2 = rep ? a2 : b2, ec2 = rep ? a2 : c2;
        const int bx = rep ? A.mv[0] : B.mv[0], by = rep ? A.mv[1] : B.mv[1];
        const int cx = rep ? A.mv[0] : C.mv[0], cy = rep ? A.mv[1] : C.mv[1];
        const int one = (a2 && !eb2 && !ec2) ? 0 : ((eb2 && !ec2 && !a2) ? 1 : ((ec2 && !eb2 && !a2) ? 2 : -1));
        sel = sel >= 0 ? sel : one;
        // (a directional pick of B or C needs it inter-coded, so no
        // replacement happened: bx / cx are B's / C's own motion then)
        out[0] = sel == 0 ? A.mv[0] : (sel == 1 ? bx : (sel == 2 ? cx : median3(A.mv[0], bx, cx)));
        out[1] = sel == 0 ? A.mv[1] : (sel == 1 ? by : (sel == 2 ? cy : median3(A.mv[1], by, cy)));
        return;
    }
#endif
    // named values + selects (no dynamically indexed arrays: they go to scratch)
    MvN A = nb[0], B = nb[1], C = nb[2];
    int rA = A.st == 2 ? 0 : -1, rB = B.st == 2 ? 0 : -1, rC = C.st == 2 ? 0 : -1;
    int sel = -1;
    if (ps.part_w == 16 && ps.part_h == 8 && pi == 0 && rB == 0) sel = 1;
    else if (ps.part_w == 16 && ps.part_h == 8 && pi == 1 && rA == 0) sel = 0;
    else if (ps.part_w == 8 && ps.part_h == 16 && pi == 0 && rA == 0) sel = 0;
    else if (ps.part_w == 8 && ps.part_h == 16 && pi == 1 && rC == 0) sel = 2;
    if (sel < 0) {
        if (B.st == 0 && C.st == 0 && A.st != 0) {
            B = A;
            C = A;
            rB = rC = rA;
        }
        if (rA == 0 && rB != 0 && rC != 0) sel = 0;
        else if (rB == 0 && rC != 0 && rA != 0) sel = 1;
        else if (rC == 0 && rB != 0 && rA != 0) sel = 2;
    }
    if (sel >= 0) {
        out[0] = sel == 0 ? A.mv[0] : (sel == 1 ? B.mv[0] : C.mv[0]);
        out[1] = sel == 0 ? A.mv[1] : (sel == 1 ? B.mv[1] : C.mv[1]);
        return;
    }
    out[0] = median3(A.mv[0], B.mv[0], C.mv[0]);
    out[1] = median3(A.mv[1], B.mv[1], C.mv[1]);
}

// 8.4.1.1 P_Skip motion vector (utils.c:709-748)
HD void skip_mv(const Shared& S, int out[2])
{
    MvN nb[3];
    nb_motion(S, 0, 0, 16, nb);
    if (nb[0].st == 0 || nb[1].st == 0 || (nb[0].st == 2 && !nb[0].mv[0] && !nb[0].mv[1]) ||
        (nb[1].st == 2 && !nb[1].mv[0] && !nb[1].mv[1])) {
        out[0] = out[1] = 0;
        return;
    }
    const PartShape p16{16, 16, 16, 16, 0};
    mvp(S, p16, 0, 0, out);
}

// marks the 4x4 blocks of the luma rectangle as decided with motion mv
// (one lane: spreading these stores over 16 lanes measured slower, the
// extra SALU address arithmetic outweighing the stores)
HD void grid_set(Shared& S, int x, int y, int w, int h, int mvx, int mvy)
{
    for (int by = y >> 2; by < (y + h) >> 2; ++by)
        for (int bx = x >> 2; bx < (x + w) >> 2; ++bx) {
            S.mvs[by + 1][bx + 1] = 2;
            S.mvg[by + 1][bx + 1] = (mvx & 0xFFFF) | (int)((uint32_t)mvy << 16);
        }
}
HD void grid_reset_inside(Shared& S)
{
    for (int by = 0; by < 4; ++by)
        for (int bx = 0; bx < 4; ++bx) S.mvs[by + 1][bx + 1] = 0;
}

// nC of a luma-type block (residual.c:640-755): neighbour values are taken
// from the external MBs (extA/extB) or, inside the MB, through `inside`.
template <typename F>
HD int nc_luma_of(const Shared& S, int bi, F inside)
{
    const int bx = blk_x(bi), by = blk_y(bi);
    int nA = 0, nB = 0;
    bool aA, aB;
    if (bx == 0) {
        aA = S.extA[bi] >= 0;
        nA = aA ? S.extA[bi] : 0;
    }
    else {
        const int ni = blk_idx(bx - 4, by);
        aA = true;
        nA = (S.cbp_l & (1 << (ni >> 2))) ? inside(ni) : 0;
    }
    if (by == 0) {
        aB = S.extB[bi] >= 0;
        nB = aB ? S.extB[bi] : 0;
    }
    else {
        const int ni = blk_idx(bx, by - 4);
        aB = true;
        nB = (S.cbp_l & (1 << (ni >> 2))) ? inside(ni) : 0;
    }
    if (aA && aB) return (nA + nB + 1) >> 1;
    if (aA) return nA;
    if (aB) return nB;
    return 0;
}

// The entry-value bookkeeping of a speculated 8x8-family search (fam3 helper
// tasks): v of block b, read from the live TotalCoeffs the search started
// from, keeps every nC class it took part in while v stays in [lo[b], hi[b]].
template <typename T>
HD void iv_tighten(T* lo, T* hi, int b, int l, int h)
{
    if (lo[b] < l) lo[b] = (T)l;
    if (hi[b] > h) hi[b] = (T)(h > 127 ? 127 : h);
}
// the interval of an entry value v (or of a sum of two) that keeps the nC
// class of a read: both neighbours available -> nC = (nA + nB + 1) >> 1, else
// the one available value.  sum: nA + nB (both), else v.
HD void iv_of_sum(int sm, int& l, int& h)  // classes of (sm + 1) >> 1: sm <= 2, 3..6, 7..14, >= 15
{
    l = sm <= 2 ? 0 : (sm <= 6 ? 3 : (sm <= 14 ? 7 : 15));
    h = sm <= 2 ? 2 : (sm <= 6 ? 6 : (sm <= 14 ? 14 : 127));
}
HD void iv_of_one(int v, int& l, int& h)  // classes of v: 0-1, 2-3, 4-7, >= 8
{
    l = v < 2 ? 0 : (v < 4 ? 2 : (v < 8 ? 4 : 8));
    h = v < 2 ? 1 : (v < 4 ? 3 : (v < 8 ? 7 : 127));
}
// nC (as nc_luma_of) where inside(ni, entry) also tells whether the value is
// an entry value; each such read tightens [lo, hi] of its block; a read of
// both neighbours of block bi at once, [lo[16 + bi], hi[16 + bi]] of their sum
template <typename F, typename T>
HD int nc_luma_iv(const Shared& S, int bi, F inside, T* lo, T* hi)
{
    const int bx = blk_x(bi), by = blk_y(bi);
    int nA = 0, nB = 0, ia = -1, ib = -1;
    bool aA, aB;
    if (bx == 0) {
        aA = S.extA[bi] >= 0;
        nA = aA ? S.extA[bi] : 0;
    }
    else {
        const int ni = blk_idx(bx - 4, by);
        aA = true;
        if (S.cbp_l & (1 << (ni >> 2))) {
            bool e = false;
            nA = inside(ni, e);
            if (e) ia = ni;
        }
    }
    if (by == 0) {
        aB = S.extB[bi] >= 0;
        nB = aB ? S.extB[bi] : 0;
    }
    else {
        const int ni = blk_idx(bx, by - 4);
        aB = true;
        if (S.cbp_l & (1 << (ni >> 2))) {
            bool e = false;
            nB = inside(ni, e);
            if (e) ib = ni;
        }
    }
    if (ia >= 0 || ib >= 0) {
        int l, h;
        if (aA && aB) {
            iv_of_sum(nA + nB, l, h);
            if (ia >= 0 && ib >= 0) iv_tighten(lo + 16, hi + 16, bi, l, h);  // both entry values: their sum
            else if (ia >= 0) iv_tighten(lo, hi, ia, l - nB, h - nB);
            else iv_tighten(lo, hi, ib, l - nA, h - nA);
        }
        else {
            iv_of_one(ia >= 0 ? nA : nB, l, h);
            iv_tighten(lo, hi, ia >= 0 ? ia : ib, l, h);
        }
    }
    if (aA && aB) return (nA + nB + 1) >> 1;
    if (aA) return nA;
    if (aB) return nB;
    return 0;
}
// --------------------------------------------------------------------------
// MB start: load neighbours, source, live state
// --------------------------------------------------------------------------
HD void load_nbinfo(const MbState& m, NbInfo& n)
{
    n.avail = 1;
    n.intra = (m.flags & FL_INTRA) ? 1 : 0;
    n.e_type = m.e_type;
    n.part_w = m.part_w;
    n.part_h = m.part_h;
    for (int i = 0; i < 4; ++i) {
        n.sub_w[i] = m.sub_w[i];
        n.sub_h[i] = m.sub_h[i];
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            n.mv[i][j][0] = m.mv[i][j][0];
            n.mv[i][j][1] = m.mv[i][j][1];
        }
}

// diagnostic builds (-DHL_DIAG_INPUTS): digests of everything the decision
// reads from other macroblocks, so that a parity failure names the input that
// differed
HD void mb_diag_inputs(Ctx& c)
{
#if defined(HL_DIAG_INPUTS)
    const FrameArgs& F = c.F;
    Shared& S = c.S;
    const int tid = c.tid, a = c.addr;
    // diagnostic builds: digests of everything the decision reads from other
    // macroblocks, so that a parity failure names the input that differed
    if (tid == 0) {
        auto fnv = [](const void* p, int n, uint32_t h) {
            const uint8_t* b = (const uint8_t*)p;
            for (int i = 0; i < n; ++i) h = (h ^ b[i]) * 16777619u;
            return h;
        };
#if defined(__HIP_DEVICE_COMPILE__)
        uint32_t* d = S.recb.dbg;  // stored with the record at the MB end
        (void)F;
        (void)a;
#else
        uint32_t* d = F.rec[a].dbg;
#endif
        d[0] = fnv(S.top, sizeof(S.top), 2166136261u);
        d[1] = fnv(S.left, sizeof(S.left), 2166136261u);
        d[2] = fnv(S.cleft, sizeof(S.cleft), fnv(S.ctop, sizeof(S.ctop), 2166136261u));
        uint32_t h = 2166136261u;
        for (int w = 1; w < 5; ++w) {
            h = fnv(&S.nb[w].avail, 4, h);
            if (S.nb[w].avail) h = fnv(&S.nb[w], sizeof(NbInfo), h);
        }
        d[3] = fnv(S.mvs, sizeof(S.mvs), fnv(S.mvg, sizeof(S.mvg), h));
        d[4] = fnv(S.extCB, 4, fnv(S.extCA, 4, fnv(S.extB, 16, fnv(S.extA, 16, fnv(S.nb_i4, sizeof(S.nb_i4), fnv(S.nb_pm0, 12, 2166136261u))))));
        d[5] = fnv(&S.cbp_c, 4, fnv(&S.cbp_l, 4, fnv(S.tcc, 8, fnv(S.tc, 16, 2166136261u))));
        d[6] = fnv(S.cac, sizeof(S.cac), fnv(S.src, 256, 2166136261u));
        d[7] = (uint32_t)(c.chain & 0xFF) | ((uint32_t)c.spec << 8);
    }
#else
    (void)c;
#endif
}

#if defined(__HIP_DEVICE_COMPILE__) && HL_MB_THREADS >= 512
// MB start on the device: every global load of the MB start is issued in one
// round -- the MB objects of this address and of A, B, C, D (16-byte words),
// the source samples, the intra neighbour samples of the current picture and
// the CAVLC length tables -- and lands in LDS; the derivations then run from
// LDS, each on its own lanes.  Same results as the host version below.
// The lane assignment needs 512 lanes (smaller workgroups take the generic
// strided version below).
__device__ __forceinline__ void mb_begin(Ctx& c)
{
    const FrameArgs& F = c.F;
    Shared& S = c.S;
    const int tid = c.tid;
    const int a = c.addr;
    const int hasA = c.mbx > 0, hasB = c.mby > 0, hasC = c.mby > 0 && c.mbx < F.mbw - 1, hasD = c.mbx > 0 && c.mby > 0;
    const int xc = c.xL >> 1, yc = c.yL >> 1;
    constexpr int kW = (int)(sizeof(MbState) / 16);  // 16-byte words per MB object
    static_assert(5 * kW + 32 <= 448 && kMbThreads >= 464, "mb_begin lane map");
    // ---- round 1: loads (addresses clamped to valid memory, values unused there)
    uint4 q = make_uint4(0, 0, 0, 0);
    int b1 = kNA, b2 = 0, b3 = 0, b4 = 0;
    if (tid < 5 * kW) {
        const int w = tid / kW, i = tid - w * kW;
        const int off = w == 0 ? 0 : (w == 1 ? -1 : (w == 2 ? -F.mbw : (w == 3 ? -F.mbw + 1 : -F.mbw - 1)));
        const bool avw = w == 0 || (w == 1 ? hasA : (w == 2 ? hasB : (w == 3 ? hasC : hasD)));
        q = gmem(reinterpret_cast<const uint4*>(F.st + (avw ? a + off : a)))[i];
    }
    else if (tid < 5 * kW + 16) {
        q = *gmem(reinterpret_cast<const uint4*>(F.src[0] + (size_t)(c.yL + tid - 5 * kW) * F.W + c.xL));
    }
    else if (tid < 5 * kW + 32) {
        const int k = tid - 5 * kW - 16, comp = k >> 3;
        const uint2 d = *gmem(reinterpret_cast<const uint2*>(F.src[1 + comp] + (size_t)(yc + (k & 7)) * F.Wc + xc));
        q.x = d.x;
        q.y = d.y;
    }
    // intra neighbour samples from the (unfiltered) current picture
    if (tid < 25) {
        const int x = tid - 1;
        if (x < 0 ? hasD : (x < 16 ? hasB : (x < 20 ? hasC : false))) b1 = gmem(F.cur[0])[(size_t)(c.yL - 1) * F.W + c.xL + x];
    }
    else if (tid >= 32 && tid < 48) {
        if (hasA) b1 = gmem(F.cur[0])[(size_t)(c.yL + tid - 32) * F.W + c.xL - 1];
    }
    else if (tid >= 64 && tid < 82) {
        const int comp = (tid - 64) / 9, x = (tid - 64) % 9 - 1;
        if (x < 0 ? hasD : hasB) b1 = gmem(F.cur[1 + comp])[(size_t)(yc - 1) * F.Wc + xc + x];
    }
    else if (tid >= 96 && tid < 112) {
        const int comp = (tid - 96) >> 3, y = (tid - 96) & 7;
        if (hasA) b1 = gmem(F.cur[1 + comp])[(size_t)(yc + y) * F.Wc + xc - 1];
    }
    if (tid < 15 * 16) b2 = kTzLen[tid >> 4][tid & 15];
    if (tid < 3 * 4 * 17) b3 = kTokLen[tid / 68][(tid / 17) % 4][tid % 17];
    if (tid >= 256) b4 = kRbTab.v[(tid - 256) >> 4][tid & 15];
    uint32_t b5 = 0;
    if (tid >= 240 && tid < 240 + 4 * 17) b5 = kTok3Tab.v[(tid - 240) / 17][(tid - 240) % 17];
    // ---- stores
    if (tid < 5 * kW) reinterpret_cast<uint4*>(S.nbst)[tid] = q;
    else if (tid < 5 * kW + 16) reinterpret_cast<uint4*>(S.src)[tid - 5 * kW] = q;
    else if (tid < 5 * kW + 32) {
        const int k = tid - 5 * kW - 16;
        *reinterpret_cast<uint2*>(&S.srcc[k >> 3][(k & 7) * 8]) = make_uint2(q.x, q.y);
    }
    if (tid < 25) S.top[tid] = (int16_t)b1;
    else if (tid >= 32 && tid < 48) S.left[tid - 32] = (int16_t)b1;
    else if (tid >= 64 && tid < 82) S.ctop[(tid - 64) / 9][(tid - 64) % 9] = (int16_t)b1;
    else if (tid >= 96 && tid < 112) S.cleft[(tid - 96) >> 3][(tid - 96) & 7] = (int16_t)b1;
    if (tid < 15 * 16) S.ct.tz[tid >> 4][tid & 15] = (uint8_t)b2;
    if (tid < 3 * 4 * 17) S.ct.tok[tid / 68][(tid / 17) % 4][tid % 17] = (uint8_t)b3;
    if (tid >= 256) S.ct.rb[(tid - 256) >> 4][tid & 15] = (uint8_t)b4;
    if (tid >= 240 && tid < 240 + 4 * 17) S.ct.tok3[(tid - 240) / 17][(tid - 240) % 17] = b5;
    if (tid >= kMbThreads - 48) (&S.be_tcm[0][0])[tid - (kMbThreads - 48)] = 0u;  // every slot empty at the MB start
    if (tid >= 448 && tid < 464) {
        const int8_t* e = kQpelTab[tid - 448];
        const uint32_t q = (uint32_t)(e[0] | (e[1] << 2) | (e[2] << 3) | ((e[3] >= 0) << 4) | ((e[3] >= 0 ? e[3] : 0) << 5) | (e[4] << 7) | (e[5] << 8));
        S.qtab[tid - 448] = q;
        const int o1 = (int)(q & 3) * F.plsz + (int)((q >> 3) & 1) * F.pstride + (int)((q >> 2) & 1);
        S.qoff[tid - 448] = make_int2(o1, (q & 16) ? (int)((q >> 5) & 3) * F.plsz + (int)((q >> 8) & 1) * F.pstride + (int)((q >> 7) & 1) : o1);
    }
    HL_SYNC();
    // ---- round 2: derivations from LDS, spread over the waves
    // availability of MB w (no dynamically indexed array: it would live in scratch)
    auto av = [&](int w) -> bool { return w == 0 || (w == 1 ? hasA : (w == 2 ? hasB : (w == 3 ? hasC : hasD))); };
    if (tid < 30) {  // motion grid: row -1 from D / B / C, column -1 from A, inside undecided
        const int gy = tid / 6, gx = tid % 6, bx = gx - 1, by = gy - 1;
        int w = 0, st = 0, v = 0;
        if (by < 0) w = bx < 0 ? 4 : (bx < 4 ? 2 : 3);
        else if (bx < 0) w = 1;
        if (w && av(w)) {
            const MbState& M = S.nbst[w];
            const int xW = (bx + 4) & 3, yW = (by + 4) & 3;  // 4x4 block of the neighbour
            if (M.flags & FL_INTRA) st = 1;
            else {
                const int x = xW * 4, y = yW * 4;
                const int pi = ((y >> lg2(M.part_h)) << (4 - lg2(M.part_w))) + (x >> lg2(M.part_w));
                const int spi = is8x8(M.e_type) ? (((y & 7) >> lg2(M.sub_h[pi])) << (3 - lg2(M.sub_w[pi]))) + ((x & 7) >> lg2(M.sub_w[pi])) : 0;
                st = 2;
                v = (M.mv[pi][spi][0] & 0xFFFF) | (int)((uint32_t)M.mv[pi][spi][1] << 16);
            }
        }
        S.mvs[gy][gx] = (int8_t)st;
        S.mvg[gy][gx] = v;
    }
    else if (tid >= 64 && tid < 128) {  // neighbour summaries: motion (one word per lane)
        const int w = ((tid - 64) >> 4) + 1, k = (tid - 64) & 15;
        if (av(w)) reinterpret_cast<int32_t*>(&S.nb[w].mv[0][0][0])[k] = reinterpret_cast<const int32_t*>(&S.nbst[w].mv[0][0][0])[k];
    }
    else if (tid >= 128 && tid < 132) {  // neighbour summaries: shape
        const int w = tid - 127;
        NbInfo& n = S.nb[w];
        if (av(w)) {
            const MbState& m = S.nbst[w];
            n.avail = 1;
            n.intra = (m.flags & FL_INTRA) ? 1 : 0;
            n.e_type = m.e_type;
            n.part_w = m.part_w;
            n.part_h = m.part_h;
            for (int i = 0; i < 4; ++i) {
                n.sub_w[i] = m.sub_w[i];
                n.sub_h[i] = m.sub_h[i];
            }
        }
        else n.avail = 0;
    }
    else if (tid >= 132 && tid < 164) {  // A / B intra modes
        const int w = ((tid - 132) >> 4) + 1, i = (tid - 132) & 15;
        if (i == 0) S.nb_pm0[w] = av(w) ? S.nbst[w].pm0 : 0;
        S.nb_i4[w][i] = av(w) ? S.nbst[w].i4mode[i] : 2;
    }
    else if (tid >= 192 && tid < 208) {  // external nC contributions (neighbour MBs are final for this frame)
        const int t = tid - 192, bx = blk_x(t), by = blk_y(t);
        int8_t ea = -2, eb = -2;
        if (bx == 0) {
            if (!hasA) ea = -1;
            else {
                const MbState& A = S.nbst[1];
                const int nb = blk_idx(12, by);
                ea = (A.e_type == ET_PSKIP || !(A.cbp_l & (1 << (nb >> 2)))) ? 0 : A.tc_luma[nb];
            }
        }
        if (by == 0) {
            if (!hasB) eb = -1;
            else {
                const MbState& B = S.nbst[2];
                const int nb = blk_idx(bx, 12);
                eb = (B.e_type == ET_PSKIP || !(B.cbp_l & (1 << (nb >> 2)))) ? 0 : B.tc_luma[nb];
            }
        }
        S.extA[t] = ea;
        S.extB[t] = eb;
    }
    else if (tid >= 208 && tid < 212) {  // chroma external nC: extCA[c*2 + row], extCB[c*2 + col]
        const int t = tid - 208, comp = t >> 1, k = t & 1;
        int8_t ea = -1, eb = -1;
        if (hasA) {
            const MbState& A = S.nbst[1];
            ea = (A.e_type == ET_PSKIP || !(A.cbp_c & 2)) ? 0 : A.tc_cac[comp][k * 2 + 1];
        }
        if (hasB) {
            const MbState& B = S.nbst[2];
            eb = (B.e_type == ET_PSKIP || !(B.cbp_c & 2)) ? 0 : B.tc_cac[comp][2 + k];
        }
        S.extCA[t] = ea;
        S.extCB[t] = eb;
    }
    else if (tid >= 256 && tid < 384) {  // live state of this address (stale from the previous frame)
        const int t = tid - 256;
        S.cac[t >> 6][(t >> 4) & 3][t & 15] = S.nbst[0].cac_level[t >> 6][(t >> 4) & 3][t & 15];
        if (t < 16) S.tc[t] = S.nbst[0].tc_luma[t];
        else if (t < 24) S.tcc[(t - 16) >> 2][(t - 16) & 3] = S.nbst[0].tc_cac[(t - 16) >> 2][(t - 16) & 3];
    }
    else if (tid >= 384 && tid < 400) {  // this MB's decision fields, initial values
        const int i = tid - 384;
        S.i4mode[i] = 2;
        S.prev_flag[i] = 0;
        S.rem_mode[i] = 0;
        reinterpret_cast<int32_t*>(&S.mvd[0][0][0])[i] = 0;
        if (i < 4) {
            S.num_sub[i] = 1;
            S.sub_type[i] = -1;
        }
        if (i == 0) {
            const MbState& M = S.nbst[0];
            S.cbp_l = M.cbp_l;
            S.cbp_c = M.cbp_c;
            S.cbp_l4x4 = 0;
            S.cbp_cac[0] = S.cbp_cac[1] = 0;
            S.cbp_cdc[0] = S.cbp_cdc[1] = 0;
            S.nb[0].avail = 1;
            S.nb[0].intra = 0;
            S.nb[0].e_type = M.e_type;
            S.num_part = 1;
            S.i16mode = 2;
            S.chroma_mode = 0;
            S.mb_type = 0;
        }
    }
    HL_SYNC();
    mb_diag_inputs(c);
}
#else
HD void mb_begin(Ctx& c)
{
    const FrameArgs& F = c.F;
    Shared& S = c.S;
    const int tid = c.tid, nthr = c.nthr;
    const int a = c.addr;
    const int hasA = c.mbx > 0, hasB = c.mby > 0, hasC = c.mby > 0 && c.mbx < F.mbw - 1, hasD = c.mbx > 0 && c.mby > 0;
    const int addrs[5] = {a, a - 1, a - F.mbw, a - F.mbw + 1, a - F.mbw - 1};
    const int av[5] = {1, hasA, hasB, hasC, hasD};
#if defined(__HIP_DEVICE_COMPILE__)
    coop_tables_init(S.ct, tid, nthr);
    for (int t = tid; t < 48; t += nthr) (&S.be_tcm[0][0])[t] = 0u;  // every slot empty at the MB start
    for (int t = tid; t < 16; t += nthr) {
        const int8_t* e = kQpelTab[t];
        const uint32_t q = (uint32_t)(e[0] | (e[1] << 2) | (e[2] << 3) | ((e[3] >= 0) << 4) | ((e[3] >= 0 ? e[3] : 0) << 5) | (e[4] << 7) | (e[5] << 8));
        S.qtab[t] = q;
        const int o1 = (int)(q & 3) * F.plsz + (int)((q >> 3) & 1) * F.pstride + (int)((q >> 2) & 1);
        S.qoff[t] = make_int2(o1, (q & 16) ? (int)((q >> 5) & 3) * F.plsz + (int)((q >> 8) & 1) * F.pstride + (int)((q >> 7) & 1) : o1);
    }
#endif
    // source samples
    for (int t = tid; t < 256; t += nthr) S.src[t] = F.src[0][(c.yL + (t >> 4)) * F.W + c.xL + (t & 15)];
    for (int t = tid; t < 128; t += nthr) {
        const int comp = t >> 6, i = t & 63;
        S.srcc[comp][i] = F.src[1 + comp][((c.yL >> 1) + (i >> 3)) * F.Wc + (c.xL >> 1) + (i & 7)];
    }
    // intra neighbour samples from the (unfiltered) current picture
    for (int t = tid; t < 25; t += nthr) {
        const int x = t - 1;
        int v = kNA;
        if (x < 0) {
            if (hasD) v = F.cur[0][(c.yL - 1) * F.W + c.xL - 1];
        }
        else if (x < 16) {
            if (hasB) v = F.cur[0][(c.yL - 1) * F.W + c.xL + x];
        }
        else if (x < 20) {
            if (hasC) v = F.cur[0][(c.yL - 1) * F.W + c.xL + x];
        }
        S.top[t] = (int16_t)v;
    }
    for (int t = tid; t < 16; t += nthr) S.left[t] = (int16_t)(hasA ? F.cur[0][(c.yL + t) * F.W + c.xL - 1] : kNA);
    for (int t = tid; t < 18; t += nthr) {
        const int comp = t / 9, x = t % 9 - 1;
        int v = kNA;
        if (x < 0) {
            if (hasD) v = F.cur[1 + comp][((c.yL >> 1) - 1) * F.Wc + (c.xL >> 1) - 1];
        }
        else if (hasB) {
            v = F.cur[1 + comp][((c.yL >> 1) - 1) * F.Wc + (c.xL >> 1) + x];
        }
        S.ctop[comp][x + 1] = (int16_t)v;
    }
    for (int t = tid; t < 16; t += nthr) {
        const int comp = t >> 3, y = t & 7;
        S.cleft[comp][y] = (int16_t)(hasA ? F.cur[1 + comp][((c.yL >> 1) + y) * F.Wc + (c.xL >> 1) - 1] : kNA);
    }
    // neighbour MB summaries
    for (int t = tid; t < 4; t += nthr) {
        const int w = t + 1;
        if (av[w]) load_nbinfo(F.st[addrs[w]], S.nb[w]);
        else S.nb[w].avail = 0;
    }
    // motion grid: row -1 from D / B / C, column -1 from A, inside undecided
    for (int t = tid; t < 30; t += nthr) {
        const int gy = t / 6, gx = t % 6, bx = gx - 1, by = gy - 1;
        int w = 0, st = 0, v = 0;
        if (by < 0) w = bx < 0 ? 4 : (bx < 4 ? 2 : 3);
        else if (bx < 0) w = 1;
        if (w && av[w]) {
            const MbState& M = F.st[addrs[w]];
            const int xW = (bx + 4) & 3, yW = (by + 4) & 3;  // 4x4 block of the neighbour
            if (M.flags & FL_INTRA) st = 1;
            else {
                const int x = xW * 4, y = yW * 4;
                const int pi = ((y >> lg2(M.part_h)) << (4 - lg2(M.part_w))) + (x >> lg2(M.part_w));
                const int spi = is8x8(M.e_type) ? (((y & 7) >> lg2(M.sub_h[pi])) << (3 - lg2(M.sub_w[pi]))) + ((x & 7) >> lg2(M.sub_w[pi])) : 0;
                st = 2;
                v = (M.mv[pi][spi][0] & 0xFFFF) | (int)((uint32_t)M.mv[pi][spi][1] << 16);
            }
        }
        S.mvs[gy][gx] = (int8_t)st;
        S.mvg[gy][gx] = v;
    }
    for (int t = tid; t < 2; t += nthr) {
        const int w = t + 1;
        S.nb_pm0[w] = av[w] ? F.st[addrs[w]].pm0 : 0;
        for (int i = 0; i < 16; ++i) S.nb_i4[w][i] = av[w] ? F.st[addrs[w]].i4mode[i] : 2;
    }
    // external nC contributions (neighbour MBs are final for this frame)
    for (int t = tid; t < 16; t += nthr) {
        const int bx = blk_x(t), by = blk_y(t);
        int8_t ea = -2, eb = -2;
        if (bx == 0) {
            if (!hasA) ea = -1;
            else {
                const MbState& A = F.st[addrs[1]];
                const int nb = blk_idx(12, by);
                ea = (A.e_type == ET_PSKIP || !(A.cbp_l & (1 << (nb >> 2)))) ? 0 : A.tc_luma[nb];
            }
        }
        if (by == 0) {
            if (!hasB) eb = -1;
            else {
                const MbState& B = F.st[addrs[2]];
                const int nb = blk_idx(bx, 12);
                eb = (B.e_type == ET_PSKIP || !(B.cbp_l & (1 << (nb >> 2)))) ? 0 : B.tc_luma[nb];
            }
        }
        S.extA[t] = ea;
        S.extB[t] = eb;
    }
    // chroma external nC: extCA[c*2 + row], extCB[c*2 + col]
    for (int t = tid; t < 4; t += nthr) {
        const int comp = t >> 1, k = t & 1;
        int8_t ea = -1, eb = -1;
        if (hasA) {
            const MbState& A = F.st[addrs[1]];
            ea = (A.e_type == ET_PSKIP || !(A.cbp_c & 2)) ? 0 : A.tc_cac[comp][k * 2 + 1];
        }
        if (hasB) {
            const MbState& B = F.st[addrs[2]];
            eb = (B.e_type == ET_PSKIP || !(B.cbp_c & 2)) ? 0 : B.tc_cac[comp][2 + k];
        }
        S.extCA[t] = ea;
        S.extCB[t] = eb;
    }
    // live state of this address (stale from the previous frame)
    const MbState& M = F.st[a];
    for (int t = tid; t < 16; t += nthr) S.tc[t] = M.tc_luma[t];
    for (int t = tid; t < 8; t += nthr) S.tcc[t >> 2][t & 3] = M.tc_cac[t >> 2][t & 3];
    for (int t = tid; t < 128; t += nthr) S.cac[t >> 6][(t >> 4) & 3][t & 15] = M.cac_level[t >> 6][(t >> 4) & 3][t & 15];
    if (tid == 0) {
        S.cbp_l = M.cbp_l;
        S.cbp_c = M.cbp_c;
        S.cbp_l4x4 = 0;
        S.cbp_cac[0] = S.cbp_cac[1] = 0;
        S.cbp_cdc[0] = S.cbp_cdc[1] = 0;
        S.nb[0].avail = 1;
        S.nb[0].intra = 0;
        S.nb[0].e_type = M.e_type;
        S.num_part = 1;
        for (int i = 0; i < 4; ++i) {
            S.num_sub[i] = 1;
            S.sub_type[i] = -1;
        }
        for (int i = 0; i < 16; ++i) {
            S.i4mode[i] = 2;
            S.prev_flag[i] = 0;
            S.rem_mode[i] = 0;
        }
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) S.mvd[i][j][0] = S.mvd[i][j][1] = 0;
        S.i16mode = 2;
        S.chroma_mode = 0;
        S.mb_type = 0;
    }
    HL_SYNC();
    mb_diag_inputs(c);
}
#endif

// --------------------------------------------------------------------------
// Inter candidate evaluation (me_ds.c:527-688 for a list of MVs)
// --------------------------------------------------------------------------
struct PartGeo {
    int px, py, pw, ph, nbw, nblk, lbw, lnb;  // lbw / lnb = log2(nbw) / log2(nblk)
};

// Quarter-pel phase table kQpelTab packed 9 bits per phase:
// plane1 | dx1 << 2 | dy1 << 3 | has2 << 4 | plane2 << 5 | dx2 << 7 | dy2 << 8
HD constexpr uint32_t qpel_entry(int ph)
{
    return (uint32_t)(kQpelTab[ph][0] | (kQpelTab[ph][1] << 2) | (kQpelTab[ph][2] << 3) | ((kQpelTab[ph][3] >= 0) << 4) |
                      ((kQpelTab[ph][3] >= 0 ? kQpelTab[ph][3] : 0) << 5) | (kQpelTab[ph][4] << 7) | (kQpelTab[ph][5] << 8));
}
HD constexpr uint64_t qpel_pack(int first, int n)
{
    uint64_t r = 0;
    for (int i = 0; i < n; ++i) r |= (uint64_t)qpel_entry(first + i) << (9 * i);
    return r;
}

// The candidate list of a step is uniform; each wave keeps its own copy in
// LDS so that no barrier is needed between choosing and evaluating it.
// (xo, yo) = luma origin of the partition inside the MB.
HD void put_cand(Ctx& c, int xo, int yo, int pw, int pht, int i, int mx, int my, int pt = 0, bool writer = true)
{
    const FrameArgs& F = c.F;
    constexpr uint64_t q0 = qpel_pack(0, 7), q1 = qpel_pack(7, 7), q2 = qpel_pack(14, 2);
    const int ph = ((my & 3) << 2) | (mx & 3);
    const uint64_t w = ph < 7 ? q0 : (ph < 14 ? q1 : q2);
    const uint32_t e = (uint32_t)(w >> (9 * (ph < 7 ? ph : (ph < 14 ? ph - 7 : ph - 14)))) & 0x1FF;
    const int X = clip3(-17, F.W + 17, c.xL + xo + (mx >> 2)) + kPad, Y = clip3(-17, F.H + 17, c.yL + yo + (my >> 2)) + kPad;
    CandSlot cs;
#if defined(__HIP_DEVICE_COMPILE__)
    // the phase's two sample offsets from the MB start's table (S.qoff)
    const int2 qo = c.S.qoff[ph];
    const int base = Y * F.pstride + X;
    cs.off1 = qo.x + base;
    cs.off2 = qo.y + base;
    (void)e;
#else
    cs.off1 = (int)(e & 3) * F.plsz + (Y + (int)((e >> 3) & 1)) * F.pstride + X + (int)((e >> 2) & 1);
    cs.off2 = (e & 16) ? (int)((e >> 5) & 3) * F.plsz + (Y + (int)((e >> 8) & 1)) * F.pstride + X + (int)((e >> 7) & 1) : cs.off1;
#endif
    cs.mvx = (int16_t)mx;
    cs.mvy = (int16_t)my;
    cs.pad = pt;  // diamond point index
    (void)pw;
    (void)pht;
    if (writer) c.S.wc[c.tid >> 6][i] = cs;
}

HD double mv_cost(const FrameArgs& F, int dist, int bits, int mvx, int mvy, const int pmv[2])
{
    const int rbc_mv = se_len(mvx - pmv[0]) + se_len(mvy - pmv[1]);
    return dadd((double)dist, dmul((double)(bits + rbc_mv), F.lambda));
}

#if defined(HL_STATS) && !defined(__HIP_DEVICE_COMPILE__)
extern long long g_hl_stats[8];
#endif

// Evaluates the candidates S.wc[wave][0..ncand) of partition g in order.
// Leaves per-candidate cost/rbc/dist/single/cbp in S.cd_*, updates the live
// TotalCoeffsLuma S.tc (last writer) and the Single_ctr chain.
// REC: the 8x8-family helper's instantiation (entry-value intervals recorded)
template <bool REC = false>
HD void eval_candidates(Ctx& c, const PartGeo& g, int ncand, const int pmv[2])
{
#if defined(HL_STATS) && !defined(__HIP_DEVICE_COMPILE__)
    g_hl_stats[0]++;
    g_hl_stats[1] += ncand;
    g_hl_stats[2] += ncand * g.nblk;
    g_hl_stats[3 + (g.nblk == 16 ? 0 : (g.nblk == 4 ? 1 : (g.nblk == 2 ? 2 : 3)))]++;
#endif
    const FrameArgs& F = c.F;
    Shared& S = c.S;
    c.par ^= 1;
    c.p3 = c.p3 == 2 ? 0 : c.p3 + 1;
    Shared::CandRes& R = S.cd[c.par];
    uint8_t(&tcb)[16][kMaxCand] = S.be_tcb[c.par];
    HL_PROF_T(tp0);
#if defined(__HIP_DEVICE_COMPILE__)
    // phase 1: one 4-lane quad per (candidate, 4x4 block), lane r = block row
    // r (hl_quad.h); every quad issues its prediction loads for both rounds
    // before computing
    {
        const int wave = c.tid >> 6, qg = c.tid >> 2, nq = c.nthr >> 2;
        const int n = ncand << g.lnb;
        const int qp = uni(F.qp);  // scalar: the quantiser's shifts and the dequantiser's form are uniform
        const int qbits = 15 + qp / 6, f = (1 << qbits) / 6;
        LaneQ Q = c.Q;
        if (HL_FRESH_ZZ & 1) Q.zz = laneq_zz_fresh(Q.r);
        const auto base = gmem(F.pl[0]);
        // single-block partitions: both nC neighbours lie outside the partition,
        // so nC is fixed for its whole search (read here, beside the loads)
        const int nc1 = g.nblk == 1 ? nc_luma_of(S, blk_idx(g.px, g.py), [&](int ni) -> int { return S.tc[ni]; }) : 0;
        if (HL_F3REC(c) && g.nblk == 1 && c.tid == 0)  // fam3_helper: its entry reads (lane 0; phase 2 does not run)
            nc_luma_iv(S, blk_idx(g.px, g.py), [&](int ni, bool& e) -> int {
                e = !((S.f3w >> ni) & 1);
                return S.tc[ni];
            }, S.f3lo, S.f3hi);
        int o1[kQPass], o2[kQPass];
        uint32_t sv[kQPass], pr[kQPass];
#pragma unroll
        for (int j = 0; j < kQPass; ++j) {
            const int item = min(qg + j * nq, n - 1);  // clamped: no divergence, valid addresses
            const int ci = item >> g.lnb, k = item & (g.nblk - 1);
            const int hx = k & (g.nbw - 1), hy = k >> g.lbw;
            const int2 cs = *reinterpret_cast<const int2*>(&S.wc[wave][ci]);
            const int o = ((hy << 2) + Q.r) * F.pstride + (hx << 2);
            o1[j] = cs.x + o;
            o2[j] = cs.y + o;
            sv[j] = *reinterpret_cast<const uint32_t*>(&S.src[(g.py + (hy << 2) + Q.r) * 16 + g.px + (hx << 2)]);
        }
        HL_PROF_T(ta0);
        {
#pragma unroll
            for (int j = 0; j < kQPass; ++j)
                if (qg + j * nq < n) pr[j] = avg_u8x4(ld_u8x4(base, o1[j]), ld_u8x4(base, o2[j]));
        }
#if defined(HL_STEP_PROF)
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // the loads' latency (profiling only)
        HL_PROF_ADD(c, 12, ta0);
#endif
        HL_PROF_T(ta1);
#pragma unroll
        for (int j = 0; j < kQPass; ++j) {
            const int item = qg + j * nq;
            if (item < n) {
#if defined(HL_NOP_PROBE)  // timing experiment: HL_NOP_PROBE x 8 independent VALU issue slots per quad round
#pragma unroll
                for (int np = 0; np < HL_NOP_PROBE; ++np) asm volatile("v_nop\n v_nop\n v_nop\n v_nop\n v_nop\n v_nop\n v_nop\n v_nop");
#endif
                const int ci = item >> g.lnb, k = item & (g.nblk - 1);
                int x[4], y[4], q[4];
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) x[cc] = (int)((sv[j] >> (8 * cc)) & 255) - (int)((pr[j] >> (8 * cc)) & 255);
                quad_fwd(Q, x, y);
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) q[cc] = quad_q1(y[cc], (cc & 1) ? Q.mfO : Q.mfE, qbits, f);
                CoopStat st{0, 0, 0, -1};
                int tok = 0, dist;
                if (__ballot((q[0] | q[1] | q[2] | q[3]) != 0) == 0) {  // every block of the wave quantised to zero
                    dist = quad_sum((int)__builtin_amdgcn_sad_u8(sv[j], pr[j], 0u));  // the row's sum of |residual|
                }
                else {
                    // reconstruction distortion first: independent of the CAVLC
                    // chain, so the two interleave
                    int r[4];
                    quad_idct(Q, q, qp, r);
                    uint32_t rec = 0;  // the row's reconstructed samples, packed
#pragma unroll
                    for (int cc = 0; cc < 4; ++cc) rec |= (uint32_t)clip255((int)((pr[j] >> (8 * cc)) & 255) + r[cc]) << (8 * cc);
                    dist = quad_sum((int)__builtin_amdgcn_sad_u8(sv[j], rec, 0u));
                    st = quad_cavlc(S.ct, Q, q, 0, S.lvq[qg]);
                    if (Q.r == 0 && st.tc) tok = (int)S.ct.tok3[st.t1][st.tc];  // coeff_token lengths for the four nC classes
                }
                if (Q.r == 0) {
                    S.be_w[ci][k] = make_int4(st.tc | (st.t1 << 5) | ((st.sctr + 1) << 8), st.rest | (dist << 16), tok, 0);
                    tcb[k][ci] = (uint8_t)st.tc;
                    if (st.tc) atomicOr(&S.be_tcm[c.p3][k], 1u << ci);
                    if (g.nblk == 1) {
                        // a single-block partition: both nC neighbours lie outside it, so the
                        // nC (and the candidate's cost) needs no other block (phase 2 skipped)
                        int bits = 0;
                        if (st.tc) bits = st.rest + ((tok >> (5 * (nc1 < 2 ? 0 : (nc1 < 4 ? 1 : (nc1 < 8 ? 2 : 3))))) & 31);
                        const CandSlot cs = S.wc[wave][ci];
                        R.cost[ci] = mv_cost(F, dist, bits, cs.mvx, cs.mvy, pmv);
                        R.bits[ci] = bits;
                        R.dist[ci] = dist;
                        R.single[ci] = st.tc ? st.sctr : 0;
                        R.cbp[ci] = st.tc ? 1 << blk_idx(g.px, g.py) : 0;
                        R.last[ci] = st.tc ? st.sctr : -1;
                    }
                }
            }
        }
#if defined(HL_STEP_PROF)
        HL_PROF_ADD(c, 13, ta1);
#endif
    }
#if defined(HL_STEP_PROF)
    HL_PROF_T(tb0);
    HL_SYNC();
    HL_PROF_ADD(c, 14, tb0);
#else
    HL_SYNC();
#endif
#if defined(__HIP_DEVICE_COMPILE__)
    // the slot the pass after next ORs into: its last readers (the phase 2
    // and commit of the pass before this one) are done, and its first
    // writer runs after the next pass's barrier above
    if (c.tid < 16) S.be_tcm[c.p3 == 0 ? 2 : c.p3 - 1][c.tid] = 0;
#endif
#if defined(HL_NBLK_PROF)  // phase 1 by partition size: slots 12..15 = 1, 2, 4, 8+ blocks
    HL_PROF_ADD(c, 12 + (g.nblk >= 8 ? 3 : g.lnb), tp0);
#endif
    HL_PROF_ADD(c, 0, tp0);
    HL_PROF_T(tp1);
    // phase 2: one row per candidate, one lane per block: nC as the reference
    // sees it at this point of the sequence (residual.c:640-755 with the live
    // TotalCoeffs of quirk 1), coeff_token, candidate sums, cost.  All LDS
    // reads are issued up front.
    // (one round at 512 lanes; smaller workgroups take more)
    constexpr int kRowRounds = (kMaxCand + kMbRows - 1) / kMbRows;
#pragma unroll
    for (int rr = 0; rr < kRowRounds; ++rr)
    if (g.nblk > 1 && c.tid + rr * kMbThreads < (ncand << 4)) {
        const int wave = c.tid >> 6, ci = (c.tid >> 4) + rr * kMbRows, k0 = c.tid & 15;
        const bool valid = k0 < g.nblk;
        const int k = valid ? k0 : 0;
        const int hx = k & (g.nbw - 1), hy = k >> g.lbw;
        const int bx = g.px + (hx << 2), by = g.py + (hy << 2);
        const int bi = blk_idx(bx, by);
        const int niA = bx ? blk_idx(bx - 4, by) : 0, niB = by ? blk_idx(bx, by - 4) : 0;
        const bool inA = bx - 4 >= g.px, inB = by - 4 >= g.py;  // neighbour inside the partition
        const int kkA = inA ? ((hy << g.lbw) + hx - 1) : 0, kkB = inB ? (((hy - 1) << g.lbw) + hx) : 0;
        const int4 wq = S.be_w[ci][k];
        const int w0 = wq.x, w1 = wq.y, w2 = wq.z;
        const int eA = S.extA[bi], eB = S.extB[bi], cbp = S.cbp_l, tA = S.tc[niA], tB = S.tc[niB];
        const int f3w = HL_F3REC(c) ? S.f3w : 0;
        const uint8_t *rA = tcb[kkA], *rB = tcb[kkB];
        const CandSlot cs = S.wc[wave][ci];
        int bits = 0, dist = 0, cs_sum = 0, last = 0;
        const int tc = w0 & 31;
        if (!HL_FAM3 || !REC) {
            // selects throughout (no exec-mask branches): the neighbours'
            // TotalCoeffs as the nC reads them (live value of the last
            // candidate up to ci that coded the block inside the partition,
            // else the live state; 0 without coded luma in the 8x8; the
            // neighbouring MB's value at the MB edge, -1 = not available)
            const uint32_t allow = ci == 31 ? ~0u : (2u << ci) - 1u;  // candidates 0..ci
            const bool cA = (cbp >> (niA >> 2)) & 1, cB = (cbp >> (niB >> 2)) & 1;
            const uint32_t mA = inA ? S.be_tcm[c.p3][kkA] & allow : 0u, mB = inB ? S.be_tcm[c.p3][kkB] & allow : 0u;
            const int vA = rA[mA ? 31 - __clz(mA) : 0], vB = rB[mB ? 31 - __clz(mB) : 0];
            const bool aA = bx ? true : eA >= 0, aB = by ? true : eB >= 0;
            const int nA = bx ? (cA ? (mA ? vA : tA) : 0) : (aA ? eA : 0);
            const int nB = by ? (cB ? (mB ? vB : tB) : 0) : (aB ? eB : 0);
            const int nC = (aA && aB) ? (nA + nB + 1) >> 1 : (aA ? nA : (aB ? nB : 0));
            const int cls = nC < 2 ? 0 : (nC < 4 ? 1 : (nC < 8 ? 2 : 3));
            const int sctr = ((w0 >> 8) & 15) - 1;
            const bool coded = valid && tc;
            dist = valid ? w1 >> 16 : 0;
            bits = coded ? (w1 & 0xFFFF) + ((w2 >> (5 * cls)) & 31) : 0;
            cs_sum = coded ? (1 << bi) | (sctr << 16) : 0;
            last = coded ? ((k + 1) << 4) | sctr : 0;
            (void)f3w;
        }
        else
        if (valid) {
            dist = w1 >> 16;
            if (tc) {
                const uint32_t allow = ci == 31 ? ~0u : (2u << ci) - 1u;  // candidates 0..ci
                int nA = 0, nB = 0;
                bool aA = true, aB = true, enA = false, enB = false;  // en: an entry value of the family (fam3_helper)
                if (bx == 0) {
                    aA = eA >= 0;
                    nA = aA ? eA : 0;
                }
                else if (cbp & (1 << (niA >> 2))) {
                    const uint32_t mA = inA ? S.be_tcm[c.p3][kkA] & allow : 0u;
                    const int v = mA ? (int)rA[31 - __clz(mA)] : -1;
                    nA = v >= 0 ? v : tA;
                    enA = HL_F3REC(c) && v < 0 && !((f3w >> niA) & 1);
                }
                if (by == 0) {
                    aB = eB >= 0;
                    nB = aB ? eB : 0;
                }
                else if (cbp & (1 << (niB >> 2))) {
                    const uint32_t mB = inB ? S.be_tcm[c.p3][kkB] & allow : 0u;
                    const int v = mB ? (int)rB[31 - __clz(mB)] : -1;
                    nB = v >= 0 ? v : tB;
                    enB = HL_F3REC(c) && v < 0 && !((f3w >> niB) & 1);
                }
                const int nC = (aA && aB) ? (nA + nB + 1) >> 1 : (aA ? nA : (aB ? nB : 0));
                if (enA || enB) {  // the interval of the entry value(s) keeping this nC's class
                    int l, h, ix;
                    if (aA && aB) {
                        iv_of_sum(nA + nB, l, h);
                        if (enA && enB) ix = 16 + bi;
                        else if (enA) {
                            ix = niA;
                            l -= nB;
                            h -= nB;
                        }
                        else {
                            ix = niB;
                            l -= nA;
                            h -= nA;
                        }
                    }
                    else {
                        iv_of_one(enA ? nA : nB, l, h);
                        ix = enA ? niA : niB;
                    }
                    atomicMax(&S.f3lo[ix], l);
                    atomicMin(&S.f3hi[ix], min(h, 127));
                }
                const int cls = nC < 2 ? 0 : (nC < 4 ? 1 : (nC < 8 ? 2 : 3));
                const int sctr = ((w0 >> 8) & 15) - 1;
                bits = (w1 & 0xFFFF) + ((w2 >> (5 * cls)) & 31);
                cs_sum = (1 << bi) | (sctr << 16);
                last = ((k + 1) << 4) | sctr;
            }
        }
        // bits (< 2^15 over 16 blocks) and distortion (< 2^17) in one row sum
        const uint32_t pk = (uint32_t)row_sum((int)((uint32_t)bits | ((uint32_t)dist << 15)));
        bits = (int)(pk & 0x7FFFu);
        dist = (int)(pk >> 15);
        cs_sum = row_sum(cs_sum);
        last = row_max(last);
        if (k0 == 0) {
            R.cost[ci] = mv_cost(F, dist, bits, cs.mvx, cs.mvy, pmv);
            R.bits[ci] = bits;
            R.dist[ci] = dist;
            R.single[ci] = cs_sum >> 16;
            R.cbp[ci] = cs_sum & 0xFFFF;
            R.last[ci] = last ? (last & 15) : -1;
        }
    }
    if (g.nblk > 1) HL_SYNC();
    HL_PROF_ADD(c, 1, tp1);
#else
    HL_PROF_T(tp2);
    const int n = ncand * g.nblk;
    // phase 1: transform / quant / CAVLC statistics / reconstruction per block
    for (int t = c.tid; t < n; t += c.nthr) {
        const int ci = t / g.nblk, k = t % g.nblk;
        const int hx = k % g.nbw, hy = k / g.nbw;
        const int mvx = S.wc[0][ci].mvx, mvy = S.wc[0][ci].mvy;
        const int X = clip3(-17, F.W + 17, c.xL + g.px + (mvx >> 2)) + (hx << 2);
        const int Y = clip3(-17, F.H + 17, c.yL + g.py + (mvy >> 2)) + (hy << 2);
        const int bx = g.px + (hx << 2), by = g.py + (hy << 2);
        int pred[16], res[16];
        pred_luma4x4(F, X, Y, mvx & 3, mvy & 3, pred);
        bool zero = true;
        for (int i = 0; i < 16; ++i) {
            res[i] = (int)S.src[(by + (i >> 2)) * 16 + bx + (i & 3)] - pred[i];
            zero = zero && res[i] == 0;
        }
        int nz = 0, dist = 0;
        CavlcStat st = {0, 0, 0, -1};
        if (!zero) {
            int w[16], q[16], lv[16];
            fwd4x4(res, w);
            quant4x4(F.qp, false, w, q);
            bool lz = true;
            for (int i = 0; i < 16; ++i) {
                lv[i] = q[kZigzag[i]];
                lz = lz && lv[i] == 0;
            }
            if (!lz) {
                nz = 1;
                st = cavlc_stat(lv, 16, 15, false);
                int r[16];
                dequant_idct(F.qp, q, false, r);
                for (int i = 0; i < 16; ++i) dist += iabs(res[i] - (clip255(pred[i] + r[i]) - pred[i]));
            }
            else {
                for (int i = 0; i < 16; ++i) dist += iabs(res[i]);
            }
        }
        S.be_nz[ci][k] = nz;
        S.be_tc[ci][k] = st.tc;
        S.be_t1[ci][k] = st.t1;
        S.be_sctr[ci][k] = st.sctr;
        S.be_bits[ci][k] = st.rest;
        S.be_dist[ci][k] = dist;
    }
    // phase 2: nC as the reference sees it at this point of the sequence
    for (int t = c.tid; t < n; t += c.nthr) {
        const int ci = t / g.nblk, k = t % g.nblk;
        if (!S.be_nz[ci][k]) continue;
        const int hx = k % g.nbw, hy = k / g.nbw;
        const int bi = blk_idx(g.px + (hx << 2), g.py + (hy << 2));
        auto inside = [&](int ni, bool& entry) -> int {
            const int nx = blk_x(ni) - g.px, ny = blk_y(ni) - g.py;
            if (nx >= 0 && ny >= 0 && nx < g.pw && ny < g.ph) {
                const int kk = (ny >> 2) * g.nbw + (nx >> 2);
                if (S.be_nz[ci][kk]) return S.be_tc[ci][kk];
                for (int cj = ci - 1; cj >= 0; --cj)
                    if (S.be_nz[cj][kk]) return S.be_tc[cj][kk];
            }
            entry = c.f3rec && !((S.f3w >> ni) & 1);
            return S.tc[ni];
        };
        const int nC = nc_luma_iv(S, bi, inside, S.f3lo, S.f3hi);
        S.be_bits[ci][k] += token_len(nC, S.be_tc[ci][k], S.be_t1[ci][k]);
    }
    // phase 3: per-candidate sums
    for (int t = 0; t < ncand; ++t) {
        int bits = 0, dist = 0, single = 0, cbp = 0, last = -1;
        for (int k = 0; k < g.nblk; ++k) {
            dist += S.be_dist[t][k];
            if (S.be_nz[t][k]) {
                const int hx = k % g.nbw, hy = k / g.nbw;
                bits += S.be_bits[t][k];
                single += S.be_sctr[t][k];
                cbp |= 1 << blk_idx(g.px + (hx << 2), g.py + (hy << 2));
                last = S.be_sctr[t][k];
            }
        }
        R.cost[t] = mv_cost(F, dist, bits, S.wc[0][t].mvx, S.wc[0][t].mvy, pmv);
        R.bits[t] = bits;
        R.dist[t] = dist;
        R.single[t] = single;
        R.cbp[t] = cbp;
        R.last[t] = last;
    }
#endif
}

// The live state left by the first n candidates of the last evaluation, in
// order (the reference's sequence of trial CAVLC writes): TotalCoeffsLuma of
// every block = its last writer (residual.c:796-806); rdo.Single_ctr = the
// last candidate that wrote it (residual.c:881-897).  The next reader of
// S.tc is behind a barrier.
// last_l: candidate (tid & 31)'s R.last when the caller has it in a register
// (device; -2 = read it here)
template <bool REC = false>
HD void commit_candidates(Ctx& c, const PartGeo& g, int n, int last_l = -2)
{
    Shared& S = c.S;
    const Shared::CandRes& R = S.cd[c.par];
    HL_PROF_T(tp2);
#if defined(__HIP_DEVICE_COMPILE__)
    const uint8_t(&tcb)[16][kMaxCand] = S.be_tcb[c.par];
    if (c.tid < g.nblk) {
        const int k = c.tid;
        const uint32_t mk = S.be_tcm[c.p3][k] & (n >= 32 ? ~0u : (1u << n) - 1u);
        const int v = mk ? (int)tcb[k][31 - __clz(mk)] : -1;
        const int bi = blk_idx(g.px + ((k & (g.nbw - 1)) << 2), g.py + ((k >> g.lbw) << 2));
        if (v >= 0) {
            S.tc[bi] = (int8_t)v;
            if (HL_F3REC(c)) atomicOr(&S.f3w, 1 << bi);
        }
    }
    {  // last candidate that wrote the counter (vectorised over the pass)
        const int l = c.tid & 31;
        const int v = l < n ? (last_l == -2 ? R.last[l] : last_l) : -1;
        const unsigned long long bal = __ballot(v >= 0) & 0xFFFFFFFFull;
        if (bal) chain_write(c, __builtin_amdgcn_readlane(v, 63 - __clzll((long long)bal)));
    }
#else
    (void)last_l;
    for (int k = 0; k < g.nblk; ++k) {
        const int hx = k % g.nbw, hy = k / g.nbw;
        const int bi = blk_idx(g.px + (hx << 2), g.py + (hy << 2));
        for (int cj = n - 1; cj >= 0; --cj)
            if (S.be_nz[cj][k]) {
                S.tc[bi] = (int8_t)S.be_tc[cj][k];
                if (c.f3rec) S.f3w |= 1 << bi;
                break;
            }
    }
    for (int ci = n - 1; ci >= 0; --ci)
        if (R.last[ci] >= 0) {
            chain_write(c, R.last[ci]);
            break;
        }
#endif
    HL_PROF_ADD(c, 2, tp2);
}

// The sequential strict-< scan of one step's candidates (me_ds.c:339-347):
// index of the first candidate with the smallest cost, and that cost.
HD int pick_first_min(const Ctx& c, int lo, int hi, double& m)  // candidates [lo, hi), hi > lo
{
    const Shared& S = c.S;
#if defined(__HIP_DEVICE_COMPILE__)
    const int l = c.tid & 31;
    const bool in = l >= lo && l < hi;
    const double v = in ? S.cd[c.par].cost[l] : 1.7976931348623157e308;
    double mn = row_min_f64(v);
    mn = fmin(mn, __shfl_xor(mn, 16, 64));  // both 16-lane rows of the half-wave
    const unsigned long long bal = __ballot(in && v == mn) & 0xFFFFFFFFull;
    m = uni(mn);
    return uni(__ffsll((long long)bal) - 1);
#else
    int bi = lo;
    m = S.cd[c.par].cost[lo];
    for (int ci = lo + 1; ci < hi; ++ci)
        if (S.cd[c.par].cost[ci] < m) {
            m = S.cd[c.par].cost[ci];
            bi = ci;
        }
    return bi;
#endif
}

// Search state of one (sub)partition, uniform across lanes
struct Best {
    double cost;
    int dist, single, cbp, mv[2];
};

HD int ilog2_small(int v) { return v >= 16 ? 4 : (v >= 8 ? 3 : (v >= 4 ? 2 : (v >= 2 ? 1 : 0))); }

// Pipelined runs (hl_pipeline.h): the task of a picture after which the
// quarter-pel planes of all its MBs (X' <= X, Y' <= Y) are final.  Plane
// blocks of (X, Y) run in task (X+2, Y+2), in the last rows in (X+3, mbh-1)
// (trig_pl); a finished task implies every task before it in both
// wavefront directions.  Model-checked by tests/test_pipeline_schedule.py.
HD void reach_task(int X, int Y, int mbw, int mbh, int& tx, int& ty)
{
    ty = Y + 2 < mbh - 1 ? Y + 2 : mbh - 1;
    const int k = ty == mbh - 1 ? 3 : 2;
    tx = X + k < mbw - 1 ? X + k : mbw - 1;
}

// Pipelined runs: before a partition search, make sure the reference
// picture's planes cover its motion window.  The integer diamond stays
// within +-me_range of its start (the MVP or (0,0), me_ds.c:302-358); the
// half and quarter stages add at most me_range / 2 + me_range / 4 pels
// (me_ds.c:360-470), and a quarter-pel fetch reads one sample further: the
// last sample read lies within start + 1.75 * me_range + 2 of the block.
// The task start guarantees MBs up to (gx, gy); a window reaching further
// waits for the reference picture's task that covers it.  Negative
// directions are always covered.
HD void reach_wait(Ctx& c, const PartGeo& g, const int pmv[2])
{
#if defined(__HIP_DEVICE_COMPILE__)
    const FrameArgs& F = c.F;
    if (!F.ref_done) return;
    const int ext = F.me_range + (F.me_range >> 1) + ((F.me_range + 3) >> 2) + 2;
    const int px = c.xL + g.px + g.pw - 1 + (pmv[0] > 0 ? pmv[0] >> 2 : 0) + ext;
    const int py = c.yL + g.py + g.ph - 1 + (pmv[1] > 0 ? pmv[1] >> 2 : 0) + ext;
    int X = min(F.mbw - 1, max(0, px >> 4)), Y = min(F.mbh - 1, max(0, py >> 4));
    if (X <= c.gx && Y <= c.gy) return;
    X = max(X, c.gx);
    Y = max(Y, c.gy);
    HL_PROF_T(tw);
    if (c.tid == 0) {
        int tx, ty;
        reach_task(X, Y, F.mbw, F.mbh, tx, ty);
        spin_ge(F.ref_done + ty * F.mbw + tx, F.ref_epoch, F.perr);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, HL_ACQ_SCOPE);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    HL_SYNC();
    HL_PROF_ADD(c, 9, tw);
    c.gx = X;
    c.gy = Y;
#else
    (void)c;
    (void)g;
    (void)pmv;
#endif
}

// Diamond search of one (sub)partition, me_ds.c:104-477.  Returns true when
// the P_Skip probe fired (16x16 only).
template <bool REC = false>
HD bool search_partition(Ctx& c, const PartDef& pd, int pi, int spi, bool probe)
{
    // (no HL_FRESH_TID here: ROCm 7.2's greedy register allocator crashes on it)
    Shared& S = c.S;
    HL_PROF_T(tsp);
    const int xP = part_x(pi, pd.part_w), yP = part_y(pi, pd.part_w, pd.part_h);
    int xS = 0, yS = 0;
    if (pd.num_part == 4) {
        xS = sub_x(spi, pd.sub_w);
        yS = sub_y(spi, pd.sub_w, pd.sub_h);
    }
    PartGeo g;
    g.px = xP + xS;
    g.py = yP + yS;
    g.pw = pd.sub_w;
    g.ph = pd.sub_h;
    g.nbw = g.pw >> 2;
    g.nblk = (g.pw >> 2) * (g.ph >> 2);
    g.lbw = ilog2_small(g.nbw);
    g.lnb = ilog2_small(g.nblk);
    Best b;
    b.cost = 1.7976931348623157e308;
    b.dist = 0x7fffffff;
    b.single = 9;
    b.cbp = 0;
    b.mv[0] = b.mv[1] = 0;
    bool probably = false;
    int pmv[2];
    {
        HL_PROF_T(tm);
        const PartShape ps{pd.part_w, pd.part_h, pd.sub_w, pd.sub_h, pd.num_part == 4};
        mvp(S, ps, pi, spi, pmv);
        pmv[0] = uni(pmv[0]);
        pmv[1] = uni(pmv[1]);
        HL_PROF_ADD(c, 4, tm);
    }
    reach_wait(c, g, pmv);
    if (probe) {  // me_ds.c:229-261 (the probe's predictor is the 16x16 one, pmv)
        int smv[2];
        skip_mv(S, smv);
        smv[0] = uni(smv[0]);
        smv[1] = uni(smv[1]);
        if (pmv[0] == smv[0] && pmv[1] == smv[1]) {
            put_cand(c, g.px, g.py, g.pw, g.ph, 0, pmv[0], pmv[1], 0, (c.tid & 63) == 0);
            eval_candidates<REC>(c, g, 1, pmv);
            commit_candidates<REC>(c, g, 1);
            if (uni(S.cd[c.par].bits[0]) == 0 || uni(S.cd[c.par].single[0]) < 6) {
                probably = true;
                b.cost = 0.0;
                b.single = uni(S.cd[c.par].single[0]);
                b.dist = uni(S.cd[c.par].dist[0]);
                b.cbp = uni(S.cd[c.par].cbp[0]);
                b.mv[0] = pmv[0];
                b.mv[1] = pmv[1];
            }
        }
    }
    // The search is a sequence of steps (me_ds.c:280-470): the MVP and (0,0)
    // candidates (stage 3), then diamond steps of the integer (2), half (1)
    // and quarter (0) stages.  A step that finds no better point ends its
    // stage, and the next stage's first step is then fully determined by the
    // unchanged best MV; after the MVP/(0,0) step the next step is known
    // once its winner is (the MVP is predicted).  One evaluation pass
    // therefore holds a chain of up to kMaxSeg steps -- the current one and
    // the speculative continuations that fit the pass (at most kMaxCand
    // candidates, kMaxPass rows per lane) -- in the reference's evaluation
    // order, so every nC (quirk 1) and cost in the chain is exact for as long
    // as the speculation holds.  The chain is resolved step by step; at the
    // first step whose outcome differs from the prediction the rest is
    // dropped, and only the candidates of the resolved steps are committed
    // to the live state.
    // diamond stages, me_ds.c:302-470.  The point offsets and visited-point
    // masks are packed into immediates (3-bit offsets + 2, 9-bit masks).
    // integer: {0,2},{-1,1},{1,1},{-2,0},{0,0},{2,0},{-1,-1},{1,-1},{0,-2}
    // half:    {0,1},{-1,0},{0,-1},{1,0},{0,0}
    // quarter: {-1,1},{0,1},{1,1},{-1,0},{0,0},{1,0},{-1,-1},{0,-1},{1,-1}
    auto pk3 = [](const int* v, int n) -> uint32_t {
        uint32_t r = 0;
        for (int i = 0; i < n; ++i) r |= (uint32_t)(v[i] + 2) << (3 * i);
        return r;
    };
    static constexpr int kIntX[9] = {0, -1, 1, -2, 0, 2, -1, 1, 0}, kIntY[9] = {2, 1, 1, 0, 0, 0, -1, -1, -2};
    static constexpr int kHalfX[5] = {0, -1, 0, 1, 0}, kHalfY[5] = {1, 0, -1, 0, 0};
    static constexpr int kQuarX[9] = {-1, 0, 1, -1, 0, 1, -1, 0, 1}, kQuarY[9] = {1, 1, 1, 0, 0, 0, -1, -1, -1};
    const uint32_t pIntX = pk3(kIntX, 9), pIntY = pk3(kIntY, 9), pHalfX = pk3(kHalfX, 5), pHalfY = pk3(kHalfY, 5);
    const uint32_t pQuarX = pk3(kQuarX, 9), pQuarY = pk3(kQuarY, 9);
    // visited-point masks after a move to point i (low 9 bits; bit 4 = centre)
    auto mask_of = [](int shift, int i) -> int {
        constexpr uint64_t mi0 = (uint64_t)(0x1FF & ~(16 | 64 | 256 | 128)) | (uint64_t)(0x1FF & ~(16 | 32 | 256)) << 9 |
                                 (uint64_t)(0x1FF & ~(16 | 2 | 8 | 64 | 256 | 128)) << 18 | (uint64_t)(0x1FF & ~(16 | 4 | 32 | 128)) << 27 |
                                 (uint64_t)0x1FF << 36 | (uint64_t)(0x1FF & ~(16 | 2 | 8 | 64)) << 45 |
                                 (uint64_t)(0x1FF & ~(16 | 1 | 2 | 128 | 32 | 4)) << 54;
        constexpr uint32_t mi1 = (0x1FF & ~(16 | 1 | 2 | 8 | 64 | 4)) | (0x1FF & ~(16 | 4 | 1 | 2)) << 9;
        constexpr uint64_t mh = (uint64_t)(0x1FF & ~(16 | 4)) | (uint64_t)(0x1FF & ~(16 | 8)) << 9 | (uint64_t)(0x1FF & ~(16 | 1)) << 18 |
                                (uint64_t)(0x1FF & ~(16 | 2)) << 27 | (uint64_t)0x1FF << 36;
        constexpr uint64_t mq0 = (uint64_t)(0x1FF & ~(16 | 32 | 256 | 128)) | (uint64_t)(0x1FF & ~(16 | 8 | 64 | 128 | 256 | 32)) << 9 |
                                 (uint64_t)(0x1FF & ~(16 | 8 | 1 | 2 | 4 | 32)) << 18 | (uint64_t)(0x1FF & ~(16 | 2 | 4 | 32 | 256 | 128)) << 27 |
                                 (uint64_t)0x1FF << 36 | (uint64_t)(0x1FF & ~(16 | 1 | 2 | 8 | 64 | 128)) << 45 |
                                 (uint64_t)(0x1FF & ~(16 | 2 | 4 | 32)) << 54;
        constexpr uint32_t mq1 = (0x1FF & ~(16 | 1 | 2 | 4 | 8 | 32)) | (0x1FF & ~(16 | 1 | 2 | 8)) << 9;
        uint64_t w;
        int k = i;
        if (shift == 1) w = mh;
        else if (i < 7) w = shift == 2 ? mi0 : mq0;
        else {
            w = shift == 2 ? mi1 : mq1;
            k = i - 7;
        }
        return (int)((w >> (9 * k)) & 0x1FF);
    };
    const int range = c.F.me_range;
    const int budget = g.nblk <= kSpecMaxBlocks ? min(kMaxCand, kPassItems >> g.lnb) : 0;  // 0: one step per pass
    const int nc0 = (pmv[0] != 0 || pmv[1] != 0) ? 2 : 1;
    int stage = 3, flags = 0x1FF, cx = 0, cy = 0, left = 0, right = 0, top = 0, bottom = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    // a pass's candidate results, lane l (and l + 32) holding candidate l:
    // loaded once per pass, then every pick and take is register work
    double pv_cost = 0.0;
    int pv_single = 0, pv_dist = 0, pv_cbp = 0, pv_mvx = 0, pv_mvy = 0, pv_pad = 0, pv_last = -1;
    auto take = [&](int bi, double m) {
        b.cost = m;
        b.single = __builtin_amdgcn_readlane(pv_single, bi);
        b.dist = __builtin_amdgcn_readlane(pv_dist, bi);
        b.cbp = __builtin_amdgcn_readlane(pv_cbp, bi);
        b.mv[0] = __builtin_amdgcn_readlane(pv_mvx, bi);
        b.mv[1] = __builtin_amdgcn_readlane(pv_mvy, bi);
        return __builtin_amdgcn_readlane(pv_pad, bi);
    };
    // the sequential strict-< scan of candidates [lo, hi) (me_ds.c:339-347):
    // index of the first candidate with the smallest cost, and that cost
    auto pick = [&](int lo, int hi, double& m) -> int {
        const int l = c.tid & 31;
        const bool in = l >= lo && l < hi;
        const double v = in ? pv_cost : 1.7976931348623157e308;
        const double rm = row_min_f64(v);
        const unsigned long long b0 = __builtin_bit_cast(unsigned long long, rm);
        const double m0 = __builtin_bit_cast(double, (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(b0 >> 32), 0) << 32 |
                                                         (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b0, 0));
        const double m1 = __builtin_bit_cast(double, (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(b0 >> 32), 16) << 32 |
                                                         (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b0, 16));
        const double mn = fmin(m0, m1);
        const unsigned long long bal = __ballot(in && v == mn) & 0xFFFFFFFFull;
        m = mn;
        return __ffsll((long long)bal) - 1;
    };
#else
    auto take = [&](int bi, double m) {
        b.cost = m;
        b.single = uni(S.cd[c.par].single[bi]);
        b.dist = uni(S.cd[c.par].dist[bi]);
        b.cbp = uni(S.cd[c.par].cbp[bi]);
        b.mv[0] = uni((int)S.wc[c.tid >> 6][bi].mvx);
        b.mv[1] = uni((int)S.wc[c.tid >> 6][bi].mvy);
        return uni(S.wc[c.tid >> 6][bi].pad);
    };
    auto pick = [&](int lo, int hi, double& m) -> int { return pick_first_min(c, lo, hi, m); };
#endif
    // first step of stage st from best MV (mx, my): window re-centred, every
    // point enabled; the half stage starts at the integer MV value read as
    // half-pel (me_ds.c:360)
    auto centre_of = [](int st, int m) { return st == 0 ? m : m >> 2; };
    while (stage >= 0) {
        HL_PROF_T(tgap);
        // the chain: step 0 = the current step, then fresh stages from the
        // predicted best MV (pmv after the MVP/(0,0) step, else unchanged)
        const int pmx = stage == 3 ? pmv[0] : b.mv[0], pmy = stage == 3 ? pmv[1] : b.mv[1];
        // steps that fit the pass after the current one (each its stage's full
        // point count: 5 half-pel, 9 otherwise), in closed form: the uniform
        // loop this replaces ran as an exec-mask loop
        static_assert(kMaxSeg == 4, "three continuation steps");
        const int room0 = budget - (stage == 3 ? 2 : 9);
        const int c1 = stage - 1 == 1 ? 5 : 9, c2 = stage - 2 == 1 ? 5 : 9, c3 = stage - 3 == 1 ? 5 : 9;
        const bool ok1 = stage >= 1 && room0 >= c1, ok2 = ok1 && stage >= 2 && room0 - c1 >= c2;
        const bool ok3 = ok2 && stage >= 3 && room0 - c1 - c2 >= c3;
        const int nseg = 1 + (int)ok1 + (int)ok2 + (int)ok3;
        int lo[kMaxSeg] = {0, 0, 0, 0}, n[kMaxSeg] = {0, 0, 0, 0};
#if defined(__HIP_DEVICE_COMPILE__)
#if defined(HL_STEP_PROF)
        HL_PROF_T(tgen);
#endif
        {  // lane 16 j + i of every wave checks point i of step j; enabled points are compacted in order
            const int i = c.tid & 63, j = i >> 4, pt = min(i & 15, 8);
            const int st = stage - j;  // step j's stage (3 = MVP/(0,0))
            // (both kinds of step computed and selected: the lanes' steps differ,
            // so branches on them would run both sides under exec masks anyway)
            const uint32_t pkx = st == 2 ? pIntX : (st == 1 ? pHalfX : pQuarX);
            const uint32_t pky = st == 2 ? pIntY : (st == 1 ? pHalfY : pQuarY);
            const bool fresh = j > 0 || stage == 3;
            const int ccx = fresh ? centre_of(st, pmx) : cx, ccy = fresh ? centre_of(st, pmy) : cy;
            const int l0 = fresh ? ccx - range : left, r0 = fresh ? ccx + range : right;
            const int t0 = fresh ? ccy - range : top, b0 = fresh ? ccy + range : bottom;
            const int fl = fresh ? 0x1FF : flags;
            const int dmx = ccx + (int)((pkx >> (3 * pt)) & 7) - 2, dmy = ccy + (int)((pky >> (3 * pt)) & 7) - 2;
            const bool den = (i & 15) < (st == 1 ? 5 : 9) && ((fl >> (i & 15)) & 1) && dmx >= l0 && dmx <= r0 && dmy >= t0 && dmy <= b0;
            const bool s3 = st == 3;
            const bool en = j < nseg && (s3 ? (i & 15) < nc0 : den);
            const int mx = s3 ? ((i & 15) ? 0 : pmv[0]) : dmx, my = s3 ? ((i & 15) ? 0 : pmv[1]) : dmy;
            const int sh = st == 2 ? 2 : (st == 1 ? 1 : 0);
            const unsigned long long bal = __ballot(en);
            for (int k = 0; k < kMaxSeg; ++k) {
                lo[k] = __popcll(bal & ((1ull << (16 * k)) - 1ull));
                n[k] = __popcll(bal & (0xFFFFull << (16 * k)));
            }
            if (en) put_cand(c, g.px, g.py, g.pw, g.ph, __popcll(bal & ((1ull << i) - 1ull)), mx * (1 << sh), my * (1 << sh), i & 15, true);
        }
#if defined(HL_STEP_PROF)
        HL_PROF_ADD(c, 19, tgen);  // the pass's candidates generated and stored
#endif
#else
        {
            int tot = 0;
            for (int j = 0; j < nseg; ++j) {
                const int st = stage - j;
                lo[j] = tot;
                if (st == 3) {
                    put_cand(c, g.px, g.py, g.pw, g.ph, tot++, pmv[0], pmv[1], 0, true);
                    if (nc0 == 2) put_cand(c, g.px, g.py, g.pw, g.ph, tot++, 0, 0, 1, true);
                }
                else {
                    const uint32_t pkx = st == 2 ? pIntX : (st == 1 ? pHalfX : pQuarX);
                    const uint32_t pky = st == 2 ? pIntY : (st == 1 ? pHalfY : pQuarY);
                    const bool fresh = j > 0 || stage == 3;
                    const int ccx = fresh ? centre_of(st, pmx) : cx, ccy = fresh ? centre_of(st, pmy) : cy;
                    const int l0 = fresh ? ccx - range : left, r0 = fresh ? ccx + range : right;
                    const int t0 = fresh ? ccy - range : top, b0 = fresh ? ccy + range : bottom;
                    const int fl = fresh ? 0x1FF : flags;
                    const int sh = st == 2 ? 2 : (st == 1 ? 1 : 0);
                    for (int pt = 0; pt < (st == 1 ? 5 : 9); ++pt) {
                        if (!((fl >> pt) & 1)) continue;
                        const int mx = ccx + (int)((pkx >> (3 * pt)) & 7) - 2, my = ccy + (int)((pky >> (3 * pt)) & 7) - 2;
                        if (mx < l0 || mx > r0 || my < t0 || my > b0) continue;
                        put_cand(c, g.px, g.py, g.pw, g.ph, tot++, mx * (1 << sh), my * (1 << sh), pt, true);
                    }
                }
                n[j] = tot - lo[j];
            }
        }
#endif
        const int total = lo[nseg - 1] + n[nseg - 1];
        if (total) {
            HL_PROF_ADD(c, 16, tgap);
            eval_candidates<REC>(c, g, total, pmv);
        }
        HL_PROF_T(tsel);
#if defined(__HIP_DEVICE_COMPILE__)
        {
            const int l = c.tid & 31;
            const Shared::CandRes& R = S.cd[c.par];
            const CandSlot cs = S.wc[c.tid >> 6][l];
            pv_cost = R.cost[l];
            pv_single = R.single[l];
            pv_dist = R.dist[l];
            pv_cbp = R.cbp[l];
            pv_last = R.last[l];
            pv_mvx = cs.mvx;
            pv_mvy = cs.mvy;
            pv_pad = cs.pad;
        }
        // The sequential strict-< scans of every step of the chain
        // (me_ds.c:339-347) at once: four independent DPP minimum chains over
        // the candidate lanes of each step, then each step's smallest cost and
        // the first candidate holding it as uniform values.  Resolving the
        // chain below is then scalar work.
        double sm[kMaxSeg];
        int sb[kMaxSeg];
        {
            const int l = c.tid & 31;
            bool in[kMaxSeg];
            double v[kMaxSeg], rm[kMaxSeg];
#pragma unroll
            for (int j = 0; j < kMaxSeg; ++j) {
                in[j] = j < nseg && l >= lo[j] && l < lo[j] + n[j];
                v[j] = in[j] ? pv_cost : 1.7976931348623157e308;
                rm[j] = row_min_f64(v[j]);
            }
#pragma unroll
            for (int j = 0; j < kMaxSeg; ++j) {
                const unsigned long long b0 = __builtin_bit_cast(unsigned long long, rm[j]);
                const double m0 = __builtin_bit_cast(double, (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(b0 >> 32), 0) << 32 |
                                                                 (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b0, 0));
                const double m1 = __builtin_bit_cast(double, (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(b0 >> 32), 16) << 32 |
                                                                 (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b0, 16));
                sm[j] = fmin(m0, m1);
                sb[j] = __ffsll((long long)(__ballot(in[j] && v[j] == sm[j]) & 0xFFFFFFFFull)) - 1;
            }
        }
#if defined(HL_STEP_PROF)
        HL_PROF_ADD(c, 15, tsel);  // results loaded, the steps' minima found
        HL_PROF_T(tres);
#endif
        auto seg_pick = [&](int j, double& m) -> int {
            m = sm[j];
            return sb[j];
        };
#else
        auto seg_pick = [&](int j, double& m) -> int { return pick(lo[j], lo[j] + n[j], m); };
#endif
        // Resolve the chain (me_ds.c:280-470 applied to its steps, in closed
        // form): the MVP/(0,0) step (stage 3, always first) may take its
        // winner; from then on the best cost stays fixed until a step moves,
        // so the chain moves at its first later step with a candidate below
        // that cost, and every step before it ends its stage.  The stage's
        // window is the one re-centred when it began (kept by a move).
        int used;
        {
            int j0 = 0;
            bool cut = false;  // the (0,0) candidate won: the continuations assumed the MVP
            if (stage == 3) {  // MVP / (0,0)
                double m;
                const int bi = seg_pick(0, m);
                if (m < b.cost) take(bi, m);
                stage = 2;
                j0 = 1;
                cut = b.mv[0] != pmv[0] || b.mv[1] != pmv[1];
                cx = centre_of(2, b.mv[0]);
                cy = centre_of(2, b.mv[1]);
                flags = 0x1FF;
                left = cx - range;
                right = cx + range;
                top = cy - range;
                bottom = cy + range;
            }
            unsigned mv_mask = 0;  // steps with a candidate below the best cost
            double sj[kMaxSeg];
            int bj[kMaxSeg];
#pragma unroll
            for (int j = 0; j < kMaxSeg; ++j) {
                bj[j] = 0;
                sj[j] = 1.7976931348623157e308;
                if (j >= j0 && j < nseg && n[j]) {
                    bj[j] = seg_pick(j, sj[j]);
                    if (sj[j] < b.cost) mv_mask |= 1u << j;
                }
            }
            if (cut) used = lo[0] + n[0];
            else if (mv_mask) {
                const int jm = __builtin_ctz(mv_mask);
                if (jm > j0) {  // the steps before it ended their stages: the stage began at step jm
                    stage -= jm - j0;
                    const int wx = centre_of(stage, b.mv[0]), wy = centre_of(stage, b.mv[1]);
                    left = wx - range;
                    right = wx + range;
                    top = wy - range;
                    bottom = wy + range;
                }
                // moved: the stage goes on from the new centre (window kept, me_ds.c:309)
                const int best = take(bj[jm], sj[jm]);
                cx = b.mv[0] >> stage;
                cy = b.mv[1] >> stage;
                flags = mask_of(stage, best);  // points the move already visited
                used = lo[jm] + n[jm];
            }
            else {  // no step moved: each ended its stage
                stage -= nseg - j0;
                if (stage >= 0) {
                    cx = centre_of(stage, b.mv[0]);
                    cy = centre_of(stage, b.mv[1]);
                    flags = 0x1FF;
                    left = cx - range;
                    right = cx + range;
                    top = cy - range;
                    bottom = cy + range;
                }
                used = lo[nseg - 1] + n[nseg - 1];
            }
        }
#if defined(__HIP_DEVICE_COMPILE__)
#if defined(HL_STEP_PROF)
        HL_PROF_ADD(c, 18, tres);  // the chain resolved
#endif
        if (used) commit_candidates<REC>(c, g, used, pv_last);
#else
        if (used) commit_candidates<REC>(c, g, used);
#endif
        HL_PROF_ADD(c, 17, tsel);
    }
    // (no barrier before these stores: after the last pass, waves still read
    // only the pass's candidate results, S.cd / S.wc / S.be_tcb, which lane 0
    // does not write here; the barrier below orders them for the next search)
    if (c.tid == 0) {
        S.bcost[pi][spi] = b.cost;
        S.bdist[pi][spi] = b.dist;
        S.bsingle[pi][spi] = b.single;
        S.bcbp[pi][spi] = b.cbp;
        S.bmv[pi][spi][0] = (int16_t)b.mv[0];
        S.bmv[pi][spi][1] = (int16_t)b.mv[1];
        S.bmvp[pi][spi][0] = (int16_t)pmv[0];
        S.bmvp[pi][spi][1] = (int16_t)pmv[1];
        S.nb[0].mv[pi][spi][0] = (int16_t)b.mv[0];  // MvL0 feeds the MVP of later partitions
        S.nb[0].mv[pi][spi][1] = (int16_t)b.mv[1];
#if !defined(__HIP_DEVICE_COMPILE__)
        grid_set(S, g.px, g.py, g.pw, g.ph, b.mv[0], b.mv[1]);
#endif
    }
#if defined(__HIP_DEVICE_COMPILE__)
    // the partition's 4x4 blocks in the motion grid, lane k of wave 0 block k
    // (shifts by the partition's log2 width, no division)
    if (c.tid < g.nblk) {
        const int bx = (g.px >> 2) + (c.tid & (g.nbw - 1)), by = (g.py >> 2) + (c.tid >> g.lbw);
        S.mvs[by + 1][bx + 1] = 2;
        S.mvg[by + 1][bx + 1] = (b.mv[0] & 0xFFFF) | (int)((uint32_t)b.mv[1] << 16);
    }
#endif
    HL_SYNC();
    HL_PROF_ADD(c, 3, tsp);
    return probably;
}
// --------------------------------------------------------------------------
// Intra prediction (8.3, pred_intra.c:326-1220)
// --------------------------------------------------------------------------
// luma sample at (x, y) relative to the MB origin as intra prediction sees it
HD int intra_sample(const Shared& S, int x, int y)
{
    if (y < 0) return S.top[x + 1];
    if (x < 0) return S.left[y];
    return S.rec[y * 16 + x];
}

HD void i4_neighbours(const Shared& S, int blk, int p[13])
{
    const int xO = blk_x(blk), yO = blk_y(blk);
    for (int i = 0; i < 13; ++i) {
        const int X = i < 5 ? -1 : i - 5, Y = i < 5 ? i - 1 : -1;
        const int x = xO + X, y = yO + Y;
        int v;
        if (x > 15 && y >= 0) v = kNA;
        else if (X > 3 && (blk == 3 || blk == 11)) v = kNA;
        else if (x < 0 && y >= 0) v = S.left[y];
        else if (y < 0) v = S.top[x + 1];
        else v = S.rec[y * 16 + x];
        p[i] = v;
    }
    if (p[9] == kNA && p[8] != kNA) p[9] = p[10] = p[11] = p[12] = p[8];
}

#define HL_P4(x, y) p[(x) == -1 ? (y) + 1 : (x) + 5]
template <typename PT>
HD bool i4_avail(int mode, const PT& p)
{
    if ((mode == 0 || mode == 3 || mode == 7) && p[5] == kNA) return false;
    if ((mode == 1 || mode == 8) && p[1] == kNA) return false;
    if ((mode == 4 || mode == 5 || mode == 6) && p[0] == kNA) return false;
    return true;
}
// Intra4x4 prediction of sample (x, y), modes 0-8 (8.3.1.2); p is the
// 13-sample neighbour array (p[0] = corner, p[1..4] left, p[5..12] top).
template <typename PT>
constexpr HD int i4_pred_px(int mode, const PT& p, int x, int y)
{
    {
        {
            int v;
            switch (mode) {
            case 0: v = p[5 + x]; break;
            case 1: v = p[1 + y]; break;
            case 2: {
                const bool xa = p[5] != kNA && p[6] != kNA && p[7] != kNA && p[8] != kNA;
                const bool ya = p[1] != kNA && p[2] != kNA && p[3] != kNA && p[4] != kNA;
                if (xa && ya) v = (p[5] + p[6] + p[7] + p[8] + p[1] + p[2] + p[3] + p[4] + 4) >> 3;
                else if (ya) v = (p[1] + p[2] + p[3] + p[4] + 2) >> 2;
                else if (xa) v = (p[5] + p[6] + p[7] + p[8] + 2) >> 2;
                else v = 128;
                break;
            }
            case 3:
                v = (x == 3 && y == 3) ? (p[11] + 3 * p[12] + 2) >> 2
                                       : (HL_P4(x + y, -1) + 2 * HL_P4(x + y + 1, -1) + HL_P4(x + y + 2, -1) + 2) >> 2;
                break;
            case 4:
                if (x > y) v = (HL_P4(x - y - 2, -1) + 2 * HL_P4(x - y - 1, -1) + HL_P4(x - y, -1) + 2) >> 2;
                else if (x < y) v = (HL_P4(-1, y - x - 2) + 2 * HL_P4(-1, y - x - 1) + HL_P4(-1, y - x) + 2) >> 2;
                else v = (p[5] + 2 * p[0] + p[1] + 2) >> 2;
                break;
            case 5: {
                const int z = 2 * x - y;
                if (z >= 0 && !(z & 1)) v = (HL_P4(x - (y >> 1) - 1, -1) + HL_P4(x - (y >> 1), -1) + 1) >> 1;
                else if (z >= 0) v = (HL_P4(x - (y >> 1) - 2, -1) + 2 * HL_P4(x - (y >> 1) - 1, -1) + HL_P4(x - (y >> 1), -1) + 2) >> 2;
                else if (z == -1) v = (p[1] + 2 * p[0] + p[5] + 2) >> 2;
                else v = (HL_P4(-1, y - 1) + 2 * HL_P4(-1, y - 2) + HL_P4(-1, y - 3) + 2) >> 2;
                break;
            }
            case 6: {
                const int z = 2 * y - x;
                if (z >= 0 && !(z & 1)) v = (HL_P4(-1, y - (x >> 1) - 1) + HL_P4(-1, y - (x >> 1)) + 1) >> 1;
                else if (z >= 0) v = (HL_P4(-1, y - (x >> 1) - 2) + 2 * HL_P4(-1, y - (x >> 1) - 1) + HL_P4(-1, y - (x >> 1)) + 2) >> 2;
                else if (z == -1) v = (p[1] + 2 * p[0] + p[5] + 2) >> 2;
                else v = (HL_P4(x - 1, -1) + 2 * HL_P4(x - 2, -1) + HL_P4(x - 3, -1) + 2) >> 2;
                break;
            }
            case 7:
                if (y == 0) v = (HL_P4(x, -1) + HL_P4(x + 1, -1) + 1) >> 1;
                else if (y == 2) v = (HL_P4(x + 1, -1) + HL_P4(x + 2, -1) + 1) >> 1;
                else if (y == 1) v = (HL_P4(x, -1) + 2 * HL_P4(x + 1, -1) + HL_P4(x + 2, -1) + 2) >> 2;
                else v = (HL_P4(x + 1, -1) + 2 * HL_P4(x + 2, -1) + HL_P4(x + 3, -1) + 2) >> 2;
                break;
            default: {
                const int z = x + 2 * y;
                if (z == 0 || z == 2 || z == 4) v = (HL_P4(-1, y + (x >> 1)) + HL_P4(-1, y + (x >> 1) + 1) + 1) >> 1;
                else if (z == 1 || z == 3) v = (HL_P4(-1, y + (x >> 1)) + 2 * HL_P4(-1, y + (x >> 1) + 1) + HL_P4(-1, y + (x >> 1) + 2) + 2) >> 2;
                else if (z == 5) v = (p[3] + 3 * p[4] + 2) >> 2;
                else v = p[4];
                break;
            }
            }
            return v;
        }
    }
}
// Every Intra4x4 mode except DC predicts a sample as (w0 p[i0] + w1 p[i1] +
// w2 p[i2] + 2) >> 2 over the 13 neighbours (two-tap averages are weights
// 2, 2; copies weight 4).  The table holds (i0, i1, i2, w0, w1, w2) per
// (mode, sample), derived at compile time by probing i4_pred_px with unit
// neighbours; DC reads p[13] = its value.  The device evaluates all nine
// modes branch-free from it (one row per mode, no per-mode code path);
// tests/test_emu_golden.py::test_i4_prediction_table checks it against
// i4_pred_px on random neighbourhoods.
struct I4Tab {
    uint32_t e[9][16];
};
constexpr I4Tab make_i4_tab()
{
    I4Tab t{};
    for (int m = 0; m < 9; ++m)
        for (int pos = 0; pos < 16; ++pos) {
            uint32_t e = 0;
            if (m == 2) e = 13u | (4u << 12);
            else {
                int n = 0;
                for (int k = 0; k < 13; ++k) {
                    int pv[13] = {};
                    pv[k] = 256;
                    const int w = i4_pred_px(m, pv, pos & 3, pos >> 2) / 64;
                    if (w) {
                        e |= (uint32_t)k << (4 * n) | (uint32_t)w << (12 + 3 * n);
                        ++n;
                    }
                }
            }
            t.e[m][pos] = e;
        }
    return t;
}
constexpr I4Tab kI4Tab = make_i4_tab();
HD int i4_tab_pred(uint32_t e, int a, int b, int c)  // a, b, c = p[i0], p[i1], p[i2]
{
    return ((int)((e >> 12) & 7) * a + (int)((e >> 15) & 7) * b + (int)((e >> 18) & 7) * c + 2) >> 2;
}
// DC prediction value of a 13-sample neighbourhood (mode 2 of i4_pred_px)
HD int i4_dc(const int p[13]) { return i4_pred_px(2, p, 0, 0); }

HD void i4_pred(int mode, const int p[13], int* pr)
{
    for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) pr[y * 4 + x] = i4_pred_px(mode, p, x, y);
}

// Intra16x16 prediction of sample (x, y) (pred_intra.c:855-1041); p33 layout
// is S.top / S.left.
HD int i16_pred(const Shared& S, int mode, int x, int y, int dcv, int pa, int pb, int pc)
{
    if (mode == 0) return S.top[1 + x];
    if (mode == 1) return S.left[y];
    if (mode == 2) return dcv;
    return clip255((pa + pb * (x - 7) + pc * (y - 7) + 16) >> 5);
    (void)pc;
}
HD void i16_params(const Shared& S, int mode, int& dcv, int& pa, int& pb, int& pc)
{
    dcv = pa = pb = pc = 0;
    if (mode == 2) {
        bool xa = true, ya = true;
        int xs = 0, ys = 0;
        // no early exit: a sum is only used when its side had no kNA, so the
        // loads are independent and issue together
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            xa = xa && S.top[1 + k] != kNA;
            ya = ya && S.left[k] != kNA;
            xs += S.top[1 + k];
            ys += S.left[k];
        }
        if (xa && ya) dcv = (xs + ys + 16) >> 5;
        else if (ya) dcv = (ys + 8) >> 4;
        else if (xa) dcv = (xs + 8) >> 4;
        else dcv = 128;
    }
    else if (mode == 3) {
        int H = 0, V = 0;
        for (int i = 0; i < 7; ++i) {
            H += (i + 1) * (S.top[1 + 8 + i] - S.top[1 + 6 - i]);
            V += (i + 1) * (S.left[8 + i] - S.left[6 - i]);
        }
        H += 8 * (S.top[16] - S.top[0]);
        V += 8 * (S.left[15] - S.top[0]);
        pa = (S.left[15] + S.top[16]) << 4;
        pb = (5 * H + 32) >> 6;
        pc = (5 * V + 32) >> 6;
    }
}

// --------------------------------------------------------------------------
// Chroma reconstruction (rdo.c:2502-2701 + transf.c:161-294)
// --------------------------------------------------------------------------
// S.predc holds the chroma prediction; writes recon to the picture.
HD void reconstruct_chroma(Ctx& c, bool intra_flag)
{
    HL_FRESH_TID_K(c, 1);
    const FrameArgs& F = c.F;
    Shared& S = c.S;
#if defined(HL_PROF_MISC)
    HL_PROF_T(trc);
#endif
#if defined(__HIP_DEVICE_COMPILE__)
    // one 4-lane quad per chroma 4x4 block (lanes 0-31: Cb blocks 0-3, Cr
    // blocks 0-3), lane r = block row r (hl_quad.h) at the chroma QP
    const LaneQ Qc = make_laneq(c.tid, F.qpc);
    const int qbc = 15 + F.qpc / 6, fqc = (1 << qbc) / 3;  // intra rounding for every MB (rdo.c:2588,2618)
    if (c.tid < 32) {
        const int t = c.tid >> 2, r = c.tid & 3, comp = t >> 2, b = t & 3, xO = (b & 1) * 4, yO = (b >> 1) * 4;
        const uint32_t sv = *reinterpret_cast<const uint32_t*>(&S.srcc[comp][(yO + r) * 8 + xO]);
        const int* pc = &S.predc[comp][(yO + r) * 8 + xO];
        int x[4];
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) x[cc] = (int)((sv >> (8 * cc)) & 255) - pc[cc];
        int dc = 0, cacb = 0, cdcb = 0, tc = 0, sctr = -1;
        if (quad_or(x[0] | x[1] | x[2] | x[3]) != 0) {  // (quad-uniform)
            int y[4], q[4];
            quad_fwd(Qc, x, y);
            int mb = 0;
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                q[cc] = quad_q1(y[cc], (cc & 1) ? Qc.mfO : Qc.mfE, qbc, fqc);
                const int zz = (int)((Qc.zz >> (4 * cc)) & 15);
                if (zz) {  // ChromaACLevel: scan positions 1-15 at list index 0-14
                    S.cac[comp][b][zz - 1] = (int16_t)q[cc];
                    mb |= q[cc] ? (1 << (zz - 1)) | ((q[cc] == 1 || q[cc] == -1) << (zz + 15)) : 0;
                }
            }
            // list index 15 is read stale, as the CAVLC statistics see it
            const int st = S.cac[comp][b][15];
            const uint32_t masks = (uint32_t)quad_or(mb) | (st ? (1u << 15) | ((uint32_t)(st == 1 || st == -1) << 31) : 0u);
            const uint32_t nz = masks & 0xFFFFu, ones = masks >> 16;
            dc = dpp_x<0x00>(y[0]);  // coefficient (0, 0): lane 0 of the quad (quad_perm 0,0,0,0)
            cacb = nz != 0;
            cdcb = dc != 0;
            if (cacb) {  // cavlc_stat's TotalCoeff and single-coefficient counter
                const int hi = 31 - __clz(nz);
                tc = __popc(nz);
                sctr = (tc == 1 && ones == nz) ? (hi == 0 ? 3 : (hi < 3 ? 2 : (hi < 6 ? 1 : 0))) : 9;
            }
        }
        if (r == 0) {
            S.cres_dc[comp][b] = dc;
            S.cres_cac[comp][b] = cacb;
            S.cres_cdc[comp][b] = cdcb;
            S.cres_tc[comp][b] = tc;
            S.cres_sctr[comp][b] = sctr;
        }
    }
#else
    for (int t = c.tid; t < 8; t += c.nthr) {
        const int comp = t >> 2, b = t & 3, xO = (b & 1) * 4, yO = (b >> 1) * 4;
        int res[16];
        bool zero = true;
        for (int i = 0; i < 16; ++i) {
            const int o = (yO + (i >> 2)) * 8 + xO + (i & 3);
            res[i] = (int)S.srcc[comp][o] - S.predc[comp][o];
            zero = zero && res[i] == 0;
        }
        int dc = 0, cacb = 0, cdcb = 0;
        CavlcStat st = {0, 0, 0, -1};
        if (!zero) {
            int w[16], q[16];
            fwd4x4(res, w);
            quant4x4(F.qpc, true, w, q);  // intra rounding for every MB (rdo.c:2588,2618)
            bool az = true;
            int lv[16];  // the block's ChromaACLevel as the CAVLC statistics read it (entry 15 stays stale)
            for (int i = 1; i < 16; ++i) {
                lv[i - 1] = (int16_t)q[kZigzag[i]];
                S.cac[comp][b][i - 1] = (int16_t)lv[i - 1];
                az = az && lv[i - 1] == 0;
            }
            lv[15] = S.cac[comp][b][15];
            az = az && lv[15] == 0;
            dc = w[0];
            cacb = !az;
            cdcb = w[0] != 0;
            if (cacb) st = cavlc_stat(lv, 16, 15, false);
        }
        S.cres_dc[comp][b] = dc;
        S.cres_cac[comp][b] = cacb;
        S.cres_cdc[comp][b] = cdcb;
        S.cres_tc[comp][b] = st.tc;
        S.cres_sctr[comp][b] = st.sctr;
    }
#endif
    HL_SYNC();
    // sequential single-coefficient gating (uniform)
    int single[2] = {0, 0}, tcs[2] = {0, 0}, cac[2] = {0, 0}, cdc[2] = {0, 0};
#if defined(__HIP_DEVICE_COMPILE__)
    // as selects (uniform values in VGPRs: each if would be an exec-mask branch)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int comp = 0; comp < 2; ++comp) {
            const int ca = S.cres_cac[comp][b], sc = S.cres_sctr[comp][b];
            cac[comp] |= ca << b;
            cdc[comp] |= S.cres_cdc[comp][b] << b;
            const bool w = single[comp] < 7 && ca;
            single[comp] += w ? sc : 0;
            tcs[comp] += w ? S.cres_tc[comp][b] : 0;
            c.chain = w ? sc : c.chain;  // chain_write
            c.fresh = w ? 1 : c.fresh;
            c.spec = w ? 0 : c.spec;
        }
#else
    for (int b = 0; b < 4; ++b)
        for (int comp = 0; comp < 2; ++comp) {
            cac[comp] |= S.cres_cac[comp][b] << b;
            cdc[comp] |= S.cres_cdc[comp][b] << b;
            if (single[comp] < 7 && S.cres_cac[comp][b]) {
                single[comp] += S.cres_sctr[comp][b];
                tcs[comp] += S.cres_tc[comp][b];
                chain_write(c, S.cres_sctr[comp][b]);
            }
        }
#endif
    // TotalCoeffs are written only for blocks passed to write_block (lane 0)
    if (c.tid == 0) {
        int sg[2] = {0, 0};
        for (int b = 0; b < 4; ++b)
            for (int comp = 0; comp < 2; ++comp)
                if (sg[comp] < 7 && S.cres_cac[comp][b]) {
                    sg[comp] += S.cres_sctr[comp][b];
                    S.tcc[comp][b] = (int8_t)S.cres_tc[comp][b];
                }
    }
#pragma unroll
    for (int comp = 0; comp < 2; ++comp) cac[comp] = (single[comp] < 7 && tcs[comp] == 1) ? 0 : cac[comp];
    int dcl[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
    for (int comp = 0; comp < 2; ++comp)
        if (cdc[comp]) {
            const int* D = S.cres_dc[comp];
            const int t00 = D[0] + D[2], t01 = D[1] + D[3], t10 = D[0] - D[2], t11 = D[1] - D[3];
            dcl[comp][0] = quant_dc(F.qpc, intra_flag, t00 + t01);
            dcl[comp][1] = quant_dc(F.qpc, intra_flag, t00 - t01);
            dcl[comp][2] = quant_dc(F.qpc, intra_flag, t10 + t11);
            dcl[comp][3] = quant_dc(F.qpc, intra_flag, t10 - t11);
            cdc[comp] = (dcl[comp][0] ? 1 : 0) | (dcl[comp][1] ? 2 : 0) | (dcl[comp][2] ? 4 : 0) | (dcl[comp][3] ? 8 : 0);
        }
    if (c.tid == 0) {
        for (int comp = 0; comp < 2; ++comp) {
            S.cbp_cac[comp] = cac[comp];
            S.cbp_cdc[comp] = cdc[comp];
            for (int i = 0; i < 4; ++i) S.cdc_level[comp][i] = dcl[comp][i];
        }
    }
    // decode (transf.c:161-294)
#if defined(__HIP_DEVICE_COMPILE__)
    if (c.tid < 32) {  // the quads of the first pass: lane r writes row r of its block
        const int t = c.tid >> 2, r = c.tid & 3, comp = t >> 2, b = t & 3, xO = (b & 1) * 4, yO = (b >> 1) * 4;
        const int* pc = &S.predc[comp][(yO + r) * 8 + xO];
        int rr[4] = {0, 0, 0, 0};
        if (cdc[comp] || cac[comp]) {
            int dcc = 0;
            if (cdc[comp]) {
                const int qP = F.qpc, scale = level_scale(qP % 6, 0, 0);
                const int* L = dcl[comp];
                const int f00 = (L[0] + L[2]) + (L[1] + L[3]), f01 = (L[0] + L[2]) - (L[1] + L[3]);
                const int f10 = (L[0] - L[2]) + (L[1] - L[3]), f11 = (L[0] - L[2]) - (L[1] - L[3]);
                const int f = b == 0 ? f00 : (b == 1 ? f01 : (b == 2 ? f10 : f11));
                dcc = ((f * scale) * (1 << (qP / 6))) >> 5;
            }
            if (dcc || (cac[comp] & (1 << b))) {  // (quad-uniform)
                int q[4];
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) {
                    const int zz = (int)((Qc.zz >> (4 * cc)) & 15);
                    q[cc] = zz ? S.cac[comp][b][zz - 1] : 0;
                }
                quad_idct(Qc, q, F.qpc, rr, true, dcc);
            }
        }
        uint32_t rec = 0;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) rec |= (uint32_t)clip255(pc[cc] + rr[cc]) << (8 * cc);
        *reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(gmem(F.cur[1 + comp]) + ((c.yL >> 1) + yO + r) * F.Wc + (c.xL >> 1) + xO) = rec;
    }
#else
    for (int t = c.tid; t < 8; t += c.nthr) {
        const int comp = t >> 2, b = t & 3, xO = (b & 1) * 4, yO = (b >> 1) * 4;
        int r[16];
        bool have = false;
        if (cdc[comp] || cac[comp]) {
            int dcc = 0;
            if (cdc[comp]) {
                const int qP = F.qpc, scale = level_scale(qP % 6, 0, 0);
                const int* L = dcl[comp];
                const int f00 = (L[0] + L[2]) + (L[1] + L[3]), f01 = (L[0] + L[2]) - (L[1] + L[3]);
                const int f10 = (L[0] - L[2]) + (L[1] - L[3]), f11 = (L[0] - L[2]) - (L[1] - L[3]);
                const int f = b == 0 ? f00 : (b == 1 ? f01 : (b == 2 ? f10 : f11));
                dcc = ((f * scale) * (1 << (qP / 6))) >> 5;
            }
            if (dcc || (cac[comp] & (1 << b))) {
                int list[16], m[16];
                list[0] = dcc;
                for (int i = 1; i < 16; ++i) list[i] = S.cac[comp][b][i - 1];
                unscan(list, m);
                dequant_idct(F.qpc, m, true, r);
                have = true;
            }
        }
        for (int i = 0; i < 16; ++i) {
            const int o = (yO + (i >> 2)) * 8 + xO + (i & 3);
            const int v = have ? clip255(S.predc[comp][o] + r[i]) : S.predc[comp][o];
            gmem(F.cur[1 + comp])[((c.yL >> 1) + yO + (i >> 2)) * F.Wc + (c.xL >> 1) + xO + (i & 3)] = (uint8_t)v;
        }
    }
#endif
    HL_SYNC();
#if defined(HL_PROF_MISC)
    HL_PROF_ADD(c, 14, trc);
#endif
}

HD void guess_cbp(Shared& S)  // rdo.c:2703-2782 (lane 0)
{
    if (S.pm0 == PM_I16) S.cbp_l = S.cbp_l4x4 ? 15 : 0;
    else {
        S.cbp_l = 0;
        for (int i8 = 0; i8 < 4; ++i8)
            if (S.cbp_l4x4 & (0xF << (i8 * 4))) S.cbp_l |= 1 << i8;
    }
    if ((S.cbp_cdc[0] || S.cbp_cdc[1]) && (!S.cbp_cac[0] && !S.cbp_cac[1])) S.cbp_c = 1;
    else if (S.cbp_cac[0] || S.cbp_cac[1]) S.cbp_c = 2;
    else S.cbp_c = 0;
    S.cbp = (S.cbp_c << 4) | S.cbp_l;
    if (S.cbp > 47) {
        S.cbp -= 16;
        S.cbp_c = S.cbp >> 4;
    }
}

// intra chroma prediction into S.predc (pred_intra.c:1043-1220)
HD void intra_chroma_pred(Ctx& c, int mode)
{
    Shared& S = c.S;
    for (int t = c.tid; t < 128; t += c.nthr) {
        const int comp = t >> 6, i = t & 63, x = i & 7, y = i >> 3;
        const int16_t* top = &S.ctop[comp][1];
        const int16_t* left = S.cleft[comp];
        int v;
        if (mode == 0) {
            // availability flags are sticky across the four blocks (pred_intra.c:1046)
            bool xa = true, ya = true;
            int t4 = 128;
            for (int b = 0; b <= ((y >> 2) << 1 | (x >> 2)); ++b) {
                const int xO = (b & 1) * 4, yO = (b >> 1) * 4;
                int xs = 0, ys = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    xa = xa && top[xO + k] != kNA;
                    ya = ya && left[yO + k] != kNA;
                    xs += top[xO + k];
                    ys += left[yO + k];
                }
                t4 = 128;
                if ((xO == 0 && yO == 0) || (xO > 0 && yO > 0)) {
                    if (xa && ya) t4 = (xs + ys + 4) >> 3;
                    else if (!xa && ya) t4 = (ys + 2) >> 2;
                    else if (!ya && xa) t4 = (xs + 2) >> 2;
                }
                else if (xO > 0 && yO == 0) {
                    if (xa) t4 = (xs + 2) >> 2;
                    else if (ya) t4 = (ys + 2) >> 2;
                }
                else {
                    if (ya) t4 = (ys + 2) >> 2;
                    else if (xa) t4 = (xs + 2) >> 2;
                }
            }
            v = t4;
        }
        else if (mode == 1) v = left[y];
        else if (mode == 2) v = top[x];
        else {
            int H = 0, V = 0;
            for (int k = 0; k < 3; ++k) {
                H += (k + 1) * (top[4 + k] - top[2 - k]);
                V += (k + 1) * (left[4 + k] - left[2 - k]);
            }
            H += 4 * (top[7] - top[-1]);
            V += 4 * (left[7] - top[-1]);
            const int a = (left[7] + top[7]) << 4, bb = (34 * H + 32) >> 6, cc = (34 * V + 32) >> 6;
            v = clip255((a + bb * (x - 3) + cc * (y - 3) + 16) >> 5);
        }
        S.predc[comp][i] = v;
    }
    HL_SYNC();
}

// --------------------------------------------------------------------------
// Intra 16x16 RDO (rdo.c:1526-1809)
// --------------------------------------------------------------------------
// Pipelined runs: the exact rdo.Single_ctr for a stale read (residual.c:881-897,
// DESIGN.md §5) while this MB's value is still a row-start speculation.  It is
// the value left by the last MB that wrote the counter: the end of the nearest
// earlier row with a fresh write, walking back through this picture, then the
// earlier pictures of the run, then the value entering the run.  Those rows
// never wait on this task (they precede it in the wavefront and in picture
// order), so the walk cannot deadlock; every wait is bounded.  Rare: about one
// per 1088p I picture, none in the P pictures of the test content.
HD void resolve_chain(Ctx& c)
{
    HL_FRESH_TID_K(c, 2);
#if defined(__HIP_DEVICE_COMPILE__)
    const FrameArgs& F = c.F;
    Shared& S = c.S;
    const int nmb = F.mbw * F.mbh, lane = c.tid & 63;
    if (c.tid < 64) {
        if (c.tid == 0) atomicAdd(F.perr + 1, 1);  // walk counter (diagnostics, hl_amd_last_chain_walks)
        int val = F.carry_in, pos = F.run_pos, y = c.mby - 1;
        for (;;) {
            if (y < 0) {
                if (pos == 0) break;
                --pos;
                y = F.mbh - 1;
            }
            const int32_t* done = F.run_done + (size_t)pos * nmb + (size_t)y * F.mbw;
            const MbChain* row = F.run_chain + (size_t)pos * nmb + (size_t)y * F.mbw;
            if (lane == 0) spin_ge(done + F.mbw - 1, 1, F.perr);  // the row's last MB: the whole row is final
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, HL_ACQ_SCOPE);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bool fr = false;
            for (int x = lane; x < F.mbw; x += 64) fr = fr || ld_relaxed(&row[x].fresh) != 0;
            if (__ballot(fr)) {
                val = ld_relaxed(&row[F.mbw - 1].s_out);
                break;
            }
            --y;
        }
        if (c.tid == 0) S.chain_x = val;
    }
    HL_SYNC();
    c.chain = uni(S.chain_x);
    c.spec = 0;
#else
    (void)c;
#endif
}

// Intra16x16 modes the neighbourhood allows (rdo.c:1541-1560), uniform
HD bool i16_mode_avail(const Shared& S, int mode)
{
    if (mode == 0) return uni((int)S.top[1]) != kNA;
    if (mode == 1) return uni((int)S.left[0]) != kNA;
    if (mode == 3) return uni((int)S.top[0]) != kNA;
    return true;
}
HD int nc_class(int nC) { return nC < 2 ? 0 : (nC < 4 ? 1 : (nC < 8 ? 2 : 3)); }  // the coeff_token table nC selects

// Intra16x16, the part of every mode that depends only on the MB's source and
// its final neighbours (rdo.c:1526-1700): prediction, transform,
// quantisation and CAVLC statistics of each 4x4 block and of the DC block,
// the reconstruction with the residual and the distortions with and without
// it.  Into S.ih (blk, dcs, dist) and S.ih_rec / ih_pred / ih_ac / ih_dcl.
HD void i16_heavy(Ctx& c)
{
    HL_FRESH_TID_K(c, 3);
    const FrameArgs& F = c.F;
    Shared& S = c.S;
#if defined(__HIP_DEVICE_COMPILE__)
    // Wave m evaluates mode m on its own (waves 0-3): one 4-lane quad per 4x4
    // block, lane r = block row r (hl_quad.h); the DC block on lanes 0-15 of
    // the wave (16-lane Hadamard, hl_coop.h); the mode's distortions summed
    // over its quads.  Only the waves' LDS writes need ordering inside the
    // wave, so the four modes run without a workgroup barrier.
    static_assert(kMbThreads >= 256, "one wave per Intra16x16 mode");
    const int mode = c.tid >> 6, lane = c.tid & 63, blk = lane >> 2, r = lane & 3;
    if (mode < 4 && i16_mode_avail(S, mode)) {  // (wave-uniform)
        const int qp = uni(F.qp), qbits = 15 + qp / 6, fq = (1 << qbits) / 3;
        LaneQ Q = c.Q;
        if (HL_FRESH_ZZ & 2) Q.zz = laneq_zz_fresh(Q.r);
        int dcv, pa, pb, pc;
        i16_params(S, mode, dcv, pa, pb, pc);
        dcv = uni(dcv);
        pa = uni(pa);
        pb = uni(pb);
        pc = uni(pc);
        const int xO = blk_x(blk), y = blk_y(blk) + r;
        const uint32_t sv = *reinterpret_cast<const uint32_t*>(&S.src[y * 16 + xO]);
        int x[4], w[4], q[4];
        uint32_t pr = 0;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
            const int p = i16_pred(S, mode, xO + cc, y, dcv, pa, pb, pc);
            pr |= (uint32_t)p << (8 * cc);
            x[cc] = (int)((sv >> (8 * cc)) & 255) - p;
        }
        *reinterpret_cast<uint32_t*>(&S.ih_pred[mode][y * 16 + xO]) = pr;
        // blocks: transform, quant, AC statistics
        quad_fwd(Q, x, w);
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
            q[cc] = quad_q1(w[cc], (cc & 1) ? Q.mfO : Q.mfE, qbits, fq);
            const int zz = (int)((Q.zz >> (4 * cc)) & 15);
            S.ih_ac[mode][blk][zz == 0 ? 15 : zz - 1] = (int16_t)(zz == 0 ? 0 : q[cc]);
        }
        const bool qz = quad_or(q[0] | q[1] | q[2] | q[3]) == 0;
        const CoopStat st = quad_cavlc(S.ct, Q, q, 1, S.lvq[c.tid >> 2]);
        if (r == 0) {
            S.i16_dcc[mode * 16 + blk] = w[0];  // the block's DC coefficient (lane 0 holds coefficient row 0)
            S.ih.blk[mode][blk] = (qz ? 0 : 1) | (st.tc << 1) | (st.t1 << 6) | ((st.sctr + 1) << 8) | (st.rest << 16);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane < 16) {  // the DC block: Hadamard, quant, CAVLC, scaling
            const int hh = coop_lin(c.k().had, S.i16_dcc[mode * 16 + kDcPos[c.k().p]]) >> 1;
            const int qd = quant_dc(qp, true, hh);
            const CoopStat sd = coop_cavlc(S.ct, qd, c.k().s, S.lvs[c.tid >> 4]);
            S.ih_dcl[mode][c.k().s] = (int16_t)qd;
            const int f = coop_lin(c.k().had, qd);
            const int scale = level_scale(qp % 6, 0, 0), q6 = qp / 6;
            S.dcY[mode * 16 + c.k().p] = qp >= 36 ? (f * scale) * (1 << (q6 - 6)) : (f * scale + (1 << (5 - q6))) >> (6 - q6);
            if (lane == 0) {  // block 0's nC neighbours lie outside the MB: the DC rate is fixed
                const int nC = nc_luma_of(S, 0, [&](int ni) -> int { return S.tc[ni]; });
                S.ih.dcs[mode][0] = sd.rest + coop_token_len(S.ct, nC, sd.tc, sd.t1);
                S.ih.dcs[mode][1] = sd.tc;
                S.ih.dcs[mode][2] = sd.sctr;
                S.ih.dcs[mode][3] = 0;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // reconstruction with the residual (the scaled DC kept); both distortions
        int rr[4];
        quad_idct(Q, q, qp, rr, true, S.dcY[mode * 16 + kDcPos[blk]]);
        uint32_t rec = 0;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) rec |= (uint32_t)clip255((int)((pr >> (8 * cc)) & 255) + rr[cc]) << (8 * cc);
        *reinterpret_cast<uint32_t*>(&S.ih_rec[mode][y * 16 + xO]) = rec;
        // per-row sums of |residual| over the wave, then its four 16-lane rows
        const int df = row_sum((int)__builtin_amdgcn_sad_u8(sv, rec, 0u)), dz = row_sum((int)__builtin_amdgcn_sad_u8(sv, pr, 0u));
        const int tf = __builtin_amdgcn_readlane(df, 0) + __builtin_amdgcn_readlane(df, 16) + __builtin_amdgcn_readlane(df, 32) + __builtin_amdgcn_readlane(df, 48);
        const int tz = __builtin_amdgcn_readlane(dz, 0) + __builtin_amdgcn_readlane(dz, 16) + __builtin_amdgcn_readlane(dz, 32) + __builtin_amdgcn_readlane(dz, 48);
        if (lane == 0) {
            S.ih.dist[mode][0] = tf;
            S.ih.dist[mode][1] = tz;
        }
    }
    HL_SYNC();
#else
    for (int mode = 0; mode < 4; ++mode) {
        if (!i16_mode_avail(S, mode)) continue;
        int dcv, pa, pb, pc;
        i16_params(S, mode, dcv, pa, pb, pc);
        for (int t = 0; t < 256; ++t) S.ih_pred[mode][t] = (uint8_t)i16_pred(S, mode, t & 15, t >> 4, dcv, pa, pb, pc);
        int dcc[16];
        for (int t = 0; t < 16; ++t) {  // blocks: transform, quant, AC statistics
            const int xO = blk_x(t), yO = blk_y(t);
            int res[16], w[16], q[16];
            for (int i = 0; i < 16; ++i) {
                const int o = (yO + (i >> 2)) * 16 + xO + (i & 3);
                res[i] = (int)S.src[o] - S.ih_pred[mode][o];
            }
            fwd4x4(res, w);
            quant4x4(F.qp, true, w, q);
            bool qz = true;
            for (int i = 0; i < 16; ++i) qz = qz && q[i] == 0;
            for (int i = 1; i < 16; ++i) S.ih_ac[mode][t][i - 1] = (int16_t)q[kZigzag[i]];
            S.ih_ac[mode][t][15] = 0;
            dcc[t] = w[0];
            CavlcStat st = {0, 0, 0, -1};
            if (!qz) st = cavlc_stat(S.ih_ac[mode][t], 16, 15, false);
            S.ih.blk[mode][t] = (qz ? 0 : 1) | (st.tc << 1) | (st.t1 << 6) | ((st.sctr + 1) << 8) | (st.rest << 16);
        }
        // the DC block: Hadamard, quant, CAVLC (block 0's nC neighbours lie outside the MB)
        int h[16], hh[16], qd[16], dcl[16];
        for (int b = 0; b < 16; ++b) h[kDcPos[b]] = dcc[b];
        hadamard4x4_fwd(h, hh);
        for (int i = 0; i < 16; ++i) qd[i] = quant_dc(F.qp, true, hh[i]);
        for (int i = 0; i < 16; ++i) dcl[i] = qd[kZigzag[i]];
        const CavlcStat st = cavlc_stat(dcl, 16, 15, false);
        const int nC = nc_luma_of(S, 0, [&](int ni) -> int { return S.tc[ni]; });
        S.ih.dcs[mode][0] = st.rest + token_len(nC, st.tc, st.t1);
        S.ih.dcs[mode][1] = st.tc;
        S.ih.dcs[mode][2] = st.sctr;
        S.ih.dcs[mode][3] = 0;
        for (int i = 0; i < 16; ++i) S.ih_dcl[mode][i] = (int16_t)dcl[i];
        // scale DC (8.5.10), then the inverse of every block with it
        int cm[16], dcY[16];
        unscan(dcl, cm);
        {
            int d[16], f[16];
            for (int j = 0; j < 4; ++j) {
                d[0 * 4 + j] = cm[0 * 4 + j] + cm[1 * 4 + j] + cm[2 * 4 + j] + cm[3 * 4 + j];
                d[1 * 4 + j] = cm[0 * 4 + j] + cm[1 * 4 + j] - cm[2 * 4 + j] - cm[3 * 4 + j];
                d[2 * 4 + j] = cm[0 * 4 + j] - cm[1 * 4 + j] - cm[2 * 4 + j] + cm[3 * 4 + j];
                d[3 * 4 + j] = cm[0 * 4 + j] - cm[1 * 4 + j] + cm[2 * 4 + j] - cm[3 * 4 + j];
            }
            for (int i = 0; i < 4; ++i) {
                f[i * 4 + 0] = d[i * 4 + 0] + d[i * 4 + 1] + d[i * 4 + 2] + d[i * 4 + 3];
                f[i * 4 + 1] = d[i * 4 + 0] + d[i * 4 + 1] - d[i * 4 + 2] - d[i * 4 + 3];
                f[i * 4 + 2] = d[i * 4 + 0] - d[i * 4 + 1] - d[i * 4 + 2] + d[i * 4 + 3];
                f[i * 4 + 3] = d[i * 4 + 0] - d[i * 4 + 1] + d[i * 4 + 2] - d[i * 4 + 3];
            }
            const int scale = level_scale(F.qp % 6, 0, 0), q6 = F.qp / 6;
            for (int i = 0; i < 16; ++i) dcY[i] = F.qp >= 36 ? (f[i] * scale) * (1 << (q6 - 6)) : (f[i] * scale + (1 << (5 - q6))) >> (6 - q6);
        }
        int df = 0, dz = 0;
        for (int t = 0; t < 16; ++t) {
            const int xO = blk_x(t), yO = blk_y(t);
            int list[16], m[16], r[16];
            list[0] = dcY[kDcPos[t]];
            bool nzl = list[0] != 0;
            for (int i = 1; i < 16; ++i) {
                list[i] = S.ih_ac[mode][t][i - 1];
                nzl = nzl || list[i] != 0;
            }
            if (nzl) {
                unscan(list, m);
                dequant_idct(F.qp, m, true, r);
            }
            for (int i = 0; i < 16; ++i) {
                const int o = (yO + (i >> 2)) * 16 + xO + (i & 3);
                const int p = S.ih_pred[mode][o];
                const int v = nzl ? clip255(p + r[i]) : p;
                S.ih_rec[mode][o] = (uint8_t)v;
                df += iabs((int)S.src[o] - v);
                dz += iabs((int)S.src[o] - p);
            }
        }
        S.ih.dist[mode][0] = df;
        S.ih.dist[mode][1] = dz;
    }
#endif
}

// Intra16x16, the part that depends on the live state (rdo.c:1700-1809), from
// the modes' statistics in S.ih, modes in order: each mode's coded blocks
// rewrite the live TotalCoeffs (quirk 1) and read or write rdo.Single_ctr, its
// DC block writes both.  spec: the intra helper's guess of the live state
// (no row-start validation of the counter).  Returns the best mode's cost,
// coded-block mask, distortion and index.
HD void i16_light(Ctx& c, double& best_cost, int& best_cbp, int& best_dist, int& best_mode, bool spec)
{
    HL_FRESH_TID_K(c, 4);
    const FrameArgs& F = c.F;
    Shared& S = c.S;
    best_dist = 0;
    best_cost = 1.7976931348623157e308;
    best_cbp = 0;
    best_mode = 2;
    if (c.tid == 0) {
        S.e_type = ET_I16;
        S.flags = FL_INTRA;
        S.pm0 = PM_I16;
        S.i16mode = 2;
    }
#if defined(__HIP_DEVICE_COMPILE__)
    // The four modes at once, every wave alike (registers only): lane 16 m + t
    // holds block t of mode m.  The modes' sequential effects -- the live
    // TotalCoeffs (quirk 1) each mode's coded blocks leave for the nC of the
    // next, the DC block's write of block 0, the rdo.Single_ctr chain -- are
    // resolved in mode order as scalar work, with the results of the
    // reference's mode loop (host version below).
    const bool av[4] = {i16_mode_avail(S, 0), i16_mode_avail(S, 1), true, i16_mode_avail(S, 3)};
    const int l = c.tid & 63, m = l >> 4, t = l & 15;
    const bool avm = m == 0 ? av[0] : (m == 1 ? av[1] : (m == 2 ? true : av[3]));
    const int w = S.ih.blk[m][t];
    const int tc0 = S.tc[t];  // live TotalCoeff before the modes (lane t of every row)
    const bool called = avm && (w & 1);
    const int tcb = (w >> 1) & 31, sct = ((w >> 8) & 255) - 1;
    const unsigned long long BC = __ballot(called), BW = __ballot(called && tcb > 0);
    {
        // per mode: sum over its coded blocks of the counter of the last
        // writer at or before them (blocks before the first writer read the
        // entry value: counted below)
        const unsigned bwl = (unsigned)(BW >> (16 * m)) & 0xFFFFu;
        const unsigned upto = bwl & ((2u << t) - 1u);
        const int sv = __shfl(sct, (l & 48) | (upto ? 31 - __clz(upto) : 0), 64);
        const int s1 = row_sum(called && upto ? sv : 0);
        int bcbpm[4] = {0, 0, 0, 0};
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
            if (!av[mm]) continue;
            const unsigned bc = (unsigned)(BC >> (16 * mm)) & 0xFFFFu, bw = (unsigned)(BW >> (16 * mm)) & 0xFFFFu;
            const unsigned before = bw ? (bw & (0u - bw)) - 1u : 0xFFFFu;  // blocks before the first writer
            if (!spec && (bc & before) && !c.fresh) {
                // pipelined run: a speculated value is resolved here; once it
                // is exact (resolved in this MB or to its left) the read is
                // exact too.  The per-picture path records the stale read for
                // the host's row validation.
                if (!F.run_done) c.dep = 1;
                else if (c.spec) resolve_chain(c);
            }
            const int single = __builtin_amdgcn_readlane(s1, 16 * mm) + __popc(bc & before) * c.chain;
            if (bw) chain_write(c, __builtin_amdgcn_readlane(sct, 16 * mm + 31 - __clz(bw)));
            int bcbp = (int)bc;
            if (bcbp && single < 6) bcbp = 0;
            if (bcbp && uni(S.ih.dcs[mm][1]) > 0) chain_write(c, uni(S.ih.dcs[mm][2]));
            bcbpm[mm] = bcbp;
        }
        // AC rates: nC of every coded block with the live TotalCoeffs its mode sees
        int bits = 0;
        if (called) {
            const int nC = nc_luma_of(S, t, [&](int ni) -> int {
                const int wn = S.ih.blk[m][ni];
                if (wn & 1) return (wn >> 1) & 31;  // coded earlier in this mode
                int v = S.tc[ni];  // (written only after the barrier below)
#pragma unroll
                for (int mm = 0; mm < 3; ++mm) {
                    if (mm >= m || !av[mm]) continue;
                    const int wp = S.ih.blk[mm][ni];
                    if (wp & 1) v = (wp >> 1) & 31;
                    if (ni == 0 && bcbpm[mm]) v = S.ih.dcs[mm][1];
                }
                return v;
            });
            bits = (w >> 16) + coop_token_len(S.ct, nC, tcb, (w >> 6) & 3);
        }
        const int rate_ac = row_sum(bits);
        int fin = tc0;  // block t's live TotalCoeff after the modes (lanes 0-15)
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
            if (!av[mm]) continue;
            const int bcbp = bcbpm[mm];
            const int rate = __builtin_amdgcn_readlane(rate_ac, 16 * mm) + (bcbp ? uni(S.ih.dcs[mm][0]) : 0);
            const int dist = uni(S.ih.dist[mm][bcbp ? 0 : 1]);
            const double cost = dadd((double)dist, dmul(F.lambda, (double)rate));
            if (cost < best_cost) {
                best_cost = cost;
                best_dist = dist;
                best_cbp = bcbp;
                best_mode = mm;
            }
            const int wf = __shfl(w, 16 * mm + t, 64);
            if (wf & 1) fin = (wf >> 1) & 31;
            if (t == 0 && bcbp) fin = S.ih.dcs[mm][1];
        }
        HL_SYNC();  // every wave's reads of S.tc are done
        if (c.tid < 16) S.tc[c.tid] = (int8_t)fin;
        if (c.tid == 0) S.i16mode = best_mode;
        HL_SYNC();
    }
#else
    for (int mode = 0; mode < 4; ++mode) {
        if (!i16_mode_avail(S, mode)) continue;
        int single, bcbp, rate;
        int bits[16];
        for (int t = 0; t < 16; ++t) {
            const int w = S.ih.blk[mode][t];
            if (!(w & 1)) continue;
            const int nC = nc_luma_of(S, t, [&](int ni) -> int {
                const int wn = S.ih.blk[mode][ni];
                return (wn & 1) ? (wn >> 1) & 31 : S.tc[ni];
            });
            bits[t] = (w >> 16) + token_len(nC, (w >> 1) & 31, (w >> 6) & 3);
        }
        single = bcbp = rate = 0;
        for (int b = 0; b < 16; ++b) {
            const int w = S.ih.blk[mode][b];
            if (!(w & 1)) continue;
            rate += bits[b];
            bcbp |= 1 << b;
            if (((w >> 1) & 31) > 0) chain_write(c, ((w >> 8) & 255) - 1);
            else if (!spec && !c.fresh) c.dep = 1;
            single += c.chain;
        }
        for (int t = 0; t < 16; ++t)
            if (S.ih.blk[mode][t] & 1) S.tc[t] = (int8_t)((S.ih.blk[mode][t] >> 1) & 31);
        if (bcbp && single < 6) bcbp = 0;
        if (bcbp) {  // the DC block
            rate += uni(S.ih.dcs[mode][0]);
            if (uni(S.ih.dcs[mode][1]) > 0) chain_write(c, uni(S.ih.dcs[mode][2]));
            if (c.tid == 0) S.tc[0] = (int8_t)S.ih.dcs[mode][1];
        }
        const int dist = uni(S.ih.dist[mode][bcbp ? 0 : 1]);
        const double cost = dadd((double)dist, dmul(F.lambda, (double)rate));
        if (cost < best_cost) {
            best_cost = cost;
            best_dist = dist;
            best_cbp = bcbp;
            best_mode = mode;
            if (c.tid == 0) S.i16mode = mode;
        }
    }
#endif
}

// The chosen Intra16x16 mode's levels and reconstruction into S.i16_best_*:
// from this MB's own i16_heavy results in LDS, or from its intra helper's in
// global memory (hin)
HD void i16_copy_best(Ctx& c, int mode, bool coded, const IntraSpec* hin)
{
    HL_FRESH_TID_K(c, 5);
    Shared& S = c.S;
#if defined(__HIP_DEVICE_COMPILE__)
    const int t = c.tid;
    if (hin) {
        if (t < 16) reinterpret_cast<uint4*>(S.i16_best_rec)[t] = gmem(reinterpret_cast<const uint4*>(coded ? hin->rec[mode] : hin->pred[mode]))[t];
        else if (t < 48) reinterpret_cast<uint4*>(&S.i16_best_ac[0][0])[t - 16] = gmem(reinterpret_cast<const uint4*>(&hin->ac[mode][0][0]))[t - 16];
        else if (t < 50) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (coded) v = gmem(reinterpret_cast<const uint4*>(hin->dcl[mode]))[t - 48];
            reinterpret_cast<uint4*>(S.i16_best_dc)[t - 48] = v;
        }
    }
    else {
        if (t < 16) reinterpret_cast<uint4*>(S.i16_best_rec)[t] = reinterpret_cast<const uint4*>(coded ? S.ih_rec[mode] : S.ih_pred[mode])[t];
        else if (t < 48) reinterpret_cast<uint4*>(&S.i16_best_ac[0][0])[t - 16] = reinterpret_cast<const uint4*>(&S.ih_ac[mode][0][0])[t - 16];
        else if (t < 50) reinterpret_cast<uint4*>(S.i16_best_dc)[t - 48] = coded ? reinterpret_cast<const uint4*>(S.ih_dcl[mode])[t - 48] : make_uint4(0, 0, 0, 0);
    }
    HL_SYNC();
#else
    const uint8_t* rec = hin ? (coded ? hin->rec[mode] : hin->pred[mode]) : (coded ? S.ih_rec[mode] : S.ih_pred[mode]);
    const int16_t* ac = hin ? &hin->ac[mode][0][0] : &S.ih_ac[mode][0][0];
    const int16_t* dcl = hin ? hin->dcl[mode] : S.ih_dcl[mode];
    for (int t = 0; t < 256; ++t) {
        S.i16_best_rec[t] = rec[t];
        S.i16_best_ac[t >> 4][t & 15] = ac[t];
    }
    for (int i = 0; i < 16; ++i) S.i16_best_dc[i] = coded ? dcl[i] : 0;
#endif
}

HD void guess_i16(Ctx& c, double& best_cost, int& best_cbp, int& best_dist)
{
    i16_heavy(c);
    int bm;
    i16_light(c, best_cost, best_cbp, best_dist, bm, false);
    i16_copy_best(c, bm, best_cbp != 0, nullptr);
}

// --------------------------------------------------------------------------
// Intra 4x4 RDO (rdo.c:1813-2098)
// --------------------------------------------------------------------------
HD void guess_i4(Ctx& c, double& best_cost, int& cbp4, int& best_dist)
{
    HL_FRESH_TID_K(c, 6);
    best_dist = 0;
    const FrameArgs& F = c.F;
    Shared& S = c.S;
    best_cost = 0.0;
    cbp4 = 0;
    if (c.tid == 0) {
        S.e_type = ET_I_NXN;
        S.flags = FL_INTRA;
        S.pm0 = PM_I4;
    }
#if defined(__HIP_DEVICE_COMPILE__)
    // 4x4-block wavefront: step d runs the blocks with bx + 2 by = d (at most
    // two, z-order indices below).  Every block's left, top, top-left and
    // available top-right neighbours lie on earlier steps, and so do the
    // blocks whose TotalCoeffs its nC reads; the z-order effects (cost sum,
    // counter writes, CBP) are applied in z-order after the wavefront.
    // Wave s runs slot s of every step on its own: the block's neighbour
    // samples (lanes 0-13), its nine modes as nine 4-lane quads (hl_quad.h:
    // lane r = block row r), the resolution from the quads' registers and the
    // chosen quad's reconstruction and levels; one workgroup barrier per step
    // orders the two slots' writes before the next step reads them.
    constexpr uint8_t kWave[10][2] = {{0, 255}, {1, 255}, {2, 4}, {3, 5}, {6, 8}, {7, 9}, {10, 12}, {11, 13}, {14, 255}, {15, 255}};
    static_assert(kMbThreads >= 128, "one wave per wavefront slot");
    const int lane = c.tid & 63, sl = c.tid >> 6;
    const int qp = uni(F.qp), qbits = 15 + qp / 6, fq = (1 << qbits) / 3;
    const int m = min(lane >> 2, 8), rr = lane & 3;  // this quad's mode, this lane's block row
    LaneQ Q = c.Q;
    if (HL_FRESH_ZZ & 2) Q.zz = laneq_zz_fresh(Q.r);
    uint32_t te[4];  // the prediction taps of the lane's four samples (kI4Tab)
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) te[cc] = kI4Tab.e[m][rr * 4 + cc];
    for (int d = 0; d < 10; ++d) {
#if defined(HL_I4_PROF)
        HL_PROF_T(ti1);
#endif
        const int blk = sl == 0 ? kWave[d][0] : (sl == 1 ? kWave[d][1] : 255);
        if (blk != 255) {  // (wave-uniform)
            const int xO = blk_x(blk), yO = blk_y(blk);
            // nC first: its LDS reads overlap the neighbour gather
            // (nC is the same for all nine modes of a block: they only rewrite it)
            const int nC = uni(nc_luma_of(S, blk, [&](int ni) -> int { return S.tc[ni]; }));
            // lane i < 13: neighbour sample i (i4_neighbours, one sample per
            // lane); lane 13: the DC value (mode 2 of i4_pred_px); every lane
            // computes (the reads are clamped in range), lanes 0-13 are read
            // back with ds_bpermute (no LDS store, no wave barrier)
            int nbv;
            {
                const int i = lane & 15;
                const int X = i < 5 ? -1 : i - 5, Y = i < 5 ? i - 1 : -1;
                const int x = xO + X, y = yO + Y;
                const bool na = i >= 13 || (x > 15 && y >= 0) || (X > 3 && (blk == 3 || blk == 11));
                const int vl = S.left[y < 0 ? 0 : y], vt = S.top[min(max(x + 1, 0), 24)], vr = S.rec[(y < 0 ? 0 : y) * 16 + min(max(x, 0), 15)];
                int v = na ? kNA : ((x < 0 && y >= 0) ? vl : (y < 0 ? vt : vr));
                const int s8 = __builtin_amdgcn_readlane(v, 8), s9 = __builtin_amdgcn_readlane(v, 9);
                if (i >= 9 && i <= 12 && s9 == kNA && s8 != kNA) v = s8;
                const bool isl = i >= 1 && i <= 4, ist = i >= 5 && i <= 8;
                const int suml = row_sum(isl ? v : 0), sumt = row_sum(ist ? v : 0);
                const unsigned al = (unsigned)__ballot(isl && v != kNA) & 0xFFFFu, at = (unsigned)__ballot(ist && v != kNA) & 0xFFFFu;
                const bool ya = al == 0x1Eu, xa = at == 0x1E0u;
                const int dc = (xa && ya) ? (sumt + suml + 4) >> 3 : (ya ? (suml + 2) >> 2 : (xa ? (sumt + 2) >> 2 : 128));
                nbv = i == 13 ? dc : v;
            }
#if defined(HL_I4_PROF)
            HL_PROF_ADD(c, 12, ti1);  // neighbours, nC
            HL_PROF_T(ti3);
#endif
            struct {
                int v;
                __device__ int operator[](int i) const { return __builtin_amdgcn_readlane(v, i); }  // constant indices (i4_avail)
            } nbr{nbv};
            const bool ok = (lane >> 2) < 9 && i4_avail(m, nbr);
            const uint32_t sv4 = *reinterpret_cast<const uint32_t*>(&S.src[(yO + rr) * 16 + xO]);
            int x[4], y[4], q[4], r[4];
            uint32_t pr4 = 0;
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                const uint32_t e = te[cc];
                const int pred = i4_tab_pred(e, __shfl(nbv, (int)(e & 15), 64), __shfl(nbv, (int)((e >> 4) & 15), 64),
                                             __shfl(nbv, (int)((e >> 8) & 15), 64));
                x[cc] = (int)((sv4 >> (8 * cc)) & 255) - pred;
                pr4 |= (uint32_t)pred << (8 * cc);
            }
            const bool exact = quad_or(x[0] | x[1] | x[2] | x[3]) == 0;
            quad_fwd(Q, x, y);
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) q[cc] = quad_q1(y[cc], (cc & 1) ? Q.mfO : Q.mfE, qbits, fq);
            // reconstruction before the CAVLC chain: the two interleave
            quad_idct(Q, q, qp, r);
            uint32_t rec4 = 0;
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) rec4 |= (uint32_t)clip255((int)((pr4 >> (8 * cc)) & 255) + r[cc]) << (8 * cc);
            const int dd = quad_sum((int)__builtin_amdgcn_sad_u8(sv4, rec4, 0u));
            const CoopStat st = quad_cavlc(S.ct, Q, q, 0, S.lvq[c.tid >> 2]);
            const int bits = st.tc ? st.rest + coop_token_len(S.ct, nC, st.tc, st.t1) : 0;
            const double cost = exact ? 0.0 : dadd((double)dd, dmul(F.lambda, (double)bits));
#if defined(HL_I4_PROF)
            HL_PROF_ADD(c, 13, ti3);  // the nine modes
            HL_PROF_T(ti4);
#endif
            // resolution in mode order (rdo.c:1931-2014), lane 4 m standing for
            // mode m: the scan stops at the first exact mode; before it, the
            // last coded mode writes the counter and the first strict minimum wins
            const bool v0 = ok && rr == 0;
            const unsigned long long bex = __ballot(v0 && exact), bnz = __ballot(v0 && st.tc > 0);
            const int limitl = bex ? __ffsll((long long)bex) - 1 : 36;
            const unsigned long long W = bnz & ((1ull << limitl) - 1ull);
            const int lastwl = W ? 63 - __clzll((long long)W) : -1;
            double dmin;
            int bestl;
            bool best_zero;
            if (bex) {
                dmin = 0.0;
                bestl = limitl;
                best_zero = true;
            }
            else {
                const double rm = row_min_f64(v0 ? cost : 1.7976931348623157e308);  // rows 0-2 hold the nine modes
                double mn = 1.7976931348623157e308;
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const unsigned long long b64 = __builtin_bit_cast(unsigned long long, rm);
                    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b64 >> 32), 16 * k);
                    const unsigned lw = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b64, 16 * k);
                    mn = fmin(mn, __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lw));
                }
                dmin = mn;
                bestl = __ffsll((long long)__ballot(v0 && cost == mn)) - 1;
                best_zero = !((W >> bestl) & 1);
            }
            // (every value from registers, each stored by the lane that holds it:
            // no readlane; the stores carry no dependent load)
            if (lane == 0) {
                S.i4r_dmin[blk] = dmin;
                S.i4r_zero[blk] = best_zero;
                S.i4mode[blk] = (int8_t)(bestl >> 2);
                // the verification record (i4_verify): the costs used an nC
                // only without an exact mode and with a coded one
                S.ih.i4_ncls[blk] = (int8_t)(!bex && W ? nc_class(nC) : -1);
                if (lastwl < 0) {
                    S.i4r_sct[blk] = -1;
                    S.ih.i4_lwtc[blk] = -1;
                }
            }
            if (lane == bestl) S.i4r_dist[blk] = dd;  // d_min_dist4x4 (rdo.c:2011, 2023); 0 for an exact mode
            if (lane == lastwl) {  // the last coded mode before the scan stopped writes the counter and TotalCoeff
                S.i4r_sct[blk] = st.sctr;
                S.tc[blk] = (int8_t)st.tc;
                S.ih.i4_lwtc[blk] = (int8_t)st.tc;
            }
            if ((lane >> 2) == (bestl >> 2)) {  // the chosen mode's quad: its reconstruction rows and levels
                *reinterpret_cast<uint32_t*>(&S.rec[(yO + rr) * 16 + xO]) = rec4;
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) S.luma_level[blk][(Q.zz >> (4 * cc)) & 15] = q[cc];
            }
#if defined(HL_I4_PROF)
            HL_PROF_ADD(c, 15, ti4);  // the resolution
#endif
        }
#if defined(HL_I4_PROF)
        HL_PROF_T(ti2);
#endif
        HL_SYNC();
#if defined(HL_I4_PROF)
        HL_PROF_ADD(c, 14, ti2);  // the step's barrier
#endif
    }
    int last_sct = -1;
    for (int blk = 0; blk < 16; ++blk) {  // z-order: cost sum, distortion, CBP, counter writes
        best_cost = dadd(best_cost, uni(S.i4r_dmin[blk]));
        best_dist += uni(S.i4r_dist[blk]);
        if (!uni(S.i4r_zero[blk])) cbp4 |= 1 << blk;
        const int sct = uni(S.i4r_sct[blk]);
        if (sct >= 0) {
            chain_write(c, sct);
            last_sct = sct;
        }
    }
    if (c.tid == 0) {
        S.ih.i4_cbp = cbp4;
        S.ih.i4_dist = best_dist;
        S.ih.i4_sct = last_sct;
        S.ih.i4_cost = best_cost;
    }
#else
    S.ih.i4_sct = -1;
    for (int blk = 0; blk < 16; ++blk) {
        const int xO = blk_x(blk), yO = blk_y(blk);
        int p[13];
        i4_neighbours(S, blk, p);
        // nC is the same for all nine modes: they only rewrite this block
        const int nC = nc_luma_of(S, blk, [&](int ni) -> int { return S.tc[ni]; });
        HL_SYNC();
        for (int m = c.tid; m < 9; m += c.nthr) {
            S.i4_cost_ok[0][m] = i4_avail(m, p);
            if (!S.i4_cost_ok[0][m]) continue;
            int pred[16], res[16];
            i4_pred(m, p, pred);
            bool zero = true;
            for (int i = 0; i < 16; ++i) {
                res[i] = (int)S.src[(yO + (i >> 2)) * 16 + xO + (i & 3)] - pred[i];
                zero = zero && res[i] == 0;
            }
            S.i4_exact[0][m] = zero;
            S.i4_nz[0][m] = 0;
            S.i4_tc[0][m] = 0;
            S.i4_sctr[0][m] = -1;
            if (zero) {
                for (int i = 0; i < 16; ++i) {
                    S.i4_rec[0][m][i] = (uint8_t)pred[i];
                    S.i4_lv[0][m][i] = 0;
                }
                S.i4_cost[0][m] = 0.0;
                S.i4_dist[0][m] = 0;
                continue;
            }
            int w[16], q[16], lv[16];
            fwd4x4(res, w);
            quant4x4(F.qp, true, w, q);
            bool lz = true;
            for (int i = 0; i < 16; ++i) {
                lv[i] = q[kZigzag[i]];
                lz = lz && lv[i] == 0;
                S.i4_lv[0][m][i] = (int16_t)lv[i];
            }
            int bits = 0, d = 0;
            if (!lz) {
                const CavlcStat st = cavlc_stat(lv, 16, 15, false);
                bits = st.rest + token_len(nC, st.tc, st.t1);
                S.i4_nz[0][m] = 1;
                S.i4_tc[0][m] = st.tc;
                S.i4_sctr[0][m] = st.sctr;
                int r[16];
                dequant_idct(F.qp, q, false, r);
                for (int i = 0; i < 16; ++i) {
                    const int v = clip255(pred[i] + r[i]);
                    S.i4_rec[0][m][i] = (uint8_t)v;
                    d += iabs(res[i] + pred[i] - v);
                }
            }
            else {
                for (int i = 0; i < 16; ++i) {
                    S.i4_rec[0][m][i] = (uint8_t)pred[i];
                    d += iabs(res[i]);
                }
            }
            S.i4_dist[0][m] = d;
            S.i4_cost[0][m] = dadd((double)d, dmul(F.lambda, (double)bits));
        }
        HL_SYNC();
        // uniform resolution in mode order (rdo.c:1931-2014)
        double dmin = 1.7976931348623157e308;
        int best = 2, lastw = -1;
        bool best_zero = false, exact = false;
        for (int m = 0; m < 9; ++m) {
            if (!S.i4_cost_ok[0][m]) continue;
            if (S.i4_exact[0][m]) {
                dmin = 0.0;
                best = m;
                best_zero = true;
                exact = true;
                break;
            }
            if (S.i4_nz[0][m]) lastw = m;
            if (S.i4_cost[0][m] < dmin) {
                dmin = S.i4_cost[0][m];
                best = m;
                best_zero = !S.i4_nz[0][m];
            }
        }
        // the verification record (i4_verify): the costs used an nC only
        // without an exact mode and with a coded one
        S.ih.i4_ncls[blk] = (int8_t)(!exact && lastw >= 0 ? nc_class(nC) : -1);
        S.ih.i4_lwtc[blk] = (int8_t)(lastw >= 0 ? S.i4_tc[0][lastw] : -1);
        if (lastw >= 0) {
            chain_write(c, S.i4_sctr[0][lastw]);
            S.ih.i4_sct = S.i4_sctr[0][lastw];
        }
        best_cost = dadd(best_cost, dmin);
        best_dist += S.i4_dist[0][best];
        if (!best_zero) cbp4 |= 1 << blk;
        for (int t = c.tid; t < 16; t += c.nthr) {
            S.rec[(yO + (t >> 2)) * 16 + xO + (t & 3)] = S.i4_rec[0][best][t];
            S.luma_level[blk][t] = S.i4_exact[0][best] ? 0 : S.i4_lv[0][best][t];
        }
        if (c.tid == 0) {
            S.i4mode[blk] = (int8_t)best;
            if (lastw >= 0) S.tc[blk] = (int8_t)S.i4_tc[0][lastw];
        }
        HL_SYNC();
    }
    S.ih.i4_cbp = cbp4;
    S.ih.i4_dist = best_dist;
    S.ih.i4_cost = best_cost;
#endif
}

HD void pred_modes_4x4(Shared& S)  // pred_intra.c:541-615 (lane 0)
{
    for (int blk = 0; blk < 16; ++blk) {
        const int bx = blk_x(blk), by = blk_y(blk);
        int mA, mB;
        bool aA, aB;
        int pmA, pmB, iA, iB;
        if (bx == 0) {
            aA = S.nb[1].avail;
            pmA = S.nb_pm0[1];
            iA = aA ? S.nb_i4[1][blk_idx(12, by)] : 2;
        }
        else {
            aA = true;
            pmA = PM_I4;
            iA = S.i4mode[blk_idx(bx - 4, by)];
        }
        if (by == 0) {
            aB = S.nb[2].avail;
            pmB = S.nb_pm0[2];
            iB = aB ? S.nb_i4[2][blk_idx(bx, 12)] : 2;
        }
        else {
            aB = true;
            pmB = PM_I4;
            iB = S.i4mode[blk_idx(bx, by - 4)];
        }
        const bool dcf = !aA || !aB;
        mA = (dcf || pmA != PM_I4) ? 2 : iA;
        mB = (dcf || pmB != PM_I4) ? 2 : iB;
        const int pred = mA < mB ? mA : mB;
        if (pred == S.i4mode[blk]) S.prev_flag[blk] = 1;
        else {
            S.prev_flag[blk] = 0;
            S.rem_mode[blk] = (int8_t)(S.i4mode[blk] < pred ? S.i4mode[blk] : S.i4mode[blk] - 1);
        }
    }
}

// Intra4x4 decided by the intra helper under its guess of the live
// TotalCoeffs (S.ih, imported): every block whose mode costs used an nC must
// see the same nC class in the live state the MB left after its Intra16x16
// trials (S.tc).  Inside the MB a neighbour's TotalCoeff is the one its own
// resolution wrote, if any; by induction over the blocks' order every block
// then saw the same neighbours and costs.  Uniform.
HD bool i4_verify(Ctx& c)
{
    Shared& S = c.S;
#if defined(__HIP_DEVICE_COMPILE__)
    const int b = c.tid & 15, want = S.ih.i4_ncls[b];
    bool ok = true;
    if (want >= 0) {
        const int nC = nc_luma_of(S, b, [&](int ni) -> int {
            const int lw = S.ih.i4_lwtc[ni];
            return lw >= 0 ? lw : S.tc[ni];
        });
        ok = nc_class(nC) == want;
    }
    return (__ballot(!ok) & 0xFFFFull) == 0;
#else
    for (int b = 0; b < 16; ++b) {
        const int want = S.ih.i4_ncls[b];
        if (want < 0) continue;
        const int nC = nc_luma_of(S, b, [&](int ni) -> int {
            const int lw = S.ih.i4_lwtc[ni];
            return lw >= 0 ? lw : S.tc[ni];
        });
        if (nc_class(nC) != want) return false;
    }
    return true;
#endif
}

// The helper's Intra4x4 decision, verified, applied to the live MB as
// guess_i4 would have left it
HD void i4_apply(Ctx& c, const IntraSpec* hin, double& c4, int& cbp4, int& d4)
{
    HL_FRESH_TID_K(c, 7);
    Shared& S = c.S;
    if (c.tid == 0) {
        S.e_type = ET_I_NXN;
        S.flags = FL_INTRA;
        S.pm0 = PM_I4;
    }
#if defined(__HIP_DEVICE_COMPILE__)
    const int t = c.tid;
    if (t < 16) {
        const int lw = S.ih.i4_lwtc[t];
        if (lw >= 0) S.tc[t] = (int8_t)lw;
        S.i4mode[t] = S.ih.i4_mode[t];
        reinterpret_cast<uint4*>(S.rec)[t] = gmem(reinterpret_cast<const uint4*>(hin->i4_rec))[t];
    }
    else if (t < 16 + 128) {  // LumaLevel, two levels per lane
        const int k = t - 16;
        const uint32_t w = gmem(reinterpret_cast<const uint32_t*>(&hin->i4_lv[0][0]))[k];
        S.luma_level[k >> 3][(k & 7) * 2] = (int16_t)(w & 0xFFFF);
        S.luma_level[k >> 3][(k & 7) * 2 + 1] = (int16_t)(w >> 16);
    }
#else
    for (int t = 0; t < 16; ++t) {
        if (S.ih.i4_lwtc[t] >= 0) S.tc[t] = S.ih.i4_lwtc[t];
        S.i4mode[t] = S.ih.i4_mode[t];
    }
    for (int t = 0; t < 256; ++t) {
        S.rec[t] = hin->i4_rec[t];
        S.luma_level[t >> 4][t & 15] = hin->i4_lv[t >> 4][t & 15];
    }
#endif
    c4 = uni(S.ih.i4_cost);
    cbp4 = uni(S.ih.i4_cbp);
    d4 = uni(S.ih.i4_dist);
    const int sct = uni(S.ih.i4_sct);
    if (sct >= 0) chain_write(c, sct);
    HL_SYNC();
}

// hl_codec_264_rdo_mb_guess_best_intra_pred_avc, rdo.c:99-299.  Returns the
// best intra cost (the reference's static last_best_intra_cost).  hin: the
// results of this MB's intra helper task (S.ih already imported), or null.
HD double guess_intra(Ctx& c, const IntraSpec* hin = nullptr)
{
    HL_FRESH_TID_K(c, 8);
    const FrameArgs& F = c.F;
    Shared& S = c.S;
    double c16, c4;
    int cbp16, cbp4 = 0, d16 = 0, d4 = 0, m16;
    HL_PROF_T(t16);
    if (!hin) i16_heavy(c);
    i16_light(c, c16, cbp16, d16, m16, false);
    i16_copy_best(c, m16, cbp16 != 0, hin);
    HL_PROF_ADD(c, 10, t16);
    HL_PROF_T(t4);
    if (c16 == 0.0) c4 = 1.7976931348623157e308;
    else if (hin && uni(S.ih.i4_valid) && i4_verify(c)) {
        i4_apply(c, hin, c4, cbp4, d4);
#if defined(__HIP_DEVICE_COMPILE__)
        if (c.tid == 0 && F.perr) atomicAdd(F.perr + 2, 1);  // helper's Intra4x4 kept (hl_amd_last_helper_stats)
#else
        if (F.perr) ++F.perr[2];
#endif
    }
    else {
#if defined(__HIP_DEVICE_COMPILE__)
        if (hin && c.tid == 0 && F.perr) atomicAdd(F.perr + 3, 1);  // helper's Intra4x4 rejected
#else
        if (hin && F.perr) ++F.perr[3];
#endif
        guess_i4(c, c4, cbp4, d4);
    }
    HL_PROF_ADD(c, 11, t4);
#if defined(HL_PROF_MISC)
    HL_PROF_T(ttl);
#endif
    HL_SYNC();
    const int i16mode = S.i16mode;
    const int cmode = i16mode == 0 ? 2 : (i16mode == 3 ? 3 : (i16mode == 1 ? 1 : 0));
    bool is_i16 = false;
    if (c4 < c16) {
#if defined(__HIP_DEVICE_COMPILE__)
        // the predicted modes of the 16 blocks at once, in lanes 0-15 of
        // every wave (pred_modes_4x4 on lane l = block l; wave 0 stores them):
        // the count of mode remainders is then known to every wave without a
        // barrier.  (The barrier above ordered every read of the fields lane 0
        // rewrites here; the next reads are behind intra_chroma_pred's.)
        const int l = c.tid & 63;
        bool pf = true;
        if (l < 16) {
            const int blk = l, bx = blk_x(blk), by = blk_y(blk), m = S.i4mode[blk];
            const bool aA = bx ? true : S.nb[1].avail != 0, aB = by ? true : S.nb[2].avail != 0;
            const int pmA = bx ? PM_I4 : S.nb_pm0[1], pmB = by ? PM_I4 : S.nb_pm0[2];
            const int iA = bx ? S.i4mode[blk_idx(bx - 4, by)] : (aA ? S.nb_i4[1][blk_idx(12, by)] : 2);
            const int iB = by ? S.i4mode[blk_idx(bx, by - 4)] : (aB ? S.nb_i4[2][blk_idx(bx, 12)] : 2);
            const bool dcf = !aA || !aB;
            const int mA = (dcf || pmA != PM_I4) ? 2 : iA, mB = (dcf || pmB != PM_I4) ? 2 : iB;
            const int pred = mA < mB ? mA : mB;
            pf = pred == m;
            if (c.tid < 16) {
                S.prev_flag[blk] = pf ? 1 : 0;
                if (!pf) S.rem_mode[blk] = (int8_t)(m < pred ? m : m - 1);
            }
        }
        const int nz = __popcll(__ballot(!pf));
        if (c.tid == 0) {
            S.mb_type = 0;
            S.e_type = ET_I_NXN;
            S.flags = FL_INTRA;
            S.pm0 = PM_I4;
            S.cbp_l4x4 = cbp4;
        }
#else
        if (c.tid == 0) {
            S.mb_type = 0;
            S.e_type = ET_I_NXN;
            S.flags = FL_INTRA;
            S.pm0 = PM_I4;
            S.cbp_l4x4 = cbp4;
            pred_modes_4x4(S);
        }
        int nz = 0;
        for (int b = 0; b < 16; ++b) nz += !S.prev_flag[b];
#endif
        c4 = dadd(c4, dmul(F.lambda, (double)(16 + nz * 3)));
    }
    if (c16 <= c4) is_i16 = true;
    if (c.tid == 0) {
        S.chroma_mode = cmode;
        S.mad = is_i16 ? d16 : d4;
        if (is_i16) {
            S.mb_type = 1;
            S.e_type = ET_I16;
            S.flags = FL_INTRA;
            S.pm0 = PM_I16;
            S.cbp_l4x4 = cbp16;
        }
    }
    intra_chroma_pred(c, cmode);
    reconstruct_chroma(c, true);
    if (is_i16) {
        for (int t = c.tid; t < 256; t += c.nthr) S.rec[t] = S.i16_best_rec[t];
    }
    HL_SYNC();
    if (c.tid == 0) {
        guess_cbp(S);
        if (is_i16) S.mb_type += (S.cbp_c << 2) + S.i16mode + (S.cbp_l ? 12 : 0);
        if (!F.is_intra) S.mb_type += 5;
    }
    HL_SYNC();
#if defined(HL_PROF_MISC)
    HL_PROF_ADD(c, 15, ttl);
#endif
    return c16 < c4 ? c16 : c4;
}

// --------------------------------------------------------------------------
// Inter prediction of the whole MB with the final partitioning
// --------------------------------------------------------------------------
HD void part_of(const Shared& S, int lx, int ly, int& pi, int& spi)
{
    const NbInfo& n = S.nb[0];
    pi = ((ly >> lg2(n.part_h)) << (4 - lg2(n.part_w))) + (lx >> lg2(n.part_w));
    if (!is8x8(n.e_type)) spi = 0;
    else spi = (((ly & 7) >> lg2(n.sub_h[pi])) << (3 - lg2(n.sub_w[pi]))) + ((lx & 7) >> lg2(n.sub_w[pi]));
}

// luma prediction of the MB into S.pred, chroma into S.predc; mv from S.nb[0].mv
HD void inter_pred_mb(Ctx& c, bool chroma_only_16x16, bool luma)
{
    HL_FRESH_TID_K(c, 9);
    const FrameArgs& F = c.F;
    Shared& S = c.S;
#if defined(HL_PROF_MISC)
    HL_PROF_T(tip);
#endif
    if (luma) {
#if defined(__HIP_DEVICE_COMPILE__)
        // one 4-lane quad per 4x4 block, lane r = row r: the quarter-pel
        // sample pairs of the search (put_cand / eval_candidates)
        if (c.tid < 64) {
            const int t = c.tid >> 2, r = c.tid & 3, bx = blk_x(t), by = blk_y(t);
            int pi, spi;
            part_of(S, bx, by, pi, spi);
            const NbInfo& n = S.nb[0];
            const int xP = part_x(pi, n.part_w), yP = part_y(pi, n.part_w, n.part_h);
            int xS = 0, yS = 0;
            if (is8x8(n.e_type)) {
                xS = sub_x(spi, n.sub_w[pi]);
                yS = sub_y(spi, n.sub_w[pi], n.sub_h[pi]);
            }
            const int mvx = n.mv[pi][spi][0], mvy = n.mv[pi][spi][1];
            const int X = clip3(-17, F.W + 17, c.xL + xP + xS + (mvx >> 2)) + kPad + bx - xP - xS;
            const int Y = clip3(-17, F.H + 17, c.yL + yP + yS + (mvy >> 2)) + kPad + by - yP - yS + r;
            const uint32_t e = S.qtab[((mvy & 3) << 2) | (mvx & 3)];
            const int o1 = (int)(e & 3) * F.plsz + (Y + (int)((e >> 3) & 1)) * F.pstride + X + (int)((e >> 2) & 1);
            const int o2 = (e & 16) ? (int)((e >> 5) & 3) * F.plsz + (Y + (int)((e >> 8) & 1)) * F.pstride + X + (int)((e >> 7) & 1) : o1;
            const auto base = gmem(F.pl[0]);
            const uint32_t pr = avg_u8x4(ld_u8x4(base, o1), ld_u8x4(base, o2));
            *reinterpret_cast<int4*>(&S.pred[(by + r) * 16 + bx]) =
                make_int4((int)(pr & 255), (int)((pr >> 8) & 255), (int)((pr >> 16) & 255), (int)(pr >> 24));
        }
#else
        for (int t = c.tid; t < 16; t += c.nthr) {
            const int bx = blk_x(t), by = blk_y(t);
            int pi, spi;
            part_of(S, bx, by, pi, spi);
            const NbInfo& n = S.nb[0];
            const int xP = part_x(pi, n.part_w), yP = part_y(pi, n.part_w, n.part_h);
            int xS = 0, yS = 0;
            if (is8x8(n.e_type)) {
                xS = sub_x(spi, n.sub_w[pi]);
                yS = sub_y(spi, n.sub_w[pi], n.sub_h[pi]);
            }
            const int mvx = n.mv[pi][spi][0], mvy = n.mv[pi][spi][1];
            const int X = clip3(-17, F.W + 17, c.xL + xP + xS + (mvx >> 2)) + bx - xP - xS;
            const int Y = clip3(-17, F.H + 17, c.yL + yP + yS + (mvy >> 2)) + by - yP - yS;
            int p[16];
            pred_luma4x4(F, X, Y, mvx & 3, mvy & 3, p);
            for (int i = 0; i < 16; ++i) S.pred[(by + (i >> 2)) * 16 + bx + (i & 3)] = p[i];
        }
#endif
    }
    for (int t = c.tid; t < 64; t += c.nthr) {
        const int cx = t & 7, cy = t >> 3;
        int pi = 0, spi = 0;
        if (!chroma_only_16x16) part_of(S, cx * 2, cy * 2, pi, spi);
        const int mvx = S.nb[0].mv[pi][spi][0], mvy = S.nb[0].mv[pi][spi][1];
        const int xi = (c.xL >> 1) + cx + (mvx >> 3), yi = (c.yL >> 1) + cy + (mvy >> 3);
        const int xF = mvx & 7, yF = mvy & 7;
        const int xa = clip3(0, F.Wc - 1, xi), xb = clip3(0, F.Wc - 1, xi + 1);
        const int ya = clip3(0, F.Hc - 1, yi), yb = clip3(0, F.Hc - 1, yi + 1);
        for (int comp = 0; comp < 2; ++comp) {
            const auto r = gmem(F.ref[1 + comp]);
            S.predc[comp][t] = ((8 - xF) * (8 - yF) * r[ya * F.Wc + xa] + xF * (8 - yF) * r[ya * F.Wc + xb] +
                                (8 - xF) * yF * r[yb * F.Wc + xa] + xF * yF * r[yb * F.Wc + xb] + 32) >> 6;
        }
    }
    HL_SYNC();
#if defined(HL_PROF_MISC)
    HL_PROF_ADD(c, 18, tip);
#endif
}

// rdo.c:2274-2500 luma part (chroma via reconstruct_chroma)
HD void reconstruct_inter_luma(Ctx& c, int single_luma)
{
    HL_FRESH_TID_K(c, 10);
    const FrameArgs& F = c.F;
    Shared& S = c.S;
#if defined(__HIP_DEVICE_COMPILE__)
    // one 4-lane quad per 4x4 block (hl_quad.h, as the search evaluated it)
    if (c.tid < 64) {
        const int t = c.tid >> 2, r = c.tid & 3, bx = blk_x(t), by = blk_y(t);
        LaneQ Q = c.Q;
        if (HL_FRESH_ZZ & 2) Q.zz = laneq_zz_fresh(Q.r);
        const int4 pv = *reinterpret_cast<const int4*>(&S.pred[(by + r) * 16 + bx]);
        const int pr[4] = {pv.x, pv.y, pv.z, pv.w};
        const uint32_t sv = *reinterpret_cast<const uint32_t*>(&S.src[(by + r) * 16 + bx]);
        int q[4] = {0, 0, 0, 0};
        bool coded = false;
        if (single_luma >= 6) {
            const int qbits = 15 + F.qp / 6, f = (1 << qbits) / 6;
            int x[4], y[4];
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) x[cc] = (int)((sv >> (8 * cc)) & 255) - pr[cc];
            quad_fwd(Q, x, y);
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) q[cc] = quad_q1(y[cc], (cc & 1) ? Q.mfO : Q.mfE, qbits, f);
            coded = quad_or(q[0] | q[1] | q[2] | q[3]) != 0;
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) S.luma_level[t][(Q.zz >> (4 * cc)) & 15] = coded ? q[cc] : 0;
        }
        uint32_t rec = 0;
        if (coded) {
            int rr[4];
            quad_idct(Q, q, F.qp, rr);
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) rec |= (uint32_t)clip255(pr[cc] + rr[cc]) << (8 * cc);
        }
        else rec = (uint32_t)pr[0] | ((uint32_t)pr[1] << 8) | ((uint32_t)pr[2] << 16) | ((uint32_t)pr[3] << 24);
        *reinterpret_cast<uint32_t*>(&S.rec[(by + r) * 16 + bx]) = rec;
        const unsigned long long bal = __ballot(coded && r == 0);
        if (c.tid == 0) {
            int cbp = 0;
#pragma unroll
            for (int b = 0; b < 16; ++b) cbp |= (int)((bal >> (4 * b)) & 1) << b;
            S.cbp_l4x4 = cbp;
        }
    }
    HL_SYNC();
#else
    for (int t = c.tid; t < 16; t += c.nthr) {
        const int xO = blk_x(t), yO = blk_y(t);
        int res[16], pred[16];
        bool zero = true;
        for (int i = 0; i < 16; ++i) {
            const int o = (yO + (i >> 2)) * 16 + xO + (i & 3);
            pred[i] = S.pred[o];
            res[i] = (int)S.src[o] - pred[i];
            zero = zero && res[i] == 0;
        }
        bool coded = false;
        int q[16];
        if (single_luma >= 6) {
            if (!zero) {
                int w[16];
                fwd4x4(res, w);
                quant4x4(F.qp, false, w, q);
                bool qz = true;
                for (int i = 0; i < 16; ++i) qz = qz && q[i] == 0;
                coded = !qz;
            }
            for (int i = 0; i < 16; ++i) S.luma_level[t][i] = coded ? q[kZigzag[i]] : 0;
        }
        int r[16];
        if (coded) dequant_idct(F.qp, q, false, r);
        for (int i = 0; i < 16; ++i) {
            const int o = (yO + (i >> 2)) * 16 + xO + (i & 3);
            S.rec[o] = (uint8_t)(coded ? clip255(pred[i] + r[i]) : pred[i]);
        }
        S.i16_called[t] = coded;  // reuse as per-block coded flag
    }
    HL_SYNC();
    if (c.tid == 0) {
        int cbp = 0;
        for (int b = 0; b < 16; ++b) cbp |= S.i16_called[b] << b;
        S.cbp_l4x4 = cbp;
    }
    HL_SYNC();
#endif
}

// --------------------------------------------------------------------------
// Early termination (me_early_term_flag), rdo.c:888-931 (JVT-O079
// 2.1.3.4.3.1): after the 16x16 search only the partition modes the source
// MB's homogeneity allows are searched.  Homogeneity of an 8x8 quadrant is
// the Sobel-like edge energy of hl_math_homogeneousity8x8_u8_cpp
// (hl_math.c:470-486); the quadrants of border MBs are shifted one sample
// inwards (rdo.c:895-896).  Returns the mode mask, bit j + 1 = kParts[j].
// One wave per quadrant, one lane per sample.
// --------------------------------------------------------------------------
constexpr int kHomoTh16x16 = 20000, kHomoTh8x8 = 5000, kHomoTh8x4 = 7500;  // hl_codec_264_defs.h:61-63

HD int homo_sample(const FrameArgs& F, int x, int y)  // |dx| + |dy| at source sample (x, y), eq. 2-35
{
    const auto u = gmem(F.src[0]) + y * F.W + x;
    const auto um = u - F.W, up = u + F.W;
    const int dx = up[-1] + (up[0] << 1) + up[1] - um[-1] - (um[0] << 1) - um[1];
    const int dy = um[1] + (u[1] << 1) + up[1] - um[-1] - (u[-1] << 1) - up[-1];
    return iabs(dx) + iabs(dy);
}

HD int early_term_modes(Ctx& c)
{
    const FrameArgs& F = c.F;
    Shared& S = c.S;
    const int xs = c.xL == 0 ? 1 : (c.xL == F.W - 16 ? F.W - 17 : c.xL);
    const int ys = c.yL == 0 ? 1 : (c.yL == F.H - 16 ? F.H - 17 : c.yL);
#if defined(__HIP_DEVICE_COMPILE__)
    const int q = c.tid >> 6, i = c.tid & 63;
    if (q < 4) {
        int v = homo_sample(F, xs + (q & 1) * 8 + (i & 7), ys + (q >> 1) * 8 + (i >> 3));
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (i == 0) S.homo[q] = v;
    }
#else
    for (int q = 0; q < 4; ++q) {
        int v = 0;
        for (int i = 0; i < 64; ++i) v += homo_sample(F, xs + (q & 1) * 8 + (i & 7), ys + (q >> 1) * 8 + (i >> 3));
        S.homo[q] = v;
    }
#endif
    HL_SYNC();
    const int h0 = uni(S.homo[0]), h1 = uni(S.homo[1]), h2 = uni(S.homo[2]), h3 = uni(S.homo[3]);
    if (h0 < kHomoTh8x8 && h1 < kHomoTh8x8 && h2 < kHomoTh8x8 && h3 < kHomoTh8x8) return 1 << 1;
    if (h0 + h1 + h2 + h3 < kHomoTh16x16) return (h0 < kHomoTh8x8 && h1 < kHomoTh8x8) ? (1 << 1) | (1 << 2) : (1 << 1) | (1 << 3);
    if (h0 < kHomoTh8x4 && h1 < kHomoTh8x4 && h2 < kHomoTh8x4 && h3 < kHomoTh8x4) return 0x7E;  // all but the 4x4 sub-partitions
    return 0xFFFF;
}

// --------------------------------------------------------------------------
// The MB's intra helper task (pipelined runs, FrameArgs::hstate): take the
// task over if no workgroup has claimed it yet (the MB then decides intra
// itself), else wait until the helper has published -- it waits on nothing,
// so the wait ends.  use: import the helper's IntraHead into S.ih.  Returns
// the helper's results, or null.  Called once per P macroblock, before
// mb_end: the per-address results buffer is free again once the MB ends.
// --------------------------------------------------------------------------
HD const IntraSpec* helper_join(Ctx& c, bool use)
{
    const FrameArgs& F = c.F;
    if (!F.hstate) return nullptr;
#if defined(__HIP_DEVICE_COMPILE__)
    Shared& S = c.S;
    if (c.tid < 64) {
        if (c.tid == 0) {
            int s = atomicCAS(F.hstate + c.addr, HS_FREE, HS_MAIN);
            if (s == HS_CLAIMED) {
                const int e0 = F.perr ? ld_relaxed(F.perr) : 0;
                spin_ge(F.hstate + c.addr, HS_DONE, F.perr);
                s = F.perr && ld_relaxed(F.perr) != e0 ? HS_MAIN : HS_DONE;  // gave up: decide intra here
            }
            if (s == HS_MAIN && F.perr) atomicAdd(F.perr + 4, 1);  // helper not claimed in time
            S.hs_x = s;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    HL_SYNC();
    if (!use || uni(S.hs_x) != HS_DONE) return nullptr;
    const IntraSpec* hin = F.ispec + c.addr;
    constexpr int kHW = (int)(sizeof(IntraHead) / 16);
    if (c.tid < kHW) reinterpret_cast<uint4*>(&S.ih)[c.tid] = gmem(reinterpret_cast<const uint4*>(&hin->h))[c.tid];
    HL_SYNC();
    return hin;
#else
    if (F.hstate[c.addr] != HS_DONE || !use) return nullptr;
    const IntraSpec* hin = F.ispec + c.addr;
    c.S.ih = hin->h;
    return hin;
#endif
}

// --------------------------------------------------------------------------
// P macroblock decision, rdo.c:678-1271
// --------------------------------------------------------------------------
HD int32_t fam_etype(int f) { return f < 3 ? ET_P16x16 + f : ET_P8x8REF0; }

// One partitioning j of family fam searched (rdo.c:731-760): the partition
// mode's best cost (header bits not added), its Single_ctr sum and
// distortion; returns the P_Skip probe's outcome (16x16 only).
template <bool REC>
HD bool search_family_part(Ctx& c, int j, int fam, double& cost_sum, int& single_sum, int& dist_sum)
{
    Shared& S = c.S;
    const PartDef& pd = kParts[j];
    HL_SYNC();
    if (c.tid == 0) {
        S.e_type = fam_etype(fam);
        S.nb[0].e_type = fam_etype(fam);
        S.nb[0].part_w = pd.part_w;
        S.nb[0].part_h = pd.part_h;
        for (int i = 0; i < 4; ++i) {
            S.nb[0].sub_w[i] = pd.sub_w;
            S.nb[0].sub_h[i] = pd.sub_h;
        }
        grid_reset_inside(S);
    }
    HL_SYNC();
    bool prob = false;
    for (int pi = 0; pi < pd.num_part; ++pi)
        for (int spi = 0; spi < pd.num_sub; ++spi) {
            const bool p = search_partition<REC>(c, pd, pi, spi, j == 0 && pi == 0 && spi == 0);
            if (j == 0 && pi == 0 && spi == 0) prob = p;
        }
    for (int pi = 0; pi < pd.num_part; ++pi)
        for (int spi = 0; spi < pd.num_sub; ++spi) {
            cost_sum = dadd(cost_sum, uni(S.bcost[pi][spi]));
            single_sum += uni(S.bsingle[pi][spi]);
            dist_sum += uni(S.bdist[pi][spi]);
        }
    return prob;
}

// --------------------------------------------------------------------------
// Partitioning helper tasks of the 8x8 family (lone pictures): while a P
// macroblock searches 16x16 / 16x8 / 8x16, idle workgroups search the P8x8
// partitionings (kParts[3..6]), one task per partitioning, each from the
// MB-start live TotalCoeffs.  A partitioning reads the live TotalCoeffs it
// starts from only through nC classes, and only until it overwrites a block
// itself; the helper records, for every such read, the interval of the entry
// value (or of the sum of two) that keeps the class (Shared::f3lo / f3hi).  A
// partitioning never reads rdo.Single_ctr, nor the motion another one left.
// So if the macroblock's real entry values for partitioning j -- what j - 1
// left, imported or searched -- lie in every interval of j's helper, j's every
// cost, decision and write is the helper's, and the macroblock takes them
// (f3_import); otherwise it searches j itself.  The four run side by side:
// the macroblock's 8x8-family latency is that of its longest partitioning
// (4x4, 16 searches), not of the family's 36 searches in a row.
// --------------------------------------------------------------------------
// The macroblock's real entry values e (its live TotalCoeffs) against the helper's intervals
template <typename P>
HD bool f3_verify(const int8_t* e, P h)
{
    bool ok = true;
    for (int i = 0; i < 16; ++i) {
        const int v = e[i];
        ok = ok && v >= h->lo[i] && v <= h->hi[i];
        if (blk_x(i) > 0 && blk_y(i) > 0) {
            const int sm = e[blk_idx(blk_x(i) - 4, blk_y(i))] + e[blk_idx(blk_x(i), blk_y(i) - 4)];
            ok = ok && sm >= h->lo[16 + i] && sm <= h->hi[16 + i];
        }
    }
    return ok;
}

// f3out: run as the macroblock's helper task of partitioning hj (3..6) instead
// (that partitioning only, recorded for f3_verify, into f3out; see above)
HD void guess_inter(Ctx& c, Fam3Out* f3out = nullptr, int hj = 3)
{
    const FrameArgs& F = c.F;
    Shared& S = c.S;
    auto fam_first = [](int f) -> int { return f < 4 ? f : 7; };  // {0, 1, 2, 3, 7}
    double best_cost = 1.7976931348623157e308;
    int best_single = 9, best_part = -1, best_fam = -1, best_dist = 0;
    bool best_found = false, pskip = false;
    // b_probably_pskip is function-scoped in the reference (rdo.c:691): a mode
    // skipped by early termination leaves the last searched mode's value
    bool probably = false;
    int mode_flags = 0xFFFF;  // rdo.c:874
    if (c.tid == 0) S.flags = FL_INTER;
    // were this macroblock's partitioning helpers queued?  (HS_MAIN: no;
    // read at the start, used at the 8x8 family)
#if defined(__HIP_DEVICE_COMPILE__)
    if (HL_FAM3 && F.hstate3 && !f3out && c.tid == 0) S.f3b[1] = ld_relaxed(F.hstate3 + c.addr * 4) != HS_MAIN;
#else
    if (HL_FAM3 && F.hstate3 && !f3out && c.tid == 0) S.f3b[1] = F.hstate3[c.addr * 4] != HS_MAIN;
#endif
    // a partitioning's results against the best so far (rdo.c:1148-1160)
    auto take_part = [&](int j, int fam, double cost_sum, int single_sum, int dist_sum, auto bmv, auto bmvp) {
        const PartDef& pd = kParts[j];
        cost_sum = dadd(cost_sum, dmul(F.lambda, (double)pd.hdr_bits));
        if (cost_sum < best_cost) {
            best_cost = cost_sum;
            best_single = single_sum;
            best_dist = dist_sum;
            best_part = j;
            best_fam = fam;
            HL_SYNC();
            if (c.tid == 0) {
                for (int pi = 0; pi < pd.num_part; ++pi)
                    for (int spi = 0; spi < pd.num_sub; ++spi) {
                        const int o = (pi * 4 + spi) * 2;
                        S.best_mv[pi][spi][0] = bmv[o];
                        S.best_mv[pi][spi][1] = bmv[o + 1];
                        S.best_mvp[pi][spi][0] = bmvp[o];
                        S.best_mvp[pi][spi][1] = bmvp[o + 1];
                    }
            }
            HL_SYNC();
        }
    };
    // the helper: the MB-start state, the recording on
    if (HL_FAM3 && f3out) {
        if (F.early_term) mode_flags = early_term_modes(c);
        for (int i = c.tid; i < 32; i += c.nthr) {
            S.f3lo[i] = 0;
            S.f3hi[i] = 127;
        }
        if (c.tid == 0) {
            S.f3w = 0;
            S.f3b[0] = 0;  // searched (mode_flags)
        }
        HL_SYNC();
        c.f3rec = 1;
        c.fresh = 0;
    }
    for (int fam = HL_FAM3 && f3out ? 3 : 0; fam < 4 && !best_found; ++fam) {
        const int jlo = HL_FAM3 && f3out ? hj : fam_first(fam), jhi = HL_FAM3 && f3out ? hj + 1 : fam_first(fam + 1);
        for (int j = jlo; j < jhi; ++j) {
            if (!((1 << (j + 1)) & mode_flags)) continue;
            // partitioning j's helper (8x8 family): taken over if no workgroup
            // claimed it yet, else waited for (it waits on nothing) and taken
            // if its intervals hold for the real entry state (the live
            // TotalCoeffs partitioning j - 1 left)
            if (HL_FAM3 && fam == 3 && F.hstate3 && !f3out && uni(S.f3b[1])) {
                const int hx = c.addr * 4 + (j - 3);  // its state and results
#if defined(__HIP_DEVICE_COMPILE__)
                if (c.tid == 0) {
                    const int st = atomicCAS(F.hstate3 + hx, HS_FREE, HS_MAIN);
#if defined(HL_PROFILE)
                    if (F.prof) atomicAdd(F.prof + (st == HS_FREE ? 60 : (st == HS_CLAIMED ? 61 : 62)), 1ull);  // taken over / still running / done
#endif
                    S.f3b[4 + j - 3] = st == HS_FREE ? HS_MAIN : st;
                }
                if (c.tid < 64) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                HL_SYNC();
#else
                if (c.tid == 0) S.f3b[4 + j - 3] = F.hstate3[hx] == HS_FREE ? HS_MAIN : F.hstate3[hx];
#endif
                int h3 = uni(S.f3b[4 + j - 3]);
#if defined(__HIP_DEVICE_COMPILE__)
                if (h3 == HS_CLAIMED) {
                    if (c.tid < 64) {
                        if (c.tid == 0) {
                            spin_ge(F.hstate3 + hx, HS_DONE, F.perr);
                            S.f3b[4 + j - 3] = ld_relaxed(F.hstate3 + hx) == HS_DONE ? HS_DONE : HS_MAIN;  // (a wait that gave up: searched here)
                        }
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                    HL_SYNC();
                    h3 = uni(S.f3b[4 + j - 3]);
                }
                const auto h = gmem(F.f3 + hx);
#else
                const Fam3Out* h = F.f3 + hx;
#endif
                if (h3 == HS_DONE) {
                    if (((uni((int)h->done_mask) >> (j - 3)) & 1) && f3_verify(S.tc, h)) {
                        // the helper's partitioning from the entry state: its
                        // results against the best so far, the live TotalCoeffs
                        // it wrote, rdo.Single_ctr, the partition state it leaves
                        const int wm = uni((int)h->wmask);
                        take_part(j, 3, uni((double)h->cost[j - 3]), uni((int)h->single[j - 3]), uni((int)h->dist[j - 3]), &h->bmv[j - 3][0][0][0],
                                  &h->bmvp[j - 3][0][0][0]);
                        HL_SYNC();
                        for (int i = c.tid; i < 16; i += c.nthr)
                            if ((wm >> i) & 1) S.tc[i] = h->tc[i];
                        for (int i = c.tid; i < 32; i += c.nthr) {
                            (&S.nb[0].mv[0][0][0])[i] = (&h->nbmv[0][0][0])[i];
                            (&S.bmv[0][0][0])[i] = (&h->bmv[j - 3][0][0][0])[i];
                            (&S.bmvp[0][0][0])[i] = (&h->bmvp[j - 3][0][0][0])[i];
                        }
                        for (int i = c.tid; i < 36; i += c.nthr) {
                            (&S.mvg[0][0])[i] = (&h->mvg[0][0])[i];
                            (&S.mvs[0][0])[i] = (&h->mvs[0][0])[i];
                        }
                        if (c.tid == 0) {
                            const PartDef& pd = kParts[j];
                            S.e_type = fam_etype(3);
                            S.nb[0].e_type = fam_etype(3);
                            S.nb[0].part_w = pd.part_w;
                            S.nb[0].part_h = pd.part_h;
                            for (int i = 0; i < 4; ++i) {
                                S.nb[0].sub_w[i] = pd.sub_w;
                                S.nb[0].sub_h[i] = pd.sub_h;
                            }
                        }
                        if (uni((int)h->fresh)) chain_write(c, uni((int)h->chain));
                        probably = false;  // (the probe is 16x16's; partitioning j was the last searched)
                        HL_SYNC();
#if defined(__HIP_DEVICE_COMPILE__)
                        if (c.tid == 0 && F.perr) atomicAdd(F.perr + 5, 1);
#else
                        if (F.perr) ++F.perr[5];
#endif
                        continue;
                    }
#if defined(__HIP_DEVICE_COMPILE__)
                    if (c.tid == 0 && F.perr) atomicAdd(F.perr + 6, 1);
#else
                    if (F.perr) ++F.perr[6];
#endif
                }
            }
            if (F.early_term && j == 0) {
#if !defined(HL_STEP_PROF) && !defined(HL_I4_PROF) && !defined(HL_NBLK_PROF)
                HL_PROF_T(tet);
#endif
                mode_flags = early_term_modes(c);
#if !defined(HL_STEP_PROF) && !defined(HL_I4_PROF) && !defined(HL_NBLK_PROF)
                HL_PROF_ADD(c, 12, tet);  // early termination's homogeneity
#endif
            }
            double cost_sum = 0.0;
            int single_sum = 0, dist_sum = 0;
            // (one call site: every copy of the search is inlined)
            // (the helper runs its own instantiation, with the recording)
            if (HL_FAM3 && f3out) probably = search_family_part<true>(c, j, fam, cost_sum, single_sum, dist_sum);
            else probably = search_family_part<false>(c, j, fam, cost_sum, single_sum, dist_sum);
            if (HL_FAM3 && f3out) {  // the helper: this partitioning's results
                HL_SYNC();
#if defined(__HIP_DEVICE_COMPILE__)
                auto o = gmem(f3out);
#else
                Fam3Out* o = f3out;
#endif
                if (c.tid == 0) {
                    o->cost[j - 3] = cost_sum;
                    o->single[j - 3] = single_sum;
                    o->dist[j - 3] = dist_sum;
                    S.f3b[0] |= 1 << (j - 3);
                }
                for (int i = c.tid; i < 32; i += c.nthr)  // best MVs and MVPs, 16 words each
                    (i < 16 ? reinterpret_cast<int32_t*>(&o->bmv[j - 3][0][0][0]) : reinterpret_cast<int32_t*>(&o->bmvp[j - 3][0][0][0]))[i & 15] =
                        reinterpret_cast<const int32_t*>(i < 16 ? &S.bmv[0][0][0] : &S.bmvp[0][0][0])[i & 15];
                continue;
            }
            if (!probably && cost_sum != 0.0 && single_sum < 6 && fam == 0) {
                int smv[2];
                skip_mv(S, smv);
                probably = uni(smv[0]) == uni(S.bmvp[0][0][0]) && uni(smv[1]) == uni(S.bmvp[0][0][1]) &&
                           uni(S.bmv[0][0][0]) == uni(S.bmvp[0][0][0]) && uni(S.bmv[0][0][1]) == uni(S.bmvp[0][0][1]);
            }
            take_part(j, fam, cost_sum, single_sum, dist_sum, &S.bmv[0][0][0], &S.bmvp[0][0][0]);
        }
        pskip = probably;
        if (pskip) {  // _is_zeros_inter16x16_chroma, rdo.c:2140-2215
            HL_SYNC();
            if (c.tid == 0) {
                S.nb[0].mv[0][0][0] = S.best_mv[0][0][0];
                S.nb[0].mv[0][0][1] = S.best_mv[0][0][1];
            }
            HL_SYNC();
            inter_pred_mb(c, true, false);
            reconstruct_chroma(c, false);
            pskip = !uni(S.cbp_cac[0]) && !uni(S.cbp_cac[1]) && !uni(S.cbp_cdc[0]) && !uni(S.cbp_cdc[1]);
        }
        best_found = best_found || best_cost == 0.0 || pskip;
    }
    if (HL_FAM3 && f3out) {  // the helper: the partitioning's end state (the task publishes it with its release)
        HL_SYNC();
#if defined(__HIP_DEVICE_COMPILE__)
        auto o = gmem(f3out);
#else
        Fam3Out* o = f3out;
#endif
        if (c.tid == 0) {
            o->done_mask = S.f3b[0];
            o->wmask = S.f3w;
            o->chain = c.chain;
            o->fresh = c.fresh;
            o->e_last = hj;
        }
        for (int i = c.tid; i < 16; i += c.nthr) o->tc[i] = S.tc[i];
        for (int i = c.tid; i < 32; i += c.nthr) {
            o->lo[i] = (int8_t)S.f3lo[i];
            o->hi[i] = (int8_t)S.f3hi[i];
            (&o->nbmv[0][0][0])[i] = (&S.nb[0].mv[0][0][0])[i];
        }
        for (int i = c.tid; i < 36; i += c.nthr) {
            (&o->mvg[0][0])[i] = (&S.mvg[0][0])[i];
            (&o->mvs[0][0])[i] = (&S.mvs[0][0])[i];
        }
        return;
    }
#if defined(__HIP_DEVICE_COMPILE__)
    // the helpers of partitionings the macroblock did not reach (a P_Skip or a
    // zero cost ended the search, or early termination left them out): not
    // started yet, they are cancelled (a running one writes only its own slot)
    if (HL_FAM3 && F.hstate3 && c.tid < 4 && S.f3b[1]) atomicCAS(F.hstate3 + c.addr * 4 + c.tid, HS_FREE, HS_MAIN);
#endif
    if (!pskip) {
        HL_PROF_T(ti);
        HL_PROF_T(tj);
        const IntraSpec* hin = helper_join(c, true);
#if !defined(HL_STEP_PROF)
        HL_PROF_ADD(c, 19, tj);  // joining the intra helper
#endif
#if defined(HL_SKIP_INTRA_P)  // timing experiment only (not bit-exact): the P macroblocks' intra fallback skipped
        const double ic = 1.7976931348623157e308;
        (void)hin;
#else
        const double ic = guess_intra(c, hin);
#endif
        HL_PROF_ADD(c, 5, ti);
        if (ic <= best_cost) return;
    }
    else helper_join(c, false);  // not needed: cancelled, or its results are not read
    // finalize (rdo.c:1167-1262)
#if !defined(HL_STEP_PROF) && !defined(HL_I4_PROF) && !defined(HL_NBLK_PROF)
    HL_PROF_T(tfin);
#endif
    const PartDef& bp = kParts[best_part];
    HL_SYNC();
    if (c.tid == 0) {
        S.mad = best_dist;
        S.flags = FL_INTER;
        S.pm0 = PM_L0;
        S.e_type = fam_etype(best_fam);
        S.mb_type = S.e_type - 301;
        S.num_part = bp.num_part;
        S.nb[0].intra = 0;
        S.nb[0].e_type = S.e_type;
        S.nb[0].part_w = bp.part_w;
        S.nb[0].part_h = bp.part_h;
        for (int pi = 0; pi < 4; ++pi) {
            S.nb[0].sub_w[pi] = bp.sub_w;
            S.nb[0].sub_h[pi] = bp.sub_h;
            S.num_sub[pi] = pi < bp.num_part ? bp.num_sub : 1;
            S.sub_type[pi] = pi < bp.num_part ? bp.sub_type : -1;
        }
        for (int pi = 0; pi < bp.num_part; ++pi)
            for (int spi = 0; spi < bp.num_sub; ++spi) {
                S.nb[0].mv[pi][spi][0] = S.best_mv[pi][spi][0];
                S.nb[0].mv[pi][spi][1] = S.best_mv[pi][spi][1];
                S.mvd[pi][spi][0] = (int16_t)(S.best_mv[pi][spi][0] - S.best_mvp[pi][spi][0]);
                S.mvd[pi][spi][1] = (int16_t)(S.best_mv[pi][spi][1] - S.best_mvp[pi][spi][1]);
            }
    }
    HL_SYNC();
    if (pskip) {
        inter_pred_mb(c, false, true);
        for (int t = c.tid; t < 256; t += c.nthr) S.rec[t] = (uint8_t)S.pred[t];
        HL_SYNC();
        if (c.tid == 0) {
            S.e_type = ET_PSKIP;
            S.nb[0].e_type = ET_PSKIP;
            S.flags = FL_INTER | FL_SKIP;
            S.mb_type = ET_PSKIP - 301;
            S.cbp = 0;
            S.cbp_c = 0;
            S.cbp_l4x4 = 0;
            S.cbp_l = 0;
        }
        HL_SYNC();
    }
    else {
        inter_pred_mb(c, false, true);
        reconstruct_inter_luma(c, best_single);
        reconstruct_chroma(c, false);
        if (c.tid == 0) guess_cbp(S);
        HL_SYNC();
    }
    if (!(uni(S.flags) & FL_SKIP) && uni(S.cbp) == 0 && uni(S.e_type) == ET_P16x16 && uni(S.mvd[0][0][0]) == 0 && uni(S.mvd[0][0][1]) == 0) {
        int smv[2];
        skip_mv(S, smv);
        if (uni(smv[0]) == uni(S.best_mvp[0][0][0]) && uni(smv[1]) == uni(S.best_mvp[0][0][1])) {
            HL_SYNC();
            if (c.tid == 0) {
                S.e_type = ET_PSKIP;
                S.nb[0].e_type = ET_PSKIP;
                S.mb_type = ET_PSKIP - 301;
            }
            HL_SYNC();
        }
    }
#if !defined(HL_STEP_PROF) && !defined(HL_I4_PROF) && !defined(HL_NBLK_PROF)
    HL_PROF_ADD(c, 13, tfin);  // the inter finalize (prediction, reconstruction, CBP, skip check)
#endif
}

// --------------------------------------------------------------------------
// Final CAVLC write side effects (mb.c:543-892): TotalCoeff updates and the
// nC of every written block, recorded for the host writer.  Lane 0.
// --------------------------------------------------------------------------
template <typename T>
HD int count_tc(const T* lv, int n)
{
    int k = 0;
    for (int i = 0; i < n; ++i) k += lv[i] != 0;
    return k;
}

HD void final_write(Shared& S)
{
    for (int i = 0; i < 16; ++i) S.nc_luma[i] = 0;
    for (int i = 0; i < 8; ++i) S.nc_cac[i >> 2][i & 3] = 0;
    S.nc_dc = 0;
    if (S.e_type == ET_PSKIP) return;
    if (!(S.cbp_l > 0 || S.cbp_c > 0 || S.pm0 == PM_I16)) return;
    auto inside = [&](int ni) -> int { return S.tc[ni]; };
    if (S.pm0 == PM_I16) {
        S.nc_dc = (int8_t)nc_luma_of(S, 0, inside);
        S.tc[0] = (int8_t)count_tc(S.i16_best_dc, 16);
    }
    for (int i8 = 0; i8 < 4; ++i8)
        for (int i4 = 0; i4 < 4; ++i4)
            if (S.cbp_l & (1 << i8)) {
                const int blk = i8 * 4 + i4;
                S.nc_luma[blk] = (int8_t)nc_luma_of(S, blk, inside);
                S.tc[blk] = (int8_t)(S.pm0 == PM_I16 ? count_tc(S.i16_best_ac[blk], 15) : count_tc(S.luma_level[blk], 16));
            }
    for (int comp = 0; comp < 2; ++comp)
        for (int i4 = 0; i4 < 4; ++i4)
            if (S.cbp_c & 2) {
                int nA, nB;
                bool aA, aB;
                if (i4 & 1) {
                    aA = true;
                    nA = (S.cbp_c & 2) ? S.tcc[comp][i4 - 1] : 0;
                }
                else {
                    aA = S.extCA[comp * 2 + (i4 >> 1)] >= 0;
                    nA = aA ? S.extCA[comp * 2 + (i4 >> 1)] : 0;
                }
                if (i4 & 2) {
                    aB = true;
                    nB = (S.cbp_c & 2) ? S.tcc[comp][i4 - 2] : 0;
                }
                else {
                    aB = S.extCB[comp * 2 + (i4 & 1)] >= 0;
                    nB = aB ? S.extCB[comp * 2 + (i4 & 1)] : 0;
                }
                S.nc_cac[comp][i4] = (int8_t)(aA && aB ? (nA + nB + 1) >> 1 : (aA ? nA : (aB ? nB : 0)));
                S.tcc[comp][i4] = (int8_t)((S.cbp_cac[comp] & (1 << i4)) ? count_tc(S.cac[comp][i4], 15) : 0);
            }
}

// --------------------------------------------------------------------------
// MB end: write recon, persistent state and the record
// --------------------------------------------------------------------------
#if defined(__HIP_DEVICE_COMPILE__)
// count of non-zero entries
template <typename T>
__device__ __forceinline__ int count_nz(const T* v, int n)
{
    int k = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) k += (i < n && v[i] != 0) ? 1 : 0;
    return k;
}

// MB end on the device: final_write's TotalCoeff updates and nC (one lane
// per block: the z-order loop of mb.c:543-892 reads only neighbours that
// precede the block, whose values are final by then), then the new MB
// object and the record assembled in LDS by many lanes at once and stored
// as 16-byte words (the record to the host-mapped copy of a pipelined run
// and / or device memory).  Same results as the host version below.
__device__ __forceinline__ void mb_end(Ctx& c)
{
    HL_FRESH_TID_K(c, 11);
    const FrameArgs& F = c.F;
    Shared& S = c.S;
    const int tid = c.tid;
    const int e_type = S.e_type, pm0 = S.pm0, cbp_l = S.cbp_l, cbp_c = S.cbp_c;
    const bool coded = e_type != ET_PSKIP && (cbp_l > 0 || cbp_c > 0 || pm0 == PM_I16);
    const bool intra = (S.flags & FL_INTRA) != 0;
    // ---- TotalCoeffs after the write
    if (tid < 16) {
        const int blk = tid;
        int t = S.tc[blk];
        if (coded) {
            if (cbp_l & (1 << (blk >> 2))) t = pm0 == PM_I16 ? count_nz(S.i16_best_ac[blk], 15) : count_nz(S.luma_level[blk], 16);
            else if (blk == 0 && pm0 == PM_I16) t = count_nz(S.i16_best_dc, 16);
        }
        S.tcn[blk] = (int8_t)t;
    }
    else if (tid >= 64 && tid < 72) {
        const int comp = (tid - 64) >> 2, i4 = (tid - 64) & 3;
        int t = S.tcc[comp][i4];
        if (coded && (cbp_c & 2)) t = (S.cbp_cac[comp] & (1 << i4)) ? count_nz(S.cac[comp][i4], 15) : 0;
        S.tccn[comp][i4] = (int8_t)t;
    }
    HL_SYNC();
    // ---- nC of every written block
    if (tid < 16) {
        const int blk = tid;
        int nc = 0;
        if (coded && (cbp_l & (1 << (blk >> 2)))) nc = nc_luma_of(S, blk, [&](int ni) -> int { return S.tcn[ni]; });
        S.nc_luma[blk] = (int8_t)nc;
        if (blk == 0) S.nc_dc = (int8_t)(coded && pm0 == PM_I16 ? nc_luma_of(S, 0, [&](int ni) -> int { return S.tcn[ni]; }) : 0);
    }
    else if (tid >= 64 && tid < 72) {
        const int comp = (tid - 64) >> 2, i4 = (tid - 64) & 3;
        int nc = 0;
        if (coded && (cbp_c & 2)) {
            int nA, nB;
            bool aA, aB;
            if (i4 & 1) {
                aA = true;
                nA = S.tccn[comp][i4 - 1];
            }
            else {
                aA = S.extCA[comp * 2 + (i4 >> 1)] >= 0;
                nA = aA ? S.extCA[comp * 2 + (i4 >> 1)] : 0;
            }
            if (i4 & 2) {
                aB = true;
                nB = S.tccn[comp][i4 - 2];
            }
            else {
                aB = S.extCB[comp * 2 + (i4 & 1)] >= 0;
                nB = aB ? S.extCB[comp * 2 + (i4 & 1)] : 0;
            }
            nc = aA && aB ? (nA + nB + 1) >> 1 : (aA ? nA : (aB ? nB : 0));
        }
        S.nc_cac[comp][i4] = (int8_t)nc;
    }
    HL_SYNC();
    // ---- the MB object (over the one loaded at the MB start) and the record, in LDS
    MbState& M = S.nbst[0];
    MbRecord& R = S.recb;
    if (tid < 64) {  // ChromaACLevel of both
        const int32_t w = reinterpret_cast<const int32_t*>(&S.cac[0][0][0])[tid];
        reinterpret_cast<int32_t*>(&M.cac_level[0][0][0])[tid] = w;
        reinterpret_cast<int32_t*>(&R.cac[0][0][0])[tid] = w;
    }
    else if (tid < 192) {  // LumaLevel / Intra16x16ACLevel, two levels per lane
        const int k = (tid - 64) * 2, b = k >> 4, i = k & 15;
        const int l0 = pm0 == PM_I16 ? S.i16_best_ac[b][i] : S.luma_level[b][i];
        const int l1 = pm0 == PM_I16 ? S.i16_best_ac[b][i + 1] : S.luma_level[b][i + 1];
        reinterpret_cast<int32_t*>(&R.luma[0][0])[k >> 1] = (int32_t)((l0 & 0xFFFF) | ((uint32_t)l1 << 16));
    }
    else if (tid < 208) {  // motion: the record's mvd and mv, the object's mv (inter MBs)
        const int k = tid - 192;
        const int32_t mv = reinterpret_cast<const int32_t*>(&S.nb[0].mv[0][0][0])[k];
        reinterpret_cast<int32_t*>(&R.mvd[0][0][0])[k] = reinterpret_cast<const int32_t*>(&S.mvd[0][0][0])[k];
        reinterpret_cast<int32_t*>(&R.mv[0][0][0])[k] = mv;
        if (!intra) reinterpret_cast<int32_t*>(&M.mv[0][0][0])[k] = mv;
    }
    else if (tid < 224) {  // per-block bytes and the I16x16 DC levels
        const int i = tid - 208;
        R.prev_flag[i] = S.prev_flag[i];
        R.rem_mode[i] = S.rem_mode[i];
        R.i4mode[i] = S.i4mode[i];
        R.nc_luma[i] = S.nc_luma[i];
        R.i16dc[i] = S.i16_best_dc[i];
        M.i4mode[i] = S.i4mode[i];
        M.tc_luma[i] = S.tcn[i];
        if (i < 8) {
            R.nc_cac[i >> 2][i & 3] = S.nc_cac[i >> 2][i & 3];
            R.cdc[i >> 2][i & 3] = (int16_t)S.cdc_level[i >> 2][i & 3];
            M.tc_cac[i >> 2][i & 3] = S.tccn[i >> 2][i & 3];
        }
        if (i < 4) {
            R.num_sub[i] = S.num_sub[i];
            R.sub_mb_type[i] = S.sub_type[i];
            if (!intra) {
                M.sub_w[i] = S.nb[0].sub_w[i];
                M.sub_h[i] = S.nb[0].sub_h[i];
            }
        }
    }
    else if (tid == 224) {  // the scalar fields
        M.e_type = e_type;
        M.flags = S.flags;
        M.pm0 = pm0;
        M.cbp_l = cbp_l;
        M.cbp_c = cbp_c;
        M.cbp_l4x4 = S.cbp_l4x4;
        if (!intra) {
            M.num_part = S.num_part;
            M.part_w = S.nb[0].part_w;
            M.part_h = S.nb[0].part_h;
        }
        R.e_type = e_type;
        R.mb_type = S.mb_type;
        R.flags = S.flags;
        R.pm0 = pm0;
        R.cbp = S.cbp;
        R.cbp_l = cbp_l;
        R.cbp_c = cbp_c;
        R.cbp_l4x4 = S.cbp_l4x4;
        for (int i = 0; i < 2; ++i) {
            R.cbp_cdc[i] = S.cbp_cdc[i];
            R.cbp_cac[i] = S.cbp_cac[i];
        }
        R.num_part = S.num_part;
        R.chroma_mode = S.chroma_mode;
        R.i16mode = S.i16mode;
        R.nc_dc = S.nc_dc;
        R.pad0[0] = R.pad0[1] = R.pad0[2] = 0;
        R.mad = S.mad;
        R.pad1 = 0;
        const auto ch = gmem(F.chain) + c.addr;
        ch->s_out = c.chain;
        ch->dep = c.dep;
        ch->fresh = c.fresh;
        ch->spec = c.spec;
    }
    HL_SYNC();
    // ---- 16-byte stores: the reconstruction, the MB object, the record
    constexpr int kSW = (int)(sizeof(MbState) / 16), kRW = (int)(sizeof(MbRecord) / 16);
    static_assert(sizeof(MbRecord) % 16 == 0, "MbRecord in whole 16-byte words");
    if (tid < 16)
        *gmem(reinterpret_cast<uint4*>(F.cur[0] + (size_t)(c.yL + tid) * F.W + c.xL)) = reinterpret_cast<const uint4*>(S.rec)[tid];
    else if (tid >= 64 && tid < 64 + kSW)
        gmem(reinterpret_cast<uint4*>(F.st + c.addr))[tid - 64] = reinterpret_cast<const uint4*>(&M)[tid - 64];
    else if (tid >= 128 && tid < 128 + kRW) {
        const uint4 w = reinterpret_cast<const uint4*>(&R)[tid - 128];
        if (F.hrec) gmem(reinterpret_cast<uint4*>(F.hrec + c.addr))[tid - 128] = w;
        if (F.rec_dev) gmem(reinterpret_cast<uint4*>(F.rec + c.addr))[tid - 128] = w;
    }
    HL_SYNC();
}
#else
HD void mb_end(Ctx& c)
{
    const FrameArgs& F = c.F;
    Shared& S = c.S;
    for (int t = c.tid; t < 256; t += c.nthr) F.cur[0][(c.yL + (t >> 4)) * F.W + c.xL + (t & 15)] = S.rec[t];
    if (c.tid == 0) final_write(S);
    HL_SYNC();
    MbState& M = F.st[c.addr];
    MbRecord& R = F.rec[c.addr];
    for (int t = c.tid; t < 128; t += c.nthr) {
        M.cac_level[t >> 6][(t >> 4) & 3][t & 15] = S.cac[t >> 6][(t >> 4) & 3][t & 15];
        R.cac[t >> 6][(t >> 4) & 3][t & 15] = S.cac[t >> 6][(t >> 4) & 3][t & 15];
    }
    for (int t = c.tid; t < 256; t += c.nthr) {
        const int b = t >> 4, i = t & 15;
        R.luma[b][i] = (int16_t)(S.pm0 == PM_I16 ? S.i16_best_ac[b][i] : S.luma_level[b][i]);
    }
    if (c.tid == 0) {
        M.e_type = S.e_type;
        M.flags = S.flags;
        M.pm0 = S.pm0;
        M.cbp_l = S.cbp_l;
        M.cbp_c = S.cbp_c;
        M.cbp_l4x4 = S.cbp_l4x4;
        const bool intra = (S.flags & FL_INTRA) != 0;
        if (!intra) {
            M.num_part = S.num_part;
            M.part_w = S.nb[0].part_w;
            M.part_h = S.nb[0].part_h;
            for (int i = 0; i < 4; ++i) {
                M.sub_w[i] = S.nb[0].sub_w[i];
                M.sub_h[i] = S.nb[0].sub_h[i];
            }
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) {
                    M.mv[i][j][0] = S.nb[0].mv[i][j][0];
                    M.mv[i][j][1] = S.nb[0].mv[i][j][1];
                }
        }
        for (int i = 0; i < 16; ++i) {
            M.i4mode[i] = S.i4mode[i];
            M.tc_luma[i] = S.tc[i];
        }
        for (int i = 0; i < 8; ++i) M.tc_cac[i >> 2][i & 3] = S.tcc[i >> 2][i & 3];
        R.e_type = S.e_type;
        R.mb_type = S.mb_type;
        R.flags = S.flags;
        R.pm0 = S.pm0;
        R.cbp = S.cbp;
        R.cbp_l = S.cbp_l;
        R.cbp_c = S.cbp_c;
        R.cbp_l4x4 = S.cbp_l4x4;
        for (int i = 0; i < 2; ++i) {
            R.cbp_cdc[i] = S.cbp_cdc[i];
            R.cbp_cac[i] = S.cbp_cac[i];
        }
        R.num_part = S.num_part;
        for (int i = 0; i < 4; ++i) {
            R.num_sub[i] = S.num_sub[i];
            R.sub_mb_type[i] = S.sub_type[i];
        }
        R.chroma_mode = S.chroma_mode;
        R.i16mode = S.i16mode;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                R.mvd[i][j][0] = S.mvd[i][j][0];
                R.mvd[i][j][1] = S.mvd[i][j][1];
                R.mv[i][j][0] = S.nb[0].mv[i][j][0];
                R.mv[i][j][1] = S.nb[0].mv[i][j][1];
            }
        for (int i = 0; i < 16; ++i) {
            R.prev_flag[i] = S.prev_flag[i];
            R.rem_mode[i] = S.rem_mode[i];
            R.i4mode[i] = S.i4mode[i];
            R.nc_luma[i] = S.nc_luma[i];
            R.i16dc[i] = S.i16_best_dc[i];
        }
        for (int i = 0; i < 8; ++i) {
            R.nc_cac[i >> 2][i & 3] = S.nc_cac[i >> 2][i & 3];
            R.cdc[i >> 2][i & 3] = (int16_t)S.cdc_level[i >> 2][i & 3];
        }
        R.nc_dc = S.nc_dc;
        R.mad = S.mad;
        MbChain& ch = F.chain[c.addr];
        ch.s_out = c.chain;
        ch.dep = c.dep;
        ch.fresh = c.fresh;
        ch.spec = c.spec;
    }
    HL_SYNC();
}
#endif

#if defined(HL_EMU_BUILD) && !defined(__HIP_DEVICE_COMPILE__)
extern int g_emu_bad_guess;
extern int g_emu_bad_guess3;
#endif
// The intra helper task of P macroblock addr (pipelined runs): the parts of
// its intra fallback that do not depend on its inter search, into out --
// every Intra16x16 mode's statistics and results (i16_heavy), and the
// Intra4x4 decision under the live state the Intra16x16 trials leave when
// the inter search left this address's previous TotalCoeffs and the entry
// value s_in of rdo.Single_ctr (i16_light with spec, guess_i4).  The MB keeps
// that decision only if i4_verify holds.  Reads what the MB's mb_begin reads
// (all final when the MB is ready) and writes only out.
#if defined(HL_HELPER_NOINLINE)
__host__ __device__ __attribute__((noinline)) void intra_helper(
#else
HD void intra_helper(
#endif
    const FrameArgs& F, Shared& S, int addr, int tid, int nthr, int s_in, IntraSpec* out)
{
    Ctx c{F, S, tid, nthr, addr, addr % F.mbw, addr / F.mbw, (addr % F.mbw) * 16, (addr / F.mbw) * 16, s_in, 0, 0};
#if defined(__HIP_DEVICE_COMPILE__)
    if (tid < 16) S.lk[tid] = make_lanek(tid, F.qp, F.qpc);
    c.Q = make_laneq(tid, F.qp);
#endif
    mb_begin(c);
#if defined(HL_EMU_BUILD) && !defined(__HIP_DEVICE_COMPILE__)
    if (g_emu_bad_guess)  // tests: a wrong guess of the live TotalCoeffs, so that i4_verify must reject
        for (int i = 0; i < 16; ++i) S.tc[i] = (int8_t)((i * 5 + addr) % 11);
#endif
    i16_heavy(c);
    double c16, c4;
    int cbp16, d16, m16, cbp4, d4;
    i16_light(c, c16, cbp16, d16, m16, true);
    guess_i4(c, c4, cbp4, d4);
#if defined(__HIP_DEVICE_COMPILE__)
    if (tid < 16) S.ih.i4_mode[tid] = S.i4mode[tid];
    if (tid == 0) S.ih.i4_valid = 1;
    HL_SYNC();
    // 16-byte stores: the head, the modes' bulk results, the Intra4x4 results
    constexpr int kHW = (int)(sizeof(IntraHead) / 16);
    const auto o = gmem(reinterpret_cast<uint4*>(out));
    static_assert(offsetof(IntraSpec, i4_lv) == sizeof(IntraHead) + 16 * (64 + 64 + 128 + 8 + 16), "IntraSpec layout");
    for (int k = tid; k < kHW + 64 + 64 + 128 + 8 + 16; k += nthr) {
        uint4 v;
        if (k < kHW) v = reinterpret_cast<const uint4*>(&S.ih)[k];
        else if (k < kHW + 64) v = reinterpret_cast<const uint4*>(S.ih_rec)[k - kHW];
        else if (k < kHW + 128) v = reinterpret_cast<const uint4*>(S.ih_pred)[k - kHW - 64];
        else if (k < kHW + 256) v = reinterpret_cast<const uint4*>(S.ih_ac)[k - kHW - 128];
        else if (k < kHW + 264) v = reinterpret_cast<const uint4*>(S.ih_dcl)[k - kHW - 256];
        else v = reinterpret_cast<const uint4*>(S.rec)[k - kHW - 264];
        o[k] = v;  // IntraSpec: h, rec, pred, ac, dcl, i4_rec in this order
    }
    if (tid < 128) {  // LumaLevel, two levels per lane
        const uint32_t w = (uint32_t)(S.luma_level[tid >> 3][(tid & 7) * 2] & 0xFFFF) | ((uint32_t)S.luma_level[tid >> 3][(tid & 7) * 2 + 1] << 16);
        gmem(reinterpret_cast<uint32_t*>(&out->i4_lv[0][0]))[tid] = w;
    }
#else
    for (int i = 0; i < 16; ++i) S.ih.i4_mode[i] = S.i4mode[i];
    S.ih.i4_valid = 1;
    out->h = S.ih;
    memcpy(out->rec, S.ih_rec, sizeof(out->rec));
    memcpy(out->pred, S.ih_pred, sizeof(out->pred));
    memcpy(out->ac, S.ih_ac, sizeof(out->ac));
    memcpy(out->dcl, S.ih_dcl, sizeof(out->dcl));
    memcpy(out->i4_rec, S.rec, sizeof(out->i4_rec));
    for (int t = 0; t < 256; ++t) out->i4_lv[t >> 4][t & 15] = (int16_t)S.luma_level[t >> 4][t & 15];
#endif
}

// One macroblock, start to end.  s_in = rdo.Single_ctr on entry (spec_in = 1
// while it is a row-start speculation); (gx, gy) = reference region already
// known complete (pipelined runs; see reach_wait).
// f3out: the macroblock's helper task of 8x8-family partitioning hj instead (guess_inter)
HD void encode_mb(const FrameArgs& F, Shared& S, int addr, int tid, int nthr, int s_in, int gx = 1 << 20, int gy = 1 << 20,
               int spec_in = 1, Fam3Out* f3out = nullptr, int hj = 3)
{
    Ctx c{F, S, tid, nthr, addr, addr % F.mbw, addr / F.mbw, (addr % F.mbw) * 16, (addr / F.mbw) * 16, s_in, 0, 0};
    c.gx = gx;
    c.gy = gy;
    c.spec = spec_in;
#if defined(__HIP_DEVICE_COMPILE__)
    // (first read after mb_begin's barriers)
    if (tid < 16) S.lk[tid] = make_lanek(tid, F.qp, F.qpc);
    c.Q = make_laneq(tid, F.qp);
#endif
    if (tid == 0 && !f3out) gmem(F.chain + addr)->s_in = s_in;
#if defined(__HIP_DEVICE_COMPILE__) && defined(HL_PROFILE) && defined(HL_BAR_PROF)
    if ((tid & 63) == 0) g_bar_acc[tid >> 6][0] = g_bar_acc[tid >> 6][1] = 0;
#if HL_BAR_PROF >= 2
    for (int k = tid; k < kBarSites; k += nthr) {
        g_bar_site[k] = 0;
        g_bar_cnt[k] = 0;
    }
    __syncthreads();
#endif
#endif
    HL_PROF_T(t0);
    mb_begin(c);
    HL_PROF_ADD(c, 6, t0);
    if (f3out) {
        // the entry guess: one coefficient in every block.  The live values
        // at the 8x8 family are those the 16x16 / 16x8 / 8x16 searches of
        // this picture left, mostly 1 or 2; the address's values from the
        // previous picture (an intra MB's after an I picture) miss their nC
        // classes far more often (fam3_guess_stats.py, emulator, 1088p bench
        // stream: rejections 23.9 -> 14.3 % over its first three P pictures)
        for (int t = tid; t < 16; t += nthr) S.tc[t] = 1;
        HL_SYNC();
#if defined(HL_EMU_BUILD) && !defined(__HIP_DEVICE_COMPILE__)
        if (g_emu_bad_guess3)  // tests: a wrong guess of the entry values, so that f3_verify must reject
            for (int i = 0; i < 16; ++i) S.tc[i] = (int8_t)((i * 5 + addr) % 11);
#endif
        if (HL_FAM3) guess_inter(c, f3out, hj);
        return;
    }
    if (F.is_intra) guess_intra(c);
    else guess_inter(c);
    HL_PROF_T(t1);
    mb_end(c);
    HL_PROF_ADD(c, 7, t1);
    HL_PROF_ADD(c, 8, t0);
#if defined(HL_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
#if defined(HL_BAR_PROF)
    // slot 14: barrier cycles summed over the waves (count: barriers of wave
    // 0); slot 15: the most waiting wave's, slot 18: the least waiting wave's
    __syncthreads();
    if (tid == 0) {
        unsigned long long sum = 0, mx = 0, mn = ~0ull;
        for (int w = 0; w < nthr / 64; ++w) {
            sum += g_bar_acc[w][0];
            mx = max(mx, g_bar_acc[w][0]);
            mn = min(mn, g_bar_acc[w][0]);
        }
        c.pacc[14] = sum;
        c.pcnt[14] = (int)g_bar_acc[0][1];
        c.pacc[15] = mx;
        c.pcnt[15] = 1;
        c.pacc[18] = mn;
        c.pcnt[18] = 1;
    }
#if HL_BAR_PROF >= 2
    if (F.prof) {
        unsigned long long* site = F.prof + 64 + 4 * F.mbw * F.mbh;
        for (int k = tid; k < kBarSites; k += nthr)
            if (g_bar_cnt[k]) {
                atomicAdd(site + 2 * k, g_bar_site[k]);
                atomicAdd(site + 2 * k + 1, (unsigned long long)g_bar_cnt[k]);
            }
    }
#endif
#endif
    if (tid == 0 && F.prof) {
        for (int i = 0; i < kProfSlots; ++i) {
            atomicAdd(&F.prof[2 * i], c.pacc[i]);
            atomicAdd(&F.prof[2 * i + 1], (unsigned long long)c.pcnt[i]);
        }
        F.prof[64 + addr] = c.pacc[8];
    }
#endif
}

}  // namespace hl
