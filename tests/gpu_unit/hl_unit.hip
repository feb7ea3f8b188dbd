// hl_unit.hip -- TEST INFRASTRUCTURE.  GPU unit kernels that diff the
// product's cooperative 16-lane 4x4 pipeline (hartallo_amd/csrc/hl_coop.h)
// against the scalar primitives (hl_prims.h) on the same random blocks, so a
// parity failure of the full encoder can be narrowed to one primitive.
#include <hip/hip_runtime.h>
#include <string.h>

#include "../../hartallo_amd/csrc/hl_coop.h"
#include "../../hartallo_amd/csrc/hl_quad.h"
#include "../../hartallo_amd/csrc/hl_filters.h"
#include "../../hartallo_amd/csrc/hl_mbcore.h"
#include "../../hartallo_amd/csrc/hl_cavlc.h"

using namespace hl;

struct UnitOut {
    int32_t tc, t1, rest, sctr, dist;
    int32_t q[16], rec[16];
};

// mode 0: inter 4x4 (f = 2^qbits/6), 1: intra 4x4 (/3), 2: AC list (scan 1..15, intra rounding)
__global__ __launch_bounds__(64) void k_unit_scalar(const uint8_t* src, const uint8_t* pred, int n, int qp, int mode, UnitOut* out)
{
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= n) return;
    const uint8_t* s = src + 16 * b;
    const uint8_t* p = pred + 16 * b;
    int res[16], w[16], q[16], lv[16], r[16];
    for (int i = 0; i < 16; ++i) res[i] = (int)s[i] - p[i];
    fwd4x4(res, w);
    quant4x4(qp, mode != 0, w, q);
    if (mode == 2) {
        for (int i = 1; i < 16; ++i) lv[i - 1] = q[kZigzag[i]];
        lv[15] = 0;
    }
    else
        for (int i = 0; i < 16; ++i) lv[i] = q[kZigzag[i]];
    bool lz = true;
    for (int i = 0; i < 16; ++i) lz = lz && lv[i] == 0;
    CavlcStat st = {0, 0, 0, -1};
    if (!lz) st = cavlc_stat(lv, 16, 15, false);
    dequant_idct(qp, q, false, r);
    int dist = 0;
    UnitOut& o = out[b];
    for (int i = 0; i < 16; ++i) {
        const int v = clip255(p[i] + r[i]);
        dist += iabs((int)s[i] - v);
        o.q[i] = q[i];
        o.rec[i] = v;
    }
    o.tc = st.tc;
    o.t1 = st.t1;
    o.rest = st.rest;
    o.sctr = st.sctr;
    o.dist = dist;
}

__global__ __launch_bounds__(256) void k_unit_coop(const uint8_t* src, const uint8_t* pred, int n, int qp, int mode, UnitOut* out)
{
    __shared__ CoopTables T;
    __shared__ int lvs[16][16];
    coop_tables_init(T, threadIdx.x, 256);
    __syncthreads();
    const LaneK K = make_lanek(threadIdx.x, qp, qp);
    const int grp = threadIdx.x >> 4;
    const int b = blockIdx.x * 16 + grp;
    if (b >= n) return;  // whole rows
    const int sv = src[16 * b + K.p], pv = pred[16 * b + K.p];
    const int w = coop_fwd(K, sv - pv);
    const int qbits = 15 + qp / 6;
    const int f = (1 << qbits) / (mode != 0 ? 3 : 6);
    const int q = coop_quant(w, K.mf, qbits, f);
    const int li = mode == 2 ? K.s - 1 : K.s;
    const CoopStat st = coop_cavlc(T, q, li, lvs[grp]);
    const int r = coop_idct(K, coop_dequant(q, K.ls, qp));
    const int v = clip255(pv + r);
    const int dist = row_sum(iabs(sv - v));
    UnitOut& o = out[b];
    o.q[K.p] = q;
    o.rec[K.p] = v;
    if (K.p == 0) {
        o.tc = st.tc;
        o.t1 = st.t1;
        o.rest = st.rest;
        o.sctr = st.sctr;
        o.dist = dist;
    }
}

// the quad pipeline (hl_quad.h): one 4-lane quad per block, lane r = row r
__global__ __launch_bounds__(256) void k_unit_quad(const uint8_t* src, const uint8_t* pred, int n, int qp, int mode, UnitOut* out)
{
    __shared__ CoopTables T;
    __shared__ int lvs[64][16];
    coop_tables_init(T, threadIdx.x, 256);
    __syncthreads();
    const LaneQ Q = make_laneq(threadIdx.x, qp);
    const int qg = threadIdx.x >> 2;
    const int b = blockIdx.x * 64 + qg;
    if (b >= n) return;  // whole quads
    int x[4], y[4], q[4], r[4], sv[4], pv[4];
    for (int c = 0; c < 4; ++c) {
        sv[c] = src[16 * b + 4 * Q.r + c];
        pv[c] = pred[16 * b + 4 * Q.r + c];
        x[c] = sv[c] - pv[c];
    }
    quad_fwd(Q, x, y);
    const int qbits = 15 + qp / 6;
    const int f = (1 << qbits) / (mode != 0 ? 3 : 6);
    for (int c = 0; c < 4; ++c) q[c] = quad_q1(y[c], (c & 1) ? Q.mfO : Q.mfE, qbits, f);
    const CoopStat st = quad_cavlc(T, Q, q, mode == 2 ? 1 : 0, lvs[qg]);
    quad_idct(Q, q, qp, r);
    int d = 0;
    UnitOut& o = out[b];
    for (int c = 0; c < 4; ++c) {
        const int v = clip255(pv[c] + r[c]);
        d += iabs(sv[c] - v);
        o.q[4 * quad_coef_row(Q.r) + c] = q[c];
        o.rec[4 * Q.r + c] = v;
    }
    const int dist = quad_sum(d);
    if (Q.r == 0) {
        o.tc = st.tc;
        o.t1 = st.t1;
        o.rest = st.rest;
        o.sctr = st.sctr;
        o.dist = dist;
    }
}

extern "C" int unit_run(const uint8_t* h_src, const uint8_t* h_pred, int n, int qp, int mode, int coop, UnitOut* h_out)
{
    uint8_t *d_src = nullptr, *d_pred = nullptr;
    UnitOut* d_out = nullptr;
    if (hipMalloc(&d_src, 16 * (size_t)n) || hipMalloc(&d_pred, 16 * (size_t)n) || hipMalloc(&d_out, sizeof(UnitOut) * (size_t)n)) return -1;
    (void)hipMemcpy(d_src, h_src, 16 * (size_t)n, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_pred, h_pred, 16 * (size_t)n, hipMemcpyHostToDevice);
    (void)hipMemset(d_out, 0xFF, sizeof(UnitOut) * (size_t)n);
    if (coop == 2) k_unit_quad<<<(n + 63) / 64, 256>>>(d_src, d_pred, n, qp, mode, d_out);
    else if (coop) k_unit_coop<<<(n + 15) / 16, 256>>>(d_src, d_pred, n, qp, mode, d_out);
    else k_unit_scalar<<<(n + 63) / 64, 64>>>(d_src, d_pred, n, qp, mode, d_out);
    const hipError_t e = hipDeviceSynchronize();
    (void)hipMemcpy(h_out, d_out, sizeof(UnitOut) * (size_t)n, hipMemcpyDeviceToHost);
    (void)hipFree(d_src);
    (void)hipFree(d_pred);
    (void)hipFree(d_out);
    return e == hipSuccess ? 0 : -2;
}

extern "C" int unit_sizeof_out() { return (int)sizeof(UnitOut); }

// The product's quarter-pel plane kernel (k_planes, hl_filters.h) and the
// per-sample definition it implements (qpel_plane_sample, run on the host)
// on the same picture: out_gpu / out_host hold the four padded planes, each
// pstride x (H + 2 kPad) with pstride = (W + 2 kPad + 63) & ~63.
extern "C" int unit_planes(const uint8_t* h_ref, int W, int H, uint8_t* out_gpu, uint8_t* out_host)
{
    const int pstride = (W + 2 * kPad + 63) & ~63, ph = H + 2 * kPad;
    const size_t plsz = (size_t)pstride * ph;
    uint8_t *d_ref = nullptr, *d_pl = nullptr;
    if (hipMalloc(&d_ref, (size_t)W * H) || hipMalloc(&d_pl, 4 * plsz)) return 1;
    if (hipMemcpy(d_ref, h_ref, (size_t)W * H, hipMemcpyHostToDevice) || hipMemset(d_pl, 0, 4 * plsz)) return 2;
    const dim3 grid((W + 2 * kPad + kPlTileW - 1) / kPlTileW, (H + 2 * kPad + kPlTileH - 1) / kPlTileH);
    k_planes<<<grid, 256>>>(d_ref, W, H, d_pl, pstride, (int)plsz);
    if (hipDeviceSynchronize() || hipMemcpy(out_gpu, d_pl, 4 * plsz, hipMemcpyDeviceToHost)) return 3;
    (void)hipFree(d_ref);
    (void)hipFree(d_pl);
    memset(out_host, 0, 4 * plsz);
    for (int p = 0; p < 4; ++p)
        for (int y = 0; y < ph; ++y)
            for (int x = 0; x < W + 2 * kPad; ++x) out_host[p * plsz + (size_t)y * pstride + x] = qpel_plane_sample(h_ref, W, H, p, x - kPad, y - kPad);
    return 0;
}

// ---------------------------------------------------------------------------
// Op-level parity against the reference's own kernels (tests/test_gpu_ops.py,
// tests/golden/ops_*.npz made by tests/golden/make_op_golden.py through
// oracle/_ref/ref_ops)
// ---------------------------------------------------------------------------

// CAVLC residual blocks from scan-order level lists.
//   cavlc_block (hl_cavlc.h, the GPU slice writer) -> the bits themselves;
//   quad_cavlc (hl_quad.h, the candidate evaluation's and Intra16x16's rate)
//   for kinds 0 / 4 -> rest + the coeff_token length of the nC class (tc >
//   0; -1 else)
struct UnitCavlcIn {
    int32_t kind, nC, level[16];  // kind 0 luma 4x4, 1 Intra16x16 AC, 2 chroma DC, 3 chroma AC, 4 AC as the RDO prices it
};
struct UnitCavlcOut {
    int32_t nbits, quad_bits, tc, pad;
    uint32_t words[24];
};

__global__ __launch_bounds__(64) void k_unit_cavlc_block(const UnitCavlcIn* in, int n, UnitCavlcOut* out)
{
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const UnitCavlcIn& x = in[i];
    const int maxn = (x.kind == 0 || x.kind == 4) ? 16 : (x.kind == 2 ? 4 : 15);
    BitOr bw{out[i].words, 0};
    cavlc_block(bw, x.level, maxn - 1, maxn, x.nC);
    out[i].nbits = (int)bw.pos;
}

__global__ __launch_bounds__(256) void k_unit_cavlc_quad(const UnitCavlcIn* in, int n, UnitCavlcOut* out)
{
    __shared__ CoopTables T;
    __shared__ int lvs[64][16];
    coop_tables_init(T, threadIdx.x, 256);
    __syncthreads();
    const LaneQ Q = make_laneq(threadIdx.x, 28);  // (the scan word does not depend on the QP)
    const int qg = threadIdx.x >> 2;
    const int b = blockIdx.x * 64 + qg;
    if (b >= n) return;  // whole quads
    const UnitCavlcIn& x = in[b];
    const int ac = (x.kind == 1 || x.kind == 4) ? 1 : 0;
    int L[4];
    for (int c = 0; c < 4; ++c) {  // this lane's coefficient row, raster: the level at its scan index
        const int li = (int)((Q.zz >> (4 * c)) & 15) - ac;
        L[c] = li >= 0 ? x.level[li] : 0;
    }
    const CoopStat st = quad_cavlc(T, Q, L, ac, lvs[qg]);
    if (Q.r == 0 && (x.kind == 0 || x.kind == 4)) {  // the RDO's 16-entry lists (rdo.c:1676, 1981)
        const int cls = x.nC < 2 ? 0 : (x.nC < 4 ? 1 : (x.nC < 8 ? 2 : 3));
        out[b].quad_bits = st.tc ? st.rest + (int)((T.tok3[st.t1][st.tc] >> (5 * cls)) & 31) : -1;
        out[b].tc = st.tc;
    }
}

extern "C" int unit_cavlc(const UnitCavlcIn* h_in, int n, UnitCavlcOut* h_out)
{
    UnitCavlcIn* d_in = nullptr;
    UnitCavlcOut* d_out = nullptr;
    if (hipMalloc(&d_in, sizeof(UnitCavlcIn) * (size_t)n) || hipMalloc(&d_out, sizeof(UnitCavlcOut) * (size_t)n)) return -1;
    if (hipMemcpy(d_in, h_in, sizeof(UnitCavlcIn) * (size_t)n, hipMemcpyHostToDevice) ||
        hipMemset(d_out, 0, sizeof(UnitCavlcOut) * (size_t)n))
        return -2;
    k_unit_cavlc_block<<<(n + 63) / 64, 64>>>(d_in, n, d_out);
    k_unit_cavlc_quad<<<(n + 63) / 64, 256>>>(d_in, n, d_out);
    const hipError_t e = hipDeviceSynchronize();
    (void)hipMemcpy(h_out, d_out, sizeof(UnitCavlcOut) * (size_t)n, hipMemcpyDeviceToHost);
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return e == hipSuccess ? 0 : -3;
}
extern "C" int unit_sizeof_cavlc_out() { return (int)sizeof(UnitCavlcOut); }

// 16x16 luma inter predictions as the macroblock's finalize computes them
// (hl_mbcore.h inter_pred_mb: the partition origin clamped to [-17, W + 17]
// like interpol.c, the quarter-pel phase's two samples of the k_planes
// planes via qpel_entry (kQpelTab), their rounded average); one 4-lane quad
// per (record, 4x4 block), lane r = row r.
struct UnitPredIn {
    int32_t mbx, mby, mvx, mvy;
};
__global__ __launch_bounds__(256) void k_unit_lpred(const uint8_t* pl, int W, int H, int pstride, int plsz, const UnitPredIn* in, int n,
                                                    uint8_t* out)
{
    const int q = (blockIdx.x * 256 + threadIdx.x) >> 2, r = threadIdx.x & 3;
    const int i = q >> 4, t = q & 15;
    if (i >= n) return;
    const UnitPredIn x = in[i];
    const int bx = (t & 3) * 4, by = (t >> 2) * 4;
    const int X = clip3(-17, W + 17, 16 * x.mbx + (x.mvx >> 2)) + kPad + bx;
    const int Y = clip3(-17, H + 17, 16 * x.mby + (x.mvy >> 2)) + kPad + by + r;
    const uint32_t e = qpel_entry(((x.mvy & 3) << 2) | (x.mvx & 3));
    const int o1 = (int)(e & 3) * plsz + (Y + (int)((e >> 3) & 1)) * pstride + X + (int)((e >> 2) & 1);
    const int o2 = (e & 16) ? (int)((e >> 5) & 3) * plsz + (Y + (int)((e >> 8) & 1)) * pstride + X + (int)((e >> 7) & 1) : o1;
#if defined(__HIP_DEVICE_COMPILE__)
    const auto base = gmem(pl);
    const uint32_t pr = avg_u8x4(ld_u8x4(base, o1), ld_u8x4(base, o2));
    *reinterpret_cast<uint32_t*>(out + 256 * (size_t)i + (by + r) * 16 + bx) = pr;
#endif
}

extern "C" int unit_lpred(const uint8_t* h_ref, int W, int H, const UnitPredIn* h_in, int n, uint8_t* h_out)
{
    const int pstride = (W + 2 * kPad + 63) & ~63, ph = H + 2 * kPad;
    const size_t plsz = (size_t)pstride * ph;
    uint8_t *d_ref = nullptr, *d_pl = nullptr, *d_out = nullptr;
    UnitPredIn* d_in = nullptr;
    // (+64: the 4-byte loads read whole aligned words past the last plane's end)
    if (hipMalloc(&d_ref, (size_t)W * H) || hipMalloc(&d_pl, 4 * plsz + 64) || hipMalloc(&d_in, sizeof(UnitPredIn) * (size_t)n) ||
        hipMalloc(&d_out, 256 * (size_t)n))
        return 1;
    for (int i = 0; i < n; ++i)  // the kernel's addressing assumes the records' blocks inside the padded planes
        if (h_in[i].mbx < 0 || h_in[i].mby < 0 || 16 * h_in[i].mbx >= W || 16 * h_in[i].mby >= H) return 2;
    if (hipMemcpy(d_ref, h_ref, (size_t)W * H, hipMemcpyHostToDevice) || hipMemset(d_pl, 0, 4 * plsz + 64) ||
        hipMemcpy(d_in, h_in, sizeof(UnitPredIn) * (size_t)n, hipMemcpyHostToDevice))
        return 3;
    const dim3 grid((W + 2 * kPad + kPlTileW - 1) / kPlTileW, (H + 2 * kPad + kPlTileH - 1) / kPlTileH);
    k_planes<<<grid, 256>>>(d_ref, W, H, d_pl, pstride, (int)plsz);
    k_unit_lpred<<<(n * 64 + 255) / 256, 256>>>(d_pl, W, H, pstride, (int)plsz, d_in, n, d_out);
    const hipError_t e = hipDeviceSynchronize();
    (void)hipMemcpy(h_out, d_out, 256 * (size_t)n, hipMemcpyDeviceToHost);
    (void)hipFree(d_ref);
    (void)hipFree(d_pl);
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return e == hipSuccess ? 0 : 4;
}

// Deblocking of 8 lines across one edge (p[k][l] = pk of line l) with the
// product's line filter (hl_filters.h deblock_line, kAlpha / kBeta / kTc0),
// one lane per line.
struct UnitDbIn {
    uint8_t p[4][8], q[4][8];
    int32_t bS, indexA, chroma;
};
struct UnitDbOut {
    uint8_t p[3][8], q[3][8];
};
__global__ __launch_bounds__(64) void k_unit_dblk(const UnitDbIn* in, int n, UnitDbOut* out)
{
    const int g = blockIdx.x * 64 + threadIdx.x;
    const int i = g >> 3, l = g & 7;
    if (i >= n) return;
    const UnitDbIn& x = in[i];
    uint8_t s[8];
    for (int k = 0; k < 4; ++k) {
        s[3 - k] = x.p[k][l];
        s[4 + k] = x.q[k][l];
    }
    const int ia = x.indexA;
    deblock_line(s + 4, 1, x.bS, x.chroma != 0, ia, kAlpha[ia], kBeta[ia]);
    for (int k = 0; k < 3; ++k) {
        out[i].p[k][l] = s[3 - k];
        out[i].q[k][l] = s[4 + k];
    }
}

extern "C" int unit_dblk(const UnitDbIn* h_in, int n, UnitDbOut* h_out)
{
    UnitDbIn* d_in = nullptr;
    UnitDbOut* d_out = nullptr;
    for (int i = 0; i < n; ++i)  // table indices the kernel reads
        if (h_in[i].indexA < 0 || h_in[i].indexA > 51 || h_in[i].bS < 1 || h_in[i].bS > 4) return -4;
    if (hipMalloc(&d_in, sizeof(UnitDbIn) * (size_t)n) || hipMalloc(&d_out, sizeof(UnitDbOut) * (size_t)n)) return -1;
    if (hipMemcpy(d_in, h_in, sizeof(UnitDbIn) * (size_t)n, hipMemcpyHostToDevice)) return -2;
    k_unit_dblk<<<(n * 8 + 63) / 64, 64>>>(d_in, n, d_out);
    const hipError_t e = hipDeviceSynchronize();
    (void)hipMemcpy(h_out, d_out, sizeof(UnitDbOut) * (size_t)n, hipMemcpyDeviceToHost);
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return e == hipSuccess ? 0 : -3;
}
