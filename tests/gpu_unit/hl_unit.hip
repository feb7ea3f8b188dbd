// hl_unit.hip -- TEST INFRASTRUCTURE.  GPU unit kernels that diff the
// product's cooperative 16-lane 4x4 pipeline (hartallo_amd/csrc/hl_coop.h)
// against the scalar primitives (hl_prims.h) on the same random blocks, so a
// parity failure of the full encoder can be narrowed to one primitive.
#include <hip/hip_runtime.h>
#include <string.h>

#include "../../hartallo_amd/csrc/hl_coop.h"
#include "../../hartallo_amd/csrc/hl_quad.h"
#include "../../hartallo_amd/csrc/hl_filters.h"

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
