// fetch_calib.hip -- development tool: calibrates rocprofv3's FETCH_SIZE on
// gfx950 for the access pattern of the macroblock search's prediction loads
// (MI355X_MICROARCH.md: FETCH_SIZE reads exactly half the bytes of a wide
// streaming read; "other access widths are uncalibrated").
//
//   hipcc --offload-arch=gfx950 -O3 -o build/fetch_calib tools/fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d <dir> -o run --output-format csv -- build/fetch_calib
//
// Three kernels over cold buffers larger than the 256 MiB Infinity Cache (a
// 768 MiB flush stream, also k_stream, runs before each: dispatches 1, 3, 5
// are flushes), so that every line they touch comes from HBM exactly once:
//   k_stream   16 bytes per lane, consecutive (the guide's reference case)
//   k_gather   the eval's prediction loads (hl_mbcore.h eval_candidates /
//              hl_quad.h ld_u8x4): per 4-lane quad, lane r reads row Y + r
//              of a 2048-byte-stride plane at column X (any alignment) as two
//              aligned dwords, twice (the two planes of a quarter-pel phase);
//              every quad at its own lines
//   k_bytes    one dword per lane at a 128-byte stride (one line per lane)
//   k_wstream / k_wpiece16 / k_wpiece4: writes of 16 bytes per lane
//              streaming, and 16 / 4 bytes in each 128-byte line (WRITE_SIZE)
// The program prints, for each kernel, the bytes of the distinct 128-, 64-
// and 32-byte blocks it touches (counted on the host from the same address
// formula); FETCH_SIZE per dispatch divided by those gives the factor that
// turns the counter into bytes for that pattern.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>


constexpr size_t kBuf = (size_t)1536 << 20;  // 1.5 GiB: far beyond the Infinity Cache
constexpr int kStride = 2048;                // plane stride (hl_encoder.hip: 1088p planes)

__global__ void k_stream(const uint4* p, size_t n, unsigned* out)
{
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// quad q: column X = (q * 97) % 1900 + (q & 3), rows Y..Y+3 with Y = 8 * (q / 1900 * 4 + ...):
// each quad owns rows of its own so that no two quads share a line.
__host__ __device__ inline void gather_addr(unsigned q, int r, int plane, size_t& a0)
{
    const unsigned col = (q % 15) * 128 + 3 + (q & 1);                 // 15 quads per row band, one line each, misaligned
    const unsigned band = q / 15;                                      // 4 rows per band
    const size_t planeoff = (size_t)plane * (kBuf / 2);
    a0 = planeoff + ((size_t)band * 4 + r) * kStride + col;            // the sample's byte address
}

__global__ void k_gather(const uint8_t* p, unsigned nquads, unsigned* out)
{
    const unsigned q = (blockIdx.x * blockDim.x + threadIdx.x) >> 2;
    const int r = threadIdx.x & 3;
    if (q >= nquads) return;
    unsigned acc = 0;
    for (int plane = 0; plane < 2; ++plane) {
        size_t a;
        gather_addr(q, r, plane, a);
        const unsigned* w = reinterpret_cast<const unsigned*>(p + (a & ~(size_t)3));
        acc += __builtin_amdgcn_alignbyte(w[1], w[0], (unsigned)(a & 3));
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// writes: 16 bytes per lane streaming; 16 bytes per 128-byte line (a task's
// plane-block and recon-row pieces); 4 bytes per line
__global__ void k_wstream(uint4* p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = make_uint4(1, 2, 3, (unsigned)i);
}
__global__ void k_wpiece16(uint8_t* p, unsigned n)
{
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) *reinterpret_cast<uint4*>(p + (size_t)i * 128 + 32) = make_uint4(i, 1, 2, 3);
}
__global__ void k_wpiece4(uint8_t* p, unsigned n)
{
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) *reinterpret_cast<unsigned*>(p + (size_t)i * 128 + 8) = i;
}

__global__ void k_bytes(const uint8_t* p, unsigned n, unsigned* out)
{
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned v = *reinterpret_cast<const unsigned*>(p + (size_t)i * 128 + 8);
    if (v == 0x12345678u) out[0] = v;
}

int main()
{
    // one cold buffer per measured kernel, and a flush buffer streamed before
    // each of them so that none of its lines is still in the Infinity Cache
    uint8_t *a = nullptr, *b = nullptr, *c = nullptr, *f = nullptr;
    unsigned* out = nullptr;
    const size_t nflush = (size_t)768 << 20;
    if (hipMalloc(&a, kBuf) || hipMalloc(&b, kBuf) || hipMalloc(&c, kBuf) || hipMalloc(&f, nflush) || hipMalloc(&out, 64)) return 1;
    if (hipMemset(a, 1, kBuf) || hipMemset(b, 1, kBuf) || hipMemset(c, 1, kBuf) || hipMemset(f, 1, nflush)) return 1;
    auto flush = [&] { k_stream<<<4096, 256>>>(reinterpret_cast<const uint4*>(f), nflush / 16, out); };
    flush();
    k_stream<<<4096, 256>>>(reinterpret_cast<const uint4*>(a), kBuf / 16, out);
    flush();
    // the gather: bands over each plane half (each band 4 rows x 2048 B)
    const unsigned bands = (unsigned)((kBuf / 2) / (4 * (size_t)kStride)) - 1;
    const unsigned nquads = bands * 15;
    k_gather<<<(nquads * 4 + 255) / 256, 256>>>(b, nquads, out);
    flush();
    const unsigned nlines = (unsigned)(kBuf / 128);
    k_bytes<<<(nlines + 255) / 256, 256>>>(c, nlines, out);
    flush();
    k_wstream<<<4096, 256>>>(reinterpret_cast<uint4*>(a), kBuf / 16);
    flush();
    k_wpiece16<<<(nlines + 255) / 256, 256>>>(b, nlines);
    flush();
    k_wpiece4<<<(nlines + 255) / 256, 256>>>(c, nlines);
    if (hipDeviceSynchronize()) return 2;
    // distinct blocks of the gather: every (quad, row, plane) reads two
    // aligned dwords at (q % 15) * 128 + 0 or 4 of its own row of its own
    // band, so each touches one 32-, 64- and 128-byte block of its own
    const size_t nacc = (size_t)nquads * 4 * 2;
    struct { size_t size() const { return n; } size_t n; } l128{nacc}, l64{nacc}, l32{nacc};
    printf("{\"stream_bytes\": %zu, \"gather_quads\": %u, \"gather_useful_bytes\": %llu, \"gather_lines128_bytes\": %zu, "
           "\"gather_sectors64_bytes\": %zu, \"gather_sectors32_bytes\": %zu, \"bytes_kernel_lines\": %u, \"bytes_kernel_lines128_bytes\": %zu}\n",
           kBuf, nquads, (unsigned long long)nquads * 4 * 2 * 4, l128.size() * 128, l64.size() * 64, l32.size() * 32, nlines,
           (size_t)nlines * 128);
    return 0;
}
