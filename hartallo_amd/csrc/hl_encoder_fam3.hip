// hl_encoder_fam3.hip -- k_pipeline again, built with the 8x8-family helper
// tasks (HL_FAM3=1, hl_mbcore.h guess_inter with f3out), for
// runs of a single picture.
//
// A lone picture keeps at most 60 of the 256 workgroups busy on its
// wavefront, so the helpers that search a macroblock's P8x8 partitionings
// beside it shorten the picture (the per-frame path of hl_codec_encode).  In
// a run of many pictures the device is full and the helpers' registers cost
// every macroblock more than they win, so hl_encoder.hip's own k_pipeline
// (HL_FAM3=0) serves those.  This translation unit compiles hl_encoder.hip's
// kernel section inside a namespace of its own (its headers' types and
// inline functions become hl_fam3::hl::..., no clash with the product's);
// the argument structs are the same layout in both builds.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stddef.h>
#include <stdint.h>
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

#define HL_FAM3 1
#define HL_KERNELS_ONLY 1
namespace hl_fam3 {
#include "hl_encoder.hip"
}

// Launches the HL_FAM3=1 k_pipeline on `stream` with the product's PipeArgs
// (psz = its size, checked against this build's).
extern "C" __attribute__((visibility("hidden"))) hipError_t hl_fam3_launch_pipeline(const void* args, size_t psz, int mbw, int mbh,
                                                                                      int workgroups, hipStream_t stream)
{
    if (psz != sizeof(hl_fam3::hl::PipeArgs)) return hipErrorInvalidValue;
    hl_fam3::hl::PipeArgs P;
    memcpy(&P, args, psz);
    hl_fam3::k_pipeline<<<workgroups, hl_fam3::hl::kMbThreads, 0, stream>>>(P, mbw, mbh);
    return hipGetLastError();
}

// Resident workgroups per CU of this build's k_pipeline (its register use
// differs from the HL_FAM3=0 build's); the persistent launch must not hold
// more workgroups than fit at once.
extern "C" __attribute__((visibility("hidden"))) hipError_t hl_fam3_pipeline_occupancy(int* per_cu)
{
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, hl_fam3::k_pipeline, hl_fam3::hl::kMbThreads, 0);
}
