// lfm_misc.hip -- device helpers of the HIP shim: synthetic light-field input
// generator, device query, debug switches.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include "lfm_hip.h"

namespace lfm {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ int64_t tri(int64_t a)
{
    int64_t m = a % 2048;
    return m > 1024 ? m - 1024 : 1024 - m;
}

// v = 100 + lens*field/256 + noise  (<= 3235), one thread per 8 pixels (16-byte stores)
__global__ __launch_bounds__(256) void synth_kernel(uint16_t* __restrict__ out, int X, int Y, int Z, int T, int t,
                                                    int z0, uint64_t idx0, uint64_t seed)
{
    const uint64_t total = (uint64_t)X * Y * Z;
    const int64_t half = T / 2;
    const int64_t rm = 2 * half * half + 1;
    for (uint64_t i8 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 8; i8 < total;
         i8 += (uint64_t)gridDim.x * blockDim.x * 8) {
        uint16_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint64_t i = i8 + j;
            if (i >= total) { v[j] = 0; continue; }
            const int64_t x = (int64_t)(i % X);
            const int64_t y = (int64_t)((i / X) % Y);
            const int64_t z = z0 + (int64_t)(i / ((uint64_t)X * Y));
            const int64_t du = (x % T) - half, dv = (y % T) - half;
            const int64_t lens = (1024 * (rm - (du * du + dv * dv))) / rm;
            const int64_t field = 256 + tri(3 * x + 40 * z + 97 * t) / 4 + tri(2 * y) / 4;
            const uint64_t idx = idx0 + i;
            const int64_t noise = (int64_t)(splitmix64(seed ^ (idx * 0x9E3779B97F4A7C15ull)) >> 58);
            v[j] = (uint16_t)(100 + (lens * field) / 256 + noise);
        }
        if (i8 + 8 <= total && ((reinterpret_cast<uintptr_t>(out + i8) & 15) == 0)) {
            uint4 w;
            w.x = v[0] | ((uint32_t)v[1] << 16);
            w.y = v[2] | ((uint32_t)v[3] << 16);
            w.z = v[4] | ((uint32_t)v[5] << 16);
            w.w = v[6] | ((uint32_t)v[7] << 16);
            *reinterpret_cast<uint4*>(out + i8) = w;
        } else {
            for (int j = 0; j < 8 && i8 + j < total; ++j) out[i8 + j] = v[j];
        }
    }
}

} // namespace lfm

extern "C" int lfm_hip_synth(uint16_t* d_out, int X, int Y, int Z, int T, int t_index, int z0, uint64_t idx0, uint64_t seed,
                             void* stream)
{
    if (!d_out || X <= 0 || Y <= 0 || Z <= 0 || T <= 0 || z0 < 0) return LFM_HIP_EINVAL;
    const uint64_t total = (uint64_t)X * Y * Z;
    const uint64_t threads = (total + 7) / 8;
    const int grid = (int)(threads < 256ull * 2048 ? (threads + 255) / 256 : 2048);
    hipLaunchKernelGGL(lfm::synth_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, d_out, X, Y, Z, T, t_index,
                       z0, idx0, seed);
    return hipGetLastError() == hipSuccess ? LFM_HIP_OK : LFM_HIP_ERUNTIME;
}

extern "C" int lfm_hip_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" int lfm_hip_force_generic(void)
{
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("LFM_FORCE_GENERIC");
        v = (e && e[0] == '1') ? 1 : 0;
    }
    return v;
}
