// membench2.hip -- more copy-pattern probes for the predictor's memory ceiling
// (not part of the product).  hipcc --offload-arch=gfx950 -O3 scripts/membench2.hip -o exp/membench2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <string>

__global__ void k_copy4(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

// WG w copies rows [w*R, w*R+R) of 4 KiB rows (contiguous R*4 KiB), 256 threads x 16 B per row,
// PF rows in flight per thread
template <int PF>
__global__ __launch_bounds__(256) void k_rows(const uint4* __restrict__ a, uint4* __restrict__ b, int R, int nrows)
{
    const int r0 = blockIdx.x * R;
    const int r1 = min(nrows, r0 + R);
    const int t = threadIdx.x;
    for (int r = r0; r < r1; r += PF) {
        uint4 v[PF];
#pragma unroll
        for (int u = 0; u < PF; ++u) v[u] = r + u < r1 ? a[(size_t)(r + u) * 256 + t] : uint4{};
#pragma unroll
        for (int u = 0; u < PF; ++u)
            if (r + u < r1) b[(size_t)(r + u) * 256 + t] = v[u];
    }
}

// persistent: grid G WGs; WG g takes row blocks g, g+G, ... (R rows each)
template <int PF>
__global__ __launch_bounds__(256) void k_rows_persist(const uint4* __restrict__ a, uint4* __restrict__ b, int R,
                                                      int nrows)
{
    const int t = threadIdx.x;
    const int nblk = (nrows + R - 1) / R;
    for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        const int r0 = blk * R, r1 = min(nrows, r0 + R);
        for (int r = r0; r < r1; r += PF) {
            uint4 v[PF];
#pragma unroll
            for (int u = 0; u < PF; ++u) v[u] = r + u < r1 ? a[(size_t)(r + u) * 256 + t] : uint4{};
#pragma unroll
            for (int u = 0; u < PF; ++u)
                if (r + u < r1) b[(size_t)(r + u) * 256 + t] = v[u];
        }
    }
}

int main()
{
    const int W = 2048, H = 2048, Z = 64;
    const size_t px = (size_t)W * H * Z, bytes = px * 2;
    const int nrows = H * Z;
    uint16_t *a, *b;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMemset(a, 1, bytes);
    hipMemset(b, 0, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const std::string& name, auto launch) {
        launch();
        hipDeviceSynchronize();
        const int it = 20;
        hipEventRecord(e0);
        for (int i = 0; i < it; ++i) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= it;
        printf("{\"probe\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name.c_str(), ms, 2.0 * bytes / ms / 1e9);
        fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep) {
        for (int g : {512, 768, 1024, 1280, 1536, 2048})
            run("copy4_grid" + std::to_string(g), [&] {
                hipLaunchKernelGGL(k_copy4, dim3(g), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, bytes / 16);
            });
        for (int R : {8, 16, 32, 64, 128}) {
            const int grid = (nrows + R - 1) / R;
            run("rows_R" + std::to_string(R) + "_pf4", [&] {
                hipLaunchKernelGGL((k_rows<4>), dim3(grid), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, R, nrows);
            });
            run("rows_R" + std::to_string(R) + "_pf8", [&] {
                hipLaunchKernelGGL((k_rows<8>), dim3(grid), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, R, nrows);
            });
        }
        for (int G : {512, 1024, 2048})
            for (int R : {8, 32}) {
                run("persist_G" + std::to_string(G) + "_R" + std::to_string(R) + "_pf4", [&] {
                    hipLaunchKernelGGL((k_rows_persist<4>), dim3(G), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, R,
                                       nrows);
                });
            }
    }
    hipFree(a);
    hipFree(b);
    return 0;
}
