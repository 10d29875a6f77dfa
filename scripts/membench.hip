// membench.hip -- access-pattern probes for the predictor kernel's memory
// ceiling on MI355X (not part of the product).
//   hipcc --offload-arch=gfx950 -O3 scripts/membench.hip -o exp/membench
// k_copy4:    grid-stride float4 copy (the guide's 6.29 TB/s reference point)
// k_strip16:  512-pixel strips marching down rows, 16 B per lane load + store,
//             U rows in flight per wave (our read pattern, wide stores)
// k_strip2:   same loads, stores as 8 x 2-byte lane-interleaved stores
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void k_copy4(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

template <int U, bool NT>
__global__ void k_copyU(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i + u * stride < n ? a[i + u * stride] : uint4{};
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * stride < n) {
                if constexpr (NT) {
                    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                    const u32x4 t = {v[u].x, v[u].y, v[u].z, v[u].w};
                    __builtin_nontemporal_store(t, (u32x4*)(b + i + u * stride));
                }
                else b[i + u * stride] = v[u];
            }
    }
}

template <int U>
__global__ void k_read(const uint4* __restrict__ a, size_t n, uint32_t* sink)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i + u * stride < n ? a[i + u * stride] : uint4{};
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) *sink = acc;
}

// one wave per (frame, strip, piece); W = 2048, strip 512 px = 1 KiB
template <int U, bool NARROW>
__global__ __launch_bounds__(256) void k_strip(const uint16_t* __restrict__ in, uint16_t* __restrict__ out, int W,
                                               int H, int nz, int rows_per_piece)
{
    const int lane = threadIdx.x & 63;
    const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int nstrip = W / 512, npiece = (H + rows_per_piece - 1) / rows_per_piece;
    const int strip = wid % nstrip;
    const int piece = (wid / nstrip) % npiece;
    const int fz = wid / (nstrip * npiece);
    if (fz >= nz) return;
    const size_t base = (size_t)fz * W * H + strip * 512;
    const int y0 = piece * rows_per_piece, y1 = min(H, y0 + rows_per_piece);
    for (int y = y0; y < y1; y += U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int yy = min(y + u, y1 - 1);
            v[u] = *(const uint4*)(in + base + (size_t)yy * W + lane * 8);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (y + u >= y1) break;
            uint16_t* o = out + base + (size_t)(y + u) * W;
            if constexpr (!NARROW) {
                *(uint4*)(o + lane * 8) = v[u];
            } else {
                // write the same bytes lane-interleaved: lane l stores px 64j + l
                const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    // value of px 64j+lane lives in lane (64j+lane)/8, slot (lane%8)
                    const int src = (64 * j + lane) >> 3;
                    const int sl = lane & 7;
                    uint32_t x = 0;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint32_t t = __shfl(w[q], src);
                        x = (sl >> 1) == q ? t : x;
                    }
                    o[64 * j + lane] = (uint16_t)((sl & 1) ? (x >> 16) : (x & 0xffff));
                }
            }
        }
    }
}

int main()
{
    const int W = 2048, H = 2048, Z = 64;
    const size_t px = (size_t)W * H * Z, bytes = px * 2;
    uint16_t *a, *b;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMemset(a, 1, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch) {
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
        printf("{\"probe\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name, ms, 2.0 * bytes / ms / 1e9);
        fflush(stdout);
    };
    for (int g : {1024, 2048, 4096, 8192})
        run((std::string("copy4_grid") + std::to_string(g)).c_str(), [&] {
            hipLaunchKernelGGL(k_copy4, dim3(g), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, bytes / 16);
        });
    uint32_t* sink;
    hipMalloc(&sink, 4);
    for (int g : {1024, 2048, 4096}) {
        run((std::string("copyU4_grid") + std::to_string(g)).c_str(), [&] {
            hipLaunchKernelGGL((k_copyU<4, false>), dim3(g), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, bytes / 16);
        });
        run((std::string("copyU4nt_grid") + std::to_string(g)).c_str(), [&] {
            hipLaunchKernelGGL((k_copyU<4, true>), dim3(g), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, bytes / 16);
        });
        run((std::string("read_U4_grid(x0.5: bytes read only)") + std::to_string(g)).c_str(), [&] {
            hipLaunchKernelGGL((k_read<4>), dim3(g), dim3(256), 0, 0, (const uint4*)a, bytes / 16, sink);
        });
    }
    for (int rpp : {128, 256}) {
        const int waves = Z * 4 * ((H + rpp - 1) / rpp);
        const int grid = (waves + 3) / 4;
        run((std::string("strip16_U4_rpp") + std::to_string(rpp)).c_str(), [&] {
            hipLaunchKernelGGL((k_strip<4, false>), dim3(grid), dim3(256), 0, 0, a, b, W, H, Z, rpp);
        });
        run((std::string("strip16_U8_rpp") + std::to_string(rpp)).c_str(), [&] {
            hipLaunchKernelGGL((k_strip<8, false>), dim3(grid), dim3(256), 0, 0, a, b, W, H, Z, rpp);
        });
        run((std::string("strip2_U4_rpp") + std::to_string(rpp)).c_str(), [&] {
            hipLaunchKernelGGL((k_strip<4, true>), dim3(grid), dim3(256), 0, 0, a, b, W, H, Z, rpp);
        });
    }
    hipFree(a);
    hipFree(b);
    return 0;
}
