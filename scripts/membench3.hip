// membench3.hip -- strip-width probe for the predictor's access pattern (not
// part of the product): a 256-thread workgroup copies a SW-pixel-wide strip
// of a 2048 x 2048 x 64 uint16 stack down `rpp` rows (16 B per lane, U
// row-groups in flight), grid = frames x pieces x strips, XCD-interleaved
// like the predictor's launcher.
//   hipcc --offload-arch=gfx950 -O3 scripts/membench3.hip -o exp/membench3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <string>

template <int SW, int U>
__global__ __launch_bounds__(256) void k_strip(const uint16_t* __restrict__ in, uint16_t* __restrict__ out, int W,
                                               int H, int nz, int rpp)
{
    constexpr int LPR = SW / 8;        // lanes per row
    constexpr int RPI = 256 / LPR;     // rows per iteration
    const int t = threadIdx.x;
    const int nstrip = W / SW, npiece = (H + rpp - 1) / rpp;
    const int b = blockIdx.x;
    const int strip = b % nstrip, group = b / nstrip;
    const int piece = group % npiece, fz = group / npiece;
    if (fz >= nz) return;
    const size_t base = (size_t)fz * W * H + strip * SW + (t % LPR) * 8;
    const int y0 = piece * rpp, y1 = min(H, y0 + rpp);
    for (int y = y0 + t / LPR; y < y1; y += RPI * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int yy = min(y + u * RPI, y1 - 1);
            v[u] = *(const uint4*)(in + base + (size_t)yy * W);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (y + u * RPI < y1) *(uint4*)(out + base + (size_t)(y + u * RPI) * W) = v[u];
    }
}

int main()
{
    const int W = 2048, H = 2048, Z = 64;
    const size_t bytes = (size_t)W * H * Z * 2;
    uint16_t *a = nullptr, *b = nullptr;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
    (void)hipMemset(a, 1, bytes);
    (void)hipMemset(b, 0, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](const std::string& name, auto launch) {
        launch();
        (void)hipDeviceSynchronize();
        const int it = 20;
        (void)hipEventRecord(e0);
        for (int i = 0; i < it; ++i) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= it;
        printf("{\"probe\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name.c_str(), ms, 2.0 * bytes / ms / 1e9);
        fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep)
        for (int rpp : {64, 256, 512}) {
            const int np = (H + rpp - 1) / rpp;
            run("sw512_rpp" + std::to_string(rpp), [&] {
                hipLaunchKernelGGL((k_strip<512, 4>), dim3(Z * np * 4), dim3(256), 0, 0, a, b, W, H, Z, rpp);
            });
            run("sw1024_rpp" + std::to_string(rpp), [&] {
                hipLaunchKernelGGL((k_strip<1024, 4>), dim3(Z * np * 2), dim3(256), 0, 0, a, b, W, H, Z, rpp);
            });
            run("sw2048_rpp" + std::to_string(rpp), [&] {
                hipLaunchKernelGGL((k_strip<2048, 4>), dim3(Z * np), dim3(256), 0, 0, a, b, W, H, Z, rpp);
            });
            run("sw2048_u8_rpp" + std::to_string(rpp), [&] {
                hipLaunchKernelGGL((k_strip<2048, 8>), dim3(Z * np), dim3(256), 0, 0, a, b, W, H, Z, rpp);
            });
        }
    return 0;
}
