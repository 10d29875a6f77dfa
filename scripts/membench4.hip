// membench4.hip -- same-box copy ceilings and stencil-shaped access patterns
// for the predictor kernel (not part of the product).
//   hipcc --offload-arch=gfx950 -O3 scripts/membench4.hip -o exp/membench4
// Every probe moves the config-3 stack (2048 x 2048 x 64 uint16, 512 MiB in,
// 512 MiB out unless it is read-only) and prints ms and TB/s of ALGORITHMIC
// bytes (what a copy needs), so the rows compare directly with the predictor.
//   copy4_G*         guide's float4 grid-stride copy
//   rows_R8*         each workgroup copies 8 whole consecutive 4 KiB rows
//   strip512_rpp512  the round-2 predictor's pattern (512-px strip down 512 rows)
//   read_ldsdma*     read-only LDS-DMA stream (1 KiB per wave instruction)
//   band_R*          stencil-shaped: a workgroup owns R whole output rows and
//                    loads the rows the T=15 stencil reaches (y, y-1, y-T,
//                    y-T-1): two bands of R+1 rows, the second a re-read of
//                    rows the pieces above loaded (L2 hits if they are close)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <string>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ void k_copy4(const v4u* __restrict__ a, v4u* __restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

template <int PF, bool NT>
__global__ __launch_bounds__(256) void k_rows(const v4u* __restrict__ a, v4u* __restrict__ b, int R, int nrows)
{
    const int r0 = blockIdx.x * R;
    const int r1 = min(nrows, r0 + R);
    const int t = threadIdx.x;
    for (int r = r0; r < r1; r += PF) {
        v4u v[PF];
#pragma unroll
        for (int u = 0; u < PF; ++u) v[u] = r + u < r1 ? a[(size_t)(r + u) * 256 + t] : v4u{0,0,0,0};
#pragma unroll
        for (int u = 0; u < PF; ++u)
            if (r + u < r1) {
                if constexpr (NT) __builtin_nontemporal_store(v[u], &b[(size_t)(r + u) * 256 + t]);
                else b[(size_t)(r + u) * 256 + t] = v[u];
            }
    }
}

template <int SW, int U>
__global__ __launch_bounds__(256) void k_strip(const uint16_t* __restrict__ in, uint16_t* __restrict__ out, int W,
                                               int H, int nz, int rpp)
{
    constexpr int LPR = SW / 8;
    constexpr int RPI = 256 / LPR;
    const int t = threadIdx.x;
    const int nstrip = W / SW, npiece = (H + rpp - 1) / rpp;
    const int b = blockIdx.x;
    const int q = b >> 3;
    const int strip = q % nstrip, group = (q / nstrip) * 8 + (b & 7);
    const int piece = group % npiece, fz = group / npiece;
    if (fz >= nz) return;
    const size_t base = (size_t)fz * W * H + strip * SW + (t % LPR) * 8;
    const int y0 = piece * rpp, y1 = min(H, y0 + rpp);
    for (int y = y0 + t / LPR; y < y1; y += RPI * U) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int yy = min(y + u * RPI, y1 - 1);
            v[u] = *(const v4u*)(in + base + (size_t)yy * W);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (y + u * RPI < y1) __builtin_nontemporal_store(v[u], (v4u*)(out + base + (size_t)(y + u * RPI) * W));
    }
}

// read-only LDS-DMA stream: each wave streams consecutive 1 KiB pieces into a
// private 8 KiB LDS ring, 8 in flight
template <bool NT>
__global__ __launch_bounds__(256) void k_read_ldsdma(const uint8_t* __restrict__ a, size_t nbytes, uint32_t* sink)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 8192];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t nwaves = (size_t)gridDim.x * 4;
    const size_t w = (size_t)blockIdx.x * 4 + wave;
    const size_t npieces = nbytes / 1024;
    uint8_t* ring = lds + wave * 8192;
    int slot = 0;
    for (size_t p = w; p < npieces; p += nwaves) {
        const uint8_t* g = a + p * 1024 + lane * 16;
        const uint32_t m0 = __builtin_amdgcn_readfirstlane(
            (uint32_t)(size_t)(const __attribute__((address_space(3))) void*)(ring + slot * 1024));
        if constexpr (NT)
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt" ::"s"(m0), "v"(g)
                         : "memory");
        else
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m0), "v"(g)
                         : "memory");
        slot = (slot + 1) & 7;
        asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0 && ring[lane] == 0x5a && blockIdx.x == 0x7fffffff) sink[0] = ring[1];
}

// stencil-shaped: workgroup = 256 lanes x 16 B = one 4 KiB row; owns output
// rows [ys, ys + R) of frame z and loads rows ys-1 .. ys+R-1 and
// ys-T-1 .. ys-T+R-1 (clamped at 0).  ORD 0: blockIdx = z * npiece + piece;
// ORD 1: frame z on XCD z % 8, each XCD walks its frames' pieces in order.
template <int R, int TT, int ORD, bool NT>
__global__ __launch_bounds__(256) void k_band(const v4u* __restrict__ in, v4u* __restrict__ out, int H, int nz)
{
    const int npiece = (H + R - 1) / R;
    const int b = blockIdx.x;
    int z, piece;
    if constexpr (ORD == 0) {
        z = b / npiece;
        piece = b % npiece;
    } else {
        const int x = b & 7, q = b >> 3;
        z = (q / npiece) * 8 + x;
        piece = q % npiece;
    }
    if (z >= nz) return;
    const int t = threadIdx.x;
    const int ys = piece * R;
    const v4u* f = in + (size_t)z * H * 256 + t;
    v4u* o = out + (size_t)z * H * 256 + t;
    v4u bb[R + 1], aa[R + 1];
#pragma unroll
    for (int i = 0; i <= R; ++i) {
        const int yb = max(0, min(H - 1, ys - 1 + i));
        bb[i] = f[(size_t)yb * 256];
    }
#pragma unroll
    for (int i = 0; i <= R; ++i) {
        const int ya = max(0, min(H - 1, ys - TT - 1 + i));
        aa[i] = f[(size_t)ya * 256];
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
        if (ys + i >= H) break;
        v4u v;
        v.x = bb[i + 1].x ^ (bb[i].x >> 1) ^ aa[i + 1].x ^ (aa[i].x << 1);
        v.y = bb[i + 1].y ^ (bb[i].y >> 1) ^ aa[i + 1].y ^ (aa[i].y << 1);
        v.z = bb[i + 1].z ^ (bb[i].z >> 1) ^ aa[i + 1].z ^ (aa[i].z << 1);
        v.w = bb[i + 1].w ^ (bb[i].w >> 1) ^ aa[i + 1].w ^ (aa[i].w << 1);
        if constexpr (NT) __builtin_nontemporal_store(v, &o[(size_t)(ys + i) * 256]);
        else o[(size_t)(ys + i) * 256] = v;
    }
}

// WG w copies rows [w*R, w*R+R) in order (ROT = 0) or starting at a per-WG
// phase and wrapping inside its piece (ROT = 1): with long pieces and every
// WG in lock step, rows w*R + s of all WGs share their low address bits
template <int PF, bool ROT>
__global__ __launch_bounds__(256) void k_rows_rot(const v4u* __restrict__ a, v4u* __restrict__ b, int R, int nrows)
{
    const int r0 = blockIdx.x * R;
    const int t = threadIdx.x;
    const int phase = ROT ? (int)((blockIdx.x * 2654435761u) >> 7) % R : 0;
    for (int s = 0; s < R; s += PF) {
        v4u v[PF];
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            int rr = s + u + phase;
            rr = rr >= R ? rr - R : rr;
            v[u] = a[(size_t)(r0 + rr) * 256 + t];
        }
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            int rr = s + u + phase;
            rr = rr >= R ? rr - R : rr;
            __builtin_nontemporal_store(v[u], &b[(size_t)(r0 + rr) * 256 + t]);
        }
    }
}

int main()
{
    const int W = 2048, H = 2048, Z = 64;
    const size_t bytes = (size_t)W * H * Z * 2;
    const int nrows = H * Z;
    uint16_t *a = nullptr, *b = nullptr;
    uint32_t* sink = nullptr;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess)
        return 1;
    (void)hipMemset(a, 1, bytes);
    (void)hipMemset(b, 0, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](const std::string& name, double alg_bytes, auto launch) {
        launch();
        if (hipDeviceSynchronize() != hipSuccess) { printf("{\"probe\": \"%s\", \"error\": 1}\n", name.c_str()); return; }
        const int it = 20;
        (void)hipEventRecord(e0);
        for (int i = 0; i < it; ++i) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= it;
        printf("{\"probe\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f, \"frac_8TBs\": %.4f}\n", name.c_str(), ms,
               alg_bytes / ms / 1e9, alg_bytes / ms / 1e9 / 8.0);
        fflush(stdout);
    };
    const double cp = 2.0 * bytes;
    for (int rep = 0; rep < 2; ++rep) {
        for (int g : {1024, 2048})
            run("copy4_G" + std::to_string(g), cp, [&] {
                hipLaunchKernelGGL(k_copy4, dim3(g), dim3(256), 0, 0, (const v4u*)a, (v4u*)b, bytes / 16);
            });
        run("rows_R8_pf4", cp, [&] {
            hipLaunchKernelGGL((k_rows<4, false>), dim3(nrows / 8), dim3(256), 0, 0, (const v4u*)a, (v4u*)b, 8,
                               nrows);
        });
        run("rows_R8_pf4_ntst", cp, [&] {
            hipLaunchKernelGGL((k_rows<4, true>), dim3(nrows / 8), dim3(256), 0, 0, (const v4u*)a, (v4u*)b, 8,
                               nrows);
        });
        run("rows_R16_pf8_ntst", cp, [&] {
            hipLaunchKernelGGL((k_rows<8, true>), dim3(nrows / 16), dim3(256), 0, 0, (const v4u*)a, (v4u*)b, 16,
                               nrows);
        });
        for (int R : {128, 512})
            for (int rot = 0; rot < 2; ++rot)
                run("rows_R" + std::to_string(R) + (rot ? "_rot" : "_seq"), cp, [&] {
                    if (rot)
                        hipLaunchKernelGGL((k_rows_rot<4, true>), dim3(nrows / R), dim3(256), 0, 0, (const v4u*)a,
                                           (v4u*)b, R, nrows);
                    else
                        hipLaunchKernelGGL((k_rows_rot<4, false>), dim3(nrows / R), dim3(256), 0, 0, (const v4u*)a,
                                           (v4u*)b, R, nrows);
                });
        run("strip512_rpp512", cp, [&] {
            hipLaunchKernelGGL((k_strip<512, 4>), dim3(Z * 4 * 4), dim3(256), 0, 0, a, b, W, H, Z, 512);
        });
        for (int g : {1024, 2048}) {
            run("read_ldsdma_G" + std::to_string(g), (double)bytes, [&] {
                hipLaunchKernelGGL((k_read_ldsdma<false>), dim3(g), dim3(256), 0, 0, (const uint8_t*)a, bytes, sink);
            });
            run("read_ldsdma_nt_G" + std::to_string(g), (double)bytes, [&] {
                hipLaunchKernelGGL((k_read_ldsdma<true>), dim3(g), dim3(256), 0, 0, (const uint8_t*)a, bytes, sink);
            });
        }
#define BAND(RR, ORD, NT)                                                                                          \
    run(std::string("band_R" #RR "_ord" #ORD) + (NT ? "_ntst" : ""), cp, [&] {                                                    \
        hipLaunchKernelGGL((k_band<RR, 15, ORD, NT>), dim3(Z * ((H + RR - 1) / RR)), dim3(256), 0, 0,              \
                           (const v4u*)a, (v4u*)b, H, Z);                                                     \
    });
        BAND(4, 0, true) BAND(4, 1, true)
        BAND(8, 0, true) BAND(8, 1, true) BAND(8, 1, false)
        BAND(14, 0, true) BAND(14, 1, true)
#undef BAND
    }
    (void)hipFree(a);
    (void)hipFree(b);
    (void)hipFree(sink);
    return 0;
}
