// tiles_probe.hip -- timing / PMC harness for the vectorised predictor kernel
// (not part of the product): includes csrc/lfm_predict.hip and times the
// launcher the product uses (launch_vec) on the BASELINE shapes, warm and
// back to back, checking every output against predict_generic (one thread
// per pixel, neighbours from global memory) bit for bit.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include/lfm \
//         -I lightfieldmicroscopy_pc-bzip2_amd/csrc scripts/tiles_probe.hip -o exp/tiles_probe
//   exp/tiles_probe [probe|all] [iterations]
//
// probes: tilesP4 (2048x2048x64, Nnum 15, spatial), tilesP4_video (same, video
// bit: odd frames temporal), tilesP4_c5 (one config-5 volume: 4096x4096x32,
// Nnum 13, video), angleP4 (config 3), copy (angle shape, K = 0),
// copy_c5_video (the tiles shape as a copy through its rings, config-5
// volume).  With a single probe name and no check (third argument 0) only
// that kernel runs: the PMC passes filter on it.
#define LFM_PREDICT_NO_ENTRY
#include "../lightfieldmicroscopy_pc-bzip2_amd/csrc/lfm_predict.hip"
#include <cstdio>
#include <cstring>
#include <string>

extern "C" int lfm_hip_force_generic(void) { return 0; }

using namespace lfm;

// light-field-like test data: a lens-periodic pattern plus noise, all 16 bits
__global__ void fill_kernel(uint16_t* p, size_t n, int W, int H, int T, uint32_t seed)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 13;
        h *= 0x5bd1e995u;
        h ^= h >> 15;
        const uint32_t x = (uint32_t)(i % W), y = (uint32_t)((i / W) % H), z = (uint32_t)(i / ((size_t)W * H));
        const uint32_t u = x % T, v = y % T;
        const uint32_t lens = 4000u + 900u * ((u * u + v * v) < (uint32_t)(T * T / 4)) + ((x / T + 3 * (y / T)) & 255);
        p[i] = (uint16_t)(lens + 17 * z + (h & 255) + ((h >> 20) == 0 ? 50000u : 0u));
    }
}

__global__ void cmp_kernel(const uint16_t* a, const uint16_t* b, size_t n, unsigned long long* bad)
{
    unsigned long long c = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        c += a[i] != b[i];
    if (c) atomicAdd(bad, c);
}

static hipEvent_t e0, e1;

template <class F>
static float time_it(F launch, int it)
{
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int i = 0; i < it; ++i) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / it;
}

struct Shape {
    int W, H, Z, T, video;
};

int main(int argc, char** argv)
{
    const std::string which = argc > 1 ? argv[1] : "all";
    const int it = argc > 2 ? std::atoi(argv[2]) : 20;
    const bool check = argc > 3 ? std::atoi(argv[3]) != 0 : true;
    const size_t maxn = (size_t)4096 * 4096 * 32;
    uint16_t *in = nullptr, *ref = nullptr, *out = nullptr;
    unsigned long long* bad = nullptr;
    if (hipMalloc(&in, maxn * 2) || hipMalloc(&ref, maxn * 2) || hipMalloc(&out, maxn * 2) || hipMalloc(&bad, 8))
        return 1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    // prep(p) -> the FrameSet both the reference and the kernel run on
    auto ident = [](FrameSet p) { return p; };
    auto run_prep = [&](const char* name, Shape s, int fam, int k, auto launch, auto prep) {
        if (which != "all" && which != name) return;
        const size_t n = (size_t)s.W * s.H * s.Z;
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, in, n, s.W, s.H, s.T, 0x5EEDu + s.W);
        FrameSet p = prep(FrameSet{in, nullptr, out, s.W, s.H, s.T, s.Z, 0, s.video, 0});
        long long mism = -1;
        if (check && k > 0) {
            (void)hipMemset(ref, 0, n * 2);
            FrameSet pr = p;
            pr.out = ref + (p.out - out);
            const int grid = (int)std::min<size_t>((n + 255) / 256, 256 * 16);
            switch (fam * 8 + k) {
            case 0 * 8 + 4: hipLaunchKernelGGL((predict_generic<0, 4>), dim3(grid), dim3(256), 0, 0, pr); break;
            case 1 * 8 + 4: hipLaunchKernelGGL((predict_generic<1, 4>), dim3(grid), dim3(256), 0, 0, pr); break;
            default: break;
            }
            (void)hipMemset(out, 0, n * 2);
        }
        const float ms = time_it([&] { (void)launch(p); }, it);
        if (check && k > 0) {
            (void)hipMemset(bad, 0, 8);
            hipLaunchKernelGGL(cmp_kernel, dim3(4096), dim3(256), 0, 0, out, ref, n, bad);
            unsigned long long h = 0;
            (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
            mism = (long long)h;
        }
        // algorithmic bytes: every input pixel read once, every symbol written
        // once (the previous frame of a temporal frame is the volume's own
        // frame z - 1, already counted)
        const double alg = 4.0 * n;
        // per-frame accounting (SURVEY 8(d) as stated: +2 B per temporal pixel)
        const double alg6 = alg + (s.video ? 2.0 * (double)s.W * s.H * (s.Z / 2) : 0.0);
        printf("{\"probe\": \"%s\", \"shape\": [%d, %d, %d, %d, %d], \"ms\": %.4f, \"frac_8TBs\": %.4f, "
               "\"frac_8TBs_per_frame_bytes\": %.4f, \"mismatch\": %lld}\n",
               name, s.W, s.H, s.Z, s.T, s.video, ms, alg / ms / 1e6 / 8000.0, alg6 / ms / 1e6 / 8000.0, mism);
        fflush(stdout);
    };
    auto run = [&](const char* name, Shape s, int fam, int k, auto launch) { run_prep(name, s, fam, k, launch, ident); };
    const Shape c3{2048, 2048, 64, 15, 0}, c3v{2048, 2048, 64, 15, 1}, c5{4096, 4096, 32, 13, 1};
    run("tilesP4", c3, 0, 4, [](const FrameSet& p) { return launch_vec<0, 4>(p, 0); });
#define SHAPE(WPR, NCW, RPW, PD)                                                                             \
    run("tilesP4_w" #WPR "_c" #NCW "_r" #RPW "_pd" #PD, c3, 0, 4,                                          \
        [](const FrameSet& p) { return launch_vec_shape<0, 4, 15, WPR, NCW, RPW, PD>(p, 0); });
    SHAPE(1, 4, 1, 3)
    SHAPE(1, 8, 1, 3)
    SHAPE(2, 8, 1, 3)
    SHAPE(1, 4, 2, 2)
    SHAPE(2, 4, 1, 3)
#undef SHAPE
    run("tilesP4_video", c3v, 0, 4, [](const FrameSet& p) { return launch_vec<0, 4>(p, 0); });
    // angle P4 schedules: the product shape with the
    // row pieces cut shorter (more items than resident slots, frame-major
    // order, consecutive pieces of a frame on one XCD or spread), as the
    // predictor (K = 4) and as a copy through the same ring (K = 0)
    auto sched = [](const FrameSet& p, int K, int rows, int xcd) -> hipError_t {
        const void* fn = K ? (const void*)predict_vec<1, 4, 15, 1, 4, 1, 3> : (const void*)predict_vec<1, 0, 15, 1, 4, 1, 3>;
        Plan pl;
        hipError_t e = make_plan_shape(p, fn, 4 * 64 + 64, 4, 3, 512, kVHalo, 1, pl);
        if (e != hipSuccess) return e;
        if (rows > 0) {
            pl.rows_per_piece = rows;
            pl.npiece = (p.H + rows - 1) / rows;
            pl.grid = p.nz * pl.npiece * pl.nstrip;
        }
        if (xcd >= 0) pl.xcd_map = xcd && (p.nz * pl.npiece) % 8 == 0 && pl.nstrip > 1;
        return launch_plan(fn, p, pl, 4, 1, 0);
    };
#define SCHED(K, ROWS, XCD)                                                                                  \
    run("angle_sched_k" #K "_rows" #ROWS "_xcd" #XCD, c3, 1, K,                                            \
        [&](const FrameSet& p) { return sched(p, K, ROWS, XCD); });
    SCHED(4, 0, -1) SCHED(0, 0, -1)
    SCHED(4, 0, 0) SCHED(0, 0, 0)
    SCHED(4, 256, 1) SCHED(0, 256, 1)
    SCHED(4, 128, 1) SCHED(0, 128, 1)
    SCHED(4, 64, 1) SCHED(0, 64, 1)
    SCHED(4, 2048, 1) SCHED(0, 2048, 1)
    SCHED(4, 128, 0) SCHED(0, 128, 0)
#undef SCHED
    run("tilesP4_c5", c5, 0, 4, [](const FrameSet& p) { return launch_vec<0, 4>(p, 0); });
    using S0v = VecShape<0>;
    run("tilesP4_c5_single", c5, 0, 4,  // round-3 path: temporal frames re-read frame z - 1 (P ring)
        [](const FrameSet& p) { return launch_vec_shape<0, 4, 13, S0v::WPR, S0v::NCW, S0v::RPW, S0v::PD>(p, 0); });
#define PAIR(WPR, NCW, RPW, PD)                                                                              \
    run("tilesP4_c5_pair_w" #WPR "_c" #NCW "_r" #RPW "_pd" #PD, c5, 0, 4,                                  \
        [](const FrameSet& p) { return launch_vec_pairs<0, 4, 13, WPR, NCW, RPW, PD>(p, 0); });
    PAIR(1, 8, 1, 3)
    PAIR(1, 4, 1, 3)
    PAIR(1, 8, 1, 2)
    PAIR(2, 8, 1, 3)
    PAIR(1, 8, 2, 2)
    PAIR(1, 12, 1, 3)
#undef PAIR
    // frames 1..31 of a config-5 volume as a slab starting at an odd frame
    // (temporal frame 0 with prev, 15 pairs)
    run_prep("tilesP4_c5_odd_slab", c5, 0, 4, [](const FrameSet& p) { return launch_vec<0, 4>(p, 0); },
             [](FrameSet p) {
                 const size_t fs = (size_t)p.W * p.H;
                 p.prev = p.in;
                 p.in += fs;
                 p.out += fs;
                 p.z0 = 1;
                 p.nz -= 1;
                 return p;
             });
    // frames 0..30: 15 pairs and a last spatial frame alone
    run_prep("tilesP4_c5_odd_count", c5, 0, 4, [](const FrameSet& p) { return launch_vec<0, 4>(p, 0); },
             [](FrameSet p) {
                 p.nz -= 1;
                 return p;
             });
    run("angleP4", c3, 1, 4, [](const FrameSet& p) { return launch_vec<1, 4>(p, 0); });
    run("copy", c3, 1, 0, [](const FrameSet& p) { return launch_vec_shape<1, 0, 15, 1, 4, 1, 3>(p, 0); });
    using S0 = VecShape<0>;
    run("copy_c5_video", c5, 0, 0,
        [](const FrameSet& p) { return launch_vec_shape<0, 0, 13, S0::WPR, S0::NCW, S0::RPW, S0::PD>(p, 0); });
    (void)hipFree(in);
    (void)hipFree(ref);
    (void)hipFree(out);
    (void)hipFree(bad);
    return 0;
}
