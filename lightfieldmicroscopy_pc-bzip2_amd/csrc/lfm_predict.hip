// lfm_predict.hip -- fused forward predictor + zig-zag symbolize for gfx950.
//
// Replaces the reference's per-frame launches of _predictorK_{tiles,angle,space}
// (lfm_Predictors*.cu, one 1024-thread block per lens, 16-22 % of lanes active)
// followed by symbolizeKernel (lfm_Predictors.cu:2769) and the per-frame
// host<->device copies of Predictor_both (klb_imageIO.cpp:1244-1313).
//
// Fast kernel layout (W % 8 == 0, Nnum <= 31):
//   * one workgroup = 4 waves owns a 512-pixel-wide strip of a frame and
//     marches down a segment of rows; the input rows stream HBM -> VGPR
//     (16 B per lane, prefetched two steps ahead) -> an LDS ring of T+9 row
//     slots (32-pixel left halo + 512 pixels);
//   * each step every wave computes one row: lane l handles columns
//     l, l+64, ..., l+448 so every LDS neighbour read is conflict-free;
//   * residual -> int16 -> symbol in registers, one 2-byte store per pixel
//     (128 contiguous bytes per wave instruction);
//   * all frames of a stack in one launch, workgroups grid-stride over
//     (frame, row segment, strip) work items.
// Every input pixel is read from HBM once (+ the 32-pixel halo per strip and
// the T+1 primed rows per segment, served mostly from L2 / MALL); every symbol
// is written once.  Algorithmic traffic: 2 B read + 2 B written per pixel,
// +2 B read on temporal frames.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "lfm_cases.h"
#include "lfm_hip.h"

namespace lfm {

constexpr int kStrip = 512;           // pixels per strip (64 lanes x 8)
constexpr int kHalo = 32;             // left halo pixels (covers x - T - 1 for T <= 31)
constexpr int kSlot = kHalo + kStrip; // pixels per LDS row slot (1088 bytes)
constexpr int kWaves = 4;
constexpr int kThreads = kWaves * 64;
constexpr int kPrefetch = 2;          // steps of rows kept in flight per wave
constexpr int kMaxFastT = 31;

struct FrameSet {
    const uint16_t* in;    // nz frames, frame stride W*H
    const uint16_t* prev;  // raw frame preceding in[0] (needed if frame 0 is temporal) or null
    uint16_t* out;         // symbols, same layout
    int W, H, T, nz, z0, video;
};

__device__ __forceinline__ bool frame_temporal(const FrameSet& p, int fz)
{
    return ((p.video & (p.z0 + fz)) & 1) != 0;    // z_flag = video_bit & z (klb_imageIO.cpp:1270)
}
__device__ __forceinline__ const uint16_t* frame_prev(const FrameSet& p, int fz)
{
    size_t fs = (size_t)p.W * p.H;
    return fz > 0 ? p.in + (size_t)(fz - 1) * fs : p.prev;
}

// ----------------------------------------------------------- generic path --
struct GlobalNb {
    const uint16_t* f;
    int W, T, x, y;
    template <int N>
    __device__ __forceinline__ int at() const
    {
        int dx = 0, dy = 0;
        if constexpr (N == NB_A) { dx = -1; }
        if constexpr (N == NB_B) { dy = -1; }
        if constexpr (N == NB_C) { dx = -1; dy = -1; }
        if constexpr (N == NB_AP) { dx = -T; }
        if constexpr (N == NB_BP) { dy = -T; }
        if constexpr (N == NB_CP) { dx = -T; dy = -T; }
        if constexpr (N == NB_AP1) { dx = -T - 1; }
        if constexpr (N == NB_BP1) { dy = -T - 1; }
        if constexpr (N == NB_ABP) { dx = -1; dy = -T; }
        if constexpr (N == NB_BAP) { dx = -T; dy = -1; }
        return (int)f[(size_t)(y + dy) * W + (x + dx)];
    }
};

template <int FAM, int K, bool TEMP, class G>
__device__ __forceinline__ int residual_any_case(G& g, int tc, int uc, int I, int P)
{
    switch (tc * 4 + uc) {
#define LFM_CASE(TC_, UC_) \
    case TC_ * 4 + UC_: return case_residual<FAM, K, TC_, UC_, TEMP>(g, I, P);
    LFM_CASE(0, 0) LFM_CASE(0, 1) LFM_CASE(0, 2) LFM_CASE(0, 3)
    LFM_CASE(1, 0) LFM_CASE(1, 1) LFM_CASE(1, 2) LFM_CASE(1, 3)
    LFM_CASE(2, 0) LFM_CASE(2, 1) LFM_CASE(2, 2) LFM_CASE(2, 3)
    LFM_CASE(3, 0) LFM_CASE(3, 1) LFM_CASE(3, 2) LFM_CASE(3, 3)
#undef LFM_CASE
    }
    return 0;
}

__device__ __forceinline__ int tile_case(int tx, int ty) { return tx == 0 ? (ty == 0 ? 0 : 1) : (ty == 0 ? 2 : 3); }
__device__ __forceinline__ int pos_case(int u, int v) { return u == 0 ? (v > 0 ? 0 : 1) : (v == 0 ? 2 : 3); }

// One thread per pixel, neighbours straight from global memory (any W, any T).
template <int FAM, int K>
__global__ __launch_bounds__(256) void predict_generic(FrameSet p)
{
    const size_t fs = (size_t)p.W * p.H;
    const size_t total = fs * p.nz;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        int fz = (int)(i / fs);
        size_t r = i - (size_t)fz * fs;
        int y = (int)(r / p.W), x = (int)(r - (size_t)y * p.W);
        const uint16_t* f = p.in + (size_t)fz * fs;
        GlobalNb g{f, p.W, p.T, x, y};
        int tc = tile_case(x / p.T, y / p.T), uc = pos_case(x % p.T, y % p.T);
        int I = f[r];
        int res;
        if (frame_temporal(p, fz)) {
            int P = frame_prev(p, fz)[r];
            res = residual_any_case<FAM, K, true>(g, tc, uc, I, P);
        } else {
            res = residual_any_case<FAM, K, false>(g, tc, uc, I, 0);
        }
        p.out[(size_t)fz * fs + r] = (uint16_t)symbolize16(res);
    }
}

// -------------------------------------------------------------- fast path --
struct RingNb {
    const uint16_t* ring;
    int s0, s1, sT, sT1;  // LDS offsets (pixels) of rows y, y-1, y-T, y-T-1 at column c
    int T;
    template <int N>
    __device__ __forceinline__ int at() const
    {
        if constexpr (N == NB_A) return ring[s0 - 1];
        if constexpr (N == NB_B) return ring[s1];
        if constexpr (N == NB_C) return ring[s1 - 1];
        if constexpr (N == NB_AP) return ring[s0 - T];
        if constexpr (N == NB_BP) return ring[sT];
        if constexpr (N == NB_CP) return ring[sT - T];
        if constexpr (N == NB_AP1) return ring[s0 - T - 1];
        if constexpr (N == NB_BP1) return ring[sT1];
        if constexpr (N == NB_ABP) return ring[sT - 1];
        if constexpr (N == NB_BAP) return ring[s1 - T];
        return 0;
    }
};

// residual of one pixel inside a row whose (ty==0, v==0) pair is fixed
template <int FAM, int K, bool TEMP, bool TY0, bool V0>
__device__ __forceinline__ int row_residual(RingNb& g, int I, int P, bool u0, bool tx0)
{
    constexpr int tcX = TY0 ? TC_X0 : TC_XY;
    constexpr int tc0 = TY0 ? TC_00 : TC_0Y;
    constexpr int ucU = V0 ? UC_CORNER : UC_COL;
    constexpr int ucI = V0 ? UC_ROW : UC_IN;
    int r_in = case_residual<FAM, K, tcX, ucI, TEMP>(g, I, P);
    int r_u0 = case_residual<FAM, K, tcX, ucU, TEMP>(g, I, P);
    int r = u0 ? r_u0 : r_in;
    if (tx0) {  // only lanes of strip 0 with x < T (wave-divergent but rare)
        r = u0 ? case_residual<FAM, K, tc0, ucU, TEMP>(g, I, P) : case_residual<FAM, K, tc0, ucI, TEMP>(g, I, P);
    }
    return r;
}

template <int FAM, int K, bool TEMP, bool TY0, bool V0>
__device__ __forceinline__ void compute_row(const FrameSet& p, const uint16_t* ring, int slot_y, int slot_y1,
                                            int slot_yT, int slot_yT1, int y, int xs, int lane,
                                            const uint16_t* prevf, uint16_t* outf)
{
#pragma unroll
    for (int j = 0; j < kStrip / 64; ++j) {
        const int c = j * 64 + lane;
        const int x = xs + c;
        if (x < p.W) {
            const int cc = kHalo + c;
            RingNb g{ring, slot_y + cc, slot_y1 + cc, slot_yT + cc, slot_yT1 + cc, p.T};
            const int I = ring[slot_y + cc];
            const int P = TEMP ? (int)prevf[(size_t)y * p.W + x] : 0;
            const bool u0 = (x % p.T) == 0;
            const bool tx0 = x < p.T;
            int r = row_residual<FAM, K, TEMP, TY0, V0>(g, I, P, u0, tx0);
            outf[(size_t)y * p.W + x] = (uint16_t)symbolize16(r);
        }
    }
}

template <int FAM, int K, bool TEMP>
__device__ __forceinline__ void compute_row_dispatch(const FrameSet& p, const uint16_t* ring, int R, int y, int xs,
                                                     int lane, const uint16_t* prevf, uint16_t* outf)
{
    const int T = p.T;
    auto slot = [&](int yy) { int s = yy % R; return (s < 0 ? s + R : s) * kSlot; };
    const int s0 = slot(y), s1 = slot(y - 1), sT = slot(y - T), sT1 = slot(y - T - 1);
    const bool ty0 = y < T;
    const bool v0 = (y % T) == 0;
    if (ty0) {
        if (v0) compute_row<FAM, K, TEMP, true, true>(p, ring, s0, s1, sT, sT1, y, xs, lane, prevf, outf);
        else compute_row<FAM, K, TEMP, true, false>(p, ring, s0, s1, sT, sT1, y, xs, lane, prevf, outf);
    } else {
        if (v0) compute_row<FAM, K, TEMP, false, true>(p, ring, s0, s1, sT, sT1, y, xs, lane, prevf, outf);
        else compute_row<FAM, K, TEMP, false, false>(p, ring, s0, s1, sT, sT1, y, xs, lane, prevf, outf);
    }
}

struct RowChunk {
    uint4 main;
    uint4 halo;
};

__device__ __forceinline__ RowChunk load_row(const uint16_t* f, int W, int y, int xs, int lane)
{
    RowChunk rc;
    rc.main = make_uint4(0, 0, 0, 0);
    rc.halo = make_uint4(0, 0, 0, 0);
    const uint16_t* row = f + (size_t)y * W;
    const int x = xs + lane * 8;
    if (x < W) rc.main = *reinterpret_cast<const uint4*>(row + x);
    if (lane < kHalo / 8 && xs > 0) rc.halo = *reinterpret_cast<const uint4*>(row + xs - kHalo + lane * 8);
    return rc;
}

__device__ __forceinline__ void store_row_lds(uint16_t* ring, int R, int y, int lane, const RowChunk& rc)
{
    uint16_t* s = ring + (y % R) * kSlot;
    *reinterpret_cast<uint4*>(s + kHalo + lane * 8) = rc.main;
    if (lane < kHalo / 8) *reinterpret_cast<uint4*>(s + lane * 8) = rc.halo;
}

template <int FAM, int K>
__global__ __launch_bounds__(kThreads) void predict_fast(FrameSet p, int rows_per_seg, int nseg, int nstrip)
{
    extern __shared__ __attribute__((aligned(16))) uint16_t ring[];
    const int R = p.T + 9;  // rows y-T-1 .. y+3 live during a step, plus the 4 being written
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const size_t fs = (size_t)p.W * p.H;
    const int items = p.nz * nseg * nstrip;

    for (int item = blockIdx.x; item < items; item += gridDim.x) {
        const int strip = item % nstrip;
        const int seg = (item / nstrip) % nseg;
        const int fz = item / (nstrip * nseg);
        const int xs = strip * kStrip;
        const int ys = seg * rows_per_seg;
        const int ye = min(ys + rows_per_seg, p.H);
        const uint16_t* f = p.in + (size_t)fz * fs;
        uint16_t* outf = p.out + (size_t)fz * fs;
        const bool temporal = frame_temporal(p, fz);
        const uint16_t* prevf = temporal ? frame_prev(p, fz) : nullptr;

        __syncthreads();  // previous item's readers are done with the ring
        // prime rows ys-T-1 .. ys-1
        for (int y = max(0, ys - p.T - 1) + wave; y < ys; y += kWaves) {
            RowChunk rc = load_row(f, p.W, y, xs, lane);
            store_row_lds(ring, R, y, lane, rc);
        }
        RowChunk pf[kPrefetch];
#pragma unroll
        for (int d = 0; d < kPrefetch; ++d) {
            const int y = ys + d * kWaves + wave;
            if (y < ye) pf[d] = load_row(f, p.W, y, xs, lane);
        }
        const int nsteps = (ye - ys + kWaves - 1) / kWaves;
        for (int s0 = 0; s0 < nsteps; s0 += kPrefetch) {
#pragma unroll
            for (int d = 0; d < kPrefetch; ++d) {
                const int s = s0 + d;
                if (s < nsteps) {  // uniform across the workgroup
                    const int y = ys + s * kWaves + wave;
                    if (y < ye) store_row_lds(ring, R, y, lane, pf[d]);
                    const int yn = y + kPrefetch * kWaves;
                    if (yn < ye) pf[d] = load_row(f, p.W, yn, xs, lane);
                    __syncthreads();
                    if (y < ye) {
                        if (temporal) compute_row_dispatch<FAM, K, true>(p, ring, R, y, xs, lane, prevf, outf);
                        else compute_row_dispatch<FAM, K, false>(p, ring, R, y, xs, lane, prevf, outf);
                    }
                }
            }
        }
    }
}

// -------------------------------------------------------------- launchers --
template <int FAM, int K>
static hipError_t launch_k(const FrameSet& p, hipStream_t st, int force_generic)
{
    const bool fast = !force_generic && p.T <= kMaxFastT && (p.W % 8) == 0 && p.W >= kHalo;
    if (!fast) {
        size_t total = (size_t)p.W * p.H * p.nz;
        int grid = (int)std::min<size_t>((total + 255) / 256, 256 * 16);
        hipLaunchKernelGGL((predict_generic<FAM, K>), dim3(grid), dim3(256), 0, st, p);
        return hipGetLastError();
    }
    const int R = p.T + 9;
    const size_t lds = (size_t)R * kSlot * sizeof(uint16_t);
    const int rows_per_seg = 128;
    const int nseg = (p.H + rows_per_seg - 1) / rows_per_seg;
    const int nstrip = (p.W + kStrip - 1) / kStrip;
    const int items = p.nz * nseg * nstrip;
    int occ = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)predict_fast<FAM, K>, kThreads, lds);
    if (e != hipSuccess || occ <= 0) occ = 1;
    int dev = 0, ncu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
    const int resident = occ * ncu;
    // equal item counts per workgroup where possible
    const int rounds = (items + resident - 1) / resident;
    const int grid = std::max(1, (items + rounds - 1) / rounds);
    hipLaunchKernelGGL((predict_fast<FAM, K>), dim3(grid), dim3(kThreads), lds, st, p, rows_per_seg, nseg, nstrip);
    return hipGetLastError();
}

template <int FAM>
static hipError_t launch_fam(int k, const FrameSet& p, hipStream_t st, int force_generic)
{
    switch (k) {
    case 1: return launch_k<FAM, 1>(p, st, force_generic);
    case 2: return launch_k<FAM, 2>(p, st, force_generic);
    case 3: return launch_k<FAM, 3>(p, st, force_generic);
    case 4: return launch_k<FAM, 4>(p, st, force_generic);
    case 5: return launch_k<FAM, 5>(p, st, force_generic);
    case 6: return launch_k<FAM, 6>(p, st, force_generic);
    case 7: return launch_k<FAM, 7>(p, st, force_generic);
    }
    return hipErrorInvalidValue;
}

} // namespace lfm

extern "C" int lfm_hip_predict(const uint16_t* d_in, const uint16_t* d_prev, uint16_t* d_out, int W, int H,
                               int nframes, int T, int family, int predictor, int video_bit, int z0,
                               void* stream_)
{
    hipStream_t stream = (hipStream_t)stream_;
    if (W <= 0 || H <= 0 || nframes <= 0 || T <= 0 || predictor < 0 || predictor > 7 || family < 0 || family > 2)
        return LFM_HIP_EINVAL;
    const size_t bytes = (size_t)W * H * nframes * sizeof(uint16_t);
    if (predictor == 0) {  // candidate 0: the raw frames (klb_imageIO.cpp:1690, :1258)
        return hipMemcpyAsync(d_out, d_in, bytes, hipMemcpyDeviceToDevice, stream) == hipSuccess ? LFM_HIP_OK
                                                                                                   : LFM_HIP_ERUNTIME;
    }
    lfm::FrameSet p{d_in, d_prev, d_out, W, H, T, nframes, z0, video_bit & 1};
    if ((video_bit & 1) && ((z0 & 1) != 0) && d_prev == nullptr) return LFM_HIP_EINVAL;
    const int force_generic = lfm_hip_force_generic();
    hipError_t e = hipErrorInvalidValue;
    switch (family) {
    case 0: e = lfm::launch_fam<0>(predictor, p, stream, force_generic); break;
    case 1: e = lfm::launch_fam<1>(predictor, p, stream, force_generic); break;
    case 2: e = lfm::launch_fam<2>(predictor, p, stream, force_generic); break;
    }
    return e == hipSuccess ? LFM_HIP_OK : LFM_HIP_ERUNTIME;
}
