// lfm_predict.hip -- fused forward predictor + zig-zag symbolize for gfx950.
//
// Replaces the reference's per-frame launches of _predictorK_{tiles,angle,space}
// (lfm_Predictors*.cu, one 1024-thread block per lens, 16-22 % of lanes active)
// followed by symbolizeKernel (lfm_Predictors.cu:2769) and the per-frame
// host<->device copies of Predictor_both (klb_imageIO.cpp:1244-1313).
//
// Main kernel (predict_vec, Nnum 13 / 15, W % 8 == 0; see its section): the
// ring below with a lane owning 8 CONSECUTIVE pixels -- neighbours from 16-byte
// LDS windows, packed 16-bit arithmetic for shift-free formulas, one 16-byte
// symbol store per lane.  predict_ring (other Nnum <= 31) and predict_generic
// (anything else) keep the layouts described next.
//
// Ring kernel layout (W % 8 == 0, Nnum <= 31):
//   * one workgroup = NCW compute waves + 1 loader wave owns a 512-pixel strip
//     of one frame and marches down a piece of its rows;
//   * the loader wave streams rows HBM -> LDS with LDS-DMA
//     (global_load_lds_dwordx4: 16 B per lane, one instruction per 512-pixel
//     row + one for the left halo) PD steps ahead into a ring of
//     NCW*RPW*(PD+1)+T+1 row slots (halo + 512 pixels), counting its own
//     vmcnt so compute waves never wait on memory they do not need;
//   * each step every compute wave computes RPW rows: lane l handles columns
//     l, l+64, ..., l+448, so every LDS neighbour read is conflict-free;
//   * residual -> int16 -> symbol in registers, one 2-byte store per pixel
//     (128 contiguous bytes per wave instruction);
//   * all frames of a stack in one launch; the launcher splits frames into
//     row pieces so the (frame, piece, strip) items fill the GPU about once.
// Every input pixel is read from HBM once (+ the 16/32-pixel halo per strip
// row, an L2 hit under the XCD-aware mapping, and the T+1 primed rows per
// piece); every symbol is written once.  Algorithmic traffic: 2 B read + 2 B
// written per pixel, +2 B read on temporal frames.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include "lfm_cases.h"
#include "lfm_hip.h"

namespace lfm {

// Symbols are written once and not re-read by this launch: non-temporal
// stores (measured 1-3 % faster than plain stores; nt loads were 3 % slower).
__device__ __forceinline__ void store_sym(uint16_t* p, uint16_t v) { __builtin_nontemporal_store(v, p); }

constexpr int kStrip = 512;           // pixels per strip (64 lanes x 8)
// LDS row slot = left halo + 512 strip pixels; the halo covers x - T - 1:
// 16 pixels for Nnum <= 15, 32 for Nnum <= 31 (runtime, see launch_k)
constexpr int kMaxFastT = 31;

struct FrameSet {
    const uint16_t* in;    // nz frames, frame stride W*H
    const uint16_t* prev;  // raw frame preceding in[0] (needed if frame 0 is temporal) or null
    uint16_t* out;         // symbols, same layout
    int W, H, T, nz, z0, video;
    int halo;  // fast kernel only: left halo pixels of an LDS row slot
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
// Per-lane pointers into the LDS ring for the four rows a pixel can reach
// (y, y-1, y-T, y-T-1), already offset by the lane's column; pixel group j of
// a lane is 64*j columns further, so every neighbour read below is a
// ds_read_u16 with an immediate offset off one of these bases.
struct RowPtrs {
    const uint16_t* q0;
    const uint16_t* q1;
    const uint16_t* qT;
    const uint16_t* qT1;
    int T;
};

template <int J>
struct PxNb {
    const RowPtrs& r;
    template <int N>
    __device__ __forceinline__ int at() const
    {
        constexpr int o = J * 64;
        if constexpr (N == NB_A) return r.q0[o - 1];
        if constexpr (N == NB_B) return r.q1[o];
        if constexpr (N == NB_C) return r.q1[o - 1];
        if constexpr (N == NB_AP) return r.q0[o - r.T];
        if constexpr (N == NB_BP) return r.qT[o];
        if constexpr (N == NB_CP) return r.qT[o - r.T];
        if constexpr (N == NB_AP1) return r.q0[o - r.T - 1];
        if constexpr (N == NB_BP1) return r.qT1[o];
        if constexpr (N == NB_ABP) return r.qT[o - 1];
        if constexpr (N == NB_BAP) return r.q1[o - r.T];
        return 0;
    }
};

// runtime-case neighbour accessor for the rare rows / columns
struct PxNbDyn {
    const RowPtrs& r;
    int o;
    template <int N>
    __device__ __forceinline__ int at() const
    {
        if constexpr (N == NB_A) return r.q0[o - 1];
        if constexpr (N == NB_B) return r.q1[o];
        if constexpr (N == NB_C) return r.q1[o - 1];
        if constexpr (N == NB_AP) return r.q0[o - r.T];
        if constexpr (N == NB_BP) return r.qT[o];
        if constexpr (N == NB_CP) return r.qT[o - r.T];
        if constexpr (N == NB_AP1) return r.q0[o - r.T - 1];
        if constexpr (N == NB_BP1) return r.qT1[o];
        if constexpr (N == NB_ABP) return r.qT[o - 1];
        if constexpr (N == NB_BAP) return r.q1[o - r.T];
        return 0;
    }
};

// Any row, any strip: full per-pixel case logic (rows y < T, the last partial
// strip).  Correct everywhere, used only where the fast row does not apply.
template <int FAM, int K, bool TEMP>
__device__ __forceinline__ void slow_row(const RowPtrs& r, int y, int xs, int W, int lane, const uint16_t* prow,
                                         uint16_t* orow)
{
    if constexpr (K == 0) return;
    const int T = r.T;
    const int ty = y / T, v = y - ty * T;
    for (int j = 0; j < kStrip / 64; ++j) {
        const int c = j * 64 + lane;
        const int x = xs + c;
        if (x >= W) break;
        PxNbDyn g{r, j * 64};
        const int tx = x / T, u = x - tx * T;
        const int I = r.q0[j * 64];
        const int P = TEMP ? (int)prow[j * 64] : 0;
        const int res = residual_any_case<FAM, K, TEMP>(g, tile_case(tx, ty), pos_case(u, v), I, P);
        store_sym(orow + j * 64, (uint16_t)symbolize16(res));
    }
}

// Rows y >= T of full strips: tile case is TC_XY except the columns x < T of
// strip 0 (TC_0Y); the position case is fixed by (u == 0, v == 0).
template <int FAM, int K, bool TEMP, bool V0, bool FIRST, int J>
__device__ __forceinline__ void fast_px(const RowPtrs& r, uint32_t u0bits, int lane, const uint16_t* prow,
                                        uint16_t* orow)
{
    constexpr int ucU = V0 ? UC_CORNER : UC_COL;
    constexpr int ucI = V0 ? UC_ROW : UC_IN;
    PxNb<J> g{r};
    const int I = r.q0[J * 64];
    const int P = TEMP ? (int)prow[J * 64] : 0;
    if constexpr (K == 0) {  // diagnostic ablation: same loads / LDS / stores, no prediction
        store_sym(orow + J * 64, (uint16_t)(I + P));
        return;
    }
    // both candidates are evaluated and blended with a mask: no divergent branch
    const int m0 = -(int)((u0bits >> J) & 1u);
    const int r_u = case_residual<FAM, K, TC_XY, ucU, TEMP>(g, I, P);
    const int r_i = case_residual<FAM, K, TC_XY, ucI, TEMP>(g, I, P);
    int res = r_i ^ ((r_u ^ r_i) & m0);
    if constexpr (FIRST && J == 0) {
        const int mt = -(int)(lane < r.T);  // x < T: first lens column
        const int t_u = case_residual<FAM, K, TC_0Y, ucU, TEMP>(g, I, P);
        const int t_i = case_residual<FAM, K, TC_0Y, ucI, TEMP>(g, I, P);
        const int rt = t_i ^ ((t_u ^ t_i) & m0);
        res = res ^ ((rt ^ res) & mt);
    }
    store_sym(orow + J * 64, (uint16_t)symbolize16(res));
}

template <int FAM, int K, bool TEMP, bool V0, bool FIRST>
__device__ __forceinline__ void fast_row(const RowPtrs& r, uint32_t u0bits, int lane, const uint16_t* prow,
                                         uint16_t* orow)
{
    fast_px<FAM, K, TEMP, V0, FIRST, 0>(r, u0bits, lane, prow, orow);
    fast_px<FAM, K, TEMP, V0, FIRST, 1>(r, u0bits, lane, prow, orow);
    fast_px<FAM, K, TEMP, V0, FIRST, 2>(r, u0bits, lane, prow, orow);
    fast_px<FAM, K, TEMP, V0, FIRST, 3>(r, u0bits, lane, prow, orow);
    fast_px<FAM, K, TEMP, V0, FIRST, 4>(r, u0bits, lane, prow, orow);
    fast_px<FAM, K, TEMP, V0, FIRST, 5>(r, u0bits, lane, prow, orow);
    fast_px<FAM, K, TEMP, V0, FIRST, 6>(r, u0bits, lane, prow, orow);
    fast_px<FAM, K, TEMP, V0, FIRST, 7>(r, u0bits, lane, prow, orow);
}

// sy = slot of row y in the ring (y mod R), v = y mod T, both tracked
// incrementally by the caller (no integer division per row).  prow: P-ring
// slot of row y (temporal frames).
template <int FAM, int K, bool TEMP>
__device__ __forceinline__ void compute_row(const FrameSet& p, const uint16_t* ring, int R, int y, int sy, int v,
                                            int xs, int lane, bool full, uint32_t u0bits, const uint16_t* prow,
                                            uint16_t* outf)
{
    const int T = p.T;
    auto wrap = [&](int s) { return s < 0 ? s + R : s; };
    const int slot = p.halo + kStrip;
    const uint16_t* r0 = ring + sy * slot;
    const uint16_t* r1 = ring + wrap(sy - 1) * slot;
    const uint16_t* rT = ring + wrap(sy - T) * slot;
    const uint16_t* rT1 = ring + wrap(sy - T - 1) * slot;
    uint16_t* orow0 = outf + (size_t)y * p.W + xs;
    if (!full || y < T) {
        const int h = p.halo + lane;
        const RowPtrs r{r0 + h, r1 + h, rT + h, rT1 + h, T};
        slow_row<FAM, K, TEMP>(r, y, xs, p.W, lane, TEMP ? prow + lane : nullptr, orow0 + lane);
        return;
    }
    const bool first = xs == 0;
    const int h = p.halo + lane;
    const RowPtrs r{r0 + h, r1 + h, rT + h, rT1 + h, T};
    const uint16_t* pr = TEMP ? prow + lane : nullptr;
    if (v == 0) {
        if (first) fast_row<FAM, K, TEMP, true, true>(r, u0bits, lane, pr, orow0 + lane);
        else fast_row<FAM, K, TEMP, true, false>(r, u0bits, lane, pr, orow0 + lane);
    } else {
        if (first) fast_row<FAM, K, TEMP, false, true>(r, u0bits, lane, pr, orow0 + lane);
        else fast_row<FAM, K, TEMP, false, false>(r, u0bits, lane, pr, orow0 + lane);
    }
}

// LDS-DMA (global_load_lds_dwordx4: 16 B per lane into LDS at M0 + 16*lane),
// issued from inline asm so the compiler's waitcnt pass does not treat every
// later ds_read of the computing waves as a reader of an in-flight DMA (it
// would insert vmcnt(0) there, i.e. wait for the wave's own stores).  The
// loader wave counts its DMAs itself (wait_vmcnt below).
__device__ __forceinline__ void glds16(const void* g, const void* lds)
{
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(
        (uint32_t)(size_t)(const __attribute__((address_space(3))) void*)lds);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m0), "v"(g)
                 : "memory", "m0");
}

// Loader wave: one LDS-DMA (global_load_lds_dwordx4, 16 B per lane, 1 KiB per
// instruction) for the 512 strip pixels of a row and one for its 32-pixel left
// halo (lanes 0-3).  Addresses are clamped to valid pixels so the count of
// instructions per row never changes (the vmcnt waits below are counted).
__device__ __forceinline__ void dma_row(uint16_t* ring, int slot_idx, const uint16_t* f, int W, int halo,
                                        int src_row, int xs, int lane)
{
    uint16_t* slot = ring + slot_idx * (halo + kStrip);
    const uint16_t* srow = f + (size_t)src_row * W;
    const int x = min(xs + lane * 8, W - 8);
    glds16(srow + x, slot + halo);
    if (lane < halo / 8) {
        const int hx = xs > 0 ? xs - halo + lane * 8 : lane * 8;
        glds16(srow + hx, slot);
    }
}

__device__ __forceinline__ void dma_prev_row(uint16_t* pring, int pslot_idx, const uint16_t* pf, int W, int src_row,
                                             int xs, int lane)
{
    uint16_t* slot = pring + pslot_idx * kStrip;
    const int x = min(xs + lane * 8, W - 8);
    glds16(pf + (size_t)src_row * W + x, slot);
}

// rows ys+4s .. ys+4s+3; slot0 / pslot0 = ring slots of row ys+4s
template <int NCW, bool TEMP>
__device__ __forceinline__ void dma_step(uint16_t* ring, int R, int slot0, uint16_t* pring, int RP, int pslot0,
                                         const uint16_t* f, const uint16_t* pf, int W, int halo, int ys, int ye, int s,
                                         int xs, int lane)
{
#pragma unroll
    for (int i = 0; i < NCW; ++i) {
        const int row = ys + s * NCW + i;
        const int src = min(row, ye - 1);
        int si = slot0 + i;
        si = si >= R ? si - R : si;
        dma_row(ring, si, f, W, halo, src, xs, lane);
        if constexpr (TEMP) {
            int pi = pslot0 + i;
            pi = pi >= RP ? pi - RP : pi;
            dma_prev_row(pring, pi, pf, W, src, xs, lane);
        }
    }
}

template <int N>
__device__ __forceinline__ void wait_vmcnt()
{
    static_assert(N >= 0 && N < 64, "vmcnt field is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// One work item (frame, row segment, strip) of the workgroup: waves 0-3
// compute rows ys+4s+wave, wave 4 streams rows PD steps ahead into the ring.
template <int FAM, int K, int NCW, int RPW, int PD, bool TEMP>
__device__ __forceinline__ void ring_item(const FrameSet& p, uint16_t* ring, int R, uint16_t* pring, int RP,
                                          const uint16_t* f, const uint16_t* pf, uint16_t* outf, int xs, int ys,
                                          int ye, int wave, int lane)
{
    constexpr int RS = NCW * RPW;  // rows per step; compute wave w owns rows w, w+NCW, ... of the step
    constexpr int kLoadsPerStep = RS * (TEMP ? 3 : 2);
    const bool loader = wave == NCW;
    const int nsteps = (ye - ys + RS - 1) / RS;
    const bool full = xs + kStrip <= p.W;
    const int T = p.T;
    auto adv = [](int v, int d, int m) { v += d; while (v >= m) v -= m; return v; };
    uint32_t u0bits = 0;  // bit j: column xs + 64j + lane starts a lens (u == 0)
    // compute waves: row y = ys + wave + 4s, its ring slot, its P slot, y mod T
    int y = ys + wave, sy = 0, py = 0, vy = 0;
    // loader: ring / P slots of the first row of step s + PD
    int lslot = 0, lpslot = 0;
    if (!loader) {
#pragma unroll
        for (int j = 0; j < kStrip / 64; ++j) u0bits |= (uint32_t)(((xs + j * 64 + lane) % T) == 0) << j;
        sy = y % R;
        py = TEMP ? y % RP : 0;
        vy = y % T;
    } else {
        const int r0 = max(0, ys - T - 1);
        int ps = r0 % R;
        for (int row = r0; row < ys; ++row) {
            dma_row(ring, ps, f, p.W, p.halo, row, xs, lane);
            ps = ps + 1 == R ? 0 : ps + 1;
        }
        int slot0 = ys % R, pslot0 = TEMP ? ys % RP : 0;
        for (int s = 0; s < PD && s < nsteps; ++s) {
            dma_step<RS, TEMP>(ring, R, slot0, pring, RP, pslot0, f, pf, p.W, p.halo, ys, ye, s, xs, lane);
            slot0 = adv(slot0, RS, R);
            if (TEMP) pslot0 = adv(pslot0, RS, RP);
        }
        lslot = slot0;
        lpslot = pslot0;
    }
    for (int s = 0; s < nsteps; ++s) {
        if (loader) {
            if (s + PD < nsteps) wait_vmcnt<(kLoadsPerStep * (PD - 1) < 63 ? kLoadsPerStep * (PD - 1) : 63)>();
            else wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();
        if (loader) {
            if (s + PD < nsteps) {
                dma_step<RS, TEMP>(ring, R, lslot, pring, RP, lpslot, f, pf, p.W, p.halo, ys, ye, s + PD, xs, lane);
                lslot = adv(lslot, RS, R);
                if (TEMP) lpslot = adv(lpslot, RS, RP);
            }
        } else {
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                if (y < ye) {
                    const uint16_t* prow = TEMP ? pring + py * kStrip : nullptr;
                    compute_row<FAM, K, TEMP>(p, ring, R, y, sy, vy, xs, lane, full, u0bits, prow, outf);
                }
                y += NCW;
                sy = adv(sy, NCW, R);
                if (TEMP) py = adv(py, NCW, RP);
                vy = adv(vy, NCW, T);
            }
        }
    }
    // every wave is done reading the ring before the next item's loads
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

// One workgroup per item (frame, row piece, strip).  With xcd_map the nstrip
// workgroups of one (frame, piece) are blockIdx b, b+8, b+16, ... which the
// dispatcher deals to one XCD: the 32-byte left halo of a strip row is then
// an L2 hit on the row its neighbour strip streamed a few microseconds
// earlier instead of a second HBM fetch of that 128-byte line.
template <int FAM, int K, int NCW, int RPW, int PD>
__global__ __launch_bounds__(NCW * 64 + 64) void predict_ring(FrameSet p, int rows_per_piece, int npiece, int nstrip,
                                                              int xcd_map, int R, int RP)
{
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    uint16_t* ring = lds;
    uint16_t* pring = lds + R * (p.halo + kStrip);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // wave-uniform
    const size_t fs = (size_t)p.W * p.H;
    const int b = blockIdx.x;
    int strip, group;
    if (xcd_map) {
        const int q = b >> 3;
        strip = q % nstrip;
        group = (q / nstrip) * 8 + (b & 7);
    } else {
        strip = b % nstrip;
        group = b / nstrip;
    }
    const int piece = group % npiece;
    const int fz = group / npiece;
    if (fz >= p.nz) return;
    const int xs = strip * kStrip;
    const int ys = piece * rows_per_piece;
    const int ye = min(ys + rows_per_piece, p.H);
    if (ys >= ye) return;
    const uint16_t* f = p.in + (size_t)fz * fs;
    uint16_t* outf = p.out + (size_t)fz * fs;
    if (frame_temporal(p, fz))
        ring_item<FAM, K, NCW, RPW, PD, true>(p, ring, R, pring, RP, f, frame_prev(p, fz), outf, xs, ys, ye, wave, lane);
    else
        ring_item<FAM, K, NCW, RPW, PD, false>(p, ring, R, pring, RP, f, nullptr, outf, xs, ys, ye, wave, lane);
}

// All seven spatial candidates of one frame in one launch (selection pass,
// klb_imageIO.cpp:1671-1746 runs them as seven serial launch sequences):
// blockIdx.y = k - 1 writes candidate k to out + (k - 1) * W * H.
template <int FAM, int NCW, int RPW, int PD>
__global__ __launch_bounds__(NCW * 64 + 64) void predict_cands(FrameSet p, int rows_per_piece, int npiece, int nstrip,
                                                               int xcd_map, int R, int RP)
{
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // wave-uniform
    const int b = blockIdx.x;
    int strip, piece;
    if (xcd_map) {
        const int q = b >> 3;
        strip = q % nstrip;
        piece = (q / nstrip) * 8 + (b & 7);
    } else {
        strip = b % nstrip;
        piece = b / nstrip;
    }
    const int xs = strip * kStrip;
    const int ys = piece * rows_per_piece;
    const int ye = min(ys + rows_per_piece, p.H);
    if (ys >= ye) return;
    uint16_t* outf = p.out + (size_t)blockIdx.y * p.W * p.H;
    switch (blockIdx.y) {
#define LFM_CAND(KK)                                                                                                  \
    case KK - 1:                                                                                                      \
        ring_item<FAM, KK, NCW, RPW, PD, false>(p, lds, R, nullptr, RP, p.in, nullptr, outf, xs, ys, ye, wave, lane); \
        break;
        LFM_CAND(1) LFM_CAND(2) LFM_CAND(3) LFM_CAND(4) LFM_CAND(5) LFM_CAND(6) LFM_CAND(7)
#undef LFM_CAND
    }
}

// ---------------------------------------------------- vectorised ring path --
// Nnum T in {13, 15}, W % 8 == 0.  Same loader wave / LDS ring / barrier
// protocol as predict_ring, but a lane owns 8 CONSECUTIVE pixels of a row:
//   * its neighbours come from three 16-byte LDS reads per ring row (the
//     24-pixel window [x0 - 16, x0 + 8) holds every left reach <= T + 1 = 16),
//     i.e. 3 ds_read_b128 per row instead of one ds_read_u16 per pixel and
//     neighbour; the values are picked out of the window's dwords with
//     compile-time shifts (T is a template parameter);
//   * its 8 symbols leave as ONE 16-byte non-temporal store (1 KiB per wave
//     instruction instead of 128 B).
// A strip is SW = WPR * 512 pixels wide; WPR compute waves share each row
// (wave w: row group w / WPR, quarter w % WPR), so SW = 2048 streams whole
// 4 KiB rows per workgroup.
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int kVHalo = 16;  // left halo pixels per ring slot (T + 1 <= 16)

struct Win24 {  // pixels [x0 - 16, x0 + 8) of one ring row
    uint32_t w[12];
    template <int I>
    __device__ __forceinline__ int px() const
    {
        static_assert(I >= 0 && I < 24, "window index");
        return (int)((w[I >> 1] >> ((I & 1) * 16)) & 0xFFFFu);
    }
};

// p: the lane's first pixel in the ring slot (16-byte aligned); blocks the
// caller never reads are removed by the compiler
__device__ __forceinline__ void load_win(const uint16_t* p, Win24& r)
{
    const v4u* q = (const v4u*)(p - 16);
    const v4u a = q[0], b = q[1], c = q[2];
    r.w[0] = a.x; r.w[1] = a.y; r.w[2] = a.z; r.w[3] = a.w;
    r.w[4] = b.x; r.w[5] = b.y; r.w[6] = b.z; r.w[7] = b.w;
    r.w[8] = c.x; r.w[9] = c.y; r.w[10] = c.z; r.w[11] = c.w;
}

// neighbours of pixel J of the lane's 8 (window index 16 + J - dx)
template <int T, int J>
struct VecNb {
    const Win24& r0;   // row y
    const Win24& r1;   // row y - 1
    const Win24& rT;   // row y - T
    const Win24& rT1;  // row y - T - 1
    template <int N>
    __device__ __forceinline__ int at() const
    {
        if constexpr (N == NB_A) return r0.template px<15 + J>();
        if constexpr (N == NB_B) return r1.template px<16 + J>();
        if constexpr (N == NB_C) return r1.template px<15 + J>();
        if constexpr (N == NB_AP) return r0.template px<16 + J - T>();
        if constexpr (N == NB_BP) return rT.template px<16 + J>();
        if constexpr (N == NB_CP) return rT.template px<16 + J - T>();
        if constexpr (N == NB_AP1) return r0.template px<15 + J - T>();
        if constexpr (N == NB_BP1) return rT1.template px<16 + J>();
        if constexpr (N == NB_ABP) return rT.template px<15 + J>();
        if constexpr (N == NB_BAP) return r1.template px<16 + J - T>();
        return 0;
    }
};

struct VecRows {
    Win24 r0, r1, rT, rT1;
    uint32_t p[4];  // previous frame, pixels x0 .. x0+7 (temporal frames)
    template <int J>
    __device__ __forceinline__ int prev() const
    {
        return (int)((p[J >> 1] >> ((J & 1) * 16)) & 0xFFFFu);
    }
};

// Per-lane bit masks of a work item's lanes, one 64-bit (SGPR pair) mask per
// pixel J of the lane's 8: u[J] = lanes whose pixel J starts a lens column
// (u == 0); t[J] = lanes whose pixel J lies in the frame's first lens column
// (x < T).  Computed once per item by ballots, so a row selects between two
// case formulas with one v_cndmask per pixel instead of rebuilding a mask.
struct LaneMasks {
    uint64_t u[8];
    uint64_t t[8];
};

__device__ __forceinline__ LaneMasks lane_masks(uint32_t u0bits, int x0, int T)
{
    LaneMasks m;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        m.u[j] = __builtin_amdgcn_ballot_w64(((u0bits >> j) & 1u) != 0);
        m.t[j] = __builtin_amdgcn_ballot_w64(x0 + j < T);
    }
    return m;
}

// m's bit for this lane ? if_set : if_clear (v_cndmask_b32 with an SGPR-pair mask)
__device__ __forceinline__ int lane_sel(uint64_t m, int if_set, int if_clear)
{
    int r;
    asm("" : "+s"(m));  // an SGPR pair even where the mask is a known constant
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(m));
    return r;
}

// residual (32 bits, before the int16 store) of pixel J on a row y >= T of a
// full strip: tile case TC_XY except x < T (TC_0Y, FIRST strip only);
// position case by (u == 0) per pixel and V0 per row
template <int FAM, int K, int T, bool TEMP, bool V0, bool FIRST, int J>
__device__ __forceinline__ int vec_fast_res(const VecRows& rw, const LaneMasks& lm, int x0)
{
    constexpr int ucU = V0 ? UC_CORNER : UC_COL;
    constexpr int ucI = V0 ? UC_ROW : UC_IN;
    VecNb<T, J> g{rw.r0, rw.r1, rw.rT, rw.rT1};
    const int I = rw.r0.template px<16 + J>();
    const int P = TEMP ? rw.template prev<J>() : 0;
    if constexpr (K == 0) {
        return I + P;  // diagnostic: copy through the ring
    } else {
    constexpr int Fu = case_formula(FAM, K, TC_XY, ucU), Fi = case_formula(FAM, K, TC_XY, ucI);
    constexpr int Gu = case_formula(FAM, K, TC_0Y, ucU), Gi = case_formula(FAM, K, TC_0Y, ucI);
    constexpr int kind = finish_kind(FAM, K, TC_XY, ucI, TEMP), sh = formula_shift(Fi);
    constexpr bool same_xy = finish_kind(FAM, K, TC_XY, ucU, TEMP) == kind && formula_shift(Fu) == sh;
    constexpr bool same_0y = finish_kind(FAM, K, TC_0Y, ucU, TEMP) == kind && formula_shift(Gu) == sh &&
                             finish_kind(FAM, K, TC_0Y, ucI, TEMP) == kind && formula_shift(Gi) == sh;
    constexpr bool kind_xy = finish_kind(FAM, K, TC_XY, ucU, TEMP) == kind;
    constexpr bool kind_0y = finish_kind(FAM, K, TC_0Y, ucU, TEMP) == kind &&
                             finish_kind(FAM, K, TC_0Y, ucI, TEMP) == kind;
    if constexpr (same_xy && (!FIRST || same_0y)) {
        // one inner sum selected per pixel, one shift, one finish
        int S = lane_sel(lm.u[J], eval_inner<Fu>(g), eval_inner<Fi>(g));
        if constexpr (FIRST) {
            if (x0 < T)  // lanes of the first lens column (uniform per lane)
                S = lane_sel(lm.t[J], lane_sel(lm.u[J], eval_inner<Gu>(g), eval_inner<Gi>(g)), S);
        }
        return finish_residual<kind>(S >> sh, I, P);
    } else if constexpr (kind_xy && (!FIRST || kind_0y)) {
        // different shifts: one prediction selected per pixel, one finish
        int pred = lane_sel(lm.u[J], eval_formula<Fu>(g), eval_formula<Fi>(g));
        if constexpr (FIRST) {
            if (x0 < T)
                pred = lane_sel(lm.t[J], lane_sel(lm.u[J], eval_formula<Gu>(g), eval_formula<Gi>(g)), pred);
        }
        return finish_residual<kind>(pred, I, P);
    }
    const int r_u = case_residual<FAM, K, TC_XY, ucU, TEMP>(g, I, P);
    const int r_i = case_residual<FAM, K, TC_XY, ucI, TEMP>(g, I, P);
    int res = lane_sel(lm.u[J], r_u, r_i);
    if constexpr (FIRST) {
        if (x0 < T) {  // lanes of the first lens column (uniform per lane)
            const int t_u = case_residual<FAM, K, TC_0Y, ucU, TEMP>(g, I, P);
            const int t_i = case_residual<FAM, K, TC_0Y, ucI, TEMP>(g, I, P);
            res = lane_sel(lm.t[J], lane_sel(lm.u[J], t_u, t_i), res);
        }
    }
    return res;
    }
}

// the residuals of pixels 2M, 2M+1 as one packed pair (v_perm of their low
// halves) and their zig-zag symbols in packed 16-bit arithmetic
template <int FAM, int K, int T, bool TEMP, bool V0, bool FIRST, int M>
__device__ __forceinline__ uint32_t vec_fast_pair(const VecRows& rw, const LaneMasks& lm, int x0)
{
    const int r0 = vec_fast_res<FAM, K, T, TEMP, V0, FIRST, 2 * M>(rw, lm, x0);
    const int r1 = vec_fast_res<FAM, K, T, TEMP, V0, FIRST, 2 * M + 1>(rw, lm, x0);
    // (inline asm: seen as reading only the low halves, the builtin lets the
    // compiler narrow the residual arithmetic to 16 bits, where an exact
    // (a + b) >> 1 costs 4 instructions instead of 2)
    uint32_t pr;
    asm("v_perm_b32 %0, %1, %2, %3" : "=v"(pr) : "v"(r1), "v"(r0), "s"(0x05040100u));
    if constexpr (K == 0) return pr;
    typedef short s16x2_ __attribute__((ext_vector_type(2)));
    const s16x2_ v = __builtin_bit_cast(s16x2_, pr);
    const s16x2_ one{1, 1}, fifteen{15, 15};
    return __builtin_bit_cast(uint32_t, v << one) ^ __builtin_bit_cast(uint32_t, v >> fifteen);
}

// any pixel J (rows y < T): full per-pixel case logic
template <int FAM, int K, int T, bool TEMP, int J>
__device__ __forceinline__ uint32_t vec_slow_px(const VecRows& rw, int x0, int ty, int v)
{
    VecNb<T, J> g{rw.r0, rw.r1, rw.rT, rw.rT1};
    const int I = rw.r0.template px<16 + J>();
    const int P = TEMP ? rw.template prev<J>() : 0;
    if constexpr (K == 0) return (uint32_t)(I + P) & 0xFFFFu;
    const int x = x0 + J;
    const int tx = x / T, u = x - tx * T;
    return zigzag16(residual_any_case<FAM, K, TEMP>(g, tile_case(tx, ty), pos_case(u, v), I, P));
}

// ---- packed pairs: formulas without a shift ((A + B - C), B, Bp + Ap - Cp,
// ...) are needed only mod 2^16 (the residual is stored as int16), so two
// pixels go through each 32-bit register with packed 16-bit adds; the
// symbol is the zig-zag (r << 1) ^ (r >> 15) of the int16 residual, which
// equals 2|r| + (r >> 31) (lfm_Predictors.cu:16-26) including r = -32768.
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s16x2 as_pk(uint32_t v) { return __builtin_bit_cast(s16x2, v); }
__device__ __forceinline__ uint32_t as_u32(s16x2 v) { return __builtin_bit_cast(uint32_t, v); }

// pixels I, I+1 of a window as one packed register
template <int I>
__device__ __forceinline__ uint32_t win_pair(const Win24& r)
{
    static_assert(I >= 0 && I + 1 < 24, "window pair");
    if constexpr ((I & 1) == 0) return r.w[I >> 1];
    else return __builtin_amdgcn_alignbit(r.w[(I + 1) >> 1], r.w[I >> 1], 16);
}

template <int F>
__host__ __device__ constexpr bool pk_formula()
{
    return F == F_Z || F == F_A || F == F_B || F == F_C || F == F_AP || F == F_BP || F == F_CP || F == F_ABC ||
           F == F_BAC || F == F_ABC_SUM || F == F_P4_CORNER;
}

// neighbours of the pixel pair 2M, 2M+1 (window index 16 + 2M - dx)
template <int T, int M>
struct VecNbPk {
    const Win24& r0;
    const Win24& r1;
    const Win24& rT;
    const Win24& rT1;
    template <int N>
    __device__ __forceinline__ s16x2 at() const
    {
        if constexpr (N == NB_A) return as_pk(win_pair<15 + 2 * M>(r0));
        if constexpr (N == NB_B) return as_pk(win_pair<16 + 2 * M>(r1));
        if constexpr (N == NB_C) return as_pk(win_pair<15 + 2 * M>(r1));
        if constexpr (N == NB_AP) return as_pk(win_pair<16 + 2 * M - T>(r0));
        if constexpr (N == NB_BP) return as_pk(win_pair<16 + 2 * M>(rT));
        if constexpr (N == NB_CP) return as_pk(win_pair<16 + 2 * M - T>(rT));
        return s16x2{0, 0};
    }
};

template <int F, class G>
__device__ __forceinline__ s16x2 pk_eval(const G& g)
{
    static_assert(pk_formula<F>(), "formula has a shift: not exact in 16 bits");
    if constexpr (F == F_Z) return s16x2{0, 0};
    if constexpr (F == F_A) return g.template at<NB_A>();
    if constexpr (F == F_B) return g.template at<NB_B>();
    if constexpr (F == F_C) return g.template at<NB_C>();
    if constexpr (F == F_AP) return g.template at<NB_AP>();
    if constexpr (F == F_BP) return g.template at<NB_BP>();
    if constexpr (F == F_CP) return g.template at<NB_CP>();
    if constexpr (F == F_ABC || F == F_BAC) return g.template at<NB_A>() + g.template at<NB_B>() - g.template at<NB_C>();
    if constexpr (F == F_ABC_SUM || F == F_P4_CORNER)
        return g.template at<NB_BP>() + g.template at<NB_AP>() - g.template at<NB_CP>();
    return s16x2{0, 0};
}

__device__ __forceinline__ uint32_t pk_zigzag(s16x2 r)
{
    const s16x2 one{1, 1}, fifteen{15, 15};
    return as_u32(r << one) ^ as_u32(r >> fifteen);
}

// the row's formulas for (tile case, u == 0 / u > 0) are all shift-free
template <int FAM, int K, bool TEMP, bool V0, bool FIRST>
__host__ __device__ constexpr bool pk_row_ok()
{
    if constexpr (TEMP || K < 1) {
        return false;
    } else {
        constexpr int ucU = V0 ? UC_CORNER : UC_COL, ucI = V0 ? UC_ROW : UC_IN;
        return pk_formula<case_formula(FAM, K, TC_XY, ucU)>() && pk_formula<case_formula(FAM, K, TC_XY, ucI)>() &&
               (!FIRST || (pk_formula<case_formula(FAM, K, TC_0Y, ucU)>() &&
                           pk_formula<case_formula(FAM, K, TC_0Y, ucI)>()));
    }
}

// per-lane masks of a packed pair: 0xFFFF in the half whose pixel has the bit
__device__ __forceinline__ uint32_t pair_mask(uint32_t bits, int m)
{
    return (((bits >> (2 * m)) & 1u) ? 0xFFFFu : 0u) | (((bits >> (2 * m + 1)) & 1u) ? 0xFFFF0000u : 0u);
}

template <int FAM, int K, int T, bool V0, bool FIRST, int M>
__device__ __forceinline__ uint32_t vec_pk_pair(const VecRows& rw, uint32_t u0bits, uint32_t firstbits, int x0)
{
    constexpr int ucU = V0 ? UC_CORNER : UC_COL, ucI = V0 ? UC_ROW : UC_IN;
    VecNbPk<T, M> g{rw.r0, rw.r1, rw.rT, rw.rT1};
    const s16x2 I = as_pk(win_pair<16 + 2 * M>(rw.r0));
    const uint32_t mk = pair_mask(u0bits, M);
    const uint32_t r_u = as_u32(I - pk_eval<case_formula(FAM, K, TC_XY, ucU)>(g));
    const uint32_t r_i = as_u32(I - pk_eval<case_formula(FAM, K, TC_XY, ucI)>(g));
    uint32_t res = (r_u & mk) | (r_i & ~mk);
    if constexpr (FIRST) {
        if (x0 < T) {
            const uint32_t mt = pair_mask(firstbits, M);
            const uint32_t t_u = as_u32(I - pk_eval<case_formula(FAM, K, TC_0Y, ucU)>(g));
            const uint32_t t_i = as_u32(I - pk_eval<case_formula(FAM, K, TC_0Y, ucI)>(g));
            const uint32_t rt = (t_u & mk) | (t_i & ~mk);
            res = (rt & mt) | (res & ~mt);
        }
    }
    return pk_zigzag(as_pk(res));
}

template <int FAM, int K, int T, bool TEMP, bool V0, bool FIRST>
__device__ __forceinline__ v4u vec_fast_row(const VecRows& rw, uint32_t u0bits, const LaneMasks& lm, int x0)
{
    if constexpr (pk_row_ok<FAM, K, TEMP, V0, FIRST>()) {
        uint32_t firstbits = 0;
        if constexpr (FIRST) {
#pragma unroll
            for (int j = 0; j < 8; ++j) firstbits |= (uint32_t)(x0 + j < T) << j;
        }
        v4u o;
        o.x = vec_pk_pair<FAM, K, T, V0, FIRST, 0>(rw, u0bits, firstbits, x0);
        o.y = vec_pk_pair<FAM, K, T, V0, FIRST, 1>(rw, u0bits, firstbits, x0);
        o.z = vec_pk_pair<FAM, K, T, V0, FIRST, 2>(rw, u0bits, firstbits, x0);
        o.w = vec_pk_pair<FAM, K, T, V0, FIRST, 3>(rw, u0bits, firstbits, x0);
        return o;
    }
    v4u o;
    o.x = vec_fast_pair<FAM, K, T, TEMP, V0, FIRST, 0>(rw, lm, x0);
    o.y = vec_fast_pair<FAM, K, T, TEMP, V0, FIRST, 1>(rw, lm, x0);
    o.z = vec_fast_pair<FAM, K, T, TEMP, V0, FIRST, 2>(rw, lm, x0);
    o.w = vec_fast_pair<FAM, K, T, TEMP, V0, FIRST, 3>(rw, lm, x0);
    return o;
}

template <int FAM, int K, int T, bool TEMP>
__device__ __forceinline__ v4u vec_slow_row(const VecRows& rw, int x0, int ty, int v)
{
    v4u o;
    o.x = vec_slow_px<FAM, K, T, TEMP, 0>(rw, x0, ty, v) | (vec_slow_px<FAM, K, T, TEMP, 1>(rw, x0, ty, v) << 16);
    o.y = vec_slow_px<FAM, K, T, TEMP, 2>(rw, x0, ty, v) | (vec_slow_px<FAM, K, T, TEMP, 3>(rw, x0, ty, v) << 16);
    o.z = vec_slow_px<FAM, K, T, TEMP, 4>(rw, x0, ty, v) | (vec_slow_px<FAM, K, T, TEMP, 5>(rw, x0, ty, v) << 16);
    o.w = vec_slow_px<FAM, K, T, TEMP, 6>(rw, x0, ty, v) | (vec_slow_px<FAM, K, T, TEMP, 7>(rw, x0, ty, v) << 16);
    return o;
}

// loader: row src_row of strip xs into ring slot slot_idx (WPR 1-KiB DMAs for
// the strip + one for the 16-pixel left halo); P ring rows have no halo
template <int WPR>
__device__ __forceinline__ void vdma_row(uint16_t* ring, int slot_idx, const uint16_t* f, int W, int src_row, int xs,
                                         int lane)
{
    constexpr int SW = WPR * 512;
    uint16_t* slot = ring + slot_idx * (kVHalo + SW);
    const uint16_t* srow = f + (size_t)src_row * W;
#pragma unroll
    for (int q = 0; q < WPR; ++q) {
        const int x = min(xs + q * 512 + lane * 8, W - 8);
        glds16(srow + x, slot + kVHalo + q * 512);
    }
    if (lane < kVHalo / 8) glds16(srow + (xs > 0 ? xs - kVHalo + lane * 8 : lane * 8), slot);
}

template <int WPR>
__device__ __forceinline__ void vdma_prev_row(uint16_t* pring, int pslot_idx, const uint16_t* pf, int W, int src_row,
                                              int xs, int lane)
{
    constexpr int SW = WPR * 512;
    uint16_t* slot = pring + pslot_idx * SW;
#pragma unroll
    for (int q = 0; q < WPR; ++q) {
        const int x = min(xs + q * 512 + lane * 8, W - 8);
        glds16(pf + (size_t)src_row * W + x, slot + q * 512);
    }
}

template <int WPR, int RS, bool TEMP>
__device__ __forceinline__ void vdma_step(uint16_t* ring, int R, int slot0, uint16_t* pring, int RP, int pslot0,
                                          const uint16_t* f, const uint16_t* pf, int W, int ys, int ye, int s, int xs,
                                          int lane)
{
#pragma unroll
    for (int i = 0; i < RS; ++i) {
        const int src = min(ys + s * RS + i, ye - 1);
        int si = slot0 + i;
        si = si >= R ? si - R : si;
        vdma_row<WPR>(ring, si, f, W, src, xs, lane);
        if constexpr (TEMP) {
            int pi = pslot0 + i;
            pi = pi >= RP ? pi - RP : pi;
            vdma_prev_row<WPR>(pring, pi, pf, W, src, xs, lane);
        }
    }
}

// One work item (frame, row piece, strip) of a vec workgroup: NCW compute
// waves (row group w / WPR, quarter w % WPR) + one loader wave (wave NCW).
template <int FAM, int K, int T, int WPR, int NCW, int RPW, int PD, bool TEMP>
__device__ __forceinline__ void vec_item(const FrameSet& p, uint16_t* ring, int R, uint16_t* pring, int RP,
                                         const uint16_t* f, const uint16_t* pf, uint16_t* outf, int xs, int ys, int ye,
                                         int wave, int lane)
{
    constexpr int SW = WPR * 512;
    constexpr int RG = NCW / WPR;  // rows computed side by side
    constexpr int RS = RG * RPW;   // rows per step
    constexpr int kLoadsPerStep = RS * (WPR + 1 + (TEMP ? WPR : 0));
    constexpr int kWait = kLoadsPerStep * (PD - 1) < 63 ? kLoadsPerStep * (PD - 1) : 63;
    static_assert(NCW % WPR == 0, "compute waves per row");
    constexpr int slot = kVHalo + SW;
    const bool loader = wave == NCW;
    const int nsteps = (ye - ys + RS - 1) / RS;
    auto adv = [](int v, int d, int m) { v += d; while (v >= m) v -= m; return v; };
    auto wrap = [&](int s) { return s < 0 ? s + R : s; };
    const int rg = wave / WPR, sub = wave - (wave / WPR) * WPR;
    const int xl = sub * 512 + lane * 8;  // lane's first pixel in the strip
    const int x0 = xs + xl;
    const bool lane_in = x0 < p.W;
    const bool full = xs + SW <= p.W;
    uint32_t u0bits = 0;
    LaneMasks lm{};
    int y = ys + rg, sy = 0, py = 0, vy = 0;
    int lslot = 0, lpslot = 0;
    if (!loader) {
        const int u0 = x0 % T;
#pragma unroll
        for (int j = 0; j < 8; ++j) u0bits |= (uint32_t)(((u0 + j) % T) == 0) << j;
        sy = y % R;
        py = TEMP ? y % RP : 0;
        vy = y % T;
    } else {
        const int r0 = max(0, ys - T - 1);
        int ps = r0 % R;
        for (int row = r0; row < ys; ++row) {
            vdma_row<WPR>(ring, ps, f, p.W, row, xs, lane);
            ps = ps + 1 == R ? 0 : ps + 1;
        }
        int slot0 = ys % R, pslot0 = TEMP ? ys % RP : 0;
        for (int s = 0; s < PD && s < nsteps; ++s) {
            vdma_step<WPR, RS, TEMP>(ring, R, slot0, pring, RP, pslot0, f, pf, p.W, ys, ye, s, xs, lane);
            slot0 = adv(slot0, RS, R);
            if (TEMP) pslot0 = adv(pslot0, RS, RP);
        }
        lslot = slot0;
        lpslot = pslot0;
    }
    lm = lane_masks(u0bits, x0, T);  // every lane of the wave (the loader's are unused)
    for (int s = 0; s < nsteps; ++s) {
        if (loader) {
            if (s + PD < nsteps) wait_vmcnt<kWait>();
            else wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();
        if (loader) {
            if (s + PD < nsteps) {
                vdma_step<WPR, RS, TEMP>(ring, R, lslot, pring, RP, lpslot, f, pf, p.W, ys, ye, s + PD, xs, lane);
                lslot = adv(lslot, RS, R);
                if (TEMP) lpslot = adv(lpslot, RS, RP);
            }
        } else {
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                if (y < ye && lane_in) {
                    const int h = kVHalo + xl;
                    VecRows rw;
                    load_win(ring + sy * slot + h, rw.r0);
                    load_win(ring + wrap(sy - 1) * slot + h, rw.r1);
                    load_win(ring + wrap(sy - T) * slot + h, rw.rT);
                    load_win(ring + wrap(sy - T - 1) * slot + h, rw.rT1);
                    if constexpr (TEMP) {
                        const v4u pv = *(const v4u*)(pring + py * SW + xl);
                        rw.p[0] = pv.x; rw.p[1] = pv.y; rw.p[2] = pv.z; rw.p[3] = pv.w;
                    }
                    v4u o;
                    if (y < T || !full) {
                        o = vec_slow_row<FAM, K, T, TEMP>(rw, x0, y / T, vy);
                    } else if (x0 < 512) {  // the strip that starts the frame: first lens column
                        o = vy == 0 ? vec_fast_row<FAM, K, T, TEMP, true, true>(rw, u0bits, lm, x0)
                                    : vec_fast_row<FAM, K, T, TEMP, false, true>(rw, u0bits, lm, x0);
                    } else {
                        o = vy == 0 ? vec_fast_row<FAM, K, T, TEMP, true, false>(rw, u0bits, lm, x0)
                                    : vec_fast_row<FAM, K, T, TEMP, false, false>(rw, u0bits, lm, x0);
                    }
                    __builtin_nontemporal_store(o, (v4u*)(outf + (size_t)y * p.W + x0));
                }
                y += RG;
                sy = adv(sy, RG, R);
                if (TEMP) py = adv(py, RG, RP);
                vy = adv(vy, RG, T);
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

template <int FAM, int K, int T, int WPR, int NCW, int RPW, int PD>
__global__ __launch_bounds__(NCW * 64 + 64) void predict_vec(FrameSet p, int rows_per_piece, int npiece, int nstrip,
                                                             int xcd_map, int R, int RP)
{
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    uint16_t* ring = lds;
    uint16_t* pring = lds + R * (kVHalo + WPR * 512);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // wave-uniform
    const size_t fs = (size_t)p.W * p.H;
    const int b = blockIdx.x;
    int strip, group;
    if (xcd_map) {
        const int q = b >> 3;
        strip = q % nstrip;
        group = (q / nstrip) * 8 + (b & 7);
    } else {
        strip = b % nstrip;
        group = b / nstrip;
    }
    const int piece = group % npiece;
    const int fz = group / npiece;
    if (fz >= p.nz) return;
    const int xs = strip * WPR * 512;
    const int ys = piece * rows_per_piece;
    const int ye = min(ys + rows_per_piece, p.H);
    if (ys >= ye) return;
    const uint16_t* f = p.in + (size_t)fz * fs;
    uint16_t* outf = p.out + (size_t)fz * fs;
    if (frame_temporal(p, fz))
        vec_item<FAM, K, T, WPR, NCW, RPW, PD, true>(p, ring, R, pring, RP, f, frame_prev(p, fz), outf, xs, ys, ye,
                                                     wave, lane);
    else
        vec_item<FAM, K, T, WPR, NCW, RPW, PD, false>(p, ring, R, pring, RP, f, nullptr, outf, xs, ys, ye, wave,
                                                      lane);
}

// ---- video volumes: frame pairs.  With the video bit, frame z is temporal
// when z0 + z is odd and its residual needs the RAW previous frame z - 1,
// which is the volume's own input: predict_vec reads it a second time (a
// third ring of P rows per temporal item: 6 B per temporal pixel).  A pair
// item codes the spatial frame z - 1 AND the temporal frame z of one (row
// piece, strip): the loader streams both frames' rows into two rings (A: frame
// z - 1, B: frame z), compute waves 0 .. NCW/2 - 1 code frame A, the others
// frame B, and a B wave takes its P pixels from ring A's row y, which is
// already there for frame A.  Every input pixel is read once: 4 B per pixel
// for the whole volume.
template <int FAM, int K, int T, int WPR, int NCW, int RPW, int PD>
__device__ __forceinline__ void vec_pair_item(const FrameSet& p, uint16_t* ringA, uint16_t* ringB, int R,
                                              const uint16_t* fA, const uint16_t* fB, uint16_t* outA, uint16_t* outB,
                                              int xs, int ys, int ye, int wave, int lane)
{
    constexpr int SW = WPR * 512;
    constexpr int NCWF = NCW / 2;   // compute waves per frame
    constexpr int RG = NCWF / WPR;  // rows of each frame computed side by side
    constexpr int RS = RG * RPW;    // rows of each frame per step
    constexpr int kLoadsPerStep = 2 * RS * (WPR + 1);
    constexpr int kWait = kLoadsPerStep * (PD - 1) < 63 ? kLoadsPerStep * (PD - 1) : 63;
    static_assert(NCW % 2 == 0 && NCWF % WPR == 0, "compute waves per frame and row");
    constexpr int slot = kVHalo + SW;
    const bool loader = wave == NCW;
    const int nsteps = (ye - ys + RS - 1) / RS;
    auto adv = [](int v, int d, int m) { v += d; while (v >= m) v -= m; return v; };
    auto wrap = [&](int s) { return s < 0 ? s + R : s; };
    const bool onB = wave >= NCWF;  // wave-uniform
    const int w = onB ? wave - NCWF : wave;
    const int rg = w / WPR, sub = w - (w / WPR) * WPR;
    const int xl = sub * 512 + lane * 8;
    const int x0 = xs + xl;
    const bool lane_in = x0 < p.W;
    const bool full = xs + SW <= p.W;
    uint16_t* ring = onB ? ringB : ringA;
    uint16_t* outf = onB ? outB : outA;
    uint32_t u0bits = 0;
    LaneMasks lm{};
    int y = ys + rg, sy = 0, vy = 0, lslot = 0;
    if (!loader) {
        const int u0 = x0 % T;
#pragma unroll
        for (int j = 0; j < 8; ++j) u0bits |= (uint32_t)(((u0 + j) % T) == 0) << j;
        sy = y % R;
        vy = y % T;
    } else {
        const int r0 = max(0, ys - T - 1);
        int ps = r0 % R;
        for (int row = r0; row < ys; ++row) {
            vdma_row<WPR>(ringA, ps, fA, p.W, row, xs, lane);
            vdma_row<WPR>(ringB, ps, fB, p.W, row, xs, lane);
            ps = ps + 1 == R ? 0 : ps + 1;
        }
        int slot0 = ys % R;
        for (int s = 0; s < PD && s < nsteps; ++s) {
#pragma unroll
            for (int i = 0; i < RS; ++i) {
                const int src = min(ys + s * RS + i, ye - 1);
                const int si = adv(slot0, i, R);
                vdma_row<WPR>(ringA, si, fA, p.W, src, xs, lane);
                vdma_row<WPR>(ringB, si, fB, p.W, src, xs, lane);
            }
            slot0 = adv(slot0, RS, R);
        }
        lslot = slot0;
    }
    lm = lane_masks(u0bits, x0, T);  // every lane of the wave (the loader's are unused)
    for (int s = 0; s < nsteps; ++s) {
        if (loader) {
            if (s + PD < nsteps) wait_vmcnt<kWait>();
            else wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();
        if (loader) {
            if (s + PD < nsteps) {
#pragma unroll
                for (int i = 0; i < RS; ++i) {
                    const int src = min(ys + (s + PD) * RS + i, ye - 1);
                    const int si = adv(lslot, i, R);
                    vdma_row<WPR>(ringA, si, fA, p.W, src, xs, lane);
                    vdma_row<WPR>(ringB, si, fB, p.W, src, xs, lane);
                }
                lslot = adv(lslot, RS, R);
            }
        } else {
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                if (y < ye && lane_in) {
                    const int h = kVHalo + xl;
                    VecRows rw;
                    load_win(ring + sy * slot + h, rw.r0);
                    load_win(ring + wrap(sy - 1) * slot + h, rw.r1);
                    load_win(ring + wrap(sy - T) * slot + h, rw.rT);
                    load_win(ring + wrap(sy - T - 1) * slot + h, rw.rT1);
                    v4u o;
                    if (onB) {  // temporal: P = frame A's raw pixels of this row
                        const v4u pv = *(const v4u*)(ringA + sy * slot + h);
                        rw.p[0] = pv.x; rw.p[1] = pv.y; rw.p[2] = pv.z; rw.p[3] = pv.w;
                        if (y < T || !full) o = vec_slow_row<FAM, K, T, true>(rw, x0, y / T, vy);
                        else if (x0 < 512)
                            o = vy == 0 ? vec_fast_row<FAM, K, T, true, true, true>(rw, u0bits, lm, x0)
                                        : vec_fast_row<FAM, K, T, true, false, true>(rw, u0bits, lm, x0);
                        else
                            o = vy == 0 ? vec_fast_row<FAM, K, T, true, true, false>(rw, u0bits, lm, x0)
                                        : vec_fast_row<FAM, K, T, true, false, false>(rw, u0bits, lm, x0);
                    } else {
                        if (y < T || !full) o = vec_slow_row<FAM, K, T, false>(rw, x0, y / T, vy);
                        else if (x0 < 512)
                            o = vy == 0 ? vec_fast_row<FAM, K, T, false, true, true>(rw, u0bits, lm, x0)
                                        : vec_fast_row<FAM, K, T, false, false, true>(rw, u0bits, lm, x0);
                        else
                            o = vy == 0 ? vec_fast_row<FAM, K, T, false, true, false>(rw, u0bits, lm, x0)
                                        : vec_fast_row<FAM, K, T, false, false, false>(rw, u0bits, lm, x0);
                    }
                    __builtin_nontemporal_store(o, (v4u*)(outf + (size_t)y * p.W + x0));
                }
                y += RG;
                sy = adv(sy, RG, R);
                vy = adv(vy, RG, T);
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

// pair u codes frames first + 2u (spatial) and first + 2u + 1 (temporal)
template <int FAM, int K, int T, int WPR, int NCW, int RPW, int PD>
__global__ __launch_bounds__(NCW * 64 + 64) void predict_vec_pair(FrameSet p, int rows_per_piece, int npiece,
                                                                  int nstrip, int xcd_map, int R, int first)
{
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    uint16_t* ringA = lds;
    uint16_t* ringB = lds + R * (kVHalo + WPR * 512);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // wave-uniform
    const size_t fs = (size_t)p.W * p.H;
    const int b = blockIdx.x;
    int strip, group;
    if (xcd_map) {
        const int q = b >> 3;
        strip = q % nstrip;
        group = (q / nstrip) * 8 + (b & 7);
    } else {
        strip = b % nstrip;
        group = b / nstrip;
    }
    const int piece = group % npiece;
    const int fzA = first + 2 * (group / npiece);
    if (fzA + 1 >= p.nz) return;
    const int xs = strip * WPR * 512;
    const int ys = piece * rows_per_piece;
    const int ye = min(ys + rows_per_piece, p.H);
    if (ys >= ye) return;
    vec_pair_item<FAM, K, T, WPR, NCW, RPW, PD>(p, ringA, ringB, R, p.in + (size_t)fzA * fs,
                                                p.in + (size_t)(fzA + 1) * fs, p.out + (size_t)fzA * fs,
                                                p.out + (size_t)(fzA + 1) * fs, xs, ys, ye, wave, lane);
}

// -------------------------------------------------------------- launchers --
// NCW compute waves + 1 loader wave per workgroup; PD steps of NCW*RPW rows in
// flight.  Ring rows live during a step: y-T-1 .. y+NCW*RPW-1 plus the PD
// steps being loaded: R >= NCW*RPW*(PD+1) + T + 1.
// tiles formulas are the heaviest: two rows per compute wave per step
// amortise the step barrier (tiles P4 0.28 -> 0.25 ms); angle / space run
// best with one row per wave and 3 steps of prefetch (deeper prefetch costs a
// workgroup of occupancy per CU and measured 5-8 % slower).
template <int FAM>
struct RingShape {
    static constexpr int NCW = 4;
    static constexpr int RPW = FAM == 0 ? 2 : 1;
    static constexpr int PD = FAM == 0 ? 2 : 3;
};

struct Plan {
    int R, RP, halo, rows_per_piece, npiece, nstrip, xcd_map, grid;
    size_t lds;
};

// Split each frame into npiece row pieces so that the items (copies x frames
// x pieces x strips) fill the resident workgroup slots about once: a piece
// re-reads only its T+1 priming rows, so fewer, taller pieces waste less
// (1.5 % at 2048 rows / 3 pieces vs 6 % for 256-row segments).  Pieces stay
// >= 2(T+1) rows.
// rs = rows per step, sw = strip width (pixels), halo = left halo pixels per slot
// rings = haloed row rings per workgroup (2 for the frame-pair kernel)
static hipError_t make_plan_shape(const FrameSet& p, const void* fn, int threads, int rs, int pd, int sw, int halo,
                                  int copies, Plan& pl, int rings = 1)
{
    const bool any_temporal = p.video && (p.nz > 1 || (p.z0 & 1));
    pl.R = rs * (pd + 1) + p.T + 1;
    pl.RP = any_temporal ? rs * (pd + 1) : 0;
    pl.halo = halo;
    pl.lds = ((size_t)rings * pl.R * (pl.halo + sw) + (size_t)pl.RP * sw) * sizeof(uint16_t);
    pl.nstrip = (p.W + sw - 1) / sw;
    const int ncw = rs;  // rows are padded to whole steps below
    int occ = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, threads, pl.lds);
    if (e != hipSuccess || occ <= 0) occ = 1;
    int dev = 0, ncu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
    const int resident = occ * ncu;
    const int cols = copies * p.nz * pl.nstrip;
    int npiece = std::max(1, resident / std::max(1, cols));
    npiece = std::min(npiece, std::max(1, p.H / (2 * (p.T + 1))));
    int rows = (p.H + npiece - 1) / npiece;
    rows = (rows + ncw - 1) / ncw * ncw;
    pl.rows_per_piece = rows;
    pl.npiece = (p.H + rows - 1) / rows;
    const int ngroups = p.nz * pl.npiece;
    pl.xcd_map = (ngroups % 8) == 0 && pl.nstrip > 1;
    pl.grid = ngroups * pl.nstrip;
    return hipSuccess;
}

static hipError_t make_plan(const FrameSet& p, const void* fn, int ncw, int rpw, int pd, int copies, Plan& pl)
{
    return make_plan_shape(p, fn, ncw * 64 + 64, ncw * rpw, pd, kStrip, p.T <= 15 ? 16 : 32, copies, pl);
}

static hipError_t launch_plan(const void* fn, FrameSet p, const Plan& pl, int ncw, int gy, hipStream_t st)
{
    p.halo = pl.halo;
    int a_rows = pl.rows_per_piece, a_np = pl.npiece, a_nstrip = pl.nstrip, a_x = pl.xcd_map, a_R = pl.R, a_RP = pl.RP;
    void* args[] = {(void*)&p, (void*)&a_rows, (void*)&a_np, (void*)&a_nstrip, (void*)&a_x, (void*)&a_R, (void*)&a_RP};
    hipError_t e = hipLaunchKernel(fn, dim3(pl.grid, gy), dim3(ncw * 64 + 64), args, pl.lds, st);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

static bool fast_ok(const FrameSet& p, int force_generic)
{
    return !force_generic && p.T <= kMaxFastT && (p.W % 8) == 0 && p.W >= 32;
}

// vectorised path shape per family (WPR waves per row = strip of WPR * 512
// pixels, NCW compute waves, RPW rows per compute wave and step, PD steps of
// prefetch).  Measured on config 3 (scripts/pred_probe.hip, profiles/r03_pred_probe*.jsonl):
// angle / space run their (packed, shift-free) formulas at copy speed with
// one 512-pixel strip, 4 compute waves, 3 steps ahead; the tiles formulas
// (shifted sums, 32-bit) need more waves per CU to hide their VALU chains:
// 1024-pixel strips, 8 compute waves (0.227 vs 0.251 ms, round-2 ring 0.236).
#ifndef LFM_VEC_PD
#define LFM_VEC_PD 3  // steps of prefetch, angle / space
#endif
#ifndef LFM_VEC_NCW
#define LFM_VEC_NCW 4  // compute waves, angle / space
#endif
#ifndef LFM_VEC_RPW
#define LFM_VEC_RPW 1  // rows per compute wave and step, angle / space
#endif
template <int FAM>
struct VecShape {
    static constexpr int WPR = FAM == 0 ? 2 : 1;
    static constexpr int NCW = FAM == 0 ? 8 : LFM_VEC_NCW;
    static constexpr int RPW = FAM == 0 ? 1 : LFM_VEC_RPW;
    static constexpr int PD = FAM == 0 ? 3 : LFM_VEC_PD;
};

template <int FAM, int K, int T, int WPR, int NCW, int RPW, int PD>
static hipError_t launch_vec_shape(const FrameSet& p, hipStream_t st)
{
    const void* fn = (const void*)predict_vec<FAM, K, T, WPR, NCW, RPW, PD>;
    Plan pl;
    hipError_t e = make_plan_shape(p, fn, NCW * 64 + 64, (NCW / WPR) * RPW, PD, WPR * 512, kVHalo, 1, pl);
    if (e != hipSuccess) return e;
    return launch_plan(fn, p, pl, NCW, 1, st);
}

// frame-pair shape (video volumes): NCW compute waves, NCW / 2 per frame
template <int FAM>
struct PairShape {
    static constexpr int WPR = 1;
    static constexpr int NCW = 8;
    static constexpr int RPW = 1;
    static constexpr int PD = 3;
};

// A video volume: its (spatial, temporal) frame pairs in one predict_vec_pair
// launch; a temporal frame 0 (z0 odd: its previous frame is p.prev) and an
// unpaired last spatial frame go through predict_vec on their own.
template <int FAM, int K, int T, int WPR, int NCW, int RPW, int PD>
static hipError_t launch_vec_pairs(const FrameSet& p, hipStream_t st)
{
    const size_t fs = (size_t)p.W * p.H;
    const int first = (p.z0 & 1) ? 1 : 0;
    const int npairs = (p.nz - first) / 2;
    using S = VecShape<FAM>;
    auto single = [&](int fz) -> hipError_t {
        FrameSet q = p;
        q.in = p.in + (size_t)fz * fs;
        q.out = p.out + (size_t)fz * fs;
        q.prev = fz ? p.in + (size_t)(fz - 1) * fs : p.prev;
        q.nz = 1;
        q.z0 = p.z0 + fz;
        return launch_vec_shape<FAM, K, T, S::WPR, S::NCW, S::RPW, S::PD>(q, st);
    };
    if (first) {
        if (hipError_t e = single(0)) return e;
    }
    if (npairs > 0) {
        const void* fn = (const void*)predict_vec_pair<FAM, K, T, WPR, NCW, RPW, PD>;
        FrameSet q = p;
        q.nz = npairs;  // planning unit: a pair
        q.video = 0;    // no P ring: frame A's ring holds the previous frame
        Plan pl;
        hipError_t e = make_plan_shape(q, fn, NCW * 64 + 64, (NCW / 2 / WPR) * RPW, PD, WPR * 512, kVHalo, 1, pl, 2);
        if (e != hipSuccess) return e;
        FrameSet a = p;
        a.halo = pl.halo;
        int a_rows = pl.rows_per_piece, a_np = pl.npiece, a_nstrip = pl.nstrip, a_x = pl.xcd_map, a_R = pl.R,
            a_first = first;
        void* args[] = {(void*)&a, (void*)&a_rows, (void*)&a_np, (void*)&a_nstrip, (void*)&a_x, (void*)&a_R,
                        (void*)&a_first};
        e = hipLaunchKernel(fn, dim3(pl.grid), dim3(NCW * 64 + 64), args, pl.lds, st);
        if (e != hipSuccess) return e;
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (first + 2 * npairs < p.nz) return single(p.nz - 1);
    return hipSuccess;
}

template <int FAM, int K>
static hipError_t launch_vec(const FrameSet& p, hipStream_t st)
{
    using S = VecShape<FAM>;
    using PS = PairShape<FAM>;
    const bool pairs = p.video && p.nz >= 2;
    if (p.T == 15) {
        if (pairs) return launch_vec_pairs<FAM, K, 15, PS::WPR, PS::NCW, PS::RPW, PS::PD>(p, st);
        return launch_vec_shape<FAM, K, 15, S::WPR, S::NCW, S::RPW, S::PD>(p, st);
    }
    if (pairs) return launch_vec_pairs<FAM, K, 13, PS::WPR, PS::NCW, PS::RPW, PS::PD>(p, st);
    return launch_vec_shape<FAM, K, 13, S::WPR, S::NCW, S::RPW, S::PD>(p, st);
}

static bool vec_ok(const FrameSet& p, int force_generic)
{
    return !force_generic && (p.T == 13 || p.T == 15) && (p.W % 8) == 0 && p.W >= 32;
}

template <int FAM, int K>
static hipError_t launch_k(const FrameSet& p, hipStream_t st, int force_generic)
{
    if (vec_ok(p, force_generic)) return launch_vec<FAM, K>(p, st);
    if (!fast_ok(p, force_generic)) {
        size_t total = (size_t)p.W * p.H * p.nz;
        int grid = (int)std::min<size_t>((total + 255) / 256, 256 * 16);
        hipLaunchKernelGGL((predict_generic<FAM, K>), dim3(grid), dim3(256), 0, st, p);
        return hipGetLastError();
    }
    using RS = RingShape<FAM>;
    const void* fn = (const void*)predict_ring<FAM, K, RS::NCW, RS::RPW, RS::PD>;
    Plan pl;
    hipError_t e = make_plan(p, fn, RS::NCW, RS::RPW, RS::PD, 1, pl);
    if (e != hipSuccess) return e;
    return launch_plan(fn, p, pl, RS::NCW, 1, st);
}

template <int FAM>
static hipError_t launch_cands(const FrameSet& p, hipStream_t st)
{
    using RS = RingShape<FAM>;
    const void* fn = (const void*)predict_cands<FAM, RS::NCW, RS::RPW, RS::PD>;
    Plan pl;
    hipError_t e = make_plan(p, fn, RS::NCW, RS::RPW, RS::PD, 7, pl);
    if (e != hipSuccess) return e;
    return launch_plan(fn, p, pl, RS::NCW, 7, st);
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

// probes (scripts/*_probe.hip) include this file for its kernels and
// launchers only: LFM_PREDICT_NO_ENTRY drops the C entry points below, which
// instantiate every kernel
#ifndef LFM_PREDICT_NO_ENTRY
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
    lfm::FrameSet p{d_in, d_prev, d_out, W, H, T, nframes, z0, video_bit & 1, 0};
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

extern "C" int lfm_hip_predict_candidates(const uint16_t* d_frame, uint16_t* d_out7, int W, int H, int T, int family,
                                          void* stream_)
{
    if (!d_frame || !d_out7 || W <= 0 || H <= 0 || T <= 0 || family < 0 || family > 2) return LFM_HIP_EINVAL;
    hipStream_t stream = (hipStream_t)stream_;
    lfm::FrameSet p{d_frame, nullptr, d_out7, W, H, T, 1, 0, 0, 0};
    if (!lfm::fast_ok(p, lfm_hip_force_generic())) {
        for (int k = 1; k <= 7; ++k) {
            const int rc = lfm_hip_predict(d_frame, nullptr, d_out7 + (size_t)(k - 1) * W * H, W, H, 1, T, family, k,
                                           0, 0, stream_);
            if (rc != LFM_HIP_OK) return rc;
        }
        return LFM_HIP_OK;
    }
    hipError_t e = hipErrorInvalidValue;
    switch (family) {
    case 0: e = lfm::launch_cands<0>(p, stream); break;
    case 1: e = lfm::launch_cands<1>(p, stream); break;
    case 2: e = lfm::launch_cands<2>(p, stream); break;
    }
    return e == hipSuccess ? LFM_HIP_OK : LFM_HIP_ERUNTIME;
}
#endif
