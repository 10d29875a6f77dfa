// lfm_unpredict.hip -- inverse predictor + unsymbolize on gfx950 (decode).
//
// Replaces the reference's inverse kernels / host loops (_unPredictorK_* in
// lfm_Predictors*.cu:1470-2739 / space :1349-2049 / angle :1416-2587, driven
// per frame from klb_imageIO.cpp:1748-1821).  Pixel (x, y) is
// I = (uint16)(r + pred) with r the unsymbolized residual and pred the
// forward formula of its (tile case, position case) evaluated on DECODED
// neighbours; tiles temporal frames (odd z of a video stack) add
// ((pred + P) >> 1) instead, P the decoded previous frame.  The angle / space
// temporal residual ((I - pred) + P) >> 1 drops a bit and is not invertible
// (the reference's inverse is wrong there too): error ENOTINV.
//
// Every neighbour is up and / or left (reach T+1), so one wave decodes a band
// of 64 rows as a skewed wavefront: lane r owns row y0 + r and handles column
// x = k - r at step k.  Row r - b has then advanced b columns further, so a
// neighbour (x - a, y - b) inside the band was produced a + b <= 2T steps ago:
// it is read from a 64-column LDS ring of that row.  Rows of earlier bands
// come from the output in memory.  All 64 rows move in lock step (one wave),
// so no barrier is needed; frames are independent (even frames first, then
// odd temporal frames on their decoded predecessors).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <climits>
#include <mutex>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "lfm_cases.h"
#include "lfm_hip.h"

namespace lfm {

constexpr int kRing = 64;  // columns kept per band row (>= 2T + 1 for T <= 31)

struct BandNb {
    const uint16_t* ring;  // this wave's ring: [64 rows][kRing]
    const uint16_t* out;   // decoded frame (rows of earlier bands)
    int W, T, x, y, r;
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
        const int rr = r + dy;
        if (rr >= 0) return ring[rr * kRing + ((x + dx) & (kRing - 1))];
        return out[(size_t)(y + dy) * W + (x + dx)];
    }
};

template <int FAM, int K, int TC, int UC, bool TEMP>
__device__ __forceinline__ int inv_case(BandNb& g, int r, int P)
{
    constexpr int F = case_formula(FAM, K, TC, UC);
    const int pr = eval_formula<F>(g);
    if constexpr (!TEMP) return r + pr;
    else if constexpr (F == F_Z) return r + P;
    else return r + ((pr + P) >> 1);
}

struct UnFrames {
    const uint16_t* sym;   // nz frames of symbols
    const uint16_t* prev;  // decoded frame before frame 0 (temporal frame 0) or null
    uint16_t* out;         // nz decoded frames
    int W, H, T, nz, z0, video;
    int first, step;       // this launch decodes local frames first, first + step, ...
    // band5 hand-over: a wait gives up after wait_ticks of the 100 MHz
    // real-time clock (or spin_limit polls: tests force a timeout), ORs
    // err_bit into *status (global memory) and from then on every wait of
    // that band returns at once; it also gives up as soon as any other band
    // has set the bit.  The launch that follows a band5 launch (the one-wave
    // kernel, `repair`) re-runs every frame when the bit is set.
    int spin_limit;
    unsigned err_bit;
    unsigned* status;
    uint64_t wait_ticks;
    int repair;            // unpredict_band only: run only if a band5 hand-over gave up
};
// status bits (the control block's word 0, reported to the caller)
constexpr unsigned kStBand5 = 1u;   // a band5 hand-over timed out (the frames are re-run)
// control block (hipMalloc'd, pooled): word 0 status, word 32 the band5
// ticket counter, words 33.. the band progress words (0 before the launch)
constexpr int kCtlTicket = 32, kCtlPos = 33;

template <int FAM, int K>
__global__ __launch_bounds__(64) void unpredict_band(UnFrames p)
{
    __shared__ uint16_t ring[64 * kRing];
    const int fz = p.first + (int)blockIdx.x * p.step;
    if (fz >= p.nz) return;
    // the re-run after a band5 launch (one wave per frame, 8 KiB of LDS, so
    // it is dispatched at once beside other work): nothing to do unless one
    // of that launch's hand-overs gave up
    if (p.repair && !(__hip_atomic_load(p.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & kStBand5)) return;
    const int r = threadIdx.x;
    const size_t fs = (size_t)p.W * p.H;
    const uint16_t* sym = p.sym + fz * fs;
    uint16_t* out = p.out + fz * fs;
    const bool temporal = p.video && ((p.z0 + fz) & 1);
    const uint16_t* prev = temporal ? (fz ? p.out + (fz - 1) * fs : p.prev) : nullptr;
    const int W = p.W, H = p.H, T = p.T;
    for (int y0 = 0; y0 < H; y0 += 64) {
        const int y = y0 + r;
        const bool row_ok = y < H;
        const int v = y % T, ty = y / T;
        int u = 0, tx = 0;  // x % T and x / T, advanced with x
        for (int k = 0; k < W + 63; ++k) {
            const int x = k - r;
            if (row_ok && x >= 0 && x < W) {
                BandNb g{ring, out, W, T, x, y, r};
                const int tc = tx == 0 ? (ty == 0 ? TC_00 : TC_0Y) : (ty == 0 ? TC_X0 : TC_XY);
                const int uc = u == 0 ? (v > 0 ? UC_COL : UC_CORNER) : (v == 0 ? UC_ROW : UC_IN);
                const int res = unsymbolize16(sym[(size_t)y * W + x]);
                const int P = temporal ? (int)prev[(size_t)y * W + x] : 0;
                int val = 0;
                if (temporal) {
                    switch (tc * 4 + uc) {
#define LFM_INV(TC_, UC_) case TC_ * 4 + UC_: val = inv_case<FAM, K, TC_, UC_, true>(g, res, P); break;
                    LFM_INV(0, 0) LFM_INV(0, 1) LFM_INV(0, 2) LFM_INV(0, 3)
                    LFM_INV(1, 0) LFM_INV(1, 1) LFM_INV(1, 2) LFM_INV(1, 3)
                    LFM_INV(2, 0) LFM_INV(2, 1) LFM_INV(2, 2) LFM_INV(2, 3)
                    LFM_INV(3, 0) LFM_INV(3, 1) LFM_INV(3, 2) LFM_INV(3, 3)
#undef LFM_INV
                    }
                } else {
                    switch (tc * 4 + uc) {
#define LFM_INV(TC_, UC_) case TC_ * 4 + UC_: val = inv_case<FAM, K, TC_, UC_, false>(g, res, P); break;
                    LFM_INV(0, 0) LFM_INV(0, 1) LFM_INV(0, 2) LFM_INV(0, 3)
                    LFM_INV(1, 0) LFM_INV(1, 1) LFM_INV(1, 2) LFM_INV(1, 3)
                    LFM_INV(2, 0) LFM_INV(2, 1) LFM_INV(2, 2) LFM_INV(2, 3)
                    LFM_INV(3, 0) LFM_INV(3, 1) LFM_INV(3, 2) LFM_INV(3, 3)
#undef LFM_INV
                    }
                }
                const uint16_t o = (uint16_t)val;
                ring[r * kRing + (x & (kRing - 1))] = o;
                out[(size_t)y * W + x] = o;
                if (++u == T) {
                    u = 0;
                    ++tx;
                }
            }
        }
        // the band's rows are read back from memory by the next band
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
}

// Same band wavefront with the latency taken out of a step: the previous
// band's last T+1 rows stay in LDS at full width (`top`, overwritten in place
// by this band's last T+1 rows: a column is rewritten at least 64 - 2(T+1)
// steps after its last reader, so T <= 30), and each lane's symbols are
// loaded 8 steps ahead (a register delay line).  No global load on the
// dependency chain of a step; 64 + (T+1) * W * 2 B of LDS per frame.
struct BandNb2 {
    const uint16_t* ring;  // [64 rows][kRing]
    const uint16_t* top;   // [T + 1 rows][W]: rows y0 - T - 1 .. y0 - 1
    int W, TT, x, r;
    template <int N>
    __device__ __forceinline__ int at() const
    {
        int dx = 0, dy = 0;
        if constexpr (N == NB_A) { dx = -1; }
        if constexpr (N == NB_B) { dy = -1; }
        if constexpr (N == NB_C) { dx = -1; dy = -1; }
        if constexpr (N == NB_AP) { dx = -(TT - 1); }
        if constexpr (N == NB_BP) { dy = -(TT - 1); }
        if constexpr (N == NB_CP) { dx = -(TT - 1); dy = -(TT - 1); }
        if constexpr (N == NB_AP1) { dx = -TT; }
        if constexpr (N == NB_BP1) { dy = -TT; }
        if constexpr (N == NB_ABP) { dx = -1; dy = -(TT - 1); }
        if constexpr (N == NB_BAP) { dx = -(TT - 1); dy = -1; }
        const int rr = r + dy;
        if (rr >= 0) return ring[rr * kRing + ((x + dx) & (kRing - 1))];
        return top[(TT + rr) * W + (x + dx)];
    }
};

template <int FAM, int K, int TC, int UC, bool TEMP>
__device__ __forceinline__ int inv_case2(BandNb2& g, int r, int P)
{
    constexpr int F = case_formula(FAM, K, TC, UC);
    const int pr = eval_formula<F>(g);
    if constexpr (!TEMP) return r + pr;
    else if constexpr (F == F_Z) return r + P;
    else return r + ((pr + P) >> 1);
}

template <int FAM, int K, bool TEMP>
__device__ __forceinline__ int inv_any2(BandNb2& g, int tc, int uc, int res, int P)
{
    switch (tc * 4 + uc) {
#define LFM_INV(TC_, UC_) case TC_ * 4 + UC_: return inv_case2<FAM, K, TC_, UC_, TEMP>(g, res, P);
    LFM_INV(0, 0) LFM_INV(0, 1) LFM_INV(0, 2) LFM_INV(0, 3)
    LFM_INV(1, 0) LFM_INV(1, 1) LFM_INV(1, 2) LFM_INV(1, 3)
    LFM_INV(2, 0) LFM_INV(2, 1) LFM_INV(2, 2) LFM_INV(2, 3)
    LFM_INV(3, 0) LFM_INV(3, 1) LFM_INV(3, 2) LFM_INV(3, 3)
#undef LFM_INV
    }
    return 0;
}

constexpr int kSymAhead = 8;

template <int FAM, int K, bool TEMP>
__device__ __forceinline__ void band2(const UnFrames& p, int fz, uint16_t* ring, uint16_t* top)
{
    const int r = threadIdx.x;
    const size_t fs = (size_t)p.W * p.H;
    const uint16_t* sym = p.sym + fz * fs;
    uint16_t* out = p.out + fz * fs;
    const uint16_t* prev = TEMP ? (fz ? p.out + (fz - 1) * fs : p.prev) : nullptr;
    const int W = p.W, H = p.H, T = p.T, TT = T + 1, tb = 64 - TT;
    for (int y0 = 0; y0 < H; y0 += 64) {
        const int y = y0 + r;
        const bool row_ok = y < H;
        const int v = y % T, ty = y / T;
        const uint16_t* srow = sym + (size_t)(row_ok ? y : 0) * W;
        const uint16_t* prow = TEMP ? prev + (size_t)(row_ok ? y : 0) * W : nullptr;
        uint16_t* orow = out + (size_t)(row_ok ? y : 0) * W;
        uint16_t* trow = top + (r >= tb ? r - tb : 0) * W;
        // delay line: sq[j] holds the symbol (and previous-frame pixel) of
        // column k - r for the step k = k0 + j of the current round
        uint32_t sq[kSymAhead];
#pragma unroll
        for (int j = 0; j < kSymAhead; ++j) {
            const int x = j - r;
            uint32_t sv = 0;
            if (row_ok && x >= 0 && x < W) {
                sv = srow[x];
                if (TEMP) sv |= (uint32_t)prow[x] << 16;
            }
            sq[j] = sv;
        }
        int u = 0, tx = 0;  // x % T and x / T, advanced with x
        for (int k0 = 0; k0 < W + 63; k0 += kSymAhead) {
#pragma unroll
            for (int j = 0; j < kSymAhead; ++j) {
                const int k = k0 + j;
                const int x = k - r;
                const uint32_t sv = sq[j];
                {  // the load for step k + kSymAhead (column x + kSymAhead)
                    const int xn = x + kSymAhead;
                    uint32_t nv = 0;
                    if (row_ok && xn >= 0 && xn < W) {
                        nv = srow[xn];
                        if (TEMP) nv |= (uint32_t)prow[xn] << 16;
                    }
                    sq[j] = nv;
                }
                if (row_ok && x >= 0 && x < W) {
                    BandNb2 g{ring, top, W, TT, x, r};
                    const int tc = tx == 0 ? (ty == 0 ? TC_00 : TC_0Y) : (ty == 0 ? TC_X0 : TC_XY);
                    const int uc = u == 0 ? (v > 0 ? UC_COL : UC_CORNER) : (v == 0 ? UC_ROW : UC_IN);
                    const int res = unsymbolize16(sv & 0xFFFFu);
                    const int val = inv_any2<FAM, K, TEMP>(g, tc, uc, res, TEMP ? (int)(sv >> 16) : 0);
                    const uint16_t o = (uint16_t)val;
                    ring[r * kRing + (x & (kRing - 1))] = o;
                    orow[x] = o;
                    if (r >= tb) trow[x] = o;
                    if (++u == T) {
                        u = 0;
                        ++tx;
                    }
                }
            }
        }
    }
}

// band3: the band2 wavefront with the step's dependency chain cut down to
// registers.  The neighbours one step away come from registers: A = this
// lane's previous result, B / C = row r - 1's previous / second-previous
// result moved over by a DPP lane shift (row 0 takes them from `top`); every
// other neighbour was produced at least T steps earlier and is read from LDS
// before the step's own writes.  Outside the first band and the first T + 63
// steps of a band every lane is in the interior tile case, so the four
// position-case formulas are all evaluated and one is selected per lane (no
// divergent case switch); edge steps evaluate all sixteen cases and select.
struct NbVals {
    int v[NB_COUNT];
    template <int N>
    __device__ __forceinline__ int at() const { return v[N]; }
};

template <int FAM, int K, int TC, int UC, bool TEMP>
__device__ __forceinline__ int inv_case3(NbVals& g, int r, int P)
{
    constexpr int F = case_formula(FAM, K, TC, UC);
    const int pr = eval_formula<F>(g);
    if constexpr (!TEMP) return r + pr;
    else if constexpr (F == F_Z) return r + P;
    else return r + ((pr + P) >> 1);
}

// the four position cases of tile case TC, evaluated branch-free and
// selected per lane (u = x % T, v = y % T)
template <int FAM, int K, int TC, bool TEMP>
__device__ __forceinline__ int inv_tile3(NbVals& g, int res, int P, int u, int v)
{
    const int vc = inv_case3<FAM, K, TC, UC_COL, TEMP>(g, res, P);
    const int vk = inv_case3<FAM, K, TC, UC_CORNER, TEMP>(g, res, P);
    const int vr = inv_case3<FAM, K, TC, UC_ROW, TEMP>(g, res, P);
    const int vi = inv_case3<FAM, K, TC, UC_IN, TEMP>(g, res, P);
    return u == 0 ? (v > 0 ? vc : vk) : (v == 0 ? vr : vi);
}

// every tile case (edge steps: x < T in some lane, or the frame's first band)
template <int FAM, int K, bool TEMP>
__device__ __forceinline__ int inv_edge3(NbVals& g, int res, int P, int u, int v, int tx, int ty, bool all_x)
{
    const int vxy = inv_tile3<FAM, K, TC_XY, TEMP>(g, res, P, u, v);
    const int vx0 = inv_tile3<FAM, K, TC_X0, TEMP>(g, res, P, u, v);
    if (all_x) return ty == 0 ? vx0 : vxy;  // no lane has x < T
    const int v0y = inv_tile3<FAM, K, TC_0Y, TEMP>(g, res, P, u, v);
    const int v00 = inv_tile3<FAM, K, TC_00, TEMP>(g, res, P, u, v);
    return tx == 0 ? (ty == 0 ? v00 : v0y) : (ty == 0 ? vx0 : vxy);
}

template <int FAM, int K, bool TEMP>
__device__ __forceinline__ void band3(const UnFrames& p, int fz, uint16_t* ring, uint16_t* top)
{
    const int r = threadIdx.x;
    const size_t fs = (size_t)p.W * p.H;
    const uint16_t* sym = p.sym + fz * fs;
    uint16_t* out = p.out + fz * fs;
    const uint16_t* prev = TEMP ? (fz ? p.out + (fz - 1) * fs : p.prev) : nullptr;
    const int W = p.W, H = p.H, T = p.T, TT = T + 1, tb = 64 - TT;
    // LDS offset (u16 units, relative to ring) of neighbour (x + dx, y + dy)
    auto far = [&](int x, int dx, int dy) -> int {
        const int rr = r + dy;
        return rr >= 0 ? rr * kRing + ((x + dx) & (kRing - 1)) : 64 * kRing + (TT + rr) * W + (x + dx);
    };
    for (int y0 = 0; y0 < H; y0 += 64) {
        const int y = y0 + r;
        const bool row_ok = y < H;
        const int v = y % T, ty = y / T;
        const uint16_t* srow = sym + (size_t)(row_ok ? y : 0) * W;
        const uint16_t* prow = TEMP ? prev + (size_t)(row_ok ? y : 0) * W : nullptr;
        uint16_t* orow = out + (size_t)(row_ok ? y : 0) * W;
        uint16_t* trow = top + (r >= tb ? r - tb : 0) * W;
        const uint16_t* btop = top + (TT - 1) * W;  // the previous band's last row (row 0's B and C)
        // delay lines: symbol (and previous-frame pixel) of column k - r for
        // the step k = k0 + j of the current round
        uint32_t sq[kSymAhead], pq[kSymAhead];
#pragma unroll
        for (int j = 0; j < kSymAhead; ++j) {
            const int x = min(max(j - r, 0), W - 1);
            sq[j] = srow[x];
            pq[j] = TEMP ? prow[x] : 0u;
        }
        int u = 0, tx = 0;  // x % T and x / T, advanced with x
        int p1 = 0, p2 = 0; // this lane's results of the last two steps
        // far neighbours of column x (B / C slots: row 0's values from `top`)
        auto load_far = [&](NbVals& f, int x) {
            f.v[NB_B] = r == 0 && x >= 0 ? (int)btop[x] : 0;
            f.v[NB_C] = r == 0 && x >= 1 ? (int)btop[x - 1] : 0;
            f.v[NB_AP] = ring[far(x, -T, 0)];
            f.v[NB_BP] = ring[far(x, 0, -T)];
            f.v[NB_CP] = ring[far(x, -T, -T)];
            f.v[NB_AP1] = ring[far(x, -TT, 0)];
            f.v[NB_BP1] = ring[far(x, 0, -TT)];
            f.v[NB_ABP] = ring[far(x, -1, -T)];
            f.v[NB_BAP] = ring[far(x, -T, -1)];
        };
        NbVals nf;
        nf.v[NB_A] = 0;
        load_far(nf, -r);
        const int edge_k = T + 63;  // before this step some lane has x < T
        for (int k0 = 0; k0 < W + 63; k0 += kSymAhead) {
#pragma unroll
            for (int j = 0; j < kSymAhead; ++j) {
                const int k = k0 + j;
                const int x = k - r;
                const uint32_t sv = sq[j], pv = pq[j];
                {  // the loads for step k + kSymAhead (column x + kSymAhead):
                    // clamped and unconditional, so their wait lands at their use
                    const int xn = min(max(x + kSymAhead, 0), W - 1);
                    sq[j] = srow[xn];
                    if (TEMP) pq[j] = prow[xn];
                }
                const bool ok = row_ok && x >= 0 && x < W;
                // this step's far neighbours were read during the last step
                // (T >= 2: nothing they need is written by that step)
                NbVals g = nf;
                load_far(nf, x + 1);
                g.v[NB_A] = p1;
                g.v[NB_B] = __builtin_amdgcn_update_dpp(g.v[NB_B], p1, 0x138, 0xF, 0xF, false);
                g.v[NB_C] = __builtin_amdgcn_update_dpp(g.v[NB_C], p2, 0x138, 0xF, 0xF, false);
                const int res = unsymbolize16(sv);
                const int P = TEMP ? (int)pv : 0;
                int val;
                if (k >= edge_k && y0 > 0) val = inv_tile3<FAM, K, TC_XY, TEMP>(g, res, P, u, v);
                else val = inv_edge3<FAM, K, TEMP>(g, res, P, u, v, tx, ty, k >= edge_k);
                const uint16_t o = (uint16_t)val;
                if (ok) {
                    ring[r * kRing + (x & (kRing - 1))] = o;
                    orow[x] = o;
                    if (r >= tb) trow[x] = o;
                    if (++u == T) {
                        u = 0;
                        ++tx;
                    }
                }
                p2 = p1;
                p1 = (int)o;
            }
        }
    }
}

// band4: band3 with the bands of a frame pipelined over NW waves of one
// workgroup (wave w takes bands w, w + NW, ...).  Each wave publishes its
// progress (band * stride + steps done) in LDS every kSync steps, after its
// global stores have completed.  The rows a band needs from the band above
// (its last T+1 rows) are read from the output in memory, a round of kSync
// columns at a time, two rounds ahead of their use (workgroup-scope loads: the
// waves share the CU's write-through L1), into a private LDS ring of kHand
// columns: a
// wave only ever waits for the band above to be far enough ahead, so the
// waits form a chain from the first band down and cannot deadlock.
constexpr int kHand = 128;
constexpr int kSync = 32;

// XCU (cross-CU, band5 below): every band is its own workgroup, so `pos` lives
// in global memory and the progress words and the hand-over loads of the band
// above's rows use agent scope instead of workgroup scope.  The hand-over is
// write-through instead of fenced: every output store is a 16-byte `sc1`
// buffer store, drained (`s_waitcnt vmcnt(0)`) before the progress word (an
// `sc1` store) is written, and every load of another band's rows is an `sc1`
// load to registers, so neither side needs an agent-scope fence (a release
// fence is `buffer_wbl2 sc1`, a write-back of the XCD's whole L2, an acquire
// `buffer_inv sc1`; band5 issued both every 32 steps of every band).
template <int FAM, int K, bool TEMP, bool XCU = false>
__device__ __forceinline__ void band4(const UnFrames& p, int fz, int NW, int wv, uint16_t* lds, int ring_off,
                                      int hand_off, int* pos)
{
    constexpr int kScope = XCU ? __HIP_MEMORY_SCOPE_AGENT : __HIP_MEMORY_SCOPE_WORKGROUP;
    const int r = threadIdx.x & 63;
    const size_t fs = (size_t)p.W * p.H;
    const uint16_t* sym = p.sym + fz * fs;
    uint16_t* out = p.out + fz * fs;
    // write-through stores of the frame (XCU): one descriptor per wave over
    // the frame, built from wave-uniform values only
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        out, /*stride*/ 0, (int)__builtin_amdgcn_readfirstlane((int)(fs * sizeof(uint16_t))), 0x00020000);
    const uint16_t* prev = TEMP ? (fz ? p.out + (fz - 1) * fs : p.prev) : nullptr;
    const int W = p.W, H = p.H, T = p.T, TT = T + 1;
    const int nbands = (H + 63) / 64, kend = W + 63, stride = W + 64 + 3 * kSync;
    const int prodw = (wv + NW - 1) % NW;
    // (bounded in time: a wait that gives up sets its bit in *p.status -- the
    // frames of a band5 launch are then re-run on the device -- and the band
    // runs on without waiting; never a hang.)  Progress is monotonic, so a
    // stale read can only under-report it: it delays a band, never releases
    // one early.
    // XCU: `seen` is the producer's progress as last read; a read is issued
    // after every wait and consumed at the next one (a round later, so it has
    // returned), and a wait that `seen` already satisfies costs no load
    int seen = -1, pending = -1;
    bool dead = false;  // this band gave up waiting: later waits return at once
    auto wait_ge = [&](int need) {
        if constexpr (XCU) seen = max(seen, __builtin_amdgcn_readfirstlane(pending));
        if (seen < need && !dead) {
            const uint64_t t0 = (uint64_t)wall_clock64();
            for (int spin = 1;; ++spin) {
                seen = __builtin_amdgcn_readfirstlane(__hip_atomic_load(pos + prodw, __ATOMIC_RELAXED, kScope));
                if (seen >= need) break;
                if (spin >= p.spin_limit) {
                    dead = true;
                    break;
                }
                if ((spin & 63) == 0) {
                    if constexpr (XCU) {
                        // another band gave up: this launch is re-run anyway
                        if (__builtin_amdgcn_readfirstlane(
                                __hip_atomic_load(p.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) & p.err_bit) {
                            dead = true;
                            break;
                        }
                        // a long wait also drops this CU's cached lines (an
                        // agent acquire), so no cache level can keep serving
                        // an old progress word
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    }
                    if ((uint64_t)wall_clock64() - t0 > p.wait_ticks) {
                        dead = true;
                        break;
                    }
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (dead && r == 0)
                __hip_atomic_fetch_or(p.status, p.err_bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if constexpr (XCU) pending = __hip_atomic_load(pos + prodw, __ATOMIC_RELAXED, kScope);
        // XCU: every later load of the band above's rows is an sc1 load
        // (hload), so this only keeps the compiler from hoisting them
        if constexpr (XCU) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    auto far = [&](int x, int dx, int dy) -> int {
        const int rr = r + dy;
        return rr >= 0 ? ring_off + rr * kRing + ((x + dx) & (kRing - 1))
                       : hand_off + (TT + rr) * kHand + ((x + dx) & (kHand - 1));
    };
    const int btop = hand_off + (TT - 1) * kHand;
    // hand-over loader: lane l takes row l / 2 of the band above's last TT
    // rows and 8 column pairs of a kSync-column round
    const int hr = r >> 1, hc = (r & 1) * 16;
    const bool hl = hr < TT;
    uint32_t hv[8];
    for (int b = wv; b < nbands; b += NW) {
        const int y0 = b * 64;
        const int y = y0 + r;
        const bool row_ok = y < H;
        const int v = y % T, ty = y / T;
        const uint32_t* hsrc = (const uint32_t*)(out + (size_t)(b > 0 && hl ? y0 - TT + hr : 0) * W);
        auto hload = [&](int c0) {  // columns c0 + hc .. + 16 of the round starting at column c0
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int c = min(c0 + hc + 2 * q, W - 2);
                hv[q] = __hip_atomic_load(hsrc + (c >> 1), __ATOMIC_RELAXED, kScope);
            }
        };
        auto hstore = [&](int c0) {
            if (hl) {
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    *(uint32_t*)(lds + hand_off + hr * kHand + ((c0 + hc + 2 * q) & (kHand - 1))) = hv[q];
            }
        };
        // Memory operations are the same for every lane and every round of 8
        // steps, so the compiler's waits count exactly and none waits for a
        // fresh operation: lane r handles columns k0 - r .. k0 - r + 7 in the
        // round starting at step k0, i.e. the aligned 8-column groups g0 and
        // g0 + 1 (g0 = (k0 - r) >> 3, one more per round).  Symbols (and
        // previous-frame pixels) sit in a window of four groups G[q & 3] =
        // group g0 + (slot - q) loaded 3 rounds (24 steps) ahead; the 4 rounds
        // of a kSync round are unrolled so the window never moves between
        // registers.  A round starts by storing group g0 - 1 (complete) from
        // this row's LDS ring with one 16-byte store.  Lanes outside the frame
        // get an out-of-range buffer offset: the hardware drops the store and
        // returns zeros for the load.
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const int ng = W / 8;
        const uint32_t sbytes = (uint32_t)__builtin_amdgcn_readfirstlane((int)(fs * sizeof(uint16_t)));
        const __amdgpu_buffer_rsrc_t srsrc = __builtin_amdgcn_make_buffer_rsrc((void*)sym, 0, (int)sbytes, 0x00020000);
        const __amdgpu_buffer_rsrc_t prsrc =
            __builtin_amdgcn_make_buffer_rsrc((void*)(TEMP ? prev : sym), 0, (int)sbytes, 0x00020000);
        constexpr uint32_t kNoOff = 0x7FFFFFF0u;  // past every frame: dropped store / zero load
        auto goff = [&](int g) -> int {         // byte offset of group g of this lane's row
            return (row_ok && g >= 0 && g < ng) ? (int)(((uint32_t)y * (uint32_t)W + 8u * (uint32_t)g) * 2u) : (int)kNoOff;
        };
        auto gload = [&](const __amdgpu_buffer_rsrc_t& rs, int g) -> u32x4 {
            return __builtin_amdgcn_raw_buffer_load_b128(rs, goff(g), 0, 0);
        };
        const int gbase = (0 - r) >> 3;  // g0 of the first round (floor)
        u32x4 G[4], Pg[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            G[q] = gload(srsrc, gbase + q);
            if (TEMP) Pg[q] = gload(prsrc, gbase + q);
        }
        const int ph = (-r) & 7;  // column offset of step 0 of a round inside group g0
        int u = 0, tx = 0;
        int p1 = 0, p2 = 0;
        auto load_far = [&](NbVals& f, int x) {
            f.v[NB_B] = r == 0 && x >= 0 ? (int)lds[btop + (x & (kHand - 1))] : 0;
            f.v[NB_C] = r == 0 && x >= 1 ? (int)lds[btop + ((x - 1) & (kHand - 1))] : 0;
            f.v[NB_AP] = lds[far(x, -T, 0)];
            f.v[NB_BP] = lds[far(x, 0, -T)];
            f.v[NB_CP] = lds[far(x, -T, -T)];
            f.v[NB_AP1] = lds[far(x, -TT, 0)];
            f.v[NB_BP1] = lds[far(x, 0, -TT)];
            f.v[NB_ABP] = lds[far(x, -1, -T)];
            f.v[NB_BAP] = lds[far(x, -T, -1)];
        };
        if (b > 0) {  // the first two rounds' columns of the band above
            wait_ge((b - 1) * stride + min(kSync + 72, kend));
            hload(0);
            hstore(0);
        }
        NbVals nf;
        nf.v[NB_A] = 0;
        load_far(nf, -r);
        const int edge_k = T + 63;  // before this step some lane has x < T
        // the last round (k0 = W + 64) only stores every row's last group
        for (int ks = 0; ks < W + 72; ks += kSync) {
            {
                // every store issued before the last round has completed: the
                // pixels of steps < ks - 24 are in memory (a pixel of step s is
                // stored by the round starting at <= s + 15)
                if constexpr (XCU) {
                    if constexpr (TEMP) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                } else {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __builtin_amdgcn_s_waitcnt(0);
                }
                if (r == 0) __hip_atomic_store(pos + wv, b * stride + ks - 24, __ATOMIC_RELAXED, kScope);
                if (b > 0) {  // stored into the LDS ring at the end of this round
                    wait_ge((b - 1) * stride + min(ks + 2 * kSync + 72, kend));
                    hload(ks + kSync);
                }
            }
#pragma unroll
            for (int q = 0; q < kSync / 8; ++q) {
                const int k0 = ks + 8 * q;
                const int g0 = (k0 - r) >> 3;
                asm volatile("" ::: "memory");  // keeps each round's memory operations in their round
                {   // group g0 - 1 is complete: LDS ring -> one 16-byte store
                    const int gs = g0 - 1;
                    const u32x4 ov4 = *(const u32x4*)(lds + ring_off + r * kRing + ((8 * gs) & (kRing - 1)));
                    __builtin_amdgcn_raw_buffer_store_b128(ov4, orsrc, goff(gs), 0, XCU ? 16 /*sc1*/ : 0);
                }
                const u32x4 Ga = G[q & 3], Gb = G[(q + 1) & 3];
                const u32x4 Pa = TEMP ? Pg[q & 3] : Ga, Pb = TEMP ? Pg[(q + 1) & 3] : Gb;
                if (k0 < kend) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int k = k0 + j;
                        const int x = k - r;
                        const int o = ph + j;  // 0..14: column of the pair (Ga, Gb)
                        auto pick = [&](const u32x4& qa, const u32x4& qb) {  // two 64-bit halves and a shift
                            const bool hi = o >= 8;
                            const uint32_t w0 = hi ? qb.x : qa.x, w1 = hi ? qb.y : qa.y;
                            const uint32_t w2 = hi ? qb.z : qa.z, w3 = hi ? qb.w : qa.w;
                            const uint64_t lo64 = ((uint64_t)w1 << 32) | w0, hi64 = ((uint64_t)w3 << 32) | w2;
                            return (uint32_t)((((o & 4) ? hi64 : lo64) >> (16 * (o & 3)))) & 0xFFFFu;
                        };
                        const uint32_t sv = pick(Ga, Gb), pv = TEMP ? pick(Pa, Pb) : 0u;
                        const bool ok = row_ok && x >= 0 && x < W;
                        NbVals g = nf;
                        load_far(nf, x + 1);
                        g.v[NB_A] = p1;
                        g.v[NB_B] = __builtin_amdgcn_update_dpp(g.v[NB_B], p1, 0x138, 0xF, 0xF, false);
                        g.v[NB_C] = __builtin_amdgcn_update_dpp(g.v[NB_C], p2, 0x138, 0xF, 0xF, false);
                        const int res = unsymbolize16(sv);
                        const int P = TEMP ? (int)pv : 0;
                        int val;
                        if (k >= edge_k && y0 > 0) val = inv_tile3<FAM, K, TC_XY, TEMP>(g, res, P, u, v);
                        else val = inv_edge3<FAM, K, TEMP>(g, res, P, u, v, tx, ty, k >= edge_k);
                        const uint16_t o16 = (uint16_t)val;
                        if (ok) {
                            lds[ring_off + r * kRing + (x & (kRing - 1))] = o16;
                            if (++u == T) {
                                u = 0;
                                ++tx;
                            }
                        }
                        p2 = p1;
                        p1 = (int)o16;
                    }
                }
                // group g0 is used up: its slot takes group g0 + 4
                G[q & 3] = gload(srsrc, g0 + 4);
                if (TEMP) Pg[q & 3] = gload(prsrc, g0 + 4);
                // the hand-over columns loaded at the start of this round
                // (24 steps ago) are first read (lanes r <= T, one step ahead)
                // at step ks + kSync - 1; their ring slots held columns
                // < ks - 64, no longer read
                if (q == kSync / 8 - 2 && b > 0) hstore(ks + kSync);
            }
        }
        // every row's groups are stored: drain, then the band is complete
        if constexpr (XCU) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_s_waitcnt(0);
        }
        if (r == 0) __hip_atomic_store(pos + wv, b * stride + kend, __ATOMIC_RELAXED, kScope);
    }
}

// band5: the band pipeline spread over the whole chip -- one single-wave
// workgroup per (band, frame).  HIP promises neither a dispatch order nor a
// workgroup -> XCD placement, so a workgroup does not take its band from
// blockIdx: its first act is to draw a ticket (an agent-scope atomic add on
// the control block) and it decodes band ticket / nfr of frame ticket % nfr.
// Tickets go out in the order the workgroups actually started, so the band a
// workgroup waits for (ticket - nfr) belongs to a workgroup that is already
// resident, and the chain of waits always ends at a running band 0, wherever
// and whenever the workgroups were placed.  Progress words (one per band, 0
// before the launch) live in the same hipMalloc'd control block: bands
// publish with write-through (sc1) stores after draining their pixel stores
// and poll with sc1 loads (MI355X_MICROARCH.md, visibility, write-through
// form).  Config 3: 2048 waves over 256 CUs instead of 64 workgroups of 8
// waves on 64 CUs.
template <int FAM, int K>
__global__ __launch_bounds__(64) void unpredict_band5(UnFrames p, int* ctl, int nbands, int nfr)
{
    extern __shared__ __attribute__((aligned(16))) uint16_t lds5[];
    int t = 0;
    if (threadIdx.x == 0) t = __hip_atomic_fetch_add(ctl + kCtlTicket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t = __builtin_amdgcn_readfirstlane(t);
    const int b = t / nfr, fi = t - b * nfr;
    const int fz = p.first + fi * p.step;
    if (fz >= p.nz || b >= nbands) return;  // (the grid is exactly nbands * nfr)
    int* pos = ctl + kCtlPos + (size_t)fi * nbands;
    if (p.video && ((p.z0 + fz) & 1)) band4<FAM, K, true, true>(p, fz, nbands, b, lds5, 0, 64 * kRing, pos);
    else band4<FAM, K, false, true>(p, fz, nbands, b, lds5, 0, 64 * kRing, pos);
}

template <int FAM, int K>
__global__ __launch_bounds__(64) void unpredict_band3(UnFrames p)
{
    extern __shared__ __attribute__((aligned(16))) uint16_t lds3[];
    const int fz = p.first + (int)blockIdx.x * p.step;
    if (fz >= p.nz) return;
    uint16_t* ring = lds3;
    uint16_t* top = lds3 + 64 * kRing;
    if (p.video && ((p.z0 + fz) & 1)) band3<FAM, K, true>(p, fz, ring, top);
    else band3<FAM, K, false>(p, fz, ring, top);
}

template <int FAM, int K>
__global__ __launch_bounds__(64) void unpredict_band2(UnFrames p)
{
    extern __shared__ __attribute__((aligned(16))) uint16_t lds2[];
    const int fz = p.first + (int)blockIdx.x * p.step;
    if (fz >= p.nz) return;
    uint16_t* ring = lds2;
    uint16_t* top = lds2 + 64 * kRing;
    if (p.video && ((p.z0 + fz) & 1)) band2<FAM, K, true>(p, fz, ring, top);
    else band2<FAM, K, false>(p, fz, ring, top);
}

static size_t band2_lds(const UnFrames& p) { return (size_t)(64 * kRing + (p.T + 1) * p.W) * sizeof(uint16_t); }

static bool band2_ok(const UnFrames& p)
{
    return p.T <= 30 && band2_lds(p) <= 160 * 1024;
}

// waves per frame for band4 (0: not applicable; rows are read and written in
// aligned 8-column groups, so W is a multiple of 8)
static int band4_waves(const UnFrames& p)
{
    // (band4 / band5 address a frame through 31-bit buffer offsets)
    if (p.T < 2 || p.T > 30 || (p.W & 7) || (size_t)p.W * p.H * 2 >= 0x7FFFFFF0u) return 0;
    const int nw = std::min(8, (p.H + 63) / 64);
    return nw >= 2 ? nw : 0;
}

// Hand-over limits.  LFM_UNPREDICT_WAIT_MS (default 500): a band5 wait
// gives up after that long on the device's 100 MHz real-time clock.
// LFM_UNPREDICT_SPIN (tests): band5 waits give up after that many polls.
// LFM_UNPREDICT_FALLBACK=0: a band5 timeout is reported as an error instead of
// re-running the frames.  Read per call (tests set them in the
// process).
static int band5_spin_limit()
{
    const char* e = std::getenv("LFM_UNPREDICT_SPIN");
    return e ? std::max(1, std::atoi(e)) : INT_MAX;
}

static bool fallback_enabled()
{
    const char* f = std::getenv("LFM_UNPREDICT_FALLBACK");
    return !(f && std::atoi(f) == 0);
}

static uint64_t wait_ticks()
{
    const char* e = std::getenv("LFM_UNPREDICT_WAIT_MS");
    const long ms = e ? std::max(1l, std::atol(e)) : 500l;
    int khz = 0, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
        khz <= 0)
        khz = 100000;  // the gfx9 real-time clock: 100 MHz
    return (uint64_t)khz * (uint64_t)ms;
}

// Control blocks: device words (hipMalloc) for the status, the band5 ticket
// and the progress words.  A block is handed to one call at a time and taken
// again only once the event recorded behind that call's last use has fired,
// so concurrent decodes on several streams never share progress words.  (A
// stream-ordered pool allocation per launch -- hipMallocAsync / hipFreeAsync,
// round 5 -- gave no such guarantee across streams and is not the memory
// type whose cross-XCD behaviour MI355X_MICROARCH.md measured.)
struct CtlBlock {
    int dev = -1;
    int* d = nullptr;
    size_t words = 0;
    hipEvent_t done = nullptr;
    bool busy = false;
};

static std::mutex& ctl_mu()
{
    static std::mutex m;
    return m;
}

static std::vector<CtlBlock*>& ctl_pool()
{
    static std::vector<CtlBlock*> v;  // (process lifetime: a handful per device)
    return v;
}

static CtlBlock* ctl_acquire(size_t words)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(ctl_mu());
    CtlBlock* got = nullptr;
    int mine = 0;
    for (CtlBlock* c : ctl_pool()) {
        if (c->dev != dev) continue;
        ++mine;
        if (!c->busy && c->words >= words && hipEventQuery(c->done) == hipSuccess) {
            got = c;
            break;
        }
    }
    (void)hipGetLastError();  // (a pending event's hipErrorNotReady)
    if (!got && mine >= 64) {  // bounded pool: wait for the first idle block of the size
        for (CtlBlock* c : ctl_pool())
            if (c->dev == dev && !c->busy && c->words >= words && hipEventSynchronize(c->done) == hipSuccess) {
                got = c;
                break;
            }
    }
    if (!got) {
        got = new CtlBlock;
        got->dev = dev;
        got->words = std::max<size_t>(words, 1 << 16);
        if (hipMalloc((void**)&got->d, got->words * sizeof(int)) != hipSuccess ||
            hipEventCreateWithFlags(&got->done, hipEventDisableTiming) != hipSuccess) {
            if (got->d) (void)hipFree(got->d);
            (void)hipGetLastError();
            delete got;
            return nullptr;
        }
        ctl_pool().push_back(got);
    }
    got->busy = true;
    return got;
}

static void ctl_release(CtlBlock* c, hipStream_t st)
{
    std::lock_guard<std::mutex> lk(ctl_mu());
    (void)hipEventRecord(c->done, st);
    c->busy = false;
}

template <int FAM, int K_>
static hipError_t launch_band2(const UnFrames& p, int grid, hipStream_t st, int* ctl)
{
    if (band4_waves(p)) {
        const int nbands = (p.H + 63) / 64;
        const size_t lds = (size_t)(64 * kRing + (p.T + 1) * kHand) * 2;
        // ticket and progress words of this launch start at 0 (every wait
        // needs a progress > 0); the status word accumulates over the call
        hipError_t e = hipMemsetAsync(ctl + kCtlTicket, 0, (size_t)(1 + grid * nbands) * sizeof(int), st);
        UnFrames pt = p;
        pt.status = (unsigned*)ctl;
        pt.err_bit = kStBand5;
        pt.spin_limit = band5_spin_limit();
        pt.repair = 0;
        if (e == hipSuccess) {
            hipLaunchKernelGGL((unpredict_band5<FAM, K_>), dim3(grid * nbands), dim3(64), lds, st, pt, ctl, nbands,
                               grid);
            e = hipGetLastError();
        }
        // re-run on the device, no host round trip: a band that gave up
        // decoded from rows that were not ready, so when the status word
        // carries kStBand5 every frame of the launch runs again through the
        // one-wave kernel (a frame's bands are one wave's loop: nothing to
        // wait for); otherwise its waves return at once.  (The round-5 re-run
        // was band4 -- 512 threads and up to 129 KiB of LDS per frame -- whose
        // launch waited up to 9 ms for CUs held by the other decode slot's
        // bzip2 kernels even when it had nothing to do.)
        if (e == hipSuccess && fallback_enabled()) {
            UnFrames pr = p;
            pr.status = (unsigned*)ctl;
            pr.err_bit = 0;
            pr.repair = 1;
            hipLaunchKernelGGL((unpredict_band<FAM, K_>), dim3(grid), dim3(64), 0, st, pr);
            e = hipGetLastError();
        }
        return e;
    }
    const size_t lds = band2_lds(p);
    // band3 reads a step's far neighbours one step early: T >= 2
    const bool v2 = p.T < 2;
    const void* fn = v2 ? (const void*)unpredict_band2<FAM, K_> : (const void*)unpredict_band3<FAM, K_>;
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return hipErrorInvalidValue;
    if (v2) hipLaunchKernelGGL((unpredict_band2<FAM, K_>), dim3(grid), dim3(64), lds, st, p);
    else hipLaunchKernelGGL((unpredict_band3<FAM, K_>), dim3(grid), dim3(64), lds, st, p);
    return hipGetLastError();
}

template <int FAM>
static hipError_t launch_unpredict(int k, const UnFrames& p, hipStream_t st, int* ctl)
{
    const int grid = (p.nz - p.first + p.step - 1) / p.step;
    if (grid <= 0) return hipSuccess;
    if (band2_ok(p)) {
        switch (k) {
#define LFM_K(K_) case K_: return launch_band2<FAM, K_>(p, grid, st, ctl);
        LFM_K(1) LFM_K(2) LFM_K(3) LFM_K(4) LFM_K(5) LFM_K(6) LFM_K(7)
#undef LFM_K
        default: return hipErrorInvalidValue;
        }
    }
    switch (k) {
#define LFM_K(K_) case K_: hipLaunchKernelGGL((unpredict_band<FAM, K_>), dim3(grid), dim3(64), 0, st, p); break;
    LFM_K(1) LFM_K(2) LFM_K(3) LFM_K(4) LFM_K(5) LFM_K(6) LFM_K(7)
#undef LFM_K
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// (checks that compile this file for one kernel define LFM_UNPREDICT_NO_ENTRY:
// unpredict_issue and the entry points below instantiate every kernel)
#ifndef LFM_UNPREDICT_NO_ENTRY
// Queues the inverse of every frame on `st`; with a control block (band5
// shapes) its status word is copied into *h_status behind the kernels (the
// caller reads it once the stream has passed that point), else *h_status = 0.
static int unpredict_issue(const uint16_t* d_sym, const uint16_t* d_prev, uint16_t* d_out, int W, int H, int nframes,
                           int T, int family, int predictor, int video_bit, int z0, int* h_status, hipStream_t st)
{
    if (W <= 0 || H <= 0 || nframes <= 0 || T <= 0 || T > 31 || predictor < 0 || predictor > 7 || family < 0 ||
        family > 2)
        return LFM_HIP_EINVAL;
    const size_t bytes = (size_t)W * H * nframes * sizeof(uint16_t);
    if (h_status) *h_status = 0;
    if (predictor == 0)
        return hipMemcpyAsync(d_out, d_sym, bytes, hipMemcpyDeviceToDevice, st) == hipSuccess ? LFM_HIP_OK
                                                                                              : LFM_HIP_ERUNTIME;
    const int video = video_bit & 1;
    const bool any_temporal = video && (nframes > 1 || (z0 & 1));
    if (any_temporal && family != 0) return LFM_HIP_ENOTINV;  // ((I - pred) + P) >> 1 drops a bit
    if (video && (z0 & 1) && !d_prev) return LFM_HIP_EINVAL;
    UnFrames p{d_sym, d_prev, d_out, W, H, T, nframes, z0, video, 0, 1, INT_MAX, 0u, nullptr, wait_ticks(), 0};
    CtlBlock* ctl = nullptr;
    if (band2_ok(p) && band4_waves(p)) {
        const int nbands = (H + 63) / 64;
        ctl = ctl_acquire((size_t)kCtlPos + (size_t)nframes * nbands);
        if (!ctl) return LFM_HIP_ERUNTIME;
        if (hipMemsetAsync(ctl->d, 0, sizeof(int), st) != hipSuccess) {
            ctl_release(ctl, st);
            return LFM_HIP_ERUNTIME;
        }
    }
    // without video every frame is spatial: one launch; with video the
    // spatial (even global z) frames first, then the temporal ones on their
    // decoded predecessors
    const int passes = video ? 2 : 1;
    int rc = LFM_HIP_OK;
    for (int pass = 0; pass < passes && rc == LFM_HIP_OK; ++pass) {
        if (video) {
            const int want = pass;  // global parity decoded by this pass
            p.first = (z0 & 1) == want ? 0 : 1;
            p.step = 2;
        }
        hipError_t e = hipErrorInvalidValue;
        int* c = ctl ? ctl->d : nullptr;
        switch (family) {
        case 0: e = lfm::launch_unpredict<0>(predictor, p, st, c); break;
        case 1: e = lfm::launch_unpredict<1>(predictor, p, st, c); break;
        case 2: e = lfm::launch_unpredict<2>(predictor, p, st, c); break;
        }
        if (e != hipSuccess) rc = LFM_HIP_ERUNTIME;
    }
    if (ctl) {
        if (rc == LFM_HIP_OK && h_status &&
            hipMemcpyAsync(h_status, ctl->d, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess)
            rc = LFM_HIP_ERUNTIME;
        ctl_release(ctl, st);
    }
    return rc;
}
#endif

} // namespace lfm

#ifndef LFM_UNPREDICT_NO_ENTRY
extern "C" int lfm_hip_unpredict_check(int status)
{
    if (!status) return LFM_HIP_OK;
    // without the re-run (LFM_UNPREDICT_FALLBACK=0) a band5 timeout leaves
    // pixels decoded from rows that were not ready
    const bool fixed = status == (int)lfm::kStBand5 && lfm::fallback_enabled();
    std::fprintf(stderr, "lfm: inverse predictor band hand-over timed out (band5)%s\n",
                 fixed ? "; frames re-run by the one-wave kernel" : "; the decoded pixels are not valid");
    return fixed ? LFM_HIP_OK : LFM_HIP_ERUNTIME;
}

extern "C" int lfm_hip_unpredict_async(const uint16_t* d_sym, const uint16_t* d_prev, uint16_t* d_out, int W, int H,
                                       int nframes, int T, int family, int predictor, int video_bit, int z0,
                                       int* h_status, void* stream_)
{
    if (!h_status) return LFM_HIP_EINVAL;
    const int rc = lfm::unpredict_issue(d_sym, d_prev, d_out, W, H, nframes, T, family, predictor, video_bit, z0,
                                        h_status, (hipStream_t)stream_);
    // (the caller passes the status word, once the stream is past the copy,
    // to lfm_hip_unpredict_check)
    return rc;
}

extern "C" int lfm_hip_unpredict(const uint16_t* d_sym, const uint16_t* d_prev, uint16_t* d_out, int W, int H,
                                 int nframes, int T, int family, int predictor, int video_bit, int z0, void* stream_)
{
    hipStream_t st = (hipStream_t)stream_;
    int* hs = nullptr;  // pinned, per thread (the copy behind the kernels lands there)
    thread_local struct Pinned {
        int* p = nullptr;
        ~Pinned()
        {
            if (p) (void)hipHostFree(p);
        }
    } pin;
    if (!pin.p && hipHostMalloc((void**)&pin.p, sizeof(int), hipHostMallocDefault) != hipSuccess) {
        pin.p = nullptr;
        return LFM_HIP_ERUNTIME;
    }
    hs = pin.p;
    const int rc = lfm::unpredict_issue(d_sym, d_prev, d_out, W, H, nframes, T, family, predictor, video_bit, z0, hs, st);
    if (rc != LFM_HIP_OK) return rc;
    if (hipStreamSynchronize(st) != hipSuccess) return LFM_HIP_ERUNTIME;
    return lfm_hip_unpredict_check(*hs);
}
#endif
