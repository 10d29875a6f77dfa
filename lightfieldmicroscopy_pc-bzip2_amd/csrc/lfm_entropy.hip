// lfm_entropy.hip -- 2D-entropy predictor selection on gfx950.
//
// Reference semantics (klb_imageIO.cpp:2030-2093 bwt_entropy_2D;
// lfm_Predictors.cu:2883-2914 bwt_GPU, :2833-2856 static_bwt_GPU,
// :2923-2949 sum_bwt_GPU): for every chunk of <= 450000 pixels (S = 2n bytes
// c[0..S)), form pairs (key c[i], val c[i-1]) with c[-1] = 0 plus a sentinel
// (key 0, val c[S-1]); stable-sort by key into L[0..S]; count bigrams
// (L[j], L[j+1]) for j < S; H = sum over bins b < 65535 of -P ln P with
// P = h / S in float.  Candidate 0 (raw) is scaled by 0.96; the argmin takes
// the highest index on exact ties (std::map<float,int> overwrite).
//
// gfx950 pipeline, all candidates x chunks ("jobs") of one frame batched in
// every launch (the reference runs 3 kernels + a CUB radix sort + a blocking
// thrust::reduce per candidate and chunk, serialised on the default stream):
//   count   : per 4 KiB segment, key histogram (LDS)
//   scan    : per job, bucket bases (sentinel closes bucket 0) + per-segment
//             offsets
//   scatter : stable counting sort, one wave per segment; in-wave stable rank
//             from eight 64-bit ballots (peer mask), running counts in LDS
//   bigram  : per <= 61440 pairs, 65536 16-bit counters packed in 128 KiB LDS
//             (cannot overflow), run-length pre-aggregation per lane, flush of
//             non-zero bins with global atomics
//   entropy : per job, -P logf P over 65535 bins, fixed-order wave-shuffle
//             reduction (deterministic)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include "lfm_hip.h"

namespace lfm {

constexpr uint32_t kChunkPix = 450000;
constexpr uint32_t kChunkBytes = 2 * kChunkPix;
constexpr uint32_t kSeg = 4096;                                   // bytes per count/scatter segment
constexpr uint32_t kSegMax = (kChunkBytes + kSeg - 1) / kSeg;     // 220
constexpr uint32_t kPairsPerWG = 61440;                           // <= 65535 keeps 16-bit counters exact
constexpr uint32_t kBins = 65536;
constexpr uint32_t kLStride = (kChunkBytes + 1 + 255) & ~255u;

struct Jobs {
    const uint8_t* cand[8];  // candidate buffers as bytes
    uint64_t npix;
    int nchunks;
    int njobs;               // ncand * nchunks
};

__device__ __forceinline__ void job_span(const Jobs& J, int job, const uint8_t*& c, uint32_t& S)
{
    const int k = job / J.nchunks, q = job % J.nchunks;
    const uint64_t p0 = (uint64_t)q * kChunkPix;
    const uint64_t n = (J.npix - p0) < kChunkPix ? (J.npix - p0) : kChunkPix;
    c = J.cand[k] + p0 * 2;
    S = (uint32_t)(n * 2);
}

// ---------------------------------------------------------------- count --
__global__ __launch_bounds__(256) void ent_count(Jobs J, uint32_t* __restrict__ cnt)
{
    __shared__ uint32_t h[256];
    const int job = blockIdx.y;
    const uint8_t* c;
    uint32_t S;
    job_span(J, job, c, S);
    const uint32_t s0 = blockIdx.x * kSeg;
    h[threadIdx.x] = 0;
    __syncthreads();
    if (s0 < S) {
        const uint32_t e = min(S, s0 + kSeg);
        uint32_t zeros = 0;
        for (uint32_t i = s0 + threadIdx.x * 16; i < e; i += 256 * 16) {
            const uint32_t m = min(16u, e - i);
            for (uint32_t t = 0; t < m; ++t) {
                const uint8_t b = c[i + t];
                if (b == 0) ++zeros;
                else atomicAdd(&h[b], 1u);
            }
        }
        if (zeros) atomicAdd(&h[0], zeros);
    }
    __syncthreads();
    cnt[((size_t)job * kSegMax + blockIdx.x) * 256 + threadIdx.x] = h[threadIdx.x];
}

// ----------------------------------------------------------------- scan --
// offs[job][seg][k] = start of segment seg's key-k elements in L.
__global__ __launch_bounds__(256) void ent_scan(Jobs J, const uint32_t* __restrict__ cnt, uint32_t* __restrict__ offs,
                                                uint8_t* __restrict__ L)
{
    __shared__ uint32_t tot[256];
    const int job = blockIdx.x;
    const uint8_t* c;
    uint32_t S;
    job_span(J, job, c, S);
    const uint32_t nseg = (S + kSeg - 1) / kSeg;
    const int k = threadIdx.x;
    const uint32_t* cj = cnt + (size_t)job * kSegMax * 256;
    uint32_t t = 0;
    for (uint32_t s = 0; s < nseg; ++s) t += cj[s * 256 + k];
    tot[k] = t + (k == 0 ? 1u : 0u);  // sentinel closes bucket 0
    __syncthreads();
    // exclusive scan over 256 keys (serial by thread 0 is 256 adds; keep it simple and exact)
    __shared__ uint32_t base[256];
    if (k == 0) {
        uint32_t acc = 0;
        for (int i = 0; i < 256; ++i) { base[i] = acc; acc += tot[i]; }
    }
    __syncthreads();
    uint32_t acc = base[k];
    uint32_t* oj = offs + (size_t)job * kSegMax * 256;
    for (uint32_t s = 0; s < nseg; ++s) {
        oj[s * 256 + k] = acc;
        acc += cj[s * 256 + k];
    }
    if (k == 0) {
        // sentinel (key 0, val c[S-1]) sits after every key-0 element
        L[(size_t)job * kLStride + acc] = S ? c[S - 1] : 0;
    }
}

// -------------------------------------------------------------- scatter --
__global__ __launch_bounds__(256) void ent_scatter(Jobs J, const uint32_t* __restrict__ offs, uint8_t* __restrict__ L)
{
    __shared__ uint32_t run[4][256];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int job = blockIdx.y;
    const uint32_t seg = blockIdx.x * 4 + wave;
    const uint8_t* c;
    uint32_t S;
    job_span(J, job, c, S);
    const uint32_t s0 = seg * kSeg;
    if (s0 >= S) return;  // whole wave leaves; no block barrier below
    const uint32_t* oj = offs + ((size_t)job * kSegMax + seg) * 256;
    for (int i = lane; i < 256; i += 64) run[wave][i] = oj[i];
    __builtin_amdgcn_wave_barrier();
    uint8_t* Lj = L + (size_t)job * kLStride;
    const uint32_t e = min(S, s0 + kSeg);
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t g = s0; g < e; g += 64) {
        const uint32_t i = g + lane;
        const bool valid = i < e;
        const uint32_t key = valid ? c[i] : 0u;
        const uint32_t val = (valid && i > 0) ? c[i - 1] : 0u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (key >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t rank = __popcll(peers & lt);
        const uint32_t before = valid ? run[wave][key] : 0u;
        __builtin_amdgcn_wave_barrier();
        if (valid) {
            Lj[before + rank] = (uint8_t)val;
            // the highest lane of each peer group advances the bucket
            if ((peers >> lane) == 1ull) run[wave][key] = before + rank + 1;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// --------------------------------------------------------------- bigram --
__global__ __launch_bounds__(256) void ent_bigram(Jobs J, const uint8_t* __restrict__ L, uint32_t* __restrict__ hist)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t packed[];  // 32768 words = 65536 x u16
    const int job = blockIdx.y;
    const uint8_t* c;
    uint32_t S;
    job_span(J, job, c, S);
    const uint32_t p0 = blockIdx.x * kPairsPerWG;
    if (p0 >= S) return;  // uniform for the block
    for (uint32_t w = threadIdx.x; w < kBins / 2; w += 256) packed[w] = 0;
    __syncthreads();
    const uint8_t* Lj = L + (size_t)job * kLStride;
    const uint32_t p1 = min(S, p0 + kPairsPerWG);
    const uint32_t per = (kPairsPerWG + 255) / 256;
    const uint32_t a0 = p0 + threadIdx.x * per;
    const uint32_t a1 = min(p1, a0 + per);
    uint32_t cur = 0xFFFFFFFFu, n = 0;
    if (a0 < a1) {
        uint32_t prev = Lj[a0];
        for (uint32_t j = a0; j < a1; ++j) {
            const uint32_t nxt = Lj[j + 1];
            const uint32_t bin = (prev << 8) | nxt;
            prev = nxt;
            if (bin == cur) { ++n; continue; }
            if (n) atomicAdd(&packed[cur >> 1], n << ((cur & 1) * 16));
            cur = bin;
            n = 1;
        }
        if (n) atomicAdd(&packed[cur >> 1], n << ((cur & 1) * 16));
    }
    __syncthreads();
    uint32_t* hj = hist + (size_t)job * kBins;
    for (uint32_t w = threadIdx.x; w < kBins / 2; w += 256) {
        const uint32_t v = packed[w];
        if (v & 0xFFFFu) atomicAdd(&hj[2 * w], v & 0xFFFFu);
        if (v >> 16) atomicAdd(&hj[2 * w + 1], v >> 16);
    }
}

// -------------------------------------------------------------- entropy --
__global__ __launch_bounds__(256) void ent_sum(Jobs J, const uint32_t* __restrict__ hist, float* __restrict__ ent)
{
    __shared__ float part[4];
    const int job = blockIdx.x;
    const uint8_t* c;
    uint32_t S;
    job_span(J, job, c, S);
    const float fs = (float)S;
    const uint32_t* hj = hist + (size_t)job * kBins;
    float e = 0.f;
    const uint32_t b0 = threadIdx.x * 256;
    for (uint32_t b = b0; b < b0 + 256; ++b) {
        if (b >= 65535u) break;  // bin 0xFFFF is never summed by the reference
        const uint32_t h = hj[b];
        if (h) {
            const float P = (float)h / fs;
            e += -1.0f * P * logf(P);
        }
    }
    for (int off = 32; off > 0; off >>= 1) e += __shfl_xor(e, off);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = e;
    __syncthreads();
    if (threadIdx.x == 0) ent[job] = ((part[0] + part[1]) + part[2]) + part[3];
}

struct Workspace {
    uint32_t* cnt;
    uint32_t* offs;
    uint8_t* L;
    uint32_t* hist;
    float* ent;
    uint16_t* cands;  // 7 candidate buffers (select only)
};

static size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

static size_t workspace_layout(uint64_t npix, int ncand, bool with_cands, Workspace* w, uint8_t* base)
{
    const int nchunks = (int)((npix + kChunkPix - 1) / kChunkPix);
    const size_t jobs = (size_t)nchunks * ncand;
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off += align256(bytes); return base ? base + o : nullptr; };
    uint8_t* p;
    p = take(jobs * kSegMax * 256 * 4); if (w) w->cnt = (uint32_t*)p;
    p = take(jobs * kSegMax * 256 * 4); if (w) w->offs = (uint32_t*)p;
    p = take(jobs * (size_t)kLStride); if (w) w->L = p;
    p = take(jobs * kBins * 4); if (w) w->hist = (uint32_t*)p;
    p = take(jobs * 4); if (w) w->ent = (float*)p;
    p = take(with_cands ? (size_t)7 * npix * 2 : 0); if (w) w->cands = (uint16_t*)p;
    return off;
}

static hipError_t run_entropy(const Jobs& J, const Workspace& w, hipStream_t st)
{
    const uint32_t nsegBlocks = kSegMax;
    hipError_t e;
    e = hipMemsetAsync(w.hist, 0, (size_t)J.njobs * kBins * 4, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ent_count, dim3(nsegBlocks, J.njobs), dim3(256), 0, st, J, w.cnt);
    hipLaunchKernelGGL(ent_scan, dim3(J.njobs), dim3(256), 0, st, J, w.cnt, w.offs, w.L);
    hipLaunchKernelGGL(ent_scatter, dim3((nsegBlocks + 3) / 4, J.njobs), dim3(256), 0, st, J, w.offs, w.L);
    const uint32_t nbig = (kChunkBytes + kPairsPerWG - 1) / kPairsPerWG;
    hipLaunchKernelGGL(ent_bigram, dim3(nbig, J.njobs), dim3(256), (kBins / 2) * 4, st, J, w.L, w.hist);
    hipLaunchKernelGGL(ent_sum, dim3(J.njobs), dim3(256), 0, st, J, w.hist, w.ent);
    return hipGetLastError();
}

} // namespace lfm

using namespace lfm;

static int entropy_impl(const uint16_t* const* cands, int ncand, uint64_t npix, float* out, void* dws,
                        bool own_ws, hipStream_t st)
{
    Jobs J{};
    for (int k = 0; k < ncand; ++k) J.cand[k] = (const uint8_t*)cands[k];
    J.npix = npix;
    J.nchunks = (int)((npix + kChunkPix - 1) / kChunkPix);
    J.njobs = J.nchunks * ncand;
    Workspace w{};
    workspace_layout(npix, ncand, false, &w, (uint8_t*)dws);
    if (run_entropy(J, w, st) != hipSuccess) return LFM_HIP_ERUNTIME;
    float* h_ent = (float*)malloc(sizeof(float) * J.njobs);
    hipError_t e = hipMemcpyAsync(h_ent, w.ent, sizeof(float) * J.njobs, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) {
        for (int k = 0; k < ncand; ++k) {
            float acc = 0.f;  // entropy_A += per-chunk reduce, in chunk order
            for (int q = 0; q < J.nchunks; ++q) acc += h_ent[k * J.nchunks + q];
            out[k] = acc;
        }
    }
    free(h_ent);
    (void)own_ws;
    return e == hipSuccess ? LFM_HIP_OK : LFM_HIP_ERUNTIME;
}

extern "C" int lfm_hip_entropy2d(const uint16_t* d_cand, uint64_t npix, float* entropy, void* stream)
{
    if (!d_cand || !npix || !entropy) return LFM_HIP_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const size_t bytes = workspace_layout(npix, 1, false, nullptr, nullptr);
    void* ws = nullptr;
    if (hipMallocAsync(&ws, bytes, st) != hipSuccess) return LFM_HIP_ERUNTIME;
    const uint16_t* c[1] = {d_cand};
    int rc = entropy_impl(c, 1, npix, entropy, ws, true, st);
    (void)hipFreeAsync(ws, st);
    return rc;
}

extern "C" size_t lfm_hip_select_workspace_bytes(int W, int H)
{
    return workspace_layout((uint64_t)W * H, 8, true, nullptr, nullptr);
}

extern "C" int lfm_hip_select(const uint16_t* d_frame, int W, int H, int T, int family, float entropy[8],
                              int* chosen, void* d_workspace, void* stream)
{
    if (!d_frame || W <= 0 || H <= 0 || T <= 0 || !entropy || !chosen) return LFM_HIP_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const uint64_t npix = (uint64_t)W * H;
    const size_t bytes = workspace_layout(npix, 8, true, nullptr, nullptr);
    void* ws = d_workspace;
    bool own = false;
    if (!ws) {
        if (hipMallocAsync(&ws, bytes, st) != hipSuccess) return LFM_HIP_ERUNTIME;
        own = true;
    }
    Workspace w{};
    workspace_layout(npix, 8, true, &w, (uint8_t*)ws);
    const uint16_t* cands[8];
    cands[0] = d_frame;  // candidate 0: the raw frame (klb_imageIO.cpp:1690)
    int rc = LFM_HIP_OK;
    for (int k = 1; k < 8 && rc == LFM_HIP_OK; ++k) {
        uint16_t* dst = w.cands + (size_t)(k - 1) * npix;
        rc = lfm_hip_predict(d_frame, nullptr, dst, W, H, 1, T, family, k, 0, 0, st);
        cands[k] = dst;
    }
    float ent[8];
    if (rc == LFM_HIP_OK) rc = entropy_impl(cands, 8, npix, ent, ws, false, st);
    if (own) (void)hipFreeAsync(ws, st);
    if (rc != LFM_HIP_OK) return rc;
    ent[0] = (float)((double)ent[0] * 0.96);  // bwt_entropy_2D: raw candidate * 0.96 (klb_imageIO.cpp:2087-2090)
    int best = 0;
    for (int k = 0; k < 8; ++k) {
        entropy[k] = ent[k];
        if (k > 0 && ent[k] <= ent[best]) best = k;  // std::map<float,int>: equal keys keep the last index
    }
    *chosen = best;
    return LFM_HIP_OK;
}
