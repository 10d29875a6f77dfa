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
//   bigram  : per 30720-pair slice, staged in LDS, 65536 16-bit counters
//             packed in 128 KiB LDS (cannot overflow), run-length
//             pre-aggregation per thread, non-zero bins added to the job's
//             histogram with global atomics
//   entropy : per job, -P logf P per bin in parallel, then fixed-order row
//             sums and wave butterflies (deterministic)
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
// one 4 KiB segment per workgroup, 16 bytes per thread from one 16-byte load
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
    const uint32_t i = s0 + threadIdx.x * 16;
    if (i < S) {
        uint32_t w[4];
        const uint32_t m = min(16u, S - i);
        if (m == 16) {
            const uint4 v = *(const uint4*)(c + i);  // chunk starts are 16-byte aligned (450000 px * 2 B)
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        } else {
            for (int q = 0; q < 4; ++q) w[q] = 0;
            for (uint32_t t = 0; t < m; ++t) w[t >> 2] |= (uint32_t)c[i + t] << ((t & 3) * 8);
        }
        uint32_t zeros = 0;
#pragma unroll
        for (uint32_t t = 0; t < 16; ++t) {
            const uint32_t b = (w[t >> 2] >> ((t & 3) * 8)) & 0xFFu;
            if (t >= m) break;
            if (b == 0) ++zeros;
            else atomicAdd(&h[b], 1u);
        }
        if (zeros) atomicAdd(&h[0], zeros);
    }
    __syncthreads();
    // (plain stores: non-temporal ones here and in ent_scan gave no measurable
    // gain, and in ent_scatter's byte scatter they doubled the selection time;
    // profiles/r03_ab_nt_stores.txt)
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
// One wave per 4 KiB segment.  The segment (and the byte before it) is staged
// in LDS with 16-byte loads first, so the 64 rank rounds never wait on HBM.
__global__ __launch_bounds__(256) void ent_scatter(Jobs J, const uint32_t* __restrict__ offs, uint8_t* __restrict__ L)
{
    __shared__ uint32_t run[4][256];
    __shared__ __attribute__((aligned(16))) uint8_t seg_bytes[4][kSeg + 16];
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
    const uint32_t e = min(S, s0 + kSeg);
    uint8_t* sb = seg_bytes[wave] + 16;  // sb[-1] = c[s0 - 1]
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t o = (q * 64 + lane) * 16;
        if (s0 + o + 16 <= e) {
            *(uint4*)(sb + o) = *(const uint4*)(c + s0 + o);
        } else {
            for (uint32_t t = 0; t < 16; ++t) sb[o + t] = s0 + o + t < e ? c[s0 + o + t] : 0;
        }
    }
    if (lane == 0) sb[-1] = s0 > 0 ? c[s0 - 1] : 0;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    uint8_t* Lj = L + (size_t)job * kLStride;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t g = 0; g < e - s0; g += 64) {
        const uint32_t i = g + lane;
        const bool valid = s0 + i < e;
        const uint32_t key = valid ? sb[i] : 0u;
        const uint32_t val = valid ? sb[(int)i - 1] : 0u;
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
// Workgroup (slice, job) counts the bigrams of kSlice consecutive pairs of L:
// the slice is staged in LDS with 16-byte loads, every thread walks 60
// consecutive pairs (run-length pre-aggregated: the long (0,0) runs of the
// non-zero key buckets become one atomic), 65536 16-bit counters packed in
// 128 KiB of LDS (kSlice < 65536: no overflow), then the non-zero counters are
// added to the job's u32 histogram in HBM.
constexpr uint32_t kBins = 65536;
constexpr uint32_t kBigramThreads = 512;
// 60 pairs per thread: thread ranges start 15 words apart (odd), so the byte
// reads of a wave hit 64 distinct LDS banks; 128 KiB + 30 KiB of LDS
constexpr uint32_t kPerThread = 60;
constexpr uint32_t kSlice = kPerThread * kBigramThreads;

__global__ __launch_bounds__(kBigramThreads) void ent_bigram(Jobs J, const uint8_t* __restrict__ L,
                                                             uint32_t* __restrict__ hist)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t packed[];  // kBins / 2 words, then the slice bytes
    uint8_t* sl = (uint8_t*)(packed + kBins / 2);
    const int job = blockIdx.y;
    const uint8_t* c;
    uint32_t S;
    job_span(J, job, c, S);
    const uint32_t p0 = blockIdx.x * kSlice;
    if (p0 >= S) return;  // uniform for the block
    const uint32_t n = min(kSlice, S - p0);  // pairs p0 .. p0+n-1 use L[p0 .. p0+n]
    const uint8_t* Lj = L + (size_t)job * kLStride;
    // L job stride and p0 are multiples of 16: the staged span is 16-byte aligned
    for (uint32_t o = threadIdx.x * 16; o < n + 1; o += kBigramThreads * 16)
        *(uint4*)(sl + o) = *(const uint4*)(Lj + p0 + o);  // reads stay inside the L stride's slack
    for (uint32_t w = threadIdx.x; w < kBins / 2; w += kBigramThreads) packed[w] = 0;
    __syncthreads();
    const uint32_t a0 = threadIdx.x * kPerThread;
    const uint32_t a1 = min(n, a0 + kPerThread);
    uint32_t cur = 0xFFFFFFFFu, cnt = 0;
    if (a0 < a1) {
        uint32_t prev = sl[a0];
        for (uint32_t j = a0; j < a1; ++j) {
            const uint32_t nxt = sl[j + 1];
            const uint32_t bin = (prev << 8) | nxt;
            prev = nxt;
            if (bin == cur) { ++cnt; continue; }
            if (cnt) atomicAdd(&packed[cur >> 1], cnt << ((cur & 1) * 16));
            cur = bin;
            cnt = 1;
        }
        if (cnt) atomicAdd(&packed[cur >> 1], cnt << ((cur & 1) * 16));
    }
    __syncthreads();
    uint32_t* hj = hist + (size_t)job * kBins;
    for (uint32_t w = threadIdx.x; w < kBins / 2; w += kBigramThreads) {
        const uint32_t v = packed[w];
        if (v & 0xFFFFu) atomicAdd(&hj[2 * w], v & 0xFFFFu);
        if (v >> 16) atomicAdd(&hj[2 * w + 1], v >> 16);
    }
}

// -------------------------------------------------------------- entropy --
// Per job: H = sum over bins b < 65535 of -P logf P, P = h / S, in the fixed
// order the oracle restates (lfm_oracle.c lfmo_entropy_chunk): row r (bins
// 256r .. 256r+255) summed in ascending order by one lane, the 64 rows of a
// quarter combined by the wave's xor butterfly, quarters ((q0+q1)+q2)+q3.
// The per-bin terms are formed by all threads into LDS first (they do not
// depend on the order), then one wave runs the ordered row sums.
constexpr int kRow = 257;
__global__ __launch_bounds__(256) void ent_sum(Jobs J, const uint32_t* __restrict__ hist, float* __restrict__ ent)
{
    extern __shared__ float term[];  // 64 rows x kRow
    __shared__ float quarter[4];
    const int job = blockIdx.x;
    const uint8_t* c;
    uint32_t S;
    job_span(J, job, c, S);
    const float fs = (float)S;
    const uint32_t* hj = hist + (size_t)job * kBins;
    for (int q = 0; q < 4; ++q) {
        for (uint32_t i = threadIdx.x; i < 16384; i += 256) {
            const uint32_t b = q * 16384 + i;
            const uint32_t h = hj[b];
            float t = 0.f;
            if (h && b != 0xFFFFu) {  // bin 0xFFFF is never summed by the reference
                const float P = (float)h / fs;
                t = -1.0f * P * logf(P);
            }
            term[(i >> 8) * kRow + (i & 255)] = t;
        }
        __syncthreads();
        if (threadIdx.x < 64) {
            const float* row = term + threadIdx.x * kRow;
            float e = 0.f;
            for (int k = 0; k < 256; ++k) e += row[k];
            for (int off = 32; off > 0; off >>= 1) e += __shfl_xor(e, off);
            if (threadIdx.x == 0) quarter[q] = e;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) ent[job] = ((quarter[0] + quarter[1]) + quarter[2]) + quarter[3];
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
    hipError_t e = hipMemsetAsync(w.hist, 0, (size_t)J.njobs * kBins * 4, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ent_count, dim3(nsegBlocks, J.njobs), dim3(256), 0, st, J, w.cnt);
    hipLaunchKernelGGL(ent_scan, dim3(J.njobs), dim3(256), 0, st, J, w.cnt, w.offs, w.L);
    hipLaunchKernelGGL(ent_scatter, dim3((nsegBlocks + 3) / 4, J.njobs), dim3(256), 0, st, J, w.offs, w.L);
    const uint32_t nslice = (kChunkBytes + kSlice - 1) / kSlice;
    hipLaunchKernelGGL(ent_bigram, dim3(nslice, J.njobs), dim3(kBigramThreads), (kBins / 2) * 4 + kSlice + 16, st, J,
                       w.L, w.hist);
    hipLaunchKernelGGL(ent_sum, dim3(J.njobs), dim3(256), 64 * kRow * 4, st, J, w.hist, w.ent);
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
    for (int k = 1; k < 8; ++k) cands[k] = w.cands + (size_t)(k - 1) * npix;
    int rc = lfm_hip_predict_candidates(d_frame, w.cands, W, H, T, family, st);
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
