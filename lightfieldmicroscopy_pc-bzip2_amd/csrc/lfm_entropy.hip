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
// The sorted array L is never built.  In L the element after (key k, val
// c[i-1]) is the next element of the same key in index order -- the next
// occurrence i' > i of byte k, whose val is c[i'-1] -- or, for the last
// element of a key, the first element of the next non-empty key (the
// sentinel closes key 0).  So each position i has a PARTNER byte p[i], its
// bigram is bin (c[i-1] << 8) | p[i], and the histogram is a position-order
// pass over (c, p).  All candidates x chunks ("jobs") of a frame go through
// every launch (the reference runs 3 kernels + a CUB radix sort + a blocking
// thrust::reduce per candidate and chunk):
//   ent_next : per 16 KiB segment (4 waves x 4 KiB): each wave walks its
//              bytes backward in 64-position windows; a position's partner is
//              the val of the next lane with the same byte (peer masks from
//              eight ballots) or the first val of that byte in the later
//              windows (a 256-entry LDS table); the four waves are linked the
//              same way; per segment and byte: first val and last position
//   ent_link : per job, per byte (one thread each): links the segments
//              (last position of a segment <- first val of the byte in the
//              later segments) and the keys (the last element of key k <-
//              the first val of the next non-empty key; key 0's last element
//              <- the sentinel's val; the sentinel <- key >= 1's first val);
//              the one element without a partner (end of L) is recorded
//   ent_rows : per (job, quarter of the rows by val & 3): counts its bins --
//              64 rows x 256 u32 counters in LDS, written by nobody else, so
//              no 16-bit packing, no merge and no global atomics -- then the
//              -P logf P terms and the ascending row sums of its 64 rows
//   host     : per job the 256 row sums are combined in the oracle's fixed
//              order (lfm_oracle.c lfmo_entropy_chunk: the 64 rows of a
//              quarter by an xor butterfly, quarters left to right) -- the
//              same float additions the round-1..5 ent_sum kernel did.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "lfm_hip.h"

namespace lfm {

constexpr uint32_t kChunkPix = 450000;
constexpr uint32_t kChunkBytes = 2 * kChunkPix;
constexpr uint32_t kSub = 4096;                                   // bytes per wave of ent_next
constexpr uint32_t kSeg = 4 * kSub;                               // bytes per ent_next workgroup
constexpr uint32_t kSegMax = (kChunkBytes + kSeg - 1) / kSeg;     // 55
constexpr uint32_t kLStride = (kChunkBytes + 16 + 255) & ~255u;   // partner bytes per job (16-byte reads past S)
constexpr uint32_t kNoVal = 0x100;                                // "no val" (a byte is < 256)
constexpr uint32_t kNoPos = 0xFFFFFFFFu;
constexpr int kRow = 257;                                         // padded LDS row (u32 / float)

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

// 16 bytes of c at o (16-byte aligned), zeros past S (the last chunk of a
// buffer may end anywhere)
__device__ __forceinline__ uint4 load16(const uint8_t* c, uint32_t o, uint32_t S)
{
    if (o + 16 <= S) return *(const uint4*)(c + o);  // chunk starts are 16-byte aligned (450000 px * 2 B)
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t t = 0; t < 16 && o + t < S; ++t) w[t >> 2] |= (uint32_t)c[o + t] << ((t & 3) * 8);
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ uint32_t byte_of(const uint4& v, int j)
{
    const uint32_t w = j < 4 ? v.x : j < 8 ? v.y : j < 12 ? v.z : v.w;
    return (w >> ((j & 3) * 8)) & 0xFFu;
}

// ------------------------------------------------------------- ent_next --
// tab[job][seg][k] = (last position of byte k in the segment + 1) | first
// val of byte k in the segment << 20 (kNoVal: absent); 0 when absent.
__global__ __launch_bounds__(256) void ent_next(Jobs J, uint8_t* __restrict__ part, uint32_t* __restrict__ tab)
{
    __shared__ __attribute__((aligned(16))) uint8_t sbytes[4][kSub + 16];
    __shared__ uint16_t nxt[4][256];   // first val of byte k in this wave's later windows
    __shared__ uint32_t last[4][256];  // last position of byte k in this wave's bytes
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int job = blockIdx.y;
    const uint8_t* c;
    uint32_t S;
    job_span(J, job, c, S);
    const uint32_t s0 = blockIdx.x * kSeg;
    if (s0 >= S) return;  // uniform for the block
    uint8_t* pj = part + (size_t)job * kLStride;
    const uint32_t b0 = s0 + wave * kSub;
    const uint32_t len = b0 < S ? min(kSub, S - b0) : 0u;
    uint8_t* sb = sbytes[wave] + 16;  // sb[-1] = c[b0 - 1]
    for (int k = lane; k < 256; k += 64) {
        nxt[wave][k] = kNoVal;
        last[wave][k] = kNoPos;
    }
    if (len) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t o = (q * 64 + lane) * 16;
            if (o < len) *(uint4*)(sb + o) = load16(c, b0 + o, S);
        }
        if (lane == 0) sb[-1] = b0 > 0 ? c[b0 - 1] : 0;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    const uint64_t above = lane == 63 ? 0ull : (~0ull << (lane + 1));
    const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (int g = (int)((len + 63) / 64) - 1; g >= 0; --g) {
        const uint32_t i = (uint32_t)g * 64 + lane;
        const bool valid = i < len;
        const uint32_t key = valid ? sb[i] : 0u;
        const uint32_t val = valid ? sb[(int)i - 1] : 0u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (key >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint64_t hi = peers & above;
        const int src = hi ? (int)__builtin_ctzll(hi) : lane;
        const uint32_t pv = (uint32_t)__shfl((int)val, src);
        uint32_t pt = hi ? pv : (valid ? (uint32_t)nxt[wave][key] : 0u);
        __builtin_amdgcn_wave_barrier();
        if (valid) {
            // the lowest lane of a byte's group is that byte's first
            // occurrence from here on; the highest with no later occurrence
            // in this wave's bytes is the wave's last occurrence
            if (!(peers & below)) nxt[wave][key] = (uint16_t)val;
            if (pt == kNoVal) {
                last[wave][key] = b0 + i;
                pt = 0;  // (linked below or by ent_link)
            }
            pj[b0 + i] = (uint8_t)pt;
        }
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // link the four waves, byte k per thread: the last occurrence of k in a
    // wave gets the first val of k in the waves after it
    const int k = threadIdx.x;
    uint32_t carry = kNoVal, seg_last = kNoPos;
    for (int w = 3; w >= 0; --w) {
        const uint32_t lp = last[w][k];
        if (lp != kNoPos) {
            if (carry == kNoVal) seg_last = lp;
            else pj[lp] = (uint8_t)carry;
        }
        if (nxt[w][k] != kNoVal) carry = nxt[w][k];
    }
    tab[((size_t)job * kSegMax + blockIdx.x) * 256 + k] = seg_last == kNoPos ? 0u : ((seg_last + 1) | (carry << 20));
}

// ------------------------------------------------------------- ent_link --
// meta[job] = {position whose element ends L (no bigram) or kNoPos,
//              the sentinel's bin or kNoPos}
__global__ __launch_bounds__(256) void ent_link(Jobs J, uint8_t* __restrict__ part, const uint32_t* __restrict__ tab,
                                                uint32_t* __restrict__ meta)
{
    __shared__ uint32_t T[kSegMax * 256];
    __shared__ uint32_t F[256], NF[256];
    __shared__ uint32_t skip;
    const int job = blockIdx.x;
    const uint8_t* c;
    uint32_t S;
    job_span(J, job, c, S);
    uint8_t* pj = part + (size_t)job * kLStride;
    const uint32_t nseg = (S + kSeg - 1) / kSeg;
    const uint32_t* tj = tab + (size_t)job * kSegMax * 256;
    for (uint32_t o = threadIdx.x; o < nseg * 256; o += 256) T[o] = tj[o];
    if (threadIdx.x == 0) skip = kNoPos;
    __syncthreads();
    const int k = threadIdx.x;
    uint32_t carry = kNoVal, glast = kNoPos;
    for (int s = (int)nseg - 1; s >= 0; --s) {
        const uint32_t t = T[s * 256 + k];
        if (!t) continue;
        const uint32_t lp = (t & 0xFFFFFu) - 1;
        if (carry == kNoVal) glast = lp;  // the last occurrence of k in the chunk
        else pj[lp] = (uint8_t)carry;
        carry = t >> 20;
    }
    F[k] = carry;  // first val of key k (kNoVal: k absent)
    __syncthreads();
    if (k == 0) {  // NF[k] = first val of the next non-empty key > k
        uint32_t nf = kNoVal;
        for (int q = 255; q >= 0; --q) {
            NF[q] = nf;
            if (F[q] != kNoVal) nf = F[q];
        }
    }
    __syncthreads();
    const uint32_t sval = S ? c[S - 1] : 0u;  // the sentinel (key 0) closes key 0
    if (glast != kNoPos) {
        const uint32_t p = k == 0 ? sval : NF[k];
        if (p == kNoVal) skip = glast;  // the end of L (one key at most)
        else pj[glast] = (uint8_t)p;
    }
    __syncthreads();
    if (k == 0) {
        meta[2 * job] = skip;
        meta[2 * job + 1] = NF[0] == kNoVal ? kNoPos : ((sval << 8) | NF[0]);
    }
}

// ------------------------------------------------------------- ent_rows --
// Workgroup (job, quarter q) owns the 64 rows r = 4m + q (bins r * 256 ..
// r * 256 + 255, r = the bigram's first byte): it counts them over every
// position of the job, then writes the 64 row sums rows[job][r].  The
// quarters of a job are blocks b, b + 8, b + 16, b + 24 (one XCD: the job's
// bytes are read from one L2).  Bin 0 -- (0, 0), the high bytes of small
// symbols -- is counted in registers.
#ifndef LFM_ENT_ROW_THREADS
#define LFM_ENT_ROW_THREADS 1024  // (512: a config-3 selection 0.51 ms, 1 024: 0.50; profiles/r06_ab_select_ent_rows.txt)
#endif
constexpr int kRowThreads = LFM_ENT_ROW_THREADS;
__global__ __launch_bounds__(kRowThreads) void ent_rows(Jobs J, const uint8_t* __restrict__ part,
                                                        const uint32_t* __restrict__ meta, float* __restrict__ rows)
{
    extern __shared__ uint32_t cnt[];  // 64 rows x kRow
    __shared__ uint32_t zsum;
    const int blk = blockIdx.x;
    const int job = (blk >> 5) * 8 + (blk & 7), q = (blk >> 3) & 3;
    if (job >= J.njobs) return;  // uniform for the block
    const uint8_t* c;
    uint32_t S;
    job_span(J, job, c, S);
    const uint8_t* pj = part + (size_t)job * kLStride;
    for (int o = threadIdx.x; o < 64 * kRow; o += kRowThreads) cnt[o] = 0;
    if (threadIdx.x == 0) zsum = 0;
    const uint32_t skip = meta[2 * job], extra = meta[2 * job + 1];
    __syncthreads();
    uint32_t zeros = 0;
    for (uint32_t i0 = threadIdx.x * 16; i0 < S; i0 += kRowThreads * 16) {
        const uint4 pv = *(const uint4*)(pj + i0);  // (the stride holds 16 bytes past S)
        const uint4 cv = load16(c, i0, S);
        uint32_t prev = i0 ? c[i0 - 1] : 0u;  // c[-1] = 0
        const uint32_t n = min(16u, S - i0);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t val = prev, p = byte_of(pv, j);
            prev = byte_of(cv, j);
            const uint32_t i = i0 + j;
            if ((uint32_t)j >= n || i == skip) continue;
            const uint32_t bin = (val << 8) | p;
            if (bin == 0) ++zeros;
            else if ((val & 3u) == (uint32_t)q) atomicAdd(&cnt[(val >> 2) * kRow + p], 1u);
        }
    }
    if (extra != kNoPos && threadIdx.x == 0 && ((extra >> 8) & 3u) == (uint32_t)q) {
        if (extra == 0) ++zeros;
        else atomicAdd(&cnt[(extra >> 10) * kRow + (extra & 0xFFu)], 1u);
    }
    if (q == 0) {
        for (int off = 32; off > 0; off >>= 1) zeros += __shfl_xor(zeros, off);
        if ((threadIdx.x & 63) == 0 && zeros) atomicAdd(&zsum, zeros);
    }
    __syncthreads();
    if (q == 0 && threadIdx.x == 0) cnt[0] += zsum;
    __syncthreads();
    // -P logf P per bin in place (bin 0xFFFF is never summed by the
    // reference), then row sums in ascending bin order
    const float fs = (float)S;
    float* term = (float*)cnt;
    for (int o = threadIdx.x; o < 64 * 256; o += kRowThreads) {
        const int m = o >> 8, b = o & 255;
        const uint32_t bin = ((uint32_t)(4 * m + q) << 8) | (uint32_t)b;
        const uint32_t h = cnt[m * kRow + b];
        float t = 0.f;
        if (h && bin != 0xFFFFu) {
            const float P = (float)h / fs;
            t = -1.0f * P * logf(P);
        }
        term[m * kRow + b] = t;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        const float* row = term + threadIdx.x * kRow;
        float e = 0.f;
        for (int b = 0; b < 256; ++b) e += row[b];
        rows[(size_t)job * 256 + 4 * threadIdx.x + q] = e;
    }
}

struct Workspace {
    uint32_t* tab;
    uint8_t* part;
    uint32_t* meta;
    float* rows;
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
    p = take(jobs * kSegMax * 256 * 4); if (w) w->tab = (uint32_t*)p;
    p = take(jobs * (size_t)kLStride); if (w) w->part = p;
    p = take(jobs * 8); if (w) w->meta = (uint32_t*)p;
    p = take(jobs * 256 * 4); if (w) w->rows = (float*)p;
    p = take(with_cands ? (size_t)7 * npix * 2 : 0); if (w) w->cands = (uint16_t*)p;
    return off;
}

static hipError_t run_entropy(const Jobs& J, const Workspace& w, hipStream_t st)
{
    hipLaunchKernelGGL(ent_next, dim3(kSegMax, J.njobs), dim3(256), 0, st, J, w.part, w.tab);
    hipLaunchKernelGGL(ent_link, dim3(J.njobs), dim3(256), 0, st, J, w.part, w.tab, w.meta);
    const uint32_t nblk = (uint32_t)((J.njobs + 7) / 8) * 32;
    hipLaunchKernelGGL(ent_rows, dim3(nblk), dim3(kRowThreads), 64 * kRow * 4, st, J, w.part, w.meta, w.rows);
    return hipGetLastError();
}

// the oracle's fixed order (lfm_oracle.c lfmo_entropy_chunk) over one job's
// 256 row sums: the 64 rows of a quarter by an xor butterfly, then the
// quarters left to right
static float combine_rows(const float* part)
{
    float w[4];
    for (int q = 0; q < 4; ++q) {
        float v[64], nv[64];
        for (int l = 0; l < 64; ++l) v[l] = part[q * 64 + l];
        for (int off = 32; off > 0; off >>= 1) {
            for (int l = 0; l < 64; ++l) nv[l] = v[l] + v[l ^ off];
            std::memcpy(v, nv, sizeof(v));
        }
        w[q] = v[0];
    }
    return ((w[0] + w[1]) + w[2]) + w[3];
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
    std::vector<float> h_rows((size_t)J.njobs * 256);
    hipError_t e = hipMemcpyAsync(h_rows.data(), w.rows, h_rows.size() * sizeof(float), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) {
        for (int k = 0; k < ncand; ++k) {
            float acc = 0.f;  // entropy_A += per-chunk reduce, in chunk order
            for (int q = 0; q < J.nchunks; ++q) acc += combine_rows(h_rows.data() + (size_t)(k * J.nchunks + q) * 256);
            out[k] = acc;
        }
    }
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
