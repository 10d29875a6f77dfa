// lfm_bzip2.hip -- block-parallel bzip2 (libbzip2 1.0.6 byte-exact) on gfx950.
//
// The .lfm writer compresses every 5-D block as its own bzip2 stream at
// level min(9, ceil(blockBytes / 1e5)) with workFactor 30
// (klb_imageIO.cpp:108, :217).  For a default 96x96x8 uint16 block that is
// one bzip2 block per stream, and a config-3 stack has 3 872 of them: the
// unit of parallelism here is the stream.  Every stage reproduces the
// published bzip2-1.0.6 algorithm (vendored at src/external/bzip2-1.0.6 of the
// reference; restated, not copied):
//
//   rle1_crc   bzlib.c ADD_CHAR_TO_BLOCK / add_pair_to_block: runs of 4..255
//              equal bytes -> 4 bytes + (len-4); block CRC (MSB-first
//              CRC-32, poly 0x04c11db7) over the raw bytes; inUse map.
//              One workgroup per stream: per-thread chunks, a scan carries
//              the run state across chunks, CRCs of chunks are combined with
//              GF(2) shift matrices.
//   BWT        blocksort.c sorts the cyclic rotations of the RLE1 block (the
//              order is unique for a non-periodic block, so any correct sort
//              gives libbzip2's bytes): prefix doubling -- rotations sorted by
//              their first 8 bytes, then by (rank[i], rank[i+h]) for h = 8,
//              16, ... with segmented radix sorts (one segment per stream)
//              until every rank is unique.  A periodic block (equal
//              rotations) is handed back to the host library.
//   mtf        compress.c generateMTFValues: move-to-front + RUNA/RUNB zero
//              runs, one wave per stream, the 256-entry list packed 4 bytes
//              per lane, lookups by ballot.
//   huffman    compress.c sendMTFValues + huffman.c: table count by nMTF,
//              initial partition, 4 refinement passes (selector per 50
//              symbols: first minimum cost; BZ2_hbMakeCodeLengths with
//              maxLen 17 and its weight-halving retry), selector MTF, codes.
//   emit       the bit stream: "BZh" + level, block magic, CRC, origPtr,
//              mapping table, selectors, delta-coded lengths, the symbols,
//              end magic and combined CRC; MSB-first bits.  Symbol codes are
//              written by all threads at prefix-summed bit offsets.
//
// Streams whose RLE1 block reaches nblockMAX (libbzip2 would cut a second
// block) or that are periodic are flagged for the host library: the output
// stays byte-identical in every case.
#include <hip/hip_runtime.h>
#include <rocprim/block/block_exchange.hpp>
#include <rocprim/block/block_sort.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#include "lfm_hip.h"


namespace lfm {
namespace bz {

constexpr int kRleThreads = 512;
constexpr int kMaxGroups = 6;
constexpr int kMaxAlpha = 258;
constexpr int kGSize = 50;
constexpr int kIters = 4;
constexpr uint32_t kRunA = 0, kRunB = 1;

// flags
constexpr uint32_t kFlagHost = 1;  // compress this stream with the host library

__constant__ uint32_t c_crc_table[256];

struct Geometry {
    uint32_t dims[5];   // x y z c t
    uint32_t bs[5];     // block size (clamped)
    uint32_t nb[5];     // blocks per dim
    uint32_t bpp;
};

struct Batch {
    // inputs
    const uint8_t* img;      // symbols / pixels, image layout (device)
    Geometry g;
    uint32_t first_block;    // global id of stream 0 of this batch
    uint32_t nstreams;
    uint32_t raw_cap;        // bytes reserved per stream for the raw block
    uint32_t cap;            // elements reserved per stream for the RLE1 block
    uint32_t level;          // blockSize100k
    uint32_t nblock_max;     // 100000 * level - 19
    uint32_t out_cap;        // bytes reserved per stream for the compressed stream
    // work buffers (per stream s at s * cap, etc.)
    uint8_t* raw;
    uint32_t* raw_len;
    uint8_t* T;              // RLE1 blocks
    uint32_t* n;             // RLE1 length
    uint32_t* crc;           // finalised block CRC
    uint32_t* inuse;         // 8 words per stream
    uint32_t* flags;
    uint32_t* done;          // BWT finished
    uint64_t* keys_a;
    uint64_t* keys_b;
    uint32_t* vals_a;        // rotation start indices (input of a sort)
    uint32_t* sa;            // sorted rotation starts (output of a sort)
    uint32_t* rank;
    uint32_t* vals_b;        // sorted values of the compacted rounds
    uint32_t* cl0;           // slots of unresolved rotations (compacted)
    uint32_t* cl1;
    uint8_t* uflag;          // per slot / per compacted entry: still tied
    uint32_t* seg_begin;
    uint32_t* seg_end;
    uint16_t* mtfv;          // cap + 8 per stream (16-byte aligned rows)
    uint32_t* nmtf;
    uint32_t* mtf_freq;      // kMaxAlpha per stream
    uint32_t* orig_ptr;
    uint8_t* sel;            // selectors, sel_cap per stream
    uint8_t* sel_mtf;
    uint32_t sel_cap;
    uint32_t* nsel;
    uint32_t* ngroups;
    uint8_t* len;            // kMaxGroups * kMaxAlpha per stream
    uint32_t* code;          // kMaxGroups * kMaxAlpha per stream
    uint32_t* rfreq;         // kMaxGroups * kMaxAlpha per stream
    uint32_t* words;         // out_cap / 4 per stream, MSB-first bit words
    uint32_t* out_bytes;
    uint32_t* wide;          // (stream, table) tasks whose heap weights exceed 17 bits
    uint32_t* wide_cnt;
    // two-stage BWT (bwt_bucket, bwt_induce)
    uint32_t* nsub;          // rotations sorted per stream (the A or B rotations, or all of them)
    uint32_t* bwt_mode;      // per stream: kModeSortA / kModeSortB / kModeFull
    uint32_t* abcnt;         // per stream: A rotations per first byte [256], then B rotations [256]
    uint32_t* itab;          // per stream: q0, p0, p1, s0 [256] each (bwt_bucket, for bwt_place_sorted)
    uint32_t* sfin;          // the final order of every rotation (bwt_place_sorted / bwt_induce)
    uint2* ent;              // bwt_induce's entries per final position (the keys_a area, free after the sorts)
    uint32_t it_full;        // sort every rotation (no induction): the fallback for ties that need doubling
};

__device__ __forceinline__ uint32_t crc_feed(uint32_t c, uint32_t b) { return (c << 8) ^ c_crc_table[(c >> 24) ^ b]; }

// ------------------------------------------------------------- gather --
// Block id -> origin/size, x fastest (klb_imageIO.cpp:133-140); the block's
// bytes are gathered x fastest, then y, z, c, t (blockCompressor).
__device__ __forceinline__ void block_box(const Geometry& g, uint32_t id, uint32_t org[5], uint32_t sz[5])
{
#pragma unroll
    for (int d = 0; d < 5; ++d) {
        const uint32_t q = id % g.nb[d];
        id /= g.nb[d];
        org[d] = q * g.bs[d];
        sz[d] = min(g.bs[d], g.dims[d] - org[d]);
    }
}

__global__ __launch_bounds__(256) void gather_blocks(Batch B)
{
    const uint32_t s = blockIdx.y;
    uint32_t org[5], sz[5];
    block_box(B.g, B.first_block + s, org, sz);
    const uint32_t rowb = sz[0] * B.g.bpp;
    const uint32_t nrows = sz[1] * sz[2] * sz[3] * sz[4];
    uint8_t* dst = B.raw + (size_t)s * B.raw_cap;
    for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
        uint32_t q = r;
        const uint32_t y = q % sz[1]; q /= sz[1];
        const uint32_t z = q % sz[2]; q /= sz[2];
        const uint32_t c = q % sz[3]; q /= sz[3];
        const uint32_t t = q;
        const size_t src = ((((size_t)(org[4] + t) * B.g.dims[3] + (org[3] + c)) * B.g.dims[2] + (org[2] + z)) *
                                B.g.dims[1] + (org[1] + y)) * B.g.dims[0] + org[0];
        const uint8_t* sp = B.img + src * B.g.bpp;
        uint8_t* dp = dst + (size_t)r * rowb;
        for (uint32_t i = threadIdx.x; i < rowb; i += blockDim.x) dp[i] = sp[i];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) B.raw_len[s] = rowb * nrows;
}

// ----------------------------------------------------------- RLE1 + CRC --
// One workgroup per stream walks the raw block in tiles of kRleTile bytes,
// kRleChunk bytes per thread (two 16-byte loads, straight from the image when
// the block rows are 16-byte granular, else from the gathered raw block):
//   * run summary of the chunk (first / last byte, leading / trailing run),
//     scanned across the tile (wave shuffles, then the waves) on top of the
//     run carried in from the previous tiles: the bzip2 run state at the
//     chunk start (a run restarts every 255 bytes from its first byte);
//   * the chunk's RLE1 bytes (bzlib.c ADD_CHAR_TO_BLOCK / flush_RL) counted,
//     placed by a scan of the counts into an LDS copy of the tile's output and
//     stored with coalesced writes;
//   * the chunk CRC (slicing by 4, tables in LDS) from a zero register (the
//     stream's first chunk from 0xffffffff), combined over the tile by a tree
//     of GF(2) "shift by 32 << k zero bytes" matrices and folded into the
//     stream CRC; the tail of the last tile is zero padding, removed at the
//     end by the inverse shift (the CRC is linear: crc(D . 0^p) = Z^p crc(D));
//   * inUse: bytes present (register masks, OR-reduced once) and run-length
//     bytes (LDS atomics, rare).
// Run summary of a byte range, combined left to right by the scan.
struct RunSum {
    uint32_t len;    // bytes in the range (0 = identity)
    uint32_t first, last;
    uint32_t lead;   // length of the leading run
    uint32_t trail;  // length of the trailing run
};

// (selects, no early returns: the scans keep RunSums in registers)
__device__ __forceinline__ RunSum run_combine(const RunSum& a, const RunSum& b)
{
    const bool ae = a.len == 0, be = b.len == 0;
    const bool join = a.last == b.first && !ae && !be;
    RunSum r;
    r.len = a.len + b.len;
    r.first = ae ? b.first : a.first;
    r.last = be ? a.last : b.last;
    r.lead = ae ? b.lead : ((join && a.lead == a.len) ? a.len + b.lead : a.lead);
    r.trail = be ? a.trail : ((join && b.trail == b.len) ? b.len + a.trail : b.trail);
    return r;
}

__device__ __forceinline__ RunSum run_shfl_up(const RunSum& a, int d)
{
    RunSum r;
    r.len = __shfl_up(a.len, d);
    r.first = __shfl_up(a.first, d);
    r.last = __shfl_up(a.last, d);
    r.lead = __shfl_up(a.lead, d);
    r.trail = __shfl_up(a.trail, d);
    return r;
}

// Visit the bytes p[0 .. len) in order with 16-byte loads (p 16-byte aligned;
// the load may read up to 15 bytes past len, inside the stream's buffer).
template <typename F>
__device__ __forceinline__ void for_bytes(const uint8_t* p, uint32_t len, F&& f)
{
    for (uint32_t k = 0; k < len; k += 16) {
        const uint4 v = *(const uint4*)(p + k);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (uint32_t b = 0; b < 16; ++b)
            if (k + b < len) f((w[b >> 2] >> (8 * (b & 3))) & 0xFFu);
    }
}

constexpr uint32_t kRleChunk = 32;
constexpr uint32_t kRleTile = kRleThreads * kRleChunk;  // 16 KiB
constexpr int kCrcLevels = 10;                          // shift by kRleChunk << k bytes, k = 0..9 (9: one tile)
constexpr int kCrcUnshift = 14;                         // inverse shift by 2^k bytes (padding < kRleTile)
static_assert(kRleTile == (kRleChunk << (kCrcLevels - 1)) && kRleTile == (1u << kCrcUnshift), "CRC tables");

__constant__ uint32_t c_crc4[4][256];  // 4 zero feeds of a register holding byte v at byte k
__constant__ uint32_t c_crc_unshift[kCrcUnshift][32];

// 32x32 GF(2) matrix as 32 columns (column k = image of bit k); m is a
// wave-uniform constant, so its columns are scalar loads
__device__ __forceinline__ uint32_t gf2_apply(const uint32_t* m, uint32_t v)
{
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 32; ++k) r ^= ((v >> k) & 1u) ? m[k] : 0u;
    return r;
}

// CRC shift by 32 << l zero bytes as byte tables: Z(v) = T[l][0][v & 255] ^
// T[l][1][(v >> 8) & 255] ^ T[l][2][(v >> 16) & 255] ^ T[l][3][v >> 24]
// (four LDS reads instead of a 32-column GF(2) product per lane)
__constant__ uint32_t c_crc_shb[kCrcLevels][4][256];

__device__ __forceinline__ uint32_t crc_shift_b(const uint32_t (*t)[256], uint32_t v)
{
    return t[0][v & 255u] ^ t[1][(v >> 8) & 255u] ^ t[2][(v >> 16) & 255u] ^ t[3][v >> 24];
}

// The bytes of a chunk as a bitmask: bit i set when byte i equals byte i - 1
// (bit 0 clear), i < nv, four bytes per word by a zero-byte test of
// w ^ (w << 8 | previous byte)
__device__ __forceinline__ uint32_t chunk_eq_mask(const uint32_t (&w)[kRleChunk / 4], uint32_t nv)
{
    uint32_t E = 0;
#pragma unroll
    for (uint32_t q = 0; q < kRleChunk / 4; ++q) {
        const uint32_t x = w[q], pb = q ? w[q - 1] >> 24 : x & 255u;
        const uint32_t y = x ^ ((x << 8) | pb);
        const uint32_t eq = ~((((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y)) & 0x80808080u;  // bit 7: byte equal
        const uint32_t e4 = ((eq >> 7) & 1u) | ((eq >> 14) & 2u) | ((eq >> 21) & 4u) | ((eq >> 28) & 8u);
        E |= e4 << (4 * q);
    }
    return E & ~1u & (nv >= 32 ? ~0u : (1u << nv) - 1u);
}

__device__ __forceinline__ uint32_t chunk_byte(const uint32_t (&w)[kRleChunk / 4], uint32_t i)
{
    uint32_t x = w[0];
#pragma unroll
    for (uint32_t q = 1; q < kRleChunk / 4; ++q) x = (i >> 2) == q ? w[q] : x;
    return (x >> (8 * (i & 3u))) & 255u;
}

template <bool FROM_IMG>
__global__ __launch_bounds__(kRleThreads) __attribute__((amdgpu_waves_per_eu(4))) void rle1_crc(Batch B)
{
    constexpr uint32_t NW = kRleThreads / 64;
    __shared__ uint32_t crc4[4][256];
    __shared__ uint32_t crcsh[kCrcLevels][4][256];
    // the tile's RLE1 bytes at tout[po ..), po = the stream offset mod 16:
    // tout[0 .. po) holds the previous tile's last partial 16-byte unit
    __shared__ __attribute__((aligned(16))) uint8_t tout[16 + kRleTile + kRleTile / 4 + 64];
    __shared__ uint8_t junk[kRleThreads];  // where a thread's skipped byte writes land
    __shared__ RunSum wrs[NW];
    __shared__ uint32_t wcnt[NW], wcrc[NW];
    __shared__ RunSum s_carry;
    __shared__ uint32_t s_wr, s_crc;
    const uint32_t s = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint32_t org[5], sz[5];
    block_box(B.g, B.first_block + s, org, sz);
    const uint32_t rowb = sz[0] * B.g.bpp;
    const uint32_t L = rowb * sz[1] * sz[2] * sz[3] * sz[4];
    const uint8_t* raw = B.raw + (size_t)s * B.raw_cap;
    // divisions by the block's row bytes and extents: float reciprocal and
    // one correction step (exact for x < 2^23, integer division above): a
    // 32-bit integer division is ~40 instructions, four per load
    struct FDiv {
        uint32_t d;
        float inv;
        __device__ __forceinline__ uint32_t div(uint32_t x) const
        {
            if (x >= (1u << 23)) return x / d;  // (huge blocks only)
            uint32_t q = (uint32_t)((float)x * inv);
            const int32_t r = (int32_t)(x - q * d);
            q += r >= (int32_t)d ? 1u : 0u;
            q -= r < 0 ? 1u : 0u;
            return q;
        }
    };
    const FDiv frow{rowb, 1.0f / (float)rowb}, fy{sz[1], 1.0f / (float)sz[1]}, fz{sz[2], 1.0f / (float)sz[2]},
        fc{sz[3], 1.0f / (float)sz[3]};
    auto load16 = [&](uint32_t g) -> uint4 {
        if (FROM_IMG) {  // rows are whole 16-byte pieces at 16-byte aligned addresses
            const uint32_t row = frow.div(g), col = g - row * rowb;
            uint32_t q = row, qn;
            qn = fy.div(q); const uint32_t y = q - qn * sz[1]; q = qn;
            qn = fz.div(q); const uint32_t z = q - qn * sz[2]; q = qn;
            qn = fc.div(q); const uint32_t c = q - qn * sz[3]; q = qn;
            const size_t src = ((((size_t)(org[4] + q) * B.g.dims[3] + (org[3] + c)) * B.g.dims[2] + (org[2] + z)) *
                                    B.g.dims[1] + (org[1] + y)) * B.g.dims[0] + org[0];
            return *(const uint4*)(B.img + src * B.g.bpp + col);
        } else {
            return *(const uint4*)(raw + g);
        }
    };
    for (uint32_t i = t; i < 1024; i += kRleThreads) crc4[i >> 8][i & 255] = c_crc4[i >> 8][i & 255];
    for (uint32_t i = t; i < kCrcLevels * 1024; i += kRleThreads)
        crcsh[i >> 10][(i >> 8) & 3][i & 255] = c_crc_shb[i >> 10][(i >> 8) & 3][i & 255];
    if (t == 0) {
        s_carry = RunSum{0, 0, 0, 0, 0};
        s_wr = 0;
        s_crc = 0;
    }
    uint8_t* Tout = B.T + (size_t)s * B.cap;
    const uint32_t wlim = B.cap - 8;  // RLE1 bytes past this are not stored (the stream goes to the host)
    // this thread's 32 bytes of a tile; the next tile's are loaded while this
    // one is processed
    // (unconditional loads at clamped offsets: a load under a branch makes the
    // compiler wait for every outstanding load at the next use)
    const uint32_t glim = FROM_IMG ? L - 16 : B.raw_cap - 16;  // L >= 16: rows are whole 16-byte pieces
    auto load_chunk = [&](uint32_t g, uint32_t nv, uint4& a, uint4& b) {
        const uint4 va = load16(min(g, glim)), vb = load16(min(g + 16, glim));
        const uint4 z = make_uint4(0, 0, 0, 0);
        a = nv ? va : z;
        b = nv > 16 ? vb : z;
    };
    uint4 na, nb;
    {
        const uint32_t g = t * kRleChunk;
        load_chunk(g, g < L ? min(kRleChunk, L - g) : 0u, na, nb);
    }
    __syncthreads();
    for (uint32_t tb = 0; tb < L; tb += kRleTile) {
        const uint32_t g = tb + t * kRleChunk;
        const uint32_t nv = g < L ? min(kRleChunk, L - g) : 0u;
        uint32_t w[8];
        w[0] = na.x; w[1] = na.y; w[2] = na.z; w[3] = na.w;
        w[4] = nb.x; w[5] = nb.y; w[6] = nb.z; w[7] = nb.w;
        {
            const uint32_t g2 = g + kRleTile;
            load_chunk(g2, g2 < L ? min(kRleChunk, L - g2) : 0u, na, nb);
        }
        if (nv < kRleChunk) {  // zero padding past L
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) {
                if (nv <= 4 * q) w[q] = 0;
                else if (nv < 4 * q + 4) w[q] &= (1u << (8 * (nv - 4 * q))) - 1u;
            }
        }
        // chunk CRC
        uint32_t cc = g == 0 ? 0xffffffffu : 0u;
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) {
            const uint32_t x = cc ^ __builtin_bswap32(w[q]);
            cc = crc4[3][x >> 24] ^ crc4[2][(x >> 16) & 255u] ^ crc4[1][(x >> 8) & 255u] ^ crc4[0][x & 255u];
        }
        // chunk run summary from the equal-neighbour mask
        const uint32_t Ein = chunk_eq_mask(w, nv);
        const uint32_t b0 = w[0] & 255u;
        const uint32_t blast = nv == kRleChunk ? w[7] >> 24 : chunk_byte(w, nv ? nv - 1 : 0u);
        RunSum rs{nv, b0, blast, 0, 0};
        if (nv) {
            rs.lead = 1u + (uint32_t)__builtin_ctz(~(Ein >> 1));
            rs.trail = 1u + (uint32_t)__clz(~(Ein << (32u - nv)));
        }
        // scan of the run summaries: wave, then waves, on top of the carry
        RunSum inc = rs;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const RunSum o = run_shfl_up(inc, d);
            if ((int)lane >= d) inc = run_combine(o, inc);
        }
        RunSum exc = run_shfl_up(inc, 1);
        if (lane == 0) exc = RunSum{0, 0, 0, 0, 0};
        if (lane == 63) wrs[wave] = inc;
        __syncthreads();
        RunSum pre = s_carry;
#pragma unroll
        for (uint32_t w2 = 0; w2 < NW - 1; ++w2) {
            const RunSum o = wrs[w2];
            if (w2 < wave) pre = run_combine(pre, o);
        }
        pre = run_combine(pre, exc);
        // the bzip2 run state at the chunk start: byte ch0 (256: none) in a
        // run piece of rl0 bytes (a piece restarts every 255 bytes)
        const uint32_t ch0 = pre.len ? pre.last : 256u, rl0 = pre.len ? (pre.trail - 1) % 255 + 1 : 0u;
        const bool has_end = nv && g + nv == L;
        const uint32_t valid = nv >= 32 ? ~0u : (1u << nv) - 1u;
        const uint32_t E = Ein | (nv && b0 == ch0 ? 1u : 0u);
        // a piece reaching 255 bytes splits only when the carried piece is that long
        const bool slow = rl0 >= 224 && (E & 1u);
        // byte i is copied when it is among the first four of its piece, and a
        // piece of >= 4 bytes ends with its count byte (written before the
        // next piece's first byte, or at the stream end): with Y = E << 3 | the
        // carried piece's bytes, r_i >= k <=> bits i .. i + k - 2 of Y set
        const uint64_t Y = ((uint64_t)E << 3) | (rl0 >= 4 ? 1u : 0u) | (rl0 >= 3 ? 2u : 0u) | (rl0 >= 2 ? 4u : 0u);
        const uint64_t Q = Y & (Y >> 1) & (Y >> 2);  // bit i: the piece through byte i - 1 has >= 4 bytes
        const uint32_t S = ~E & valid;               // bytes starting a piece
        const uint32_t omask = ~(uint32_t)(Q & (Y >> 3)) & valid;
        const uint32_t cmask = S & (uint32_t)Q;
        const bool endc = has_end && ((Q >> nv) & 1u);
        // the same bytes by the sequential state machine (a piece reaches
        // 255 bytes inside the chunk): emit(byte, is a count byte) in order
        auto walk = [&](auto&& emit) {
            uint32_t ch = ch0, r = rl0;
            for (uint32_t i = 0; i < nv; ++i) {
                const uint32_t c = chunk_byte(w, i);
                const bool same = c == ch && r < 255;
                if (!same && r >= 4) emit(r - 4, true);
                r = same ? r + 1 : 1u;
                ch = c;
                if (r <= 4) emit(c, false);
            }
            if (has_end && r >= 4) emit(r - 4, true);  // flush_RL of the final run
        };
        uint32_t cnt = 0;
        if (!slow) {
            cnt = (uint32_t)__popc(omask) + (uint32_t)__popc(cmask) + (endc ? 1u : 0u);
        } else {
            walk([&](uint32_t, bool) { ++cnt; });
        }
        uint32_t cinc = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(cinc, d);
            if ((int)lane >= d) cinc += o;
        }
        if (lane == 63) wcnt[wave] = cinc;
        // tile CRC: tree over the wave's chunks (byte tables of the shifts)
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const uint32_t o = __shfl_xor(cc, 1 << k);
            const bool right = (lane >> k) & 1u;
            cc = crc_shift_b(crcsh[k], right ? o : cc) ^ (right ? cc : o);
        }
        if (lane == 0) wcrc[wave] = cc;
        __syncthreads();
        const uint32_t wr0 = s_wr, po = wr0 & 15u;
        uint32_t base = po + cinc - cnt, total = 0;
        for (uint32_t w2 = 0; w2 < NW; ++w2) {
            if (w2 < wave) base += wcnt[w2];
            total += wcnt[w2];
        }
        if (!slow) {
            // copies in order, the count bytes after (each a few per chunk at most)
            uint32_t pos = base;
#pragma unroll
            for (uint32_t i = 0; i < kRleChunk; ++i) {
                pos += (cmask >> i) & 1u;
                const bool of = (omask >> i) & 1u;
                uint8_t* dst = of ? &tout[pos] : &junk[t];
                *dst = (uint8_t)(w[i >> 2] >> (8 * (i & 3u)));
                pos += of ? 1u : 0u;
            }
            uint32_t cm = cmask;
            while (cm) {
                const uint32_t i = (uint32_t)__builtin_ctz(cm);
                cm &= cm - 1u;
                const uint32_t lt = (1u << i) - 1u, m = S & lt;
                const uint32_t len = m ? i - (31u - (uint32_t)__clz(m)) : rl0 + i;
                tout[base + (uint32_t)__popc(omask & lt) + (uint32_t)__popc(cmask & lt)] = (uint8_t)(len - 4u);
            }
            if (endc) {
                const uint32_t m = S & valid;
                const uint32_t len = m ? nv - (31u - (uint32_t)__clz(m)) : rl0 + nv;
                tout[base + cnt - 1u] = (uint8_t)(len - 4u);
            }
        } else {
            walk([&](uint32_t v, bool) { tout[base++] = (uint8_t)v; });
        }
        RunSum ncarry{0, 0, 0, 0, 0};
        if (t == 0) {
            ncarry = s_carry;
#pragma unroll
            for (uint32_t w2 = 0; w2 < NW; ++w2) ncarry = run_combine(ncarry, wrs[w2]);
        }
        // the tile's CRC: wave CRCs shifted by the waves after them (lane
        // w < 8 of wave 0: (7 - w) * 2048 bytes, levels 6..8), xor-reduced,
        // on top of the stream CRC shifted by the tile (level 9)
        uint32_t ncrc = 0;
        if (wave == 0) {
            static_assert(NW == 8 && kRleChunk * 64 == (32u << 6), "wave CRC levels");
            uint32_t x = lane < NW ? wcrc[lane] : 0u;
            const uint32_t sh = NW - 1 - min(lane, NW - 1);
#pragma unroll
            for (int l = 0; l < 3; ++l) {
                const uint32_t y = crc_shift_b(crcsh[6 + l], x);
                x = (sh >> l) & 1u ? y : x;
            }
            x ^= __shfl_xor(x, 1);
            x ^= __shfl_xor(x, 2);
            x ^= __shfl_xor(x, 4);
            ncrc = crc_shift_b(crcsh[9], s_crc) ^ x;
        }
        __syncthreads();
        // whole 16-byte units out (16-byte stores; a unit starting before
        // wlim ends inside the 256-aligned cap), the last partial unit kept
        {
            const uint32_t end = po + total, full = end >> 4, ub = wr0 & ~15u;
            for (uint32_t u = t; u < full; u += kRleThreads)
                if (ub + 16u * u < wlim) *(uint4*)(Tout + ub + 16u * u) = *(const uint4*)(tout + 16u * u);
            const uint8_t keep = t < 16u ? tout[16u * full + t] : (uint8_t)0;
            __syncthreads();
            if (t < 16u) tout[t] = keep;
        }
        if (t == 0) {
            s_carry = ncarry;
            s_crc = ncrc;
            s_wr = wr0 + total;
        }
    }
    __syncthreads();
    {  // the stream's last partial unit (bytes past the end are not read)
        const uint32_t wr = s_wr;
        if ((wr & 15u) && t == 0 && (wr & ~15u) < wlim) *(uint4*)(Tout + (wr & ~15u)) = *(const uint4*)tout;
    }
    if (t == 0) {
        const uint32_t total = s_wr;
        uint32_t crc = s_crc;
        const uint32_t pad = (L + kRleTile - 1) / kRleTile * kRleTile - L;
        for (int j = 0; j < kCrcUnshift; ++j)
            if ((pad >> j) & 1u) crc = gf2_apply(c_crc_unshift[j], crc);
        const bool host = total >= B.nblock_max || total > wlim;
        B.crc[s] = L ? ~crc : 0u;
        B.n[s] = total;
        B.flags[s] = host ? kFlagHost : 0u;
        B.done[s] = host ? 1u : 0u;
        B.seg_begin[s] = s * B.cap;
        B.seg_end[s] = s * B.cap + (host ? 0u : total);
    }
    // the byte map of the RLE1 text comes from bwt_bucket's histogram
    if (t < 8) B.inuse[s * 8 + t] = 0u;
}

// ------------------------------------------------------------------ BWT --
// Sort values carry the rotation start i (bits 0-23, n < 2^20) and the byte
// preceding it (bits 24-31): after sorting, that byte IS the BWT output
// column, so the MTF stage reads it in sorted order without a gather.
constexpr uint32_t kIdxMask = 0x00FFFFFFu;
#ifndef LFM_BWT_PACK
#define LFM_BWT_PACK 0  // 1: bwt_chunk_sort sorts (key - min) << LJ | slot keys only where the range allows (measured no faster)
#endif
constexpr uint32_t kKeyBytes = 8;  // first-round key: the 8-byte prefix (0.02 % of rotations tie on symbols)

// First round: every rotation by its 8-byte prefix, in two steps.
//  bwt_bucket      one workgroup per stream: a counting sort of the rotations
//                  by their leading kBucketBits bits (byte 0, top bits of byte 1), the
//                  histogram in LDS; only the values are scattered (the sorters rebuild the 8-byte big-endian keys from the text).
//                  The stream's slot range is cut at bucket ends into chunks
//                  of < 2 kChunk rotations (a cut after the bucket that holds
//                  each multiple of kChunk; a bucket larger than kChunk is a
//                  chunk of its own).
//  bwt_chunk_sort  one workgroup per chunk: the chunk's rotations sorted by the
//                  whole key in LDS (buckets are ordered by the key's top bits,
//                  so sorting a run of whole buckets sorts each bucket), and
//                  the still-tied flags (equal keys never cross a bucket).
// On light-field symbols a 147k-rotation stream has ~1 000 buckets of at most
// ~2 000 rotations: each rotation is read and written once per step; the
// previous device-wide 60-bit radix sort made 8 HBM passes.  Chunks above the
// large sorter's capacity (one bucket of > kBigCap equal-prefix rotations) go
// to a rocPRIM segmented sort.
constexpr uint32_t kBucketBits = 14;               // 64 KiB histogram, two workgroups per CU (15 bits / one workgroup
                                                   // per CU measured 3 % slower end to end, 13 bits 18 % slower: more
                                                   // buckets overflow the small sorter)
constexpr int kBucketThreads = 1024;
constexpr uint32_t kBktTile = 4096;
constexpr uint32_t kChunk = 1024;  // (512 equal, 2 048 slower end to end in round 5)
constexpr int kCsThreads = 512, kCsItems = 4;      // chunks up to 2 048 (every multi-bucket chunk); 512 x 4 measured
                                                   // 10 % faster than 256 x 8
constexpr int kBigThreads = 512, kBigItems = 8;    // single buckets up to 4 096
constexpr uint32_t kSmallCap = kCsThreads * kCsItems, kBigCap = kBigThreads * kBigItems;
constexpr uint32_t kMaxCuts = 1024;                // >= 3 * cap / kChunk + 2

// chunk lists: [3] <= kTinyCap, [0] <= kSmallCap, [1] <= kBigCap, [2] larger
// (rocPRIM segmented sort)
constexpr uint32_t kTinyCap = 1024;  // half-size sorter: the ~40 % of chunks at most
                                     // this long would pad a kSmallCap sort to twice their size
struct ChunkLists {
    uint32_t* b[4];
    uint32_t* e[4];
    uint32_t* cnt;   // counters of classes 0..2
    uint32_t* cnt3;  // counter of class 3
};

// A tile of the text for the bucket pass: T[i0 - 1 .. i0 + m + 8) cyclically
// in tile[kTOff - 1 .. kTOff + m + 8), m = min(n - i0, kBktTile) (T[i0 + k]
// at tile[kTOff + k]: word-aligned stores).  bucket_fetch loads this
// thread's part (4 bytes; one edge byte for threads 0..8) into registers, a
// tile ahead of bucket_put, which stores it into LDS: the pass is a chain of
// tiles, and waiting for each tile's loads was most of its time.  Tiles
// alternate between two buffers, so one barrier per tile orders them.
constexpr uint32_t kTOff = 4;
struct BktPart {
    uint32_t w;
    uint32_t e;
};

__device__ __forceinline__ BktPart bucket_fetch(const uint8_t* __restrict__ T, uint32_t n, uint32_t i0)
{
    // loads at clamped offsets for every thread (no load under a branch: the
    // compiler would wait for all outstanding loads at the next use)
    const uint32_t t = threadIdx.x;
    const uint32_t i0c = min(i0, n ? n - 1 : 0u);
    const uint32_t m = n > i0c ? min(n - i0c, kBktTile) : 0u;
    // 4 bytes (may read up to 3 bytes past n: inside the stream's cap)
    const uint32_t w = *(const uint32_t*)(T + min(i0c + 4 * t, n ? (n - 1) & ~3u : 0u));
    uint32_t j = n ? (t < 8 ? (i0c + m + t) % n : (i0c ? i0c - 1 : n - 1)) : 0u;
    const uint32_t e = T[j];
    BktPart p;
    p.w = (i0 < n && 4 * t < m) ? w : 0u;
    p.e = (i0 < n && t <= 8) ? e : 0u;
    return p;
}

__device__ __forceinline__ uint32_t bucket_put(const BktPart& p, uint32_t n, uint32_t i0, uint8_t* tile)
{
    const uint32_t t = threadIdx.x;
    const uint32_t m = min(n - i0, kBktTile);
    if (4 * t + 4 <= m) {
        *(uint32_t*)(tile + kTOff + 4 * t) = p.w;
    } else if (4 * t < m) {  // the last partial word: its valid bytes only (the edge bytes follow)
        for (uint32_t b = 0; b < m - 4 * t; ++b) tile[kTOff + 4 * t + b] = (uint8_t)(p.w >> (8 * b));
    }
    if (t < 8) tile[kTOff + m + t] = (uint8_t)p.e;
    else if (t == 8) tile[kTOff - 1] = (uint8_t)p.e;
    return m;  // the caller's barrier publishes the tile
}

// LDS slot of bucket `key` (BITS bits: the first byte, then the top BITS - 8
// bits of the second).  A dword's bank is its index mod 32, i.e. the key's
// low bits -- the top bits of the SECOND byte, which on 16-bit little-endian
// symbols is the high byte (mostly 0) for every other rotation: half the
// lanes of an atomic landed on one bank with different addresses.  XOR-ing
// the low 5 bits with the first byte spreads them (a bijection; every access
// to the histogram goes through it).
template <uint32_t BITS>
__device__ __forceinline__ uint32_t bkt_slot(uint32_t key)
{
    return key ^ ((key >> (BITS - 8)) & 31u);
}

// Two-stage BWT (Itoh & Tanaka).  Rotation i is of type B when it sorts
// before rotation i + 1 (T[i] < T[i + 1], or equal bytes and i + 1 of type B)
// and of type A otherwise; the types of a non-periodic block are well defined
// cyclically.  Only the rotations of ONE type (about half) go through the sort
// below (bucket pass, chunk sorts, ties); bwt_induce places the others by one
// scan of the sorted order.  Inside the bucket of first byte c the A rotations
// come first; the A rotations of a bucket are ordered as their successors are
// (i + 1 precedes i in the final order) and the B rotations likewise (i + 1
// follows i).  So with the B rotations sorted a left-to-right scan places the
// A ones (kModeSortB), with the A rotations sorted a right-to-left scan places
// the B ones (kModeSortA).  The pass sorts the A rotations unless the B ones
// are clearly fewer: on 16-bit little-endian symbols the A rotations start at
// the low bytes, whose first byte spreads them over the buckets, while the B
// ones start at the (mostly zero) high bytes.  rot_type reads tile[kTOff + k + d]
// for d <= 8 (the tile holds 8 bytes past its end): 1 = B, 0 = A, 2 = still
// undecided after 8 equal bytes (only runs of 0xFB survive RLE1 that long: the
// stream is then sorted whole, kModeFull).
constexpr uint32_t kModeSortA = 0, kModeSortB = 1, kModeFull = 2;

__device__ __forceinline__ uint32_t rot_type(const uint8_t* tile, uint32_t k, uint32_t a, uint32_t b)
{
    if (a != b) return a < b ? 1u : 0u;
#pragma unroll 1
    for (uint32_t d = 1; d < 8; ++d) {
        const uint32_t x = tile[kTOff + k + d], y = tile[kTOff + 1 + k + d];
        if (x != y) return x < y ? 1u : 0u;
    }
    return 2u;
}

// does rotation k of the tile (first bytes a, b) go through the sort in `mode`
__device__ __forceinline__ bool rot_sorted(const uint8_t* tile, uint32_t k, uint32_t a, uint32_t b, uint32_t mode)
{
    return mode == kModeFull || rot_type(tile, k, a, b) == (mode == kModeSortB ? 1u : 0u);
}

template <uint32_t BITS>
__global__ __launch_bounds__(kBucketThreads) __attribute__((amdgpu_waves_per_eu(8))) void bwt_bucket(Batch B, ChunkLists L)
{
    constexpr uint32_t kBuckets = 1u << BITS;
    __shared__ uint32_t hist[kBuckets];  // 64 KiB at 14 bits
    __shared__ __attribute__((aligned(16))) uint8_t tiles[2][kBktTile + 16];
    __shared__ uint32_t cuts[kMaxCuts];
    __shared__ uint32_t wsum[kBucketThreads / 64], wcut[kBucketThreads / 64];
    __shared__ uint32_t ccount[4], cbase[4];
    __shared__ uint32_t sinuse[8];                  // bytes present in the RLE1 text (the stream's inUse map)
    __shared__ uint32_t cnt_u[256], cnt_s[256];     // unsorted / sorted rotations per first byte
    __shared__ uint32_t undecided, n_unsorted;
    __shared__ uint32_t tsum[8];
    const uint32_t s = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (B.flags[s] & kFlagHost) return;
    const uint32_t n = B.n[s];
    const uint8_t* T = B.T + (size_t)s * B.cap;
    const uint32_t o = s * B.cap;
    if (t < 4) ccount[t] = 0;
    if (t < 8) sinuse[t] = 0;
    // histogram of the BITS-bit bucket over the rotations to sort; the pass
    // restarts (at most twice) for the B rotations when they are clearly fewer
    // and for every rotation when a type is undecided
    uint32_t mode = B.it_full ? kModeFull : kModeSortA;
    for (;;) {
        for (uint32_t b = t; b < kBuckets; b += kBucketThreads) hist[b] = 0;
        if (t < 256) cnt_u[t] = cnt_s[t] = 0;
        if (t == 0) undecided = n_unsorted = 0;
        __syncthreads();
        // unsorted rotations starting with byte 0 (the high bytes of small
        // 16-bit symbols: about half of all rotations) are counted in a
        // register -- their LDS atomics all hit one word and serialise
        uint32_t u_zero = 0;
        // sorted rotations in buckets a << (BITS - 8) for a < 4 (a small low
        // byte, then a zero high byte: the hottest buckets) likewise, in
        // 16-bit register fields
        uint32_t hot01 = 0, hot23 = 0;
        BktPart nx = bucket_fetch(T, n, 0);
        for (uint32_t i0 = 0, it = 0; i0 < n; i0 += kBktTile, ++it) {
            const BktPart cur = nx;
            nx = bucket_fetch(T, n, i0 + kBktTile);
            uint8_t* tile = tiles[it & 1];
            const uint32_t m = bucket_put(cur, n, i0, tile);
            __syncthreads();
            for (uint32_t k = t; k < m; k += kBucketThreads) {
                const uint32_t a = tile[kTOff + k], b = tile[kTOff + 1 + k];
                const uint32_t ty = mode == kModeFull ? 3u : rot_type(tile, k, a, b);
                if (ty == 2u) undecided = 1u;
                else if (mode == kModeFull || ty == (mode == kModeSortB ? 1u : 0u)) {
                    const uint32_t key = (a << (BITS - 8)) | (b >> (16 - BITS));
                    if (key < (4u << (BITS - 8)) && (key & ((1u << (BITS - 8)) - 1u)) == 0u) {
                        const uint32_t inc = 1u << (16u * (a & 1u));
                        if (a < 2u) hot01 += inc;
                        else hot23 += inc;
                    } else {
                        atomicAdd(&hist[bkt_slot<BITS>(key)], 1u);
                    }
                }
                else if (a == 0u) ++u_zero;
                else atomicAdd(&cnt_u[a], 1u);
            }
        }
        if (u_zero) atomicAdd(&cnt_u[0], u_zero);
#pragma unroll
        for (uint32_t h = 0; h < 4; ++h) {
            const uint32_t c = ((h < 2u ? hot01 : hot23) >> (16u * (h & 1u))) & 0xFFFFu;
            if (c) atomicAdd(&hist[bkt_slot<BITS>(h << (BITS - 8))], c);
        }
        __syncthreads();
        if (mode == kModeFull) break;
        if (undecided) {
            mode = kModeFull;
        } else {
            if (t < 256 && cnt_u[t]) atomicAdd(&n_unsorted, cnt_u[t]);
            __syncthreads();
            // the other type clearly fewer (by 1/8): sort it instead
            if (mode != kModeSortA || (uint64_t)n_unsorted * 8 >= (uint64_t)(n - n_unsorted) * 7) break;
            mode = kModeSortB;
        }
        __syncthreads();
    }
    // exclusive scan of the buckets; chunk cuts at bucket ends
    constexpr uint32_t per = kBuckets / kBucketThreads;
    static_assert(per <= (1u << (BITS - 8)), "a thread's buckets share their first byte");
    uint32_t sum = 0;
    for (uint32_t q = 0; q < per; ++q) sum += hist[bkt_slot<BITS>(t * per + q)];
    if (sum) atomicAdd(&cnt_s[(t * per) >> (BITS - 8)], sum);
    uint32_t isum = sum;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t a = __shfl_up(isum, d);
        if ((int)lane >= d) isum += a;
    }
    if (lane == 63) wsum[wave] = isum;
    __syncthreads();
    uint32_t psum = 0, nsub = 0;
    for (uint32_t w = 0; w < kBucketThreads / 64; ++w) {
        if (w < wave) psum += wsum[w];
        nsub += wsum[w];
    }
    const uint32_t my0 = psum + isum - sum;
    // every byte of the text starts a rotation: byte c is present iff it
    // starts a sorted or an unsorted rotation
    if (t < 256 && (cnt_u[t] | cnt_s[t])) atomicOr(&sinuse[t >> 5], 1u << (t & 31));
    // the chunk sorts flag positions < nsub; tie_compact's 16-byte loads also
    // see up to 15 bytes past nsub, which must read as "not tied"
    if (t < 16 && nsub + t < B.cap) B.uflag[o + nsub + t] = 0;
    // cut positions of this thread's buckets (ascending): after a bucket that
    // holds a multiple of kChunk, and around a bucket larger than kChunk
    auto cuts_of = [&](auto&& emit) {
        uint32_t off = my0;
        for (uint32_t q = 0; q < per; ++q) {
            const uint32_t c = hist[bkt_slot<BITS>(t * per + q)];
            if (c) {
                const uint32_t e = off + c;
                if (c > kChunk) {
                    if (off) emit(off);
                    emit(e);
                } else if ((e - 1) / kChunk >= (off + kChunk - 1) / kChunk && e - 1 >= kChunk) {
                    emit(e);
                }
            }
            off += c;
        }
    };
    uint32_t ncut = 0;
    cuts_of([&](uint32_t) { ++ncut; });
    uint32_t icut = ncut;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t a = __shfl_up(icut, d);
        if ((int)lane >= d) icut += a;
    }
    if (lane == 63) wcut[wave] = icut;
    __syncthreads();
    uint32_t pcut = 0, tcut = 0;
    for (uint32_t w = 0; w < kBucketThreads / 64; ++w) {
        if (w < wave) pcut += wcut[w];
        tcut += wcut[w];
    }
    {
        uint32_t at = pcut + icut - ncut;
        cuts_of([&](uint32_t p) {
            if (at < kMaxCuts) cuts[at] = p;
            ++at;
        });
    }
    if (t < 8) B.inuse[s * 8 + t] = sinuse[t];  // (written after the scan's barrier)
    {  // A / B rotations per first byte for bwt_induce, and bwt_place_sorted's
       // tables: q-order start of bucket c (q0), its placed part (p0 .. p1)
       // and the first sa slot of its sorted rotations (s0)
        uint32_t na = 0, nb = 0, ns = 0, x = 0, y = 0;
        if (t < 256) {
            na = mode == kModeSortA ? cnt_s[t] : cnt_u[t];
            nb = mode == kModeSortA ? cnt_u[t] : cnt_s[t];
            ns = mode == kModeSortA ? na : nb;  // (kModeFull: all in the B counts)
            B.abcnt[(size_t)s * 512 + t] = na;
            B.abcnt[(size_t)s * 512 + 256 + t] = nb;
            x = na + nb;
            y = ns;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t a = __shfl_up(x, d), b = __shfl_up(y, d);
                if ((int)lane >= d) {
                    x += a;
                    y += b;
                }
            }
            if (lane == 63) {
                tsum[wave] = x;
                tsum[4 + wave] = y;
            }
        }
        __syncthreads();
        if (t < 256) {
            for (uint32_t w = 0; w < wave; ++w) {
                x += tsum[w];
                y += tsum[4 + w];
            }
            const uint32_t qs = x - na - nb;
            uint32_t* it = B.itab + (size_t)s * 1024;
            it[t] = qs;
            it[256 + t] = mode == kModeSortA ? qs + na : qs;
            it[512 + t] = mode == kModeSortA ? qs + na + nb : (mode == kModeSortB ? qs + na : qs);
            it[768 + t] = y - ns;
        }
    }
    if (t == 0) {
        B.nsub[s] = nsub;
        B.bwt_mode[s] = mode;
    }
    // bucket starts for the scatter
    {
        uint32_t off = my0;
        for (uint32_t q = 0; q < per; ++q) {
            const uint32_t c = hist[bkt_slot<BITS>(t * per + q)];
            hist[bkt_slot<BITS>(t * per + q)] = off;
            off += c;
        }
    }
    __syncthreads();
    // chunks = runs between consecutive cuts (the last ends at nsub)
    const uint32_t nch = min(tcut, kMaxCuts - 1) + 1;
    uint32_t cb = 0, ce = 0, cls = 0, slot = 0;
    if (t < nch) {
        cb = t ? cuts[t - 1] : 0u;
        ce = t + 1 < nch ? cuts[t] : nsub;
        const uint32_t m = ce > cb ? ce - cb : 0u;
        cls = m <= kTinyCap ? 3u : (m <= kSmallCap ? 0u : (m <= kBigCap ? 1u : 2u));
        if (m) slot = atomicAdd(&ccount[cls], 1u);
        else cb = ce;
    }
    __syncthreads();
    if (t < 4) cbase[t] = ccount[t] ? atomicAdd(t < 3 ? &L.cnt[t] : L.cnt3, ccount[t]) : 0u;
    __syncthreads();
    if (t < nch && ce > cb) {
        L.b[cls][cbase[cls] + slot] = o + cb;
        L.e[cls][cbase[cls] + slot] = o + ce;
    }
    // scatter of the values only (start | preceding byte << 24): the sorters
    // rebuild the 8-byte keys from the text (rot_key8_fast), which the L2s
    // hold, instead of 8-byte scattered key writes and their re-read
    BktPart nx = bucket_fetch(T, n, 0);
    for (uint32_t i0 = 0, it = 0; i0 < n; i0 += kBktTile, ++it) {
        const BktPart cur = nx;
        nx = bucket_fetch(T, n, i0 + kBktTile);
        uint8_t* tile = tiles[it & 1];
        const uint32_t m = bucket_put(cur, n, i0, tile);
        __syncthreads();
        for (uint32_t k = t; k < m; k += kBucketThreads) {
            const uint8_t* p = tile + kTOff + k;
            const uint32_t a = p[0], b = p[1];
            if (rot_sorted(tile, k, a, b, mode)) {
                const uint32_t pos = atomicAdd(&hist[bkt_slot<BITS>((a << (BITS - 8)) | (b >> (16 - BITS)))], 1u);
                B.vals_a[o + pos] = (i0 + k) | ((uint32_t)p[-1] << 24);
            }
        }
    }
}


// the first-round key of rotation i of a stream's text T (length n): its
// 8-byte prefix, big endian.  Away from the wrap, three aligned dwords (the
// stream's cap leaves >= 8 bytes after n) funnel-shifted; else byte by byte.
__device__ __forceinline__ uint64_t rot_key8_fast(const uint8_t* __restrict__ T, uint32_t n, uint32_t i)
{
    if (i + 8 <= n) {
        const uint32_t* w = (const uint32_t*)(T + (i & ~3u));
        const uint32_t d0 = w[0], d1 = w[1], d2 = w[2];
        const uint32_t sh = (i & 3u) * 8u;
        const uint64_t x = (uint64_t)d0 | ((uint64_t)d1 << 32);
        const uint64_t le = sh ? (x >> sh) | ((uint64_t)d2 << (64u - sh)) : x;
        return __builtin_bswap64(le);
    }
    uint64_t k = 0;
    uint32_t j = i;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        k = (k << 8) | T[j];
        j = j + 1 == n ? 0u : j + 1;
    }
    return k;
}

// text_prev4: T[i-2] | T[i-3] << 8 | T[i-4] << 16 | T[i-5] << 24 (cyclic)
__device__ __forceinline__ uint32_t text_prev4(const uint8_t* __restrict__ T, uint32_t n, uint32_t i)
{
    // two aligned dwords around T[i-5 .. i-2] (i - 1 < n: inside the text),
    // loaded at a clamped address; the first five rotations wrap
    const uint32_t a = i >= 5 ? i - 5 : 0u;
    const uint32_t* w = (const uint32_t*)(T + (a & ~3u));
    const uint64_t x = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    uint32_t r = __builtin_bswap32((uint32_t)(x >> ((a & 3u) * 8u)));
    if (i < 5) {
        r = 0;
        for (uint32_t k = 2; k <= 5; ++k) r |= (uint32_t)T[(i + 5 * n - k) % n] << (8 * (k - 2));
    }
    return r;
}

// keys_a for the chunks the rocPRIM segmented sort takes (one workgroup per chunk)
__global__ __launch_bounds__(256) void bwt_chunk_keys(Batch B, const uint32_t* __restrict__ cbp,
                                                      const uint32_t* __restrict__ cep)
{
    const uint32_t cb = cbp[blockIdx.x], ce = cep[blockIdx.x];
    const uint32_t s = cb / B.cap, n = B.n[s];
    const uint8_t* T = B.T + (size_t)s * B.cap;
    for (uint32_t j = cb + threadIdx.x; j < ce; j += 256) B.keys_a[j] = rot_key8_fast(T, n, B.vals_a[j] & kIdxMask);
}

// Runs of rotations whose 8-byte prefixes are equal, resolved right after the
// chunk sorts when short: at most kTieRunMax rotations, ordered by insertion
// on their cyclic text from byte kKeyBytes on, kTieCmpBytes at most per
// comparison (bzip2 orders the rotations of the block lexicographically).  A
// longer run, or one with a comparison still equal after kTieCmpBytes, is left
// to the device-wide tie rounds, whose result does not depend on the order
// the run is left in.
constexpr uint32_t kTieRunMax = 32;
constexpr uint32_t kTieCmpBytes = 64;

// -1 / 1: rotation i sorts before / after rotation j, given equal first
// kKeyBytes bytes; 0: still equal after kTieCmpBytes more
__device__ __forceinline__ int tie_cmp(const uint8_t* __restrict__ T, uint32_t n, uint32_t i, uint32_t j)
{
    uint32_t a = (i + kKeyBytes) % n, b = (j + kKeyBytes) % n;
    for (uint32_t d = 0; d < kTieCmpBytes; d += 8) {
        const uint64_t ka = rot_key8_fast(T, n, a), kb = rot_key8_fast(T, n, b);
        if (ka != kb) return ka < kb ? -1 : 1;
        a = (a + 8) % n;
        b = (b + 8) % n;
    }
    return 0;
}

// One thread per run of the tied list (the still-tied slots after the chunk
// sorts, in slot order; a run is consecutive slots of one prefix): the run's
// values in sa sorted in place.  The slots keep their flags, so tie rounds
// that still run (some run here too long or undecided: counted in *unres)
// re-sort the resolved runs to the same order; with *unres == 0 the host
// skips them.  A separate launch keeps the chunk sort's registers (inlined
// there, this code took it from 37 to 88 VGPRs and 8 to 5 waves per SIMD).
__global__ __launch_bounds__(256) void tie_runs_direct(Batch B, const uint32_t* __restrict__ cl,
                                                  const uint32_t* __restrict__ cnt_p, uint32_t* __restrict__ unres)
{
    const uint32_t cnt = *cnt_p;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < cnt; c += gridDim.x * blockDim.x) {
        const uint32_t slot = cl[c];
        const uint32_t s = slot / B.cap, n = B.n[s];
        const uint8_t* T = B.T + (size_t)s * B.cap;
        const uint64_t K = rot_key8_fast(T, n, B.sa[slot] & kIdxMask);
        if (c > 0 && cl[c - 1] == slot - 1 && rot_key8_fast(T, n, B.sa[slot - 1] & kIdxMask) == K) continue;
        uint32_t g = 1;
        while (c + g < cnt && g <= kTieRunMax && cl[c + g] == slot + g &&
               rot_key8_fast(T, n, B.sa[slot + g] & kIdxMask) == K)
            ++g;
        if (g > kTieRunMax) {
            atomicAdd(unres, 1u);
            continue;
        }
        uint32_t* sv = B.sa + slot;
        bool ok = true;
        for (uint32_t x = 1; x < g && ok; ++x) {
            const uint32_t vx = sv[x];
            uint32_t y = x;
            while (y > 0) {
                const int cmp = tie_cmp(T, n, sv[y - 1] & kIdxMask, vx & kIdxMask);
                if (cmp == 0) {  // undecided: the rounds re-sort the run (same elements, any order)
                    ok = false;
                    break;
                }
                if (cmp < 0) break;
                sv[y] = sv[y - 1];
                --y;
            }
            sv[y] = vx;
        }
        if (!ok) atomicAdd(unres, 1u);
    }
}

// Thread t's items of chunk [cb, cb + m), striped (item q is slot q * TH + t:
// coalesced): the values and their 8-byte keys rebuilt from the text; items
// past m get key ~0, value 0.  Every load is unconditional (clamped
// indices) and all of one kind are issued before any is used: one memory
// round trip for the values and one for the text of all IPT items (under
// per-item branches the compiler waited for each item's loads in turn: 2 IPT
// round trips).
template <int TH, int IPT>
__device__ __forceinline__ void chunk_load(const Batch& B, uint32_t cb, uint32_t m, uint32_t t, uint64_t (&k)[IPT],
                                           uint32_t (&v)[IPT])
{
    const uint32_t s = cb / B.cap, n = B.n[s];
    const uint8_t* T = B.T + (size_t)s * B.cap;
#pragma unroll
    for (int q = 0; q < IPT; ++q) v[q] = B.vals_a[cb + min(q * TH + t, m ? m - 1u : 0u)];
    uint32_t d[IPT][3];
#pragma unroll
    for (int q = 0; q < IPT; ++q) {
        const uint32_t i = v[q] & kIdxMask;
        const uint32_t* w = (const uint32_t*)(T + ((i + 8u <= n ? i : 0u) & ~3u));
        d[q][0] = w[0];
        d[q][1] = w[1];
        d[q][2] = w[2];
    }
#pragma unroll
    for (int q = 0; q < IPT; ++q) {
        const uint32_t j = q * TH + t, i = v[q] & kIdxMask;
        if (j >= m) {
            k[q] = ~0ull;
            v[q] = 0u;
        } else if (i + 8u <= n) {  // rot_key8_fast's fast path on the loaded dwords
            const uint32_t sh = (i & 3u) * 8u;
            const uint64_t x = (uint64_t)d[q][0] | ((uint64_t)d[q][1] << 32);
            k[q] = __builtin_bswap64(sh ? (x >> sh) | ((uint64_t)d[q][2] << (64u - sh)) : x);
        } else {
            k[q] = rot_key8_fast(T, n, i);
        }
    }
}

// The chunk's keys / values are loaded striped (element q * TH + t: coalesced),
// sorted (rocPRIM block merge sort: thread t ends with sorted positions
// t * IPT .. t * IPT + IPT - 1), the still-tied flags come from the
// neighbours in registers (each thread's edge keys through LDS), and sa /
// uflag go back striped through LDS.  The sorted keys are not stored: the few
// consumers (tie groups) recompute them from the text (rot_key8).
template <int TH, int IPT>
__global__ __launch_bounds__(TH) void bwt_chunk_sort(Batch B, const uint32_t* __restrict__ cbp,
                                                     const uint32_t* __restrict__ cep, uint32_t nch, uint32_t per)
{
    // per > 0: XCD-aware order (workgroup b runs on XCD b % 8; chunks
    // x * per .. x * per + per - 1, consecutive and mostly of one stream, all
    // go to XCD x, so a stream's text is pulled into one L2)
    const uint32_t c = per ? (blockIdx.x & 7u) * per + (blockIdx.x >> 3) : blockIdx.x;
    if (c >= nch) return;
    static_assert(IPT == 2 || IPT == 4 || IPT == 8, "flags are packed 2, 4 or 8 per thread");
    using Sort = rocprim::block_sort<uint64_t, TH, IPT, uint32_t, rocprim::block_sort_algorithm::merge_sort>;
    using SortK = rocprim::block_sort<uint64_t, TH, IPT, rocprim::empty_type, rocprim::block_sort_algorithm::merge_sort>;
    using ExK = rocprim::block_exchange<uint64_t, TH, IPT>;
    using ExV = rocprim::block_exchange<uint32_t, TH, IPT>;
    constexpr uint32_t NI = TH * IPT, NW = TH / 64;
    struct Xch {
        uint64_t first[TH], last[TH];
        uint32_t sv[NI];
        uint8_t fl[NI];
    };
    struct Packed {
        typename SortK::storage_type s;
        uint32_t sv[NI];  // the values by load slot
    };
    __shared__ union alignas(16) {
        typename Sort::storage_type s;
        typename ExK::storage_type ek;
        typename ExV::storage_type ev;
        Packed pk;
        Xch x;
    } sm;
    const uint32_t cb = cbp[c], ce = cep[c], m = ce - cb, t = threadIdx.x;
    uint64_t k[IPT];
    uint32_t v[IPT];
    chunk_load<TH, IPT>(B, cb, m, t, k, v);
    bool packed = false;
#if LFM_BWT_PACK
    // Keys only when they fit: the chunk's key range below 2^(64 - LJ), LJ
    // the bits of a load slot j < m, sorts (k - kmin) << LJ | j as one 64-bit
    // key (a third less to move per merge step than key + value; slots past m
    // get ~0, above every packed key, so the whole tile is sorted without a
    // valid count or a striped-to-blocked exchange); the values come back
    // through LDS by slot.
    {
        __shared__ uint64_t wlo[NW], whi[NW];
        uint64_t lo = ~0ull, hi = 0;
#pragma unroll
        for (int q = 0; q < IPT; ++q)
            if (q * TH + t < m) {
                lo = min(lo, k[q]);
                hi = max(hi, k[q]);
            }
        for (int d = 32; d > 0; d >>= 1) {
            lo = min(lo, (uint64_t)__shfl_xor(lo, d));
            hi = max(hi, (uint64_t)__shfl_xor(hi, d));
        }
        if ((t & 63) == 0) {
            wlo[t >> 6] = lo;
            whi[t >> 6] = hi;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t x = 0; x < NW; ++x) {
            lo = min(lo, wlo[x]);
            hi = max(hi, whi[x]);
        }
        const uint32_t LJ = 32u - (uint32_t)__builtin_clz(max(m, 2u) - 1u);
        if (((hi - lo) >> (64u - LJ)) == 0) {
            packed = true;
#pragma unroll
            for (int q = 0; q < IPT; ++q) {
                const uint32_t j = q * TH + t;
                if (j < m) sm.pk.sv[j] = v[q];
                k[q] = j < m ? ((k[q] - lo) << LJ) | j : ~0ull;
            }
            SortK().sort(k, sm.pk.s);
            __syncthreads();
            const uint64_t jm = (1ull << LJ) - 1ull;
#pragma unroll
            for (int q = 0; q < IPT; ++q) {
                const uint32_t pos = t * IPT + q;
                v[q] = pos < m ? sm.pk.sv[(uint32_t)(k[q] & jm)] : 0u;
                k[q] >>= LJ;  // (the tie flags compare these; positions >= m are never compared)
            }
            __syncthreads();
        }
    }
#endif
    if (!packed) {
        // the sort's valid-item count refers to the blocked arrangement
        ExK().striped_to_blocked(k, k, sm.ek);
        __syncthreads();
        ExV().striped_to_blocked(v, v, sm.ev);
        __syncthreads();
        Sort().sort(k, v, sm.s, m);
        __syncthreads();
    }
    sm.x.first[t] = k[0];
    sm.x.last[t] = k[IPT - 1];
    __syncthreads();
    const uint64_t kprev = t ? sm.x.last[t - 1] : 0ull, knext = t + 1 < (uint32_t)TH ? sm.x.first[t + 1] : 0ull;
    uint32_t nt = 0;
    uint64_t fpack = 0;
#pragma unroll
    for (int q = 0; q < IPT; ++q) {
        const uint32_t pos = t * IPT + q;
        const uint64_t lo = q ? k[q - 1] : kprev, hi = q + 1 < IPT ? k[q + 1] : knext;
        const bool f = pos < m && ((pos > 0 && lo == k[q]) || (pos + 1 < m && hi == k[q]));
        nt += f ? 1u : 0u;
        fpack |= (uint64_t)(f ? 1u : 0u) << (8 * q);
    }
    if constexpr (IPT == 2) {
        *(uint2*)&sm.x.sv[t * IPT] = make_uint2(v[0], v[1]);
        *(uint16_t*)&sm.x.fl[t * IPT] = (uint16_t)fpack;
    } else {
#pragma unroll
        for (int q = 0; q < IPT; q += 4) *(uint4*)&sm.x.sv[t * IPT + q] = make_uint4(v[q], v[q + 1], v[q + 2], v[q + 3]);
        if constexpr (IPT == 8) *(uint64_t*)&sm.x.fl[t * IPT] = fpack;
        else *(uint32_t*)&sm.x.fl[t * IPT] = (uint32_t)fpack;
    }
    __syncthreads();
    for (uint32_t j = t; j < m; j += TH) {
        B.sa[cb + j] = sm.x.sv[j];
        B.uflag[cb + j] = sm.x.fl[j];
    }
    if (__any(nt)) {
        for (int d = 32; d > 0; d >>= 1) nt += __shfl_xor(nt, d);
        if ((threadIdx.x & 63) == 0 && nt) atomicAdd(&B.done[cb / B.cap], nt);
    }
}

// bwt_chunk_rsort: bwt_chunk_sort's contract (a chunk's rotations ordered by
// their 8-byte big-endian prefix into sa, the still-tied flags into uflag and
// B.done) as a hand-written LDS radix sort, least significant digit first,
// over only the key bits that vary inside the chunk: D = OR(k) & ~AND(k) over
// its keys, and each pass takes the 8-bit digit at s, the next one at the
// lowest varying bit >= s + 8.  Bits constant across the chunk -- the
// bucket's leading bits, the zero high bits of small symbols' bytes -- cost no
// pass.  Ranking: a wave finds the lanes sharing an item's digit with 8
// ballots, keeps a running count per (digit, wave) in LDS, and one exclusive
// scan over the digit-major (digit, wave) counts gives every digit's start.
// Positions are ordered by wave, then item, then lane, so each pass is stable
// as LSD needs.  The order of equal keys is free (tie_runs_direct and the tie
// rounds order them), so the first pass ranks the items as loaded.
template <int TH, int IPT>
__global__ __launch_bounds__(TH) void bwt_chunk_rsort(Batch B, const uint32_t* __restrict__ cbp,
                                                      const uint32_t* __restrict__ cep, uint32_t nch, uint32_t per)
{
    const uint32_t c = per ? (blockIdx.x & 7u) * per + (blockIdx.x >> 3) : blockIdx.x;  // (XCD order, as bwt_chunk_sort)
    if (c >= nch) return;
    constexpr uint32_t NW = TH / 64, NI = TH * IPT, WI = 64 * IPT;
    static_assert(256 * NW == 4 * TH, "four (digit, wave) counters per thread");
    __shared__ uint64_t sk[NI];
    __shared__ uint32_t sv[NI];
    __shared__ uint32_t hist[256 * NW];  // [digit][wave]
    __shared__ uint32_t wsum[NW];
    __shared__ uint64_t wor[NW], wand[NW];
    const uint32_t cb = cbp[c], ce = cep[c], m = ce - cb, t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint64_t k[IPT];
    uint32_t v[IPT];
    chunk_load<TH, IPT>(B, cb, m, t, k, v);
    {  // the varying bits
        uint64_t o = 0, a = ~0ull;
#pragma unroll
        for (int q = 0; q < IPT; ++q)
            if (q * TH + t < m) {
                o |= k[q];
                a &= k[q];
            }
        for (int d = 32; d > 0; d >>= 1) {
            o |= __shfl_xor(o, d);
            a &= __shfl_xor(a, d);
        }
        if (lane == 0) {
            wor[w] = o;
            wand[w] = a;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) hist[4 * t + e] = 0;
    }
    __syncthreads();
    uint64_t D = 0, A = ~0ull;
#pragma unroll
    for (uint32_t x = 0; x < NW; ++x) {
        D |= wor[x];
        A &= wand[x];
    }
    D &= ~A;
    const uint64_t lt = (1ull << lane) - 1ull;
    bool first = true;
    for (uint32_t s = D ? (uint32_t)__builtin_ctzll(D) : 64u; s < 64u;) {
        uint32_t r[IPT], dg[IPT];
#pragma unroll
        for (int q = 0; q < IPT; ++q) {
            const bool ok = first ? q * TH + t < m : w * WI + q * 64 + lane < m;
            const uint32_t d = (uint32_t)(k[q] >> s) & 0xFFu;
            uint64_t same = __ballot(ok);
#pragma unroll
            for (int b = 0; b < 8; ++b) {  // keep the lanes whose bit b equals this lane's
                const int32_t e = (int32_t)(d << (31 - b)) >> 31;  // 0 / -1
                const uint64_t bb = __ballot(e != 0);
                same &= ~(bb ^ (uint64_t)(int64_t)e);
            }
            const uint32_t below = __popcll(same & lt);
            uint32_t* h = &hist[d * NW + w];
            const uint32_t base = ok ? *h : 0u;
            if (ok && below == 0) *h = base + __popcll(same);
            r[q] = ok ? base + below : ~0u;
            dg[q] = d;
        }
        __syncthreads();
        {  // exclusive scan of the counts, digit-major
            const uint32_t x0 = hist[4 * t], x1 = hist[4 * t + 1], x2 = hist[4 * t + 2], x3 = hist[4 * t + 3];
            const uint32_t sum = x0 + x1 + x2 + x3;
            uint32_t inc = sum;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(inc, d);
                if ((int)lane >= d) inc += y;
            }
            if (lane == 63) wsum[w] = inc;
            __syncthreads();
            uint32_t p = inc - sum;
            for (uint32_t x = 0; x < w; ++x) p += wsum[x];
            hist[4 * t] = p;
            hist[4 * t + 1] = p + x0;
            hist[4 * t + 2] = p + x0 + x1;
            hist[4 * t + 3] = p + x0 + x1 + x2;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < IPT; ++q)
            if (r[q] != ~0u) {
                const uint32_t to = hist[dg[q] * NW + w] + r[q];
                sk[to] = k[q];
                sv[to] = v[q];
            }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < IPT; ++q) {
            const uint32_t p = w * WI + q * 64 + lane;
            k[q] = sk[p];
            v[q] = sv[p];
        }
        // this wave's counters back to zero (every wave has read its
        // digits' starts before the barrier; only this wave counts into them)
#pragma unroll
        for (int e = 0; e < 4; ++e) hist[(lane + 64 * e) * NW + w] = 0;
        first = false;
        const uint64_t rest = s + 8u < 64u ? D >> (s + 8u) : 0ull;
        s = rest ? s + 8u + (uint32_t)__builtin_ctzll(rest) : 64u;
    }
    if (first) {  // every key equal: no pass ran, the items as loaded
#pragma unroll
        for (int q = 0; q < IPT; ++q)
            if (q * TH + t < m) {
                sk[q * TH + t] = k[q];
                sv[q * TH + t] = v[q];
            }
        __syncthreads();
    }
    uint32_t nt = 0;
    for (uint32_t j = t; j < m; j += TH) {
        const uint64_t kj = sk[j];
        const bool f = (j > 0 && sk[j - 1] == kj) || (j + 1 < m && sk[j + 1] == kj);
        B.sa[cb + j] = sv[j];
        B.uflag[cb + j] = f ? 1 : 0;
        nt += f ? 1u : 0u;
    }
    if (__any(nt)) {
        for (int d = 32; d > 0; d >>= 1) nt += __shfl_xor(nt, d);
        if (lane == 0 && nt) atomicAdd(&B.done[cb / B.cap], nt);
    }
}

// the first-round key of rotation i of stream s: its 8-byte prefix, big endian
__device__ __forceinline__ uint64_t rot_key8(const Batch& B, uint32_t s, uint32_t i)
{
    const uint32_t n = B.n[s];
    const uint8_t* T = B.T + (size_t)s * B.cap;
    uint64_t k = 0;
    uint32_t j = i;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        k = (k << 8) | T[j];
        j = j + 1 == n ? 0u : j + 1;
    }
    return k;
}

// still-tied flag of sorted position j of a chunk [cb, ce) (keys_b)
__device__ __forceinline__ uint8_t tied_flag(const uint64_t* __restrict__ K, uint32_t cb, uint32_t ce, uint32_t j,
                                             uint64_t k)
{
    return ((j > cb && K[j - 1] == k) || (j + 1 < ce && K[j + 1] == k)) ? 1 : 0;
}

// flags of the chunks sorted by rocPRIM (one workgroup per chunk)
__global__ __launch_bounds__(256) void bwt_chunk_flags(Batch B, const uint32_t* __restrict__ cbp,
                                                       const uint32_t* __restrict__ cep)
{
    const uint32_t cb = cbp[blockIdx.x], ce = cep[blockIdx.x];
    uint32_t nt = 0;
    for (uint32_t j = cb + threadIdx.x; j < ce; j += blockDim.x) {
        const uint8_t f = tied_flag(B.keys_b, cb, ce, j, B.keys_b[j]);
        B.uflag[j] = f;
        nt += f;
    }
    for (int d = 32; d > 0; d >>= 1) nt += __shfl_xor(nt, d);
    if ((threadIdx.x & 63) == 0 && nt) atomicAdd(&B.done[cb / B.cap], nt);
}

// The tied list (slots whose 8-byte prefix is shared), in slot order: per
// stream offsets of the tie counts (one workgroup), then each stream with
// ties compacts its flags (B.done = ties per stream -> exclusive offsets).
__global__ __launch_bounds__(1024) void tie_offsets(Batch B, uint32_t* __restrict__ total)
{
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x, ns = B.nstreams;
    const uint32_t per = (ns + 1023) / 1024;
    const uint32_t s0 = min(ns, t * per), s1 = min(ns, s0 + per);
    uint32_t sum = 0;
    for (uint32_t s = s0; s < s1; ++s) sum += B.done[s];
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint32_t v = t >= off ? part[t - off] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t acc = part[t] - sum;
    for (uint32_t s = s0; s < s1; ++s) {
        const uint32_t c = B.done[s];
        B.done[s] = c ? acc : ~0u;
        acc += c;
    }
    if (t == 1023) *total = part[1023];
}

__global__ __launch_bounds__(256) void tie_compact(Batch B, uint32_t* __restrict__ cl)
{
    __shared__ uint32_t wsum[4];
    __shared__ uint32_t carry;
    const uint32_t s = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t base = B.done[s];
    if (base == ~0u) return;
    const uint32_t n = B.nsub[s], o = s * B.cap;
    if (t == 0) carry = base;
    __syncthreads();
    for (uint32_t j0 = 0; j0 < n; j0 += 256 * 16) {
        const uint32_t j = j0 + 16 * t;
        uint4 w = make_uint4(0, 0, 0, 0);
        if (j < n) w = *(const uint4*)(B.uflag + o + j);  // uflag is zero past n (cap is a multiple of 256)
        const uint32_t c = __popc(w.x) + __popc(w.y) + __popc(w.z) + __popc(w.w);  // flags are 0 / 1 bytes
        uint32_t inc = c;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t a = __shfl_up(inc, d);
            if ((int)lane >= d) inc += a;
        }
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        uint32_t at = carry + inc - c;
        for (uint32_t w2 = 0; w2 < wave; ++w2) at += wsum[w2];
        if (c) {
            const uint32_t words[4] = {w.x, w.y, w.z, w.w};
            for (int q = 0; q < 16; ++q)
                if ((words[q >> 2] >> (8 * (q & 3))) & 1u) cl[at++] = o + j + q;
        }
        __syncthreads();
        if (t == 255) carry = at;
        __syncthreads();
    }
}

// After the first sort (6-byte prefixes, sa): rank[sa[j]] = first
// sorted position of j's group, uflag[slot] = 1 where j's group has more than
// one rotation.  Tiles of 1024 consecutive positions keep every load
// coalesced; the group start is a running max carried across tiles.
__global__ __launch_bounds__(1024) void bwt_rank0(Batch B)
{
    __shared__ uint32_t wmax[16];
    __shared__ uint32_t carry;
    const uint32_t s = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (B.flags[s] & kFlagHost) return;
    const uint32_t n = B.n[s];
    const size_t o = (size_t)s * B.cap;
    const uint32_t* SA = B.sa + o;
    auto K = [&](uint32_t j) { return rot_key8(B, s, SA[j] & kIdxMask); };  // keys from the text (fallback path)
    if (t == 0) carry = 0;
    __syncthreads();
    for (uint32_t j0 = 0; j0 < n; j0 += 1024) {
        const uint32_t j = j0 + t;
        bool head = false, next_head = true;
        if (j < n) {
            // Flag contract: the chunk sort flags every slot whose 8-byte key
            // equals a neighbour's; tie_runs_direct re-orders such runs from
            // the text but leaves their flags set, so the rounds below re-sort
            // them to the same order.  A slot joins its predecessor's group
            // when it is flagged and its key equals the predecessor's.  Equal
            // keys never straddle a chunk (chunks end at bucket ends), so an
            // equal key implies the flag; the flag test only saves the key
            // comparison for unflagged slots.  Both flags are read before the
            // barrier ahead of the rewrite.
            const bool fj = B.uflag[o + j] != 0;
            const bool fn = j + 1 < n && B.uflag[o + j + 1] != 0;
            const uint64_t k = K(j);
            head = j == 0 || !fj || k != K(j - 1);
            next_head = j + 1 >= n || !fn || K(j + 1) != k;
        }
        uint32_t v = head ? j : 0u;
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t u = __shfl_up(v, off);
            if ((int)lane >= off) v = max(v, u);
        }
        if (lane == 63) wmax[wave] = v;
        __syncthreads();
        uint32_t pre = carry;
        for (uint32_t w = 0; w < wave; ++w) pre = max(pre, wmax[w]);
        const uint32_t g = max(pre, v);
        if (j < n) {
            B.rank[o + (SA[j] & kIdxMask)] = g;
            B.uflag[o + j] = (head && next_head) ? 0 : 1;
        }
        __syncthreads();
        if (t == 1023) carry = g;
        __syncthreads();
    }
}

// Tie resolution by more text.  After the first sort only the rotations in
// a group of equal 6-byte prefixes are still unordered (2.4 % on light-field
// symbols, 0.01 % after 11 bytes): they are re-sorted inside their groups by
// the next 5 bytes of text, kTextRounds times, without the inverse suffix
// array (a random 4-byte scatter per rotation) that prefix doubling needs.
// Only ties that survive those rounds (long repeats) fall back to doubling.
constexpr int kTextRounds = 3;
constexpr uint32_t kTextBytes = 5;

__global__ __launch_bounds__(256) void text_gather_keys(Batch B, const uint32_t* __restrict__ cl,
                                                        const uint32_t* __restrict__ cnt_p, uint64_t* __restrict__ gk)
{
    const uint32_t cnt = *cnt_p;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < cnt; c += gridDim.x * blockDim.x) {
        const uint32_t slot = cl[c];
        gk[c] = rot_key8(B, slot / B.cap, B.sa[slot] & kIdxMask);
    }
}

// group starts of the tied list (equal keys, same stream)
__global__ __launch_bounds__(256) void text_bounds(Batch B, const uint32_t* __restrict__ cl,
                                                   const uint32_t* __restrict__ cnt_p, const uint64_t* __restrict__ gk,
                                                   uint32_t* __restrict__ bnd)
{
    const uint32_t cnt = *cnt_p;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < cnt; c += gridDim.x * blockDim.x)
        bnd[c] = (c == 0 || gk[c] != gk[c - 1] || cl[c] / B.cap != cl[c - 1] / B.cap) ? 1u : 0u;
}

// key = (group index, next kTextBytes of the rotation at offset `off`)
__global__ __launch_bounds__(256) void text_keys(Batch B, const uint32_t* __restrict__ cl,
                                                 const uint32_t* __restrict__ cnt_p, const uint32_t* __restrict__ gidx,
                                                 uint32_t off, uint32_t tb)
{
    const uint32_t cnt = *cnt_p;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < cnt; c += gridDim.x * blockDim.x) {
        const uint32_t slot = cl[c];
        const uint32_t s = slot / B.cap;
        const uint32_t n = B.n[s];
        const uint8_t* T = B.T + (size_t)s * B.cap;
        const uint32_t v = B.sa[slot];
        uint32_t j = (v & kIdxMask) + (off % n);
        if (j >= n) j -= n;
        uint64_t k = 0;
#pragma unroll
        for (uint32_t q = 0; q < kTextBytes; ++q) {
            if (q < tb) {
                k = (k << 8) | T[j];
                j = j + 1 == n ? 0 : j + 1;
            }
        }
        B.keys_a[c] = ((uint64_t)(gidx[c] - 1) << (8 * tb)) | k;
        B.vals_a[c] = v;
    }
}

// refined order back into sa; still-tied flags of the list
__global__ __launch_bounds__(256) void text_write(Batch B, const uint32_t* __restrict__ cl,
                                                  const uint32_t* __restrict__ cnt_p)
{
    const uint32_t cnt = *cnt_p;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < cnt; c += gridDim.x * blockDim.x) {
        B.sa[cl[c]] = B.vals_b[c];
        const uint64_t k = B.keys_b[c];
        B.uflag[c] = ((c > 0 && B.keys_b[c - 1] == k) || (c + 1 < cnt && B.keys_b[c + 1] == k)) ? 1 : 0;
    }
}

// fallback to doubling: rank[i] = sorted slot of rotation i for every rotation
// (the tied ones are fixed up to their group start by text_rank_tied)
__global__ __launch_bounds__(256) void bwt_rank_all(Batch B, size_t N)
{
    for (size_t slot = blockIdx.x * (size_t)blockDim.x + threadIdx.x; slot < N;
         slot += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s = (uint32_t)(slot / B.cap);
        const uint32_t j = (uint32_t)(slot - (size_t)s * B.cap);
        const uint32_t n = (B.flags[s] & kFlagHost) ? 0u : B.n[s];
        if (j < n) B.rank[(size_t)s * B.cap + (B.sa[slot] & kIdxMask)] = j;
    }
}

__global__ __launch_bounds__(256) void text_head_slots(const uint32_t* __restrict__ cl, const uint32_t* __restrict__ cnt_p,
                                                       const uint32_t* __restrict__ bnd, uint32_t* __restrict__ hv)
{
    const uint32_t cnt = *cnt_p;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < cnt; c += gridDim.x * blockDim.x)
        hv[c] = bnd[c] ? cl[c] : 0u;
}

__global__ __launch_bounds__(256) void text_rank_tied(Batch B, const uint32_t* __restrict__ cl,
                                                      const uint32_t* __restrict__ cnt_p, const uint32_t* __restrict__ hvs)
{
    const uint32_t cnt = *cnt_p;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < cnt; c += gridDim.x * blockDim.x) {
        const uint32_t head = hvs[c];
        const size_t o = (size_t)(head / B.cap) * B.cap;
        B.rank[o + (B.sa[cl[c]] & kIdxMask)] = (uint32_t)(head - o);
    }
}

// keys of a compacted doubling round: (stream slot of the group start,
// rank[i + h]) -- groups never mix, and inside a group the order is by the
// rank of the rotation h further on
__global__ __launch_bounds__(256) void bwt_comp_keys(Batch B, const uint32_t* __restrict__ cl,
                                                     const uint32_t* __restrict__ cnt_p, uint32_t h)
{
    const uint32_t cnt = *cnt_p;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < cnt; c += gridDim.x * blockDim.x) {
        const uint32_t slot = cl[c];
        const uint32_t s = slot / B.cap;
        const size_t o = (size_t)s * B.cap;
        const uint32_t n = B.n[s];
        const uint32_t v = B.sa[slot];
        const uint32_t i = v & kIdxMask;
        uint32_t i2 = i + (h % n);
        if (i2 >= n) i2 -= n;
        B.keys_a[c] = ((uint64_t)(o + B.rank[o + i]) << 20) | B.rank[o + i2];
        B.vals_a[c] = v;
    }
}

// write the refined order back into sa and mark the new group heads
__global__ __launch_bounds__(256) void bwt_comp_heads(Batch B, const uint32_t* __restrict__ cl,
                                                      const uint32_t* __restrict__ cnt_p, uint32_t* __restrict__ hv)
{
    const uint32_t cnt = *cnt_p;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < cnt; c += gridDim.x * blockDim.x) {
        B.sa[cl[c]] = B.vals_b[c];
        const bool head = c == 0 || B.keys_b[c] != B.keys_b[c - 1];
        hv[c] = head ? cl[c] : 0u;
    }
}

// new ranks (slot of the new group head) and the still-tied flags
__global__ __launch_bounds__(256) void bwt_comp_rank(Batch B, const uint32_t* __restrict__ cnt_p,
                                                     const uint32_t* __restrict__ hvs)
{
    const uint32_t cnt = *cnt_p;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < cnt; c += gridDim.x * blockDim.x) {
        const uint32_t head_slot = hvs[c];
        const uint32_t s = head_slot / B.cap;
        const size_t o = (size_t)s * B.cap;
        B.rank[o + (B.vals_b[c] & kIdxMask)] = (uint32_t)(head_slot - o);
        const bool head = c == 0 || B.keys_b[c] != B.keys_b[c - 1];
        const bool next_head = c + 1 >= cnt || B.keys_b[c + 1] != B.keys_b[c];
        B.uflag[c] = (head && next_head) ? 0 : 1;
    }
}

// rotations still tied after h covers the whole block: equal rotations of a
// periodic block -> the host library produces that stream
__global__ __launch_bounds__(256) void bwt_flag_periodic(Batch B, const uint32_t* __restrict__ cl,
                                                         const uint32_t* __restrict__ cnt_p)
{
    const uint32_t cnt = *cnt_p;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < cnt; c += gridDim.x * blockDim.x)
        atomicOr(&B.flags[cl[c] / B.cap], kFlagHost);
}

__device__ __forceinline__ void make_u2s(const Batch& B, uint32_t s, uint8_t* u2s, uint32_t lane, uint32_t* nin_out)
{
    uint32_t inu[8], nin = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        inu[q] = B.inuse[s * 8 + q];
        nin += __popc(inu[q]);
    }
    for (uint32_t c = lane; c < 256; c += 64) {
        uint32_t below = 0;
        for (uint32_t q = 0; q < (c >> 5); ++q) below += __popc(inu[q]);
        below += __popc(inu[c >> 5] & ((1u << (c & 31)) - 1u));
        u2s[c] = (uint8_t)below;
    }
    *nin_out = nin;
}

// ------------------------------------------------------------ induction --
// bwt_place_sorted + bwt_induce: the final order from the sorted rotations.
// In the final order (position q) bucket c (first byte c) holds its A
// rotations, then its B rotations.  One type is sorted (sa); the other is
// placed by one scan: kModeSortB scans left to right placing the A rotations,
// kModeSortA scans right to left placing the B rotations.  In "scan order" v
// (q, or n - 1 - q) with bytes mirrored the same way (x' = x, or 255 - x),
// bucket u = c' starts with its placed part, and the rotation i met in bucket u
// induces i - 1 when b' = T[i-1]' > u, or b' == u and i was placed itself;
// i - 1 takes the next free slot of bucket b''s placed part (head[b']).
//
// Entries: lo = i | nprev << 20 | placed << 23 | T[i-1] << 24 (the sort
// value's layout, bits 20-23 free since n < 2^20), hi = T[i-2] | T[i-3] << 8
// | T[i-4] << 16 | T[i] << 24: nprev of the three bytes before T[i-1] are
// valid (3 for a sorted rotation, one fewer per induction: a longer chain of
// placed rotations reads the text), and T[i] is the rotation's bucket.
// bwt_place_sorted writes the sorted entries to their final positions in
// `ent` and kIndPend to every position still to place; bwt_induce then
// reads nothing else, and writes every position's sort value to sfin.
constexpr uint32_t kIndPend = 0xFFFFFFFFu;  // never an entry: nprev <= 3
constexpr uint32_t kIndIdx = 0xFFFFFu;      // n < nblock_max < 2^20
constexpr uint32_t kIndPlaced = 1u << 23;
constexpr uint32_t kPlaceChunk = 2048;  // (1 024, 4 096, 8 192 equal or slower end to end)  // sorted slots / positions per bwt_place_sorted workgroup

// One workgroup per kPlaceChunk sorted slots and final positions of a
// stream, the chunks of a stream consecutive on one XCD (workgroup w runs on
// XCD w % 8): the text reads are random inside the stream, so a stream's text
// should stay in one L2 while its chunks run.
__global__ __launch_bounds__(256) void bwt_place_sorted(Batch B, uint32_t chunks)
{
    __shared__ uint32_t q0[256], p0[256], p1[256], s0[256];
    __shared__ uint8_t u2s[256];
    const uint32_t t = threadIdx.x, k = blockIdx.x >> 3;
    const uint32_t s = (blockIdx.x & 7u) + 8u * (k / chunks), base = (k % chunks) * kPlaceChunk;
    if (s >= B.nstreams || (B.flags[s] & kFlagHost)) return;
    const uint32_t n = B.n[s], ns = B.nsub[s], mode = B.bwt_mode[s];
    if (base >= n) return;
    if (mode == kModeFull && t < 64) {
        uint32_t nin;
        make_u2s(B, s, u2s, t, &nin);
    }
    {
        const uint32_t* it = B.itab + (size_t)s * 1024;
        q0[t] = it[t];
        p0[t] = it[256 + t];
        p1[t] = it[512 + t];
        s0[t] = it[768 + t];
    }
    __syncthreads();
    const size_t o = (size_t)s * B.cap;
    const uint8_t* T = B.T + o;
    uint8_t* LL = (uint8_t*)B.mtfv + o;  // the BWT output symbols (mtf_last<true> and mtf_win read them)
    uint2* E = B.ent + o;
    // the sorted slots [base, base + kPlaceChunk): sa, then T[i-4 .. i], all
    // loads issued before any is used
    constexpr int K = kPlaceChunk / 256;
    uint32_t v[K], w0[K], w1[K];
#pragma unroll
    for (int q = 0; q < K; ++q) v[q] = B.sa[o + min(base + q * 256 + t, ns ? ns - 1 : 0u)];
#pragma unroll
    for (int q = 0; q < K; ++q) {  // two aligned dwords (clamped; the first four rotations wrap)
        const uint32_t i = v[q] & kIdxMask, a = i >= 4 ? i - 4 : 0u;
        const uint32_t* w = (const uint32_t*)(T + (a & ~3u));
        w0[q] = w[0];
        w1[q] = w[1];
    }
#pragma unroll
    for (int q = 0; q < K; ++q) {
        const uint32_t j = base + q * 256 + t;
        if (j >= ns) break;
        const uint32_t i = v[q] & kIdxMask;
        uint32_t x;  // T[i-4] | T[i-3] << 8 | T[i-2] << 16 | T[i-1] << 24
        uint32_t c;  // T[i]
        if (i >= 4) {
            const uint32_t sh = ((i - 4) & 3u) * 8u;
            const uint64_t d = (uint64_t)w0[q] | ((uint64_t)w1[q] << 32);
            x = (uint32_t)(d >> sh);
            c = (uint32_t)(d >> (sh + 32)) & 0xFFu;
        } else {
            x = 0;
            for (uint32_t r = 1; r <= 4; ++r) x |= (uint32_t)T[(i + 4 * n - r) % n] << (32 - 8 * r);
            c = T[i];
        }
        const uint32_t qq = (mode == kModeSortA ? q0[c] : p1[c]) + (j - s0[c]);
        if (mode == kModeFull) {  // the final order already: the symbol, and origPtr at rotation 0
            LL[qq] = u2s[v[q] >> 24];
            if (i == 0) B.orig_ptr[s] = qq;
        }
        else
            E[qq] = make_uint2(v[q] | (3u << 20),
                               ((x >> 16) & 0xFFu) | (((x >> 8) & 0xFFu) << 8) | ((x & 0xFFu) << 16) | (c << 24));
    }
    // the positions [base, base + kPlaceChunk) still to place: the buckets
    // overlapping the range, from the last one starting at or before base
    const uint32_t end = min(n, base + kPlaceChunk);
    uint32_t lo = 0, hi = 255;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (q0[mid] <= base) lo = mid;
        else hi = mid - 1;
    }
    for (uint32_t c = lo; c < 256 && q0[c] < end; ++c)
        for (uint32_t q = max(p0[c], base) + t; q < min(p1[c], end); q += 256) E[q] = make_uint2(kIndPend, 0u);
}

// bwt_induce: one wave per stream scans in scan order, in blocks of
// kIndSlices slices of 64 positions through an LDS ring of two blocks:
// entries placed into the current or the next block go to the ring, those
// further ahead to `ent`; while a block is scanned the next block's entries
// are loaded (LDS-DMA, 16 bytes per lane) and written into the ring after the
// scan (kIndPend = not placed yet).  The final values of a block collect in
// LDS and leave in 16-byte stores: the wave's memory instructions, not its
// arithmetic, bound the scan (each store stays outstanding for thousands of
// cycles with every CU storing), so there are few and wide ones.  The
// inducing lanes of a slice are ranked per b' with one ballot per distinct b'
// (the predecessors of a run of sorted rotations take few distinct bytes), so
// the slots follow the scan order; an entry still pending when its slice is
// scanned is placed by an earlier lane of the same slice: the step then runs
// in rounds up to its first pending lane.
constexpr uint32_t kIndSlices = 8;
constexpr uint32_t kIndBlock = 64 * kIndSlices;
constexpr int kIndStepSlices = 4;  // slices scanned together (2 and 8 measured slower in the pipeline)
constexpr uint32_t kIndRing = 2 * kIndBlock;

// LDS-DMA of 16 bytes per lane into LDS at `lds` + 16 * lane, from L2 (sc1:
// the entries were written by this wave earlier, and a line may sit in the
// L1 from the previous block's load).  Inline asm: the compiler does not
// track the DMA, so nothing of it ties up VGPRs while the wave works
// (bwt_induce waits with vm_drain before it reads the staged entries).
__device__ __forceinline__ void glds16(const void* g, const void* lds)
{
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(
        (uint32_t)(size_t)(const __attribute__((address_space(3))) void*)lds);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc1" ::"s"(m0), "v"(g) : "memory", "m0");
}

__device__ __forceinline__ void glds4(const uint32_t* g, const void* lds)  // 4 bytes per lane
{
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(
        (uint32_t)(size_t)(const __attribute__((address_space(3))) void*)lds);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dword %1, off sc1" ::"s"(m0), "v"(g) : "memory", "m0");
}

__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__global__ __launch_bounds__(64) void bwt_induce(Batch B)
{
    __shared__ uint32_t head[256];            // next free scan position of bucket u's placed part
    __shared__ uint2 ring[kIndRing];
    __shared__ __attribute__((aligned(16))) uint2 stg[kIndBlock + 32];      // the next block's entries, in q order
    __shared__ __attribute__((aligned(16))) uint8_t fin[kIndBlock + 32];  // the block's symbols, in q order
    __shared__ uint8_t u2s[256];
    const uint32_t s = blockIdx.x, lane = threadIdx.x;
    if (B.flags[s] & kFlagHost) return;
    const uint32_t n = B.n[s];
    const uint32_t mode = B.bwt_mode[s];
    if (n == 0 || mode == kModeFull) return;  // kModeFull: bwt_place_sorted wrote the final order
    const bool rev = mode == kModeSortA;      // right to left, mirrored bytes
    const uint32_t mir = rev ? 255u : 0u;
    const size_t o = (size_t)s * B.cap;
    uint8_t* LL = (uint8_t*)B.mtfv + o;  // the BWT output symbols (mtf_last<true> and mtf_win read them)
    uint2* E = B.ent + o;
    const uint8_t* T = B.T + o;
    uint32_t nin;
    make_u2s(B, s, u2s, lane, &nin);
    const bool u2s_id = nin == 256;  // every byte in use: the map is the identity
    {  // head[u] = scan-order start of bucket u (its placed part comes first)
        uint32_t nt[4], l = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t c = (4 * lane + q) ^ mir;
            nt[q] = B.abcnt[(size_t)s * 512 + c] + B.abcnt[(size_t)s * 512 + 256 + c];
            l += nt[q];
        }
        uint32_t x = l;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d);
            if ((int)lane >= d) x += y;
        }
        x -= l;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            head[4 * lane + q] = x;
            x += nt[q];
        }
    }
    for (uint32_t i = lane; i < kIndRing; i += 64) ring[i].x = kIndPend;
    // position in `ent` / ll of scan position v.  A block [vb, vb + kIndBlock)
    // covers q in [qwin(vb), qwin(vb) + kIndBlock); stg holds it from q =
    // qwin & ~1, fin from q = qwin & ~15 (16-byte aligned transfers)
    const uint32_t qa = rev ? n - 1 : 0u;
    auto qof = [&](uint32_t v) { return rev ? qa - v : v; };
    auto qwin = [&](uint32_t vb) { return rev ? (int)n - (int)kIndBlock - (int)vb : (int)vb; };
    // slot of the block's t-th position in a buffer starting d before qwin
    auto wof = [&](uint32_t t, int d) { return rev ? (uint32_t)d + kIndBlock - 1 - t : t; };
    const int qmax = (int)B.cap - 2;
    auto issue = [&](uint32_t vb) {  // the block at vb into stg (clamped: every lane loads)
        const int qw = qwin(vb), qs = qw & ~1;
#pragma unroll
        for (uint32_t j = 0; j < kIndBlock / 128; ++j) {
            const int q = min(max(qs + (int)(128 * j + 2 * lane), 0), qmax);
            glds16(E + q, &stg[128 * j]);
        }
        if (qw & 1) {  // the block's last slot: entry qs + kIndBlock, one dword per lane 0 and 1
            const int q = min(max(qs + (int)kIndBlock, 0), qmax);
            glds4((const uint32_t*)(E + q) + min(lane, 1u), &stg[kIndBlock]);
        }
    };
    auto stage = [&](uint32_t vb) {  // into the ring: entries known when loaded
        const int d = qwin(vb) & 1;
        vm_drain();
        uint2 x[kIndSlices];
#pragma unroll
        for (uint32_t k = 0; k < kIndSlices; ++k) x[k] = stg[wof(64 * k + lane, d)];
        asm volatile("" ::: "memory");  // every read issued before the first write
#pragma unroll
        for (uint32_t k = 0; k < kIndSlices; ++k) {
            const uint32_t v = vb + 64 * k + lane;
            if (v < n && x[k].x != kIndPend) ring[v % kIndRing] = x[k];
        }
    };
    auto flush = [&](uint32_t vb) {  // the block's symbols to ll, 16 bytes per lane
        const int qw = qwin(vb), qf = qw & ~15;
        const int lo = max(qw, 0), hi = min(qw + (int)kIndBlock, (int)n);  // the block's positions
        const uint32_t w = 16 * lane;
        if (w < kIndBlock + 32 && (int)w < hi - qf) {
            uint4 f = *(const uint4*)&fin[w];  // the bytes before each rotation, mapped to symbols here
            if (!u2s_id) {
                uint32_t* fw = &f.x;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t x = fw[r];
                    fw[r] = (uint32_t)u2s[x & 255u] | ((uint32_t)u2s[(x >> 8) & 255u] << 8) |
                            ((uint32_t)u2s[(x >> 16) & 255u] << 16) | ((uint32_t)u2s[x >> 24] << 24);
                }
            }
            const int q = qf + (int)w;
            if (q >= lo && q + 15 < hi) {
                *(uint4*)(LL + q) = f;
            } else {
                const uint32_t fv[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (q + r >= lo && q + r < hi) LL[q + r] = (uint8_t)(fv[r >> 2] >> (8 * (r & 3)));
            }
        }
    };
    __syncthreads();
    issue(0);
    stage(0);
    bool bad = false;  // inconsistent counts or a pending entry no earlier lane places (never)
    uint32_t org = ~0u;
    for (uint32_t v0 = 0; v0 < n && !bad; v0 += kIndBlock) {
        // the next block's ring slots held the previous block: not placed yet
#pragma unroll
        for (uint32_t k = 0; k < kIndSlices; ++k) ring[(v0 + kIndBlock + 64 * k + lane) % kIndRing].x = kIndPend;
        const bool more = v0 + kIndBlock < n;
        if (more) issue(v0 + kIndBlock);
        // steps of kIndStepSlices slices: item k of lane l is position
        // vs + 64 k + l, and the scan order is (k, l)
        for (uint32_t vs = v0; vs < min(n, v0 + kIndBlock) && !bad; vs += 64 * kIndStepSlices) {
            constexpr int KS = kIndStepSlices;
            uint2 e[KS];
            uint64_t todo[KS];
#pragma unroll
            for (int k = 0; k < KS; ++k) {
                const uint32_t v = vs + 64 * k + lane;
                todo[k] = __ballot(v < n);
                e[k] = ring[v % kIndRing];
            }
            // rounds up to the first pending entry: one round unless an entry
            // of the step is placed by an earlier one of the same step
            for (;;) {
                uint64_t act[KS], pend[KS], anyp = 0;
#pragma unroll
                for (int k = 0; k < KS; ++k) {
                    pend[k] = __ballot(e[k].x == kIndPend) & todo[k];
                    anyp |= pend[k];
                }
                if (!anyp) {
#pragma unroll
                    for (int k = 0; k < KS; ++k) act[k] = todo[k];
                } else {
                    bool seen = false;
                    uint64_t any = 0;
#pragma unroll
                    for (int k = 0; k < KS; ++k) {
                        const uint64_t pk = pend[k];
                        act[k] = seen ? 0ull : (pk ? todo[k] & ((pk & (0ull - pk)) - 1ull) : todo[k]);
                        seen = seen || pk;
                        any |= act[k];
                    }
                    if (!any) {
                        bad = true;
                        break;
                    }
                }
                uint32_t b[KS];
                bool ind[KS];
                uint64_t rem[KS], left = 0;
#pragma unroll
                for (int k = 0; k < KS; ++k) {
                    const bool me = (act[k] >> lane) & 1u;
                    const uint32_t lo = e[k].x, hi = e[k].y;
                    b[k] = (lo >> 24) ^ mir;
                    const uint32_t u = (hi >> 24) ^ mir;
                    ind[k] = me && (b[k] > u || (b[k] == u && (lo & kIndPlaced)));
                    if (me) fin[wof(vs - v0 + 64 * k + lane, qwin(v0) & 15)] = (uint8_t)(lo >> 24);
                    org = me && (lo & kIndIdx) == 0 ? qof(vs + 64 * k + lane) : org;  // origPtr: rotation 0
                    rem[k] = __ballot(ind[k]);
                    left |= rem[k];
                }
                if (left) {
                    // ranks among the inducing entries with the same b, in
                    // scan order: a round of ballots per distinct b
                    uint32_t rank[KS], tot_of[KS];
                    bool inm[KS];
#pragma unroll
                    for (int k = 0; k < KS; ++k) {
                        rank[k] = 0;
                        tot_of[k] = 0;
                    }
                    while (left) {
                        uint32_t bl = 0;
                        bool got = false;
#pragma unroll
                        for (int k = 0; k < KS; ++k)
                            if (!got && rem[k]) {
                                bl = (uint32_t)__builtin_amdgcn_readlane((int)b[k], __builtin_ctzll(rem[k]));
                                got = true;
                            }
                        uint32_t sb = 0;
                        left = 0;
#pragma unroll
                        for (int k = 0; k < KS; ++k) {
                            const uint64_t m = __ballot(b[k] == bl) & rem[k];
                            inm[k] = (m >> lane) & 1u;
                            const uint32_t r =
                                sb + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                            rank[k] = inm[k] ? r : rank[k];
                            sb += (uint32_t)__popcll(m);
                            rem[k] &= ~m;
                            left |= rem[k];
                        }
#pragma unroll
                        for (int k = 0; k < KS; ++k) tot_of[k] = inm[k] ? sb : tot_of[k];
                    }
                    uint32_t dest[KS];
#pragma unroll
                    for (int k = 0; k < KS; ++k) dest[k] = head[b[k]] + rank[k];  // all reads first
#pragma unroll
                    for (int k = 0; k < KS; ++k)
                        if (ind[k] && rank[k] == 0) head[b[k]] = dest[k] + tot_of[k];
                    bool over = false, np0 = false;
                    uint32_t plo[KS], phi[KS];
#pragma unroll
                    for (int k = 0; k < KS; ++k) {
                        over = over || (ind[k] && dest[k] >= n);
                        // entry of i - 1: T[p-1] = T[i-2] ... and T[p] = T[i-1]
                        const uint32_t lo = e[k].x, hi = e[k].y;
                        const uint32_t idx = lo & kIndIdx, np = (lo >> 20) & 7u;
                        const uint32_t p = idx ? idx - 1 : n - 1;
                        plo[k] = p | ((np - 1) << 20) | kIndPlaced | ((hi & 0xFFu) << 24);
                        phi[k] = ((hi >> 8) & 0xFFFFu) | (lo & 0xFF000000u);
                        np0 = np0 || (ind[k] && np == 0);
                    }
                    if (__any(over)) {
                        bad = true;
                        break;
                    }
                    if (__any(np0)) {
#pragma unroll
                        for (int k = 0; k < KS; ++k) {
                            const uint32_t lo = e[k].x;
                            if (!ind[k] || ((lo >> 20) & 7u)) continue;
                            // a chain of placed rotations longer than the carried bytes
                            const uint32_t idx = lo & kIndIdx, p = idx ? idx - 1 : n - 1;
                            const uint32_t x = text_prev4(T, n, p + 1);  // T[p-1] .. T[p-4]
                            plo[k] = p | (3u << 20) | kIndPlaced | ((x & 0xFFu) << 24);
                            phi[k] = ((x >> 8) & 0xFFFFFFu) | (lo & 0xFF000000u);
                        }
                    }
#pragma unroll
                    for (int k = 0; k < KS; ++k) {
                        const bool near = dest[k] < v0 + kIndRing;
                        if (ind[k] && near) ring[dest[k] % kIndRing] = make_uint2(plo[k], phi[k]);
                        if (ind[k] && !near) E[qof(dest[k])] = make_uint2(plo[k], phi[k]);
                    }
                }
                if (!anyp) break;
                uint64_t rest = 0;
#pragma unroll
                for (int k = 0; k < KS; ++k) {
                    todo[k] &= ~act[k];
                    rest |= todo[k];
                }
                if (!rest) break;
#pragma unroll
                for (int k = 0; k < KS; ++k) e[k] = ring[(vs + 64 * k + lane) % kIndRing];
            }
        }
        if (!bad) flush(v0);
        if (more && !bad) stage(v0 + kIndBlock);
    }
    if (bad && lane == 0) B.flags[s] |= kFlagHost;  // the host library redoes the stream
    if (org != ~0u) B.orig_ptr[s] = org;
}

// ------------------------------------------------------------------ MTF --
// compress.c generateMTFValues in three parallel steps.  The move-to-front
// list in front of position j is a function of the last occurrences before
// j: symbols ordered by their last occurrence (most recent first), then the
// never-seen symbols in their initial order.  So every 4096-symbol segment of
// a stream can run its own MTF once those last occurrences are known:
//   mtf_last    per segment: the sorted symbols ll[j] (inUse-mapped bytes
//               before each sorted rotation) and each symbol's last position
//   mtf_prefix  per stream: exclusive running max over the segments
//   mtf_seg     per segment, one wave: initial list from the ranks of those
//               positions, then the sequential MTF (list packed 4 entries per
//               lane; lookups by ballot, shifts by a one-lane wave rotate)
//   rle2        per stream: zero runs -> RUNA/RUNB digits, v -> v + 1, EOB,
//               symbol frequencies (the run state is carried across thread
//               chunks by a scan, as in rle1_crc)
constexpr uint32_t kSeg = 4096;


// FROM_LL: bwt_place_sorted / bwt_induce already wrote the symbols ll[] (and
// origPtr); else (a batch sorted whole) they come from sa here
template <bool FROM_LL>
__global__ __launch_bounds__(256) void mtf_last(Batch B, uint32_t nseg_max, int32_t* __restrict__ seg_last)
{
    __shared__ uint8_t u2s[4][256];
    __shared__ int32_t last[4][256];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t s = blockIdx.y, k = blockIdx.x * 4 + wave;
    if (B.flags[s] & kFlagHost) return;
    const uint32_t n = B.n[s];
    const uint32_t j0 = k * kSeg;
    if (j0 >= n) return;
    const size_t o = (size_t)s * B.cap;
    uint32_t nin;
    make_u2s(B, s, u2s[wave], lane, &nin);
    for (uint32_t c = lane; c < 256; c += 64) last[wave][c] = -1;
    __builtin_amdgcn_wave_barrier();
    uint8_t* llbuf = (uint8_t*)B.mtfv + o;  // the mtfv area is free until rle2
    const uint32_t j1 = min(n, j0 + kSeg);
    // four consecutive positions per lane (16-byte loads of sa, 4-byte stores
    // of the symbols), loaded an iteration ahead at a clamped, aligned index
    // (sa holds cap >= n + 8 entries per stream)
    const uint32_t jlast = (j1 - 1) & ~3u;
    uint4 vn;
    uint32_t wn = 0;
    if constexpr (FROM_LL) wn = *(const uint32_t*)(llbuf + min(j0 + 4 * lane, jlast));
    else vn = *(const uint4*)(B.sa + o + min(j0 + 4 * lane, jlast));
    for (uint32_t jb = j0; jb < j1; jb += 256) {
        const uint32_t j = jb + 4 * lane;
        uint32_t ll[4];
        if constexpr (FROM_LL) {
            const uint32_t w4 = wn;
            wn = *(const uint32_t*)(llbuf + min(j + 256, jlast));
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) ll[q] = (w4 >> (8 * q)) & 0xFFu;
        } else {
            const uint4 v4 = vn;
            vn = *(const uint4*)(B.sa + o + min(j + 256, jlast));
            const uint32_t v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
                ll[q] = u2s[wave][v[q] >> 24];
                if (j + q < j1 && (v[q] & kIdxMask) == 0) B.orig_ptr[s] = j + q;  // BZ2_blockSort: origPtr = sorted position of rotation 0
            }
            if (j + 3 < j1) {
                *(uint32_t*)(llbuf + j) = ll[0] | (ll[1] << 8) | (ll[2] << 16) | (ll[3] << 24);
            } else {
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q)
                    if (j + q < j1) llbuf[j + q] = (uint8_t)ll[q];
            }
        }
        // only the last position of each run of equal symbols can be the
        // symbol's last: the BWT output is runs, and 64 lanes on one LDS word
        // serialise
        const uint32_t nxt0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)ll[0], 0x130, 0xF, 0xF, false);  // wave_shl:1
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            const uint32_t pos = j + q;
            const uint32_t nx = q < 3 ? ll[q + 1] : nxt0;
            const bool end = pos + 1 >= j1 || (q == 3 && lane == 63) || nx != ll[q];
            if (pos < j1 && end) atomicMax(&last[wave][ll[q]], (int32_t)pos);
        }
    }
    __builtin_amdgcn_wave_barrier();
    int32_t* dst = seg_last + ((size_t)s * nseg_max + k) * 256;
    for (uint32_t c = lane; c < 256; c += 64) dst[c] = last[wave][c];
}

__global__ __launch_bounds__(256) void mtf_prefix(Batch B, uint32_t nseg_max, int32_t* __restrict__ seg_last)
{
    const uint32_t s = blockIdx.x, c = threadIdx.x;
    if (B.flags[s] & kFlagHost) return;
    const uint32_t nseg = (B.n[s] + kSeg - 1) / kSeg;
    int32_t lb = -1;
    for (uint32_t k = 0; k < nseg; ++k) {
        int32_t* p = seg_last + ((size_t)s * nseg_max + k) * 256 + c;
        const int32_t v = *p;
        *p = lb;
        lb = max(lb, v);
    }
}

// Window-parallel MTF (the default): one wave per 4096-symbol segment walks it
// in windows of 64 positions, one lane per position, with the list state
// (P = place of each symbol, L = symbol at each place) in LDS.  For position
// l of a window whose symbol c occurred earlier in the window at p:
//     m = number of distinct symbols at positions (p, l),
// otherwise (first occurrence in the window)
//     m = P(c) + number of distinct earlier window symbols d with P(d) > P(c),
// P taken at the window start.  Distinct counts come from the match masks
// (ds_or_b64 per symbol): position i is the last occurrence before l of its
// symbol unless some k < l has i as its previous occurrence, so with
// U_l = OR_{k<l} bit(prev_k) the distinct symbols of (p, l) are the bits of
// lanemask_lt(l) & ~U_l above p.  After the window the list becomes the window
// symbols by last occurrence (most recent first) followed by the old list
// without them.
__device__ __forceinline__ void wsync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t ballot64(bool p) { return __ballot(p); }

// exclusive prefix OR of a 64-bit value over the wave's lanes with DPP row
// shifts and row broadcasts (VALU only: the ds_bpermute shuffles it replaces
// were a chain of 14 LDS round trips per 64-position window)
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_get(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_or_scan_excl32(uint32_t x)
{
    x |= dpp_get<0x111, 0xF>(x);  // row_shr:1
    x |= dpp_get<0x112, 0xF>(x);  // row_shr:2
    x |= dpp_get<0x114, 0xF>(x);  // row_shr:4
    x |= dpp_get<0x118, 0xF>(x);  // row_shr:8
    x |= dpp_get<0x142, 0xA>(x);  // row_bcast:15 into rows 1 and 3
    x |= dpp_get<0x143, 0xC>(x);  // row_bcast:31 into rows 2 and 3
    return dpp_get<0x138, 0xF>(x);  // wave_shr:1: exclusive
}
__device__ __forceinline__ uint64_t wave_or_scan_excl(uint64_t x)
{
    return ((uint64_t)wave_or_scan_excl32((uint32_t)(x >> 32)) << 32) | wave_or_scan_excl32((uint32_t)x);
}

#ifndef LFM_MTF_BALLOT
#define LFM_MTF_BALLOT 0  // 1: mtf_win's match masks by eight ballots instead of LDS atomicOr (measured slower)
#endif
__global__ __launch_bounds__(256) void mtf_win(Batch B, uint32_t nseg_max, const int32_t* __restrict__ seg_last)
{
    __shared__ int32_t key[4][256];
#if !LFM_MTF_BALLOT
    __shared__ uint64_t mt[4][256];
#endif
    __shared__ uint8_t Pt[4][256], Lt[4][256], inw[4][256];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t s = blockIdx.y, k = blockIdx.x * 4 + wave;
    if (B.flags[s] & kFlagHost) return;
    const uint32_t n = B.n[s];
    const uint32_t js = k * kSeg;
    if (js >= n) return;
    const size_t o = (size_t)s * B.cap;
    uint32_t nin = 0;
    for (int q = 0; q < 8; ++q) nin += __popc(B.inuse[s * 8 + q]);
    // list at js: seen symbols by last position (descending), then the unseen
    // ones by symbol index (ascending) -- key(unseen c) = -1 - c
    const int32_t* lb = seg_last + ((size_t)s * nseg_max + k) * 256;
    for (uint32_t c = lane; c < 256; c += 64) {
        const int32_t v = c < nin ? lb[c] : INT32_MIN;
        key[wave][c] = (c < nin && v < 0) ? -1 - (int32_t)c : v;
        inw[wave][c] = 0;
    }
    wsync();
    for (uint32_t c = lane; c < nin; c += 64) {
        const int32_t kc = key[wave][c];
        uint32_t r = 0;
        for (uint32_t d = 0; d < nin; ++d) r += key[wave][d] > kc ? 1u : 0u;
        Pt[wave][c] = (uint8_t)r;
        Lt[wave][r] = (uint8_t)c;
    }
    wsync();
    const uint8_t* llbuf = (const uint8_t*)B.mtfv + o;
    uint8_t* mraw = B.uflag + o;
    const uint32_t je = min(n, js + kSeg);
    const uint64_t lt = (1ull << lane) - 1ull, gt = ~lt & ~(1ull << lane);
    // the next window's symbol is loaded a window ahead, unconditionally (a
    // clamped index): a load under a branch made the compiler wait for every
    // outstanding load at the next use
    uint32_t cn = llbuf[min(js + lane, je - 1)];
    for (uint32_t j0 = js; j0 < je; j0 += 64) {
        const uint32_t j = j0 + lane;
        const bool valid = j < je;
        const uint32_t c = valid ? cn : 0u;
        cn = llbuf[min(j + 64, je - 1)];
        // match mask of c in this window
#if LFM_MTF_BALLOT
        // eight ballots, one per bit of c: the lanes whose byte equals this
        // lane's (VALU and scalar masks only; the LDS atomicOr per lane
        // serialised on the long runs of one byte in the BWT output)
        uint64_t M = ballot64(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const int32_t e = (int32_t)(c << (31 - b)) >> 31;  // 0 / -1
            M &= ~(ballot64(e != 0) ^ (uint64_t)(int64_t)e);
        }
        M = valid ? M : 0ull;
#else
        if (valid) mt[wave][c] = 0;
        wsync();
        if (valid) atomicOr((unsigned long long*)&mt[wave][c], 1ull << lane);
        wsync();
        const uint64_t M = valid ? mt[wave][c] : 0ull;
#endif
        const uint64_t before = M & lt;
        const bool has_prev = before != 0ull;
        const uint32_t p_in = has_prev ? 63u - (uint32_t)__clzll(before) : 0u;
        const uint32_t P0 = Pt[wave][c];
        // U = OR over lanes k < lane of bit(prev_k)  (exclusive prefix OR)
        const uint64_t U = wave_or_scan_excl(has_prev ? (1ull << p_in) : 0ull);
        uint32_t m;
        if (has_prev) {
            m = (uint32_t)__popcll((lt & ~U) >> (p_in + 1));
        } else {
            m = P0;
        }
        // first occurrences: earlier first-occurrence symbols placed behind c.
        // Their ranks at the window start are distinct, so the count is the
        // number of bits above P0 in the exclusive prefix OR of the earlier
        // first-occurrence lanes' one-hot ranks (8 words, DPP scans); a
        // serial loop over them (~27 per window, a readlane each) was
        // scalar-unit bound
        // only the words from the lowest to the highest first-occurrence
        // rank carry bits that count (usually one or two of the eight)
        const bool isF = valid && !has_prev;
        const uint32_t wm = (uint32_t)__builtin_amdgcn_readlane(
            (int)(wave_or_scan_excl32(isF ? 1u << (P0 >> 5) : 0u) | (isF ? 1u << (P0 >> 5) : 0u)), 63);
        const uint32_t wlo = wm ? (uint32_t)__builtin_ctz(wm) : 8u, whi = wm ? 31u - (uint32_t)__clz(wm) : 0u;
        {
            const uint32_t pw = P0 >> 5, pb = P0 & 31u;
            uint32_t cnt = 0;
            for (uint32_t wd = wlo; wd <= whi; ++wd) {
                const uint32_t oh = (isF && pw == wd) ? (1u << pb) : 0u;
                const uint32_t pre = wave_or_scan_excl32(oh);
                const uint32_t above = wd > pw ? ~0u : (wd == pw ? (pb == 31 ? 0u : ~0u << (pb + 1)) : 0u);
                cnt += (uint32_t)__popc(pre & above);
            }
            if (isF) m += cnt;
        }
        if (valid) mraw[j] = (uint8_t)m;
        // list update: window symbols by last occurrence, then the rest.  The
        // window symbols' old places (their first occurrences' P0) are below
        // 32 * (whi + 1), and every entry past them keeps its place (nw
        // removed before it, nw inserted in front), so only the blocks of 64
        // places up to there move (place p = 64 q + lane)
        const bool is_last = valid && (M & gt) == 0ull;
        const uint64_t Lw = ballot64(is_last);
        const uint32_t nw = (uint32_t)__popcll(Lw);
        const uint32_t nblk = whi / 2u + 1u;  // wave-uniform
        if (isF) inw[wave][P0] = 1;  // flags by old place: the update reads them in order
        wsync();
        uint32_t sym[4], fl[4];
        uint64_t fb[4];
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            if (q < nblk) {
                const uint32_t p = 64u * q + lane;
                sym[q] = Lt[wave][p];
                fl[q] = p < nin ? inw[wave][p] : 1u;
                fb[q] = ballot64(fl[q] != 0);
            }
        }
        wsync();
        uint32_t fl_blocks = 0;  // flagged places in the blocks before q
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            if (q < nblk) {
                const uint32_t p = 64u * q + lane;
                if (!fl[q]) {
                    const uint32_t np = nw + p - (fl_blocks + (uint32_t)__popcll(fb[q] & lt));
                    Lt[wave][np] = (uint8_t)sym[q];
                    Pt[wave][sym[q]] = (uint8_t)np;
                }
                fl_blocks += (uint32_t)__popcll(fb[q]);
            }
        }
        if (is_last) {
            const uint32_t np = (uint32_t)__popcll(Lw & gt);
            Lt[wave][np] = (uint8_t)c;
            Pt[wave][c] = (uint8_t)np;
        }
        if (isF) inw[wave][P0] = 0;
        wsync();
    }
}

// zero-run digits of a run of z >= 1 zeros (compress.c: z-1, then RUNA/RUNB
// by bit, (z-2)/2 ... : bijective base 2, whose length is floor(log2(z + 1)))
__device__ __forceinline__ uint32_t run_digits(uint32_t z) { return 31u - (uint32_t)__clz(z + 1u); }

// A (stream, table) heap is "narrow" when every node weight of
// BZ2_hbMakeCodeLengths fits 17 bits: the table's frequencies sum to at most
// nMTF, and each zero frequency counts 1.  Narrow heaps (nearly every default
// 96x96x8 uint16 block: nMTF ~ 95-100k) take u32 entries in huff_lengths_heap,
// the others u64 entries (rle2 lists those streams).
constexpr uint32_t kNarrowWeight = 1u << 17;
__device__ __forceinline__ bool heap_narrow(const Batch& B, uint32_t s, int alphaSize)
{
    return B.nmtf[s] + (uint32_t)alphaSize < kNarrowWeight;
}

constexpr int kRle2Threads = 256;  // (512 and 1 024 measured slower)
constexpr uint32_t kRle2Per = 64;                        // m values per thread and tile
constexpr uint32_t kRle2Tile = kRle2Threads * kRle2Per;  // 16384

// One workgroup per stream walks it in tiles of 16384 MTF values, 64 per
// thread.  A thread's zero values are a 64-bit mask; the zero run pending at
// each thread's first value comes from a scan (trailing zeros, all zero) over
// the tile on top of the run carried from the previous tiles.  Every nonzero
// value v ends the zero run before it: the run's RUNA / RUNB digits, then
// v + 1, go into an LDS copy of the tile's output (placed by a scan of the
// counts; the digits of a run of z zeros are the bits of z + 1 below its top
// bit, lowest first) and out with coalesced stores.  Frequencies: RUNA / RUNB
// and the four hottest symbols in registers, the others by LDS atomics.
__device__ __forceinline__ uint64_t zero_byte_mask64(const uint32_t (&q)[kRle2Per / 4])
{
    uint64_t Z = 0;
#pragma unroll
    for (uint32_t k = 0; k < kRle2Per / 4; ++k) {
        const uint32_t y = q[k];
        const uint32_t z = ~((((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y)) & 0x80808080u;  // bit 7: byte zero
        const uint32_t z4 = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
        Z |= (uint64_t)z4 << (4 * k);
    }
    return Z;
}

// tile_out index swizzle: a thread writes its outputs at its own offset, and
// the offsets of the 64 lanes lie one thread's output count apart -- often a
// multiple of 32 words, i.e. one LDS bank.  XOR-ing the word index's low 5
// bits with its 32-word row number spreads them over the banks; rows stay
// whole, so the coalesced read-out (consecutive indices) is a permutation
// inside each row, conflict-free as well.
#ifndef LFM_RLE2_SWZ
#define LFM_RLE2_SWZ 1
#endif
__device__ __forceinline__ uint32_t rle2_swz(uint32_t p)
{
    if constexpr (LFM_RLE2_SWZ) return p ^ (((p >> 6) & 31u) << 1);
    else return p;
}

__global__ __launch_bounds__(kRle2Threads) __attribute__((amdgpu_waves_per_eu(4))) void rle2(Batch B)
{
    constexpr uint32_t NW = kRle2Threads / 64;
    __shared__ uint32_t wz[NW], wa[NW], wc[NW];  // per-wave scan totals
    // freq[kMaxAlpha + t] and tile_out[kRle2Tile + 64 + t]: thread t's junk slots
    __shared__ uint32_t freq[kMaxAlpha + kRle2Threads];
    __shared__ uint16_t tile_out[kRle2Tile + 64 + kRle2Threads];
    __shared__ uint32_t s_carry, s_wr;
    const uint32_t s = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (B.flags[s] & kFlagHost) return;
    const uint32_t n = B.n[s];
    const size_t o = (size_t)s * B.cap;
    const uint8_t* m = B.uflag + o;
    uint16_t* out = B.mtfv + (size_t)s * (B.cap + 8);
    uint32_t nin = 0;
    for (int q = 0; q < 8; ++q) nin += __popc(B.inuse[s * 8 + q]);
    const uint32_t EOB = nin + 1;
    for (uint32_t v = t; v < kMaxAlpha; v += kRle2Threads) freq[v] = 0;
    if (t == 0) {
        s_carry = 0;
        s_wr = 0;
    }
    uint32_t nrunA = 0, nrunB = 0;
    uint64_t hot = 0;  // symbols 2 .. 5 (values 1 .. 4): 16-bit counters
    // zero-run scan element: (trailing zeros, all zeros); a then b
    auto zcomb = [](uint32_t atz, uint32_t aaz, uint32_t btz, uint32_t baz, uint32_t& rtz, uint32_t& raz) {
        rtz = baz ? atz + btz : btz;
        raz = aaz & baz;
    };
    // this thread's 64 values of a tile, in registers, loaded a tile ahead
    uint4 nq[kRle2Per / 16];
    auto load_vals = [&](uint32_t tb2) {
        const uint32_t a0 = min(n, tb2 + t * kRle2Per), l2 = min(n, a0 + kRle2Per) - a0;
#pragma unroll
        for (uint32_t i = 0; i < kRle2Per / 16; ++i)
            nq[i] = 16 * i < l2 ? *(const uint4*)(m + a0 + 16 * i) : make_uint4(0, 0, 0, 0);
    };
    load_vals(0);
    __syncthreads();
    for (uint32_t tb = 0; tb < n; tb += kRle2Tile) {
        const uint32_t c0 = min(n, tb + t * kRle2Per), c1 = min(n, c0 + kRle2Per), len = c1 - c0;
        const bool last_tile = tb + kRle2Tile >= n;
        uint32_t q[kRle2Per / 4];
#pragma unroll
        for (uint32_t i = 0; i < kRle2Per / 16; ++i) {
            q[4 * i] = nq[i].x; q[4 * i + 1] = nq[i].y; q[4 * i + 2] = nq[i].z; q[4 * i + 3] = nq[i].w;
        }
        load_vals(tb + kRle2Tile);
        const uint64_t valid = len >= 64 ? ~0ull : (1ull << len) - 1ull;
        const uint64_t Z = zero_byte_mask64(q) & valid, NZ = ~Z & valid;
        // chunk summary: trailing zeros, all-zero (empty chunks pass the carry through)
        const uint32_t az = NZ == 0ull ? 1u : 0u;
        const uint32_t tz = az ? len : (uint32_t)__clzll(NZ << (64u - len));
        // inclusive scan over the wave, then the waves before
        uint32_t itz = tz, iaz = az;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t otz = (uint32_t)__shfl_up((int)itz, d), oaz = (uint32_t)__shfl_up((int)iaz, d);
            if ((int)lane >= d) zcomb(otz, oaz, itz, iaz, itz, iaz);
        }
        if (lane == 63) {
            wz[wave] = itz;
            wa[wave] = iaz;
        }
        const uint32_t tile_carry = s_carry;
        __syncthreads();
        uint32_t ptz = tile_carry, paz = 1;  // everything before the wave, the tile carry first
        for (uint32_t w2 = 0; w2 < wave; ++w2) zcomb(ptz, paz, wz[w2], wa[w2], ptz, paz);
        uint32_t etz = (uint32_t)__shfl_up((int)itz, 1), eaz = (uint32_t)__shfl_up((int)iaz, 1);
        if (lane == 0) { etz = 0; eaz = 1; }
        uint32_t carry, cz;  // zeros pending at the chunk start
        zcomb(ptz, paz, etz, eaz, carry, cz);
        uint32_t tile_end_zeros = tile_carry, tez = 1;
        for (uint32_t w2 = 0; w2 < NW; ++w2) zcomb(tile_end_zeros, tez, wz[w2], wa[w2], tile_end_zeros, tez);
        const bool has_last = last_tile && len && c1 == n;
        // zero runs ending here: at a nonzero value after a zero (or after
        // the carried zeros), and the stream's final run
        const uint64_t R = NZ & ((Z << 1) | (carry ? 1ull : 0ull));
        const uint32_t zend = az ? carry + len : tz;  // zeros at the chunk end (the stream's final run when has_last)
        auto run_len = [&](uint32_t i) {  // zeros before the nonzero value i
            const uint64_t below = NZ & ((1ull << i) - 1ull);
            return below ? i - 1u - (63u - (uint32_t)__clzll(below)) : carry + i;
        };
        uint32_t ndig = 0;
        for (uint64_t r = R; r; r &= r - 1ull) ndig += run_digits(run_len((uint32_t)__builtin_ctzll(r)));
        const uint32_t dend = has_last && zend ? run_digits(zend) : 0u;
        const uint32_t w = (uint32_t)__popcll(NZ) + ndig + dend + (has_last ? 1u : 0u);
        // output offsets: scan of the counts
        uint32_t ic = w;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t oc = (uint32_t)__shfl_up((int)ic, d);
            if ((int)lane >= d) ic += oc;
        }
        if (lane == 63) wc[wave] = ic;
        __syncthreads();
        uint32_t wr = ic - w, tile_total = 0;
        for (uint32_t w2 = 0; w2 < NW; ++w2) {
            if (w2 < wave) wr += wc[w2];
            tile_total += wc[w2];
        }
        // the digits of a run of z zeros at p .. p + d - 1
        auto digits = [&](uint32_t p, uint32_t z) {
            const uint32_t d = run_digits(z), x = z + 1u;
            const uint32_t nb = (uint32_t)__popc(x & ((1u << d) - 1u));
            nrunB += nb;
            nrunA += d - nb;
            for (uint32_t k = 0; k < d; ++k) tile_out[rle2_swz(p + k)] = (uint16_t)((x >> k) & 1u);
        };
        // symbols v + 1: one write per value (zeros into a junk slot), the
        // position advanced past the digits of the run each one ends
        {
            uint32_t pos = wr, z = carry;
#pragma unroll
            for (uint32_t i = 0; i < kRle2Per; ++i) {
                const uint32_t v = (q[i >> 2] >> (8 * (i & 3))) & 0xFFu;
                const bool nz = (NZ >> i) & 1u;
                pos += nz && z ? run_digits(z) : 0u;
                tile_out[rle2_swz(nz ? pos : kRle2Tile + 64 + t)] = (uint16_t)(v + 1u);
                atomicAdd(&freq[nz && v > 4u ? v + 1u : kMaxAlpha + t], 1u);
                hot += nz && v <= 4u ? 1ull << (16u * (v - 1u)) : 0ull;
                pos += nz ? 1u : 0u;
                z = nz ? 0u : z + 1u;
            }
        }
        // the digits, each run before the nonzero value ending it
        {
            uint32_t dsum = 0;  // digits of the runs ending before i
            for (uint64_t r = R; r; r &= r - 1ull) {
                const uint32_t i = (uint32_t)__builtin_ctzll(r), z = run_len(i);
                digits(wr + (uint32_t)__popcll(NZ & ((1ull << i) - 1ull)) + dsum, z);
                dsum += run_digits(z);
            }
        }
        if (has_last) {
            if (zend) digits(wr + w - 1u - dend, zend);
            tile_out[rle2_swz(wr + w - 1u)] = (uint16_t)EOB;
            atomicAdd(&freq[EOB], 1u);
        }
        __syncthreads();
        const uint32_t base = s_wr;
        for (uint32_t i = t; i < tile_total; i += kRle2Threads) out[base + i] = tile_out[rle2_swz(i)];
        __syncthreads();
        if (t == 0) {
            s_wr = base + tile_total;
            s_carry = tile_end_zeros;
        }
        __syncthreads();
    }
    static_assert(kRunA == 0 && kRunB == 1, "RUNA / RUNB are symbols 0 and 1");
    // wave sums of the register counters, one atomic per wave and symbol
    uint32_t cnts[6] = {nrunA, nrunB, (uint32_t)(hot & 0xFFFFu), (uint32_t)((hot >> 16) & 0xFFFFu),
                        (uint32_t)((hot >> 32) & 0xFFFFu), (uint32_t)(hot >> 48)};
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        uint32_t c = cnts[r];
        for (int d = 32; d > 0; d >>= 1) c += (uint32_t)__shfl_xor((int)c, d);
        if (lane == 0 && c) atomicAdd(&freq[r], c);
    }
    __syncthreads();
    if (t == 0) {
        B.nmtf[s] = s_wr;
        if (!heap_narrow(B, s, (int)nin + 2)) B.wide[atomicAdd(B.wide_cnt, 1u)] = s;  // u64 Huffman heaps
    }
    for (uint32_t v = t; v < kMaxAlpha; v += kRle2Threads) B.mtf_freq[(size_t)s * kMaxAlpha + v] = freq[v];
}

// --------------------------------------------------------------- huffman --
constexpr int kHuffThreads = 256;

// sendMTFValues split across launches so the sequential part (the heap of
// BZ2_hbMakeCodeLengths) runs SIMT, one table per lane:
//   huff_init     nGroups and the initial partition (len 0 / 15)
//   huff_select   x4: selector per 50 symbols (first minimum cost, all tables
//                 summed at once in 10-bit fields), then symbol frequencies
//                 per selected table
//   huff_lengths  x4: BZ2_hbMakeCodeLengths (huffman.c, restated: nodes and
//                 heap from 1, entry 0 the sentinel, weights carry the depth
//                 in the low byte), one lane per (stream, table)
//   huff_final    selector MTF and the codes (BZ2_hbAssignCodes)
__device__ __forceinline__ uint32_t stream_nin(const Batch& B, uint32_t s)
{
    uint32_t nin = 0;
    for (int q = 0; q < 8; ++q) nin += __popc(B.inuse[s * 8 + q]);
    return nin;
}

// compress.c's initial partition: the frequencies go to LDS (the greedy walk
// is sequential and would otherwise wait on a global load per symbol), one
// lane walks them, all lanes write the lengths
__global__ __launch_bounds__(64) void huff_init(Batch B)
{
    __shared__ int mf[kMaxAlpha];
    __shared__ int pgs[kMaxGroups], pge[kMaxGroups];
    const uint32_t s = blockIdx.x, t = threadIdx.x;
    if (B.flags[s] & kFlagHost) return;
    const uint32_t nMTF = B.nmtf[s];
    const int alphaSize = (int)stream_nin(B, s) + 2;
    const uint32_t* mfreq = B.mtf_freq + (size_t)s * kMaxAlpha;
    uint8_t* len = B.len + (size_t)s * kMaxGroups * kMaxAlpha;
    const int nGroups = nMTF < 200 ? 2 : nMTF < 600 ? 3 : nMTF < 1200 ? 4 : nMTF < 2400 ? 5 : 6;
    for (int v = t; v < kMaxAlpha; v += 64) mf[v] = v < alphaSize ? (int)mfreq[v] : 0;
    __syncthreads();
    if (t == 0) {
        int nPart = nGroups, remF = (int)nMTF, gs = 0;
        while (nPart > 0) {
            const int tFreq = remF / nPart;
            int ge = gs - 1, aFreq = 0;
            while (aFreq < tFreq && ge < alphaSize - 1) {
                ++ge;
                aFreq += mf[ge];
            }
            if (ge > gs && nPart != nGroups && nPart != 1 && ((nGroups - nPart) % 2 == 1)) {
                aFreq -= mf[ge];
                --ge;
            }
            pgs[nPart - 1] = gs;
            pge[nPart - 1] = ge;
            --nPart;
            gs = ge + 1;
            remF -= aFreq;
        }
        B.ngroups[s] = (uint32_t)nGroups;
        B.nsel[s] = (nMTF + kGSize - 1) / kGSize;
    }
    __syncthreads();
    for (int i = t; i < kMaxGroups * kMaxAlpha; i += 64) {
        const int q = i / kMaxAlpha, v = i - q * kMaxAlpha;
        len[i] = (q < nGroups && v < alphaSize && v >= pgs[q] && v <= pge[q]) ? 0 : 15;
    }
}

// huff_select with a group's 50 symbols loaded straight into registers (25
// dword loads from its 100 bytes; a row is 16-byte aligned and 100 is a
// multiple of 4): no LDS tile, so ~8 KiB of LDS per workgroup and more
// workgroups per CU to hide the loads.  The last, partial group pads with
// symbol kMaxAlpha, whose packed lengths are 0 and which is not counted.
// (A 25 KiB LDS tile of the symbols measured 3.4x slower: fewer workgroups per CU.)
__global__ __launch_bounds__(kHuffThreads) void huff_select_reg(Batch B)
{
    __shared__ uint32_t rfreq[kMaxGroups][kMaxAlpha];
    __shared__ uint64_t lpack[kMaxAlpha + 1];
    __shared__ uint32_t junk[kHuffThreads];
    const uint32_t s = blockIdx.x, t = threadIdx.x;
    if (B.flags[s] & kFlagHost) return;
    const uint32_t nMTF = B.nmtf[s], nSel = B.nsel[s];
    const int nGroups = (int)B.ngroups[s];
    const int alphaSize = (int)stream_nin(B, s) + 2;
    const uint8_t* len = B.len + (size_t)s * kMaxGroups * kMaxAlpha;
    const uint16_t* mtfv = B.mtfv + (size_t)s * (B.cap + 8);
    uint8_t* sel = B.sel + (size_t)s * B.sel_cap;
    for (int i = t; i < kMaxGroups * kMaxAlpha; i += kHuffThreads) rfreq[i / kMaxAlpha][i % kMaxAlpha] = 0;
    for (int v = t; v <= kMaxAlpha; v += kHuffThreads) {
        uint64_t lp = 0;
        if (v < alphaSize)
            for (int q = 0; q < nGroups; ++q) lp |= (uint64_t)len[q * kMaxAlpha + v] << (10 * q);
        lpack[v] = lp;
    }
    __syncthreads();
    uint64_t lp_hot[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) lp_hot[f] = lpack[f];
    for (uint32_t g = t; g < nSel; g += kHuffThreads) {
        const uint32_t gs = g * kGSize, cnt = min(nMTF - gs, (uint32_t)kGSize);
        uint32_t w[kGSize / 2];
        if (cnt == (uint32_t)kGSize) {
            const uint32_t* p = (const uint32_t*)(mtfv + gs);
#pragma unroll
            for (int q = 0; q < kGSize / 2; ++q) w[q] = p[q];
        } else {
#pragma unroll
            for (int q = 0; q < kGSize / 2; ++q) {
                const uint32_t lo = 2u * q < cnt ? mtfv[gs + 2 * q] : (uint32_t)kMaxAlpha;
                const uint32_t hi = 2u * q + 1 < cnt ? mtfv[gs + 2 * q + 1] : (uint32_t)kMaxAlpha;
                w[q] = lo | (hi << 16);
            }
        }
        // a group's cost under every table at once (10-bit fields, as
        // huff_select); symbols 0 .. 3 (most of them) are counted in 8-bit
        // fields and priced from registers, their lanes read the pad entry
        // (one broadcast address instead of bank conflicts on 4 hot words)
        uint32_t hot = 0;
        uint64_t acc = 0;
#pragma unroll
        for (int q = 0; q < kGSize / 2; ++q) {
            const uint32_t lo = w[q] & 0xFFFFu, hi = w[q] >> 16;
            hot += lo < 4u ? 1u << (8u * lo) : 0u;
            hot += hi < 4u ? 1u << (8u * hi) : 0u;
            acc += lpack[lo < 4u ? (uint32_t)kMaxAlpha : lo] + lpack[hi < 4u ? (uint32_t)kMaxAlpha : hi];
        }
#pragma unroll
        for (uint32_t f = 0; f < 4; ++f) acc += (uint64_t)((hot >> (8u * f)) & 0xFFu) * lp_hot[f];
        int bt = -1;
        uint32_t bc = 999999999u;
        for (int q = 0; q < nGroups; ++q) {
            const uint32_t cq = (uint32_t)(acc >> (10 * q)) & 1023u;
            if (cq < bc) { bc = cq; bt = q; }
        }
        sel[g] = (uint8_t)bt;
        // symbols 0 .. 3 (RUNA, RUNB and the two smallest values: most of
        // them) go to rfreq from their 8-bit fields, the others by LDS atomics
        // (the hot bins' atomics serialised on bank conflicts); a lane's other
        // symbols land in its own junk word
#pragma unroll
        for (int q = 0; q < kGSize / 2; ++q) {
            const uint32_t lo = w[q] & 0xFFFFu, hi = w[q] >> 16;
            atomicAdd(lo >= 4u && lo != (uint32_t)kMaxAlpha ? &rfreq[bt][lo] : &junk[t], 1u);
            atomicAdd(hi >= 4u && hi != (uint32_t)kMaxAlpha ? &rfreq[bt][hi] : &junk[t], 1u);
        }
#pragma unroll
        for (uint32_t f = 0; f < 4; ++f)
            if ((hot >> (8u * f)) & 0xFFu) atomicAdd(&rfreq[bt][f], (hot >> (8u * f)) & 0xFFu);
    }
    __syncthreads();
    uint32_t* rf = B.rfreq + (size_t)s * kMaxGroups * kMaxAlpha;
    for (int i = t; i < kMaxGroups * kMaxAlpha; i += kHuffThreads) rf[i] = rfreq[i / kMaxAlpha][i % kMaxAlpha];
}

// BZ2_hbMakeCodeLengths, kL (stream, table) heaps per wave, one per lane,
// with wave-uniform heap walks.  A heap entry is one word: the weight as
// (freq << 5 | height) above bit 10, the node in bits 0..9; the order of
// (freq << 5 | height) is huffman.c's order of (freq << 8 | depth) because
// height <= 17 -- a node of height 18 already means a code longer than
// maxLen 17, so the lane keeps going on garbage and then redoes the tree with
// halved weights, the retry huffman.c takes after building it.  Narrow heaps
// (heap_narrow: weights < 2^17) use u32 entries (~1 KB of LDS per heap, so
// many heaps are resident), the others u64 entries in a second launch over the
// list the first one built (kList).
//   * Entries sit in per-lane quads (entries 4q .. 4q + 3 contiguous): a
//     node's children are half a quad, its grandchildren a whole quad, so a
//     sift level reads the NEXT level's candidates (one ds_read_b128) while it
//     decides the current one -- one LDS latency per level, not latency plus
//     the compare chain.
//   * The sift / upheap loops are uniform: every lane runs the level, selects
//     instead of branches, one ballot per level (divergent per-lane exits cost
//     ~20 scalar exec-mask instructions per level, and a CU's one scalar unit
//     serves all its waves).
//   * Parents go to global memory (the stream's code table, unused until
//     huff_final) and come back for the depth pass, whose depths overlay the
//     lane's own entries.
template <typename Ent>
struct HeapQuad {
    Ent e[4];
};

// entries 0 .. 259, then one quad of sentinels (the grandchildren of every
// node past 64 read as sentinels)
constexpr int kHeapQuads = (kMaxAlpha + 2 + 3) / 4 + 1;

// kL heaps with Ent entries in the LDS area hb (kHeapQuads * kL quads);
// this lane's heap is (stream s, table tb)
template <typename Ent, int kL>
__device__ __forceinline__ void heap_code_lengths(const Batch& B, char* hb, uint32_t lane, uint32_t s, uint32_t tb)
{
    constexpr int kQuads = kHeapQuads;
    constexpr uint32_t QB = sizeof(HeapQuad<Ent>);   // bytes per lane per quad
    constexpr uint32_t QS = QB * kL;                 // bytes per quad row
    constexpr uint32_t ES = sizeof(Ent);
    const uint32_t lb = lane * QB;
    auto ent = [&](uint32_t e) -> Ent& { return *(Ent*)(hb + (e >> 2) * QS + lb + (e & 3) * ES); };
    {
        const int A = (int)stream_nin(B, s) + 2;
        const uint32_t* freq = B.rfreq + ((size_t)s * kMaxGroups + tb) * kMaxAlpha;
        uint8_t* len = B.len + ((size_t)s * kMaxGroups + tb) * kMaxAlpha;
        uint16_t* parent = (uint16_t*)(B.code + ((size_t)s * kMaxGroups + tb) * kMaxAlpha);  // nodes 1 .. 2A - 2
        // depth of node k (<= 515): u16 number k % (ES / 2) of the lane's entry k / (ES / 2)
        auto dep = [&](uint32_t k) -> uint16_t& {
            return *(uint16_t*)((char*)&ent(k / (ES / 2)) + 2 * (k % (ES / 2)));
        };
        // rows are 8-byte aligned (258 words): pairs of words, a few loads ahead
        auto ld2 = [](const void* p, int i) { return *(const uint2*)((const uint32_t*)p + (i > 0 ? i : 0)); };
        // a < b on weights (bits 10 and up) <=> a < (b with its node bits
        // cleared) <=> (a with its node bits set) < b
        constexpr Ent kW = ~(Ent)1023;
        // every position past the heap holds kSent (greater than any entry:
        // heights stop at 30), so the sift needs no bounds: a pop writes kSent
        // where the last entry was, a push overwrites the first one
        constexpr Ent kSent = ~(Ent)0;
        // downheap from the root with key k; returns the new root.  Per level:
        // the grandchildren quad is read first (it holds the children of
        // either next node), then the level is decided from the children in
        // registers; ea = address of the entry the key may land in, ca = the
        // children pair of zz (ea of the next level is ca + 4 * right)
        auto sift = [&](Ent k) {
            const Ent kk = k | (Ent)1023;
            uint32_t zz = 1, ea = lb + ES, ca = lb + 2u * ES;
            Ent cx = ent(2), cy = ent(3), root = k;
            bool go = true, first = true;
            while (true) {
                const uint32_t ga = min(zz, (uint32_t)kQuads - 1u) * QS + lb;
                const HeapQuad<Ent> g = *(const HeapQuad<Ent>*)(hb + ga);
                __builtin_amdgcn_sched_barrier(0);  // the read goes out before the level's compares
                const uint32_t r = (cy | (Ent)1023) < cx ? 1u : 0u;
                const Ent ky = r ? cy : cx;
                go = go && !(kk < ky);
                *(Ent*)(hb + ea) = ky;  // a stopped lane's stray write is overwritten below
                if (first) root = go ? ky : k;
                first = false;
                const uint32_t zn = (zz << 1) | r, en = ca + r * ES;
                ca = ga + r * (2u * ES);
                ea = go ? en : ea;
                zz = go ? zn : zz;
                __builtin_amdgcn_sched_barrier(0);  // the quad is waited for last
                cx = r ? g.e[2] : g.e[0];
                cy = r ? g.e[3] : g.e[1];
                if (!__builtin_amdgcn_ballot_w64(go)) break;
            }
            *(Ent*)(hb + ea) = k;
            return root;
        };
        auto upheap = [&](uint32_t z, Ent k) {  // returns the final position
            bool go = true;
            while (true) {
                const Ent up = ent(z >> 1);
                go = go && k < (up & kW);  // the sentinel 0 stops it
                ent(z) = go ? up : k;
                z = go ? z >> 1 : z;
                if (!__any(go)) break;
            }
            return z;
        };
        // upheap for the initial inserts (z = i is the same in every lane
        // still inserting): the positions z >> j on the way to the root are
        // read at once, then every one is rewritten without a branch -- the
        // parent's entry where the key climbs past it (lt), the key where it
        // stops, the old entry above (the ancestors' weights only grow
        // downwards, so lt holds for a prefix of the levels; position 0, the
        // sentinel 0, ends it)
        auto upheap_init = [&](uint32_t z) {
            constexpr int D = 9;  // z < 512: z >> 9 is position 0
            Ent v[D + 1];
#pragma unroll
            for (int j = 0; j <= D; ++j) v[j] = ent(z >> j);  // v[0]: the key, the leaf at z
            __builtin_amdgcn_sched_barrier(0);  // every read goes out before the first wait
            const Ent k = v[0], kk = k | (Ent)1023;
            bool below = true;  // the key climbed past the level below
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const bool lt = kk < v[j + 1];
                ent(z >> j) = lt ? v[j + 1] : (below || j == 0 ? k : v[j]);
                below = lt;
            }
        };
        int retries = 0, nNodes = A;
        while (true) {
            // leaves at heap positions 1 .. A first (an insertion's upheap only
            // touches positions below it), then inserted in order; sentinels
            // past them
            ent(0) = 0;
            for (int q = (A + 1) >> 2; q < kQuads; ++q) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (4 * q + j > A) ent((uint32_t)(4 * q + j)) = kSent;
            }
            // 32 frequencies per batch of 16 loads (one memory latency per
            // batch, not per load: the compiler drains vmcnt at loop edges)
            for (int i0 = 1; i0 <= A; i0 += 32) {
                uint2 f[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) f[q] = ld2(freq, min(i0 - 1 + 2 * q, kMaxAlpha - 2));
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int i = i0 + 2 * q;
                    uint32_t w0 = f[q].x ? f[q].x : 1u, w1 = f[q].y ? f[q].y : 1u;
                    for (int r = 0; r < retries; ++r) {
                        w0 = 1u + w0 / 2u;
                        w1 = 1u + w1 / 2u;
                    }
                    if (i <= A) ent(i) = ((Ent)w0 << 15) | (Ent)i;
                    if (i + 1 <= A) ent(i + 1) = ((Ent)w1 << 15) | (Ent)(i + 1);
                }
            }
            for (int i = 1; i <= A; ++i) upheap_init((uint32_t)i);
            int nHeap = A;
            nNodes = A;
            uint32_t tooLong = 0;
            Ent top = ent(1);
            while (nHeap > 1) {
                const Ent k1 = top;
                const Ent l1 = ent(nHeap);
                ent(nHeap) = kSent;
                --nHeap;
                const Ent k2 = sift(l1);
                const Ent l2 = ent(nHeap);
                ent(nHeap) = kSent;
                --nHeap;
                const Ent r2 = sift(l2);
                ++nNodes;
                parent[(uint32_t)k1 & 1023u] = (uint16_t)nNodes;
                parent[(uint32_t)k2 & 1023u] = (uint16_t)nNodes;
                const uint32_t h1 = (uint32_t)(k1 >> 10) & 31u, h2 = (uint32_t)(k2 >> 10) & 31u;
                const uint32_t h = min(30u, 1u + max(h1, h2));
                tooLong |= h > 17u ? 1u : 0u;
                const Ent kn = ((((k1 >> 15) + (k2 >> 15)) << 5 | (Ent)h) << 10) | (Ent)nNodes;
                ++nHeap;
                top = upheap((uint32_t)nHeap, kn) == 1u ? kn : r2;
            }
            if (!tooLong) break;
            ++retries;
        }
        if (retries) atomicAdd(B.wide_cnt + 1, (uint32_t)retries);  // statistics (LFM_BZ2_STATS)
        // depths top-down (a parent is created after its children)
        dep(nNodes) = 0;
        // 64 parents per batch of 16 loads, highest nodes first
        for (int kc = (nNodes - 1) & ~63; kc >= 0; kc -= 64) {
            uint2 pw[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) pw[q] = ld2(parent, min(kc / 2 + 2 * q, (2 * kMaxAlpha) / 2 - 2));
            // four nodes b .. b + 3 per LDS round trip: their parents' depths
            // are read together, a parent inside the four (the root included)
            // is taken from registers instead
#pragma unroll
            for (int q = 15; q >= 0; --q) {
                const int b = kc + 4 * q;
                const uint32_t p4[4] = {pw[q].x & 0xFFFFu, pw[q].x >> 16, pw[q].y & 0xFFFFu, pw[q].y >> 16};
                uint32_t d[4], dn[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) d[r] = dep(min(p4[r], 2u * kMaxAlpha));
#pragma unroll
                for (int r = 3; r >= 0; --r) {
                    const int k = b + r;
                    uint32_t x = d[r];
#pragma unroll
                    for (int u = r + 1; u < 4; ++u) x = p4[r] == (uint32_t)(b + u) ? dn[u] : x;
                    dn[r] = k == nNodes ? 0u : x + 1u;
                    if (k >= 1 && k < nNodes) dep(k) = (uint16_t)dn[r];
                }
            }
        }
        for (int i = 1; i <= A; ++i) len[i - 1] = (uint8_t)dep(i);
    }
}

// Workgroups [0, nwg_wide): kL / 2 heaps of the wide streams (B.wide,
// listed by rle2 and counted by the host) with u64 entries, first so their
// chains start first; the rest: kL (stream, table) heaps each with u32
// entries (lanes of wide streams exit).  One launch, so a wide heap's chain
// runs beside the narrow ones.
template <int kL>
__global__ __launch_bounds__(64) void huff_lengths_heap(Batch B, uint32_t nwg_wide, uint32_t nwide_streams)
{
    __shared__ HeapQuad<uint32_t> hq[kHeapQuads * kL];
    char* hb = (char*)hq;
    const uint32_t lane = threadIdx.x;
    if (blockIdx.x >= nwg_wide) {
        const uint32_t task = (blockIdx.x - nwg_wide) * kL + lane;
        const uint32_t s = task / kMaxGroups, tb = task % kMaxGroups;
        if (lane >= (uint32_t)kL || s >= B.nstreams || (B.flags[s] & kFlagHost) || tb >= B.ngroups[s]) return;
        if (!heap_narrow(B, s, (int)stream_nin(B, s) + 2)) return;
        heap_code_lengths<uint32_t, kL>(B, hb, lane, s, tb);
    } else {
        constexpr int kW = kL / 2;
        const uint32_t i = blockIdx.x * kW + lane;
        if (lane >= (uint32_t)kW || i >= nwide_streams * kMaxGroups) return;
        const uint32_t s = B.wide[i / kMaxGroups], tb = i % kMaxGroups;
        if ((B.flags[s] & kFlagHost) || tb >= B.ngroups[s]) return;
        heap_code_lengths<uint64_t, kW>(B, hb, lane, s, tb);
    }
}

// One wave per stream.  Selector MTF (compress.c, 6 entries): the list is a
// register of 4-bit entries, a step finds the entry by a zero-nibble test and
// rotates the nibbles in front of it; 64 selectors are loaded at a time and
// walked with readlane.  Codes (BZ2_hbAssignCodes) per table in parallel:
// code = (codes of all shorter lengths, doubled per length) + rank of the
// symbol among the same-length symbols before it (ballots per length).
__global__ __launch_bounds__(64) void huff_final(Batch B)
{
    const uint32_t s = blockIdx.x, lane = threadIdx.x;
    if (B.flags[s] & kFlagHost) return;
    const uint32_t nGroups = B.ngroups[s];
    const uint32_t nSel = B.nsel[s];
    const uint32_t alphaSize = stream_nin(B, s) + 2;
    const uint8_t* len = B.len + (size_t)s * kMaxGroups * kMaxAlpha;
    {
        const uint8_t* sel = B.sel + (size_t)s * B.sel_cap;
        uint8_t* sm = B.sel_mtf + (size_t)s * B.sel_cap;
        uint32_t pos = 0x543210u;  // entry i in nibble i
        for (uint32_t i0 = 0; i0 < nSel; i0 += 64) {
            const uint32_t cnt = min(64u, nSel - i0);
            const uint32_t v = lane < cnt ? sel[i0 + lane] : 0u;
            uint32_t out = 0;
            for (uint32_t g = 0; g < cnt; ++g) {
                const uint32_t ll = __builtin_amdgcn_readlane(v, g);
                const uint32_t x = pos ^ (ll * 0x111111u);
                const uint32_t z = (x - 0x111111u) & ~x & 0x888888u;  // lowest set: the first zero nibble
                const uint32_t j = (uint32_t)__builtin_ctz(z) >> 2;
                const uint32_t m = (1u << (4 * (j + 1))) - 1u;
                pos = (pos & ~m) | (((pos << 4) | ll) & m);
                out = lane == g ? j : out;
            }
            if (lane < cnt) sm[i0 + lane] = (uint8_t)out;
        }
    }
    const uint64_t lt = (1ull << lane) - 1ull;
    for (uint32_t q = 0; q < nGroups; ++q) {
        const uint8_t* lq = len + q * kMaxAlpha;
        uint32_t* code = B.code + ((size_t)s * kMaxGroups + q) * kMaxAlpha;
        uint32_t L[5], c[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint32_t i = 64 * k + lane;
            L[k] = i < alphaSize ? lq[i] : 0u;
            c[k] = 0;
        }
        uint32_t vec = 0;
        for (uint32_t nl = 1; nl <= 20; ++nl) {
            uint32_t before = 0;
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const uint64_t b = __ballot(L[k] == nl);
                if (L[k] == nl) c[k] = vec + before + (uint32_t)__popcll(b & lt);
                before += (uint32_t)__popcll(b);
            }
            // BZ2_hbAssignCodes: vec <<= 1 after every length from minLen on
            vec = (vec + before) << 1;
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint32_t i = 64 * k + lane;
            if (i < alphaSize) code[i] = c[k];
        }
    }
}

// ------------------------------------------------------------------ emit --
constexpr int kEmitThreads = 256;

// MSB-first bit writer into 32-bit words (bit p is bit 31 - p%32 of word p/32)
__device__ __forceinline__ void put_bits_atomic(uint32_t* words, uint64_t pos, uint32_t nbits, uint32_t v)
{
    if (!nbits) return;
    const uint32_t w = (uint32_t)(pos >> 5), o = (uint32_t)(pos & 31);
    const uint64_t sh = ((uint64_t)v << (64 - nbits)) >> o;  // bits aligned at the top of a 64-bit window
    const uint32_t hi = (uint32_t)(sh >> 32), lo = (uint32_t)sh;
    if (hi) atomicOr(&words[w], hi);
    if (lo) atomicOr(&words[w + 1], lo);
}

constexpr uint32_t kSelLds = 8192;  // selectors cached in LDS (level <= 4 always fits)

// header bits are assembled in LDS (one writer, no atomics; a global atomic
// per header field serialised the lane on memory latency), then copied out
constexpr uint32_t kHdrWords = 4096;  // 128 kbit: every level-1..9 header but extreme ones

__device__ __forceinline__ void put_bits_hdr(uint32_t* hdr, uint32_t* words, uint64_t pos, uint32_t nbits, uint32_t v)
{
    if (!nbits) return;
    const uint32_t w = (uint32_t)(pos >> 5), o = (uint32_t)(pos & 31);
    const uint64_t sh = ((uint64_t)v << (64 - nbits)) >> o;
    const uint32_t hi = (uint32_t)(sh >> 32), lo = (uint32_t)sh;
    if (w + 1 < kHdrWords) {
        hdr[w] |= hi;
        hdr[w + 1] |= lo;
    } else {  // overflow past the LDS buffer: straight to memory
        if (hi) atomicOr(&words[w], hi);
        if (lo) atomicOr(&words[w + 1], lo);
    }
}

// header items written by many threads: neighbours share words (atomicOr)
__device__ __forceinline__ void put_bits_hdr_atomic(uint32_t* hdr, uint32_t* words, uint64_t pos, uint32_t nbits,
                                                    uint32_t v)
{
    if (!nbits) return;
    const uint32_t w = (uint32_t)(pos >> 5), o = (uint32_t)(pos & 31);
    const uint64_t sh = ((uint64_t)v << (64 - nbits)) >> o;
    const uint32_t hi = (uint32_t)(sh >> 32), lo = (uint32_t)sh;
    if (w + 1 < kHdrWords) {
        if (hi) atomicOr(&hdr[w], hi);
        if (lo) atomicOr(&hdr[w + 1], lo);
    } else {
        if (hi) atomicOr(&words[w], hi);
        if (lo) atomicOr(&words[w + 1], lo);
    }
}

// up to 64 bits, MSB first
__device__ __forceinline__ void put_bits64_hdr_atomic(uint32_t* hdr, uint32_t* words, uint64_t pos, uint32_t nbits,
                                                      uint64_t v)
{
    if (nbits > 32) {
        put_bits_hdr_atomic(hdr, words, pos, nbits - 32, (uint32_t)(v >> 32));
        put_bits_hdr_atomic(hdr, words, pos + nbits - 32, 32, (uint32_t)v);
    } else {
        put_bits_hdr_atomic(hdr, words, pos, nbits, (uint32_t)v);
    }
}

// exclusive scan over the workgroup (wave shuffles, then the waves); *total = sum
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t* total)
{
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(inc, d);
        if ((int)lane >= d) inc += o;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < NT / 64; ++w) {
        const uint32_t x = wsum[w];
        pre += w < wave ? x : 0u;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return pre + inc - v;
}

// The header: the fixed fields and the mapping table by one lane, then the
// selectors (unary MTF values) and the delta-coded code lengths as items
// written by all threads at prefix-summed bit offsets.
constexpr uint32_t kEmitC = 16;  // symbols per thread and round
constexpr uint32_t kEmitBufWords = (kEmitThreads * kEmitC * 17 + 31) / 32 + 2;  // code lengths <= 17 bits

__global__ __launch_bounds__(kEmitThreads) void emit_stream(Batch B)
{
    __shared__ uint32_t wsum[kEmitThreads / 64];
    __shared__ uint32_t obuf[kEmitBufWords];
    __shared__ uint64_t s_hdr_bits;
    __shared__ uint32_t hdr[kHdrWords];
    __shared__ uint32_t lc[kMaxGroups * kMaxAlpha];  // code | len << 24 per (table, symbol)
    __shared__ uint8_t sel_l[kSelLds];
    const uint32_t s = blockIdx.x, t = threadIdx.x;
    if (B.flags[s] & kFlagHost) {
        if (t == 0) B.out_bytes[s] = 0;
        return;
    }
    uint32_t* words = B.words + (size_t)s * (B.out_cap / 4);
    const uint32_t nMTF = B.nmtf[s], nSel = B.nsel[s], nGroups = B.ngroups[s];
    const uint8_t* len = B.len + (size_t)s * kMaxGroups * kMaxAlpha;
    const uint32_t* code = B.code + (size_t)s * kMaxGroups * kMaxAlpha;
    const uint8_t* sel = B.sel + (size_t)s * B.sel_cap;
    const uint16_t* mtfv = B.mtfv + (size_t)s * (B.cap + 8);
    uint32_t inu[8];
    uint32_t nin = 0;
    for (int q = 0; q < 8; ++q) {
        inu[q] = B.inuse[s * 8 + q];
        nin += __popc(inu[q]);
    }
    const uint32_t alphaSize = nin + 2;
    for (uint32_t w = t; w < kHdrWords; w += kEmitThreads) hdr[w] = 0;
    {
        // the word buffer is not cleared: a header that could spill past the
        // LDS copy (OR-ed straight into memory) gets its spill words zeroed here
        const uint64_t bound = 32 + 48 + 32 + 1 + 24 + 16 + 256 + 3 + 15 + (uint64_t)nSel * (kMaxGroups + 1) +
                               (uint64_t)nGroups * (5 + 33ull * alphaSize);
        if (bound >= (uint64_t)(kHdrWords - 1) * 32)
            for (uint64_t w = kHdrWords - 1 + t; w < (bound >> 5) + 2; w += kEmitThreads) words[w] = 0;
    }
    for (uint32_t i = t; i < nGroups * kMaxAlpha; i += kEmitThreads) lc[i] = code[i] | ((uint32_t)len[i] << 24);
    for (uint32_t i = t; i < min(nSel, kSelLds); i += kEmitThreads) sel_l[i] = sel[i];
    __syncthreads();
    // header (thread 0, sequential, into LDS)
    if (t == 0) {
        uint64_t p = 0;
        auto put = [&](uint32_t nb, uint32_t v) {
            put_bits_hdr(hdr, words, p, nb, v);
            p += nb;
        };
        put(8, 'B'); put(8, 'Z'); put(8, 'h'); put(8, '0' + B.level);
        put(8, 0x31); put(8, 0x41); put(8, 0x59); put(8, 0x26); put(8, 0x53); put(8, 0x59);
        put(32, B.crc[s]);
        put(1, 0);
        put(24, B.orig_ptr[s]);
        uint32_t in16 = 0;
        for (int i = 0; i < 16; ++i) {
            const uint32_t bits16 = (inu[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu;
            if (bits16) in16 |= 1u << i;
        }
        for (int i = 0; i < 16; ++i) put(1, (in16 >> i) & 1u);
        for (int i = 0; i < 16; ++i)
            if ((in16 >> i) & 1u)
                for (int j = 0; j < 16; ++j) {
                    const uint32_t c = i * 16 + j;
                    put(1, (inu[c >> 5] >> (c & 31)) & 1u);
                }
        put(3, nGroups);
        put(15, nSel);
        s_hdr_bits = p;
    }
    __syncthreads();
    {
        uint64_t p = s_hdr_bits;
        uint32_t total = 0;
        // selectors: MTF value k as k ones and a zero (k < nGroups <= 6)
        {
            const uint8_t* sm = B.sel_mtf + (size_t)s * B.sel_cap;
            const uint32_t per = (nSel + kEmitThreads - 1) / kEmitThreads;
            const uint32_t a = min(nSel, t * per), b = min(nSel, a + per);
            uint32_t nb = 0;
            for (uint32_t i = a; i < b; ++i) nb += sm[i] + 1u;
            uint64_t q = p + block_excl_scan<kEmitThreads>(nb, wsum, &total);
            for (uint32_t i = a; i < b; ++i) {
                const uint32_t k = sm[i];
                put_bits_hdr_atomic(hdr, words, q, k + 1, ((1u << k) - 1u) << 1);
                q += k + 1;
            }
            p += total;
        }
        // code lengths: per table 5 bits of the first length, then per symbol
        // |d| x ("10" up / "11" down) and a zero, d = change from the previous
        {
            const uint32_t nl = nGroups * alphaSize;
            const uint32_t per = (nl + kEmitThreads - 1) / kEmitThreads;
            const uint32_t a = min(nl, t * per), b = min(nl, a + per);
            auto item = [&](uint32_t e, uint32_t& nbits, uint64_t& v) {
                const uint32_t q = e / alphaSize, i = e - q * alphaSize;
                const uint8_t* lq = len + q * kMaxAlpha;
                const int cur = lq[i], prev = i ? lq[i - 1] : cur;
                const int d = cur - prev;
                const uint32_t ad = (uint32_t)(d < 0 ? -d : d);
                v = 0;
                for (uint32_t r = 0; r < ad; ++r) v = (v << 2) | (d > 0 ? 2u : 3u);
                v <<= 1;
                nbits = 2 * ad + 1;
                if (i == 0) {
                    v |= (uint64_t)cur << nbits;
                    nbits += 5;
                }
            };
            uint32_t nb = 0;
            for (uint32_t e = a; e < b; ++e) {
                uint32_t k;
                uint64_t v;
                item(e, k, v);
                nb += k;
            }
            uint64_t q = p + block_excl_scan<kEmitThreads>(nb, wsum, &total);
            for (uint32_t e = a; e < b; ++e) {
                uint32_t k;
                uint64_t v;
                item(e, k, v);
                put_bits64_hdr_atomic(hdr, words, q, k, v);
                q += k;
            }
            p += total;
        }
        if (t == 0) s_hdr_bits = p;
    }
    __syncthreads();
    // data bits, in rounds of kEmitC symbols per thread (thread t codes
    // symbols r0 + t * kEmitC ..): a round's bits are contiguous across the
    // threads, so they are assembled in LDS and leave in coalesced word
    // stores; the round's partial last word carries into the next round.
    // (Each thread writing its own stretch of the stream straight to memory
    // made every store instruction touch 64 scattered lines.)
    const uint64_t hb = s_hdr_bits;
    {
        // header words; the word holding the data's first bit starts the carry
        const uint32_t full = (uint32_t)min<uint64_t>(hb >> 5, kHdrWords - 1);
        for (uint32_t w = t; w < full; w += kEmitThreads) words[w] = hdr[w];
        if (t == 0 && (hb >> 5) >= kHdrWords - 1) atomicOr(&words[kHdrWords - 1], hdr[kHdrWords - 1]);
        for (uint32_t i = t; i < kEmitBufWords; i += kEmitThreads) obuf[i] = 0;
    }
    __syncthreads();
    if (t == 0)  // a spilled header's last word is in memory (OR-ed there), else in LDS
        obuf[0] = (hb >> 5) < kHdrWords - 1 ? hdr[hb >> 5] : atomicOr(&words[hb >> 5], 0u);
    __syncthreads();
    auto sym_lc = [&](uint32_t i, uint32_t v) {
        const uint32_t g = i / kGSize;
        const uint32_t tb = g < kSelLds ? sel_l[g] : sel[g];
        return lc[tb * kMaxAlpha + v];
    };
    uint64_t bitpos = hb;
    for (uint32_t r0 = 0; r0 < nMTF; r0 += kEmitThreads * kEmitC) {
        const uint32_t i0 = min(nMTF, r0 + t * kEmitC), i1 = min(nMTF, i0 + kEmitC);
        uint32_t e[kEmitC];
        uint32_t nb = 0;
        {
            const uint4 v0 = i0 < i1 ? *(const uint4*)(mtfv + i0) : make_uint4(0, 0, 0, 0);
            const uint4 v1 = i0 + 8 < i1 ? *(const uint4*)(mtfv + i0 + 8) : make_uint4(0, 0, 0, 0);
            const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
            for (uint32_t k = 0; k < kEmitC; ++k) {
                e[k] = i0 + k < i1 ? sym_lc(i0 + k, (w[k >> 1] >> (16 * (k & 1))) & 0xFFFFu) : 0u;
                nb += e[k] >> 24;
            }
        }
        uint32_t rbits = 0;
        const uint32_t lb0 = (uint32_t)(bitpos & 31) + block_excl_scan<kEmitThreads>(nb, wsum, &rbits);
        if (nb) {
            uint64_t acc = 0;      // pending bits, left aligned at bit 63
            uint32_t wpos = lb0 >> 5, nacc = lb0 & 31;
            bool first_word = true;
#pragma unroll
            for (uint32_t k = 0; k < kEmitC; ++k) {
                const uint32_t l = e[k] >> 24;
                if (l) {
                    acc |= ((uint64_t)(e[k] & 0xFFFFFFu) << (64 - l)) >> nacc;
                    nacc += l;
                    if (nacc >= 32) {
                        const uint32_t wv = (uint32_t)(acc >> 32);
                        if (first_word) atomicOr(&obuf[wpos], wv);
                        else obuf[wpos] = wv;
                        first_word = false;
                        ++wpos;
                        acc <<= 32;
                        nacc -= 32;
                    }
                }
            }
            if (nacc > 0) atomicOr(&obuf[wpos], (uint32_t)(acc >> 32));
        }
        __syncthreads();
        const uint32_t nfull = (uint32_t)(((bitpos & 31) + rbits) >> 5);
        uint32_t* dst = words + (bitpos >> 5);
        // non-temporal: the stream words are read once more (compaction), and
        // dirty lines left in the caches slow the next encode's predictor
        for (uint32_t i = t; i < nfull; i += kEmitThreads) __builtin_nontemporal_store(obuf[i], &dst[i]);
        const uint32_t cv = obuf[nfull];
        __syncthreads();
        for (uint32_t i = 1 + t; i <= nfull; i += kEmitThreads) obuf[i] = 0;
        if (t == 0) obuf[0] = cv;
        __syncthreads();
        bitpos += rbits;
    }
    const uint64_t data_end = bitpos;
    if (t == 0) {  // the last partial word, and zeros under the end marker
        words[data_end >> 5] = (data_end & 31) ? obuf[0] : 0u;
        for (uint64_t w = (data_end >> 5) + 1; w <= ((data_end + 80) >> 5) + 1; ++w) words[w] = 0;
    }
    if (t == 0) {
        uint64_t p = data_end;
        auto put = [&](uint32_t nb2, uint32_t v) {
            put_bits_atomic(words, p, nb2, v);
            p += nb2;
        };
        put(8, 0x17); put(8, 0x72); put(8, 0x45); put(8, 0x38); put(8, 0x50); put(8, 0x90);
        put(32, B.crc[s]);  // combined CRC of a one-block stream: rotl(0, 1) ^ blockCRC
        B.out_bytes[s] = (uint32_t)((p + 7) >> 3);
    }
}

// copy the streams (MSB-first words) to their byte offsets in the payload:
// one workgroup per stream; the payload words wholly inside the stream are
// assembled from two source words (byte-swapped) and stored 4 bytes at a
// time, the at most 3 + 3 edge bytes one by one
__global__ __launch_bounds__(256) void compact_streams(Batch B, const uint64_t* __restrict__ offs,
                                                       uint8_t* __restrict__ payload)
{
    const uint32_t s = blockIdx.x, t = threadIdx.x;
    const uint32_t nbytes = B.out_bytes[s];
    if (!nbytes) return;
    const uint32_t* words = B.words + (size_t)s * (B.out_cap / 4);
    const uint64_t o = offs[s], e = o + nbytes;
    const uint64_t a0 = (o + 3) >> 2, a1 = e >> 2;
    auto byte_at = [&](uint64_t k) { return (uint8_t)(words[k >> 2] >> (24 - 8 * (k & 3))); };
    if (a0 >= a1) {  // no whole word: bytes only
        for (uint64_t k = t; k < nbytes; k += 256) payload[o + k] = byte_at(k);
        return;
    }
    if (t < 4 && o + t < 4 * a0) payload[o + t] = byte_at(t);
    if (t >= 4 && t < 8 && 4 * a1 + (t - 4) < e) payload[4 * a1 + (t - 4)] = byte_at(4 * a1 + (t - 4) - o);
    uint32_t* p32 = (uint32_t*)payload;
    const uint32_t r = (uint32_t)((4 * a0 - o) & 3), sh = 8 * r;
    const uint64_t j0 = (4 * a0 - o) >> 2;  // source word of the first whole payload word
    for (uint64_t a = a0 + t; a < a1; a += 256) {
        const uint64_t w = j0 + (a - a0);
        const uint32_t x = r ? (words[w] << sh) | (words[w + 1] >> (32 - sh)) : words[w];
        __builtin_nontemporal_store(__builtin_bswap32(x), &p32[a]);  // read next by the SDMA copy
    }
}

// exclusive offsets of the streams' byte counts: one workgroup, every thread
// sums a contiguous run, one block scan, then every thread writes its run
__global__ __launch_bounds__(1024) void scan_offsets(const uint32_t* __restrict__ nbytes, uint32_t n,
                                                     uint64_t* __restrict__ offs)
{
    __shared__ uint64_t wsum64[16];
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t per = (n + 1023) / 1024;
    const uint32_t a = min(n, t * per), b = min(n, a + per);
    uint64_t sum = 0;
    for (uint32_t i = a; i < b; ++i) sum += nbytes[i];
    uint64_t inc = sum;
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(inc, d);
        if ((int)lane >= d) inc += o;
    }
    if (lane == 63) wsum64[wave] = inc;
    __syncthreads();
    uint64_t acc = inc - sum;
    for (uint32_t w = 0; w < wave; ++w) acc += wsum64[w];
    for (uint32_t i = a; i < b; ++i) {
        offs[i] = acc;
        acc += nbytes[i];
    }
    if (b == n && a < b) offs[n] = acc;
    if (n == 0 && t == 0) offs[0] = 0;
}

} // namespace bz
} // namespace lfm

// =============================================================== host side
using namespace lfm::bz;

namespace {

uint32_t host_crc_table[256];
uint32_t host_crc4[4][256];
uint32_t host_crc_shift[kCrcLevels][32];
uint32_t host_crc_unshift[kCrcUnshift][32];
uint32_t host_crc_shb[kCrcLevels][4][256];  // host_crc_shift as byte tables
bool crc_ready = false;

void ensure_crc_table()
{
    if (crc_ready) return;
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i << 24;
        for (int k = 0; k < 8; ++k) c = (c & 0x80000000u) ? (c << 1) ^ 0x04c11db7u : (c << 1);
        host_crc_table[i] = c;
    }
    // slicing-by-4 tables: 4 zero feeds of a register holding byte v at byte k
    auto feed0 = [](uint32_t c) { return (c << 8) ^ host_crc_table[c >> 24]; };
    for (uint32_t k = 0; k < 4; ++k)
        for (uint32_t v = 0; v < 256; ++v) {
            uint32_t c = v << (8 * k);
            for (int r = 0; r < 4; ++r) c = feed0(c);
            host_crc4[k][v] = c;
        }
    // one zero feed and its inverse (the table's low byte identifies its index)
    uint32_t inv_low[256];
    bool seen[256] = {};
    for (uint32_t x = 0; x < 256; ++x) {
        const uint32_t lo = host_crc_table[x] & 0xFFu;
        if (seen[lo]) std::abort();  // never for CRC-32: the map is a bijection
        seen[lo] = true;
        inv_low[lo] = x;
    }
    auto unfeed0 = [&](uint32_t c) {
        const uint32_t x = inv_low[c & 0xFFu];
        return ((c ^ host_crc_table[x]) >> 8) | (x << 24);
    };
    auto mat_apply = [](const uint32_t* m, uint32_t v) {
        uint32_t r = 0;
        for (int k = 0; k < 32; ++k)
            if ((v >> k) & 1u) r ^= m[k];
        return r;
    };
    auto mat_square = [&](const uint32_t* m, uint32_t* out) {
        for (int k = 0; k < 32; ++k) out[k] = mat_apply(m, m[k]);
    };
    uint32_t z[32];
    for (int k = 0; k < 32; ++k) z[k] = feed0(1u << k);
    for (uint32_t b = 1; b < kRleChunk; b <<= 1) {  // Z^kRleChunk
        uint32_t t2[32];
        mat_square(z, t2);
        std::memcpy(z, t2, sizeof(z));
    }
    std::memcpy(host_crc_shift[0], z, sizeof(z));
    for (int l = 1; l < kCrcLevels; ++l) mat_square(host_crc_shift[l - 1], host_crc_shift[l]);
    for (int l = 0; l < kCrcLevels; ++l)
        for (uint32_t j = 0; j < 4; ++j)
            for (uint32_t v = 0; v < 256; ++v) host_crc_shb[l][j][v] = mat_apply(host_crc_shift[l], v << (8 * j));
    for (int k = 0; k < 32; ++k) host_crc_unshift[0][k] = unfeed0(1u << k);
    for (int l = 1; l < kCrcUnshift; ++l) mat_square(host_crc_unshift[l - 1], host_crc_unshift[l]);
    crc_ready = true;
}

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// stage boundary events of the calling thread (lfm_hip_bzip2_last_stage_ms)
struct StageEvents {
    int dev = -1;
    hipEvent_t ev[6] = {};
    float last_ms[5] = {};
    bool valid = false;
    ~StageEvents()
    {
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
    }
    bool ready(int d)
    {
        if (dev == d) return true;
        for (hipEvent_t& e : ev) {
            if (e) (void)hipEventDestroy(e);
            e = nullptr;
            if (hipEventCreate(&e) != hipSuccess) return false;
        }
        dev = d;
        return true;
    }
};
thread_local StageEvents t_stage;
thread_local void (*t_hook)(void*, int) = nullptr;
thread_local void* t_hook_ctx = nullptr;

// rocPRIM temporary storage for the largest use of each primitive in a batch
// of `count` streams (size queries only: no device work).  Carved out of the
// caller's workspace: a per-call stream-ordered allocation of these
// gigabyte-sized buffers stalled every stream of the device for ~0.3 s.
size_t prim_tmp_bytes(uint32_t count, uint32_t cap)
{
    const size_t N = (size_t)count * cap;
    uint64_t* k = nullptr;
    uint32_t* v = nullptr;
    uint8_t* f = nullptr;
    size_t tmp = 0, q = 0;
    const size_t max_seg = (size_t)count * (cap / kBigCap + 1);
    (void)rocprim::segmented_radix_sort_pairs(nullptr, q, k, k, v, v, (unsigned)N, (unsigned)max_seg, v, v, 0,
                                              64 - kBucketBits);
    tmp = std::max(tmp, q);
    (void)rocprim::radix_sort_pairs(nullptr, q, k, k, v, v, (unsigned)N, 0, 64);
    tmp = std::max(tmp, q);

    (void)rocprim::select(nullptr, q, rocprim::counting_iterator<uint32_t>(0), f, v, v, N);
    tmp = std::max(tmp, q);
    (void)rocprim::select(nullptr, q, v, f, v, v, N);
    tmp = std::max(tmp, q);
    (void)rocprim::inclusive_scan(nullptr, q, v, v, N, rocprim::maximum<uint32_t>());
    tmp = std::max(tmp, q);
    return tmp;
}

} // namespace

extern "C" size_t lfm_hip_bzip2_workspace_bytes(uint32_t nstreams, uint32_t raw_cap)
{
    const uint32_t cap = (uint32_t)align_up((size_t)raw_cap + raw_cap / 4 + 64, 256);
    const uint32_t out_cap = (uint32_t)align_up((size_t)raw_cap + raw_cap / 50 + 4096, 256);
    const uint32_t sel_cap = (uint32_t)align_up(cap / kGSize + 8, 64);
    const size_t N = (size_t)nstreams * cap;
    size_t b = 0;
    b += align_up((size_t)nstreams * align_up(raw_cap, 16), 256);   // raw
    b += align_up(N, 256);                                      // T
    b += 2 * align_up(N * 8, 256);                              // keys
    b += 6 * align_up(N * 4, 256);                              // vals_a, sa, rank, vals_b, cl0, cl1
    b += align_up(N, 256);                                      // uflag
    b += align_up((size_t)nstreams * (cap + 8) * 2, 256);       // mtfv
    b += 2 * align_up((size_t)nstreams * sel_cap, 256);         // sel, sel_mtf
    b += align_up((size_t)nstreams * kMaxGroups * kMaxAlpha, 256);       // len
    b += 2 * align_up((size_t)nstreams * kMaxGroups * kMaxAlpha * 4, 256);   // code, rfreq
    b += align_up((size_t)nstreams * out_cap, 256);             // words
    b += align_up((size_t)nstreams * kMaxAlpha * 4, 256);       // mtf_freq
    b += align_up((size_t)nstreams * 8 * 4, 256);               // inuse
    b += align_up((size_t)nstreams * kMaxGroups * 4 + 64, 256);  // wide heap list
    b += align_up((size_t)nstreams * 512 * 4, 256);             // A / B rotations per first byte
    b += align_up((size_t)nstreams * 1024 * 4, 256);            // placement tables
    b += 16 * align_up((size_t)nstreams * 4 + 64, 256);         // small per-stream arrays
    b += align_up(((size_t)nstreams + 1) * 8 + 32, 256);        // offsets + counters
    b += align_up(prim_tmp_bytes(nstreams, cap), 256);          // rocPRIM temporary storage
    return b;
}

// Compress streams [first, first + count) of the block grid of `img`
// (device, image layout) into `payload` (device, contiguous in block order);
// sizes[i] = compressed size of stream i, flags[i] != 0 -> the stream must be
// produced by the host library (its bytes are absent from the payload).
extern "C" int lfm_hip_bzip2_blocks(const void* d_img, const uint32_t dims[5], const uint32_t bs[5], uint32_t bpp,
                                    uint32_t first, uint32_t count, uint32_t level, void* d_ws, size_t ws_bytes,
                                    void* d_payload, uint64_t* h_sizes, uint32_t* h_flags, void* stream_)
{
    hipStream_t st = (hipStream_t)stream_;
    if (!d_img || !dims || !bs || !bpp || !count || level < 1 || level > 9 || !d_ws || !d_payload) return LFM_HIP_EINVAL;
    ensure_crc_table();
    static thread_local int crc_dev = -1;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (crc_dev != dev) {
        if (hipMemcpyToSymbol(HIP_SYMBOL(c_crc_table), host_crc_table, sizeof(host_crc_table)) != hipSuccess ||
            hipMemcpyToSymbol(HIP_SYMBOL(c_crc4), host_crc4, sizeof(host_crc4)) != hipSuccess ||
            hipMemcpyToSymbol(HIP_SYMBOL(c_crc_shb), host_crc_shb, sizeof(host_crc_shb)) != hipSuccess ||
            hipMemcpyToSymbol(HIP_SYMBOL(c_crc_unshift), host_crc_unshift, sizeof(host_crc_unshift)) != hipSuccess)
            return LFM_HIP_ERUNTIME;
        crc_dev = dev;
    }
    StageEvents& SE = t_stage;
    SE.valid = false;
    const bool timed = SE.ready(dev);
    auto mark = [&](int i) {
        if (timed) (void)hipEventRecord(SE.ev[i], st);
    };
    Batch B{};
    B.img = (const uint8_t*)d_img;
    uint32_t raw_cap = bpp;
    for (int d = 0; d < 5; ++d) {
        B.g.dims[d] = dims[d];
        B.g.bs[d] = bs[d];
        B.g.nb[d] = (uint32_t)((dims[d] + bs[d] - 1) / bs[d]);
        raw_cap *= bs[d];
    }
    B.g.bpp = bpp;
    B.first_block = first;
    B.nstreams = count;
    B.raw_cap = (uint32_t)align_up(raw_cap, 16);  // stream stride of the raw blocks (16-byte loads)
    B.cap = (uint32_t)align_up((size_t)raw_cap + raw_cap / 4 + 64, 256);
    B.out_cap = (uint32_t)align_up((size_t)raw_cap + raw_cap / 50 + 4096, 256);
    B.sel_cap = (uint32_t)align_up(B.cap / kGSize + 8, 64);
    B.level = level;
    B.nblock_max = 100000u * level - 19u;
    if (ws_bytes < lfm_hip_bzip2_workspace_bytes(count, raw_cap)) return LFM_HIP_EINVAL;
    const size_t N = (size_t)count * B.cap;
    if (N >= (1ull << 32)) return LFM_HIP_EINVAL;
    uint8_t* p = (uint8_t*)d_ws;
    auto take = [&](size_t bytes) { uint8_t* r = p; p += align_up(bytes, 256); return r; };
    B.raw = take((size_t)count * B.raw_cap);
    B.T = take(N);
    B.keys_a = (uint64_t*)take(N * 8);
    B.keys_b = (uint64_t*)take(N * 8);
    B.vals_a = (uint32_t*)take(N * 4);
    B.sa = (uint32_t*)take(N * 4);
    B.rank = (uint32_t*)take(N * 4);
    B.vals_b = (uint32_t*)take(N * 4);
    B.cl0 = (uint32_t*)take(N * 4);
    B.cl1 = (uint32_t*)take(N * 4);
    B.uflag = take(N);
    B.mtfv = (uint16_t*)take((size_t)count * (B.cap + 8) * 2);
    B.sel = take((size_t)count * B.sel_cap);
    B.sel_mtf = take((size_t)count * B.sel_cap);
    B.len = take((size_t)count * kMaxGroups * kMaxAlpha);
    B.code = (uint32_t*)take((size_t)count * kMaxGroups * kMaxAlpha * 4);
    B.rfreq = (uint32_t*)take((size_t)count * kMaxGroups * kMaxAlpha * 4);
    B.words = (uint32_t*)take((size_t)count * B.out_cap);
    B.mtf_freq = (uint32_t*)take((size_t)count * kMaxAlpha * 4);
    B.inuse = (uint32_t*)take((size_t)count * 8 * 4);
    B.wide = (uint32_t*)take((size_t)count * kMaxGroups * 4 + 64);
    B.abcnt = (uint32_t*)take((size_t)count * 512 * 4);
    B.itab = (uint32_t*)take((size_t)count * 1024 * 4);
    uint32_t** small[] = {&B.raw_len, &B.n, &B.crc, &B.flags, &B.done, &B.seg_begin, &B.seg_end, &B.nmtf,
                          &B.orig_ptr, &B.nsel, &B.ngroups, &B.out_bytes, &B.nsub, &B.bwt_mode};
    for (uint32_t** q : small) *q = (uint32_t*)take((size_t)count * 4 + 64);
    for (int k = (int)(sizeof(small) / sizeof(small[0])); k < 16; ++k) (void)take((size_t)count * 4 + 64);
    uint64_t* offs = (uint64_t*)take(((size_t)count + 1) * 8 + 32);
    size_t tmp_bytes = prim_tmp_bytes(count, B.cap);
    void* tmp = take(tmp_bytes);

    hipError_t e = hipSuccess;
    auto ok = [&]() { return (e = hipGetLastError()) == hipSuccess; };
    // RLE1 reads the image directly when every block row is whole 16-byte
    // pieces at 16-byte aligned addresses (the default uint16 96-pixel
    // blocks); other geometries gather the blocks first
    const bool from_img = ((uintptr_t)d_img & 15) == 0 && (bs[0] * bpp) % 16 == 0 && (dims[0] * bpp) % 16 == 0 &&
                          ((dims[0] % bs[0]) * bpp) % 16 == 0;
    mark(0);
    if (from_img) {
        hipLaunchKernelGGL(rle1_crc<true>, dim3(count), dim3(kRleThreads), 0, st, B);
    } else {
        hipLaunchKernelGGL(gather_blocks, dim3(64, count), dim3(256), 0, st, B);
        hipLaunchKernelGGL(rle1_crc<false>, dim3(count), dim3(kRleThreads), 0, st, B);
    }
    if (!ok()) return LFM_HIP_ERUNTIME;
    // counters after offs: [0..2] chunk classes 0..2 of the bucket pass (then
    // the tied-list counts [0], [1]); [3] wide Huffman streams, [4] Huffman
    // retries, [5] chunk class 3
    uint32_t* d_cnt = (uint32_t*)(offs + count + 1);
    B.wide_cnt = d_cnt + 3;
    mark(1);
    // BWT: the B rotations sorted (round 0 = bucket pass + chunk sorts by the
    // 8-byte prefix, then the tie rounds), every other rotation placed by
    // bwt_induce.  Ties that would need prefix doubling (long repeats) restart
    // the batch with every rotation sorted (B.it_full: doubling ranks every
    // rotation), which also finds the periodic blocks.
    uint32_t* cl = B.cl0;
    uint32_t* cl_next = B.cl1;
    uint32_t covered = kKeyBytes;
    bool none_left = false;  // a count read 0 and no kernel ran since: skip the later reads
    uint32_t first_ties = 0, left_runs = 0;  // tied slots after the chunk sorts, runs tie_runs_direct left (LFM_BZ2_STATS)
#ifndef LFM_BWT_FORCE_FULL
#define LFM_BWT_FORCE_FULL 0  // timing variants: every rotation sorted, no induction
#endif
#ifndef LFM_BWT_RSORT
#define LFM_BWT_RSORT 0  // 1: the hand-written radix chunk sort (bwt_chunk_rsort) instead of rocPRIM's merge sort
#endif
#if LFM_BWT_RSORT
#define LFM_CHUNK_SORT bwt_chunk_rsort
#else
#define LFM_CHUNK_SORT bwt_chunk_sort
#endif
    for (B.it_full = LFM_BWT_FORCE_FULL;; B.it_full = 1) {
        ChunkLists CL;
        const size_t q = N / 4;  // chunk lists in the cl0 / cl1 areas (at most 3 n / kChunk + 1 chunks per stream)
        for (int c = 0; c < 4; ++c) {
            CL.b[c] = B.cl0 + c * q;
            CL.e[c] = B.cl1 + c * q;
        }
        CL.cnt = d_cnt;
        CL.cnt3 = d_cnt + 5;
        uint32_t nch[6] = {0, 0, 0, 0, 0, 0};
        if (hipMemsetAsync(d_cnt, 0, 32, st) != hipSuccess ||
            hipMemsetAsync(B.done, 0, (size_t)count * 4, st) != hipSuccess)
            return LFM_HIP_ERUNTIME;
        hipLaunchKernelGGL(bwt_bucket<kBucketBits>, dim3(count), dim3(kBucketThreads), 0, st, B, CL);
        if (!ok() || hipMemcpyAsync(nch, d_cnt, 24, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return LFM_HIP_ERUNTIME;
        // chunks in XCD-aware order: workgroup b runs on XCD b % 8
        auto cs_grid = [&](uint32_t nc, uint32_t& per) {
            per = (nc + 7) / 8;
            return dim3(8 * per);
        };
        uint32_t per = 0;
        if (nch[5]) {
            const dim3 g = cs_grid(nch[5], per);
            hipLaunchKernelGGL((LFM_CHUNK_SORT<kTinyCap / kCsItems, kCsItems>), g, dim3(kTinyCap / kCsItems), 0, st, B,
                               CL.b[3], CL.e[3], nch[5], per);
        }
        if (nch[0]) {
            const dim3 g = cs_grid(nch[0], per);
            hipLaunchKernelGGL((LFM_CHUNK_SORT<kCsThreads, kCsItems>), g, dim3(kCsThreads), 0, st, B, CL.b[0], CL.e[0],
                               nch[0], per);
        }
        if (nch[1]) {
            const dim3 g = cs_grid(nch[1], per);
            hipLaunchKernelGGL((LFM_CHUNK_SORT<kBigThreads, kBigItems>), g, dim3(kBigThreads), 0, st, B, CL.b[1],
                               CL.e[1], nch[1], per);
        }
        if (nch[2]) {
            hipLaunchKernelGGL(bwt_chunk_keys, dim3(nch[2]), dim3(256), 0, st, B, CL.b[2], CL.e[2]);
            e = rocprim::segmented_radix_sort_pairs(tmp, tmp_bytes, B.keys_a, B.keys_b, B.vals_a, B.sa, (unsigned)N,
                                                    nch[2], CL.b[2], CL.e[2], 0, 64 - kBucketBits, st);
            if (e == hipSuccess)
                hipLaunchKernelGGL(bwt_chunk_flags, dim3(nch[2]), dim3(256), 0, st, B, CL.b[2], CL.e[2]);
        }
        if (!ok()) return LFM_HIP_ERUNTIME;
        cl = B.cl0;
        cl_next = B.cl1;
        hipLaunchKernelGGL(tie_offsets, dim3(1), dim3(1024), 0, st, B, d_cnt);
        hipLaunchKernelGGL(tie_compact, dim3(count), dim3(256), 0, st, B, B.cl0);
        hipLaunchKernelGGL(tie_runs_direct, dim3(1024), dim3(256), 0, st, B, B.cl0, d_cnt, d_cnt + 7);
        if (!ok()) return LFM_HIP_ERUNTIME;
        covered = kKeyBytes;
        none_left = false;
        // text rounds over the tied list (group keys: u64 per entry in the rank
        // area, group index / bounds in the mtfv area -- both free here)
        uint64_t* gk = (uint64_t*)B.rank;
        uint32_t* bnd = (uint32_t*)B.mtfv;
        for (int r = 0; r < kTextRounds && e == hipSuccess; ++r) {
            // counters: [0] tied slots, [7] runs tie_runs_direct left (read with the first round's count)
            uint32_t c8[8] = {};
            if (hipMemcpyAsync(c8, d_cnt, r == 0 ? 32 : 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess) {
                e = hipErrorUnknown;
                break;
            }
            const uint32_t cnt = c8[0];
            if (r == 0) {
                first_ties = cnt;
                left_runs = c8[7];
            }
            if (cnt == 0 || (r == 0 && c8[7] == 0)) {  // nothing tied, or tie_runs_direct sorted every run
                none_left = true;
                break;
            }
            if ((size_t)cnt * 4 > N) break;
            unsigned gbits = 1;
            while ((1u << gbits) < cnt) ++gbits;
            // group index above the text bytes in one 64-bit key: fewer text
            // bytes when the tied list is longer than 2^24
            const uint32_t tb = std::min<uint32_t>(kTextBytes, (64 - gbits) / 8);
            uint32_t* gidx = bnd + cnt;
            const uint32_t grid = std::min<uint32_t>(4096, (cnt + 255) / 256);
            if (r == 0) hipLaunchKernelGGL(text_gather_keys, dim3(grid), dim3(256), 0, st, B, cl, d_cnt, gk);
            hipLaunchKernelGGL(text_bounds, dim3(grid), dim3(256), 0, st, B, cl, d_cnt, gk, bnd);
            e = rocprim::inclusive_scan(tmp, tmp_bytes, bnd, gidx, (size_t)cnt, rocprim::plus<uint32_t>(), st);
            if (e != hipSuccess) break;
            hipLaunchKernelGGL(text_keys, dim3(grid), dim3(256), 0, st, B, cl, d_cnt, gidx, covered, tb);
            e = rocprim::radix_sort_pairs(tmp, tmp_bytes, B.keys_a, B.keys_b, B.vals_a, B.vals_b, cnt, 0,
                                          8 * tb + gbits, st);
            if (e != hipSuccess) break;
            hipLaunchKernelGGL(text_write, dim3(grid), dim3(256), 0, st, B, cl, d_cnt);
            covered += tb;
            e = rocprim::select(tmp, tmp_bytes, B.keys_b, B.uflag, gk, d_cnt + 1, (size_t)cnt, st);
            if (e == hipSuccess) e = rocprim::select(tmp, tmp_bytes, cl, B.uflag, cl_next, d_cnt, (size_t)cnt, st);
            std::swap(cl, cl_next);
        }
        if (e != hipSuccess) return LFM_HIP_ERUNTIME;
        // ties left (long repeats)
        uint32_t cnt = 0;
        if (!none_left && (hipMemcpyAsync(&cnt, d_cnt, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                           hipStreamSynchronize(st) != hipSuccess))
            return LFM_HIP_ERUNTIME;
        if (cnt == 0) {
            none_left = true;
            break;
        }
        if (!B.it_full) continue;  // doubling needs the rank of every rotation: sort them all
        // ranks of every rotation for doubling: group bounds of the remaining
        // list from the last text keys, or from the first-round keys when no
        // text round ran
        uint64_t* gsrc = gk;
        const uint32_t grid = std::min<uint32_t>(4096, (cnt + 255) / 256);
        if (covered == kKeyBytes) gsrc = (uint64_t*)B.vals_b;  // cnt * 8 <= N * 4 when cnt <= N / 2: rank0 otherwise
        if (covered == kKeyBytes && (size_t)cnt * 2 > N) {
            hipLaunchKernelGGL(bwt_rank0, dim3(count), dim3(1024), 0, st, B);
        } else {
            if (covered == kKeyBytes) hipLaunchKernelGGL(text_gather_keys, dim3(grid), dim3(256), 0, st, B, cl, d_cnt, gsrc);
            uint32_t* bnd2 = (uint32_t*)B.keys_a;  // 2 * cnt u32 fit the keys area
            uint32_t* hv = bnd2 + cnt;
            uint32_t* hvs = (uint32_t*)B.cl1 == cl ? (uint32_t*)B.cl0 : (uint32_t*)B.cl1;
            hipLaunchKernelGGL(text_bounds, dim3(grid), dim3(256), 0, st, B, cl, d_cnt, gsrc, bnd2);
            hipLaunchKernelGGL(text_head_slots, dim3(grid), dim3(256), 0, st, cl, d_cnt, bnd2, hv);
            e = rocprim::inclusive_scan(tmp, tmp_bytes, hv, hvs, (size_t)cnt, rocprim::maximum<uint32_t>(), st);
            hipLaunchKernelGGL(bwt_rank_all, dim3(8192), dim3(256), 0, st, B, N);
            hipLaunchKernelGGL(text_rank_tied, dim3(grid), dim3(256), 0, st, B, cl, d_cnt, hvs);
            cl_next = hvs == (uint32_t*)B.cl0 ? B.cl0 : B.cl1;
        }
        break;
    }
    // doubling rounds over what the text rounds left (long repeats only, B.it_full)
    uint32_t h = covered;
    const uint32_t max_n = B.cap;
    while (e == hipSuccess && !none_left) {
        uint32_t cnt = 0;
        if (hipMemcpyAsync(&cnt, d_cnt, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            e = hipErrorUnknown;
            break;
        }
        if (cnt == 0) break;
        if (h >= max_n) {  // every remaining tie is a pair of equal rotations
            hipLaunchKernelGGL(bwt_flag_periodic, dim3(256), dim3(256), 0, st, B, cl, d_cnt);
            break;
        }
        const uint32_t grid = std::min<uint32_t>(4096, (cnt + 255) / 256);
        hipLaunchKernelGGL(bwt_comp_keys, dim3(grid), dim3(256), 0, st, B, cl, d_cnt, h);
        e = rocprim::radix_sort_pairs(tmp, tmp_bytes, B.keys_a, B.keys_b, B.vals_a, B.vals_b, cnt, 0, 52, st);
        if (e != hipSuccess) break;
        uint32_t* hv = (uint32_t*)B.keys_a;  // the sort has consumed keys_a
        uint32_t* hvs = hv + cnt;
        hipLaunchKernelGGL(bwt_comp_heads, dim3(grid), dim3(256), 0, st, B, cl, d_cnt, hv);
        e = rocprim::inclusive_scan(tmp, tmp_bytes, hv, hvs, (size_t)cnt, rocprim::maximum<uint32_t>(), st);
        if (e != hipSuccess) break;
        hipLaunchKernelGGL(bwt_comp_rank, dim3(grid), dim3(256), 0, st, B, d_cnt, hvs);
        e = rocprim::select(tmp, tmp_bytes, cl, B.uflag, cl_next, d_cnt, (size_t)cnt, st);
        std::swap(cl, cl_next);
        h *= 2;
    }
    if (e != hipSuccess) return LFM_HIP_ERUNTIME;
    if (!B.it_full) {
        // the other type placed by one scan; the final order in the vals_b area
        B.sfin = B.vals_b;
        B.ent = (uint2*)B.keys_a;
        const uint32_t chunks = (B.cap + kPlaceChunk - 1) / kPlaceChunk;
        hipLaunchKernelGGL(bwt_place_sorted, dim3(8 * chunks * ((count + 7) / 8)), dim3(256), 0, st, B, chunks);
        hipLaunchKernelGGL(bwt_induce, dim3(count), dim3(64), 0, st, B);
        if (!ok()) return LFM_HIP_ERUNTIME;
        B.sa = B.sfin;
    }
    mark(2);
    if (t_hook) t_hook(t_hook_ctx, 1);  // the doubling / tie rounds above end with a host synchronisation
    {
        const uint32_t nseg_max = (B.cap + kSeg - 1) / kSeg;
        int32_t* seg_last = (int32_t*)B.keys_a;  // free after the BWT (count * nseg_max KiB << N * 8 bytes)
        const dim3 g((nseg_max + 3) / 4, count);
        if (B.it_full) hipLaunchKernelGGL(mtf_last<false>, g, dim3(256), 0, st, B, nseg_max, seg_last);
        else hipLaunchKernelGGL(mtf_last<true>, g, dim3(256), 0, st, B, nseg_max, seg_last);
        hipLaunchKernelGGL(mtf_prefix, dim3(count), dim3(256), 0, st, B, nseg_max, seg_last);
        hipLaunchKernelGGL(mtf_win, g, dim3(256), 0, st, B, nseg_max, (const int32_t*)seg_last);
        hipLaunchKernelGGL(rle2, dim3(count), dim3(kRle2Threads), 0, st, B);
    }
    // streams whose Huffman weights need u64 heap entries (listed by rle2)
    uint32_t nwide = 0;
    if (!ok() || hipMemcpyAsync(&nwide, B.wide_cnt, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess || nwide > count)
        return LFM_HIP_ERUNTIME;
    mark(3);
    if (t_hook) t_hook(t_hook_ctx, 2);  // after the wide-stream count's synchronisation: rle2 has run
    hipLaunchKernelGGL(huff_init, dim3(count), dim3(64), 0, st, B);
    // stage hook 3 once the Huffman tables are done (emission and compaction
    // still queued): a caller may start its next work beside this tail
    // (earlier, after the second or third code-length round, measured slower:
    // the next encode's kernels then slow these latency-bound rounds)
    // (one per thread, destroyed when the thread exits: gpu_compress starts
    // its slot threads per call)
    static thread_local struct TablesEvent {
        hipEvent_t ev = nullptr;
        int dev = -1;
        ~TablesEvent()
        {
            if (ev) (void)hipEventDestroy(ev);
        }
    } tables_ev;
    if (t_hook && tables_ev.dev != dev) {
        if (tables_ev.ev) (void)hipEventDestroy(tables_ev.ev);
        tables_ev.ev = nullptr;
        tables_ev.dev = -1;
        if (hipEventCreateWithFlags(&tables_ev.ev, hipEventDisableTiming) == hipSuccess) tables_ev.dev = dev;
    }
    hipEvent_t ev_tables = tables_ev.ev;
    for (int it = 0; it < kIters; ++it) {
        hipLaunchKernelGGL(huff_select_reg, dim3(count), dim3(kHuffThreads), 0, st, B);
        // uniform heaps, 32 per workgroup: u32 entries for the narrow tables,
        // u64 for the streams rle2 listed, in one launch
#ifndef LFM_HUFF_PLANE
#define LFM_HUFF_PLANE 32
#endif
        constexpr uint32_t kPlane = LFM_HUFF_PLANE;  // (stream, table) heaps per wave
        const uint32_t nn = (count * kMaxGroups + kPlane - 1) / kPlane;
        const uint32_t nw = (nwide * kMaxGroups + kPlane / 2 - 1) / (kPlane / 2);
        hipLaunchKernelGGL(huff_lengths_heap<kPlane>, dim3(nn + nw), dim3(64), 0, st, B, nw, nwide);
    }
    hipLaunchKernelGGL(huff_final, dim3(count), dim3(64), 0, st, B);
    mark(4);
    const bool hook3 = t_hook && ev_tables && hipEventRecord(ev_tables, st) == hipSuccess;
    hipLaunchKernelGGL(emit_stream, dim3(count), dim3(kEmitThreads), 0, st, B);
    hipLaunchKernelGGL(scan_offsets, dim3(1), dim3(1024), 0, st, B.out_bytes, count, offs);
    hipLaunchKernelGGL(compact_streams, dim3(count), dim3(256), 0, st, B, offs, (uint8_t*)d_payload);
    mark(5);
    if (!ok()) return LFM_HIP_ERUNTIME;
    if (hook3 && hipEventSynchronize(ev_tables) == hipSuccess) t_hook(t_hook_ctx, 3);
    static const bool stats = std::getenv("LFM_BZ2_STATS") && std::atoi(std::getenv("LFM_BZ2_STATS")) != 0;
    if (stats) {
        uint32_t c[8] = {};
        if (hipMemcpyAsync(c, d_cnt, 32, hipMemcpyDeviceToHost, st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess)
            std::fprintf(stderr, "lfm_bzip2 stats: %u streams, %u with u64 Huffman heaps, Huffman retries %u, "
                         "tied after the chunk sorts %u, runs left to the tie rounds %u\n", count, c[3], c[4], first_ties,
                         left_runs);
    }
    std::vector<uint32_t> nbytes(count);
    if (hipMemcpyAsync(nbytes.data(), B.out_bytes, count * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(h_flags, B.flags, count * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return LFM_HIP_ERUNTIME;
    for (uint32_t i = 0; i < count; ++i) h_sizes[i] = nbytes[i];
    if (timed) {
        SE.valid = true;
        for (int i = 0; i < 5; ++i)
            if (hipEventElapsedTime(&SE.last_ms[i], SE.ev[i], SE.ev[i + 1]) != hipSuccess) SE.valid = false;
    }
    return LFM_HIP_OK;
}

extern "C" void lfm_hip_bzip2_set_stage_hook(void (*fn)(void*, int), void* ctx)
{
    t_hook = fn;
    t_hook_ctx = ctx;
}

extern "C" int lfm_hip_bzip2_last_stage_ms(float ms[5])
{
    if (!ms || !t_stage.valid) return 3;
    for (int i = 0; i < 5; ++i) ms[i] = t_stage.last_ms[i];
    return 0;
}
