// lfm_bunzip2.hip -- GPU decode of the .lfm block streams (bzip2, one block per
// stream) on gfx950: the decode side of SURVEY.md 8(f2).
//
// The reference decodes every block with libbzip2 on the host
// (klb_imageIO.cpp:1748-1821 via BZ2_bzBuffToBuffDecompress); here a batch of
// streams is decoded on the device, restating bzip2-1.0.6's decompress.c:
//
//   bzd_huff    one wave per stream: stream / block headers, the mapping
//               table, selectors (unary MTF), delta-coded code lengths, the
//               decode tables (an 8-bit lookup table per Huffman table plus
//               limit / base / perm for longer codes, BZ2_hbCreateDecodeTables),
//               then the symbols: RUNA/RUNB runs and move-to-front (the list
//               in registers, 4 entries per lane), giving the BWT last column
//               ll[] and the block length n.  Anything else (several blocks,
//               randomised blocks, a malformed stream) is flagged for the host.
//   bzd_tt      one workgroup per stream: byte counts, then LF(i) = C[ll[i]] +
//               Occ(ll[i], i) (ranks among equal bytes by 8-ballot matches,
//               stable), tt[LF(i)] = i << 8 | ll[LF(i)] (decompress.c's fast
//               tt), and the inverse BWT as a parallel walk: markers every kMark
//               nodes of the cycle (plus its start, tt[origPtr] >> 8), each
//               walker follows tt from its marker to the next one, counting and
//               keeping the first kWalkKeep bytes it passes, one lane chains the
//               segments to their output offsets, the kept bytes are copied into
//               place (a wave per segment) and only the rare longer segments
//               are walked again from where their walker stopped keeping.
//   bzd_rle1    one wave per stream: RLE1 decode (4 equal bytes + a count) into
//               the output block from 64 text segments (their start states
//               resolved by running every start state), CRC-32 of the block in
//               64 segments combined by polynomial shifts, checked against the
//               header.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "lfm_hip.h"

#ifndef LFM_BZD_PROBE
#define LFM_BZD_PROBE 0  // timing probes of bzd_huff (scripts only; 0 in the library)
#endif

namespace lfm {
namespace bzd {

constexpr int kMaxGroups = 6;
constexpr int kMaxAlpha = 258;
constexpr int kMaxSel = 18002;
constexpr int kMaxLen = 20;
constexpr uint32_t kMark = 128;  // cycle nodes per inverse-BWT walker (on average)
constexpr uint32_t kWalkKeep = 512;  // bytes a walker keeps from its one walk (segments are
                                     // geometric, mean kMark: 1.8 % of them are longer)

// flags
constexpr uint32_t kHost = 1;      // decode with the host library
constexpr uint32_t kCrcFail = 2;   // decoded, but the block CRC does not match

__constant__ uint32_t c_dcrc[256];

struct Dec {
    const uint8_t* payload;   // 4-byte aligned
    const uint64_t* offs;     // count + 1 byte offsets
    uint32_t count;
    uint32_t cap;             // RLE1 / ll capacity per stream
    uint32_t out_stride;
    uint8_t* out;
    uint8_t* ll;              // cap per stream
    uint32_t* tt;             // cap per stream
    uint8_t* rle;             // cap per stream (the same buffer as ll)
    uint32_t mcap;            // markers per stream
    uint32_t* mnext;
    uint32_t* mlen;
    uint32_t* mstart;
    uint32_t* mres;           // node a walker stopped keeping bytes at (segments > kWalkKeep)
    uint8_t* wkeep;           // kWalkKeep bytes per walker
    uint32_t* n;
    uint32_t* orig;
    uint32_t* crc;
    uint32_t* flags;
    uint32_t* out_len;
    uint32_t sel_cap;         // selectors that fit the decoder's LDS
};

// MSB-first bit reader over the payload: a 64-bit window of two big-endian
// words, refilled one aligned word at a time.
struct BitReader {
    const uint32_t* w;
    uint64_t pos;    // absolute bit position
    uint64_t wpos;   // word index of the window's first word
    uint64_t win;
    uint64_t end;    // bit position past the stream
    __device__ __forceinline__ uint32_t word(uint64_t i) const { return __builtin_bswap32(w[i]); }
    __device__ __forceinline__ void init(const uint8_t* payload, uint64_t byte0, uint64_t byte1)
    {
        w = (const uint32_t*)payload;
        pos = byte0 * 8;
        end = byte1 * 8;
        wpos = pos >> 5;
        win = ((uint64_t)word(wpos) << 32) | word(wpos + 1);
    }
    __device__ __forceinline__ uint32_t peek(uint32_t nb) const  // nb in 1..32
    {
        const uint32_t off = (uint32_t)(pos - 32 * wpos);
        return (uint32_t)((win << off) >> (64 - nb));
    }
    __device__ __forceinline__ void skip(uint32_t nb)
    {
        pos += nb;
        while (pos - 32 * wpos >= 32) {
            ++wpos;
            win = (win << 32) | word(wpos + 1);
        }
    }
    __device__ __forceinline__ uint32_t get(uint32_t nb)
    {
        const uint32_t v = peek(nb);
        skip(nb);
        return v;
    }
    __device__ __forceinline__ bool over() const { return pos > end; }
};

// ----------------------------------------------------------------- huffman --
// One wave per stream.  The decode is one sequential chain per stream, so
// every lane runs the same (wave-uniform) header and symbol code; what the
// wave buys is storage and wide steps:
//  * the decode tables live in LDS (an LB-bit lookup table per Huffman table:
//    one broadcast LDS read decodes most symbols; longer codes walk bzip2's
//    limit table).  The LDS per stream is kept near 10 KB so that a whole
//    batch (~16 streams per CU) is resident at once: the decode is latency
//    bound per wave, so resident waves are throughput;
//  * the move-to-front list holds the output bytes themselves (seqToUnseq
//    applied up front), 4 entries per lane: a move-to-front of position m is
//    one lane shift and a byte select, not m serial moves; list[m] is one
//    readlane;
//  * the bit window is refilled from a vector window: lane l holds payload
//    word base + l and a second register the next 64 words, loaded 64 words
//    (~300 symbols) before they are needed; a refill is one readlane (a
//    scalar-register queue made the compiler wait for every refill load right
//    where it was issued);
//  * the symbols go a group (50 symbols, one Huffman table) at a time: the
//    Huffman loop only decodes (symbol k of the group into lane k), then the
//    lanes work out the RUNA/RUNB digits (digit j of a run adds (sym + 1) << j
//    copies of the list front, so each digit lane owns its own stretch of the
//    output), the move-to-front chain runs over the group's non-run symbols
//    only (s_ff1 over their ballot), a prefix sum over the lanes gives every
//    lane its output offset and the lanes store their bytes.  The per-symbol
//    scalar code is a third of the earlier single loop's (which did the run
//    bookkeeping, the move to front and a 64-byte output staging per symbol),
//    and the decode is bound by that code: ~16 waves per CU share one scalar
//    unit (PMC: 43 SALU + 20 VALU + 11 branch instructions per symbol before).
// Output: the BWT last column ll[], n, origPtr, the block CRC.
struct WaveBits {
    const uint32_t* w;   // the stream's first (aligned) payload word
    uint32_t nw;         // words that start inside the stream (later ones read as 0)
    uint32_t base;       // word held by lane 0 of vq
    uint32_t vq, vn;     // per lane: word base + lane (byte-swapped), base + 64 + lane (raw)
    uint32_t wi;         // next word to enter the bit window
    uint64_t win;        // 64 bits from the current word on
    uint32_t off;        // bits of win already consumed (< 32)
    uint32_t total;      // bits in the stream, counted from the first word's first bit
    // raw (unswapped) load with a clamped index: no branch and no use of the
    // value next to the load, so the wait lands where the word is first needed
    __device__ __forceinline__ uint32_t raw(uint32_t i) const { return w[min(i, nw - 1)]; }
    __device__ __forceinline__ uint32_t fix(uint32_t v, uint32_t i) const { return i < nw ? __builtin_bswap32(v) : 0u; }
    __device__ __forceinline__ uint32_t next()
    {
        if (wi - base == 64) {
            base += 64;
            vq = fix(vn, base + threadIdx.x);
            vn = raw(base + 64 + threadIdx.x);
        }
        return (uint32_t)__builtin_amdgcn_readlane((int)vq, (int)(wi++ - base));
    }
    __device__ __forceinline__ void init(const uint8_t* payload, uint64_t byte0, uint64_t byte1)
    {
        w = (const uint32_t*)payload + (byte0 >> 2);
        nw = (uint32_t)((byte1 - (byte0 & ~3ull) + 3) >> 2);
        off = (uint32_t)(byte0 & 3) * 8;
        total = (uint32_t)(byte1 - byte0) * 8 + off;
        base = 0;
        vq = fix(raw(threadIdx.x), threadIdx.x);
        vn = raw(64 + threadIdx.x);
        wi = 2;
        win = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)vq, 0) << 32) |
              (uint32_t)__builtin_amdgcn_readlane((int)vq, 1);
    }
    __device__ __forceinline__ uint32_t peek(uint32_t nb) const  // nb in 1..32
    {
        return (uint32_t)((win << off) >> (64 - nb));
    }
    __device__ __forceinline__ void skip(uint32_t nb)  // nb <= 32
    {
        off += nb;
        if (off >= 32) {
            off -= 32;
            win = (win << 32) | next();
        }
    }
    __device__ __forceinline__ uint32_t get(uint32_t nb)
    {
        const uint32_t v = peek(nb);
        skip(nb);
        return v;
    }
    // bits consumed past the stream's end (win holds words wi - 2 and wi - 1)
    __device__ __forceinline__ bool over() const { return 32 * (wi - 2) + off > total; }
};

// The symbol loop's bit reader in vector registers (bzd_huff<LB, true>):
// every lane holds the same window, so the lookup is an LDS broadcast read,
// the decode arithmetic is VALU -- four SIMDs per CU -- and only loop control
// stays on the CU's one scalar unit, which the ~16 resident streams share
// (PMC: the scalar unit ~53 % busy with ~21 SALU instructions per symbol in
// the wave-uniform reader).  Refills read the vector window by ds_bpermute.
struct LaneBits {
    const uint32_t* w;
    uint32_t nw, base, vq, vn, wi, off, total;
    uint64_t win;
    __device__ __forceinline__ uint32_t raw(uint32_t i) const { return w[min(i, nw - 1)]; }
    __device__ __forceinline__ uint32_t fix(uint32_t v, uint32_t i) const { return i < nw ? __builtin_bswap32(v) : 0u; }
    __device__ __forceinline__ void from(const WaveBits& b)
    {
        // the copies go through a lane shuffle so the compiler keeps the
        // state in vector registers (a shuffle's result is divergent to it)
        w = b.w;
        nw = b.nw;
        base = (uint32_t)__shfl((int)b.base, 0);
        vq = b.vq;
        vn = b.vn;
        wi = (uint32_t)__shfl((int)b.wi, 0);
        off = (uint32_t)__shfl((int)b.off, 0);
        total = b.total;
        win = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(b.win >> 32), 0) << 32) |
              (uint32_t)__shfl((int)(uint32_t)b.win, 0);
    }
    __device__ __forceinline__ void to(WaveBits& b) const
    {
        auto U = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); };
        b.base = U(base);
        b.vq = vq;
        b.vn = vn;
        b.wi = U(wi);
        b.off = U(off);
        b.win = ((uint64_t)U((uint32_t)(win >> 32)) << 32) | U((uint32_t)win);
    }
    __device__ __forceinline__ uint32_t next()
    {
        if (wi - base == 64) {
            base += 64;
            vq = fix(vn, base + threadIdx.x);
            vn = raw(base + 64 + threadIdx.x);
        }
        return (uint32_t)__shfl((int)vq, (int)(wi++ - base));
    }
    __device__ __forceinline__ uint32_t peek(uint32_t nb) const { return (uint32_t)((win << off) >> (64 - nb)); }
    __device__ __forceinline__ void skip(uint32_t nb)
    {
        off += nb;
        if (off >= 32) {
            off -= 32;
            win = (win << 32) | next();
        }
    }
    // skip with the refill test on a scalar copy of off (equal in every
    // lane): a uniform s_cbranch instead of an exec-mask branch (save / test
    // / restore exec on the CU's one scalar unit, per symbol)
    __device__ __forceinline__ void skip_u(uint32_t nb)
    {
        off += nb;
        if ((uint32_t)__builtin_amdgcn_readfirstlane((int)off) >= 32u) {
            off -= 32;
            win = (win << 32) | next();
        }
    }
    __device__ __forceinline__ bool over() const { return 32 * (wi - 2) + off > total; }
};

// inclusive wave sum by DPP row shifts and row broadcasts (no LDS round
// trips; the lanes a step has no source for add 0)
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_in(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_sum_incl(uint32_t x)
{
    x += dpp_in<0x111, 0xF>(x);  // row_shr:1
    x += dpp_in<0x112, 0xF>(x);  // row_shr:2
    x += dpp_in<0x114, 0xF>(x);  // row_shr:4
    x += dpp_in<0x118, 0xF>(x);  // row_shr:8
    x += dpp_in<0x142, 0xA>(x);  // row_bcast:15 into rows 1 and 3
    x += dpp_in<0x143, 0xC>(x);  // row_bcast:31 into rows 2 and 3
    return x;
}

template <int LB, bool VB>
__global__ __launch_bounds__(64) void bzd_huff(Dec D)
{
    __shared__ uint16_t lut[kMaxGroups << LB];
    __shared__ int32_t slimit[kMaxGroups][kMaxLen + 2];
    __shared__ int32_t sbase[kMaxGroups][kMaxLen + 2];
    __shared__ uint16_t sperm[kMaxGroups][kMaxAlpha];
    __shared__ uint8_t slen[kMaxAlpha];
    __shared__ int scnt[kMaxLen + 2], sstart[kMaxLen + 2];
    // selectors in LDS, 8 per word (dynamic: sized for the batch's largest
    // block level; a uniform global load of what lane 0 just stored could be
    // served by the incoherent scalar cache)
    extern __shared__ uint32_t sel[];
    const uint32_t lane = threadIdx.x;
    const uint32_t s = blockIdx.x;
    uint32_t flag = 0;
    WaveBits br;
    const uint64_t b0 = D.offs[s], b1 = D.offs[s + 1];
    br.init(D.payload, b0, b1);
    uint8_t* ll = D.ll + (size_t)s * D.cap;
    uint32_t nblock = 0, origPtr = 0, bcrc = 0;
    uint32_t s2u = 0;  // seqToUnseq, entries 4 * lane .. 4 * lane + 3
    // LDS reads of wave-uniform values go through readfirstlane so that the
    // decode's control flow stays scalar
    auto U = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); };
    do {
        if (b1 - b0 < 14) { flag = kHost; break; }
        if (br.get(24) != 0x425A68u) { flag = kHost; break; }  // "BZh"
        const uint32_t lv = br.get(8);
        if (lv < '1' || lv > '9') { flag = kHost; break; }
        const uint32_t m1 = br.get(24), m2 = br.get(24);
        if (m1 != 0x314159u || m2 != 0x265359u) { flag = kHost; break; }  // no block (empty) or damaged
        bcrc = br.get(32);
        if (br.get(1)) { flag = kHost; break; }  // randomised block (bzip2 0.9.0 style)
        origPtr = br.get(24);
        // mapping table -> seqToUnseq
        const uint32_t in16 = br.get(16);
        uint32_t nInUse = 0;
        for (int i = 0; i < 16; ++i)
            if ((in16 >> (15 - i)) & 1u) {
                const uint32_t bits = br.get(16);
                for (int j = 0; j < 16; ++j)
                    if ((bits >> (15 - j)) & 1u) {
                        if ((nInUse >> 2) == lane) s2u |= (uint32_t)(i * 16 + j) << (8 * (nInUse & 3));
                        ++nInUse;
                    }
            }
        if (nInUse == 0) { flag = kHost; break; }
        const int alphaSize = (int)nInUse + 2;
        const int nGroups = (int)br.get(3);
        const uint32_t nSel = br.get(15);
        if (nGroups < 2 || nGroups > kMaxGroups || nSel < 1 || nSel > D.sel_cap) { flag = kHost; break; }
        {  // selectors: unary MTF values, then the inverse MTF
            uint32_t pos = 0x543210u, word = 0;
            for (uint32_t i = 0; i < nSel && !flag; ++i) {
                uint32_t j = 0;
                while (br.get(1)) {
                    if (++j >= (uint32_t)nGroups) { flag = kHost; break; }
                }
                const uint32_t v = (pos >> (4 * j)) & 15u;
                const uint32_t m = (1u << (4 * (j + 1))) - 1u;
                pos = (pos & ~m) | (((pos << 4) | v) & m);
                word |= v << (4 * (i & 7));
                if ((i & 7) == 7 || i + 1 == nSel) {
                    if (lane == 0) sel[i >> 3] = word;
                    word = 0;
                }
            }
            if (flag) break;
        }
        __syncthreads();
        // code lengths and decode tables (BZ2_hbCreateDecodeTables, restated)
        for (int t = 0; t < nGroups && !flag; ++t) {
            int curr = (int)br.get(5);
            int mn = 32, mx = 0;
            for (int i = 0; i < alphaSize; ++i) {
                while (true) {
                    if (curr < 1 || curr > kMaxLen) { flag = kHost; break; }
                    if (!br.get(1)) break;
                    curr += br.get(1) ? -1 : 1;
                }
                if (flag) break;
                if (lane == 0) slen[i] = (uint8_t)curr;
                mn = min(mn, curr);
                mx = max(mx, curr);
            }
            if (flag) break;
            __syncthreads();
            if (lane == 0) {
                for (int l = 0; l < kMaxLen + 2; ++l) scnt[l] = 0;
                for (int i = 0; i < alphaSize; ++i) ++scnt[slen[i]];
                int pp = 0;
                for (int l = 0; l < kMaxLen + 2; ++l) {
                    sstart[l] = pp;
                    pp += scnt[l];
                }
                for (int i = 0; i < alphaSize; ++i) sperm[t][sstart[slen[i]]++] = (uint16_t)i;
                int vec = 0, firstIdx = 0;
                for (int l = 0; l < kMaxLen + 2; ++l) {
                    if (l < mn || l > mx) {
                        slimit[t][l] = l < mn ? -1 : 0x7FFFFFFF;
                        sbase[t][l] = 0;
                        continue;
                    }
                    sbase[t][l] = vec - firstIdx;  // code vec has perm index firstIdx
                    vec += scnt[l];
                    firstIdx += scnt[l];
                    slimit[t][l] = vec - 1;
                    vec <<= 1;
                }
            }
            __syncthreads();
            // lookup table: entry = sym | length << 9 (length 0: a longer code)
            uint16_t* lt = lut + (t << LB);
            for (int e = lane; e < (1 << LB); e += 64) {
                uint16_t ent = 0;
                for (int l = mn; l <= min(mx, LB); ++l) {
                    const int c = e >> (LB - l);  // the first l bits of e
                    if (c <= slimit[t][l] && c > slimit[t][l] - scnt[l]) {
                        ent = (uint16_t)(sperm[t][c - sbase[t][l]] | (l << 9));
                        break;
                    }
                }
                lt[e] = ent;
            }
            __syncthreads();
        }
        if (flag) break;
        // symbols, a group at a time
        uint32_t mtfw = s2u;   // the move-to-front list, as output bytes, 4 per lane
        const uint32_t EOB = nInUse + 1;
        const uint32_t cap = D.cap;
        const uint64_t ltmask = (1ull << lane) - 1ull;
        const int kk0 = 1 - 4 * (int)lane;
        uint32_t rs = 0;       // digits of a run still open at the end of the previous group
        uint32_t g = 0;
        bool eob = false;
        LaneBits lb;
        if constexpr (VB) lb.from(br);
        while (!eob) {
            if (g >= nSel || (VB ? U((uint32_t)lb.over()) != 0 : br.over())) { flag = kHost; break; }
            const uint32_t tb = ((U(sel[g >> 3]) >> (4 * (g & 7))) & 15u) << LB;
            ++g;
            // 1. Huffman: symbol k of the group into lane k
            auto decode1 = [&]() -> uint32_t {
                const uint32_t e = U(lut[tb + br.peek(LB)]);
                uint32_t len = e >> 9;
                uint32_t sym = e & 511u;
                if (len == 0) {  // longer than LB bits: bzip2's limit walk
                    const uint32_t t = tb >> LB;
                    uint32_t zn = LB + 1;
                    int32_t zvec = (int32_t)br.peek(zn);
                    while (zn <= kMaxLen && zvec > (int32_t)U((uint32_t)slimit[t][zn])) {
                        ++zn;
                        zvec = (int32_t)br.peek(zn);
                    }
                    const int idx = zvec - (int32_t)U((uint32_t)sbase[t][min(zn, (uint32_t)kMaxLen)]);
                    if (zn > kMaxLen || idx < 0 || idx >= alphaSize) {
                        flag = kHost;
                        zn = 1;
                        sym = EOB;
                    } else {
                        sym = U(sperm[t][idx]);
                    }
                    len = zn;
                }
                br.skip(len);
                return sym;
            };
            // symv[lane G] = sym (sym and G are wave-uniform; lane select in m0)
            auto put = [](uint32_t& v, uint32_t sym, uint32_t G) {
                asm("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(v) : "s"(sym), "s"(G) : "m0");
            };
            // the same decode with the reader in vector registers (VB): the
            // symbol is a VGPR, equal in all lanes; a bad code marks the lane
            bool vbad = false;
            auto decode1v = [&]() -> uint32_t {
                const uint32_t e = lut[tb + lb.peek(LB)];
                uint32_t len = e >> 9;
                uint32_t sym = e & 511u;
                // a code longer than LB bits: a uniform (scalar) branch, see skip_u
                if (__builtin_amdgcn_readfirstlane((int)len) == 0) {
                    const uint32_t t = tb >> LB;
                    uint32_t zn = LB + 1;
                    int32_t zvec = (int32_t)lb.peek(zn);
                    while (zn <= kMaxLen && zvec > slimit[t][zn]) {
                        ++zn;
                        zvec = (int32_t)lb.peek(zn);
                    }
                    const int idx = zvec - sbase[t][min(zn, (uint32_t)kMaxLen)];
                    if (zn > kMaxLen || idx < 0 || idx >= alphaSize) {
                        vbad = true;
                        zn = 1;
                        sym = EOB;
                    } else {
                        sym = sperm[t][idx];
                    }
                    len = zn;
                }
                lb.skip_u(len);
                return sym;
            };
            uint32_t symv = 0, G = 0;
            if (g < nSel) {  // not the last group: 50 symbols, none of them EOB (libbzip2 writes
                             // one selector per group, EOB in the last; anything else -> host)
                if constexpr (VB) {
                    // 5 x 10 symbols: the lane compare against a constant, loop
                    // control once per 10 symbols
                    for (uint32_t G0 = 0; G0 < 50; G0 += 10) {
                        const uint32_t dl = lane - G0;
#pragma unroll
                        for (uint32_t u = 0; u < 10; ++u) {
                            const uint32_t sym = decode1v();
                            symv = dl == u ? sym : symv;
                        }
                    }
                    G = 50;
                } else {
                    for (G = 0; G < 50; ++G) put(symv, decode1(), G);
                }
                if (__ballot(lane < 50 && symv == EOB)) flag = kHost;
            } else {
                do {
                    uint32_t sym;
                    if constexpr (VB) {
                        sym = U(decode1v());
                        symv = lane == G ? sym : symv;
                    } else {
                        sym = decode1();
                        put(symv, sym, G);
                    }
                    ++G;
                    eob = sym == EOB;
                } while (G < 50 && !eob);
            }
            if (VB && __ballot(vbad)) flag = kHost;
            if (flag) break;
#if LFM_BZD_PROBE >= 3  // timing probe (wrong output): the symbol decode alone
            nblock = min(nblock + G, D.cap - 64);
            continue;
#endif
            // 2. runs and counts over the lanes
            const bool valid = lane < G;
            const bool isrun = valid && symv <= 1u;
            const bool isnorm = valid && symv > 1u && symv != EOB;
            const uint64_t below = ~__ballot(isrun) & ltmask;   // non-run lanes before this one
            const int p = 63 - (int)__clzll(below);             // the last of them, -1: none
            const uint32_t j = (uint32_t)((int)lane - p - 1) + (p < 0 ? rs : 0u);  // digit index in its run
            if (__ballot(isrun && j >= 21)) { flag = kHost; break; }  // run of 2^21 or more (decompress.c)
            const uint32_t cnt = isrun ? (symv + 1u) << j : (isnorm ? 1u : 0u);
            // the move-to-front chain over the group's ordinary symbols
            const uint32_t front0 = (uint32_t)__builtin_amdgcn_readlane((int)mtfw, 0) & 0xFFu;
            uint32_t outb = 0;
            // per-lane operands of the steps, worked out for all lanes at once
            // (each step reads its three by readlane): the list word and byte
            // shift of position nn = sym - 1, and 8 * nn for the entry mask
            const uint32_t nnv = symv - 1u;
            const uint32_t wiv = (nnv >> 2) & 63u, shv = 8u * (nnv & 3u), nn8v = 8u * nnv;
            const int kk08 = 8 * kk0;
#if LFM_BZD_PROBE >= 1  // timing probe (wrong output): no move-to-front chain
            outb = symv;
            for (uint64_t nm = 0; nm;) {
#else
            for (uint64_t nm = __ballot(isnorm); nm;) {
#endif
                const uint32_t k = (uint32_t)__builtin_ctzll(nm);
                asm("s_bitset0_b64 %0, %1" : "+s"(nm) : "s"(k));  // (one SALU op, not shift + and-not)
                const uint32_t wi = (uint32_t)__builtin_amdgcn_readlane((int)wiv, (int)k);
                const uint32_t sh = (uint32_t)__builtin_amdgcn_readlane((int)shv, (int)k);
                const int nn8 = __builtin_amdgcn_readlane((int)nn8v, (int)k);
                // v = list[nn] (the low byte of vw; the output keeps only that byte)
                const uint32_t vw = (uint32_t)__builtin_amdgcn_readlane((int)mtfw, (int)wi) >> sh;
                uint32_t v24;  // vw << 24 straight into a VGPR (the DPP's lane-0 value)
                asm("v_lshlrev_b32_e64 %0, 24, %1" : "=v"(v24) : "s"(vw));
                // move to front: entries 0 .. nn shift up by one, v goes to 0
                // lane l - 1's word (DPP wave_shr:1, a VALU op); lane 0 gets v << 24
                const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp((int)v24, (int)mtfw, 0x138, 0xF, 0xF, false);
                const uint32_t shf = __builtin_amdgcn_alignbit(mtfw, up, 24);  // (mtfw << 8) | (up >> 24)
                // this lane's entries above nn keep their place: the bytes from
                // 8 * clamp(nn + 1 - 4 * lane, 0, 4) up (all of them: 0, none: 32)
                const int t8 = min(32, max(0, nn8 + kk08));
                const uint32_t keep = (uint32_t)(~0ull << t8);
                mtfw = (mtfw & keep) | (shf & ~keep);
                // (lane select in m0: an SGPR source and an SGPR lane select
                // together exceed gfx9's one constant-bus read)
                asm("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(outb) : "s"(vw), "s"(k) : "m0");
            }
            outb &= 0xFFu;
            // a run repeats the list front: the byte of the last ordinary symbol before it
            const uint32_t fb = (uint32_t)__shfl((int)outb, max(p, 0));
            const uint32_t b = isrun ? (p < 0 ? front0 : fb) : outb;
            // 3. offsets (exclusive prefix sum of the counts) and the stores
            const uint32_t incl = wave_sum_incl(cnt);
            const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            if (nblock + total > cap) { flag = kHost; break; }
            const uint32_t at = nblock + incl - cnt;
#if LFM_BZD_PROBE >= 2  // timing probe (wrong output): no stores
            if (nblock > cap) 
#endif
            if (isnorm || (isrun && cnt <= 8u))
                for (uint32_t q = 0; q < cnt; ++q) ll[at + q] = (uint8_t)b;
            for (uint64_t big = __ballot(isrun && cnt > 8u); big; big &= big - 1) {  // long stretches: all lanes
                const int k = __builtin_ctzll(big);
                const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)at, k);
                const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cnt, k);
                const uint8_t bb = (uint8_t)__builtin_amdgcn_readlane((int)b, k);
                for (uint32_t q = lane; q < c; q += 64) ll[o + q] = bb;
            }
            nblock += total;
            rs = (uint32_t)__builtin_amdgcn_readlane((int)(isrun ? j + 1u : 0u), (int)(G - 1));
        }
        if (flag) break;
        if constexpr (VB) lb.to(br);
        if (origPtr >= nblock || nblock == 0) { flag = kHost; break; }
        // end of stream: exactly one block
        const uint32_t e1 = br.get(24), e2 = br.get(24);
        if (e1 != 0x177245u || e2 != 0x385090u) { flag = kHost; break; }
        const uint32_t ccrc = br.get(32);
        if (ccrc != bcrc) { flag = kHost; break; }  // one block: combined CRC = rotl(0, 1) ^ blockCRC
    } while (false);
#if LFM_BZD_PROBE
    if (flag) flag = kCrcFail;  // (never the host library: the probes' streams are not decoded)
#endif
    if (lane == 0) {
        D.flags[s] = flag;
        D.n[s] = flag ? 0u : nblock;
        D.orig[s] = origPtr;
        D.crc[s] = bcrc;
    }
}

// ------------------------------------------------------------ inverse BWT --
constexpr int kTtThreads = 256;

// ll is read 16 bytes per thread, a step ahead, with every load
// unconditional (clamped) and loop trip counts uniform: the byte-per-thread
// loads of a tile, each used right away, made all three passes wait one
// memory latency per 256 positions (ll and tt live in 256-aligned stream
// regions of cap bytes / words, so whole 16-byte chunks up to n stay inside)
template <int NT>
__global__ __launch_bounds__(NT) void bzd_tt(Dec D)
{
    constexpr uint32_t kBlk = 16u * NT;  // ll bytes per staged block (16 tiles)
    __shared__ uint32_t cf[256];       // C[c]: bytes < c
    __shared__ uint32_t run[256];      // occurrences of c before the current tile
    __shared__ uint32_t wc[NT / 64][256];
    __shared__ __attribute__((aligned(16))) uint8_t sll[kBlk];
    const uint32_t s = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (D.flags[s]) return;
    const uint32_t n = D.n[s];
    const uint8_t* ll = D.ll + (size_t)s * D.cap;
    uint32_t* tt = D.tt + (size_t)s * D.cap;
    const uint32_t nch = (n + 15u) / 16u;  // 16-byte chunks of ll
    auto ldc = [&](uint32_t ci) { return *(const uint4*)(ll + 16u * min(ci, nch ? nch - 1u : 0u)); };
    for (uint32_t c = t; c < 256; c += NT) {
        run[c] = 0;
        for (int w = 0; w < NT / 64; ++w) wc[w][c] = 0;
    }
    __syncthreads();
    {  // byte counts: chunk k * NT + t in step k, two chunk registers in turn
        const uint32_t K = (nch + NT - 1u) / NT;
        auto count = [&](const uint4& q, uint32_t ci) {
            if (ci < nch) {
                const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    if (16u * ci + j < n) atomicAdd(&run[(w[j >> 2] >> (8 * (j & 3))) & 0xFFu], 1u);
            }
        };
        uint4 qa = ldc(t), qb = ldc(NT + t);
        for (uint32_t k = 0; k < K; k += 2) {
            count(qa, k * NT + t);
            qa = ldc((k + 2) * NT + t);
            count(qb, (k + 1) * NT + t);
            qb = ldc((k + 3) * NT + t);
        }
    }
    __syncthreads();
    if (t < 64) {  // exclusive scan of the 256 counts, 4 per lane
        uint32_t v[4], sum = 0;
        for (int q = 0; q < 4; ++q) {
            v[q] = run[4 * t + q];
            sum += v[q];
        }
        uint32_t inc = sum;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(inc, d);
            if ((int)t >= d) inc += o;
        }
        uint32_t acc = inc - sum;
        for (int q = 0; q < 4; ++q) {
            cf[4 * t + q] = acc;
            acc += v[q];
        }
    }
    __syncthreads();
    for (uint32_t c = t; c < 256; c += NT) run[c] = 0;
    const uint64_t lt = (1ull << lane) - 1ull;
    // LF(i) = C[c] + Occ(c, i) in tiles of NT positions; ll staged in LDS a
    // block of 16 tiles at a time, the next block's chunk loaded meanwhile
    uint4 nb = ldc(t);
    for (uint32_t b0 = 0; b0 < n; b0 += kBlk) {
        __syncthreads();  // the previous block's tiles have read sll
        *(uint4*)(sll + 16u * t) = nb;
        nb = ldc((b0 + kBlk) / 16u + t);
        __syncthreads();
        for (uint32_t i0 = b0; i0 < min(n, b0 + kBlk); i0 += NT) {
            const uint32_t i = i0 + t;
            const bool ok = i < n;
            const uint32_t c = ok ? (uint32_t)sll[i - b0] : 256u;
            uint64_t mm = __ballot(ok);
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const uint64_t bb = __ballot(ok && ((c >> b) & 1u));
                mm &= ((c >> b) & 1u) ? bb : ~bb;
            }
            const uint32_t rw = (uint32_t)__popcll(mm & lt);
            const bool leader = ok && (mm & lt) == 0;
            if (leader) wc[wave][c] = (uint32_t)__popcll(mm);
            __syncthreads();
            uint32_t before = 0, total = 0;
            if (ok) {
                for (uint32_t w = 0; w < NT / 64; ++w) {
                    const uint32_t x = wc[w][c];
                    before += w < wave ? x : 0u;
                    total += x;
                }
                const uint32_t lf = cf[c] + run[c] + before + rw;
                tt[lf] = i;
            }
            __syncthreads();
            // the last occurrence of c in the tile advances the running count
            if (ok && before + rw + 1 == total) run[c] += total;
            if (leader) wc[wave][c] = 0;
            __syncthreads();
        }
    }
    __syncthreads();
    {  // decompress.c's fast tt: tt[j] = next << 8 | ll[j], 4 entries per thread
        const uint32_t ng = (n + 3u) / 4u, K = (ng + NT - 1u) / NT;
        auto ldg = [&](uint32_t g, uint4& v, uint32_t& b) {
            const uint32_t gc = min(g, ng ? ng - 1u : 0u);
            v = *(const uint4*)(tt + 4u * gc);
            b = *(const uint32_t*)(ll + 4u * gc);
        };
        auto put = [&](uint32_t g, const uint4& v, uint32_t b) {
            if (g < ng)
                *(uint4*)(tt + 4u * g) = make_uint4((v.x << 8) | (b & 0xFFu), (v.y << 8) | ((b >> 8) & 0xFFu),
                                                    (v.z << 8) | ((b >> 16) & 0xFFu), (v.w << 8) | (b >> 24));
        };
        uint4 va, vb;
        uint32_t ba, bb;
        ldg(t, va, ba);
        ldg(NT + t, vb, bb);
        for (uint32_t k = 0; k < K; k += 2) {
            put(k * NT + t, va, ba);
            ldg((k + 2) * NT + t, va, ba);
            put((k + 1) * NT + t, vb, bb);
            ldg((k + 3) * NT + t, vb, bb);
        }
    }
}

// marker id of node j (or ~0u): every kMark-th node, and the walk's start
__device__ __forceinline__ uint32_t marker_id(uint32_t j, uint32_t v0, uint32_t nm)
{
    if (j % kMark == 0) return j / kMark;
    return j == v0 ? nm : ~0u;
}

// LDSM: the marker tables (successor, length, output offset, restart node)
// live in LDS, so the one-lane chaining of the segments reads LDS instead of
// making ~1 150 dependent global round trips per stream
template <int NT, bool LDSM>
__global__ __launch_bounds__(NT) void bzd_walk(Dec D)
{
    extern __shared__ uint32_t wsm[];  // LDSM: 4 x mcap words
    __shared__ uint32_t s_total;
    const uint32_t s = blockIdx.x, t = threadIdx.x;
    if (D.flags[s]) return;
    const uint32_t n = D.n[s];
    const uint32_t* tt = D.tt + (size_t)s * D.cap;
    uint8_t* rle = D.rle + (size_t)s * D.cap;
    uint32_t* mnext = LDSM ? wsm : D.mnext + (size_t)s * D.mcap;
    uint32_t* mlen = LDSM ? wsm + D.mcap : D.mlen + (size_t)s * D.mcap;
    uint32_t* mstart = LDSM ? wsm + 2 * D.mcap : D.mstart + (size_t)s * D.mcap;
    uint32_t* mres = LDSM ? wsm + 3 * D.mcap : D.mres + (size_t)s * D.mcap;
    const uint32_t v0 = tt[D.orig[s]] >> 8;
    const uint32_t nm = (n + kMark - 1) / kMark;  // regular markers 0 .. nm-1, the start is nm
    const bool extra = (v0 % kMark) != 0;
    const uint32_t nwalk = nm + (extra ? 1u : 0u);
    auto node_of = [&](uint32_t id) { return id < nm ? id * kMark : v0; };
    uint8_t* keep = D.wkeep + (size_t)s * D.mcap * kWalkKeep;
    // pass 1: segment lengths and successors; the walker keeps the bytes it
    // passes (the low byte of each tt entry it reads) in dwords
    for (uint32_t id = t; id < nwalk; id += NT) {
        uint32_t pos = node_of(id), len = 0, nx = ~0u, acc = 0, res = 0;
        uint32_t* kp = (uint32_t*)(keep + (size_t)id * kWalkKeep);
        do {
            if (len == kWalkKeep) res = pos;
            const uint32_t e = tt[pos];
            if (len < kWalkKeep) {
                acc |= (e & 0xFFu) << (8 * (len & 3u));
                if ((len & 3u) == 3u) {
                    kp[len >> 2] = acc;
                    acc = 0;
                }
            }
            pos = e >> 8;
            ++len;
            nx = marker_id(pos, v0, nm);
        } while (nx == ~0u && len <= n);
        if (len < kWalkKeep && (len & 3u)) kp[len >> 2] = acc;
        mnext[id] = nx;
        mlen[id] = len;
        mres[id] = res;
    }
    __syncthreads();
    // chain the segments from the start (one lane)
    if (t == 0) {
        uint32_t id = extra ? nm : v0 / kMark, off = 0, k = 0;
        while (k < nwalk && off < n) {
            mstart[id] = off;
            off += mlen[id];
            id = mnext[id];
            ++k;
        }
        s_total = off == n && k == nwalk ? 1u : 0u;
    }
    __syncthreads();
    if (!s_total) {
        if (t == 0) D.flags[s] = kHost;  // not one cycle: not a valid bzip2 block
        return;
    }
    // pass 2: the kept bytes into place, one wave per segment
    const uint32_t lane = t & 63, wave = t >> 6;
    for (uint32_t id = wave; id < nwalk; id += NT / 64) {
        const uint32_t o = mstart[id], m = min(mlen[id], kWalkKeep);
        const uint8_t* src = keep + (size_t)id * kWalkKeep;
        for (uint32_t k = lane; k < m; k += 64) rle[o + k] = src[k];
    }
    // segments longer than kWalkKeep: walk on from where their walker stopped keeping
    for (uint32_t id = t; id < nwalk; id += NT) {
        const uint32_t len = mlen[id];
        if (len <= kWalkKeep) continue;
        uint32_t pos = mres[id], o = mstart[id] + kWalkKeep;
        for (uint32_t k = kWalkKeep; k < len; ++k) {
            const uint32_t e = tt[pos];
            rle[o++] = (uint8_t)e;
            pos = e >> 8;
        }
    }
}

// -------------------------------------------------------------------- RLE1 --
// One wave per stream.  RLE1 decoding is a 5-state machine over the text
// (state = equal bytes seen, 0 right after a count byte; in state 4 the byte
// is a count: it repeats the previous byte that many times), so the text is
// cut into 64 lane segments (16-byte aligned) and decoded in three steps:
//  A  every lane runs its segment from all five start states at once (the
//     paths meet after a few bytes in any real stream, then one path runs
//     alone) and keeps, per start state, the end state and the output length;
//  B  one uniform pass over the 64 lanes chains them: each lane's start state
//     and output offset;
//  C  every lane decodes its segment again, writing its bytes at its offset.
// The block CRC then runs over the output in 64 equal segments aligned to its
// end (leading zero bytes do not change a zero-initialised CRC), combined in
// a 6-level tree: crc(L || R) = crc(L) * x^(8|R|) mod P ^ crc(R).
__constant__ uint32_t c_xpow[24];  // x^(8 * 2^k) mod P

// a(x) * b(x) mod P, MSB-first CRC-32 polynomials (P = x^32 + 0x04C11DB7)
__device__ __forceinline__ uint32_t crc_mulmod(uint32_t a, uint32_t b)
{
    uint32_t r = 0;
#pragma unroll
    for (int i = 31; i >= 0; --i) {
        r = (r << 1) ^ ((r >> 31) ? 0x04C11DB7u : 0u);
        r ^= ((b >> i) & 1u) ? a : 0u;
    }
    return r;
}

// x^(8 L) mod P: the CRC shift over L zero bytes
__device__ __forceinline__ uint32_t crc_xpow8(uint32_t L)
{
    uint32_t r = 1u;  // x^0
    for (int k = 0; k < 24 && L; ++k, L >>= 1)
        if (L & 1u) r = crc_mulmod(r, c_xpow[k]);
    return r;
}

constexpr int kRleSeg = 16;  // segment alignment (bytes)

// per-lane sequential reader of the RLE1 text, 16 bytes at a time.  The load
// is unconditional (clamped address, zeros selected past the end): a load
// under a branch, or a chunk moved between registers while its load is in
// flight, made the compiler wait for it right away.
struct TextChunks {
    const uint8_t* p;
    uint32_t cap;
    __device__ __forceinline__ uint4 load(uint32_t at) const
    {
        const uint4 v = *(const uint4*)(p + min(at, cap - 16u));
        return at < cap ? v : uint4{0u, 0u, 0u, 0u};
    }
};

// visit this lane's 16-byte chunks at a, a + 16, ... while < b, with four
// chunk registers in rotation, each reloaded three chunks ahead of its use.
// The loop runs the wave's largest chunk count (a lane past its own end
// skips f but keeps loading, clamped): no divergent exit and no chunk moved
// between registers, so the compiler can count its waits.
template <typename Ld, typename F>
__device__ __forceinline__ void for_chunks4(uint32_t a, uint32_t b, Ld&& ld, F&& f)
{
    const uint32_t nc = b > a ? (b - a + 15u) / 16u : 0u;
    uint32_t N = nc;
    for (int d = 32; d > 0; d >>= 1) N = max(N, (uint32_t)__shfl_xor((int)N, d));
    N = (uint32_t)__builtin_amdgcn_readfirstlane((int)N);
    uint4 q0 = ld(a), q1 = ld(a + 16), q2 = ld(a + 32), q3 = ld(a + 48);
    for (uint32_t k = 0; k < N; k += 4) {
        const uint32_t i = a + 16u * k;
        if (k < nc) f(q0, i);
        q0 = ld(i + 64);
        if (k + 1 < nc) f(q1, i + 16);
        q1 = ld(i + 80);
        if (k + 2 < nc) f(q2, i + 32);
        q2 = ld(i + 96);
        if (k + 3 < nc) f(q3, i + 48);
        q3 = ld(i + 112);
    }
}

__device__ __forceinline__ uint32_t chunk_byte(const uint4& q, int j)  // j compile-time after unrolling
{
    const uint32_t w = j < 4 ? q.x : j < 8 ? q.y : j < 12 ? q.z : q.w;
    return (w >> (8 * (j & 3))) & 0xFFu;
}

__global__ __launch_bounds__(64) void bzd_rle1(Dec D)
{
    __shared__ uint32_t T1[256];
    __shared__ uint32_t smap[64], scnt[5][64], sst[64], soff[64];
    __shared__ uint32_t s_total;
    const uint32_t lane = threadIdx.x, s = blockIdx.x;
    for (uint32_t i = lane; i < 256; i += 64) T1[i] = c_dcrc[i];
    if (D.flags[s]) {
        if (lane == 0) D.out_len[s] = 0;
        return;
    }
    const uint32_t n = D.n[s];
    const uint8_t* rle = D.rle + (size_t)s * D.cap;
    uint8_t* out = D.out + (size_t)s * D.out_stride;
    const uint32_t cap = D.out_stride;
    const TextChunks tx{rle, D.cap};
    const uint32_t seg = ((n + 63) / 64 + kRleSeg - 1) / kRleSeg * kRleSeg;
    const uint32_t a = min(n, lane * seg), b = min(n, a + seg);
    const uint32_t before = a ? (uint32_t)rle[a - 1] : 256u;  // the text byte before the segment
    // A: all five start states until their paths meet, then one path
    {
        uint32_t st[5] = {0, 1, 2, 3, 4}, cnt[5] = {0, 0, 0, 0, 0};
        uint32_t prevb = before, s1 = 0, c1 = 0;
        bool met = false;
        for_chunks4(a, b, [&](uint32_t at) { return tx.load(at); }, [&](const uint4& q, uint32_t i) {
            if (!met) {
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    if (i + j < b) {
                        const uint32_t c = chunk_byte(q, j);
                        const bool eq = c == prevb;
#pragma unroll
                        for (int p = 0; p < 5; ++p) {
                            const bool c4 = st[p] == 4;
                            cnt[p] += c4 ? c : 1u;
                            st[p] = c4 ? 0u : ((st[p] == 0 || !eq) ? 1u : st[p] + 1u);
                        }
                        prevb = c;
                    }
                }
                met = st[0] == st[1] && st[0] == st[2] && st[0] == st[3] && st[0] == st[4];
                s1 = st[0];
            } else {
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    if (i + j < b) {
                        const uint32_t c = chunk_byte(q, j);
                        const bool c4 = s1 == 4;
                        c1 += c4 ? c : 1u;
                        s1 = c4 ? 0u : ((s1 == 0 || c != prevb) ? 1u : s1 + 1u);
                        prevb = c;
                    }
                }
            }
        });
        uint32_t map = 0;
#pragma unroll
        for (int p = 0; p < 5; ++p) {
            map |= (met ? s1 : st[p]) << (3 * p);
            scnt[p][lane] = cnt[p] + c1;
        }
        smap[lane] = map;
    }
    __syncthreads();
    // B: chain the lanes
    if (lane == 0) {
        uint32_t stt = 0, off = 0;
        for (uint32_t l = 0; l < 64; ++l) {
            sst[l] = stt;
            soff[l] = off;
            off += scnt[stt][l];
            stt = (smap[l] >> (3 * stt)) & 7u;
        }
        s_total = off;
    }
    __syncthreads();
    const uint32_t tot = s_total;
    if (tot > cap) {
        if (lane == 0) {
            D.out_len[s] = tot;
            D.flags[s] = kHost;
        }
        return;
    }
    // C: decode the segment from its start state.  Whole aligned 16-byte
    // pieces of the lane's output leave as one store each (byte stores made
    // every store instruction touch 64 scattered lines); the partial pieces at
    // the ends, shared with the neighbouring lanes, go byte by byte.
    {
        uint32_t s1 = sst[lane], o = soff[lane], prevb = before;
        const uint32_t oend = lane < 63 ? soff[lane + 1] : tot;
        // pieces are aligned in memory: po = o + (out's address mod 16)
        const uint32_t ab = (uint32_t)((uintptr_t)out & 15u);
        const uint32_t hbeg = min(((o + ab + 15) & ~15u) - ab, oend);
        const uint32_t tbeg = max(((oend + ab) & ~15u) - ab, hbeg);
        uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;  // the piece holding o
        auto put = [&](uint32_t c) {
            if (o < hbeg || o >= tbeg) {
                out[o] = (uint8_t)c;
            } else {
                const uint32_t po = o + ab;
                const uint32_t k = (po >> 2) & 3u, v = c << (8 * (po & 3u));
                a0 |= k == 0 ? v : 0u;
                a1 |= k == 1 ? v : 0u;
                a2 |= k == 2 ? v : 0u;
                a3 |= k == 3 ? v : 0u;
                if ((po & 15u) == 15u) {
                    *(uint4*)(out + (o - 15)) = make_uint4(a0, a1, a2, a3);
                    a0 = a1 = a2 = a3 = 0;
                }
            }
            ++o;
        };
        for_chunks4(a, b, [&](uint32_t at) { return tx.load(at); }, [&](const uint4& q, uint32_t i) {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                if (i + j < b) {
                    const uint32_t c = chunk_byte(q, j);
                    if (s1 == 4) {  // count byte: c more copies of the previous byte
                        for (uint32_t k = 0; k < c; ++k) put(prevb);
                        s1 = 0;
                    } else {
                        put(c);
                        s1 = (s1 == 0 || c != prevb) ? 1u : s1 + 1u;
                    }
                    prevb = c;
                }
            }
        });
    }
    // the other lanes' bytes are read back below (same wave, L1 write-through)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    __syncthreads();
    // CRC: 64 segments of segc bytes aligned to the end of the output
    const uint32_t segc = (tot + 63) / 64;
    const int64_t e = (int64_t)tot - (int64_t)(63 - lane) * segc;
    const uint32_t c0 = (uint32_t)max<int64_t>(0, e - (int64_t)segc), c1 = (uint32_t)max<int64_t>(0, e);
    uint32_t r = 0;
    if (c1 > c0) {  // aligned 16-byte chunks (a chunk holding a valid byte lies in its page)
        const uintptr_t u0 = (uintptr_t)(out + c0), u1 = (uintptr_t)(out + c1);
        const uintptr_t first = u0 & ~(uintptr_t)15, last = (u1 - 1) & ~(uintptr_t)15;
        const uint32_t nb = (uint32_t)(last - first) + 16u;  // bytes of the chunks
        auto ld = [&](uint32_t at) { return *(const uint4*)(first + min((uintptr_t)at, last - first)); };
        const uint32_t lo = (uint32_t)(u0 - first), hi = (uint32_t)(u1 - first);
        for_chunks4(0u, nb, ld, [&](const uint4& q, uint32_t i) {
#pragma unroll
            for (int j = 0; j < 16; ++j)
                if (i + j >= lo && i + j < hi) r = (r << 8) ^ T1[(r >> 24) ^ chunk_byte(q, j)];
        });
    }
    uint32_t X = crc_xpow8(segc);  // wave-uniform
    for (int j = 0; j < 6; ++j) {
        const uint32_t left = __shfl_up(r, 1u << j);
        if (((lane + 1) & ((2u << j) - 1)) == 0) r = crc_mulmod(left, X) ^ r;
        X = crc_mulmod(X, X);
    }
    if (lane == 63) {
        const uint32_t crc = ~(crc_mulmod(0xFFFFFFFFu, crc_xpow8(tot)) ^ r);
        D.out_len[s] = tot;
        if (crc != D.crc[s]) D.flags[s] = kCrcFail;
    }
}

} // namespace bzd
} // namespace lfm

using namespace lfm::bzd;

namespace {

size_t al(size_t v) { return (v + 255) / 256 * 256; }

uint32_t dec_cap(uint32_t out_stride)
{
    // a .lfm block of B bytes is compressed at level min(9, ceil(B / 1e5))
    // (klb_imageIO.cpp:108): its RLE1 block is at most 100000 * level bytes
    const uint32_t level = std::min<uint32_t>(9, std::max<uint32_t>(1, (out_stride + 99999) / 100000));
    return (uint32_t)al(100000u * level + 64);
}

uint32_t mark_cap(uint32_t cap) { return (cap + kMark - 1) / kMark + 2; }

uint32_t host_dcrc[256];
uint32_t host_xpow[24];
bool dcrc_ready = false;

} // namespace

extern "C" size_t lfm_hip_bunzip2_workspace_bytes(uint32_t count, uint32_t out_stride)
{
    const size_t cap = dec_cap(out_stride), mc = mark_cap((uint32_t)cap);
    size_t b = 0;
    b += al(((size_t)count + 1) * 8);
    b += al((size_t)count * cap);          // ll, then the RLE1 text (ll is dead once tt holds its bytes)
    b += al((size_t)count * cap * 4);      // tt
    b += 4 * al((size_t)count * mc * 4);
    b += al((size_t)count * mc * kWalkKeep);  // walkers' kept bytes
    b += 6 * al((size_t)count * 4 + 64);
    return b;
}

// Decode streams [0, count) of the device payload (byte ranges h_offs[i] ..
// h_offs[i + 1]; the payload buffer must be 4-byte aligned and readable 8 bytes
// past its end) into d_out + i * out_stride.  h_lens[i] = decoded bytes,
// h_flags[i]: 0 ok, 1 decode with the host library, 2 CRC mismatch.
extern "C" int lfm_hip_bunzip2_blocks(const void* d_payload, const uint64_t* h_offs, uint32_t count, void* d_out,
                                      uint32_t out_stride, void* d_ws, size_t ws_bytes, uint32_t* h_lens,
                                      uint32_t* h_flags, void* stream_)
{
    const int rc = lfm_hip_bunzip2_issue(d_payload, h_offs, count, d_out, out_stride, d_ws, ws_bytes, h_lens, h_flags,
                                         stream_);
    if (rc != LFM_HIP_OK) return rc;
    return hipStreamSynchronize((hipStream_t)stream_) == hipSuccess ? LFM_HIP_OK : LFM_HIP_ERUNTIME;
}

// the same, returning once the kernels and the copies of h_lens / h_flags
// (pinned host memory: the copies are asynchronous) are queued on the stream
extern "C" int lfm_hip_bunzip2_issue(const void* d_payload, const uint64_t* h_offs, uint32_t count, void* d_out,
                                     uint32_t out_stride, void* d_ws, size_t ws_bytes, uint32_t* h_lens,
                                     uint32_t* h_flags, void* stream_)
{
    hipStream_t st = (hipStream_t)stream_;
    if (!d_payload || !h_offs || !count || !d_out || !out_stride || !d_ws) return LFM_HIP_EINVAL;
    if (ws_bytes < lfm_hip_bunzip2_workspace_bytes(count, out_stride) || ((uintptr_t)d_payload & 3)) return LFM_HIP_EINVAL;
    if (!dcrc_ready) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i << 24;
            for (int k = 0; k < 8; ++k) c = (c & 0x80000000u) ? (c << 1) ^ 0x04c11db7u : (c << 1);
            host_dcrc[i] = c;
        }
        auto mulmod = [](uint32_t x, uint32_t y) {
            uint32_t r = 0;
            for (int i = 31; i >= 0; --i) {
                r = (r << 1) ^ ((r >> 31) ? 0x04C11DB7u : 0u);
                if ((y >> i) & 1u) r ^= x;
            }
            return r;
        };
        host_xpow[0] = 0x100u;  // x^8
        for (int k = 1; k < 24; ++k) host_xpow[k] = mulmod(host_xpow[k - 1], host_xpow[k - 1]);
        dcrc_ready = true;
    }
    static thread_local int crc_dev = -1;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (crc_dev != dev) {
        if (hipMemcpyToSymbol(HIP_SYMBOL(c_dcrc), host_dcrc, sizeof(host_dcrc)) != hipSuccess ||
            hipMemcpyToSymbol(HIP_SYMBOL(c_xpow), host_xpow, sizeof(host_xpow)) != hipSuccess)
            return LFM_HIP_ERUNTIME;
        crc_dev = dev;
    }
    Dec D{};
    D.payload = (const uint8_t*)d_payload;
    D.count = count;
    D.cap = dec_cap(out_stride);
    D.mcap = mark_cap(D.cap);
    D.out_stride = out_stride;
    D.out = (uint8_t*)d_out;
    uint8_t* p = (uint8_t*)d_ws;
    auto take = [&](size_t bytes) { uint8_t* r = p; p += al(bytes); return r; };
    uint64_t* d_offs = (uint64_t*)take(((size_t)count + 1) * 8);
    D.offs = d_offs;
    D.ll = take((size_t)count * D.cap);
    D.tt = (uint32_t*)take((size_t)count * D.cap * 4);
    D.rle = D.ll;  // bzd_walk writes the text over ll (bzd_tt copied ll into tt)
    D.mnext = (uint32_t*)take((size_t)count * D.mcap * 4);
    D.mlen = (uint32_t*)take((size_t)count * D.mcap * 4);
    D.mstart = (uint32_t*)take((size_t)count * D.mcap * 4);
    D.mres = (uint32_t*)take((size_t)count * D.mcap * 4);
    D.wkeep = take((size_t)count * D.mcap * kWalkKeep);
    uint32_t** small[] = {&D.n, &D.orig, &D.crc, &D.flags, &D.out_len};
    for (uint32_t** q : small) *q = (uint32_t*)take((size_t)count * 4 + 64);
    (void)take((size_t)count * 4 + 64);
    if (hipMemcpyAsync(d_offs, h_offs, ((size_t)count + 1) * 8, hipMemcpyHostToDevice, st) != hipSuccess)
        return LFM_HIP_ERUNTIME;
    D.sel_cap = std::min<uint32_t>(kMaxSel, (D.cap + 49) / 50 + 64);
    const size_t sel_lds = ((D.sel_cap + 7) / 8 * 4 + 15) & ~(size_t)15;
    // (9- / 10-bit lookup tables and a wave-uniform scalar bit reader measured slower)
    hipLaunchKernelGGL((bzd_huff<8, true>), dim3(count), dim3(64), sel_lds, st, D);
    hipLaunchKernelGGL(bzd_tt<kTtThreads>, dim3(count), dim3(kTtThreads), 0, st, D);
    // inverse-BWT walk, 512 threads per stream, the marker tables in LDS
    // (large blocks, level 5 and up, keep them in global memory: LDS for ~2
    // workgroups per CU at most)
    const size_t wl = (size_t)D.mcap * 16;
    if (wl <= 48 * 1024) hipLaunchKernelGGL((bzd_walk<512, true>), dim3(count), dim3(512), wl, st, D);
    else hipLaunchKernelGGL((bzd_walk<512, false>), dim3(count), dim3(512), 0, st, D);
    hipLaunchKernelGGL(bzd_rle1, dim3(count), dim3(64), 0, st, D);
    if (hipGetLastError() != hipSuccess) return LFM_HIP_ERUNTIME;
    if (hipMemcpyAsync(h_lens, D.out_len, (size_t)count * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(h_flags, D.flags, (size_t)count * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
        return LFM_HIP_ERUNTIME;
    return LFM_HIP_OK;
}

// ------------------------------------------------------------ block scatter --
namespace lfm {
namespace bzd {

struct Grid5 {
    uint32_t dims[5], bs[5], nb[5], bpp;
};

// decoded blocks (x fastest, then y, z, c, t: the writer's gather order,
// klb_imageIO.cpp:133-140) back into the image
__global__ __launch_bounds__(256) void scatter_blocks(const uint8_t* __restrict__ blocks, uint32_t stride, Grid5 G,
                                                      uint32_t first, uint8_t* __restrict__ img)
{
    const uint32_t s = blockIdx.y;
    uint32_t org[5], sz[5], id = first + s;
#pragma unroll
    for (int d = 0; d < 5; ++d) {
        const uint32_t q = id % G.nb[d];
        id /= G.nb[d];
        org[d] = q * G.bs[d];
        sz[d] = min(G.bs[d], G.dims[d] - org[d]);
    }
    const uint32_t rowb = sz[0] * G.bpp;
    const uint32_t nrows = sz[1] * sz[2] * sz[3] * sz[4];
    const uint8_t* src = blocks + (size_t)s * stride;
    for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
        uint32_t q = r;
        const uint32_t y = q % sz[1]; q /= sz[1];
        const uint32_t z = q % sz[2]; q /= sz[2];
        const uint32_t c = q % sz[3]; q /= sz[3];
        const size_t dst = ((((size_t)(org[4] + q) * G.dims[3] + (org[3] + c)) * G.dims[2] + (org[2] + z)) *
                                G.dims[1] + (org[1] + y)) * G.dims[0] + org[0];
        uint8_t* dp = img + dst * G.bpp;
        const uint8_t* sp = src + (size_t)r * rowb;
        for (uint32_t i = threadIdx.x; i < rowb; i += blockDim.x) dp[i] = sp[i];
    }
}

// the same with 16-byte copies: rows of a multiple of 16 bytes, 16-byte
// aligned in both the block buffer and the image (checked by the launcher);
// thread t of the grid's x dimension takes 16-byte units t, t + stride, ...
// of the block's rows
__global__ __launch_bounds__(256) void scatter_blocks16(const uint8_t* __restrict__ blocks, uint32_t stride, Grid5 G,
                                                        uint32_t first, uint8_t* __restrict__ img)
{
    const uint32_t s = blockIdx.y;
    uint32_t org[5], sz[5], id = first + s;
#pragma unroll
    for (int d = 0; d < 5; ++d) {
        const uint32_t q = id % G.nb[d];
        id /= G.nb[d];
        org[d] = q * G.bs[d];
        sz[d] = min(G.bs[d], G.dims[d] - org[d]);
    }
    const uint32_t upr = sz[0] * G.bpp / 16;  // units per row
    const uint32_t nu = upr * sz[1] * sz[2] * sz[3] * sz[4];
    const uint4* src = (const uint4*)(blocks + (size_t)s * stride);
    for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < nu; u += gridDim.x * blockDim.x) {
        uint32_t q = u / upr;
        const uint32_t c = u - q * upr;
        const uint32_t y = q % sz[1]; q /= sz[1];
        const uint32_t z = q % sz[2]; q /= sz[2];
        const uint32_t cc = q % sz[3]; q /= sz[3];
        const size_t dst = ((((size_t)(org[4] + q) * G.dims[3] + (org[3] + cc)) * G.dims[2] + (org[2] + z)) *
                                G.dims[1] + (org[1] + y)) * G.dims[0] + org[0];
        *((uint4*)(img + dst * G.bpp) + c) = src[u];
    }
}

} // namespace bzd
} // namespace lfm

extern "C" int lfm_hip_scatter_blocks(const void* d_blocks, uint32_t stride, uint32_t first, uint32_t count,
                                      const uint32_t dims[5], const uint32_t bs[5], uint32_t bpp, void* d_img,
                                      void* stream_)
{
    if (!d_blocks || !d_img || !count || !bpp) return LFM_HIP_EINVAL;
    lfm::bzd::Grid5 G;
    for (int d = 0; d < 5; ++d) {
        if (!dims[d] || !bs[d]) return LFM_HIP_EINVAL;
        G.dims[d] = dims[d];
        G.bs[d] = bs[d];
        G.nb[d] = (dims[d] + bs[d] - 1) / bs[d];
    }
    G.bpp = bpp;
    // 16-byte units when every row of every block is a whole number of aligned
    // units on both sides (the last block of a ragged dimension included)
    bool v16 = ((uintptr_t)d_blocks & 15) == 0 && ((uintptr_t)d_img & 15) == 0 && stride % 16 == 0 &&
               ((size_t)dims[0] * bpp) % 16 == 0 && ((size_t)bs[0] * bpp) % 16 == 0;
    if (v16 && dims[0] % bs[0]) v16 = ((size_t)(dims[0] % bs[0]) * bpp) % 16 == 0;
    if (v16)
        hipLaunchKernelGGL(lfm::bzd::scatter_blocks16, dim3(8, count), dim3(256), 0, (hipStream_t)stream_,
                           (const uint8_t*)d_blocks, stride, G, first, (uint8_t*)d_img);
    else
        hipLaunchKernelGGL(lfm::bzd::scatter_blocks, dim3(64, count), dim3(256), 0, (hipStream_t)stream_,
                           (const uint8_t*)d_blocks, stride, G, first, (uint8_t*)d_img);
    return hipGetLastError() == hipSuccess ? LFM_HIP_OK : LFM_HIP_ERUNTIME;
}
