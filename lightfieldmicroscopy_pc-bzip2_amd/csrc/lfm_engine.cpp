// lfm_engine.cpp -- MI355X-native encode / decode engine.
//
// Encode = predictor stage (GPU, lfm_hip.h) + block compression (host worker
// pool, in-order sink).  The reference equivalents:
//   writeImage               klb_imageIO.cpp:2248-2492
//   predictor selection      :2273-2360 (8 candidates on frame 0, argmin)
//   Predictor_both/_angle/_space :1227-1670 (one launch + 2 PCIe copies per frame)
//   blockCompressor          :78-295    (x-fastest gather, BZ2 level rule, workFactor 30)
//   blockWriter              :1145-1225 (in-order append, offset table rewritten at the end)
// Here the whole stack is predicted by one kernel launch per (c,t) volume,
// symbols come back with one D2H copy into pinned memory, and the block
// compressors run on all host cores while the calling thread appends the
// finished blocks in order.
#include "lfm_engine.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <sys/mman.h>
#include <unistd.h>
#include <zlib.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include "bz2_sys.h"
#include "lfm_cases.h"
#include "lfm_hip.h"

namespace lfm {

namespace {
using clk = std::chrono::steady_clock;
double ms_since(clk::time_point t0) { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); }

int env_int(const char* name, int dflt)
{
    const char* e = getenv(name);
    if (!e || !*e) return dflt;
    return atoi(e);
}

std::atomic<int> g_family{-1};
} // namespace

int default_threads()
{
    int n = env_int("LFM_NUM_THREADS", 0);
    if (n <= 0) n = env_int("OMP_NUM_THREADS", 0);
    if (n <= 0) n = (int)std::thread::hardware_concurrency();
    return std::max(n, 1);
}

int current_family()
{
    int f = g_family.load();
    if (f < 0) {
        f = env_int("LFM_PREDICTOR_WAY", LFM_PREDICTOR_WAY);
        if (f < 0 || f > 2) f = LFM_PREDICTOR_WAY;
        g_family.store(f);
    }
    return f;
}
void set_family(int fam) { g_family.store(fam); }

// ------------------------------------------------------------- block grid --
BlockGrid::BlockGrid(const klb_image_header& h)
{
    nblocks = 1;
    uint64_t s = 1;
    for (int d = 0; d < 5; ++d) {
        dims[d] = h.xyzct[d];
        bs[d] = h.blockSize[d];
        nb[d] = (uint64_t)std::ceil((float)h.xyzct[d] / (float)h.blockSize[d]);  // calculateNumBlocks
        nblocks *= nb[d];
        stride[d] = s;
        s *= dims[d];
    }
}

void BlockGrid::block(uint64_t id, uint64_t origin[5], uint64_t size[5]) const
{
    for (int d = 0; d < 5; ++d) {
        const uint64_t c = id % nb[d];
        id /= nb[d];
        origin[d] = c * bs[d];
        size[d] = std::min<uint64_t>(bs[d], dims[d] - origin[d]);
    }
}

template <bool GATHER>
static void walk_block(uint8_t* img, const BlockGrid& g, uint64_t id, size_t bpp, uint8_t* blk, size_t* nbytes)
{
    uint64_t o[5], s[5];
    g.block(id, o, s);
    const size_t row = s[0] * bpp;
    size_t k = 0;
    for (uint64_t t = 0; t < s[4]; ++t)
        for (uint64_t c = 0; c < s[3]; ++c)
            for (uint64_t z = 0; z < s[2]; ++z)
                for (uint64_t y = 0; y < s[1]; ++y) {
                    const uint64_t e = (o[0]) * g.stride[0] + (o[1] + y) * g.stride[1] + (o[2] + z) * g.stride[2] +
                                       (o[3] + c) * g.stride[3] + (o[4] + t) * g.stride[4];
                    if (GATHER) std::memcpy(blk + k, img + e * bpp, row);
                    else std::memcpy(img + e * bpp, blk + k, row);
                    k += row;
                }
    if (nbytes) *nbytes = k;
}

void gather_block(const uint8_t* img, const BlockGrid& g, uint64_t id, size_t bpp, uint8_t* dst, size_t* nbytes)
{
    walk_block<true>(const_cast<uint8_t*>(img), g, id, bpp, dst, nbytes);
}
void scatter_block(const uint8_t* blk, const BlockGrid& g, uint64_t id, size_t bpp, uint8_t* img)
{
    walk_block<false>(img, g, id, bpp, const_cast<uint8_t*>(blk), nullptr);
}

// ------------------------------------------------------------------ sinks --
int FileSink::begin(const klb_image_header& h)
{
    vbuf_.resize(32 << 20);
    setvbuf(f_, vbuf_.data(), _IOFBF, vbuf_.size());
    std::vector<uint8_t> head(h.getSizeInBytes(), 0);
    klb_image_header tmp(h);
    std::fill(tmp.blockOffset, tmp.blockOffset + tmp.Nb, 0);
    tmp.serialize(head.data(), head.size());
    return std::fwrite(head.data(), 1, head.size(), f_) == head.size() ? 0 : 5;
}
int FileSink::append(const uint8_t* p, size_t n)
{
    return std::fwrite(p, 1, n, f_) == n ? 0 : 5;
}
int FileSink::finish(const klb_image_header& h)
{
    if (std::fseek(f_, (long)h.getSizeInBytesFixPortion(), SEEK_SET) != 0) return 5;
    if (h.Nb && std::fwrite(h.blockOffset, sizeof(uint64_t), h.Nb, f_) != h.Nb) return 5;
    std::fflush(f_);
    return 0;
}

PinnedBuffer::~PinnedBuffer()
{
    if (p_ && malloced_) std::free(p_);
    else if (p_) (void)hipHostFree(p_);
}
bool PinnedBuffer::reserve(size_t n)
{
    if (n <= cap_) return true;
    const size_t cap = std::max(n, cap_ + cap_ / 2);
    void* q = nullptr;
    if (hipHostMalloc(&q, cap, hipHostMallocDefault) != hipSuccess) {
        // no HIP runtime (CPU-only paths): plain memory
        (void)hipGetLastError();
        q = std::malloc(cap);
        if (!q) return false;
        if (p_ && size_) std::memcpy(q, p_, size_);
        if (p_ && malloced_) std::free(p_);
        else if (p_) (void)hipHostFree(p_);
        p_ = (uint8_t*)q;
        cap_ = cap;
        malloced_ = true;
        return true;
    }
    if (p_ && size_) par_memcpy(q, p_, size_, default_threads());
    if (p_) {
        if (malloced_) std::free(p_);
        else (void)hipHostFree(p_);
    }
    p_ = (uint8_t*)q;
    cap_ = cap;
    malloced_ = false;
    return true;
}
bool PinnedBuffer::resize(size_t n)
{
    if (!reserve(n)) return false;
    size_ = n;
    return true;
}

int MemSink::begin(const klb_image_header& h)
{
    out_->clear();
    if (!out_->resize(h.getSizeInBytes())) return 3;
    std::memset(out_->data(), 0, out_->size());
    return 0;
}
int MemSink::append(const uint8_t* p, size_t n)
{
    uint8_t* d = direct(n);
    if (!d) return 3;
    std::memcpy(d, p, n);
    return 0;
}
uint8_t* MemSink::direct(size_t n)
{
    const size_t at = out_->size();
    // grow once to the worst case; if that reservation fails, the plain
    // resize below still grows by what this append needs
    if (at + n > out_->capacity() && worst_ > at + n) (void)out_->reserve(worst_);
    if (!out_->resize(at + n)) return nullptr;
    return out_->data() + at;
}
int MemSink::finish(const klb_image_header& h)
{
    h.serialize(out_->data(), h.getSizeInBytes());
    return 0;
}

// ------------------------------------------------------------ SDMA copies --
// Device -> pinned host copies of the compressed payload on a system DMA
// engine (hsa_amd_memory_async_copy).  hipMemcpyAsync does these copies with a
// blit kernel whose PCIe-bound stores hold up the other HIP stream's kernels
// (measured 3x slower while a 140 MB payload copy runs); the SDMA engines
// leave the CUs and their caches to the compute.  Returns false (the caller
// falls back to hipMemcpyAsync) if HSA cannot take the copy; LFM_D2H_SDMA=0
// disables it.  The caller has synchronised the producing stream.
// the HSA CPU agent (SDMA copies are enabled and HSA is up), or null
static const hsa_agent_t* hsa_cpu_agent()
{
    struct Cpu {
        bool ok = false;
        hsa_agent_t agent{};
        Cpu()
        {
            const char* e = std::getenv("LFM_D2H_SDMA");
            if ((e && std::atoi(e) == 0) || hsa_init() != HSA_STATUS_SUCCESS) return;
            hsa_iterate_agents(
                [](hsa_agent_t a, void* d) {
                    hsa_device_type_t t;
                    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS &&
                        t == HSA_DEVICE_TYPE_CPU) {
                        *(hsa_agent_t*)d = a;
                        return HSA_STATUS_INFO_BREAK;
                    }
                    return HSA_STATUS_SUCCESS;
                },
                &agent);
            ok = agent.handle != 0;
        }
    };
    static Cpu cpu;
    return cpu.ok ? &cpu.agent : nullptr;
}

static bool sdma_d2h(void* dst, const void* src, size_t n)
{
    const hsa_agent_t* cpu = hsa_cpu_agent();
    if (!cpu || n == 0) return cpu != nullptr;
    hsa_amd_pointer_info_t info;
    std::memset(&info, 0, sizeof(info));
    info.size = sizeof(info);
    if (hsa_amd_pointer_info(src, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        info.type != HSA_EXT_POINTER_TYPE_HSA)
        return false;
    hsa_signal_t sig;
    if (hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) return false;
    bool ok = hsa_amd_memory_async_copy(dst, *cpu, src, info.agentOwner, n, 0, nullptr, sig) == HSA_STATUS_SUCCESS;
    if (ok)
        ok = hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED) == 0;
    hsa_signal_destroy(sig);
    return ok;
}

// the payload copy of gpu_compress: SDMA if possible, else hipMemcpyAsync
static bool payload_d2h(void* dst, const void* src, size_t n, hipStream_t st)
{
    if (hipStreamSynchronize(st) != hipSuccess) return false;
    if (sdma_d2h(dst, src, n)) return true;
    return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess;
}

// ------------------------------------------------------- block compression --
static int compress_one(int ctype, uint8_t* in, uint32_t n, uint8_t* out, uint32_t cap, uint32_t* out_len,
                        int level)
{
    switch (ctype) {
    case NONE:
        std::memcpy(out, in, n);
        *out_len = n;
        return 0;
    case BZIP2: {
        unsigned int len = cap;
        int rc = BZ2_bzBuffToBuffCompress((char*)out, &len, (char*)in, n, level, 0, 30);
        *out_len = len;
        return rc == LFM_BZ_OK ? 0 : 2;
    }
    case ZLIB: {
        z_stream s;
        std::memset(&s, 0, sizeof(s));
        if (deflateInit(&s, Z_DEFAULT_COMPRESSION) != Z_OK) return 3;
        s.next_in = in;
        s.avail_in = n;
        s.next_out = out;
        s.avail_out = cap;
        s.data_type = Z_BINARY;
        int rc = deflate(&s, Z_FINISH);
        *out_len = cap - s.avail_out;
        deflateEnd(&s);
        return (rc == Z_STREAM_END || rc == Z_OK) ? 0 : 3;
    }
    }
    return 5;
}

static int decompress_one(int ctype, const uint8_t* in, uint32_t n, uint8_t* out, uint32_t expect)
{
    switch (ctype) {
    case NONE:
        if (n != expect) return 3;
        std::memcpy(out, in, n);
        return 0;
    case BZIP2: {
        unsigned int len = expect;
        int rc = BZ2_bzBuffToBuffDecompress((char*)out, &len, (char*)in, n, 0, 0);
        return (rc == LFM_BZ_OK && len == expect) ? 0 : 2;
    }
    case ZLIB: {
        z_stream s;
        std::memset(&s, 0, sizeof(s));
        if (inflateInit(&s) != Z_OK) return 3;
        s.next_in = const_cast<uint8_t*>(in);
        s.avail_in = n;
        s.next_out = out;
        s.avail_out = expect;
        int rc = inflate(&s, Z_FINISH);
        const bool ok = (rc == Z_STREAM_END) && s.avail_out == 0;
        inflateEnd(&s);
        return ok ? 0 : 3;
    }
    }
    return 5;
}

int bzip2_level(const klb_image_header& h)
{
    return std::min(9, (int)((h.getBlockSizeBytes() + 99999) / 100000));  // klb_imageIO.cpp:108, nominal block
}

int compress_blocks(const uint8_t* sym, klb_image_header& h, Sink& sink, int threads, int level)
{
    const BlockGrid g(h);
    const uint64_t nblocks = g.nblocks;
    h.resizeBlockOffset(nblocks);
    const size_t bpp = h.getBytesPerPixel();
    const uint32_t block_bytes = h.getBlockSizeBytes();                 // nominal (clamped) block
    if (level < 1) level = bzip2_level(h);
    uint32_t cap = block_bytes;
    if (h.compressionType != NONE) cap = (uint32_t)std::ceil((float)block_bytes * 2.0f + 50.0f);
    if (h.compressionType != NONE && h.compressionType != BZIP2 && h.compressionType != ZLIB) {
        std::printf("ERROR: compression type not implemented\n");
        return 5;
    }
    threads = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(threads, 1), nblocks));

    std::vector<std::vector<uint8_t>> res(nblocks);
    std::vector<uint8_t> done(nblocks, 0);
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<uint64_t> next{0};
    std::atomic<int> err{0};

    auto worker = [&]() {
        std::vector<uint8_t> in(block_bytes), out(cap);
        for (;;) {
            const uint64_t id = next.fetch_add(1);
            if (id >= nblocks) break;
            size_t n = 0;
            gather_block(sym, g, id, bpp, in.data(), &n);
            uint32_t len = 0;
            int rc = err.load() ? 0 : compress_one(h.compressionType, in.data(), (uint32_t)n, out.data(), cap, &len, level);
            if (rc) {
                std::printf("ERROR: compressing block %llu failed (code %d)\n", (unsigned long long)id, rc);
                int z = 0;
                err.compare_exchange_strong(z, rc);
                len = 0;
            }
            std::vector<uint8_t> v(out.data(), out.data() + len);
            {
                std::lock_guard<std::mutex> lk(mu);
                res[id].swap(v);
                done[id] = 1;
            }
            cv.notify_all();
        }
    };
    std::vector<std::thread> pool;
    pool.reserve(threads);
    for (int i = 0; i < threads; ++i) pool.emplace_back(worker);

    int rc = sink.begin(h);
    uint64_t offset = 0;
    for (uint64_t id = 0; id < nblocks; ++id) {
        std::vector<uint8_t> blk;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return done[id] != 0; });
            blk.swap(res[id]);
        }
        if (!rc && !err.load()) rc = sink.append(blk.data(), blk.size());
        offset += blk.size();
        h.blockOffset[id] = offset;
    }
    for (auto& t : pool) t.join();
    if (err.load()) return err.load();
    if (rc) return rc;
    return sink.finish(h);
}

// --------------------------------------------------------------- encoder --
// GPU bzip2 (default when a GPU is usable); env LFM_GPU_BZIP2=0 selects the
// host library for every block (the same bytes, for comparison).
bool gpu_decode_enabled()
{
    static const bool on = [] {
        const char* e = std::getenv("LFM_GPU_DECODE");
        return !(e && e[0] == '0');
    }();
    return on;
}

bool gpu_bzip2_enabled()
{
    static const bool on = [] {
        const char* e = std::getenv("LFM_GPU_BZIP2");
        return !(e && e[0] == '0');
    }();
    return on;
}

// GPU bzip2 for an encode: on unless disabled (LFM_GPU_BZIP2=0), not bzip2 or
// no device; a host image of at most kHostBz2Bytes goes to the host library
// (its predictor stage, if any, still runs on the GPU): a GPU batch costs
// about a millisecond of launches and host synchronisations, more than
// libbzip2 needs on the host threads for such an image (config 1's
// 101 x 151 page: 1.3 ms through the GPU batch, 0.18 ms on the host).
constexpr uint64_t kHostBz2Bytes = 1u << 20;
static bool use_gpu_bzip2(const klb_image_header& h, bool dev)
{
    if (!gpu_bzip2_enabled() || h.compressionType != BZIP2 || lfm_hip_device_count() <= 0) return false;
    return dev || h.getImageSizeBytes() > kHostBz2Bytes;
}

// the GPU bzip2 decoder (env LFM_GPU_BUNZIP2=0: host libbz2 per block)
bool gpu_bunzip2_enabled()
{
    static const bool on = env_int("LFM_GPU_BUNZIP2", 1) != 0;
    return on;
}

Encoder::Encoder(int device) : device_(device) {}

Encoder::~Encoder()
{
    join_inflight();
    for (UploadPipe& u : up_) u.join();
    if (gpu_ready_) {
        for (UploadPipe& u : up_) {
            for (hipEvent_t e : u.ev) (void)hipEventDestroy(e);
            u.release_sdma();
        }
        if (up_stream_) (void)hipStreamDestroy(up_stream_);
        (void)hipSetDevice(device_);
        if (d_in_) (void)hipFree(d_in_);
        for (void* d : d_sym_)
            if (d) (void)hipFree(d);
        if (d_ws_) (void)hipFree(d_ws_);
        if (d_prev_) (void)hipFree(d_prev_);
        if (d_sel_) (void)hipFree(d_sel_);
        for (auto& set : bz_)
            for (BzSlot& sl : set) {
                if (sl.d_ws) (void)hipFree(sl.d_ws);
                if (sl.d_out) (void)hipFree(sl.d_out);
                if (sl.h_out) (void)hipHostFree(sl.h_out);
                if (sl.stream) (void)hipStreamDestroy(sl.stream);
            }
        for (void* hs : h_sym_)
            if (hs) (void)hipHostFree(hs);
        if (ev0_) (void)hipEventDestroy(ev0_);
        if (ev1_) (void)hipEventDestroy(ev1_);
        if (caller_ev_) (void)hipEventDestroy(caller_ev_);
        if (stream_) (void)hipStreamDestroy(stream_);
        if (copy_stream_) (void)hipStreamDestroy(copy_stream_);
    }
}

void Encoder::join_inflight()
{
    for (Inflight& f : fly_)
        if (f.th.joinable()) f.th.join();
}

void Encoder::Inflight::release()
{
    {
        std::lock_guard<std::mutex> lk(mu);
        released = true;
        mtf_done = true;
    }
    cv.notify_all();
}

void Encoder::Inflight::reach()
{
    {
        std::lock_guard<std::mutex> lk(mu);
        ++reached;
        if (need > 0 && reached >= need) released = mtf_done = true;
    }
    cv.notify_all();
}

void Encoder::Inflight::reach2()
{
    {
        std::lock_guard<std::mutex> lk(mu);
        ++reached2;
        if (need > 0 && reached2 >= need) mtf_done = true;
    }
    cv.notify_all();
}

void Encoder::Inflight::wait_mtf()
{
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return mtf_done || released; });
}

void Encoder::Inflight::wait_release()
{
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return released; });
}

int Encoder::submit(const void* img, bool dev, klb_image_header& h, int threads, const SlabSpec* slab,
                    uint64_t* ticket)
{
    static const SlabSpec whole;
    if (threads <= 0) threads = default_threads();
    if (int rc = after_caller(dev)) return rc;
    const int p = par_;
    Inflight& f = fly_[p];
    if (f.th.joinable()) f.th.join();  // the encode before last used this buffer set
    // Auto-selection (klb_imageIO.cpp:2316-2360) on the encoder's stream; the
    // request then becomes the forced 8 + k (video bit kept) for the
    // predictor stage, the bytes are the same.
    const bool gpu_bz = use_gpu_bzip2(h, dev);
    const int req0 = h.headerVersion & 0x7F;
    int pre_k = -1;
    float pre_ent[8] = {0};
    double pre_ms = 0.0;
    auto select_now = [&]() -> int {
        auto ts0 = clk::now();
        if (int rc = preselect(img, dev, h, slab ? *slab : whole, &pre_k, pre_ent)) return rc;
        pre_ms = ms_since(ts0);
        h.headerVersion = (uint8_t)((h.headerVersion & 0x80) | (8 + pre_k));
        return 0;
    };
    const bool pre = gpu_bz && req0 < NUM_PREDICTORS && h.getBytesPerPixel() == 2 && h.Nnum > 0;
    // a host stack starts its chunked upload (and the predictor on the chunks
    // that have landed) before the previous encode is released: the PCIe
    // upload runs under the previous encode's GPU bzip2.  A device stack, too,
    // runs its selection and predictor stage before that wait, beside the
    // previous encode's tail (its own buffer set; the selection then queues
    // behind that tail and the predictor kernel shares the CUs): config 3
    // pipelined 12 068-12 158 vs 11 797-11 872 Mpixel/s waiting for the
    // release first, same box (profiles/r04_ab_predict_early.txt)
    const bool host_early = gpu_bz && (upload_pipe_ok(dev, h) || dev);
    f.ticket = next_ticket_++;
    f.rc = 0;
    std::memset(&f.st, 0, sizeof(f.st));
    {
        std::lock_guard<std::mutex> lk(f.mu);
        f.reached = 0;
        f.reached2 = 0;
        f.need = 0;
        f.released = false;
        f.mtf_done = false;
    }
    if (ticket) *ticket = f.ticket;
    par_ ^= 1;
    auto fail = [&](int rc) {
        up_[p].join();
        f.rc = rc;
        f.release();
        return rc;
    };
    // LFM_SELECT_AT=2: a device stack's selection and predictor stage wait
    // until the previous encode is past its MTF stage, i.e. in its
    // latency-bound Huffman rounds, instead of sharing the CUs with its sorts
    static const int select_at = env_int("LFM_SELECT_AT", 0);
    if (select_at == 2 && dev && host_early) fly_[p ^ 1].wait_mtf();
    if (pre && host_early)
        if (int rc = select_now()) return fail(rc);
    if (pre_k >= 0) {
        f.st.select_ms = pre_ms;
        std::memcpy(f.st.entropy, pre_ent, sizeof(pre_ent));
    }
    auto t0 = clk::now();
    int level = slab ? slab->level : -1;
    if (level < 1 && slab && slab->z0 > 0 && h.getBytesPerPixel()) {
        klb_image_header nominal(h);
        for (int d = 0; d < KLB_DATA_DIMS; ++d)
            if (d != 2 && nominal.blockSize[d]) nominal.blockSize[d] = std::min(nominal.blockSize[d], h.xyzct[d]);
        if (nominal.blockSize[2] == 0) nominal.blockSize[2] = 1;
        level = bzip2_level(nominal);
    }
    const uint8_t* dsym = nullptr;
    if (host_early) {
        if (int rc = normalize_header(h)) return fail(rc);
        if (int rc = predictor_stage(img, dev, h, nullptr, &dsym, &f.st, slab ? *slab : whole, p)) return fail(rc);
    }
    fly_[p ^ 1].wait_release();        // the previous encode is in its tail
    if (pre && !host_early) {
        if (int rc = select_now()) return fail(rc);
        f.st.select_ms = pre_ms;
        std::memcpy(f.st.entropy, pre_ent, sizeof(pre_ent));
    }
    if (!gpu_bz) {  // no GPU bzip2: the whole encode here
        MemSink sink(&mem_ring[p]);
        f.rc = encode_set(img, dev, h, sink, &f.st, threads, slab, p);
        f.release();
        return f.rc;
    }
    if (!host_early &&
        ((f.rc = normalize_header(h)) || (f.rc = predictor_stage(img, dev, h, nullptr, &dsym, &f.st, slab ? *slab : whole, p))))
        return fail(f.rc);
    if ((f.rc = ensure_gpu())) return fail(f.rc);
    if (dev && dsym == (const uint8_t*)img) {
        // no predictor stage (forced predictor 0, non-16-bit data): the symbols
        // ARE the caller's image, which the caller may release or refill once
        // submit returns -- the finisher must compress a copy of it
        const size_t bytes = h.getImageSizeBytes();
        if (!dev_alloc(d_sym_[p], d_sym_cap_[p], bytes) ||
            hipMemcpyAsync(d_sym_[p], img, bytes, hipMemcpyDeviceToDevice, stream_) != hipSuccess ||
            hipStreamSynchronize(stream_) != hipSuccess) {
            f.rc = 3;
            f.release();
            return f.rc;
        }
        dsym = (const uint8_t*)d_sym_[p];
    }
    auto hh = std::make_shared<klb_image_header>(h);
    f.th = std::thread([this, &f, hh, dsym, level, p, t0]() {
        (void)hipSetDevice(device_);
        MemSink sink(&mem_ring[p]);
        auto tc = clk::now();
        f.rc = gpu_compress(dsym, *hh, sink, &f.st, level, p, &f);
        f.st.compress_ms = ms_since(tc);
        f.st.total_ms = ms_since(t0);
        f.st.header_version = hh->headerVersion;
        f.st.chosen = hh->headerVersion & 0x7F;
        f.st.out_bytes = hh->getCompressedFileSizeInBytes();
        f.release();  // in case the release stage was never reached (host paths)
    });
    UploadPipe& up = up_[p];
    if (up.active) {
        // the caller may release a host stack once submit returns: wait for
        // its upload (the finisher's GPU bzip2 already runs on the chunks)
        up.join();
        f.st.h2d_ms += up.h2d_ms;
        f.st.predict_ms += up.predict_ms;
        if (up.rc) return up.rc;  // the finisher's batches fail too; wait() reports it
    }
    return 0;
}

int Encoder::wait(uint64_t ticket, const PinnedBuffer** out, lfm_encode_stats* st)
{
    for (int p = 0; p < 2; ++p) {
        Inflight& f = fly_[p];
        if (f.ticket != ticket || ticket == 0) continue;
        if (f.th.joinable()) f.th.join();
        if (out) *out = &mem_ring[p];
        if (st) *st = f.st;
        return f.rc;
    }
    return kErrUnknownTicket;  // never submitted, already recycled (two submits ago), or 0
}

int Encoder::ensure_gpu()
{
    if (gpu_ready_) return 0;
    int n = lfm_hip_device_count();
    if (n <= 0) {
        std::printf("ERROR: the LFM predictor stage needs a HIP GPU (gfx950) and none is visible\n");
        return kErrNoGpu;
    }
    if (device_ < 0) {
        if (hipGetDevice(&device_) != hipSuccess) device_ = 0;
    }
    if (device_ >= n || hipSetDevice(device_) != hipSuccess) return kErrNoGpu;
    // the predictor stage's stream (a high-priority one measured 10 % slower
    // end to end: it took a hardware queue from the bzip2 slots)
    if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) return kErrNoGpu;
    // the first buffer set's GPU bzip2 slot streams are created right after
    // the predictor stream, so each lands on a hardware queue of its own
    // (GPU_MAX_HW_QUEUES is 4, the null stream holding one): streams created
    // later share queues, and two slots sharing one run their batches in
    // series (measured: the upload pipe's extra stream, created first, put
    // both slots on one queue, +19 ms per 2 GiB encode)
    for (int k = 0; k < bz_slot_count(); ++k)
        if (hipStreamCreateWithFlags(&bz_[0][k].stream, hipStreamNonBlocking) != hipSuccess) return kErrNoGpu;
    (void)hipEventCreate(&ev0_);
    (void)hipEventCreate(&ev1_);
    gpu_ready_ = true;
    return 0;
}

void* Encoder::dev_alloc(void*& p, size_t& cap, size_t need)
{
    if (need <= cap && p) return p;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, need) != hipSuccess) return nullptr;
    cap = need;
    return p;
}

// ---------------------------------------------------------- upload pipe --
int Encoder::UploadPipe::wait_frames(uint64_t f_end, hipStream_t st)
{
    std::unique_lock<std::mutex> lk(mu);
    if (!active) return 0;
    size_t c = (size_t)(std::lower_bound(end.begin(), end.begin() + nchunks, f_end) - end.begin());
    if (c >= nchunks) c = nchunks - 1;
    cv.wait(lk, [&] { return recorded > c || rc != 0; });
    if (rc) return 3;
    return hipStreamWaitEvent(st, ev[3 * c + 2], 0) == hipSuccess ? 0 : 3;
}

void Encoder::UploadPipe::release_sdma()
{
    for (int i = 0; i < 2; ++i) {
        if (sig[i]) hsa_signal_destroy(hsa_signal_t{sig[i]});
        if (stage[i]) (void)hipHostFree(stage[i]);
        sig[i] = 0;
        stage[i] = nullptr;
    }
    stage_cap = 0;
}

void Encoder::UploadPipe::join()
{
    if (th.joinable()) th.join();
    std::lock_guard<std::mutex> lk(mu);
    active = false;
}

int Encoder::bz_slot_count()
{
    static const int n = [] {
        const int v = env_int("LFM_BZ2_SLOTS", 0);
        return v > 0 ? std::min(v, (int)kBzSlots) : 2;
    }();
    return n;
}

bool Encoder::upload_pipe_ok(bool dev, const klb_image_header& h) const
{
    static const bool on = [] {
        const char* e = std::getenv("LFM_H2D_PIPE");
        return !(e && std::atoi(e) == 0);
    }();
    return on && !dev && h.getBytesPerPixel() == 2 && h.Nnum > 0;
}

// Upload the host stack in chunks of whole frames through a ring of device
// slots and predict each chunk (forced predictor k >= 1) into the set's
// symbol buffer as it lands (see UploadPipe).  Returns once the uploader
// thread runs; UploadPipe::join waits for it (the host image is read until
// then).  The chunk's first frame takes its temporal predecessor from the
// previous chunk's slot (or the slab's prev frame), which the ring keeps
// until the chunk after it has been predicted.
int Encoder::start_upload(const void* img, klb_image_header& h, const SlabSpec& slab, int k, int set)
{
    UploadPipe& up = up_[set];
    up.join();
    const uint64_t W = h.xyzct[0], H = h.xyzct[1], Z = h.xyzct[2];
    const uint64_t V = (uint64_t)h.xyzct[3] * h.xyzct[4];
    const size_t fpx = W * H, fs = fpx * 2;
    const int video = (h.headerVersion >> 7) & 1;
    static const size_t chunk_target = [] {
        const char* e = std::getenv("LFM_H2D_CHUNK_MB");
        const long v = e ? std::atol(e) : 0;
        return (size_t)(v > 0 ? v : 32) << 20;
    }();
    static const size_t ring_target = [] {
        const char* e = std::getenv("LFM_H2D_RING_MB");
        const long v = e ? std::atol(e) : 0;
        return (size_t)(v > 0 ? v : 1024) << 20;
    }();
    // >= chunk_target bytes of whole frames; an even count on video stacks
    // (a spatial and its temporal frame go through the pair kernel together)
    uint64_t cz = std::max<uint64_t>(1, (chunk_target + fs - 1) / fs);
    if (video && (cz & 1)) ++cz;
    cz = std::min<uint64_t>(cz, Z);
    const uint64_t per_vol = (Z + cz - 1) / cz, nch = V * per_vol;
    const size_t cbytes = cz * fs;
    // at least 3 slots: the SDMA loop issues copy c before chunk c - 1 is
    // predicted, and slot c % nslot must no longer be read by chunk
    // c - nslot + 1 (its last frame is that chunk's temporal predecessor), so
    // that chunk's predictor must already be issued when copy c waits for it
    const uint64_t nslot = std::min<uint64_t>(nch, std::max<uint64_t>(3, ring_target / cbytes));
    if (!dev_alloc(d_in_, d_in_cap_, nslot * cbytes)) return 3;
    if (!dev_alloc(d_sym_[set], d_sym_cap_[set], V * Z * fs)) return 3;
    while (up.ev.size() < 3 * nch) {
        hipEvent_t e = nullptr;
        if (hipEventCreate(&e) != hipSuccess) return 3;
        up.ev.push_back(e);
    }
    const uint16_t* d_prev = nullptr;
    if (slab.z0 > 0 && video && (slab.z0 & 1)) {
        if (V != 1 || !slab.prev) return 3;
        if (!dev_alloc(d_prev_, d_prev_cap_, fs)) return 3;
        if (hipMemcpyAsync(d_prev_, slab.prev, fs, hipMemcpyHostToDevice, stream_) != hipSuccess) return 3;
        d_prev = (const uint16_t*)d_prev_;
    }
    up.end.assign(nch, 0);
    for (uint64_t c = 0; c < nch; ++c) up.end[c] = (c / per_vol) * Z + std::min<uint64_t>(Z, (c % per_vol + 1) * cz);
    {
        std::lock_guard<std::mutex> lk(up.mu);
        up.nchunks = nch;
        up.recorded = 0;
        up.rc = 0;
        up.active = true;
        up.h2d_ms = up.predict_ms = 0.0;
    }
    const int fam = current_family(), T = h.Nnum;
    const uint32_t z0 = slab.z0;
    uint16_t* const d_in = (uint16_t*)d_in_;
    uint16_t* const d_sym = (uint16_t*)d_sym_[set];
    const uint8_t* const src = (const uint8_t*)img;
    // copies on an SDMA engine (LFM_H2D_SDMA=0: hipMemcpyAsync, whose blit
    // kernel measured ~25 ms slower for the GPU bzip2 running beside a 2 GiB
    // upload); a pinned (HSA-allocated) source goes straight to the engine,
    // a pageable one through two pinned staging chunks (host copy of one
    // overlapping the engine's copy of the other)
    static const bool sdma_on = env_int("LFM_H2D_SDMA", 1) != 0;
    const hsa_agent_t* cpu = sdma_on ? hsa_cpu_agent() : nullptr;
    hsa_agent_t gpu{};
    bool direct = false;
    if (cpu) {
        hsa_amd_pointer_info_t info;
        std::memset(&info, 0, sizeof(info));
        info.size = sizeof(info);
        if (hsa_amd_pointer_info(d_in_, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
            info.type != HSA_EXT_POINTER_TYPE_HSA)
            cpu = nullptr;
        else
            gpu = info.agentOwner;
    }
    if (cpu) {
        hsa_amd_pointer_info_t info;
        std::memset(&info, 0, sizeof(info));
        info.size = sizeof(info);
        direct = hsa_amd_pointer_info((void*)img, &info, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS &&
                 info.type == HSA_EXT_POINTER_TYPE_HSA;
        for (int i = 0; i < 2 && cpu; ++i) {
            hsa_signal_t sg;
            if (!up.sig[i]) {
                if (hsa_signal_create(0, 0, nullptr, &sg) != HSA_STATUS_SUCCESS) cpu = nullptr;
                else up.sig[i] = sg.handle;
            }
        }
        if (cpu && !direct && up.stage_cap < cbytes) {
            for (int i = 0; i < 2; ++i) {
                if (up.stage[i]) (void)hipHostFree(up.stage[i]);
                up.stage[i] = nullptr;
            }
            up.stage_cap = 0;
            if (hipHostMalloc(&up.stage[0], cbytes, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc(&up.stage[1], cbytes, hipHostMallocDefault) != hipSuccess)
                cpu = nullptr;
            else
                up.stage_cap = cbytes;
        }
    }
    // (the stream of the hipMemcpyAsync copies only: SDMA copies need none)
    if (!cpu && !up_stream_ && hipStreamCreateWithFlags(&up_stream_, hipStreamNonBlocking) != hipSuccess) return 3;
    const int cthreads = default_threads();
    up.th = std::thread([=, &up]() {
        (void)hipSetDevice(device_);
        auto t0 = clk::now();
        int rc = 0;
        auto predict = [&](uint64_t c, uint16_t* slot) -> int {
            const uint64_t v = c / per_vol, za = (c % per_vol) * cz, zb = std::min<uint64_t>(Z, za + cz);
            hipEvent_t* e = &up.ev[3 * c];
            const uint16_t* prev = nullptr;
            if (video) prev = za > 0 ? d_in + ((c - 1) % nslot) * cz * fpx + (cz - 1) * fpx : d_prev;
            (void)hipEventRecord(e[1], stream_);
            if (lfm_hip_predict(slot, prev, d_sym + (v * Z + za) * fpx, (int)W, (int)H, (int)(zb - za), T, fam, k,
                                video, (int)(z0 + za), stream_) != LFM_HIP_OK ||
                hipEventRecord(e[2], stream_) != hipSuccess)
                return 3;
            {
                std::lock_guard<std::mutex> lk(up.mu);
                up.recorded = c + 1;
            }
            up.cv.notify_all();
            return 0;
        };
        auto sig_wait = [&](int b) {
            return hsa_signal_wait_scacquire(hsa_signal_t{up.sig[b]}, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                             HSA_WAIT_STATE_BLOCKED) == 0;
        };
        // SDMA: copy c is issued before chunk c - 1 (copied) is predicted,
        // so the engine always has the next chunk while a chunk is predicted
        for (uint64_t c = 0; cpu && c < nch && !rc; ++c) {
            const uint64_t v = c / per_vol, za = (c % per_vol) * cz, zb = std::min<uint64_t>(Z, za + cz);
            const size_t len = (zb - za) * fs;
            const int b = (int)(c & 1);
            uint16_t* slot = d_in + (c % nslot) * cz * fpx;
            // the slot's last readers (chunk c - nslot and the chunk after
            // it, which reads its last frame) are predicted
            if (c >= nslot && hipEventSynchronize(up.ev[3 * (c - nslot + 1) + 2]) != hipSuccess) rc = 3;
            if (!rc && c >= 2 && !sig_wait(b)) rc = 3;  // (chunk c - 2's copy: staging chunk b is free)
            const uint8_t* from = src + (v * Z + za) * fs;
            if (!rc && !direct) {
                par_memcpy(up.stage[b], from, len, cthreads);
                from = (const uint8_t*)up.stage[b];
            }
            if (!rc) {
                hsa_signal_store_relaxed(hsa_signal_t{up.sig[b]}, 1);
                if (hsa_amd_memory_async_copy(slot, gpu, from, *cpu, len, 0, nullptr, hsa_signal_t{up.sig[b]}) !=
                    HSA_STATUS_SUCCESS) {
                    hsa_signal_store_relaxed(hsa_signal_t{up.sig[b]}, 0);
                    rc = 3;
                }
            }
            if (!rc && c >= 1) {
                if (!sig_wait((int)((c - 1) & 1))) rc = 3;
                else rc = predict(c - 1, d_in + ((c - 1) % nslot) * cz * fpx);
            }
        }
        if (cpu && !rc) {
            if (!sig_wait((int)((nch - 1) & 1))) rc = 3;
            else rc = predict(nch - 1, d_in + ((nch - 1) % nslot) * cz * fpx);
        }
        if (cpu) {  // no copy still reads the caller's image or a staging chunk
            for (int b = 0; b < 2; ++b) (void)sig_wait(b);
        }
        for (uint64_t c = 0; !cpu && c < nch && !rc; ++c) {
            const uint64_t v = c / per_vol, za = (c % per_vol) * cz, zb = std::min<uint64_t>(Z, za + cz);
            uint16_t* slot = d_in + (c % nslot) * cz * fpx;
            hipEvent_t* e = &up.ev[3 * c];
            // the slot was chunk c - nslot's; chunk c - nslot + 1 (predicted
            // after it) also reads that slot's last frame as its temporal prev
            if (c >= nslot && hipStreamWaitEvent(up_stream_, up.ev[3 * (c - nslot + 1) + 2], 0) != hipSuccess) rc = 3;
            if (!rc && hipMemcpyAsync(slot, src + (v * Z + za) * fs, (zb - za) * fs, hipMemcpyHostToDevice,
                                      up_stream_) != hipSuccess)
                rc = 3;
            if (!rc && (hipEventRecord(e[0], up_stream_) != hipSuccess ||
                        hipStreamWaitEvent(stream_, e[0], 0) != hipSuccess))
                rc = 3;
            const uint16_t* prev = nullptr;
            if (video) prev = za > 0 ? d_in + ((c - 1) % nslot) * cz * fpx + (cz - 1) * fpx : d_prev;
            if (!rc) {
                (void)hipEventRecord(e[1], stream_);
                if (lfm_hip_predict(slot, prev, d_sym + (v * Z + za) * fpx, (int)W, (int)H, (int)(zb - za), T, fam, k,
                                    video, (int)(z0 + za), stream_) != LFM_HIP_OK ||
                    hipEventRecord(e[2], stream_) != hipSuccess)
                    rc = 3;
            }
            {
                std::lock_guard<std::mutex> lk(up.mu);
                if (rc) up.rc = rc;
                else up.recorded = c + 1;
            }
            up.cv.notify_all();
        }
        // the host image is no longer read once the copies are done
        if (!cpu && hipStreamSynchronize(up_stream_) != hipSuccess) rc = 3;
        const double h2d = ms_since(t0);
        double pms = 0.0;
        if (!rc && hipEventSynchronize(up.ev[3 * (nch - 1) + 2]) == hipSuccess) {
            for (uint64_t c = 0; c < nch; ++c) {
                float ms = 0.f;
                if (hipEventElapsedTime(&ms, up.ev[3 * c + 1], up.ev[3 * c + 2]) == hipSuccess) pms += ms;
            }
        }
        {
            std::lock_guard<std::mutex> lk(up.mu);
            if (rc) up.rc = rc;
            up.h2d_ms = h2d;
            up.predict_ms = pms;
        }
        up.cv.notify_all();
    });
    return 0;
}

int Encoder::predictor_stage(const void* img, bool dev, klb_image_header& h, const uint8_t** sym,
                             const uint8_t** dsym, lfm_encode_stats* st, const SlabSpec& slab, int set)
{
    void*& d_sym_ = this->d_sym_[set];
    size_t& d_sym_cap_ = this->d_sym_cap_[set];
    void*& h_sym_ = this->h_sym_[set];
    size_t& h_sym_cap_ = this->h_sym_cap_[set];
    // dsym != nullptr: the caller compresses on the GPU -- leave the symbols
    // of every volume in device memory (*dsym) and skip the host copy.
    const bool keep = dsym != nullptr;
    const size_t bpp = h.getBytesPerPixel();
    const uint8_t hv = h.headerVersion;
    const int req = hv & 0x7F;
    const int video = (hv >> 7) & 1;
    const uint64_t W = h.xyzct[0], H = h.xyzct[1], Z = h.xyzct[2];
    const uint64_t V = (uint64_t)h.xyzct[3] * h.xyzct[4];
    const uint64_t vol = W * H * Z;
    const uint64_t total_bytes = h.getImageSizeBytes();
    const bool autosel = req < NUM_PREDICTORS;
    int k = autosel ? 0 : (hv & 0x77);  // `headerVersion & 0x7F - 8` parses as & 0x77 (klb_imageIO.cpp:2380)
    if (st) st->chosen = 0;
    if (sym) *sym = nullptr;
    if (dsym) *dsym = nullptr;

    auto host_symbols_from_device = [&](const void* d, size_t bytes) -> int {
        if (!h_sym_ || h_sym_cap_ < bytes) {
            if (h_sym_) (void)hipHostFree(h_sym_);
            h_sym_ = nullptr;
            h_sym_cap_ = 0;
            if (hipHostMalloc(&h_sym_, bytes, hipHostMallocDefault) != hipSuccess) return 3;
            h_sym_cap_ = bytes;
        }
        auto t0 = clk::now();
        if (hipMemcpyAsync(h_sym_, d, bytes, hipMemcpyDeviceToHost, stream_) != hipSuccess) return 3;
        if (hipStreamSynchronize(stream_) != hipSuccess) return 3;
        if (st) st->d2h_ms += ms_since(t0);
        *sym = (const uint8_t*)h_sym_;
        return 0;
    };

    // data without a 16-bit sample: no predictor stage (the reference would
    // reinterpret the buffer as uint16, klb_imageIO.cpp:2365)
    const bool predictable = (bpp == 2) && h.Nnum > 0;
    if (!predictable || (!autosel && k == 0)) {
        if (!autosel && k > 7) return kErrBadPredictor;
        h.headerVersion = (uint8_t)(hv & 0x80);
        if (keep) {  // the raw image is the symbol stream
            if (dev) {
                *dsym = (const uint8_t*)img;
                return 0;
            }
            if (!dev_alloc(d_sym_, d_sym_cap_, total_bytes)) return 3;
            auto t0 = clk::now();
            if (hipMemcpyAsync(d_sym_, img, total_bytes, hipMemcpyHostToDevice, stream_) != hipSuccess) return 3;
            if (hipStreamSynchronize(stream_) != hipSuccess) return 3;
            if (st) st->h2d_ms += ms_since(t0);
            *dsym = (const uint8_t*)d_sym_;
            return 0;
        }
        if (!dev) {
            *sym = (const uint8_t*)img;
            return 0;
        }
        return host_symbols_from_device(img, total_bytes);
    }
    if (!autosel && k > 7) {
        std::printf("ERROR: predictor request %d is not valid (use 0-7 for auto, 8-15 for predictor 0-7)\n", req);
        return kErrBadPredictor;
    }
    if (int rc = ensure_gpu()) return rc;
    (void)hipSetDevice(device_);
    const int fam = current_family();
    const int T = h.Nnum;

    if (keep && upload_pipe_ok(dev, h)) {
        // host stack, GPU bzip2: chunked upload overlapped with the predictor
        // and the compression (start_upload); selection first, on frame 0 of
        // volume (0, 0) or the stack's frame 0 handed in for a slab
        if (autosel) {
            auto t0 = clk::now();
            const void* frame = slab.select_frame ? slab.select_frame : (slab.z0 > 0 ? nullptr : img);
            if (!frame) return 3;  // a slab's own frame 0 is not the stack's
            float ent[8];
            if (int rc = select_host_frame(frame, (int)W, (int)H, T, fam, &k, ent)) return rc;
            if (st) {
                st->select_ms += ms_since(t0);
                std::memcpy(st->entropy, ent, sizeof(ent));
            }
        }
        if (int rc = start_upload(img, h, slab, k, set)) {
            up_[set].join();
            return rc;
        }
        h.headerVersion = (uint8_t)((hv & 0x80) | k);
        if (st) st->chosen = k;
        if (video && fam != 0 && Z > 1)
            std::fprintf(stderr, "WARNING: video stack with the %s predictor family: the odd frames are coded with the "
                                 "reference's lossy temporal residual and cannot be decoded exactly\n",
                         fam == 1 ? "angle" : "space");
        *dsym = (const uint8_t*)d_sym_;
        return 0;
    }

    const uint16_t* d_img = (const uint16_t*)img;
    // slab of a larger stack: its first frame may need the raw frame z0 - 1
    const uint16_t* d_prev = nullptr;
    if (slab.z0 > 0) {
        if (V != 1) return 3;  // slabs are z ranges of a single (c, t) volume
        if (video && (slab.z0 & 1)) {
            if (!slab.prev) return 3;
            if (dev) {
                d_prev = (const uint16_t*)slab.prev;
            } else {
                if (!dev_alloc(d_prev_, d_prev_cap_, W * H * 2)) return 3;
                if (hipMemcpyAsync(d_prev_, slab.prev, W * H * 2, hipMemcpyHostToDevice, stream_) != hipSuccess)
                    return 3;
                d_prev = (const uint16_t*)d_prev_;
            }
        }
    }
    // every volume's symbols stay on the device when they are needed there
    // (device input, or GPU compression); otherwise one volume at a time
    const bool all_on_device = dev || keep;
    if (!dev && !dev_alloc(d_in_, d_in_cap_, vol * 2)) return 3;
    if (!dev_alloc(d_sym_, d_sym_cap_, (all_on_device ? V * vol : vol) * 2)) return 3;
    if (!keep && (!h_sym_ || h_sym_cap_ < total_bytes)) {
        if (h_sym_) (void)hipHostFree(h_sym_);
        h_sym_ = nullptr;
        h_sym_cap_ = 0;
        if (hipHostMalloc(&h_sym_, total_bytes, hipHostMallocDefault) != hipSuccess) return 3;
        h_sym_cap_ = total_bytes;
    }
    float pred_ms_total = 0.f;
    for (uint64_t v = 0; v < V; ++v) {
        const uint16_t* src;
        if (dev) {
            src = d_img + v * vol;
        } else {
            auto t0 = clk::now();
            if (hipMemcpyAsync(d_in_, (const uint16_t*)img + v * vol, vol * 2, hipMemcpyHostToDevice, stream_) !=
                hipSuccess)
                return 3;
            if (hipStreamSynchronize(stream_) != hipSuccess) return 3;
            if (st) st->h2d_ms += ms_since(t0);
            src = (const uint16_t*)d_in_;
        }
        if (v == 0 && autosel) {
            // selection on frame 0 of volume (c=0, t=0) (klb_imageIO.cpp:2316-2360),
            // or on the whole stack's frame 0 handed in for a slab
            auto t0 = clk::now();
            const size_t need = lfm_hip_select_workspace_bytes((int)W, (int)H);
            if (!dev_alloc(d_ws_, d_ws_cap_, need)) return 3;
            const uint16_t* sel = src;
            if (slab.select_frame) {
                if (dev) {
                    sel = (const uint16_t*)slab.select_frame;
                } else {
                    if (!dev_alloc(d_sel_, d_sel_cap_, W * H * 2)) return 3;
                    if (hipMemcpyAsync(d_sel_, slab.select_frame, W * H * 2, hipMemcpyHostToDevice, stream_) !=
                        hipSuccess)
                        return 3;
                    sel = (const uint16_t*)d_sel_;
                }
            } else if (slab.z0 > 0) {
                return 3;  // a slab's own frame 0 is not the stack's: the caller must hand that frame in
            }
            float ent[8];
            int chosen = 0;
            int rc = lfm_hip_select(sel, (int)W, (int)H, T, fam, ent, &chosen, d_ws_, stream_);
            if (rc != LFM_HIP_OK) return 3;
            k = chosen;
            if (st) {
                st->select_ms += ms_since(t0);
                std::memcpy(st->entropy, ent, sizeof(ent));
            }
        }
        uint16_t* dst = (uint16_t*)d_sym_ + (all_on_device ? v * vol : 0);
        (void)hipEventRecord(ev0_, stream_);
        int rc = lfm_hip_predict(src, d_prev, dst, (int)W, (int)H, (int)Z, T, fam, k, video, (int)slab.z0, stream_);
        (void)hipEventRecord(ev1_, stream_);
        if (rc != LFM_HIP_OK) return 3;
        if (!all_on_device) {
            auto t0 = clk::now();
            if (hipMemcpyAsync((uint8_t*)h_sym_ + v * vol * 2, dst, vol * 2, hipMemcpyDeviceToHost, stream_) !=
                hipSuccess)
                return 3;
            if (hipStreamSynchronize(stream_) != hipSuccess) return 3;
            if (st) st->d2h_ms += ms_since(t0);
        } else if (hipEventSynchronize(ev1_) != hipSuccess) {
            return 3;
        }
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, ev0_, ev1_);
        pred_ms_total += ms;
    }
    if (st) st->predict_ms += pred_ms_total;
    h.headerVersion = (uint8_t)((hv & 0x80) | k);
    if (st) st->chosen = k;
    if (video && fam != 0 && k != 0 && Z > 1) {
        // the reference writes these bytes (reproduced), but its temporal
        // residual ((I - pred) + P) >> 1 drops a bit: no reader can restore
        // the odd frames (lfm_Predictors_space.cu:114-177, _angle.cu:136-192)
        std::fprintf(stderr, "WARNING: video stack with the %s predictor family: the odd frames are coded with the "
                             "reference's lossy temporal residual and cannot be decoded exactly\n",
                     fam == 1 ? "angle" : "space");
    }
    if (keep) {
        *dsym = (const uint8_t*)d_sym_;
        return 0;
    }
    if (dev) {
        auto t0 = clk::now();
        if (hipMemcpyAsync(h_sym_, d_sym_, total_bytes, hipMemcpyDeviceToHost, stream_) != hipSuccess) return 3;
        if (hipStreamSynchronize(stream_) != hipSuccess) return 3;
        if (st) st->d2h_ms += ms_since(t0);
    }
    *sym = (const uint8_t*)h_sym_;
    return 0;
}

// GPU bzip2 of every block (lfm_bzip2.hip), streams batched to bound the
// workspace; streams the device hands back (RLE1 block reaching nblockMAX,
// periodic blocks) are compressed by libbz2 here.  Same bytes either way.
int Encoder::gpu_compress(const uint8_t* d_sym, klb_image_header& h, Sink& sink, lfm_encode_stats* st, int level,
                          int set, Inflight* fly)
{
    void*& h_sym_ = this->h_sym_[set];
    size_t& h_sym_cap_ = this->h_sym_cap_[set];
    BzSlot* bz_ = this->bz_[set];
    const BlockGrid g(h);
    const uint64_t nblocks = g.nblocks;
    h.resizeBlockOffset(nblocks);
    const size_t bpp = h.getBytesPerPixel();
    const uint32_t block_bytes = h.getBlockSizeBytes();
    if (level < 1) level = bzip2_level(h);
    const size_t out_cap = ((size_t)block_bytes + block_bytes / 50 + 4096 + 255) / 256 * 256;
    const size_t rle_cap = ((size_t)block_bytes + block_bytes / 4 + 64 + 255) / 256 * 256;
    // Batches run in a pipeline of kBzSlots HIP streams (one host thread
    // each): one batch's latency-bound stages (MTF, Huffman tables, the
    // host-synchronised doubling rounds) overlap another batch's sorts.  The
    // workspace budget (env LFM_BZ2_GPU_BUDGET_MB, default 48 GiB) is split
    // between the slots.
    static const size_t budget = [] {
        const char* e = std::getenv("LFM_BZ2_GPU_BUDGET_MB");
        const long v = e ? std::atol(e) : 0;
        return (size_t)(v > 0 ? v : 48 * 1024) << 20;
    }();
    const size_t per_stream = lfm_hip_bzip2_workspace_bytes(1, block_bytes) + out_cap;
    // one batch per slot (smaller batches, so the in-order writer's copies
    // overlap later batches' kernels, measured slower: the latency-bound
    // stages cost per batch)
    const int slots = bz_slot_count();
    const uint64_t nway = slots;
    uint64_t batch = std::max<uint64_t>(1, std::min<uint64_t>((nblocks + nway - 1) / nway,
                                                                budget / slots / per_stream));
    batch = std::min<uint64_t>(batch, ((1ull << 32) - 1) / rle_cap);
    const uint64_t nbatch = (nblocks + batch - 1) / batch;
    const int nslots = (int)std::min<uint64_t>(slots, nbatch);
    const size_t ws = lfm_hip_bzip2_workspace_bytes((uint32_t)batch, block_bytes);
    for (int k = 0; k < nslots; ++k) {
        BzSlot& sl = bz_[k];
        if (!sl.stream && hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking) != hipSuccess) return 3;
        if (!dev_alloc(sl.d_ws, sl.d_ws_cap, ws)) return 3;
        if (!dev_alloc(sl.d_out, sl.d_out_cap, batch * out_cap)) return 3;
        if (!sl.h_out || sl.h_out_cap < batch * out_cap) {
            if (sl.h_out) (void)hipHostFree(sl.h_out);
            sl.h_out = nullptr;
            sl.h_out_cap = 0;
            if (hipHostMalloc(&sl.h_out, batch * out_cap, hipHostMallocDefault) != hipSuccess) return 3;
            sl.h_out_cap = batch * out_cap;
        }
    }
    uint32_t dims[5], bs[5];
    for (int d = 0; d < 5; ++d) {
        dims[d] = h.xyzct[d];
        bs[d] = h.blockSize[d];
    }
    // per batch: sizes / flags, and the ready / consumed hand-shake with the
    // in-order writer below (slot k reuses its buffers for batch b + kBzSlots)
    std::vector<std::vector<uint64_t>> sizes(nbatch);
    std::vector<std::vector<uint32_t>> flags(nbatch);
    std::vector<int> state(nbatch, 0);  // 0 pending, 1 ready, 2 consumed, -1 failed
    // a sink backed by pinned memory takes each batch's payload straight from
    // the device, in order, at its final offset (no host copy of the blocks)
    const bool direct = sink.direct_capable();
    std::vector<char> staged(nbatch, 1);
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<bool> abort_all{false};
    std::vector<double> d2h(nslots, 0.0);
    std::vector<std::array<double, 5>> stage_ms(nslots);  // per slot, summed over its batches
    for (auto& a : stage_ms) a.fill(0.0);
    // pipelined encodes: the next submit starts once every batch of the last
    // round has run its kernels (releasing it after the BWT or the MTF of
    // those batches measured equal or slower: the next stack's kernels slow
    // this one's latency-bound Huffman chains as much as they gain; staggering
    // the two slots measured slower too, their latency-bound stages overlap
    // each other in lockstep)
    // host stack still uploading (start_upload): a batch waits for the chunks
    // holding its last block (blocks run x -> y -> z -> c -> t, so that block
    // reaches furthest into the flattened (t, c, z) frame order)
    UploadPipe* up = nullptr;
    {
        std::lock_guard<std::mutex> lk(up_[set].mu);
        if (up_[set].active) up = &up_[set];
    }
    auto frames_needed = [&](uint64_t last_block) -> uint64_t {
        uint64_t o[5], sz[5];
        g.block(last_block, o, sz);
        return ((o[4] + sz[4] - 1) * h.xyzct[3] + (o[3] + sz[3] - 1)) * (uint64_t)h.xyzct[2] + o[2] + sz[2];
    };
    if (fly) {
        std::lock_guard<std::mutex> lk(fly->mu);
        fly->need = (int)std::min<uint64_t>(nslots, nbatch);
    }
    auto worker = [&](int k) {
        (void)hipSetDevice(device_);
        BzSlot& sl = bz_[k];
        for (uint64_t b = k; b < nbatch; b += nslots) {
            if (b >= (uint64_t)nslots) {  // wait until the writer consumed batch b - nslots
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return state[b - nslots] != 1 || abort_all.load(); });
                if (abort_all.load() || state[b - nslots] < 0) break;
            }
            const uint64_t b0 = b * batch;
            const uint32_t cnt = (uint32_t)std::min<uint64_t>(batch, nblocks - b0);
            sizes[b].assign(cnt, 0);
            flags[b].assign(cnt, 0);
            if (up && up->wait_frames(frames_needed(b0 + cnt - 1), sl.stream)) {
                std::lock_guard<std::mutex> lk(mu);
                state[b] = -1;
                cv.notify_all();
                break;
            }
            // the slot's last batch releases the next encode once its Huffman
            // tables are done (stage hook 3), so the next encode's first
            // kernels queue while this one's emission and copies finish
            const bool last = fly && b + nslots >= nbatch;
            struct ReachOnce {
                Inflight* f;
                bool done;
            } ro{fly, false};
            // (measured +2.6 % end to end against the release after the
            // batch's last copy: the ~0.45 ms host turnaround between two
            // encodes' kernels is hidden, profiles/r05_ab_early_release.jsonl)
            if (last)
                lfm_hip_bzip2_set_stage_hook(
                    [](void* c, int stage) {
                        auto* r = (ReachOnce*)c;
                        if (stage == 2) r->f->reach2();
                        if (stage == 3 && !r->done) {
                            r->done = true;
                            r->f->reach();
                        }
                    },
                    &ro);
            int ok = lfm_hip_bzip2_blocks(d_sym, dims, bs, (uint32_t)bpp, (uint32_t)b0, cnt, (uint32_t)level, sl.d_ws,
                                          ws, sl.d_out, sizes[b].data(), flags[b].data(), sl.stream) == LFM_HIP_OK;
            if (last) {
                lfm_hip_bzip2_set_stage_hook(nullptr, nullptr);
                if (!ro.done) fly->reach();
            }
            float sm[5];
            if (ok && lfm_hip_bzip2_last_stage_ms(sm) == 0)
                for (int i = 0; i < 5; ++i) stage_ms[k][i] += sm[i];
            bool any_flag = false;
            for (uint32_t i = 0; i < cnt; ++i) any_flag |= flags[b][i] != 0;
            staged[b] = !direct || any_flag;
            if (ok && staged[b]) {  // through the pinned staging buffer (the writer copies block by block)
                uint64_t tot = 0;
                for (uint32_t i = 0; i < cnt; ++i) tot += sizes[b][i];
                auto t0 = clk::now();
                ok = payload_d2h(sl.h_out, sl.d_out, tot, sl.stream);
                d2h[k] += ms_since(t0);
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                state[b] = ok ? 1 : -1;
            }
            cv.notify_all();
            if (!ok) break;
        }
    };
    std::vector<std::thread> pool;
    for (int k = 0; k < nslots; ++k) pool.emplace_back(worker, k);

    const uint8_t* h_all = nullptr;  // host copy of the symbols, only if a stream needs the host library
    std::vector<uint8_t> in(block_bytes), out((size_t)std::ceil((float)block_bytes * 2.0f + 50.0f));
    int rc = sink.begin(h);
    if (direct) sink.reserve_hint(h.getSizeInBytes() + nblocks * out_cap);
    uint64_t offset = 0;
    for (uint64_t b = 0; b < nbatch && !rc; ++b) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return state[b] != 0; });
            if (state[b] < 0) rc = 3;
        }
        if (rc) break;
        const uint64_t b0 = b * batch;
        const uint32_t cnt = (uint32_t)sizes[b].size();
        if (!staged[b]) {
            uint64_t tot = 0;
            for (uint32_t i = 0; i < cnt; ++i) tot += sizes[b][i];
            BzSlot& sl = bz_[b % nslots];
            uint8_t* dst = sink.direct(tot);
            if (!dst) {
                rc = 3;
            } else {
                auto t0 = clk::now();
                if (!payload_d2h(dst, sl.d_out, tot, sl.stream)) rc = 3;
                if (st) st->d2h_ms += ms_since(t0);
            }
            for (uint32_t i = 0; i < cnt; ++i) {
                offset += sizes[b][i];
                h.blockOffset[b0 + i] = offset;
            }
        }
        const uint8_t* p = (const uint8_t*)bz_[b % nslots].h_out;
        for (uint32_t i = 0; i < cnt && !rc && staged[b]; ++i) {
            if (flags[b][i]) {
                if (!h_all) {
                    const size_t bytes = h.getImageSizeBytes();
                    if (!h_sym_ || h_sym_cap_ < bytes) {
                        if (h_sym_) (void)hipHostFree(h_sym_);
                        h_sym_ = nullptr;
                        h_sym_cap_ = 0;
                        if (hipHostMalloc(&h_sym_, bytes, hipHostMallocDefault) != hipSuccess) { rc = 3; break; }
                        h_sym_cap_ = bytes;
                    }
                    // on this batch's own HIP stream: stream_ belongs to the
                    // caller thread's next submit (its predictor stage)
                    hipStream_t fs = bz_[b % nslots].stream;
                    if ((up && up->wait_frames(~0ull, fs)) ||
                        hipMemcpyAsync(h_sym_, d_sym, bytes, hipMemcpyDeviceToHost, fs) != hipSuccess ||
                        hipStreamSynchronize(fs) != hipSuccess) {
                        rc = 3;
                        break;
                    }
                    h_all = (const uint8_t*)h_sym_;
                }
                size_t n = 0;
                gather_block(h_all, g, b0 + i, bpp, in.data(), &n);
                uint32_t len = 0;
                rc = compress_one(BZIP2, in.data(), (uint32_t)n, out.data(), (uint32_t)out.size(), &len, level);
                if (!rc) rc = sink.append(out.data(), len);
                offset += len;
            } else {
                rc = sink.append(p, sizes[b][i]);
                p += sizes[b][i];
                offset += sizes[b][i];
            }
            h.blockOffset[b0 + i] = offset;
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            state[b] = 2;
            if (rc) abort_all = true;
        }
        cv.notify_all();
    }
    if (rc) {
        std::lock_guard<std::mutex> lk(mu);
        abort_all = true;
    }
    cv.notify_all();
    for (auto& t : pool) t.join();
    if (st) {
        for (double v : d2h) st->d2h_ms += v;
        for (int i = 0; i < 5; ++i)
            for (int k = 0; k < nslots; ++k) st->bz_stage_ms[i] = std::max(st->bz_stage_ms[i], stage_ms[k][i]);
        st->bz_in_bytes = nblocks * (uint64_t)block_bytes;
    }
    if (rc) return rc;
    return sink.finish(h);
}

int normalize_header(klb_image_header& h)
{
    if (h.getBytesPerPixel() == 0) return 5;
    for (int d = 0; d < KLB_DATA_DIMS; ++d) {
        if (h.xyzct[d] == 0) return 3;
        if (h.blockSize[d] == 0) h.blockSize[d] = 1;
        h.blockSize[d] = std::min(h.blockSize[d], h.xyzct[d]);  // klb_imageIO.cpp:2402-2404
    }
    if (h.compressionType != NONE && h.compressionType != BZIP2 && h.compressionType != ZLIB) {
        std::printf("ERROR: compression type %d not implemented\n", (int)h.compressionType);
        return 5;
    }
    return 0;
}

// selection for submit: on the slab's select_frame, else on frame 0 of the image
// A device input was written by the caller's kernels, typically on the null
// stream (torch's default stream, lfm_hip_synth without a stream); the
// encoder's streams are non-blocking, so they would not wait for that work:
// the encoder's stream waits for an event recorded on the null stream.  (A
// producer on another stream must be synchronised by the caller; the Python
// binding does that for torch's current stream.)
int Encoder::after_caller(bool dev)
{
    if (!dev) return 0;
    if (int rc = ensure_gpu()) return rc;
    (void)hipSetDevice(device_);
    if (!caller_ev_ && hipEventCreateWithFlags(&caller_ev_, hipEventDisableTiming) != hipSuccess) {
        caller_ev_ = nullptr;
        return 3;
    }
    return hipEventRecord(caller_ev_, nullptr) == hipSuccess && hipStreamWaitEvent(stream_, caller_ev_, 0) == hipSuccess
               ? 0
               : 3;
}

int Encoder::preselect(const void* img, bool dev, const klb_image_header& h, const SlabSpec& slab, int* k,
                       float ent[8])
{
    if (int rc = ensure_gpu()) return rc;
    (void)hipSetDevice(device_);
    const int W = (int)h.xyzct[0], H = (int)h.xyzct[1];
    if (W <= 0 || H <= 0) return 3;
    const void* frame = slab.select_frame ? slab.select_frame : (slab.z0 > 0 ? nullptr : img);
    if (!frame) return 3;  // a slab's own frame 0 is not the stack's
    if (!dev) return select_host_frame(frame, W, H, h.Nnum, current_family(), k, ent);
    if (!dev_alloc(d_ws_, d_ws_cap_, lfm_hip_select_workspace_bytes(W, H))) return 3;
    return lfm_hip_select((const uint16_t*)frame, W, H, h.Nnum, current_family(), ent, k, d_ws_, stream_) ==
                   LFM_HIP_OK
               ? 0
               : 3;
}

int Encoder::select_host_frame(const void* frame, int W, int H, int T, int family, int* chosen, float entropy[8])
{
    if (int rc = ensure_gpu()) return rc;
    (void)hipSetDevice(device_);
    const size_t bytes = (size_t)W * H * 2;
    if (!dev_alloc(d_in_, d_in_cap_, bytes)) return 3;
    if (!dev_alloc(d_ws_, d_ws_cap_, lfm_hip_select_workspace_bytes(W, H))) return 3;
    if (hipMemcpyAsync(d_in_, frame, bytes, hipMemcpyHostToDevice, stream_) != hipSuccess) return 3;
    return lfm_hip_select((const uint16_t*)d_in_, W, H, T, family, entropy, chosen, d_ws_, stream_) == LFM_HIP_OK ? 0
                                                                                                               : 3;
}

int Encoder::encode(const void* img, bool dev, klb_image_header& h, Sink& sink, lfm_encode_stats* st, int threads,
                    const SlabSpec* slab)
{
    join_inflight();  // a synchronous encode may use either buffer set
    return encode_set(img, dev, h, sink, st, threads, slab, 0);
}

int Encoder::encode_set(const void* img, bool dev, klb_image_header& h, Sink& sink, lfm_encode_stats* st,
                        int threads, const SlabSpec* slab, int set)
{
    static const SlabSpec whole;
    if (threads <= 0) threads = default_threads();
    auto t0 = clk::now();
    if (st) std::memset(st, 0, sizeof(*st));
    // a z-slab that starts past frame 0 lies in a stack at least one nominal
    // block deeper than its start, so the stack's nominal block keeps the
    // requested depth even where the slab's own last layer is shallower
    int level = slab ? slab->level : -1;
    if (level < 1 && slab && slab->z0 > 0 && h.getBytesPerPixel()) {
        klb_image_header nominal(h);
        for (int d = 0; d < KLB_DATA_DIMS; ++d)
            if (d != 2 && nominal.blockSize[d]) nominal.blockSize[d] = std::min(nominal.blockSize[d], h.xyzct[d]);
        if (nominal.blockSize[2] == 0) nominal.blockSize[2] = 1;
        level = bzip2_level(nominal);
    }
    if (int rc = normalize_header(h)) return rc;
    if (int rc = after_caller(dev)) return rc;
    const uint8_t* sym = nullptr;
    const uint8_t* dsym = nullptr;
    const bool gpu_bz = use_gpu_bzip2(h, dev);
    int rc = predictor_stage(img, dev, h, &sym, gpu_bz ? &dsym : nullptr, st, slab ? *slab : whole, set);
    if (rc) return rc;
    auto tc = clk::now();
    if (gpu_bz) {
        if ((rc = ensure_gpu())) {
            up_[set].join();
            return rc;
        }
        rc = gpu_compress(dsym, h, sink, st, level, set, nullptr);
        UploadPipe& up = up_[set];
        if (up.active) {  // the host image is read until the uploader is done
            up.join();
            if (!rc) rc = up.rc;
            if (st) {
                st->h2d_ms += up.h2d_ms;
                st->predict_ms += up.predict_ms;
            }
        }
    } else {
        rc = compress_blocks(sym, h, sink, threads, level);
    }
    if (st) {
        st->compress_ms = ms_since(tc);
        st->total_ms = ms_since(t0);
        st->header_version = h.headerVersion;
        st->chosen = h.headerVersion & 0x7F;
        st->out_bytes = h.getCompressedFileSizeInBytes();
    }
    return rc;
}

// ------------------------------------------------------------ z-slab merge --
int merge_slabs(const uint8_t* const* slabs, const uint64_t* lens, int n, std::vector<uint8_t>* out)
{
    if (n <= 0 || !slabs || !lens || !out) return 3;
    std::vector<klb_image_header> hs(n);
    for (int i = 0; i < n; ++i)
        if (hs[i].parseHeader(slabs[i], lens[i])) return 3;
    const klb_image_header& h0 = hs[0];
    if (h0.xyzct[3] != 1 || h0.xyzct[4] != 1) return 3;
    const uint32_t bz = h0.blockSize[2];
    uint64_t Z = 0, nb = 0, payload = 0;
    for (int i = 0; i < n; ++i) {
        const klb_image_header& hi = hs[i];
        bool same = hi.xyzct[0] == h0.xyzct[0] && hi.xyzct[1] == h0.xyzct[1] && hi.xyzct[3] == 1 &&
                    hi.xyzct[4] == 1 && hi.dataType == h0.dataType && hi.compressionType == h0.compressionType &&
                    hi.headerVersion == h0.headerVersion && hi.Nnum == h0.Nnum &&
                    std::memcmp(hi.pixelSize, h0.pixelSize, sizeof(h0.pixelSize)) == 0 &&
                    std::memcmp(hi.metadata, h0.metadata, KLB_METADATA_SIZE) == 0 &&
                    hi.blockSize[0] == h0.blockSize[0] && hi.blockSize[1] == h0.blockSize[1];
        if (i + 1 < n) same = same && hi.blockSize[2] == bz && hi.xyzct[2] % bz == 0;
        else same = same && hi.blockSize[2] == std::min(bz, hi.xyzct[2]);
        if (!same) {
            std::printf("ERROR: slab %d does not continue slab 0 (dims, type, predictor or block depth)\n", i);
            return 3;
        }
        const uint64_t hsz = hi.getSizeInBytes();
        const uint64_t body = hi.Nb ? hi.blockOffset[hi.Nb - 1] : 0;
        if (hsz + body > lens[i]) return 3;
        Z += hi.xyzct[2];
        nb += hi.Nb;
        payload += body;
    }
    klb_image_header H = h0;
    H.xyzct[2] = (uint32_t)Z;
    H.resizeBlockOffset(H.calculateNumBlocks());
    if (H.Nb != nb) return 3;
    uint64_t acc = 0, b = 0;
    for (int i = 0; i < n; ++i) {
        uint64_t prev_end = 0;
        for (size_t j = 0; j < hs[i].Nb; ++j) {
            acc += hs[i].blockOffset[j] - prev_end;
            prev_end = hs[i].blockOffset[j];
            H.blockOffset[b++] = acc;
        }
    }
    const size_t hsz = H.getSizeInBytes();
    out->assign(hsz + payload, 0);
    H.serialize(out->data(), hsz);
    uint8_t* dst = out->data() + hsz;
    for (int i = 0; i < n; ++i) {
        const uint64_t body = hs[i].Nb ? hs[i].blockOffset[hs[i].Nb - 1] : 0;
        std::memcpy(dst, slabs[i] + hs[i].getSizeInBytes(), body);
        dst += body;
    }
    return 0;
}

// ---------------------------------------------------------------- decode --
namespace {
struct HostNb {
    const uint16_t* f;
    int W, T, x, y;
    template <int N>
    int at() const
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

// prediction (spatial) or temporal prediction of the tiles family for a case
template <int FAM, int K, int TC, int UC, bool TEMP>
inline int inv_case(HostNb& g, int r, int P)
{
    constexpr int F = case_formula(FAM, K, TC, UC);
    const int pr = eval_formula<F>(g);
    if constexpr (!TEMP) return r + pr;
    else if constexpr (F == F_Z) return r + P;
    else return r + ((pr + P) >> 1);  // tiles: I = r + ((pred + P) >> 1)
}

template <int FAM, int K, bool TEMP>
void unpredict_frame(const uint16_t* sym, const uint16_t* prev, uint16_t* out, int W, int H, int T)
{
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            HostNb g{out, W, T, x, y};
            const int tx = x / T, ty = y / T, u = x % T, v = y % T;
            const int tc = tx == 0 ? (ty == 0 ? 0 : 1) : (ty == 0 ? 2 : 3);
            const int uc = u == 0 ? (v > 0 ? 0 : 1) : (v == 0 ? 2 : 3);
            const int r = unsymbolize16(sym[(size_t)y * W + x]);
            const int P = TEMP ? (int)prev[(size_t)y * W + x] : 0;
            int val = 0;
            switch (tc * 4 + uc) {
#define LFM_INV(TC_, UC_) case TC_ * 4 + UC_: val = inv_case<FAM, K, TC_, UC_, TEMP>(g, r, P); break;
            LFM_INV(0, 0) LFM_INV(0, 1) LFM_INV(0, 2) LFM_INV(0, 3)
            LFM_INV(1, 0) LFM_INV(1, 1) LFM_INV(1, 2) LFM_INV(1, 3)
            LFM_INV(2, 0) LFM_INV(2, 1) LFM_INV(2, 2) LFM_INV(2, 3)
            LFM_INV(3, 0) LFM_INV(3, 1) LFM_INV(3, 2) LFM_INV(3, 3)
#undef LFM_INV
            }
            out[(size_t)y * W + x] = (uint16_t)val;
        }
}

template <int FAM>
int unpredict_dispatch_k(int k, bool temp, const uint16_t* sym, const uint16_t* prev, uint16_t* out, int W, int H,
                         int T)
{
#define LFM_K(K_)                                                                          \
    case K_:                                                                               \
        if (temp) unpredict_frame<FAM, K_, true>(sym, prev, out, W, H, T);                 \
        else unpredict_frame<FAM, K_, false>(sym, prev, out, W, H, T);                     \
        return 0;
    switch (k) { LFM_K(1) LFM_K(2) LFM_K(3) LFM_K(4) LFM_K(5) LFM_K(6) LFM_K(7) }
#undef LFM_K
    return 3;
}

int unpredict_one(int fam, int k, bool temp, const uint16_t* sym, const uint16_t* prev, uint16_t* out, int W, int H,
                  int T)
{
    if (temp && fam != 0) return LFM_HIP_ENOTINV;  // r = ((I - pred) + P) >> 1 drops a bit
    switch (fam) {
    case 0: return unpredict_dispatch_k<0>(k, temp, sym, prev, out, W, H, T);
    case 1: return unpredict_dispatch_k<1>(k, temp, sym, prev, out, W, H, T);
    case 2: return unpredict_dispatch_k<2>(k, temp, sym, prev, out, W, H, T);
    }
    return 3;
}

template <class F>
void parallel_for(uint64_t n, int threads, F&& f)
{
    std::atomic<uint64_t> next{0};
    auto w = [&]() {
        for (;;) {
            uint64_t i = next.fetch_add(1);
            if (i >= n) break;
            f(i);
        }
    };
    threads = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(threads, 1), n));
    std::vector<std::thread> pool;
    for (int i = 1; i < threads; ++i) pool.emplace_back(w);
    w();
    for (auto& t : pool) t.join();
}

// Host <-> device copies of pageable buffers through two pinned staging
// chunks: the DMA of one chunk overlaps the multi-threaded host copy of the
// other (the runtime's own staging copies with one thread and takes the page
// faults of a fresh destination on that thread).  The pinned chunks and their
// events are kept per host thread and device.
struct Staging {
    static constexpr size_t kChunk = 32u << 20;
    void* buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool used[2] = {false, false};
    int dev = -1;
    Staging() = default;
    Staging(const Staging&) = delete;
    Staging& operator=(const Staging&) = delete;
    ~Staging() { release(); }  // a worker thread that exits frees its pinned chunks
    void release()
    {
        for (int i = 0; i < 2; ++i) {
            if (ev[i]) (void)hipEventDestroy(ev[i]);
            if (buf[i]) (void)hipHostFree(buf[i]);
            ev[i] = nullptr;
            buf[i] = nullptr;
            used[i] = false;
        }
        dev = -1;
    }
    bool ready()
    {
        int d = 0;
        if (hipGetDevice(&d) != hipSuccess) return false;
        if (dev == d && buf[0]) return true;
        for (int i = 0; i < 2; ++i) {
            if (ev[i]) (void)hipEventDestroy(ev[i]);
            ev[i] = nullptr;
            if (!buf[i] && hipHostMalloc(&buf[i], kChunk, hipHostMallocPortable) != hipSuccess) {
                buf[i] = nullptr;
                return false;
            }
            if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) return false;
        }
        dev = d;
        return true;
    }
};

Staging& staging()
{
    static thread_local Staging s;  // the pinned chunks stay for the thread's life
    return s;
}

// Multi-threaded memcpy on a persistent pool: the staged copies run one
// 32 MiB chunk at a time, and starting and joining 15 threads per chunk
// (parallel_for) cost about as much as the copy.  A copy is split into 1 MiB
// pieces that the caller and up to threads - 1 pool workers take in turn;
// several callers (the decode's upload and download threads) share the pool.
// The pool is never destroyed (its workers may still wait on it at exit).
struct CopyPool {
    struct Job {
        uint8_t* dst;
        const uint8_t* src;
        size_t n, piece;
        uint64_t np;
        int helpers;                      // pool workers still allowed to join
        int active = 0;                   // pool workers inside run() (under mu)
        std::atomic<uint64_t> next{0}, done{0};
    };
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::vector<Job*> jobs;
    int nthreads = 0;
    static void run(Job& j)
    {
        for (;;) {
            const uint64_t i = j.next.fetch_add(1);
            if (i >= j.np) return;
            const size_t o = i * j.piece;
            std::memcpy(j.dst + o, j.src + o, std::min(j.piece, j.n - o));
            j.done.fetch_add(1);
        }
    }
    void worker()
    {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return !jobs.empty(); });
            Job* j = nullptr;
            for (Job* c : jobs)
                if (c->helpers > 0 && c->next.load() < c->np) {
                    j = c;
                    break;
                }
            if (!j) {  // every queued job is fully handed out: wait for the next one
                cv.wait(lk);
                continue;
            }
            --j->helpers;
            ++j->active;
            lk.unlock();
            run(*j);
            lk.lock();
            --j->active;  // (the last touch of the job: its owner waits for this under mu)
            done_cv.notify_all();
        }
    }
    void copy(void* dst, const void* src, size_t n, int threads)
    {
        Job j;
        j.dst = (uint8_t*)dst;
        j.src = (const uint8_t*)src;
        j.n = n;
        j.piece = 1u << 20;
        j.np = (n + j.piece - 1) / j.piece;
        {
            std::lock_guard<std::mutex> lk(mu);
            while (nthreads < threads - 1) {
                std::thread(&CopyPool::worker, this).detach();
                ++nthreads;
            }
            j.helpers = (int)std::min<uint64_t>((uint64_t)threads - 1, j.np - 1);
            jobs.push_back(&j);
        }
        cv.notify_all();
        run(j);
        std::unique_lock<std::mutex> lk(mu);
        done_cv.wait(lk, [&] { return j.done.load() == j.np && j.active == 0; });
        jobs.erase(std::find(jobs.begin(), jobs.end(), &j));
    }
};

void par_memcpy_impl(void* dst, const void* src, size_t n, int threads)
{
    const size_t piece = 1u << 20;
    const uint64_t np = (n + piece - 1) / piece;
    if (threads <= 1 || np <= 1) {
        std::memcpy(dst, src, n);
        return;
    }
    static CopyPool* pool = new CopyPool;  // (never destroyed, see CopyPool)
    pool->copy(dst, src, n, std::min(threads, 64));
}

bool staged_h2d(void* d_dst, const void* h_src, size_t n, hipStream_t st, int threads)
{
    Staging& S = staging();
    if (!S.ready()) return hipMemcpyAsync(d_dst, h_src, n, hipMemcpyHostToDevice, st) == hipSuccess;
    static const bool timing = env_int("LFM_DECODE_TIMING", 0) != 0;
    double t_wait = 0, t_copy = 0;
    auto now = [] { return std::chrono::steady_clock::now(); };
    for (size_t off = 0, i = 0; off < n; off += Staging::kChunk, ++i) {
        const int b = (int)(i & 1);
        const size_t len = std::min(Staging::kChunk, n - off);
        auto t0 = now();
        if (S.used[b] && hipEventSynchronize(S.ev[b]) != hipSuccess) return false;
        auto t1 = now();
        par_memcpy_impl(S.buf[b], (const uint8_t*)h_src + off, len, threads);
        auto t2 = now();
        t_wait += std::chrono::duration<double, std::milli>(t1 - t0).count();
        t_copy += std::chrono::duration<double, std::milli>(t2 - t1).count();
        if (timing && off + len >= n)
            std::fprintf(stderr, "staged h2d: %zu bytes, host copies %.2f ms, waits %.2f ms, %d threads\n", n, t_copy,
                         t_wait, threads);
        if (hipMemcpyAsync((uint8_t*)d_dst + off, S.buf[b], len, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipEventRecord(S.ev[b], st) != hipSuccess)
            return false;
        S.used[b] = true;
    }
    return true;
}

// Host -> device through the pinned chunks with the DMA on an SDMA engine
// (HSA): the host copy of one chunk overlaps the engine's copy of the other.
// The blit-kernel copies of hipMemcpyAsync ran the decode payload upload at
// 5-47 ms depending on the process's state; the engine does not depend on
// the CUs.  Returns false if HSA cannot take the copy (nothing was issued on
// a false return before the first chunk; the caller falls back).  The
// destination stream must be idle (the caller synchronises it).
// the wait state of the staged SDMA copies' signal waits (LFM_SDMA_WAIT: 0
// blocked, the default; 1 active)
hsa_wait_state_t sdma_wait_state()
{
    static const int m = env_int("LFM_SDMA_WAIT", 0);
    return m == 1 ? HSA_WAIT_STATE_ACTIVE : HSA_WAIT_STATE_BLOCKED;
}

bool sdma_staged_h2d(void* d_dst, const void* h_src, size_t n, int threads)
{
    const hsa_agent_t* cpu = hsa_cpu_agent();
    Staging& S = staging();
    if (!cpu || !S.ready() || n == 0) return false;
    hsa_amd_pointer_info_t info;
    std::memset(&info, 0, sizeof(info));
    info.size = sizeof(info);
    if (hsa_amd_pointer_info(d_dst, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        info.type != HSA_EXT_POINTER_TYPE_HSA)
        return false;
    hsa_signal_t sig[2];
    if (hsa_signal_create(0, 0, nullptr, &sig[0]) != HSA_STATUS_SUCCESS) return false;
    if (hsa_signal_create(0, 0, nullptr, &sig[1]) != HSA_STATUS_SUCCESS) {
        hsa_signal_destroy(sig[0]);
        return false;
    }
    bool ok = true;
    static const bool timing = env_int("LFM_DECODE_TIMING", 0) != 0;
    double t_wait = 0, t_copy = 0, t_first = 0;
    auto now = [] { return std::chrono::steady_clock::now(); };
    for (size_t off = 0, i = 0; ok && off < n; off += Staging::kChunk, ++i) {
        const int b = (int)(i & 1);
        const size_t len = std::min(Staging::kChunk, n - off);
        auto t0 = now();
        if (i >= 2) ok = hsa_signal_wait_scacquire(sig[b], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                                   sdma_wait_state()) == 0;
        if (!ok) break;
        auto t1 = now();
        par_memcpy_impl(S.buf[b], (const uint8_t*)h_src + off, len, threads);
        const double w = std::chrono::duration<double, std::milli>(t1 - t0).count();
        t_wait += w;
        if (i == 2) t_first = w;
        t_copy += std::chrono::duration<double, std::milli>(now() - t1).count();
        hsa_signal_store_relaxed(sig[b], 1);
        ok = hsa_amd_memory_async_copy((uint8_t*)d_dst + off, info.agentOwner, S.buf[b], *cpu, len, 0, nullptr,
                                       sig[b]) == HSA_STATUS_SUCCESS;
        if (!ok) hsa_signal_store_relaxed(sig[b], 0);
    }
    auto t_tail = now();
    for (int b = 0; b < 2; ++b)
        if (hsa_signal_wait_scacquire(sig[b], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, sdma_wait_state()) != 0)
            ok = false;
    if (timing)
        std::fprintf(stderr,
                     "sdma h2d: %zu bytes, host copies %.2f ms, waits %.2f ms (first %.2f), last copy %.2f ms, %d threads\n",
                     n, t_copy, t_wait, t_first, std::chrono::duration<double, std::milli>(now() - t_tail).count(),
                     threads);
    hsa_signal_destroy(sig[0]);
    hsa_signal_destroy(sig[1]);
    S.used[0] = S.used[1] = false;  // the chunks are free (no HIP event pending on them)
    return ok;
}

// Device -> host through the pinned chunks with the DMA on an SDMA engine:
// the engine copies chunk i + 1 while the host threads copy chunk i out (the
// blit kernel of hipMemcpyAsync would run on the CUs beside the next decode
// chunk's kernels).  The source must be complete (the caller synchronised its
// stream).  Returns false if HSA cannot take the copy before anything was
// issued (the caller falls back); a failure after that is reported as false too.
bool sdma_staged_d2h(void* h_dst, const void* d_src, size_t n, int threads, Staging& S)
{
    const hsa_agent_t* cpu = hsa_cpu_agent();
    if (!cpu || !S.ready() || n == 0) return false;
    hsa_amd_pointer_info_t info;
    std::memset(&info, 0, sizeof(info));
    info.size = sizeof(info);
    if (hsa_amd_pointer_info((void*)d_src, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        info.type != HSA_EXT_POINTER_TYPE_HSA)
        return false;
    hsa_signal_t sig[2];
    if (hsa_signal_create(0, 0, nullptr, &sig[0]) != HSA_STATUS_SUCCESS) return false;
    if (hsa_signal_create(0, 0, nullptr, &sig[1]) != HSA_STATUS_SUCCESS) {
        hsa_signal_destroy(sig[0]);
        return false;
    }
    const size_t nc = (n + Staging::kChunk - 1) / Staging::kChunk;
    auto issue = [&](size_t i) {
        const int b = (int)(i & 1);
        const size_t off = i * Staging::kChunk, len = std::min(Staging::kChunk, n - off);
        hsa_signal_store_relaxed(sig[b], 1);
        if (hsa_amd_memory_async_copy(S.buf[b], *cpu, (const uint8_t*)d_src + off, info.agentOwner, len, 0, nullptr,
                                      sig[b]) != HSA_STATUS_SUCCESS) {
            hsa_signal_store_relaxed(sig[b], 0);
            return false;
        }
        return true;
    };
    auto wait = [&](int b) {
        return hsa_signal_wait_scacquire(sig[b], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, sdma_wait_state()) == 0;
    };
    static const bool timing = env_int("LFM_DECODE_TIMING", 0) != 0;
    double t_wait = 0, t_copy = 0;
    auto now = [] { return std::chrono::steady_clock::now(); };
    bool ok = issue(0);
    for (size_t i = 0; ok && i < nc; ++i) {
        const int b = (int)(i & 1);
        if (i + 1 < nc) ok = issue(i + 1);
        auto t0 = now();
        if (!wait(b)) ok = false;
        if (!ok) break;
        auto t1 = now();
        const size_t off = i * Staging::kChunk, len = std::min(Staging::kChunk, n - off);
        par_memcpy_impl((uint8_t*)h_dst + off, S.buf[b], len, threads);
        t_wait += std::chrono::duration<double, std::milli>(t1 - t0).count();
        t_copy += std::chrono::duration<double, std::milli>(now() - t1).count();
    }
    for (int b = 0; b < 2; ++b) (void)wait(b);  // nothing still writes a chunk
    if (timing)
        std::fprintf(stderr, "sdma d2h: %zu bytes, host copies %.2f ms, waits %.2f ms, %d threads\n", n, t_copy, t_wait,
                     threads);
    hsa_signal_destroy(sig[0]);
    hsa_signal_destroy(sig[1]);
    S.used[0] = S.used[1] = false;
    return ok;
}

bool staged_d2h(void* h_dst, const void* d_src, size_t n, hipStream_t st, int threads, Staging& S)
{
    if (!S.ready())
        return hipMemcpyAsync(h_dst, d_src, n, hipMemcpyDeviceToHost, st) == hipSuccess &&
               hipStreamSynchronize(st) == hipSuccess;
    const size_t nc = (n + Staging::kChunk - 1) / Staging::kChunk;
    auto issue = [&](size_t i) {
        const int b = (int)(i & 1);
        const size_t off = i * Staging::kChunk, len = std::min(Staging::kChunk, n - off);
        S.used[b] = true;
        return hipMemcpyAsync(S.buf[b], (const uint8_t*)d_src + off, len, hipMemcpyDeviceToHost, st) == hipSuccess &&
               hipEventRecord(S.ev[b], st) == hipSuccess;
    };
    for (size_t i = 0; i < std::min<size_t>(2, nc); ++i)
        if (!issue(i)) return false;
    for (size_t i = 0; i < nc; ++i) {
        const int b = (int)(i & 1);
        const size_t off = i * Staging::kChunk, len = std::min(Staging::kChunk, n - off);
        if (hipEventSynchronize(S.ev[b]) != hipSuccess) return false;
        par_memcpy_impl((uint8_t*)h_dst + off, S.buf[b], len, threads);
        if (i + 2 < nc && !issue(i + 2)) return false;
    }
    return true;
}

// Device buffers, streams and pinned status arrays of the GPU decode, kept
// per host thread and device between calls (LFM_DECODE_KEEP=0 releases them
// after every call): fresh device allocations are cleared by the driver
// before first use, which showed up as 20-40 ms stalls of the first upload.
// Two slots (stream, workspace, block buffer, lens / flags) for the pipelined
// chunks of gpu_decode.
struct DecodeBuffers {
    static constexpr int kSlots = 3;
    enum { PAY, SYM, OUT, WS0, BLK0 = WS0 + kSlots, N = BLK0 + kSlots };
    int dev = -1;
    hipStream_t st[kSlots] = {};
    hipStream_t dl = nullptr;                // the downloads' device -> pinned copies
    void* p[N] = {};
    size_t cap[N] = {};
    uint32_t* hs[kSlots] = {};  // pinned: lens then flags, per slot
    size_t hs_cap[kSlots] = {};
    int* us = nullptr;          // pinned: the inverse predictor's status words, per (chunk, volume piece)
    size_t us_cap = 0;
    Staging down;                            // the download thread's pinned chunks
    DecodeBuffers() = default;
    DecodeBuffers(const DecodeBuffers&) = delete;
    DecodeBuffers& operator=(const DecodeBuffers&) = delete;
    ~DecodeBuffers() { release(); }  // a worker thread that exits frees its device buffers
    void release()
    {
        for (int i = 0; i < N; ++i) {
            if (p[i]) (void)hipFree(p[i]);
            p[i] = nullptr;
            cap[i] = 0;
        }
        if (us) (void)hipHostFree(us);
        us = nullptr;
        us_cap = 0;
        for (int k = 0; k < kSlots; ++k) {
            if (hs[k]) (void)hipHostFree(hs[k]);
            hs[k] = nullptr;
            hs_cap[k] = 0;
            if (st[k]) (void)hipStreamDestroy(st[k]);
            st[k] = nullptr;
        }
        if (dl) (void)hipStreamDestroy(dl);
        dl = nullptr;
        down.release();
        dev = -1;
    }
    bool begin()
    {
        int d = 0;
        if (hipGetDevice(&d) != hipSuccess) return false;
        if (dev != d) {
            release();
            // LFM_DECODE_PRIO=1: slot 0's stream at the highest priority, the
            // others at the lowest, so the first chunk finishes (and its
            // download starts) while the second one still decodes
            static const bool prio = env_int("LFM_DECODE_PRIO", 0) != 0;
            int least = 0, greatest = 0;
            if (prio) (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
            for (int k = 0; k < kSlots; ++k)
                if ((prio ? hipStreamCreateWithPriority(&st[k], hipStreamNonBlocking, k == 0 ? greatest : least)
                          : hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking)) != hipSuccess) {
                    release();
                    return false;
                }
            if (hipStreamCreateWithFlags(&dl, hipStreamNonBlocking) != hipSuccess) {
                release();
                return false;
            }
            dev = d;
        }
        return true;
    }
    void* get(int i, size_t bytes)
    {
        if (cap[i] >= bytes) return p[i];
        if (p[i]) (void)hipFree(p[i]);
        p[i] = nullptr;
        cap[i] = 0;
        if (hipMalloc(&p[i], bytes) != hipSuccess) {
            (void)hipGetLastError();
            p[i] = nullptr;
            return nullptr;
        }
        cap[i] = bytes;
        return p[i];
    }
    uint32_t* status(int k, size_t count)  // 2 * count words: lens, flags
    {
        if (hs_cap[k] >= count) return hs[k];
        if (hs[k]) (void)hipHostFree(hs[k]);
        hs[k] = nullptr;
        hs_cap[k] = 0;
        if (hipHostMalloc((void**)&hs[k], count * 8, hipHostMallocDefault) != hipSuccess) {
            hs[k] = nullptr;
            return nullptr;
        }
        hs_cap[k] = count;
        return hs[k];
    }
    int* ustatus(size_t count)
    {
        if (us_cap >= count) return us;
        if (us) (void)hipHostFree(us);
        us = nullptr;
        us_cap = 0;
        if (hipHostMalloc((void**)&us, count * sizeof(int), hipHostMallocDefault) != hipSuccess) {
            us = nullptr;
            return nullptr;
        }
        us_cap = count;
        return us;
    }
};

DecodeBuffers& decode_buffers()
{
    static thread_local DecodeBuffers b;
    return b;
}
} // namespace

void par_memcpy(void* dst, const void* src, size_t n, int threads) { par_memcpy_impl(dst, src, n, threads); }

// GPU decode of a BZIP2 payload (lfm_bunzip2.hip), pipelined over chunks of
// whole block slabs (the blocks of one z-block row of one volume, so a chunk's
// pixels are a contiguous run of frames of the image): per chunk the payload
// bytes go up (SDMA), its streams are decoded (the few flagged ones by the
// host library), scattered into the device symbol image, run through the
// inverse predictor and come down (SDMA) into the caller's image.  Chunks
// alternate between two HIP streams, and the host works one chunk behind the
// device: while chunk c's kernels run, chunk c - 1 is finished and copied
// down and chunk c + 1's payload goes up.  Returns -1 when the GPU path does
// not apply (the caller decodes on the host).
static int gpu_decode(const uint8_t* payload, size_t len, const klb_image_header& h, uint8_t* img, int family,
                      bool predicted, int k, int video, int threads)
{
    const BlockGrid g(h);
    const uint64_t nb = g.nblocks;
    const size_t bpp = h.getBytesPerPixel();
    const uint32_t block_bytes = h.getBlockSizeBytes();
    if (!nb || !block_bytes || nb >= (1ull << 31)) return -1;
    // LFM_DECODE_TIMING=1: stage times on stderr
    static const bool timing = env_int("LFM_DECODE_TIMING", 0) != 0;
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const auto t_start = clk::now();
    double t_up = 0, t_wait = 0, t_down = 0, t_host = 0;
    std::vector<uint64_t> offs(nb + 1);
    for (uint64_t i = 0; i < nb; ++i) {
        offs[i] = h.getBlockOffset(i);
        if (i && offs[i] != offs[i - 1] + h.getBlockCompressedSizeBytes(i - 1)) return -1;  // not contiguous
    }
    offs[nb] = offs[nb - 1] + h.getBlockCompressedSizeBytes(nb - 1);
    if (offs[nb] > len) return 3;
    const size_t img_bytes = h.getImageSizeBytes();
    const uint64_t W = h.xyzct[0], H = h.xyzct[1], Z = h.xyzct[2];
    const size_t frame_bytes = (size_t)W * H * bpp;
    // chunks: whole slabs, at least two and about LFM_DECODE_CHUNK_BLOCKS
    // blocks each (default 4096, about the streams the Huffman kernel holds
    // resident at once: config 3's 3 872 streams in two chunks, a config-5
    // volume's 7 396 in two); 0 = one chunk.  With two slots a third chunk
    // cannot start before the first is finished, so smaller chunks lose (four
    // chunks of 968 streams: 75.6 vs 54.3 ms on config 3)
    const uint64_t slab = g.nb[0] * g.nb[1], nslabs = nb / slab;
    const long target = env_int("LFM_DECODE_CHUNK_BLOCKS", 4096);
    static const int slots = std::max(2, std::min(env_int("LFM_DECODE_SLOTS", 2), (int)DecodeBuffers::kSlots));
    uint64_t spc = nslabs;  // slabs per chunk
    if (target > 0) {
        const uint64_t want = std::max<uint64_t>(slots, (nb + (uint64_t)target - 1) / (uint64_t)target);
        spc = std::max<uint64_t>(1, (nslabs + want - 1) / want);
    }
    const size_t per = lfm_hip_bunzip2_workspace_bytes(1, block_bytes) + block_bytes;
    const size_t budget = (size_t)env_int("LFM_BUNZIP2_GPU_BUDGET_MB", 16 * 1024) << 20;
    spc = std::max<uint64_t>(1, std::min<uint64_t>(spc, budget / slots / per / slab));
    const uint64_t batch = spc * slab, nch = (nslabs + spc - 1) / spc;
    const size_t ws = lfm_hip_bunzip2_workspace_bytes((uint32_t)batch, block_bytes);
    static const bool keep = env_int("LFM_DECODE_KEEP", 1) != 0;
    DecodeBuffers& DB = decode_buffers();
    auto release = [&]() {
        if (!keep) {
            DB.release();
            staging().release();
        }
    };
    const int nslot = (int)std::min<uint64_t>(nch, (uint64_t)slots);
    void *d_pay = nullptr, *d_sym = nullptr, *d_out = nullptr, *d_ws[DecodeBuffers::kSlots] = {},
         *d_blk[DecodeBuffers::kSlots] = {};
    uint32_t* hs[DecodeBuffers::kSlots] = {};
    // inverse predictor status words: chunk c's volume pieces at us[c * (spc + 1) ..]
    // (a chunk's slabs lie in at most spc volumes)
    int* us = nullptr;
    const uint64_t us_per = spc + 1;
    if (DB.begin()) {
        d_pay = DB.get(DecodeBuffers::PAY, offs[nb] + 64);
        d_sym = DB.get(DecodeBuffers::SYM, img_bytes);
        d_out = predicted ? DB.get(DecodeBuffers::OUT, img_bytes) : nullptr;
        for (int q = 0; q < nslot; ++q) {
            d_ws[q] = DB.get(DecodeBuffers::WS0 + q, ws);
            d_blk[q] = DB.get(DecodeBuffers::BLK0 + q, batch * block_bytes);
            hs[q] = DB.status(q, batch);
        }
        if (predicted) {
            us = DB.ustatus(nch * us_per);
            if (us) std::fill(us, us + nch * us_per, 0);
        }
    }
    bool have = DB.st[0] && d_pay && d_sym && (!predicted || (d_out && us));
    for (int q = 0; q < nslot; ++q) have = have && d_ws[q] && d_blk[q] && hs[q];
    if (!have) {
        DB.release();
        return -1;
    }
    const auto t_alloc = clk::now();
    uint32_t dims[5], bs[5];
    for (int d = 0; d < 5; ++d) {
        dims[d] = h.xyzct[d];
        bs[d] = (uint32_t)g.bs[d];
    }
    // payload upload: the SDMA engine through the pinned chunks (LFM_DECODE_H2D
    // = 0, default; falls back to 1 when HSA cannot take it), 1 one runtime
    // copy, 2 the pinned chunks with hipMemcpyAsync -- the blit-kernel copies
    // took 5-47 ms for config 3's 277 MB depending on the process's state
    static const int up_mode = env_int("LFM_DECODE_H2D", 0);
    auto upload = [&](uint64_t lo, uint64_t hi, hipStream_t st) {  // payload bytes [lo, hi)
        lo &= ~(uint64_t)3;  // (4-byte aligned pieces; neighbours rewrite the same bytes)
        const size_t n = hi - lo;
        if (up_mode == 0 && sdma_staged_h2d((uint8_t*)d_pay + lo, payload + lo, n, threads)) return true;
        (void)hipGetLastError();
        const bool ok = up_mode == 2 ? staged_h2d((uint8_t*)d_pay + lo, payload + lo, n, st, threads)
                                     : hipMemcpyAsync((uint8_t*)d_pay + lo, payload + lo, n, hipMemcpyHostToDevice,
                                                      st) == hipSuccess;
        return ok && hipStreamSynchronize(st) == hipSuccess;
    };
    // the frames (volume-major) a chunk's slabs cover: [f0, f1)
    const uint64_t nbz = g.nb[2];
    auto frames = [&](uint64_t c, uint64_t& f0, uint64_t& f1) {
        const uint64_t s0 = c * spc, s1 = std::min(nslabs, s0 + spc) - 1;
        f0 = (s0 / nbz) * Z + (s0 % nbz) * g.bs[2];
        f1 = (s1 / nbz) * Z + std::min<uint64_t>(Z, (s1 % nbz + 1) * g.bs[2]);
    };
    std::vector<uint8_t> hb(block_bytes);
    int rc = 0;
    const double t_hb = ms(t_start, clk::now());
    // LFM_DECODE_TIMING: a timeline of the pipeline's steps (ms since start)
    std::mutex tlmu;
    std::vector<std::pair<std::string, double>> tl;
    auto mark = [&](const char* what, uint64_t c) {
        if (!timing) return;
        std::lock_guard<std::mutex> lk(tlmu);
        tl.emplace_back(std::string(what) + " " + std::to_string(c), ms(t_start, clk::now()));
    };
    // The image comes down into the caller's buffer, usually fresh pages (a
    // new numpy array, readKLBstack's malloc): the download's host copies used
    // to take a first-touch fault per 4 KiB page (config 3: 131 072 faults,
    // download 11-24 ms for 537 MB).  While the GPU decodes, a helper thread
    // asks for huge pages and touches one byte per page of the destination, so
    // the downloads copy into mapped memory (LFM_DECODE_PREFAULT=0: off).
    // LFM_DECODE_DMA_PROBE=1 (diagnosis): a 64 KiB staged SDMA upload, timed,
    // before the decode's own steps start
    if (env_int("LFM_DECODE_DMA_PROBE", 0) == 1 && offs[nb] >= 65536) {
        const auto p0 = clk::now();
        const bool pok = sdma_staged_h2d(d_pay, payload, 65536, 1);
        std::fprintf(stderr, "dma probe: 64 KiB upload %.3f ms (%s)\n", ms(p0, clk::now()), pok ? "ok" : "failed");
    }
    static const int prefault_mode = env_int("LFM_DECODE_PREFAULT", 1);  // 2: started after the first upload
    std::thread prefault;  // joined by the downloader before its first copy
    auto start_prefault = [&]() {
        prefault = std::thread([img, img_bytes, threads, &mark]() {
            const size_t pg = (size_t)sysconf(_SC_PAGESIZE), huge = (size_t)2 << 20;
            const uintptr_t a0 = ((uintptr_t)img + huge - 1) & ~(uintptr_t)(huge - 1);
            const uintptr_t a1 = ((uintptr_t)img + img_bytes) & ~(uintptr_t)(huge - 1);
            if (a1 > a0) (void)madvise((void*)a0, a1 - a0, MADV_HUGEPAGE);
            const size_t piece = (size_t)8 << 20;
            const uint64_t np = (img_bytes + piece - 1) / piece;
            parallel_for(np, std::max(1, threads / 2), [&](uint64_t i) {
                volatile uint8_t* q = (volatile uint8_t*)img;
                const size_t e = std::min(img_bytes, (size_t)(i + 1) * piece);
                for (size_t o = (size_t)i * piece; o < e; o += pg) q[o] = 0;
            });
            mark("prefault-done", 0);
        });
        mark("prefault-started", 0);
    };
    if (prefault_mode == 1) start_prefault();
    // the 64 zero bytes past the payload (the bit window's lookahead of the
    // last stream): LFM_DECODE_SLACK=1 queues them on the last chunk's stream
    // (stream order puts them before its kernels), 0 synchronises here
    static const int slack_mode = env_int("LFM_DECODE_SLACK", 1);
    {
        hipStream_t sst = slack_mode ? DB.st[(nch - 1) % nslot] : DB.st[0];
        if (hipMemsetAsync((uint8_t*)d_pay + offs[nb], 0, 64, sst) != hipSuccess) rc = 3;
        mark("memset-issued", 0);
        if (!slack_mode && hipStreamSynchronize(sst) != hipSuccess) rc = 3;
    }
    mark("memset", 0);
    // per chunk: its scatter + inverse predictor done (the download waits for it)
    std::vector<hipEvent_t> cev(nch, nullptr);
    for (uint64_t c = 0; c < nch && !rc; ++c)
        if (hipEventCreateWithFlags(&cev[c], hipEventDisableTiming) != hipSuccess) rc = 3;
    mark("events", 0);
    // host side of chunk c once its streams are decoded: host-library blocks,
    // then scatter and inverse predictor queued behind them (no wait)
    auto finish = [&](uint64_t c) -> int {
        const int q = (int)(c % nslot);
        hipStream_t st = DB.st[q];
        const uint64_t b0 = c * batch, cnt = std::min<uint64_t>(batch, nb - b0);
        auto t0 = clk::now();
        if (hipStreamSynchronize(st) != hipSuccess) return 3;
        auto t1 = clk::now();
        t_wait += ms(t0, t1);
        const uint32_t* lens = hs[q];
        const uint32_t* flags = hs[q] + batch;
        for (uint64_t i = 0; i < cnt; ++i) {
            uint64_t o[5], sz[5];
            g.block(b0 + i, o, sz);
            const uint64_t expect = bpp * sz[0] * sz[1] * sz[2] * sz[3] * sz[4];
            if (flags[i] == 1) {  // the host library decodes this stream
                const int r = decompress_one(BZIP2, payload + offs[b0 + i], (uint32_t)(offs[b0 + i + 1] - offs[b0 + i]),
                                             hb.data(), (uint32_t)expect);
                if (r) return r;
                if (hipMemcpyAsync((uint8_t*)d_blk[q] + (size_t)i * block_bytes, hb.data(), expect,
                                   hipMemcpyHostToDevice, st) != hipSuccess ||
                    hipStreamSynchronize(st) != hipSuccess)
                    return 3;
            } else if (flags[i] != 0 || lens[i] != expect) {
                std::printf("ERROR: block %llu of the payload does not decode to its %llu bytes (bzip2 CRC / length)\n",
                            (unsigned long long)(b0 + i), (unsigned long long)expect);
                return 2;
            }
        }
        if (lfm_hip_scatter_blocks(d_blk[q], block_bytes, (uint32_t)b0, (uint32_t)cnt, dims, bs, (uint32_t)bpp, d_sym,
                                   st) != LFM_HIP_OK)
            return 3;
        if (predicted) {
            uint64_t f0, f1;
            frames(c, f0, f1);
            // a temporal first frame (video, odd z) reads the previous chunk's
            // last decoded frame: wait for that chunk's inverse predictor
            if (video && c > 0 && hipStreamWaitEvent(st, cev[c - 1], 0) != hipSuccess) return 3;
            uint64_t piece = 0;
            for (uint64_t f = f0; f < f1; ++piece) {  // per volume
                const uint64_t v = f / Z, z0 = f % Z, n = std::min<uint64_t>(f1, (v + 1) * Z) - f;
                const uint16_t* prev = z0 > 0 ? (const uint16_t*)d_out + (f - 1) * W * H : nullptr;
                if (piece >= us_per) return 3;  // (cannot happen: see us_per)
                // queued only: its status word is checked with the download
                const int hr = lfm_hip_unpredict_async((const uint16_t*)d_sym + f * W * H, prev,
                                                       (uint16_t*)d_out + f * W * H, (int)W, (int)H, (int)n, h.Nnum,
                                                       family, k, video, (int)z0, us + c * us_per + piece, st);
                if (hr == LFM_HIP_ENOTINV) {
                    std::printf("ERROR: frames of this file cannot be inverted (temporal angle/space predictor)\n");
                    return 3;
                }
                if (hr != LFM_HIP_OK) return 3;
                f += n;
            }
        }
        if (hipEventRecord(cev[c], st) != hipSuccess) return 3;
        t_host += ms(t1, clk::now());
        return 0;
    };
    // the downloads run on their own thread (own pinned chunks), in chunk
    // order, each once its chunk's event fires: the loop below goes on queueing
    // the next chunks meanwhile
    std::mutex dmu;
    std::condition_variable dcv;
    uint64_t dl_ready = 0;  // chunks [0, dl_ready) may be downloaded
    bool dl_stop = false;
    int drc = 0;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::thread downloader([&]() {
        (void)hipSetDevice(dev);
        for (uint64_t c = 0; c < nch; ++c) {
            {
                std::unique_lock<std::mutex> lk(dmu);
                dcv.wait(lk, [&] { return dl_ready > c || dl_stop; });
                if (dl_ready <= c) return;  // stopped
            }
            // (started before chunk 0 was handed over; done long before it is decoded)
            if (c == 0 && prefault.joinable()) prefault.join();
            auto t0 = clk::now();
            mark("dl-start", c);
            uint64_t f0, f1;
            frames(c, f0, f1);
            const size_t o0 = f0 * frame_bytes, n = (f1 - f0) * frame_bytes;
            const uint8_t* src = (const uint8_t*)(predicted ? d_out : d_sym) + o0;
            // (its own stream: on the chunk's slot stream the copies would
            // queue behind the kernels of chunk c + nslot, issued meanwhile)
            hipStream_t st = DB.dl;
            if (hipEventSynchronize(cev[c]) != hipSuccess) {
                drc = 3;
                return;
            }
            mark("dl-ready", c);
            // the chunk's inverse predictor launches: a hand-over that timed
            // out and was not repaired on the device fails the read
            if (predicted)
                for (uint64_t i = 0; i < us_per; ++i)
                    if (lfm_hip_unpredict_check(us[c * us_per + i]) != LFM_HIP_OK) {
                        std::printf("ERROR: the inverse predictor did not complete (band hand-over timed out)\n");
                        drc = 3;
                        return;
                    }
            // the device -> pinned copies: the runtime's (57 GB/s) or an SDMA
            // engine's (28 GB/s).  The runtime's copies slow the kernels of
            // chunks still decoding (config 5, 8 chunks: 403-427 vs 325-349
            // ms), so LFM_DECODE_D2H=1 (default) takes them only for the last
            // nslot chunks, whose downloads are the decode's exposed tail
            // (config 3: 55-57 vs 62-64 ms); 2: always, 0: never
            // (profiles/r06_ab_decode_d2h*.jsonl)
            static const int d2h_mode = env_int("LFM_DECODE_D2H", 1);
            const bool rt = d2h_mode == 2 || (d2h_mode == 1 && c + nslot >= nch);
            if (((rt || !sdma_staged_d2h(img + o0, src, n, threads, DB.down)) &&
                 (!staged_d2h(img + o0, src, n, st, threads, DB.down) || hipStreamSynchronize(st) != hipSuccess))) {
                drc = 3;
                return;
            }
            t_down += ms(t0, clk::now());
            mark("dl-end", c);
        }
    });
    auto hand_over = [&](uint64_t c) {
        {
            std::lock_guard<std::mutex> lk(dmu);
            dl_ready = c + 1;
        }
        dcv.notify_all();
    };
    mark("downloader-started", 0);
    for (uint64_t c = 0; c < nch && !rc; ++c) {
        const int q = (int)(c % nslot);
        const uint64_t b0 = c * batch, cnt = std::min<uint64_t>(batch, nb - b0);
        auto t0 = clk::now();
        if (!upload(offs[b0], offs[b0 + cnt], DB.st[q])) {
            rc = 3;
            break;
        }
        t_up += ms(t0, clk::now());
        mark("uploaded", c);
        if (c == 0 && prefault_mode == 2) start_prefault();
        if (lfm_hip_bunzip2_issue(d_pay, offs.data() + b0, (uint32_t)cnt, d_blk[q], block_bytes, d_ws[q], ws, hs[q],
                                  hs[q] + batch, DB.st[q]) != LFM_HIP_OK) {
            rc = 3;
            break;
        }
        mark("issued", c);
        if (c > 0) {
            rc = finish(c - 1);
            mark("finished", c - 1);
            if (!rc) hand_over(c - 1);
        }
    }
    if (!rc) rc = finish(nch - 1);
    mark("finished", nch - 1);
    if (!rc) hand_over(nch - 1);
    {
        std::lock_guard<std::mutex> lk(dmu);
        dl_stop = true;
    }
    dcv.notify_all();
    downloader.join();
    mark("joined", nch);
    if (prefault.joinable()) prefault.join();  // (not reached: the downloader joins it first)
    if (!rc) rc = drc;
    for (int q = 0; q < nslot; ++q) (void)hipStreamSynchronize(DB.st[q]);  // nothing may still run on the buffers
    for (hipEvent_t e : cev)
        if (e) (void)hipEventDestroy(e);
    if (timing) {
        std::string line = "decode timeline: alloc@" + std::to_string(ms(t_start, t_alloc)).substr(0, 6) +
                           " hb@" + std::to_string(t_hb).substr(0, 6);
        for (auto& e : tl) line += " " + e.first + "@" + std::to_string(e.second).substr(0, 6);
        std::fprintf(stderr, "%s\n", line.c_str());
    }
    if (timing)
        std::fprintf(stderr,
                     "decode: %llu chunks of <= %llu blocks, alloc %.2f ms, upload %.2f, wait %.2f, host + kernels "
                     "after wait %.2f, download %.2f, total %.2f ms\n",
                     (unsigned long long)nch, (unsigned long long)batch, ms(t_start, t_alloc), t_up, t_wait, t_host,
                     t_down, ms(t_start, clk::now()));
    release();
    return rc;
}

int decode_payload(const uint8_t* payload, size_t len, const klb_image_header& h, uint8_t* img, int threads,
                   int family)
{
    if (threads <= 0) threads = default_threads();
    const BlockGrid g(h);
    if (g.nblocks != h.Nb) return 3;
    const size_t bpp = h.getBytesPerPixel();
    if (!bpp) return 5;
    const int k = h.headerVersion & 0x7F;
    const int video = (h.headerVersion >> 7) & 1;
    const bool predicted = bpp == 2 && k != 0;
    if (predicted && (k > 7 || h.Nnum == 0)) {
        std::printf("ERROR: unknown predictor %d in header\n", k);
        return 3;
    }
    if (h.compressionType == BZIP2 && gpu_decode_enabled() && gpu_bunzip2_enabled() && lfm_hip_device_count() > 0 &&
        (!predicted || h.Nnum <= 31)) {
        const int rc = gpu_decode(payload, len, h, img, family, predicted, k, video, threads);
        if (rc != -1) return rc;
    }
    std::vector<uint16_t> symbuf;
    uint8_t* sym = img;
    if (predicted) {
        symbuf.resize(h.getImageSizePixels());
        sym = (uint8_t*)symbuf.data();
    }
    std::atomic<int> err{0};
    const uint32_t block_bytes = h.getBlockSizeBytes();
    parallel_for(g.nblocks, threads, [&](uint64_t id) {
        thread_local std::vector<uint8_t> scratch;
        uint64_t o[5], s[5];
        g.block(id, o, s);
        const uint64_t expect = bpp * s[0] * s[1] * s[2] * s[3] * s[4];
        const uint64_t off = h.getBlockOffset(id), n = h.getBlockCompressedSizeBytes(id);
        if (off + n > len) { err.store(3); return; }
        scratch.resize(std::max<uint64_t>(expect, block_bytes));
        int rc = decompress_one(h.compressionType, payload + off, (uint32_t)n, scratch.data(), (uint32_t)expect);
        if (rc) { err.store(rc); return; }
        scatter_block(scratch.data(), g, id, bpp, sym);
    });
    if (err.load()) return err.load();
    if (!predicted) return 0;
    const int W = h.xyzct[0], H = h.xyzct[1], Z = h.xyzct[2];
    const uint64_t V = (uint64_t)h.xyzct[3] * h.xyzct[4];
    const size_t fs = (size_t)W * H;
    const uint16_t* s16 = symbuf.data();
    uint16_t* o16 = (uint16_t*)img;
    // inverse predictor on the GPU (lfm_unpredict.hip) whenever one is
    // visible; the host loop below is the reader of GPU-less machines (the
    // reference decoder itself is host code, klb_imageIO.cpp:1748-1821)
    if (gpu_decode_enabled() && lfm_hip_device_count() > 0 && h.Nnum <= 31) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        hipStream_t st = nullptr;
        void *d_s = nullptr, *d_o = nullptr;
        const size_t vb = fs * Z * 2;
        int rc = 0;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess || hipMalloc(&d_s, vb) != hipSuccess ||
            hipMalloc(&d_o, vb) != hipSuccess)
            rc = 3;
        for (uint64_t v = 0; v < V && !rc; ++v) {
            if (hipMemcpyAsync(d_s, s16 + v * Z * fs, vb, hipMemcpyHostToDevice, st) != hipSuccess) { rc = 3; break; }
            const int hr = lfm_hip_unpredict((const uint16_t*)d_s, nullptr, (uint16_t*)d_o, W, H, Z, h.Nnum, family, k,
                                             video, 0, st);
            if (hr == LFM_HIP_ENOTINV) {
                std::printf("ERROR: frames of this file cannot be inverted (temporal angle/space predictor)\n");
                rc = 3;
                break;
            }
            if (hr != LFM_HIP_OK || hipMemcpyAsync(o16 + v * Z * fs, d_o, vb, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                rc = 3;
        }
        if (d_s) (void)hipFree(d_s);
        if (d_o) (void)hipFree(d_o);
        if (st) (void)hipStreamDestroy(st);
        return rc;
    }
    // host inverse (frames in parallel; on video stacks the odd frames need
    // the decoded even frame before them)
    for (int pass = 0; pass < (video ? 2 : 1); ++pass) {
        std::vector<uint64_t> frames;
        for (uint64_t v = 0; v < V; ++v)
            for (int z = 0; z < Z; ++z) {
                const bool temp = video && (z & 1);
                if (video ? (pass == (temp ? 1 : 0)) : true) frames.push_back(v * Z + z);
            }
        parallel_for(frames.size(), threads, [&](uint64_t i) {
            const uint64_t fidx = frames[i];
            const int z = (int)(fidx % Z);
            const bool temp = video && (z & 1);
            int rc = unpredict_one(family, k, temp, s16 + fidx * fs, temp ? o16 + (fidx - 1) * fs : nullptr,
                                   o16 + fidx * fs, W, H, h.Nnum);
            if (rc) err.store(rc == LFM_HIP_ENOTINV ? 3 : rc);
        });
        if (err.load()) {
            std::printf("ERROR: frames of this file cannot be inverted (temporal angle/space predictor)\n");
            return err.load();
        }
    }
    return 0;
}

// ROI read: decode only the blocks the ROI depends on, then
// crop.  Every predictor neighbour is up and / or left in its frame, so a
// predicted ROI needs x in [0, ub0] and y in [0, ub1] of its frames (the
// inverse on that corner computes the same pixels as on the whole frame);
// a temporal (odd z) frame of a video stack also needs the frame before it.
// The blocks of that region (whole blocks, origin z even on video stacks so
// the temporal parity is unchanged) are described by a sub-header whose block
// grid is exactly those blocks in file order, their streams are gathered into
// a sub-payload, and the ordinary decode (GPU or host) runs on it.  The
// reference's own ROI path decodes the ROI's blocks and then un-predicts them
// as if they were the whole frame, which is wrong with predictors
// (klb_imageIO.cpp:2614-2682).
int decode_roi(const uint8_t* payload, size_t len, const klb_image_header& h, const uint32_t lb[5],
               const uint32_t ub[5], uint8_t* out, int threads, int family)
{
    const BlockGrid g(h);
    if (g.nblocks != h.Nb) return 3;
    const size_t bpp = h.getBytesPerPixel();
    if (!bpp) return 5;
    for (int d = 0; d < 5; ++d)
        if (ub[d] < lb[d] || ub[d] >= h.xyzct[d]) return 3;
    const int k = h.headerVersion & 0x7F;
    const bool video = (h.headerVersion >> 7) & 1;
    const bool predicted = bpp == 2 && k != 0;
    uint64_t b0[5], b1[5], o[5], n[5];
    for (int d = 0; d < 5; ++d) {
        uint64_t lo = lb[d];
        if (predicted && d < 2) lo = 0;
        if (predicted && video && d == 2 && (lo & 1)) lo -= 1;
        b0[d] = lo / g.bs[d];
        b1[d] = ub[d] / g.bs[d] + 1;
    }
    if (predicted && video)
        while (b0[2] > 0 && ((b0[2] * g.bs[2]) & 1)) --b0[2];
    klb_image_header sub(h);
    for (int d = 0; d < 5; ++d) {
        o[d] = b0[d] * g.bs[d];
        n[d] = std::min<uint64_t>(g.dims[d], b1[d] * g.bs[d]) - o[d];
        sub.xyzct[d] = (uint32_t)n[d];
    }
    const uint64_t cnt = (b1[0] - b0[0]) * (b1[1] - b0[1]) * (b1[2] - b0[2]) * (b1[3] - b0[3]) * (b1[4] - b0[4]);
    sub.resizeBlockOffset(cnt);
    std::vector<uint64_t> ids;
    ids.reserve(cnt);
    uint64_t total = 0;
    for (uint64_t t = b0[4]; t < b1[4]; ++t)
        for (uint64_t c = b0[3]; c < b1[3]; ++c)
            for (uint64_t z = b0[2]; z < b1[2]; ++z)
                for (uint64_t y = b0[1]; y < b1[1]; ++y)
                    for (uint64_t x = b0[0]; x < b1[0]; ++x) {
                        const uint64_t id = x + g.nb[0] * (y + g.nb[1] * (z + g.nb[2] * (c + g.nb[3] * t)));
                        const uint64_t e = h.getBlockOffset(id) + h.getBlockCompressedSizeBytes(id);
                        if (e > len) return 3;
                        total += h.getBlockCompressedSizeBytes(id);
                        sub.blockOffset[ids.size()] = total;
                        ids.push_back(id);
                    }
    // the region's streams: a run of consecutive blocks (whole t-volumes, a
    // z-range of whole frames) is read where it lies in the payload; anything
    // else is gathered into a buffer (no zero fill: every byte is copied)
    bool run = true;
    for (size_t i = 1; i < ids.size() && run; ++i)
        run = ids[i] == ids[i - 1] + 1 && h.getBlockOffset(ids[i]) == h.getBlockOffset(ids[i - 1]) +
                                                                         h.getBlockCompressedSizeBytes(ids[i - 1]);
    std::unique_ptr<uint8_t[]> gathered;
    const uint8_t* spay = ids.empty() ? payload : payload + h.getBlockOffset(ids[0]);
    if (!run) {
        gathered.reset(new uint8_t[total]);
        parallel_for(ids.size(), threads, [&](uint64_t i) {
            const uint64_t id = ids[i], sz = h.getBlockCompressedSizeBytes(id);
            std::memcpy(gathered.get() + (sub.blockOffset[i] - sz), payload + h.getBlockOffset(id), sz);
        });
        spay = gathered.get();
    }
    // a region that is exactly its blocks' box (e.g. whole t-volumes) is
    // decoded straight into `out`: no temporary image, no crop
    bool exact = true;
    for (int d = 0; d < 5; ++d) exact = exact && o[d] == lb[d] && n[d] == (uint64_t)ub[d] - lb[d] + 1;
    if (exact) return decode_payload(spay, total, sub, out, threads, family);
    std::unique_ptr<uint8_t[]> simg(new uint8_t[sub.getImageSizeBytes()]);  // (no zero fill: every byte is decoded)
    const int rc = decode_payload(spay, total, sub, simg.get(), threads, family);
    if (rc) return rc;
    const size_t row = (size_t)(ub[0] - lb[0] + 1) * bpp;
    const uint64_t ny = (uint64_t)ub[1] - lb[1] + 1, nz = (uint64_t)ub[2] - lb[2] + 1, nc = (uint64_t)ub[3] - lb[3] + 1;
    const uint64_t nrows = ny * nz * nc * ((uint64_t)ub[4] - lb[4] + 1);
    parallel_for(nrows, threads, [&](uint64_t r) {  // output row r = ((t * nc + c) * nz + z) * ny + y
        const uint64_t y = lb[1] + r % ny, z = lb[2] + (r / ny) % nz, c = lb[3] + (r / ny / nz) % nc,
                       t = lb[4] + r / ny / nz / nc;
        const uint64_t e = (lb[0] - o[0]) +
                           n[0] * ((y - o[1]) + n[1] * ((z - o[2]) + n[2] * ((c - o[3]) + n[3] * (t - o[4]))));
        std::memcpy(out + r * row, simg.get() + e * bpp, row);
    });
    return 0;
}

int decode_file_roi(const char* filename, klb_image_header& h, const uint32_t lb[5], const uint32_t ub[5],
                    uint8_t* out, int threads)
{
    FILE* f = std::fopen(filename, "rb");
    if (!f) {
        std::printf("ERROR: file %s could not be opened\n", filename);
        return 3;
    }
    std::fseek(f, 0, SEEK_END);
    const long size = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    std::vector<uint8_t> buf(size > 0 ? (size_t)size : 0);
    const size_t got = buf.empty() ? 0 : std::fread(buf.data(), 1, buf.size(), f);
    std::fclose(f);
    if (got != buf.size()) return 3;
    int rc = h.parseHeader(buf.data(), buf.size());
    if (rc) return rc;
    const size_t hs = h.getSizeInBytes();
    return decode_roi(buf.data() + hs, buf.size() - hs, h, lb, ub, out, threads, current_family());
}

int decode_file(const char* filename, klb_image_header& h, std::vector<uint8_t>* img_out, uint8_t* img_into,
                int threads)
{
    FILE* f = std::fopen(filename, "rb");
    if (!f) {
        std::printf("ERROR: file %s could not be opened\n", filename);
        return 3;
    }
    std::fseek(f, 0, SEEK_END);
    const long size = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    std::vector<uint8_t> buf(size > 0 ? (size_t)size : 0);
    const size_t got = buf.empty() ? 0 : std::fread(buf.data(), 1, buf.size(), f);
    std::fclose(f);
    if (got != buf.size()) return 3;
    int rc = h.parseHeader(buf.data(), buf.size());
    if (rc) return rc;
    uint8_t* dst = img_into;
    if (!dst) {
        img_out->resize(h.getImageSizeBytes());
        dst = img_out->data();
    }
    const size_t hs = h.getSizeInBytes();
    return decode_payload(buf.data() + hs, buf.size() - hs, h, dst, threads, current_family());
}

} // namespace lfm
