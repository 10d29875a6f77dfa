// lfm_multigpu.cpp -- the klb_imageIO block scheduler farmed across the GPUs
// of one node (BASELINE north_star: "the klb_imageIO block
// scheduler is reworked to farm independent xyzct blocks across the 8 GPUs").
//
// The reference scheduler is one process, one GPU and a pool of host bzip2
// threads behind an atomic block counter with an in-order writer
// (klb_imageIO.cpp:2406-2463, workers :2446-2454, writer :1145-1225).  Here
// the unit farmed to a device is a contiguous range of block layers: z-slabs
// of whole blocks for a single (c,t) volume, ranges of whole c or t otherwise
// (block ids run x -> y -> z -> c -> t, so every range is a contiguous id
// range of the file).  One host thread per worker drives its device's
// Encoder (predictor kernel + GPU bzip2) on its range; the calling thread is
// the in-order writer: it appends each range's compressed blocks as soon as
// that range and all before it are done and re-accumulates the block offset
// table (a host prefix sum of block sizes).  No data crosses between GPUs:
// the predictor is selected once on frame 0 and forced for every range, and a
// z-slab that starts at an odd frame of a video stack reads its previous raw
// frame straight from the caller's host image.  Output bytes are identical to
// the one-GPU encode (tests/test_gpu_full.py, tests/test_multigpu_gpu.py).
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "lfm_engine.h"
#include "lfm_hip.h"

namespace lfm {

namespace {
using clk = std::chrono::steady_clock;
double ms_since(clk::time_point t0) { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); }

std::mutex g_dev_mu;
std::vector<int> g_devices;  // lfm_set_devices; empty = LFM_GPUS / all visible

struct PoolEntry {
    std::mutex mu;
    std::unique_ptr<Encoder> enc;
};
std::mutex g_pool_mu;
std::map<std::pair<int, int>, std::unique_ptr<PoolEntry>> g_pool;
} // namespace

void set_encode_devices(const std::vector<int>& devs)
{
    std::lock_guard<std::mutex> lk(g_dev_mu);
    g_devices = devs;
}

namespace {
int env_int(const char* name, int dflt)
{
    const char* e = std::getenv(name);
    return (e && *e) ? std::atoi(e) : dflt;
}
} // namespace

std::vector<int> default_devices(int n, int current)
{
    std::vector<int> out;
    if (n <= 0) return out;
    // LFM_GPUS: "0,1,2,3" (a device list; repeats map several workers onto
    // one device) or "N" (devices 0 .. N-1)
    if (const char* e = std::getenv("LFM_GPUS")) {
        std::string s(e);
        if (!s.empty() && s.find(',') == std::string::npos) {
            const int k = std::atoi(s.c_str());
            for (int i = 0; i < k && i < n; ++i) out.push_back(i);
        } else {
            size_t p = 0;
            while (p < s.size()) {
                size_t q = s.find(',', p);
                if (q == std::string::npos) q = s.size();
                if (q > p) {
                    const int d = std::atoi(s.substr(p, q - p).c_str());
                    if (d >= 0 && d < n) out.push_back(d);
                }
                p = q + 1;
            }
        }
        if (!out.empty()) return out;
    }
    // A process of a multi-process job (torchrun / MPI launchers set these).
    // The number of processes on THIS node decides: one process per node owns
    // every GPU of it; several share the node, and farming to every GPU from
    // each of them would oversubscribe them all, so each takes one device --
    // its local rank modulo the visible devices (the current device is not
    // trusted: a rank that never called set_device would sit on device 0).
    // Only a global WORLD_SIZE > 1 with no local size known is taken as
    // one process per GPU.
    int local_size = env_int("LOCAL_WORLD_SIZE", -1);
    if (local_size < 0) local_size = env_int("OMPI_COMM_WORLD_LOCAL_SIZE", -1);
    const bool shared_node = local_size > 1 || (local_size < 0 && env_int("WORLD_SIZE", 1) > 1);
    if (shared_node) {
        int lr = env_int("LOCAL_RANK", -1);
        if (lr < 0) lr = env_int("OMPI_COMM_WORLD_LOCAL_RANK", -1);
        if (lr >= 0) return {lr % n};
        return {(current >= 0 && current < n) ? current : 0};
    }
    for (int i = 0; i < n; ++i) out.push_back(i);
    return out;
}

std::vector<int> encode_devices()
{
    {
        std::lock_guard<std::mutex> lk(g_dev_mu);
        if (!g_devices.empty()) return g_devices;
    }
    const int n = lfm_hip_device_count();
    int cur = -1;
    if (n <= 0 || hipGetDevice(&cur) != hipSuccess) cur = -1;
    return default_devices(n, cur);
}

// persistent encoders (device buffers kept between calls) keyed by (device,
// worker slot on that device); the caller holds the entry's lock while using it
Encoder& pooled_encoder(int dev, int slot, std::unique_lock<std::mutex>& lock)
{
    PoolEntry* e;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        auto& p = g_pool[{dev, slot}];
        if (!p) p.reset(new PoolEntry);
        e = p.get();
    }
    lock = std::unique_lock<std::mutex>(e->mu);
    if (!e->enc) e->enc.reset(new Encoder(dev));
    return *e->enc;
}

void release_pooled_encoders()
{
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (auto& kv : g_pool) {
        std::lock_guard<std::mutex> el(kv.second->mu);
        kv.second->enc.reset();
    }
}

Encoder& shared_encoder(std::unique_lock<std::mutex>& lock)
{
    int dev = 0;
    if (lfm_hip_device_count() > 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
    return pooled_encoder(std::max(0, dev), 0, lock);
}

int encode_multi(const void* img, klb_image_header& h, Sink& sink, lfm_encode_stats* st, int threads,
                 const std::vector<int>& devs)
{
    if (devs.size() < 2 || !img) return -1;
    auto t0 = clk::now();
    if (int rc = normalize_header(h)) return rc;
    const size_t bpp = h.getBytesPerPixel();
    // shard axis: t ranges, else c ranges, else z-slabs; whole blocks each
    const int axis = h.xyzct[4] > 1 ? 4 : (h.xyzct[3] > 1 ? 3 : 2);
    const uint64_t unit = h.blockSize[axis], dim = h.xyzct[axis];
    const uint64_t nunits = (dim + unit - 1) / unit;
    uint64_t per = (nunits + devs.size() - 1) / devs.size();
    const int nw = (int)((nunits + per - 1) / per);
    if (nw < 2) return -1;
    uint64_t stride = bpp;  // bytes between consecutive indices along the axis
    for (int d = 0; d < axis; ++d) stride *= h.xyzct[d];
    if (threads <= 0) threads = default_threads();
    if (st) std::memset(st, 0, sizeof(*st));

    struct Work {
        uint64_t first, count;  // along the axis
        int dev, slot;
        Encoder* enc = nullptr;
        int rc = -1;
        bool done = false, consumed = false;
        lfm_encode_stats st{};
        const uint8_t* out = nullptr;
        size_t out_len = 0;
    };
    std::vector<Work> work(nw);
    std::map<int, int> slots;
    for (int w = 0; w < nw; ++w) {
        work[w].first = w * per * unit;
        work[w].count = std::min<uint64_t>(dim, (w + 1) * per * unit) - work[w].first;
        work[w].dev = devs[w];
        work[w].slot = slots[devs[w]]++;
    }
    // Every pooled encoder this call uses is locked here, by the calling
    // thread, in one global (device, slot) order and held until the workers
    // are joined: two concurrent calls whose device lists differ in order
    // can then never hold one entry each while waiting for the other's.
    std::vector<int> order(nw);
    for (int w = 0; w < nw; ++w) order[w] = w;
    std::sort(order.begin(), order.end(), [&](int a, int b) {
        return std::make_pair(work[a].dev, work[a].slot) < std::make_pair(work[b].dev, work[b].slot);
    });
    std::vector<std::unique_lock<std::mutex>> held(nw);
    for (int w : order) work[w].enc = &pooled_encoder(work[w].dev, work[w].slot, held[w]);

    // predictor selection once, on frame 0 of volume (0,0) (klb_imageIO.cpp:2316-2360),
    // then forced (request 8 + k) for every range.  It runs on the caller's
    // thread with devs[0] current; the caller's device is restored after.
    uint8_t hv = h.headerVersion;
    const int req = hv & 0x7F;
    const bool predictable = bpp == 2 && h.Nnum > 0;
    if (predictable && req < NUM_PREDICTORS) {
        auto ts = clk::now();
        int caller_dev = -1;
        if (hipGetDevice(&caller_dev) != hipSuccess) caller_dev = -1;
        Encoder& e0 = *work[0].enc;  // (devs[0], slot 0)
        int k = 0;
        float ent[8] = {0};
        const int src = e0.select_host_frame(img, (int)h.xyzct[0], (int)h.xyzct[1], h.Nnum, current_family(), &k, ent);
        if (caller_dev >= 0) (void)hipSetDevice(caller_dev);
        if (src) return src;
        hv = (uint8_t)((hv & 0x80) | (8 + k));
        if (st) {
            st->select_ms = ms_since(ts);
            std::memcpy(st->entropy, ent, sizeof(ent));
        }
    }

    std::mutex mu;
    std::condition_variable cv;
    const int wthreads = std::max(1, threads / nw);
    const int level = bzip2_level(h);  // the whole stack's nominal block (klb_imageIO.cpp:108)
    auto worker = [&](int w) {
        Work& W = work[w];
        Encoder& enc = *W.enc;  // locked by the calling thread until every worker is joined
        klb_image_header hs(h);
        hs.headerVersion = hv;
        hs.xyzct[axis] = (uint32_t)W.count;
        hs.blockSize[axis] = std::min<uint32_t>(h.blockSize[axis], hs.xyzct[axis]);
        SlabSpec slab;
        slab.level = level;
        if (axis == 2 && W.first > 0) {
            slab.z0 = (uint32_t)W.first;
            slab.prev = (const uint8_t*)img + (W.first - 1) * stride;
        }
        MemSink ms(&enc.mem_out);
        const int rc = enc.encode((const uint8_t*)img + W.first * stride, false, hs, ms, &W.st, wthreads, &slab);
        {
            std::lock_guard<std::mutex> lk(mu);
            W.rc = rc;
            W.out = enc.mem_out.data();
            W.out_len = enc.mem_out.size();
            W.done = true;
        }
        cv.notify_all();
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return W.consumed; });
    };
    std::vector<std::thread> pool;
    pool.reserve(nw);
    for (int w = 0; w < nw; ++w) pool.emplace_back(worker, w);

    // in-order writer: the final header first (offsets rewritten at the end),
    // then each range's payload as soon as it and every range before it is done
    klb_image_header H(h);
    H.resizeBlockOffset(H.calculateNumBlocks());
    int rc = 0;
    uint64_t nb = 0, acc = 0;
    bool begun = false;
    auto consumed = [&](int w) {
        {
            std::lock_guard<std::mutex> lk(mu);
            work[w].consumed = true;
        }
        cv.notify_all();
    };
    for (int w = 0; w < nw; ++w) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return work[w].done; });
        }
        if (!rc) rc = work[w].rc;
        klb_image_header hs;
        if (!rc && hs.parseHeader(work[w].out, work[w].out_len)) rc = 3;
        if (!rc && !begun) {
            H.headerVersion = hs.headerVersion;
            rc = sink.begin(H);
            begun = true;
        }
        const uint64_t body = (!rc && hs.Nb) ? hs.blockOffset[hs.Nb - 1] : 0;
        if (!rc && (nb + hs.Nb > H.Nb || hs.getSizeInBytes() + body > work[w].out_len)) rc = 3;
        if (rc) {
            consumed(w);
            continue;
        }
        uint64_t prev_end = 0;
        for (size_t j = 0; j < hs.Nb; ++j) {
            acc += hs.blockOffset[j] - prev_end;
            prev_end = hs.blockOffset[j];
            H.blockOffset[nb++] = acc;
        }
        const uint8_t* src = work[w].out + hs.getSizeInBytes();
        if (sink.direct_capable()) {
            uint8_t* dst = sink.direct(body);
            if (!dst) rc = 3;
            else par_memcpy(dst, src, body, threads);
        } else {
            rc = sink.append(src, body);
        }
        consumed(w);
    }
    for (auto& t : pool) t.join();
    if (!rc && nb != H.Nb) rc = 3;
    if (!rc) rc = sink.finish(H);
    if (st) {
        for (const Work& W : work) {
            st->h2d_ms = std::max(st->h2d_ms, W.st.h2d_ms);
            st->predict_ms = std::max(st->predict_ms, W.st.predict_ms);
            st->d2h_ms = std::max(st->d2h_ms, W.st.d2h_ms);
            st->compress_ms = std::max(st->compress_ms, W.st.compress_ms);
        }
        st->total_ms = ms_since(t0);
        st->header_version = H.headerVersion;
        st->chosen = H.headerVersion & 0x7F;
        st->out_bytes = H.getSizeInBytes() + acc;
    }
    return rc;
}

} // namespace lfm
