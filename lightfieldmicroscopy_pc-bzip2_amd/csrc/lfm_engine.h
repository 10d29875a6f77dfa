// lfm_engine.h -- encode / decode engine behind klb_imageIO, the C ABI and
// the lfm_encoder API.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>
#include <hip/hip_runtime.h>
#include "klb_imageHeader.h"
#include "lfm_api.h"

namespace lfm {

// error codes beyond the reference's 2 / 3 / 5
constexpr int kErrBadPredictor = 6;
constexpr int kErrNoGpu = 7;
constexpr int kErrUnknownTicket = 8;  // lfm_encoder_wait: ticket never submitted or already recycled

bool gpu_bzip2_enabled();   // env LFM_GPU_BZIP2 (default on)
bool gpu_decode_enabled();  // env LFM_GPU_DECODE (default on): inverse predictor on the GPU
bool gpu_bunzip2_enabled(); // env LFM_GPU_BUNZIP2 (default on): bzip2 decode on the GPU
int default_threads();      // env LFM_NUM_THREADS, else OMP_NUM_THREADS, else hardware_concurrency
int current_family();       // lfm_set_family / env LFM_PREDICTOR_WAY / LFM_PREDICTOR_WAY
void set_family(int fam);

// x-fastest decomposition of the 5-D image into blocks (klb_imageIO.cpp:98-160)
struct BlockGrid {
    uint64_t dims[5], bs[5], nb[5], stride[5], nblocks;
    explicit BlockGrid(const klb_image_header& h);
    void block(uint64_t id, uint64_t origin[5], uint64_t size[5]) const;
};
void gather_block(const uint8_t* img, const BlockGrid& g, uint64_t id, size_t bpp, uint8_t* dst, size_t* nbytes);
void scatter_block(const uint8_t* blk, const BlockGrid& g, uint64_t id, size_t bpp, uint8_t* img);

// output of an encode: a file (reference writer order: header, blocks, then
// the offset table rewritten) or a memory buffer
class Sink {
public:
    virtual ~Sink() = default;
    virtual int begin(const klb_image_header& h) = 0;
    virtual int append(const uint8_t* p, size_t n) = 0;
    virtual int finish(const klb_image_header& h) = 0;
    // sinks backed by pinned host memory hand out the next n bytes of the
    // output so a device buffer can be copied straight into place
    virtual bool direct_capable() const { return false; }
    virtual uint8_t* direct(size_t) { return nullptr; }
    virtual void reserve_hint(size_t) {}
};

// growable pinned host buffer (the in-memory .lfm): device-to-host copies land
// in it at full DMA speed, and it is kept between encodes
class PinnedBuffer {
public:
    PinnedBuffer() = default;
    PinnedBuffer(const PinnedBuffer&) = delete;
    PinnedBuffer& operator=(const PinnedBuffer&) = delete;
    ~PinnedBuffer();
    bool reserve(size_t n);
    bool resize(size_t n);
    void clear() { size_ = 0; }
    uint8_t* data() { return p_; }
    const uint8_t* data() const { return p_; }
    size_t size() const { return size_; }
    size_t capacity() const { return cap_; }
private:
    uint8_t* p_ = nullptr;
    size_t size_ = 0, cap_ = 0;
    bool malloced_ = false;
};
class FileSink : public Sink {
public:
    explicit FileSink(FILE* f) : f_(f) {}
    int begin(const klb_image_header& h) override;
    int append(const uint8_t* p, size_t n) override;
    int finish(const klb_image_header& h) override;
private:
    FILE* f_;
    std::vector<char> vbuf_;
};
class MemSink : public Sink {
public:
    explicit MemSink(PinnedBuffer* out) : out_(out) {}
    int begin(const klb_image_header& h) override;
    int append(const uint8_t* p, size_t n) override;
    int finish(const klb_image_header& h) override;
    bool direct_capable() const override { return true; }
    uint8_t* direct(size_t n) override;
    // n is the worst case (every block stored at its raw size + bzip2's
    // overhead); beyond 8 GiB only 60 % of it is pinned up front (ratio >= 1.67
    // fits): a 100-volume config-5 stack (107 GB raw, 52 GB .lfm) would
    // otherwise pin 110 GB of host memory for its output.  A stack that
    // compresses worse grows the buffer once, straight to the worst case
    // (direct()): the peak is the old buffer plus n, 1.6 n; if n cannot be
    // pinned, the buffer grows by half its capacity at a time instead (first
    // step: 0.6 n + 0.9 n = 1.5 n).
    void reserve_hint(size_t n) override
    {
        const size_t big = (size_t)8 << 30;
        worst_ = n;
        (void)out_->reserve(n <= big ? n : std::max(big, n / 10 * 6));
    }
private:
    PinnedBuffer* out_;
    size_t worst_ = 0;
};

// Compress every block of `sym` (image layout, bpp bytes per pixel) in
// parallel and hand them to the sink in block order.  `h` must already hold
// the clamped block size; its blockOffset table is filled.
int compress_blocks(const uint8_t* sym, klb_image_header& h, Sink& sink, int threads, int level = -1);

// z-slab [z0, z0 + xyzct[2]) of a larger stack (c = t = 1): the temporal
// flag of frame z is video & (z0 + z), and the first frame's previous raw
// frame is `prev` (host or device like the image) when z0 is odd.
// level >= 1 overrides the bzip2 level rule (min(9, ceil(nominal block
// bytes / 1e5)), klb_imageIO.cpp:108): a range of a larger stack codes at the
// level of the whole stack's nominal block even when its own last block layer
// is shallower.
// select_frame: the frame auto-selection runs on (host or device like the
// image) instead of the image's own frame 0 -- the whole stack's frame 0 when
// this encode is a slab of it (klb_imageIO.cpp:2316-2360 selects on frame 0).
struct SlabSpec {
    uint32_t z0 = 0;
    const void* prev = nullptr;
    int level = -1;
    const void* select_frame = nullptr;
};

// clamp the block size to the dims and check the types (klb_imageIO.cpp:2402-2404)
int normalize_header(klb_image_header& h);
// bzip2 level of the reference's rule for the header's nominal block
int bzip2_level(const klb_image_header& h);
// multi-threaded memcpy (1 MiB pieces)
void par_memcpy(void* dst, const void* src, size_t n, int threads);

// Encoder: GPU predictor stage + block compression.  One per device; keeps
// device / pinned buffers between calls.
class Encoder {
public:
    explicit Encoder(int device);
    ~Encoder();
    // img: host pointer (dev=false) or device pointer on this encoder's device
    int encode(const void* img, bool dev, klb_image_header& h, Sink& sink, lfm_encode_stats* st, int threads,
               const SlabSpec* slab = nullptr);
    PinnedBuffer mem_out;
    int device() const { return device_; }
    // Pipelined encodes (lfm_encoder_submit / lfm_encoder_wait), two buffer
    // sets (symbols, bzip2 slots and workspaces, pinned output) used in turn:
    // submit runs the predictor stage of its stack into one set and hands the
    // GPU bzip2 + in-order assembly + payload copies to a finisher thread.
    // The next submit's GPU bzip2 starts once the previous encode's kernels
    // are done, so the next stack's kernels overlap its assembly and payload
    // copies (releasing it after its BWT or its MTF, so they also overlap its
    // latency-bound tail, measured 8 943 / 9 035 vs 9 098 Mpixel/s: the heap
    // chains slow down as much as the head gains).  At most two encodes are
    // in flight.  The input may be released when submit returns (the
    // predictor stage has consumed it).
    int submit(const void* img, bool dev, klb_image_header& h, int threads, const SlabSpec* slab, uint64_t* ticket);
    // wait for a submitted encode: its .lfm is *out (valid until the second
    // submit after it); stats as encode() reports them, d2h_ms including the
    // deferred copies
    int wait(uint64_t ticket, const PinnedBuffer** out, lfm_encode_stats* st);
    PinnedBuffer mem_ring[2];
    // predictor selection on one host frame (uploaded to this encoder's device)
    int select_host_frame(const void* frame, int W, int H, int T, int family, int* chosen, float entropy[8]);

private:
    // an encode in flight (submit): its finisher thread and the release point
    struct Inflight {
        uint64_t ticket = 0;  // 0: none
        std::thread th;       // GPU bzip2, in-order assembly, payload copies
        int rc = 0;
        lfm_encode_stats st{};
        std::mutex mu;
        std::condition_variable cv;
        int reached = 0;      // batches of the last round past the release stage
        int need = 0;         // ... needed to release the next submit (0: not yet known)
        bool released = true;
        int reached2 = 0;     // batches of the last round past the MTF stage (stage 2)
        bool mtf_done = true; // every last-round batch is past stage 2 (or released)
        void release();
        void wait_release();
        void reach();         // one last-round batch passed the release stage
        void reach2();        // one last-round batch passed its MTF stage
        void wait_mtf();
    };
    // Host stacks for the GPU bzip2 path go up in chunks of whole frames on
    // up_stream_ (one uploader thread per encode), each chunk predicted on
    // stream_ as soon as it has landed; the GPU bzip2 batches wait (event)
    // only for the chunks that hold their blocks, so the PCIe upload overlaps
    // the compression of the layers already predicted.  Chunks pass through a
    // ring of device slots (LFM_H2D_RING_MB), so the stack's size is not
    // bounded by it.  LFM_H2D_PIPE=0: the whole volume is uploaded first.
    struct UploadPipe {
        std::thread th;
        std::mutex mu;
        std::condition_variable cv;
        std::vector<hipEvent_t> ev;  // pool: 2 per chunk (predict start / end), kept between encodes
        std::vector<uint64_t> end;   // per chunk: flattened frame index (v * Z + z) past its last frame
        size_t nchunks = 0, recorded = 0;  // chunks whose "predicted" event is recorded
        int rc = 0;
        bool active = false;
        double h2d_ms = 0.0, predict_ms = 0.0;
        // SDMA copies (HSA async copies, not a blit kernel beside the GPU
        // bzip2): completion signals and, for pageable sources, two pinned
        // staging chunks; kept between encodes
        uint64_t sig[2] = {0, 0};
        void* stage[2] = {nullptr, nullptr};
        size_t stage_cap = 0;
        void release_sdma();
        // make `st` wait until frames [0, f_end) are predicted (0 or 3)
        int wait_frames(uint64_t f_end, hipStream_t st);
        void join();
    };
    int start_upload(const void* img, klb_image_header& h, const SlabSpec& slab, int k, int set);
    bool upload_pipe_ok(bool dev, const klb_image_header& h) const;
    int predictor_stage(const void* img, bool dev, klb_image_header& h, const uint8_t** sym, const uint8_t** dsym,
                        lfm_encode_stats* st, const SlabSpec& slab, int set);
    int gpu_compress(const uint8_t* d_sym, klb_image_header& h, Sink& sink, lfm_encode_stats* st, int level, int set,
                     Inflight* fly);
    int encode_set(const void* img, bool dev, klb_image_header& h, Sink& sink, lfm_encode_stats* st, int threads,
                   const SlabSpec* slab, int set);
    int preselect(const void* img, bool dev, const klb_image_header& h, const SlabSpec& slab, int* k, float ent[8]);
    int ensure_gpu();
    int after_caller(bool dev);
    void* dev_alloc(void*& p, size_t& cap, size_t need);
    void join_inflight();
    Inflight fly_[2];                         // by buffer set
    UploadPipe up_[2];                        // by buffer set
    hipStream_t up_stream_ = nullptr;         // host -> device chunk copies
    uint64_t next_ticket_ = 1;
    int par_ = 0;                             // buffer set of the next submit
    hipStream_t copy_stream_ = nullptr;       // payload copies the SDMA path cannot take
    int device_;
    bool gpu_ready_ = false;
    hipStream_t stream_ = nullptr;
    hipEvent_t ev0_ = nullptr, ev1_ = nullptr;
    hipEvent_t caller_ev_ = nullptr;          // the null stream's work before a device input
    void* d_in_ = nullptr;  size_t d_in_cap_ = 0;
    void* d_sym_[2] = {nullptr, nullptr}; size_t d_sym_cap_[2] = {0, 0};  // by buffer set
    void* d_ws_ = nullptr;  size_t d_ws_cap_ = 0;
    void* d_prev_ = nullptr; size_t d_prev_cap_ = 0;
    void* d_sel_ = nullptr; size_t d_sel_cap_ = 0;  // host select_frame uploaded
    // GPU bzip2 pipeline slots (stream, workspace, device + pinned output),
    // kBzSlots per buffer set (LFM_BZ2_SLOTS picks how many run, at most that)
    static constexpr int kBzSlots = 4;
    struct BzSlot {
        hipStream_t stream = nullptr;
        void* d_ws = nullptr; size_t d_ws_cap = 0;
        void* d_out = nullptr; size_t d_out_cap = 0;
        void* h_out = nullptr; size_t h_out_cap = 0;
    };
    BzSlot bz_[2][kBzSlots];
    static int bz_slot_count();  // slots that run (env LFM_BZ2_SLOTS, default 2)
    void* h_sym_[2] = {nullptr, nullptr}; size_t h_sym_cap_[2] = {0, 0};   // pinned, by buffer set
};

// process-wide encoders for the C ABI / klb_imageIO, one per (device, worker
// slot), kept between calls; `lock` holds the entry while it is used
Encoder& shared_encoder(std::unique_lock<std::mutex>& lock);
Encoder& pooled_encoder(int dev, int slot, std::unique_lock<std::mutex>& lock);
void release_pooled_encoders();

// devices the writer farms block ranges to: lfm_set_devices, else env
// LFM_GPUS ("0,1,2" or a count), else the current device when the process is one
// rank of a one-process-per-GPU job (WORLD_SIZE / LOCAL_WORLD_SIZE > 1), else
// every visible device
std::vector<int> encode_devices();
// the default device list for n visible devices, `current` the caller's device (-1: unknown)
std::vector<int> default_devices(int n, int current);
void set_encode_devices(const std::vector<int>& devs);

// Multi-GPU writer (lfm_multigpu.cpp): host image, block-layer ranges farmed
// to `devs` (one host thread each), selection once on frame 0, in-order
// append to `sink`.  Returns -1 when the image does not split into two or
// more ranges (the caller then encodes on one device).
int encode_multi(const void* img, klb_image_header& h, Sink& sink, lfm_encode_stats* st, int threads,
                 const std::vector<int>& devs);

// Assemble one .lfm from the .lfm files of consecutive z-slabs of a stack
// (each encoded with the same forced predictor, slab i starting at the sum of
// the previous depths, depths multiples of the block depth except the last):
// the blocks of a slab are a contiguous id range of the whole stack's blocks,
// so the payloads concatenate and the offset table is re-accumulated.
int merge_slabs(const uint8_t* const* slabs, const uint64_t* lens, int n, std::vector<uint8_t>* out);

// Decode the payload of a .lfm (bytes after the header) into img.
int decode_payload(const uint8_t* payload, size_t len, const klb_image_header& h, uint8_t* img, int threads,
                   int family);
int decode_file(const char* filename, klb_image_header& h, std::vector<uint8_t>* img_out, uint8_t* img_into,
                int threads);
// ROI read: only the blocks the ROI depends on are decoded (lb / ub inclusive)
int decode_roi(const uint8_t* payload, size_t len, const klb_image_header& h, const uint32_t lb[5],
               const uint32_t ub[5], uint8_t* out, int threads, int family);
int decode_file_roi(const char* filename, klb_image_header& h, const uint32_t lb[5], const uint32_t ub[5],
                    uint8_t* out, int threads);

} // namespace lfm
