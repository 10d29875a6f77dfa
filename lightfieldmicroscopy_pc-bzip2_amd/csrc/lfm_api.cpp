// lfm_api.cpp -- liblfm extensions (lfm_api.h).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include "lfm_api.h"
#include <cstdlib>
#include <cstring>
#include <string>
#include "klb_imageIO.h"
#include "lfm_engine.h"
#include "lfm_hip.h"
#include <vector>

struct lfm_encoder {
    lfm::Encoder enc;
    int threads;
    lfm_encoder(int device, int threads_) : enc(device), threads(threads_) {}
};

extern "C" int lfm_set_family(int family)
{
    if (family < 0 || family > 2) return 1;
    lfm::set_family(family);
    return 0;
}
extern "C" int lfm_get_family(void) { return lfm::current_family(); }
extern "C" const char* lfm_version(void) { return "lfm-mi355x 0.2 (gfx950, api 2)"; }
extern "C" int lfm_api_version(void) { return LFM_API_VERSION; }

extern "C" int writeLFMstack_c(const void* im, const char* filename, const uint32_t xyzct[KLB_DATA_DIMS],
                               int dataType, int numThreads, const float pixelSize[KLB_DATA_DIMS],
                               const uint32_t blockSize[KLB_DATA_DIMS], int compressionType,
                               const char metadata[KLB_METADATA_SIZE], int predictor_request, int Nnum, int video)
{
    klb_imageIO io{std::string(filename)};
    io.header.setHeader(xyzct, (KLB_DATA_TYPE)dataType, pixelSize, blockSize, (KLB_COMPRESSION_TYPE)compressionType,
                        metadata);
    // matlabWrapper/writeLFMstack.cpp:360-433: headerVersion |= predictor; Nnum; |= video << 7
    io.header.headerVersion = (uint8_t)(io.header.headerVersion | (uint8_t)predictor_request);
    io.header.Nnum = (uint8_t)Nnum;
    io.header.headerVersion = (uint8_t)(io.header.headerVersion | ((uint8_t)video << 7));
    return io.writeImage((const char*)im, numThreads);
}

extern "C" int readLFMstack_c(const char* filename, void* im, int numThreads, uint8_t* headerVersion, uint8_t* Nnum)
{
    klb_imageIO io{std::string(filename)};
    int e = io.readHeader();
    if (e) return e;
    e = io.readImageFull((char*)im, numThreads);
    if (headerVersion) *headerVersion = io.header.headerVersion;
    if (Nnum) *Nnum = io.header.Nnum;
    return e;
}

extern "C" lfm_encoder* lfm_encoder_create(int device, int numThreads)
{
    return new lfm_encoder(device, numThreads);
}
extern "C" void lfm_encoder_destroy(lfm_encoder* e) { delete e; }

extern "C" int lfm_encoder_encode(lfm_encoder* e, const void* img, int img_is_device,
                                  const uint32_t xyzct[KLB_DATA_DIMS], int dataType, int headerVersion, int Nnum,
                                  const uint32_t blockSize[KLB_DATA_DIMS], int compressionType,
                                  const char metadata[KLB_METADATA_SIZE], const uint8_t** out, uint64_t* out_len,
                                  lfm_encode_stats* stats)
{
    if (!e || !img || !out || !out_len) return 3;
    klb_image_header h;
    h.setHeader(xyzct, (KLB_DATA_TYPE)dataType, nullptr, blockSize, (KLB_COMPRESSION_TYPE)compressionType, metadata,
                (uint8_t)headerVersion, (uint8_t)Nnum);
    lfm::MemSink sink(&e->enc.mem_out);
    int rc = e->enc.encode(img, img_is_device != 0, h, sink, stats, e->threads);
    *out = e->enc.mem_out.data();
    *out_len = e->enc.mem_out.size();
    return rc;
}

extern "C" int lfm_encoder_encode_slab(lfm_encoder* e, const void* img, int img_is_device, const void* prev_frame,
                                       uint32_t z0, const uint32_t xyzct[KLB_DATA_DIMS], int dataType,
                                       int headerVersion, int Nnum, const uint32_t blockSize[KLB_DATA_DIMS],
                                       int compressionType, const char metadata[KLB_METADATA_SIZE],
                                       const uint8_t** out, uint64_t* out_len, lfm_encode_stats* stats)
{
    if (!e || !img || !out || !out_len) return 3;
    klb_image_header h;
    h.setHeader(xyzct, (KLB_DATA_TYPE)dataType, nullptr, blockSize, (KLB_COMPRESSION_TYPE)compressionType, metadata,
                (uint8_t)headerVersion, (uint8_t)Nnum);
    lfm::SlabSpec slab;
    slab.z0 = z0;
    slab.prev = prev_frame;
    lfm::MemSink sink(&e->enc.mem_out);
    int rc = e->enc.encode(img, img_is_device != 0, h, sink, stats, e->threads, &slab);
    *out = e->enc.mem_out.data();
    *out_len = e->enc.mem_out.size();
    return rc;
}

extern "C" int lfm_encoder_submit(lfm_encoder* e, const void* img, int img_is_device, const void* prev_frame,
                                  uint32_t z0, const uint32_t xyzct[KLB_DATA_DIMS], int dataType, int headerVersion,
                                  int Nnum, const uint32_t blockSize[KLB_DATA_DIMS], int compressionType,
                                  const char metadata[KLB_METADATA_SIZE], uint64_t* ticket)
{
    if (!e || !img || !ticket) return 3;
    klb_image_header h;
    h.setHeader(xyzct, (KLB_DATA_TYPE)dataType, nullptr, blockSize, (KLB_COMPRESSION_TYPE)compressionType, metadata,
                (uint8_t)headerVersion, (uint8_t)Nnum);
    lfm::SlabSpec slab;
    slab.z0 = z0;
    slab.prev = prev_frame;
    return e->enc.submit(img, img_is_device != 0, h, e->threads, &slab, ticket);
}

extern "C" int lfm_encoder_submit_select(lfm_encoder* e, const void* img, int img_is_device, const void* prev_frame,
                                         uint32_t z0, const void* select_frame, const uint32_t xyzct[KLB_DATA_DIMS],
                                         int dataType, int headerVersion, int Nnum,
                                         const uint32_t blockSize[KLB_DATA_DIMS], int compressionType,
                                         const char metadata[KLB_METADATA_SIZE], uint64_t* ticket)
{
    if (!e || !img || !ticket) return 3;
    klb_image_header h;
    h.setHeader(xyzct, (KLB_DATA_TYPE)dataType, nullptr, blockSize, (KLB_COMPRESSION_TYPE)compressionType, metadata,
                (uint8_t)headerVersion, (uint8_t)Nnum);
    lfm::SlabSpec slab;
    slab.z0 = z0;
    slab.prev = prev_frame;
    slab.select_frame = select_frame;
    return e->enc.submit(img, img_is_device != 0, h, e->threads, &slab, ticket);
}

extern "C" int lfm_encoder_wait(lfm_encoder* e, uint64_t ticket, const uint8_t** out, uint64_t* out_len,
                                lfm_encode_stats* stats)
{
    if (!e || !out || !out_len) return 3;
    const lfm::PinnedBuffer* b = nullptr;
    const int rc = e->enc.wait(ticket, &b, stats);
    // a failed encode leaves an earlier encode's bytes in that buffer set:
    // hand out nothing rather than a stale .lfm
    *out = (b && rc == 0) ? b->data() : nullptr;
    *out_len = (b && rc == 0) ? b->size() : 0;
    return rc;
}

extern "C" int lfm_set_devices(const int* devices, int n)
{
    if (n < 0 || (n > 0 && !devices)) return 3;
    std::vector<int> d(devices, devices + n);
    const int count = lfm_hip_device_count();
    for (int v : d)
        if (v < 0 || v >= count) return 3;
    lfm::set_encode_devices(d);
    return 0;
}

extern "C" int lfm_get_devices(int* devices, int cap)
{
    const std::vector<int> d = lfm::encode_devices();
    for (int i = 0; i < cap && i < (int)d.size(); ++i) devices[i] = d[i];
    return (int)d.size();
}

extern "C" int lfm_default_devices(int n_visible, int current, int* devices, int cap)
{
    const std::vector<int> d = lfm::default_devices(n_visible, current);
    for (int i = 0; i < cap && i < (int)d.size(); ++i) devices[i] = d[i];
    return (int)d.size();
}

extern "C" int lfm_encoder_encode_multi(lfm_encoder* e, const void* img, const uint32_t xyzct[KLB_DATA_DIMS],
                                        int dataType, int headerVersion, int Nnum,
                                        const uint32_t blockSize[KLB_DATA_DIMS], int compressionType,
                                        const char metadata[KLB_METADATA_SIZE], const uint8_t** out,
                                        uint64_t* out_len, lfm_encode_stats* stats)
{
    if (!e || !img || !out || !out_len) return 3;
    klb_image_header h;
    h.setHeader(xyzct, (KLB_DATA_TYPE)dataType, nullptr, blockSize, (KLB_COMPRESSION_TYPE)compressionType, metadata,
                (uint8_t)headerVersion, (uint8_t)Nnum);
    lfm::MemSink sink(&e->enc.mem_out);
    int rc = lfm::encode_multi(img, h, sink, stats, e->threads, lfm::encode_devices());
    if (rc == -1) rc = e->enc.encode(img, false, h, sink, stats, e->threads);
    *out = e->enc.mem_out.data();
    *out_len = e->enc.mem_out.size();
    return rc;
}

extern "C" void lfm_release_encoders(void) { lfm::release_pooled_encoders(); }

extern "C" int lfm_merge_slabs(const uint8_t* const* slabs, const uint64_t* lens, int nslabs, uint8_t** out,
                               uint64_t* out_len)
{
    if (!out || !out_len) return 3;
    *out = nullptr;
    *out_len = 0;
    std::vector<uint8_t> v;
    int rc = lfm::merge_slabs(slabs, lens, nslabs, &v);
    if (rc) return rc;
    *out = (uint8_t*)std::malloc(v.size() ? v.size() : 1);
    if (!*out) return 3;
    std::memcpy(*out, v.data(), v.size());
    *out_len = v.size();
    return 0;
}

extern "C" void lfm_free(void* p) { std::free(p); }

extern "C" int lfm_slab_info(const uint8_t* slab, uint64_t len, uint64_t* payload_bytes, uint64_t* nblocks)
{
    klb_image_header h;
    if (!slab || h.parseHeader(slab, len)) return 3;
    const uint64_t body = h.Nb ? h.blockOffset[h.Nb - 1] : 0;
    if (h.getSizeInBytes() + body > len) return 3;
    if (payload_bytes) *payload_bytes = body;
    if (nblocks) *nblocks = h.Nb;
    return 0;
}

extern "C" int lfm_place_slab(const uint8_t* slab, uint64_t slab_len, uint8_t* dst, uint64_t dst_len,
                              uint32_t total_z, uint64_t total_blocks, uint64_t block_index, uint64_t payload_offset,
                              int numThreads)
{
    klb_image_header h;
    if (!slab || !dst || h.parseHeader(slab, slab_len)) return 3;
    if (h.xyzct[3] != 1 || h.xyzct[4] != 1 || block_index + h.Nb > total_blocks) return 3;
    const uint64_t body = h.Nb ? h.blockOffset[h.Nb - 1] : 0;
    const uint64_t hsz = 320 + 8 * total_blocks;
    if (h.getSizeInBytes() + body > slab_len || hsz + payload_offset + body > dst_len) return 3;
    if (block_index == 0) {  // the whole stack's fixed header (the offset table follows from every rank)
        klb_image_header H(h);
        H.xyzct[2] = total_z;
        H.resizeBlockOffset(0);
        if (H.calculateNumBlocks() != total_blocks) return 3;
        H.serialize(dst, 320);
    }
    uint64_t* table = (uint64_t*)(dst + 320);  // little-endian host (x86-64)
    for (size_t j = 0; j < h.Nb; ++j) table[block_index + j] = payload_offset + h.blockOffset[j];
    lfm::par_memcpy(dst + hsz + payload_offset, slab + h.getSizeInBytes(), body,
                    numThreads > 0 ? numThreads : lfm::default_threads());
    return 0;
}

extern "C" int lfm_decode_memory(const uint8_t* buf, uint64_t len, void* img, int numThreads)
{
    const auto t0 = std::chrono::steady_clock::now();
    klb_image_header h;
    int rc = h.parseHeader(buf, len);
    if (rc) return rc;
    const size_t hs = h.getSizeInBytes();
    rc = lfm::decode_payload(buf + hs, len - hs, h, (uint8_t*)img, numThreads, lfm::current_family());
    if (std::getenv("LFM_DECODE_TIMING"))
        std::fprintf(stderr, "decode total (C)     %8.2f ms\n",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    return rc;
}

extern "C" int lfm_decode_memory_roi(const uint8_t* buf, uint64_t len, const uint32_t lb[KLB_DATA_DIMS],
                                     const uint32_t ub[KLB_DATA_DIMS], void* out, uint64_t out_bytes, int numThreads)
{
    if (!buf || !lb || !ub || !out) return 3;
    klb_image_header h;
    int rc = h.parseHeader(buf, len);
    if (rc) return rc;
    uint64_t need = h.getBytesPerPixel();  // the region in the file's own data type
    for (int d = 0; d < KLB_DATA_DIMS; ++d) {
        if (ub[d] < lb[d] || ub[d] >= h.xyzct[d]) return 3;
        need *= (uint64_t)(ub[d] - lb[d] + 1);
    }
    if (!need || out_bytes < need) return 3;
    const size_t hs = h.getSizeInBytes();
    return lfm::decode_roi(buf + hs, len - hs, h, lb, ub, (uint8_t*)out, numThreads, lfm::current_family());
}
