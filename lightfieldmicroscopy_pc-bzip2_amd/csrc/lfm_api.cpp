// lfm_api.cpp -- liblfm extensions (lfm_api.h).
#include "lfm_api.h"
#include <cstdlib>
#include <cstring>
#include <string>
#include "klb_imageIO.h"
#include "lfm_engine.h"

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
extern "C" const char* lfm_version(void) { return "lfm-mi355x 0.1 (gfx950)"; }

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

extern "C" int lfm_decode_memory(const uint8_t* buf, uint64_t len, void* img, int numThreads)
{
    klb_image_header h;
    int rc = h.parseHeader(buf, len);
    if (rc) return rc;
    const size_t hs = h.getSizeInBytes();
    return lfm::decode_payload(buf + hs, len - hs, h, (uint8_t*)img, numThreads, lfm::current_family());
}
