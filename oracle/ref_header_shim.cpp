// Driver for the reference's own header class (TEST INFRASTRUCTURE ONLY).
// Compiled together with /root/reference/src/klb_imageHeader.cpp by
// oracle/Makefile into oracle/_ref/libklbheader_ref.so; it lets tests produce
// the reference's header bytes (klb_imageHeader.cpp:164-176) for a given
// header state.  No reference source is copied into the repository.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "klb_imageHeader.h"

extern "C" int ref_header_bytes(const uint32_t xyzct[5], int dataType, const float pixelSize[5],
                                const uint32_t blockSize[5], int compressionType, const char metadata[256],
                                int headerVersion, int Nnum, const uint64_t* blockOffset, size_t Nb,
                                unsigned char* out, size_t outCap)
{
    klb_image_header h;
    h.setHeader(xyzct, (KLB_DATA_TYPE)dataType, pixelSize, blockSize, (KLB_COMPRESSION_TYPE)compressionType,
                metadata, (std::uint8_t)headerVersion, (std::uint8_t)Nnum);
    if (h.calculateNumBlocks() != Nb) return -1;
    h.resizeBlockOffset(Nb);
    std::memcpy(h.blockOffset, blockOffset, Nb * sizeof(uint64_t));
    char* buf = nullptr;
    size_t len = 0;
    FILE* f = open_memstream(&buf, &len);
    h.writeHeader(f);
    std::fclose(f);
    int rc = (int)len;
    if (len > outCap) rc = -2;
    else std::memcpy(out, buf, len);
    std::free(buf);
    return rc;
}

extern "C" long long ref_num_blocks(const uint32_t xyzct[5], const uint32_t blockSize[5])
{
    klb_image_header h;
    h.setHeader(xyzct, UINT16_TYPE, nullptr, blockSize);
    return (long long)h.calculateNumBlocks();
}
