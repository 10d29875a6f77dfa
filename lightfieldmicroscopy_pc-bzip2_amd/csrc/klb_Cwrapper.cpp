// klb_Cwrapper.cpp -- the reference C ABI (src/klb_Cwrapper.h:40-64) on liblfm.
#include "klb_Cwrapper.h"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include "klb_imageIO.h"
#include "lfm_engine.h"

static void report_write_error(int e)
{
    switch (e) {
    case 2: std::printf("Error during BZIP compression of one of the blocks"); break;
    case 5: std::printf("Error generating the output file in the specified location"); break;
    case lfm::kErrBadPredictor: std::printf("Error: invalid predictor request in the header"); break;
    case lfm::kErrNoGpu: std::printf("Error: the predictor stage needs a GPU"); break;
    default: std::printf("Error writing the image");
    }
}

extern "C" int writeKLBstack(const void* im, const char* filename, uint32_t xyzct[KLB_DATA_DIMS],
                             enum KLB_DATA_TYPE dataType, int numThreads, float32_t pixelSize[KLB_DATA_DIMS],
                             uint32_t blockSize[KLB_DATA_DIMS], enum KLB_COMPRESSION_TYPE compressionType,
                             char metadata[KLB_METADATA_SIZE])
{
    klb_imageIO io{std::string(filename)};
    io.header.setHeader(xyzct, dataType, pixelSize, blockSize, compressionType, metadata);  // headerVersion 0, Nnum 13
    int e = io.writeImage((const char*)im, numThreads);
    if (e > 0) report_write_error(e);
    return e;
}

extern "C" int writeKLBstackSlices(const void** im, const char* filename, uint32_t xyzct[KLB_DATA_DIMS],
                                   enum KLB_DATA_TYPE dataType, int numThreads, float32_t pixelSize[KLB_DATA_DIMS],
                                   uint32_t blockSize[KLB_DATA_DIMS], enum KLB_COMPRESSION_TYPE compressionType,
                                   char metadata[KLB_METADATA_SIZE])
{
    klb_imageIO io{std::string(filename)};
    io.header.setHeader(xyzct, dataType, pixelSize, blockSize, compressionType, metadata);
    int e = io.writeImageStackSlices((const char**)im, numThreads);
    if (e == 3) std::printf("Error: number of channels or number of time points must be 1 for this API call\n");
    else if (e > 0) report_write_error(e);
    return e;
}

extern "C" int readKLBheader(const char* filename, uint32_t xyzct[KLB_DATA_DIMS], enum KLB_DATA_TYPE* dataType,
                             float32_t pixelSize[KLB_DATA_DIMS], uint32_t blockSize[KLB_DATA_DIMS],
                             enum KLB_COMPRESSION_TYPE* compressionType, char metadata[KLB_METADATA_SIZE])
{
    klb_image_header h;
    int e = h.readHeader(filename);
    if (e) return e;
    std::memcpy(xyzct, h.xyzct, sizeof(h.xyzct));
    *dataType = h.dataType;
    *compressionType = h.compressionType;
    std::memcpy(pixelSize, h.pixelSize, sizeof(h.pixelSize));
    std::memcpy(metadata, h.metadata, KLB_METADATA_SIZE);
    std::memcpy(blockSize, h.blockSize, sizeof(h.blockSize));
    return 0;
}

extern "C" void* readKLBstack(const char* filename, uint32_t xyzct[KLB_DATA_DIMS], enum KLB_DATA_TYPE* dataType,
                              int numThreads, float32_t pixelSize[KLB_DATA_DIMS], uint32_t blockSize[KLB_DATA_DIMS],
                              enum KLB_COMPRESSION_TYPE* compressionType, char metadata[KLB_METADATA_SIZE])
{
    klb_imageIO io{std::string(filename)};
    if (io.readHeader() > 0) return nullptr;
    void* im = std::malloc(io.header.getImageSizeBytes() ? io.header.getImageSizeBytes() : 1);
    if (!im) return nullptr;
    if (io.readImageFull((char*)im, numThreads) > 0) {
        std::free(im);
        return nullptr;
    }
    std::memcpy(xyzct, io.header.xyzct, sizeof(io.header.xyzct));
    *dataType = io.header.dataType;
    if (compressionType) *compressionType = io.header.compressionType;
    if (pixelSize) std::memcpy(pixelSize, io.header.pixelSize, sizeof(io.header.pixelSize));
    if (metadata) std::memcpy(metadata, io.header.metadata, KLB_METADATA_SIZE);
    if (blockSize) std::memcpy(blockSize, io.header.blockSize, sizeof(io.header.blockSize));
    return im;
}

extern "C" int readKLBstackInPlace(const char* filename, void* im, enum KLB_DATA_TYPE* dataType, int numThreads)
{
    klb_imageIO io{std::string(filename)};
    int e = io.readHeader();
    if (e > 0) return e;
    *dataType = io.header.dataType;
    return io.readImageFull((char*)im, numThreads);
}

extern "C" int readKLBroiInPlace(const char* filename, void* im, uint32_t xyzctLB[KLB_DATA_DIMS],
                                 uint32_t xyzctUB[KLB_DATA_DIMS], int numThreads)
{
    klb_imageIO io{std::string(filename)};
    klb_ROI roi;
    for (int d = 0; d < KLB_DATA_DIMS; ++d) {
        roi.xyzctLB[d] = xyzctLB[d];
        roi.xyzctUB[d] = xyzctUB[d];
    }
    return io.readImage((char*)im, &roi, numThreads);
}
