// klb_imageIO.cpp -- the reference's klb_imageIO surface over the MI355X engine.
#include "klb_imageIO.h"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>
#include "lfm_engine.h"

klb_imageIO::klb_imageIO() : numThreads(lfm::default_threads()) {}
klb_imageIO::klb_imageIO(const std::string& filename_) : numThreads(lfm::default_threads()), filename(filename_) {}

int klb_imageIO::writeImage(const char* img, int nThreads)
{
    if (nThreads <= 0) nThreads = lfm::default_threads();
    FILE* f = std::fopen(filename.c_str(), "wb");
    if (!f) {
        std::printf("ERROR: file %s could not be opened\n", filename.c_str());
        return 5;
    }
    std::unique_lock<std::mutex> lk;
    lfm::Encoder& enc = lfm::shared_encoder(lk);
    lfm::FileSink sink(f);
    int rc = enc.encode(img, false, header, sink, nullptr, nThreads);
    std::fclose(f);
    return rc;
}

int klb_imageIO::writeImageStackSlices(const char** img, int nThreads)
{
    // one pointer per xy slice; no predictor stage (as klb_imageIO.cpp:2496-2610)
    if (header.xyzct[3] != 1 || header.xyzct[4] != 1) return 3;
    if (nThreads <= 0) nThreads = lfm::default_threads();
    const size_t slice = (size_t)header.xyzct[0] * header.xyzct[1] * header.getBytesPerPixel();
    std::vector<uint8_t> stack(slice * header.xyzct[2]);
    for (uint32_t z = 0; z < header.xyzct[2]; ++z) std::memcpy(stack.data() + z * slice, img[z], slice);
    FILE* f = std::fopen(filename.c_str(), "wb");
    if (!f) return 5;
    for (int d = 0; d < KLB_DATA_DIMS; ++d) header.blockSize[d] = std::min(header.blockSize[d], header.xyzct[d]);
    lfm::FileSink sink(f);
    int rc = lfm::compress_blocks(stack.data(), header, sink, nThreads);
    std::fclose(f);
    return rc;
}

int klb_imageIO::readImageFull(char* img, int nThreads)
{
    if (filename.empty()) return 3;
    if (nThreads <= 0) nThreads = lfm::default_threads();
    return lfm::decode_file(filename.c_str(), header, nullptr, (uint8_t*)img, nThreads);
}

int klb_imageIO::readImage(char* img, const klb_ROI* roi, int nThreads)
{
    // decode the blocks the ROI depends on (all of them up / left of it in its
    // frames when predictors are on), then crop: lfm::decode_roi.  The
    // reference's block-ROI path cannot undo predictors (klb_imageIO.cpp:2614-2682)
    if (filename.empty() || !roi) return 3;
    if (nThreads <= 0) nThreads = lfm::default_threads();
    return lfm::decode_file_roi(filename.c_str(), header, roi->xyzctLB, roi->xyzctUB, (uint8_t*)img, nThreads);
}
