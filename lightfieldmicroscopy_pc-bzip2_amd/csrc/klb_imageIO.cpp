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
    // decode the whole image, then crop (the reference's block-ROI path cannot
    // undo predictors, klb_imageIO.cpp:2614-2682)
    if (filename.empty()) return 3;
    std::vector<uint8_t> full;
    int rc = lfm::decode_file(filename.c_str(), header, &full, nullptr, nThreads);
    if (rc) return rc;
    const size_t bpp = header.getBytesPerPixel();
    uint64_t lb[5], ub[5], stride[5], s = 1;
    for (int d = 0; d < 5; ++d) {
        lb[d] = roi->xyzctLB[d];
        ub[d] = roi->xyzctUB[d];
        if (ub[d] < lb[d] || ub[d] >= header.xyzct[d]) return 3;
        stride[d] = s;
        s *= header.xyzct[d];
    }
    const size_t row = (ub[0] - lb[0] + 1) * bpp;
    uint8_t* out = (uint8_t*)img;
    for (uint64_t t = lb[4]; t <= ub[4]; ++t)
        for (uint64_t c = lb[3]; c <= ub[3]; ++c)
            for (uint64_t z = lb[2]; z <= ub[2]; ++z)
                for (uint64_t y = lb[1]; y <= ub[1]; ++y) {
                    const uint64_t e = lb[0] + y * stride[1] + z * stride[2] + c * stride[3] + t * stride[4];
                    std::memcpy(out, full.data() + e * bpp, row);
                    out += row;
                }
    return 0;
}
