// klb_imageIO.cpp -- the reference's klb_imageIO surface over the MI355X engine.
#include "klb_imageIO.h"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>
#include "lfm_engine.h"
#include "lfm_hip.h"

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
    lfm::FileSink sink(f);
    // the block scheduler farms block-layer ranges over every device of
    // lfm_set_devices / LFM_GPUS / all visible GPUs (lfm_multigpu.cpp); one
    // device, or an image of one range, encodes on the current device
    int rc = lfm::encode_multi(img, header, sink, nullptr, nThreads, lfm::encode_devices());
    if (rc == -1) {
        std::unique_lock<std::mutex> lk;
        lfm::Encoder& enc = lfm::shared_encoder(lk);
        rc = enc.encode(img, false, header, sink, nullptr, nThreads);
    }
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
    // the slices are written raw: a predictor request in the header would
    // make readers apply an inverse predictor to unpredicted data
    header.headerVersion &= 0x80;
    lfm::FileSink sink(f);
    int rc = lfm::compress_blocks(stack.data(), header, sink, nThreads);
    std::fclose(f);
    return rc;
}

float klb_imageIO::bwt_entropy_2D(uint16_t* In, float* entropy, int is_src)
{
    // klb_imageIO.cpp:2030-2093: 2D entropy of a device candidate buffer of
    // header.getImageSizePixels() symbols; candidate 0 (is_src == 0) is
    // reported x0.96, the unscaled value is returned.  The reference multiplies
    // the float by the DOUBLE literal 0.96 and stores the product back into a
    // float (`*entropy = entropy_A*0.96`, klb_imageIO.cpp:2090): promote,
    // multiply in double, round once -- e * 0.96f can differ in the last bit.
    float e = 0.f;
    if (lfm_hip_entropy2d(In, header.getImageSizePixels(), &e, nullptr) != LFM_HIP_OK) return -1.f;
    if (entropy) *entropy = is_src != 0 ? e : (float)((double)e * 0.96);
    return e;
}

int klb_imageIO::predict_and_2DEntropy(uint16_t* In, uint16_t** out, float* entropy, std::atomic<uint64_t>* blockId,
                                       int numPredictors)
{
    // klb_imageIO.cpp:2197-2225: candidates k = atomic counter < numPredictors,
    // each predicted over the header's frames (device buffers) and scored
    const int W = header.xyzct[0], H = header.xyzct[1], Z = header.xyzct[2];
    const int video = (header.headerVersion >> 7) & 1;
    for (;;) {
        const uint64_t k = blockId->fetch_add(1);
        if (k >= (uint64_t)numPredictors) break;
        if (lfm_hip_predict(In, nullptr, out[k], W, H, Z, header.Nnum, lfm::current_family(), (int)k, video, 0,
                            nullptr) != LFM_HIP_OK)
            return 1;
        if (bwt_entropy_2D(out[k], &entropy[k], (int)k) < 0.f) return 1;
    }
    return 0;
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
