/*
 * klb_imageIO.h -- encode/decode engine of the .lfm container.
 *
 * Same public surface as the reference class (src/klb_imageIO.h:47-135) so
 * the MEX sources in matlabWrapper/ relink unchanged: public `header` and
 * `numThreads`, writeImage / writeImageStackSlices / readImage /
 * readImageFull / readHeader.  The implementation is MI355X-native: the
 * predictor stage and the predictor selection run as HIP kernels on the GPU
 * (lfm_hip.h) for whole stacks at once, and so does bzip2: every block is
 * compressed on the GPU, byte-identical to libbzip2 1.0.6 (the host library
 * only takes the rare streams the device flags).  writeImage farms block-layer
 * ranges over the node's GPUs (lfm_set_devices / LFM_GPUS; one device per
 * rank in a one-process-per-GPU job) with an in-order writer; readImageFull
 * decodes on the GPU (bzip2 decode + inverse predictor).
 */
#ifndef LFM_KLB_IMAGE_IO_H
#define LFM_KLB_IMAGE_IO_H

#include <atomic>
#include <string>
#include <cstdint>
#include "klb_imageHeader.h"
#include "klb_ROI.h"

class __attribute__((visibility("default"))) klb_imageIO
{
public:
    klb_image_header header;
    int numThreads;

    klb_imageIO();
    explicit klb_imageIO(const std::string& filename_);

    std::string getFilename() const { return filename; }
    void setFilename(const std::string& filename_) { filename = filename_; }

    int readHeader() { return header.readHeader(filename.c_str()); }
    int readHeader(const std::string& filename_)
    {
        filename = filename_;
        return readHeader();
    }

    /* Encode `img` (layout x fastest, then y, z, c, t) with the current header
     * to getFilename().  headerVersion bits 0-6 < 8 auto-select the predictor
     * on frame 0, 8..15 force predictor (request - 8); bit 7 = video. */
    int writeImage(const char* img, int numThreads);
    int writeImageStackSlices(const char** img, int numThreads);

    int readImage(char* img, const klb_ROI* ROI, int numThreads);
    int readImageFull(char* img, int numThreads);

    /* Selection helpers kept public as in the reference (src/klb_imageIO.h:91,101).
     * Device pointers on the current HIP device.  bwt_entropy_2D: 2D entropy of
     * header.getImageSizePixels() symbols (x0.96 into *entropy when is_src == 0;
     * the unscaled value is returned).  predict_and_2DEntropy: candidates
     * k = (*blockId)++ < numPredictors into out[k], scored into entropy[k]. */
    float bwt_entropy_2D(uint16_t* In, float* entropy, int is_src);
    int predict_and_2DEntropy(uint16_t* In, uint16_t** out, float* entropy, std::atomic<uint64_t>* blockId,
                              int numPredictors);

private:
    std::string filename;
};

#endif
