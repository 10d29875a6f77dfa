/*
 * klb_ROI.h -- inclusive box of interest, as in the reference (src/klb_ROI.h:24-48).
 */
#ifndef LFM_KLB_ROI_H
#define LFM_KLB_ROI_H

#include <cstdint>
#include "common.h"

class __attribute__((visibility("default"))) klb_ROI
{
public:
    std::uint32_t xyzctLB[KLB_DATA_DIMS];  // first index, included
    std::uint32_t xyzctUB[KLB_DATA_DIMS];  // last index, included

    void defineSlice(int val, int dim, const std::uint32_t xyzct[KLB_DATA_DIMS]);
    void defineFullImage(const std::uint32_t xyzct[KLB_DATA_DIMS]);
    std::uint32_t getSizePixels(int dim) const { return xyzctUB[dim] - xyzctLB[dim] + 1; }
    std::uint64_t getSizePixels() const
    {
        std::uint64_t n = 1;
        for (int d = 0; d < KLB_DATA_DIMS; ++d) n *= getSizePixels(d);
        return n;
    }
};

#endif
