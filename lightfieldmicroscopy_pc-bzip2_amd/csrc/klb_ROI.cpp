// klb_ROI.cpp -- inclusive region helpers (reference src/klb_ROI.cpp).
#include "klb_ROI.h"

void klb_ROI::defineSlice(int val, int dim, const std::uint32_t xyzct[KLB_DATA_DIMS])
{
    defineFullImage(xyzct);
    xyzctLB[dim] = (std::uint32_t)val;
    xyzctUB[dim] = (std::uint32_t)val;
}

void klb_ROI::defineFullImage(const std::uint32_t xyzct[KLB_DATA_DIMS])
{
    for (int d = 0; d < KLB_DATA_DIMS; ++d) {
        xyzctLB[d] = 0;
        xyzctUB[d] = xyzct[d] - 1;
    }
}
