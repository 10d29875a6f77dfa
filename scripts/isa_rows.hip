// isa_rows.hip -- compile-only probe (not part of the product): one kernel per
// predictor row variant of predict_vec, so `hipcc -S` shows the VALU work of
// one lane-row (8 pixels) of each (family, predictor, temporal, v==0, first
// strip) case in isolation.  scripts/isa_count.py counts the instructions.
#define LFM_PREDICT_NO_ENTRY
#include "../lightfieldmicroscopy_pc-bzip2_amd/csrc/lfm_predict.hip"
using namespace lfm;

template <int FAM, int K, int T, bool TEMP, bool V0, bool FIRST>
__global__ void isa_row(const uint16_t* src, v4u* dst, int x0, uint32_t u0bits)
{
    const uint16_t* p = src + 64 * threadIdx.x;
    VecRows rw;
    load_win(p + 32, rw.r0);
    load_win(p + 64, rw.r1);
    load_win(p + 96, rw.rT);
    load_win(p + 128, rw.rT1);
    const v4u pv = *(const v4u*)(p + 160);
    rw.p[0] = pv.x; rw.p[1] = pv.y; rw.p[2] = pv.z; rw.p[3] = pv.w;
    const LaneMasks lm = lane_masks(u0bits, x0, T);
    asm volatile("; ROW_BEGIN" ::: "memory");
    const v4u o = vec_fast_row<FAM, K, T, TEMP, V0, FIRST>(rw, u0bits, lm, x0);
    asm volatile("; ROW_END" ::: "memory");
    dst[threadIdx.x] = o;
}

#define ROWS(FAM, K, T)                                                                                       \
    template __global__ void isa_row<FAM, K, T, false, false, false>(const uint16_t*, v4u*, int, uint32_t);  \
    template __global__ void isa_row<FAM, K, T, false, true, false>(const uint16_t*, v4u*, int, uint32_t);   \
    template __global__ void isa_row<FAM, K, T, false, false, true>(const uint16_t*, v4u*, int, uint32_t);   \
    template __global__ void isa_row<FAM, K, T, true, false, false>(const uint16_t*, v4u*, int, uint32_t);   \
    template __global__ void isa_row<FAM, K, T, true, true, false>(const uint16_t*, v4u*, int, uint32_t);
ROWS(1, 0, 15)
ROWS(0, 4, 15)
ROWS(0, 4, 13)
ROWS(1, 4, 15)
ROWS(0, 1, 13)
ROWS(0, 2, 13)
ROWS(0, 3, 13)
ROWS(0, 5, 13)
ROWS(0, 6, 13)
ROWS(0, 7, 13)
