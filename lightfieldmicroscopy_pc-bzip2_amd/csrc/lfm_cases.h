// lfm_cases.h -- per-case prediction formulas of the three predictor families.
//
// Every reference kernel (_predictorK_{tiles,angle,space}, lfm_Predictors*.cu)
// has the same decision tree: tile case {tx==0&&ty==0, tx==0, ty==0, other} x
// position case {u==0&&v>0, u==0&&v==0, v==0, interior}.  The tables below give
// the prediction each case uses; the HIP kernels
// select a formula per pixel from them at compile time.  oracle/audit_tables.py
// checks these tables and formula spellings against the reference source text.
#pragma once
#include <cstdint>
#include <hip/hip_runtime.h>

namespace lfm {

// position of a neighbour relative to (x, y); T = Nnum
enum Nb : int { NB_A, NB_B, NB_C, NB_AP, NB_BP, NB_CP, NB_AP1, NB_BP1, NB_ABP, NB_BAP, NB_COUNT };

enum Formula : int {
    F_Z = 0,
    F_A, F_B, F_C, F_AP, F_BP, F_CP,
    F_AVG_A_AP, F_AVG_B_BP, F_AVG_A_BP, F_AVG_C_BP, F_AVG_B_AP,
    F_AVG_C_AP, F_AVG_B_CP, F_AVG_A_CP, F_AVG_C_CP, F_AVG_A_B, F_AVG_B_A,
    F_AVG_BP_AP,
    F_ABC, F_BAC, F_ABC_SUM,
    F_P4_0Y, F_P4_X0, F_P4_COL, F_P4_CORNER, F_P4_ROW, F_P4_IN,
    F_P5_00Q,
    F_P5_0Y, F_P5_X0, F_P5_COL, F_P5_CORNER, F_P5_ROW, F_P5_IN,
    F_A_HBC, F_B_HAC,
    F_P6_0Y, F_P6_X0, F_P6_COL, F_P6_CORNER, F_P6_ROW, F_P6_IN,
    F_P7_0Y, F_P7_X0, F_P7_IN,
    F_COUNT
};

enum TileCase : int { TC_00 = 0, TC_0Y = 1, TC_X0 = 2, TC_XY = 3 };
enum PosCase : int { UC_COL = 0, UC_CORNER = 1, UC_ROW = 2, UC_IN = 3 };

// [predictor-1][tile case][position case]
constexpr uint8_t kTiles[7][4][4] = {
    {{F_B, F_Z, F_A, F_A}, {F_B, F_BP, F_A, F_A}, {F_AP, F_AP, F_AVG_A_AP, F_AVG_A_AP}, {F_AP, F_AP, F_AVG_A_AP, F_AVG_A_AP}},
    {{F_B, F_Z, F_A, F_B}, {F_AVG_B_BP, F_BP, F_BP, F_AVG_B_BP}, {F_B, F_AP, F_A, F_B}, {F_BP, F_BP, F_AVG_B_BP, F_AVG_B_BP}},
    {{F_B, F_Z, F_A, F_C}, {F_AVG_B_BP, F_BP, F_AVG_A_BP, F_AVG_C_BP}, {F_AVG_B_AP, F_AP, F_AVG_A_AP, F_AVG_C_AP}, {F_AVG_B_CP, F_CP, F_AVG_A_CP, F_AVG_C_CP}},
    {{F_B, F_Z, F_A, F_ABC}, {F_AVG_B_BP, F_BP, F_AVG_A_BP, F_P4_0Y}, {F_AVG_B_AP, F_AP, F_AVG_A_AP, F_P4_X0}, {F_P4_COL, F_P4_CORNER, F_P4_ROW, F_P4_IN}},
    {{F_B, F_Z, F_A, F_P5_00Q}, {F_AVG_B_BP, F_BP, F_AVG_A_BP, F_P5_0Y}, {F_AVG_B_AP, F_AP, F_AVG_A_AP, F_P5_X0}, {F_P5_COL, F_P5_CORNER, F_P5_ROW, F_P5_IN}},
    {{F_B, F_Z, F_A, F_B_HAC}, {F_AVG_B_BP, F_BP, F_AVG_A_BP, F_P6_0Y}, {F_AVG_B_AP, F_AP, F_AVG_A_AP, F_P6_X0}, {F_P6_COL, F_P6_CORNER, F_P6_ROW, F_P6_IN}},
    {{F_B, F_Z, F_A, F_AVG_A_B}, {F_AVG_B_BP, F_BP, F_AVG_A_BP, F_P7_0Y}, {F_AVG_B_AP, F_AP, F_AVG_A_AP, F_P7_X0}, {F_P4_COL, F_P4_CORNER, F_P4_ROW, F_P7_IN}},
};
constexpr uint8_t kAngle[7][4][4] = {
    {{F_B, F_Z, F_A, F_A}, {F_B, F_BP, F_A, F_A}, {F_B, F_AP, F_A, F_A}, {F_B, F_AP, F_A, F_A}},
    {{F_B, F_Z, F_A, F_B}, {F_B, F_BP, F_A, F_B}, {F_B, F_AP, F_A, F_B}, {F_B, F_BP, F_B, F_B}},
    {{F_B, F_Z, F_A, F_C}, {F_B, F_BP, F_A, F_C}, {F_B, F_AP, F_A, F_C}, {F_B, F_CP, F_A, F_C}},
    {{F_B, F_Z, F_A, F_ABC}, {F_B, F_BP, F_A, F_ABC}, {F_B, F_AP, F_A, F_ABC}, {F_B, F_ABC_SUM, F_A, F_BAC}},
    {{F_B, F_Z, F_A, F_A_HBC}, {F_B, F_BP, F_A, F_A_HBC}, {F_B, F_AP, F_A, F_A_HBC}, {F_B, F_P5_CORNER, F_A, F_B_HAC}},
    {{F_B, F_Z, F_A, F_B_HAC}, {F_B, F_BP, F_A, F_B_HAC}, {F_B, F_AP, F_A, F_B_HAC}, {F_B, F_P6_CORNER, F_A, F_A_HBC}},
    {{F_B, F_Z, F_A, F_AVG_A_B}, {F_B, F_BP, F_A, F_AVG_A_B}, {F_B, F_AP, F_A, F_AVG_A_B}, {F_B, F_ABC_SUM, F_A, F_AVG_B_A}},
};
constexpr uint8_t kSpace[7][4][4] = {
    {{F_B, F_Z, F_A, F_A}, {F_BP, F_BP, F_BP, F_BP}, {F_AP, F_AP, F_AP, F_AP}, {F_AP, F_AP, F_AP, F_AP}},
    {{F_B, F_Z, F_A, F_B}, {F_BP, F_BP, F_BP, F_BP}, {F_AP, F_AP, F_AP, F_AP}, {F_BP, F_BP, F_BP, F_BP}},
    {{F_B, F_Z, F_A, F_C}, {F_BP, F_BP, F_BP, F_BP}, {F_AP, F_AP, F_AP, F_AP}, {F_CP, F_CP, F_CP, F_CP}},
    {{F_B, F_Z, F_A, F_ABC}, {F_BP, F_BP, F_BP, F_BP}, {F_AP, F_AP, F_AP, F_AP}, {F_ABC_SUM, F_ABC_SUM, F_ABC_SUM, F_ABC_SUM}},
    {{F_B, F_Z, F_A, F_A_HBC}, {F_BP, F_BP, F_BP, F_BP}, {F_AP, F_AP, F_AP, F_AP}, {F_P5_CORNER, F_P5_CORNER, F_P5_CORNER, F_P5_CORNER}},
    {{F_B, F_Z, F_A, F_B_HAC}, {F_BP, F_BP, F_BP, F_BP}, {F_AP, F_AP, F_AP, F_AP}, {F_P6_CORNER, F_P6_CORNER, F_P6_CORNER, F_P6_CORNER}},
    {{F_B, F_Z, F_A, F_AVG_A_B}, {F_BP, F_BP, F_BP, F_BP}, {F_AP, F_AP, F_AP, F_AP}, {F_ABC_SUM, F_ABC_SUM, F_ABC_SUM, F_AVG_BP_AP}},
};

__host__ __device__ constexpr int case_formula(int fam, int k, int tc, int uc)
{
    return fam == 0 ? kTiles[k - 1][tc][uc] : fam == 1 ? kAngle[k - 1][tc][uc] : kSpace[k - 1][tc][uc];
}

// angle/space temporal cases where the reference applies "+P >> 1" twice
__host__ __device__ constexpr bool temporal_twice(int fam, int k, int tc, int uc)
{
    return (fam == 1 && k == 4 && tc == TC_XY && (uc == UC_CORNER || uc == UC_ROW)) ||
           (fam == 2 && k == 6 && tc == TC_00 && uc == UC_ROW);
}

// Every formula is an inner integer expression followed by an arithmetic
// right shift by formula_shift(F) (0, 1 or 2).  The kernels select between
// two cases' inner sums when their shifts (and temporal finishing, below)
// agree, and shift once.
__host__ __device__ constexpr int formula_shift(int F)
{
    return (F >= F_AVG_A_AP && F <= F_AVG_BP_AP) || F == F_P4_0Y || F == F_P4_X0 || F == F_P4_COL ||
                   F == F_P4_ROW || F == F_P4_IN || F == F_P5_00Q || F == F_P5_0Y || F == F_P5_X0 || F == F_P5_COL ||
                   F == F_P5_ROW || F == F_P5_IN || F == F_P6_0Y || F == F_P6_X0 || F == F_P6_COL || F == F_P6_ROW ||
                   F == F_P6_IN
               ? 1
               : (F == F_P7_0Y || F == F_P7_X0 || F == F_P7_IN) ? 2 : 0;
}

// The inner expression of formula F with a neighbour accessor g
// (g.template at<NB_x>()); eval_formula = eval_inner >> formula_shift.
template <int F, class G>
__host__ __device__ __forceinline__ int eval_inner(G& g)
{
#define A (g.template at<NB_A>())
#define B (g.template at<NB_B>())
#define C (g.template at<NB_C>())
#define Ap (g.template at<NB_AP>())
#define Bp (g.template at<NB_BP>())
#define Cp (g.template at<NB_CP>())
#define Ap1 (g.template at<NB_AP1>())
#define Bp1 (g.template at<NB_BP1>())
#define ABp (g.template at<NB_ABP>())
#define BAp (g.template at<NB_BAP>())
    if constexpr (F == F_Z) return 0;
    if constexpr (F == F_A) return A;
    if constexpr (F == F_B) return B;
    if constexpr (F == F_C) return C;
    if constexpr (F == F_AP) return Ap;
    if constexpr (F == F_BP) return Bp;
    if constexpr (F == F_CP) return Cp;
    if constexpr (F == F_AVG_A_AP) return A + Ap;
    if constexpr (F == F_AVG_B_BP) return B + Bp;
    if constexpr (F == F_AVG_A_BP) return A + Bp;
    if constexpr (F == F_AVG_C_BP) return C + Bp;
    if constexpr (F == F_AVG_B_AP) return B + Ap;
    if constexpr (F == F_AVG_C_AP) return C + Ap;
    if constexpr (F == F_AVG_B_CP) return B + Cp;
    if constexpr (F == F_AVG_A_CP) return A + Cp;
    if constexpr (F == F_AVG_C_CP) return C + Cp;
    if constexpr (F == F_AVG_A_B) return A + B;
    if constexpr (F == F_AVG_B_A) return B + A;
    if constexpr (F == F_AVG_BP_AP) return Bp + Ap;
    if constexpr (F == F_ABC) return A + B - C;
    if constexpr (F == F_BAC) return B + A - C;
    if constexpr (F == F_ABC_SUM) return Bp + Ap - Cp;
    if constexpr (F == F_P4_0Y) return A + B - C + Bp;
    if constexpr (F == F_P4_X0) return A + B - C + Ap;
    if constexpr (F == F_P4_COL) return Bp + Ap - Cp + B;
    if constexpr (F == F_P4_CORNER) return Bp + Ap - Cp;
    if constexpr (F == F_P4_ROW) return Bp + Ap - Cp + A;
    if constexpr (F == F_P4_IN) return Bp + Ap - Cp + B + A - C;
    if constexpr (F == F_P5_00Q) return A + (B - C);
    if constexpr (F == F_P5_0Y) return A + ((B - C) >> 1) + Bp;
    if constexpr (F == F_P5_X0) return A + ((B - C) >> 1) + Ap;
    if constexpr (F == F_P5_COL) return Bp + ((Ap - Cp) >> 1) + B;
    if constexpr (F == F_P5_CORNER) return Bp + ((Ap - Cp) >> 1);
    if constexpr (F == F_P5_ROW) return Bp + ((Ap - Cp) >> 1) + A;
    if constexpr (F == F_P5_IN) return Bp + ((Ap - Cp) >> 1) + B + ((A - C) >> 1);
    if constexpr (F == F_A_HBC) return A + ((B - C) >> 1);
    if constexpr (F == F_B_HAC) return B + ((A - C) >> 1);
    if constexpr (F == F_P6_0Y) return B + ((A - C) >> 1) + Bp;
    if constexpr (F == F_P6_X0) return B + ((A - C) >> 1) + Ap;
    if constexpr (F == F_P6_COL) return Ap + ((Bp - Cp) >> 1) + B;
    if constexpr (F == F_P6_CORNER) return Ap + ((Bp - Cp) >> 1);
    if constexpr (F == F_P6_ROW) return Ap + ((Bp - Cp) >> 1) + A;
    if constexpr (F == F_P6_IN) return Ap + ((Bp - Cp) >> 1) + A + ((B - C) >> 1);
    if constexpr (F == F_P7_0Y) return A + B + ABp + Bp1;
    if constexpr (F == F_P7_X0) return A + B + BAp + Ap1;
    if constexpr (F == F_P7_IN) return Bp1 + Ap1 + B + A;
#undef A
#undef B
#undef C
#undef Ap
#undef Bp
#undef Cp
#undef Ap1
#undef Bp1
#undef ABp
#undef BAp
    return 0;
}

// Evaluate formula F with a neighbour accessor g.
template <int F, class G>
__host__ __device__ __forceinline__ int eval_formula(G& g)
{
    return eval_inner<F>(g) >> formula_shift(F);
}

// Residual before the int16 store, for a case (FAM, K, TC, UC).
//  spatial: I - pred
//  temporal tiles:        I - ((pred + P) >> 1)      (pred == 0 case: I - P)
//  temporal angle/space:  ((I - pred) + P) >> 1       (pred == 0 case: I - P)
template <int FAM, int K, int TC, int UC, bool TEMPORAL, class G>
__host__ __device__ __forceinline__ int case_residual(G& g, int I, int P)
{
    if constexpr (K < 1) {  // predictor 0 (raw) / diagnostic builds
        return I;
    } else {
        constexpr int F = case_formula(FAM, K, TC, UC);
        if constexpr (!TEMPORAL) {
            return I - eval_formula<F>(g);
        } else if constexpr (F == F_Z) {
            return I - P;
        } else if constexpr (FAM == 0) {
            return I - ((eval_formula<F>(g) + P) >> 1);
        } else if constexpr (temporal_twice(FAM, K, TC, UC)) {
            return ((((I - eval_formula<F>(g)) + P) >> 1) + P) >> 1;
        } else {
            return ((I - eval_formula<F>(g)) + P) >> 1;
        }
    }
}

// How a case turns its prediction into the residual (as case_residual above):
// 0 spatial I - pred; 1 temporal tiles I - ((pred + P) >> 1); 2 temporal with
// no prediction I - P; 3 temporal angle / space ((I - pred) + P) >> 1; 4 the
// same with "+ P >> 1" applied twice.
__host__ __device__ constexpr int finish_kind(int fam, int k, int tc, int uc, bool temporal)
{
    return !temporal ? 0
                     : case_formula(fam, k, tc, uc) == F_Z ? 2
                                                          : fam == 0 ? 1 : temporal_twice(fam, k, tc, uc) ? 4 : 3;
}

template <int KIND>
__host__ __device__ __forceinline__ int finish_residual(int pred, int I, int P)
{
    if constexpr (KIND == 0) return I - pred;
    if constexpr (KIND == 1) return I - ((pred + P) >> 1);
    if constexpr (KIND == 2) return I - P;
    if constexpr (KIND == 3) return ((I - pred) + P) >> 1;
    return ((((I - pred) + P) >> 1) + P) >> 1;
}

// zig-zag symbol of the int16-stored residual (lfm_Predictors.cu:16-26)
__host__ __device__ __forceinline__ uint32_t symbolize16(int r)
{
    int v = (int)(int16_t)r;
    int a = v < 0 ? -v : v;
    return (uint32_t)(2 * a + (v >> 31)) & 0xFFFFu;
}

// the same symbol as a zig-zag of the low 16 bits: (r << 1) ^ (bit 15 of r
// ? all ones : 0), masked to 16 bits -- 3 integer ops instead of abs + add
__host__ __device__ __forceinline__ uint32_t zigzag16(int r)
{
    return ((uint32_t)r << 1 ^ (uint32_t)((r << 16) >> 31)) & 0xFFFFu;
}

__host__ __device__ __forceinline__ int unsymbolize16(uint32_t s)
{
    int neg = (int)(s & 1u);
    return (1 - 2 * neg) * ((int)(s + neg) >> 1);
}

} // namespace lfm
