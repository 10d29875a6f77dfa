/*
 * common.h -- shared constants and enums of the .lfm / KLB container.
 *
 * Names and numeric values are the reference's (src/common.h:12-63) so that
 * callers written against it (MEX writeLFMstack/readLFMstack, JNI) compile
 * unchanged.  LFM_PREDICTOR_WAY is the DEFAULT predictor family here; the
 * family can be changed at run time (env LFM_PREDICTOR_WAY or lfm_set_family()
 * in lfm_api.h) instead of recompiling as the reference requires.
 */
#ifndef LFM_COMMON_H
#define LFM_COMMON_H

typedef float float32_t;
typedef double float64_t;

#define KLB_DATA_DIMS (5)              /* x, y, z, c, t */
#define KLB_METADATA_SIZE (256)        /* bytes of free-form metadata */
#define KLB_DEFAULT_HEADER_VERSION (0) /* bit 7 video flag, bits 0-6 predictor request */
#define NUM_PREDICTORS (8)             /* candidate 0 = raw, 1..7 = predictors */
#define LFM_PREDICTOR_WAY (0)          /* default family: 0 tiles, 1 angle, 2 space */

enum KLB_DATA_TYPE {
    UINT8_TYPE = 0, UINT16_TYPE = 1, UINT32_TYPE = 2, UINT64_TYPE = 3,
    INT8_TYPE = 4, INT16_TYPE = 5, INT32_TYPE = 6, INT64_TYPE = 7,
    FLOAT32_TYPE = 8, FLOAT64_TYPE = 9
};

enum KLB_COMPRESSION_TYPE { NONE = 0, BZIP2 = 1, ZLIB = 2 };

enum LFM_PREDICTORS { ANGLE_AND_SPACE = 0, ANGLE = 1, SPACE = 2 };

/* spelling kept from the reference so existing callers compile */
enum LFM_PREDICTORS_TYPE {
    NO_PREIDICTORS = 0,
    PREIDCTORS_A = 1,
    PREIDCTORS_B = 2,
    PREIDCTORS_C = 3,
    PREIDCTORS_APB_DC = 4,
    PREIDCTORS_A_BDC_Div2 = 5,
    PREIDCTORS_B_ADC_Div2 = 6,
    PREIDCTORS_APB_Div2 = 7,
    PREIDCTORS_APB_Div2_Exten = 8
};

#endif
