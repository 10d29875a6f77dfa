/*
 * klb_Cwrapper.h -- the C ABI of the reference (src/klb_Cwrapper.h:40-64),
 * served by liblfm.so.  Same function names, argument order, types and
 * return codes, so the JNI wrapper (src/jni/) and any ctypes / cgo / MEX
 * caller relinks without source changes.
 *
 * Return codes: 0 ok, 2 bzip2 error, 3 zlib / file / channel error,
 * 5 cannot open output or unknown compression; liblfm adds
 * 6 invalid predictor request (header bits 0-6 >= 16) and
 * 7 the predictor stage needs a GPU and none is usable.
 * readKLBstack returns a malloc'ed buffer the caller frees, or NULL.
 */
#ifndef LFM_KLB_CWRAPPER_H
#define LFM_KLB_CWRAPPER_H

#ifdef __cplusplus
extern "C" {
#endif

#include <stdint.h>
#include "common.h"

#define DECLSPECIFIER __attribute__((visibility("default")))

/* Encode a stack. headerVersion is 0 (auto-select the predictor) and Nnum 13,
 * as in the reference (klb_Cwrapper.cpp:27); use lfm_api.h for other values. */
DECLSPECIFIER int writeKLBstack(const void* im, const char* filename, uint32_t xyzct[KLB_DATA_DIMS],
                                enum KLB_DATA_TYPE dataType, int numThreads, float32_t pixelSize[KLB_DATA_DIMS],
                                uint32_t blockSize[KLB_DATA_DIMS], enum KLB_COMPRESSION_TYPE compressionType,
                                char metadata[KLB_METADATA_SIZE]);

/* One pointer per xy slice (xyzct[3] = xyzct[4] = 1); no predictor stage. */
DECLSPECIFIER int writeKLBstackSlices(const void** im, const char* filename, uint32_t xyzct[KLB_DATA_DIMS],
                                      enum KLB_DATA_TYPE dataType, int numThreads,
                                      float32_t pixelSize[KLB_DATA_DIMS], uint32_t blockSize[KLB_DATA_DIMS],
                                      enum KLB_COMPRESSION_TYPE compressionType, char metadata[KLB_METADATA_SIZE]);

DECLSPECIFIER int readKLBheader(const char* filename, uint32_t xyzct[KLB_DATA_DIMS], enum KLB_DATA_TYPE* dataType,
                                float32_t pixelSize[KLB_DATA_DIMS], uint32_t blockSize[KLB_DATA_DIMS],
                                enum KLB_COMPRESSION_TYPE* compressionType, char metadata[KLB_METADATA_SIZE]);

DECLSPECIFIER void* readKLBstack(const char* filename, uint32_t xyzct[KLB_DATA_DIMS], enum KLB_DATA_TYPE* dataType,
                                 int numThreads, float32_t pixelSize[KLB_DATA_DIMS],
                                 uint32_t blockSize[KLB_DATA_DIMS], enum KLB_COMPRESSION_TYPE* compressionType,
                                 char metadata[KLB_METADATA_SIZE]);

DECLSPECIFIER int readKLBstackInPlace(const char* filename, void* im, enum KLB_DATA_TYPE* dataType, int numThreads);

/* inclusive bounds; decodes the full image and crops (correct with predictors) */
DECLSPECIFIER int readKLBroiInPlace(const char* filename, void* im, uint32_t xyzctLB[KLB_DATA_DIMS],
                                    uint32_t xyzctUB[KLB_DATA_DIMS], int numThreads);

#ifdef __cplusplus
}
#endif
#endif
